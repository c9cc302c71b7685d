"""Build a variant of the native library with ONE source replaced by another file (e.g. the previous
revision of a kernel, for an A/B on the same box):
    git show HEAD~1:csrc/kernels/gemm_glds.hip > /tmp/old/gemm_glds.hip
    python scripts/diag/build_variant_src.py /tmp/old/gemm_glds.hip exp/variants/_C_old.so
The replaced source is the tree's file of the same name; its relative includes resolve against
csrc/kernels. The other objects come from build/native (run the normal build first)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fluxmpi_amd import _build as B  # noqa: E402

path, out, *flags = sys.argv[1:]
srcs = B._sources()
target = next(s for s in srcs if os.path.basename(s) == os.path.basename(path))
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
obj = os.path.abspath(out) + ".o"
cmd = [os.path.abspath(path) if c == target else c for c in B._compile_cmd(target, obj)]
cmd += ["-I", os.path.dirname(target), *flags]
subprocess.run(cmd, check=True)
objs = [obj if s == target else B._obj_for(s) for s in srcs]
tl = B._torch_lib()
link = [B._tool("hipcc"), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs, f"-L{B.ROCM}/lib",
        "-lamdhip64", f"-L{tl}", "-l:librccl.so", f"-Wl,-rpath,{tl}", f"-Wl,-rpath,{B.ROCM}/lib"]
subprocess.run(link, check=True)
os.remove(obj)
print(out)
