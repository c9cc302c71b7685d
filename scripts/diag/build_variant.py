"""Build a variant of the native library with extra compile flags for ONE source (diagnostics):
    python scripts/diag/build_variant.py gemm_nt.hip exp/variants/_C_v1.so -DGNT_DBG=1
The other objects come from build/native (run the normal build first). Load the result with
scripts/diag/load_variant.py (module name _C, any path)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fluxmpi_amd import _build as B  # noqa: E402

src_name, out, *flags = sys.argv[1:]
srcs = B._sources()
target = next(s for s in srcs if os.path.basename(s) == src_name)
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
obj = os.path.abspath(out) + ".o"
cmd = B._compile_cmd(target, obj) + flags
subprocess.run(cmd, check=True)
objs = [obj if s == target else B._obj_for(s) for s in srcs]
tl = B._torch_lib()
link = [B._tool("hipcc"), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs, f"-L{B.ROCM}/lib",
        "-lamdhip64", f"-L{tl}", "-l:librccl.so", f"-Wl,-rpath,{tl}", f"-Wl,-rpath,{B.ROCM}/lib"]
subprocess.run(link, check=True)
os.remove(obj)
print(out)
