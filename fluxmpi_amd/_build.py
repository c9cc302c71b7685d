"""In-tree build of the native library ``fluxmpi_amd/_C*.so`` (no hipify, no JIT cache).

* ``*.hip`` sources: ``hipcc --offload-arch=gfx950 -O3`` (device + host code),
* ``*.cpp`` sources: ``amdclang++`` as plain host C++ against the HIP headers,
* link: ``hipcc -shared`` against ``libamdhip64`` and the ``librccl.so`` that
  PyTorch ships (same SONAME as the one ``import torch`` already loaded, so a
  process never holds two RCCL runtimes).

Objects go to ``build/native/``; a source is recompiled only when it (or a
header under ``csrc/``) is newer than its object. Run ``python -m
fluxmpi_amd._build`` or ``fluxmpi_amd.build()``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("FLUXMPI_ARCH", "gfx950")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def output_path() -> str:
    return os.path.join(ROOT, "fluxmpi_amd", "_C" + _ext_suffix())


def _sources() -> list[str]:
    srcs = sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True))
    srcs += sorted(glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True))
    return srcs


def _headers() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _torch_lib() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _tool(name: str) -> str:
    for cand in (os.path.join(ROCM, "bin", name), os.path.join(ROCM, "llvm", "bin", name), shutil.which(name)):
        if cand and os.path.exists(cand):
            return cand
    raise FileNotFoundError(f"{name} not found (ROCM_PATH={ROCM})")


def _obj_for(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


# per-file extra flags: no SLP vectorisation in the MFMA kernels — plain -O3 packs adjacent f32
# math (epilogues, softmax, operand prologues) into v_pk_*_f32, an anti-lever beside MFMAs
# (MI355X_MICROARCH.md price list). For speed only: the round-4 NaNs of the SLP gemm_nt build were
# an epilogue store-data hazard, fixed in the source (gemm_nt.hip store_guard; the SLP build is
# clean: profiles/rd5c_gemm_nt_store_hazard.md). The memory-bound elementwise kernels keep it.
_NO_SLP = ["-fno-slp-vectorize"]
EXTRA_FLAGS = {f: _NO_SLP for f in ("gemm_nt.hip", "attention.hip", "gemm_glds.hip", "gemm.hip", "conv3x3n.hip",
                                        "wgrad3x3n.hip", "linbwd.hip")}


def _compile_cmd(src: str, obj: str) -> list[str]:
    import pybind11

    common = ["-O3", "-fPIC", "-std=c++17", "-I", CSRC, "-Wall", "-Wno-unused-function",
              "-Wno-unused-variable", "-Wno-unused-but-set-variable"]
    if src.endswith(".hip"):
        return [_tool("hipcc"), f"--offload-arch={ARCH}", "-c", src, "-o", obj, *common,
                "-munsafe-fp-atomics", *EXTRA_FLAGS.get(os.path.basename(src), [])]
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{ROCM}/include"]
    return [_tool("amdclang++"), "-D__HIP_PLATFORM_AMD__=1", "-c", src, "-o", obj, *common, *inc,
            "-fvisibility=hidden"]


def _stale(obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Compile and link ``fluxmpi_amd/_C``; returns the path of the shared object."""
    os.makedirs(BUILD, exist_ok=True)
    headers = _headers()
    srcs = _sources()
    out = output_path()
    jobs = jobs or min(8, os.cpu_count() or 4)

    todo = [(s, _obj_for(s)) for s in srcs if force or _stale(_obj_for(s), [s, *headers])]

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose and (r.stderr.strip()):
            print(r.stderr, file=sys.stderr)
        return r

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda so: run(_compile_cmd(*so)), todo))

    objs = [_obj_for(s) for s in srcs]
    if force or todo or _stale(out, objs):
        tl = _torch_lib()
        cmd = [_tool("hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs,
               f"-L{ROCM}/lib", "-lamdhip64", f"-L{tl}", "-l:librccl.so", f"-Wl,-rpath,{tl}",
               f"-Wl,-rpath,{ROCM}/lib"]
        run(cmd)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":  # pragma: no cover
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
