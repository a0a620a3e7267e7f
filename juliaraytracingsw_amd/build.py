"""Build libsw.so in-tree with hipcc for gfx950 (no JIT cache, so the .so
travels to the GPU box with the repository snapshot)."""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["sw_kernels.hip", "sw_api.cpp"]
HEADERS = ["sw_fft.hpp", "sw_internal.hpp"]
OUT = os.path.join(HERE, "libsw.so")


def hipcc_path():
    p = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found")
    return p


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "sw.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(verbose=False, force=False, out=OUT, extra_flags=()):
    if not force and not needs_build(out):
        return out
    cmd = [hipcc_path(), "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
           "-Wno-unused-result", f"-I{os.path.join(ROOT, 'include')}", "-o", out + ".tmp",
           *extra_flags, *[os.path.join(CSRC, s) for s in SOURCES],
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_lib(verbose=True, force=True))
