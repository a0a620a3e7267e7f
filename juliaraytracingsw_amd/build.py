"""Build libsw.so in-tree with hipcc for gfx950 (no JIT cache, so the .so
travels to the GPU box with the repository snapshot).

The kernel file is compiled as one translation unit per transform length
(``-DSW_PART=L``, L = log2 N = 5 … 13) plus the length-independent part
(``SW_PART=0``: element-wise kernels and the dispatch), in parallel, then
linked with the host-side API (``sw_api.cpp``) and the generic engine for
grids that are not powers of two (``sw_generic.hip``)."""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["sw_kernels.hip", "sw_api.cpp", "sw_generic.hip"]
HEADERS = ["sw_fft.hpp", "sw_internal.hpp", "sw_generic.hpp"]
OUT = os.path.join(HERE, "libsw.so")
PARTS = [0, 13, 12, 11, 10, 9, 8, 7, 6, 5]  # longest first (compile time)


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


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}): {' '.join(cmd)}\n{r.stderr[-4000:]}")


def build_lib(verbose=False, force=False, out=OUT, extra_flags=(), jobs=None, parts=None):
    """parts: [L] builds transform length 2^L only (experiments: the dispatch
    then knows that length alone); default every length."""
    if not force and not needs_build(out):
        return out
    hipcc = hipcc_path()
    common = [hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wno-unused-result",
              f"-I{os.path.join(ROOT, 'include')}", *extra_flags]
    jobs = jobs or min(len(PARTS) + 1, max(1, len(os.sched_getaffinity(0))))
    with tempfile.TemporaryDirectory(prefix="libsw_build_") as tmp:
        cmds = []
        plist = [0] + [q for q in PARTS if q and (parts is None or q in parts)]
        only = [f"-DSW_ONLY_LOG2={parts[0]}"] if parts is not None and len(parts) == 1 else []
        for part in plist:
            cmds.append(common + only + ["-c", f"-DSW_PART={part}", os.path.join(CSRC, "sw_kernels.hip"),
                                         "-o", os.path.join(tmp, f"k{part}.o")])
        cmds.append(common + ["-c", os.path.join(CSRC, "sw_api.cpp"), "-o", os.path.join(tmp, "api.o")])
        # the generic engine (grids that are not powers of two, sw_generic.hpp)
        cmds.append(common + ["-c", os.path.join(CSRC, "sw_generic.hip"), "-o", os.path.join(tmp, "gen.o")])
        if verbose:
            for c in cmds:
                print(" ".join(c))
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_run, cmds))
        objs = [os.path.join(tmp, f"k{p}.o") for p in plist] + [os.path.join(tmp, "api.o"), os.path.join(tmp, "gen.o")]
        link = [hipcc, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out + ".tmp", *objs,
                "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(link))
        _run(link)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_lib(verbose=True, force=True))
