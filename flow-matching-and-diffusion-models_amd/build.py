"""Build the gfx950 HIP library in-tree: csrc/*.hip -> fmdiff/lib/libfmdiff_hip.so.

Plain ``hipcc --offload-arch=gfx950`` (no torch extension machinery): the
product's C ABI is declared in ``include/fmdiff.h`` and loaded with ctypes.
Objects are cached by source + header mtime so rebuilds are incremental.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build", "obj")
LIB_DIR = os.path.join(HERE, "fmdiff", "lib")
LIB = os.path.join(LIB_DIR, "libfmdiff_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("FMD_OFFLOAD_ARCH", "gfx950")
# -fno-slp-vectorize: packed f32 VALU (v_pk_fma/v_pk_mul + the v_mov pairs that feed them) costs more issue
# slots than scalar FMAs beside MFMAs (MI355X_MICROARCH.md constants table); measured faster end to end
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-slp-vectorize", "-I", CSRC, "-I", INCLUDE,
         *os.environ.get("FMD_EXTRA_FLAGS", "").split()]
_FLAG_TAG = format(zlib.crc32(" ".join(FLAGS).encode()), "08x")   # objects are cached per flag set


def _deps_mtime():
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(INCLUDE, "fmdiff.h"))
    return max(os.path.getmtime(h) for h in headers)


def _compile(src: str, dep_mtime: float) -> str:
    obj = os.path.join(OBJ, f"{os.path.basename(src)}.{_FLAG_TAG}.o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), dep_mtime):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    dep = _deps_mtime()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, dep), srcs))
    stamp = LIB + ".flags"
    same_flags = os.path.exists(stamp) and open(stamp).read() == _FLAG_TAG
    if not same_flags or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        with open(stamp, "w") as f:
            f.write(_FLAG_TAG)
    if verbose:
        print(f"[fmdiff] built {LIB} from {len(srcs)} sources", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build()
