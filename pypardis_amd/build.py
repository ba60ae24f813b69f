"""In-tree build of libpardis.so (hipcc, gfx950 only).

    python -m pypardis_amd.build          # incremental
    python -m pypardis_amd.build --force

The .so is written next to this file so it travels with the repo snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "_obj")
LIB = os.path.join(HERE, "libpardis.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYPARDIS_ARCH", "gfx950")

# -ffp-contract=off: the fp64 neighbour predicate must round every product
# and sum separately (sklearn's Cython does; see engine.hip).  The kernels
# also use __dmul_rn/__dadd_rn, so this is belt and braces.
CFLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
          "-fno-fast-math", "-Wall", "-Wno-unused-result", f"-I{INCLUDE}"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")]
    return hs + [os.path.join(INCLUDE, "pardis.h")]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
    dep = max([_mtime(src)] + [_mtime(h) for h in headers()])
    if _mtime(obj) >= dep:
        return obj, None
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


INGEST_SRC = os.path.join(CSRC, "ingest.cpp")
INGEST = os.path.join(HERE, "_ingest.so")


def build_ingest(force=False):
    """The host-side (key, vector) record unzip (csrc/ingest.cpp), a CPython
    extension built with the system g++ against this interpreter's headers."""
    if not force and _mtime(INGEST) >= _mtime(INGEST_SRC):
        return INGEST
    import sysconfig
    cmd = ["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-Wall",
           f"-I{sysconfig.get_paths()['include']}", INGEST_SRC, "-o", INGEST]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"ingest build failed:\n{r.stdout}\n{r.stderr}")
    return INGEST


def build(force=False, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    if force:
        for f in os.listdir(OBJ):
            os.remove(os.path.join(OBJ, f))
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(_compile, srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("libpardis build failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    build_ingest(force)
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        # librccl.so.1 (pd_comm_*): under torch the process already holds
        # torch's RCCL (same soname), so one RCCL serves both
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args()
    build(force=args.force)
