"""Build the gfx950 HIP extension in-tree.

``python -m datamining_recblr_amd.build`` compiles csrc/*.hip into
``datamining_recblr_amd/lib/libdmrecblr.so`` with hipcc.  Cross-compiles
without a GPU, so it runs in the CPU container as well as on the GPU box.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
SOURCES = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")))
HEADERS = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.h"))) + [
    os.path.join(ROOT, "include", "recblr_hip.h")]
OUT = os.path.join(_HERE, "lib", "libdmrecblr.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

# -ffp-contract=off: the reference scan is compiled with enable_fp_fusion=False
# (parallel_scan.py:92) and its gate math is separate torch ops, so no FMA
# contraction anywhere keeps our rounding close to it.
FLAGS = ["-O3", "-std=c++17", "-shared", "-fPIC", f"--offload-arch={ARCH}",
         "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + HEADERS
    return any(os.path.getmtime(s) > t for s in deps)


def build(force: bool = False, verbose: bool = False, jobs: int = 4) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *FLAGS, "-I", os.path.join(ROOT, "include"), "-o", tmp, *SOURCES]
    if jobs > 1:
        cmd.insert(1, f"-parallel-jobs={jobs}")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
