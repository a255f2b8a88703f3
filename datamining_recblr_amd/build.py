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
# measurement aids for bench.py (probes/recblr_probe.h): their own library,
# hidden visibility, never loaded by the model's path
PROBE_SOURCES = sorted(glob.glob(os.path.join(_HERE, "probes", "*.hip")))
PROBE_HEADERS = HEADERS + sorted(glob.glob(os.path.join(_HERE, "probes", "*.h")))
PROBE_OUT = os.path.join(_HERE, "lib", "libdmrecblr_probe.so")
# opt-in experimental kernels (experimental/recblr_exp.h): their own library,
# hidden visibility, loaded only when requested (RECBLR_FUSED_GRL*)
EXP_SOURCES = sorted(glob.glob(os.path.join(_HERE, "experimental", "*.hip")))
EXP_HEADERS = HEADERS + sorted(glob.glob(os.path.join(_HERE, "experimental", "*.h")))
EXP_OUT = os.path.join(_HERE, "lib", "libdmrecblr_exp.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

# -ffp-contract=off: the reference scan is compiled with enable_fp_fusion=False
# (parallel_scan.py:92) and its gate math is separate torch ops, so no FMA
# contraction anywhere keeps our rounding close to it.
FLAGS = ["-O3", "-std=c++20", "-shared", "-fPIC", f"--offload-arch={ARCH}",
         "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _stale(out, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in deps)


def _compile(out, sources, extra, verbose, jobs):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), *FLAGS, *extra, "-I", os.path.join(ROOT, "include"), "-o", tmp, *sources]
    if jobs > 1:
        cmd.insert(1, f"-parallel-jobs={jobs}")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)


def build(force: bool = False, verbose: bool = False, jobs: int = 4) -> str:
    """Build the product library (and the probe and experimental libraries
    beside it); returns the product library's path."""
    if force or _stale(OUT, SOURCES + HEADERS):
        _compile(OUT, SOURCES, [], verbose, jobs)
    if PROBE_SOURCES and (force or _stale(PROBE_OUT, PROBE_SOURCES + PROBE_HEADERS)):
        _compile(PROBE_OUT, PROBE_SOURCES, ["-fvisibility=hidden"], verbose, jobs)
    if EXP_SOURCES and (force or _stale(EXP_OUT, EXP_SOURCES + EXP_HEADERS)):
        _compile(EXP_OUT, EXP_SOURCES, ["-fvisibility=hidden"], verbose, jobs)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
