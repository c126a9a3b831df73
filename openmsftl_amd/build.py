"""Build libfedcodec.so in-tree for gfx950 (hipcc, no CMake).

    python -m openmsftl_amd.build [--force]

The .so lands next to this file so it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libfedcodec.so")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libfedcodec.so)")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
                  + [os.path.join(os.path.dirname(HERE), "include", "fedcodec.h")])


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(s) <= t for s in sources())


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc(), *FLAGS, "-o", tmp, os.path.join(CSRC, "fedcodec.hip")]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, LIB)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    print(build(force=args.force))


if __name__ == "__main__":
    sys.exit(main())
