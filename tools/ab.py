"""Same-box A/B of libfedcodec.so build variants (replaces the per-experiment tools/ab_*.sh).

    python tools/ab.py --out gpurun_out/ab_X.jsonl \
        --var base= --var wide=tools/variants/lib_wide.so \
        --probe "tools/sample_probe.py --n 134217728" \
        --probe "tools/sample_probe.py --n 134217728 --dense" [--reps 2] [--timeout 120]

Every probe is a script that accepts ``--lib PATH`` and ``--tag TAG`` and prints one JSON line
(tools/sample_probe.py, tools/kbench.py, bench.py with ``--lib``).  Variants run in turn, in
alternating order on every repetition (boxes differ by 2-4 %: compare only within one call).
Variants are built with tools/mkvar.sh (``FC_NAME=VALUE`` constants into tools/variants/lib_<name>.so);
``name=`` (empty path) is the default in-tree build.  Each result line gets ``var``, ``probe``
and ``rep``; a failing probe stops the run (no retries on the GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--var", action="append", required=True, help="tag=path ('' = in-tree build)")
    ap.add_argument("--probe", action="append", required=True)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=120)
    args = ap.parse_args()
    variants = []
    for v in args.var:
        tag, _, path = v.partition("=")
        if path and not os.path.exists(os.path.join(ROOT, path)):
            raise SystemExit(f"variant {tag}: {path} not built (tools/mkvar.sh)")
        variants.append((tag, path))
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "a") as fh:
        for rep in range(args.reps):
            order = variants if rep % 2 == 0 else variants[::-1]
            for tag, path in order:
                for probe in args.probe:
                    cmd = ["timeout", "-k", "10", str(args.timeout), sys.executable,
                           *shlex.split(probe), "--tag", tag]
                    if path:
                        cmd += ["--lib", path]
                    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
                    if p.returncode != 0:
                        sys.stderr.write(p.stderr[-3000:])
                        raise SystemExit(f"probe failed ({p.returncode}): {' '.join(cmd)}")
                    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
                    rec = json.loads(lines[-1]) if lines else {"raw": p.stdout[-500:]}
                    rec.update(var=tag, probe=probe, rep=rep)
                    fh.write(json.dumps(rec) + "\n")
                    fh.flush()
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
