"""Summaries of rocprofv3 (ROCm 7.2, rocpd SQLite) outputs, for profiles/.

    python tools/rocpd_summary.py stats <results.db> <out_kernel_stats.csv>
    python tools/rocpd_summary.py pmc <fetch.db> <write.db> <kernel-substring> <out.json> \
        [--alg-bytes B]

`stats` is the per-kernel table rocprofv3 --stats prints (calls, total/avg/min/max ns, %).
`pmc` averages FETCH_SIZE / WRITE_SIZE (kilobytes, one --pmc pass each) over the dispatches of
one kernel and converts them to HBM bytes per launch the way MI355X_MICROARCH.md §HBM
prescribes for gfx950: FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read,
so it is doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
from __future__ import annotations

import argparse
import csv
import json
import sqlite3
import statistics


def kernel_rows(db):
    """(name, duration) per dispatch; the name carries the grid when rocpd records it, so
    launches of one kernel with different batch shapes (grid.y = clients) are told apart."""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    gy = next((x for x in ("grid_size_y", "grid_y", "grid_size_y_") if x in cols), None)
    gx = next((x for x in ("grid_size_x", "grid_x") if x in cols), None)
    if gx and gy:
        return [(f"{n} [grid {x}x{y}]", d) for n, d, x, y in
                c.execute(f"select name, duration, {gx}, {gy} from kernels")]
    return c.execute("select name, duration from kernels").fetchall()


def stats(db, out):
    per = {}
    for name, dur in kernel_rows(db):
        per.setdefault(name, []).append(int(dur))
    total = sum(sum(v) for v in per.values()) or 1
    rows = sorted(per.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs",
                    "Percentage"])
        for name, d in rows:
            short = name if len(name) < 160 else name[:157] + "..."
            w.writerow([short, len(d), sum(d), round(sum(d) / len(d), 1), min(d), max(d),
                        round(100.0 * sum(d) / total, 3)])
    return rows


def pmc_values(db, counter, substr):
    c = sqlite3.connect(db)
    q = ("select kernel_name, value from counters_collection where counter_name = ? ")
    return [float(v) for name, v in c.execute(q, (counter,)) if substr in name]


def pmc(fetch_db, write_db, substr, out, alg_bytes=None, clients=1):
    f = pmc_values(fetch_db, "FETCH_SIZE", substr)
    w = pmc_values(write_db, "WRITE_SIZE", substr)
    if not f or not w:
        raise SystemExit(f"no dispatches of {substr!r} with FETCH_SIZE/WRITE_SIZE")
    fetch_kb, write_kb = statistics.mean(f), statistics.mean(w)
    hbm = 2.0 * fetch_kb * 1024 + write_kb * 1024
    res = {"kernel": substr, "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_size_kb_avg": round(fetch_kb, 1), "write_size_kb_avg": round(write_kb, 1),
           "hbm_read_bytes_per_launch": int(2.0 * fetch_kb * 1024),
           "hbm_write_bytes_per_launch": int(write_kb * 1024),
           "hbm_bytes_per_launch": int(hbm), "clients_per_launch": clients,
           "correction": "MI355X_MICROARCH.md §HBM: FETCH_SIZE x2 (gfx950 half-count of "
                         "16 B/lane streaming reads); WRITE_SIZE as reported"}
    if alg_bytes:
        res["alg_bytes_per_launch"] = int(alg_bytes)
        res["traffic_over_alg"] = round(hbm / alg_bytes, 4)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    return res


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("stats")
    s.add_argument("db")
    s.add_argument("out")
    p = sub.add_parser("pmc")
    p.add_argument("fetch_db")
    p.add_argument("write_db")
    p.add_argument("kernel")
    p.add_argument("out")
    p.add_argument("--alg-bytes", type=float, default=None)
    p.add_argument("--clients-per-launch", type=int, default=1)
    a = ap.parse_args()
    if a.cmd == "stats":
        for name, d in stats(a.db, a.out)[:12]:
            print(f"{len(d):7d} {sum(d) / len(d) / 1e3:10.2f} us  {name[:100]}")
    else:
        print(json.dumps(pmc(a.fetch_db, a.write_db, a.kernel, a.out, a.alg_bytes,
                             a.clients_per_launch), indent=1))


if __name__ == "__main__":
    main()
