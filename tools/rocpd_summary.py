"""Summaries of rocprofv3 (ROCm 7.2, rocpd SQLite) outputs, for profiles/.

    python tools/rocpd_summary.py stats <results.db> <out_kernel_stats.csv>
    python tools/rocpd_summary.py pmc <fetch.db> <write.db> <kernel-substring> <out.json> \
        [--alg-bytes B] [--calib profiles/<tag>_pmc_calib.json]
    python tools/rocpd_summary.py calib <fetch.db> <write.db> <out.json>
    python tools/rocpd_summary.py counters <db> <kernel-substring>
    python tools/rocpd_summary.py timeline <db> [last-N-dispatches]

`stats` is the per-kernel table rocprofv3 --stats prints (calls, total/avg/min/max ns, %).
`pmc` averages FETCH_SIZE / WRITE_SIZE (kilobytes, one --pmc pass each) over the dispatches of
one kernel and converts them to HBM bytes per launch.  MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) streaming read and WRITE_SIZE is exact
for 16 B/lane streaming stores; other widths must be calibrated on a known byte count.
`calib` does that with tools/pmc_calib.hip's kernels (512 MiB each, k_compact_mag1's 4 B/lane
non-temporal read and its store shapes: 16 B/lane values, 8 B/lane uint16 indices) and `pmc --calib` applies the measured factors
(read: k_read4_nt, write: k_write16) instead of the 16 B/lane defaults.
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


def timeline(db, last=60):
    """The last dispatches in start order: start / end (us, relative to the first shown),
    duration and name (with grid), to see how launches of different streams overlap."""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    st = next(x for x in ("start", "start_ns", "begin") if x in cols)
    en = next(x for x in ("end", "end_ns") if x in cols)
    gx = next((x for x in ("grid_size_x", "grid_x") if x in cols), None)
    gy = next((x for x in ("grid_size_y", "grid_y") if x in cols), None)
    q = f"select name, {st}, {en}" + (f", {gx}, {gy}" if gx and gy else "") + f" from kernels order by {st}"
    rows = [r for r in c.execute(q).fetchall() if "fc::" in r[0]][-last:]
    t0 = rows[0][1]
    for r in rows:
        grid = f" [grid {r[3]}x{r[4]}]" if len(r) > 3 else ""
        print(f"{(r[1] - t0) / 1e3:10.1f} {(r[2] - t0) / 1e3:10.1f} {(r[2] - r[1]) / 1e3:9.1f}  "
              f"{r[0][:70]}{grid}")


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


CALIB_BYTES = 512 * 1024 * 1024          # tools/pmc_calib.py: bytes per calibration dispatch


def calib(fetch_db, write_db, out):
    """Bytes / reported bytes for each calibration kernel (its known 512 MiB)."""
    res = {"known_bytes_per_dispatch": CALIB_BYTES, "source": "tools/pmc_calib.hip"}
    for kern, db, ctr in (("k_read4_nt", fetch_db, "FETCH_SIZE"), ("k_read16", fetch_db, "FETCH_SIZE"),
                          ("k_write16", write_db, "WRITE_SIZE"), ("k_write4_nt", write_db, "WRITE_SIZE"),
                          ("k_write8", write_db, "WRITE_SIZE")):
        v = pmc_values(db, ctr, kern)
        if not v:
            raise SystemExit(f"no {ctr} for {kern}")
        kb = statistics.mean(v)
        res[kern] = {"counter": ctr, "dispatches": len(v), "reported_kb_avg": round(kb, 1),
                     "factor": round(CALIB_BYTES / (kb * 1024.0), 4)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    return res


def pmc(fetch_db, write_db, substr, out, alg_bytes=None, clients=1, calib_path=None):
    f = pmc_values(fetch_db, "FETCH_SIZE", substr)
    w = pmc_values(write_db, "WRITE_SIZE", substr)
    if not f or not w:
        raise SystemExit(f"no dispatches of {substr!r} with FETCH_SIZE/WRITE_SIZE")
    fetch_kb, write_kb = statistics.mean(f), statistics.mean(w)
    rf, wf = 2.0, 1.0
    corr = ("MI355X_MICROARCH.md §HBM: FETCH_SIZE x2 (gfx950 half-count of 16 B/lane streaming "
            "reads); WRITE_SIZE as reported")
    if calib_path:
        cal = json.load(open(calib_path))
        rf, wf = cal["k_read4_nt"]["factor"], cal["k_write16"]["factor"]
        corr = (f"calibrated on known 512 MiB dispatches of the same access shapes ({calib_path}): "
                f"FETCH_SIZE x {rf} (4 B/lane non-temporal reads), WRITE_SIZE x {wf} "
                "(16 B/lane stores)")
    hbm = rf * fetch_kb * 1024 + wf * write_kb * 1024
    res = {"kernel": substr, "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_size_kb_avg": round(fetch_kb, 1), "write_size_kb_avg": round(write_kb, 1),
           "hbm_read_bytes_per_launch": int(rf * fetch_kb * 1024),
           "hbm_write_bytes_per_launch": int(wf * write_kb * 1024),
           "hbm_bytes_per_launch": int(hbm), "clients_per_launch": clients,
           "correction": corr}
    if alg_bytes:
        res["alg_bytes_per_launch"] = int(alg_bytes)
        res["traffic_over_alg"] = round(hbm / alg_bytes, 4)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    return res


def counters(db, substr):
    """Average of every collected counter over the dispatches of one kernel (name substring)."""
    c = sqlite3.connect(db)
    per = {}
    for name, ctr, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        if substr in name:
            per.setdefault(ctr, []).append(float(v))
    return {k: {"avg": statistics.mean(v), "dispatches": len(v)} for k, v in sorted(per.items())}


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
    p.add_argument("--calib", default=None)
    k = sub.add_parser("counters")
    k.add_argument("db")
    k.add_argument("kernel")
    t = sub.add_parser("timeline")
    t.add_argument("db")
    t.add_argument("last", type=int, nargs="?", default=60)
    c = sub.add_parser("calib")
    c.add_argument("fetch_db")
    c.add_argument("write_db")
    c.add_argument("out")
    a = ap.parse_args()
    if a.cmd == "stats":
        for name, d in stats(a.db, a.out)[:12]:
            print(f"{len(d):7d} {sum(d) / len(d) / 1e3:10.2f} us  {name[:100]}")
    elif a.cmd == "timeline":
        timeline(a.db, a.last)
    elif a.cmd == "counters":
        print(json.dumps(counters(a.db, a.kernel), indent=1))
    elif a.cmd == "calib":
        print(json.dumps(calib(a.fetch_db, a.write_db, a.out), indent=1))
    else:
        print(json.dumps(pmc(a.fetch_db, a.write_db, a.kernel, a.out, a.alg_bytes,
                             a.clients_per_launch, a.calib), indent=1))


if __name__ == "__main__":
    main()
