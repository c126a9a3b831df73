"""Every kernel and memory copy of a rocprofv3 database in start order (the last N), with gaps:
    python tools/timeline_all.py <db> [N]"""
import sqlite3
import sys


def main():
    db, last = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = sqlite3.connect(db)
    rows = []
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    for tab, kind in (("kernels", "K"), ("memory_copies", "M")):
        if tab not in tabs:
            continue
        cols = [r[1] for r in c.execute(f"pragma table_info({tab})")]
        st = next(x for x in ("start", "start_ns", "begin") if x in cols)
        en = next(x for x in ("end", "end_ns") if x in cols)
        nm = next((x for x in ("name", "kernel_name", "operation") if x in cols), None)
        q = f"select {nm if nm else repr(tab)}, {st}, {en} from {tab}"
        for r in c.execute(q).fetchall():
            rows.append((r[1], r[2], kind, str(r[0])))
    rows.sort()
    rows = rows[-last:]
    t0 = rows[0][0]
    prev_end = None
    for s, e, kind, name in rows:
        gap = "" if prev_end is None else f"{(s - prev_end) / 1e3:8.1f}"
        print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} {gap:>8} {kind} {name[:80]}")
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main()
