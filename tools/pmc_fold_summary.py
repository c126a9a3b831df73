"""Merge tools/pmc_fold.sh's counter passes into one profiles/ JSON with derived figures.

    python tools/pmc_fold_summary.py gpurun_out/<tag> profiles/<round>_pmc_k_fold_q.json \
        [--entries-per-packet 13421773] [--packets 128]

Derived: the split of wave cycles (issuing / issue-stalled / waiting), LDS bank-conflict share
of LDS cycles, VALU lane-ops per folded entry and HBM read bytes (FETCH_SIZE x 2 for 4 B/lane
reads, the calibration in profiles/r02_pmc_calib.json)."""
import argparse
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("out")
    ap.add_argument("--entries-per-packet", type=float, default=13_421_773)
    ap.add_argument("--packets", type=int, default=128)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    c = {}
    for part in ("sq", "fetch", "ta"):
        p = os.path.join(a.src, part + ".json")
        if os.path.exists(p):
            for k, v in json.load(open(p)).items():
                c[k] = v["avg"]
    d = {}
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        act, wait = c.get("SQ_ACTIVE_INST_ANY", 0.0), c.get("SQ_WAIT_ANY", 0.0)
        d["wave_cycles_split"] = {"active_inst": round(act / wc, 3),
                                  "issue_stall": round(max(0.0, 1 - act / wc - wait / wc), 3),
                                  "waitcnt_or_barrier": round(wait / wc, 3)}
    if c.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_share_of_lds_cycles"] = round(
            c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 3)
    entries = a.entries_per_packet * a.packets
    if c.get("SQ_INSTS_VALU"):
        d["valu_lane_ops_per_folded_entry"] = round(c["SQ_INSTS_VALU"] * 64 / entries, 1)
    if c.get("SQ_INSTS_LDS"):
        d["lds_wave_instructions_per_64_entries"] = round(c["SQ_INSTS_LDS"] * 64 / entries, 2)
    if c.get("FETCH_SIZE"):
        d["hbm_read_bytes"] = int(c["FETCH_SIZE"] * 1024 * 2)
        d["hbm_read_note"] = ("FETCH_SIZE (KiB) x 2 (profiles/r02_pmc_calib.json, 4 B/lane reads); "
                              f"{a.packets} x 6 B x entries = "
                              f"{6 * entries / 1e9:.2f} GB expected")
    rec = {"kernel": f"k_fold_q<false>, {a.packets} packets x 134,217,728 (tools/kbench.py --dec "
                     f"{a.packets}), per launch", "counters": c, "derived": d,
           "source": "tools/pmc_fold.sh (one --pmc pass per counter group, averaged over the "
                     "k_fold_q dispatches)"}
    if a.note:
        rec["note"] = a.note
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec["derived"], indent=1))


if __name__ == "__main__":
    main()
