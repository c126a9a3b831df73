# lone packet encode: no in-kernel candidate binning (k_resolve<true> bins them instead)
edits = [
    ("fc_topk.hip", "compact_mag_item<NW, MagShared, DENSE, true, !DENSE>(a0, mag_out(a0, 0u), chunk, st, x, u.m);",
     "compact_mag_item<NW, MagShared, DENSE, DENSE, !DENSE>(a0, mag_out(a0, 0u), chunk, st, x, u.m);"),
    ("fc_capi.hip", "    ra.rbin = 0;                     // k_fused_mag binned the candidates\n    return launch_resolve(ra, s);",
     "    ra.rbin = 1;\n    return launch_resolve(ra, s);"),
]
