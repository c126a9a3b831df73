# A/B: k_compact_mag1 bins its candidates into the client's candidate histogram (one device
# atomic each, as k_fused_mag does), so a batched magnitude encode's k_resolve<false> follows
# alone (no k_resolve<true> binning launch).
edits = [
    ("fc_topk.hip", "  compact_mag_item<NW, MagShared, DENSE, false, true, NTS>(a0, mag_out(a0, client), chunk, st, x, sh);",
     "  compact_mag_item<NW, MagShared, DENSE, !DENSE, true, NTS>(a0, mag_out(a0, client), chunk, st, x, sh);"),
    ("fc_capi.hip", """  const bool bin = key_mode == FC_KEY_PHILOX;   // rand-k bins its candidates while it compacts
  rc = launch_compact_key(key_mode, ca, s, 1, bin);
  if (rc) return rc;
  ra.rbin = bin ? 0 : 1;             // else the unfused compaction leaves the binning to k_resolve""",
     """  rc = launch_compact_key(key_mode, ca, s, 1, true);
  if (rc) return rc;
  ra.rbin = 0;                       // both compactions bin their candidates"""),
    ("fc_capi.hip", "  ra.rbin = 1;                       // batched compaction: k_resolve bins the candidates",
     "  ra.rbin = key_mode == FC_KEY_PHILOX ? 1 : 0;   // k_compact_mag1 bins, batched rand-k does not"),
]
