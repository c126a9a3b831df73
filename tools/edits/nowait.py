# timing only: k_fused_mag's chunk workgroups do not wait for this launch's bracket (they use
# whichever record they read first: the previous call's bracket when the same gradient is
# re-encoded) -- the floor of the fused form (profiles/r05_ab_fused_noshard_nowait.jsonl)
edits = [
    ("fc_topk.hip", """    fc_rec4 r = ld16_agent(rec);
    while (r.w != tag && ++it < kSpinMax) {
      __builtin_amdgcn_s_sleep(4);
      r = ld16_agent(rec);
    }
    if (it >= kSpinMax) st_agent(&S->err, 1u);
    MagState m;""", """    fc_rec4 r = ld16_agent(rec);
    (void)tag; (void)it;
    MagState m;"""),
]
