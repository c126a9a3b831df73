# timing only: k_fused_mag's chunk workgroups do not wait for this launch's bracket (they read
# whatever state is there: the previous call's bracket when the same gradient is re-encoded)
edits = [
    ("fc_topk.hip", "    while (ld_agent(&S->fz_pub) != pub && ++it < kSpinMax) __builtin_amdgcn_s_sleep(4);",
     "    (void)pub;"),
]
