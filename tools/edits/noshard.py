# timing only (wrong totals): the compaction's per-chunk shard-total atomics removed
edits = [
    ("fc_topk.hip", "    atomicAdd(&S->shard_ent[chunk % kShards], tot_e);\n    if (tot_c) atomicAdd(&S->shard_cnd[chunk % kShards], tot_c);",
     "    (void)S;"),
]
