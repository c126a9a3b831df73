# A/B: the scalar bracket-record load issued right AFTER the gradient loads (it has its own
# counter, so it still does not wait behind them) and enabled for the dense form too (fewer
# SGPRs live across the load issue).
edits = [
    ("fc_topk.hip", """  const bool try_s = !DENSE && chunk >= (uint32_t)FC_FUSED_SREC;
  fc_rec4 sr = {0u, 0u, 0u, 0u};
  if (try_s) sr = *(fc_crec4*)rec;
  mag_load<NW>(a0.g, chunk, a0.n, x);""", """  const bool try_s = chunk >= (uint32_t)FC_FUSED_SREC;
  fc_rec4 sr = {0u, 0u, 0u, 0u};
  mag_load<NW>(a0.g, chunk, a0.n, x);
  if (try_s) sr = *(fc_crec4*)rec;"""),
]
