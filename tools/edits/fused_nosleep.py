# A/B: no start delay for the fused launch's first round of chunk loads
edits = [("fc_topk.hip", "  if (chunk < 1024u) __builtin_amdgcn_s_sleep(90);\n", "")]
