edits = [("fc_topk.hip", "  if (chunk < 1024u) __builtin_amdgcn_s_sleep(90);", "  if (chunk < 1024u) __builtin_amdgcn_s_sleep(45);")]
