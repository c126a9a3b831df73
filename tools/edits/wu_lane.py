# A/B: goff_of's lane index from a wave-uniform SGPR (w read once with readfirstlane) instead of
# a VGPR that hipcc re-read with v_readfirstlane (+ s_nop hazards) for every 64-element group.
edits = [
    ("fc_topk.hip", "    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + w);",
     "    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + wu);"),
    ("fc_topk.hip", "  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;\n  const uint32_t base = chunk * (uint32_t)kChunk;\n  const uint32_t lbase",
     "  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;\n  const int wu = __builtin_amdgcn_readfirstlane(w);     // uniform: the readlane index below\n  const uint32_t base = chunk * (uint32_t)kChunk;\n  const uint32_t lbase"),
    ("fc_pred.hip", "    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + w);",
     "    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + wu);"),
    ("fc_pred.hip", "  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;",
     "  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;\n  const int wu = __builtin_amdgcn_readfirstlane(w);     // uniform: the readlane index below"),
]
