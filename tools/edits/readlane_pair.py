# A/B: the staged phase-2 loop reads each pair of groups' slot offsets with ONE readlane (the two
# 16-bit offsets share a word), issued before both groups' branches (hipcc re-read the word per
# group: a convergent readlane is not CSE'd across the if (p) blocks).
edits = [
    ("fc_topk.hip", """  } else if (tot_e <= (uint32_t)SH::kStageN) {          // block-uniform
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool p = mag_listed<FAST>(P, x[q]);
      const uint32_t pos = prefix_count(__ballot(p)) + goff_of(q);
      if (p) sh.st[pos] = make_uint2(FC_LOC(q), __float_as_uint(FAST ? x[q] : a.g[base + FC_LOC(q)]));
      dense_out(q, p);
    }
  } else {""", """  } else if (tot_e <= (uint32_t)SH::kStageN) {          // block-uniform
#pragma unroll
    for (int q = 0; q < NQ; q += 2) {
      const uint32_t gw = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + wu);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool p = mag_listed<FAST>(P, x[q + h]);
        const uint32_t pos = prefix_count(__ballot(p)) + (h ? gw >> 16 : gw & 0xffffu);
        if (p) sh.st[pos] = make_uint2(FC_LOC(q + h), __float_as_uint(FAST ? x[q + h] : a.g[base + FC_LOC(q + h)]));
        dense_out(q + h, p);
      }
    }
  } else {"""),
]
