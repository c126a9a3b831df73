# A/B: the candidate loop of compact_mag_body skips the prefix count and the per-lane work of a
# 64-element group with no candidate (wave-uniform branch on its ballot; ~85 % of groups at
# f = 0.1 hold none).
edits = [
    ("fc_topk.hip", """    for (int q = 0; q < NQ; ++q) {
      const bool c = mag_cand<FAST>(P, x[q]);
      const uint64_t mc = __ballot(c);
      const uint32_t pos = wc + prefix_count(mc);
      if (c) {
        const uint32_t e = base + FC_LOC(q);
        const uint32_t key = mag_key(FAST ? x[q] : a.g[e]);
        if (pos < (uint32_t)kCW) sh.cst[w * kCW + pos] = comp_of(key, e, a.ib);
        if (BIN) {
          const uint32_t bin = (key - P.t_lo) >> sbin;
          if (pos < (uint32_t)kCW) sh.cstb[w * kCW + pos] = (uint16_t)bin;
          else atomicAdd(&a.chist[bin], 1u);
        }
      }
      wc += (uint32_t)__popcll(mc);
    }""", """    for (int q = 0; q < NQ; ++q) {
      const bool c = mag_cand<FAST>(P, x[q]);
      const uint64_t mc = __ballot(c);
      if (mc == 0) continue;                            // uniform: no candidate in the group
      const uint32_t pos = wc + prefix_count(mc);
      if (c) {
        const uint32_t e = base + FC_LOC(q);
        const uint32_t key = mag_key(FAST ? x[q] : a.g[e]);
        if (pos < (uint32_t)kCW) sh.cst[w * kCW + pos] = comp_of(key, e, a.ib);
        if (BIN) {
          const uint32_t bin = (key - P.t_lo) >> sbin;
          if (pos < (uint32_t)kCW) sh.cstb[w * kCW + pos] = (uint16_t)bin;
          else atomicAdd(&a.chist[bin], 1u);
        }
      }
      wc += (uint32_t)__popcll(mc);
    }"""),
]
