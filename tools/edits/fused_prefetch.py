# A/B: the first resident round of k_fused_mag's chunk workgroups, while it waits for the
# bracket, touches the chunks the next FC_FUSED_PF rounds will read (one dword per 64 B: the
# lines land in the Infinity Cache), so the HBM is not idle during the bracket wait.
edits = [
    ("fc_topk.hip", """  mag_load<NW>(a0.g, chunk, a0.n, x);
  FC_TR(24);""", """  mag_load<NW>(a0.g, chunk, a0.n, x);
  uint32_t pf = 0;
  if (chunk < 1024u) {
    const uint32_t nch = (uint32_t)((a0.n + kChunk - 1) / kChunk);
#pragma unroll
    for (int j = 1; j <= FC_FUSED_PF; ++j) {
      const uint32_t c2 = chunk + 1024u * (uint32_t)j;
      if (c2 + 1u < nch)
        pf ^= ((const FC_G uint32_t*)a0.g)[(uint64_t)c2 * kChunk + threadIdx.x * 16u];
    }
  }
  FC_TR(24);"""),
    ("fc_topk.hip", """  __syncthreads();
  FC_TR(25);""", """  __syncthreads();
  asm volatile("" :: "v"(pf));
  FC_TR(25);"""),
    ("fc_topk.hip", """constexpr int FC_MAG1_IL = 64;""", """constexpr int FC_MAG1_IL = 64;
constexpr int FC_FUSED_PF = 1;"""),
]
