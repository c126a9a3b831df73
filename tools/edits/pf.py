# k_fused_mag: a chunk workgroup of the first resident round prefetches the chunk(s) the same
# slot (same XCD: chunk + 1024 j keeps bid % 8) will process next, into L2, while it waits for
# the bracket; the loaded value is kept live past the wait (no hazard on its VGPR)
import os
PF = int(os.environ.get("PF_ROUNDS", "1"))
edits = [
    ("fc_topk.hip", """  mag_load<NW>(a0.g, chunk, a0.n, x);
  FC_TR(24);""", f"""  mag_load<NW>(a0.g, chunk, a0.n, x);
  float pf[{PF}];
#pragma unroll
  for (int j = 0; j < {PF}; ++j) {{
    pf[j] = 0.f;
    const uint64_t e2 = (uint64_t)(chunk + 1024u * (j + 1)) * kChunk + threadIdx.x * 32u;
    if (chunk < 1024u && threadIdx.x < kChunk / 32 && e2 < a0.n)
      pf[j] = ((__attribute__((address_space(1))) const float*)a0.g)[e2];
  }}
  FC_TR(24);"""),
    ("fc_topk.hip", """  __syncthreads();
  FC_TR(25);""", f"""  __syncthreads();
#pragma unroll
  for (int j = 0; j < {PF}; ++j) asm volatile("" :: "v"(pf[j]));
  FC_TR(25);"""),
]
