# A/B (timing): the batched compaction takes client c's gradient pointer as g_slab + c * g_stride
# (rows of one slab) instead of loading it from the job table before its gradient loads; the
# hint comes from FC_AB_SLAB="base,stride" (bench.py sets it for its slab).
edits = [
    ("fc_topk.hip", """  uint32_t grid3;           // k_compact_mag1(_dense): 3-D grid (clients of a group, chunks, groups)
  uint32_t m;               // its clients (the last group may be partial)
};""", """  uint32_t grid3;           // k_compact_mag1(_dense): 3-D grid (clients of a group, chunks, groups)
  uint32_t m;               // its clients (the last group may be partial)
  const float* g_slab;
  uint64_t g_stride;
};"""),
    ("fc_topk.hip", """__device__ __forceinline__ const float* mag_g(const CompactArgs& a0, uint32_t client) {
  if (!a0.jobs) return a0.g;""", """__device__ __forceinline__ const float* mag_g(const CompactArgs& a0, uint32_t client) {
  if (!a0.jobs) return a0.g;
  if (a0.g_slab) return a0.g_slab + (uint64_t)client * a0.g_stride;"""),
    ("fc_capi.hip", """  ca.jobs = jobs; ca.ws_stride = stride;
  ResolveArgs ra;""", """  ca.jobs = jobs; ca.ws_stride = stride;
  if (const char* e = getenv("FC_AB_SLAB")) {
    unsigned long long b = 0, st = 0;
    if (sscanf(e, "%llu,%llu", &b, &st) == 2) { ca.g_slab = (const float*)(uintptr_t)b; ca.g_stride = st; }
  }
  ResolveArgs ra;"""),
]
