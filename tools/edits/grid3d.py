# k_compact_mag1: grid (clients per interleave group, chunks, groups) instead of a linear id
# divided by (chunks x group size) at every workgroup's start
edits = [
    ("fc_topk.hip", """__device__ __forceinline__ void mag_item_of(uint32_t& client, uint32_t& chunk) {
  if (FC_MAG1_IL == 1) {""", """__device__ __forceinline__ void mag_item_of(uint32_t& client, uint32_t& chunk) {
  if (gridDim.z > 1 || gridDim.x <= (uint32_t)FC_MAG1_IL) {   // 3-D grid
    client = blockIdx.z * gridDim.x + blockIdx.x; chunk = blockIdx.y;
    return;
  }
  if (FC_MAG1_IL == 1) {"""),
    ("fc_topk.hip", """  uint32_t client, chunk;
  mag_item_of(client, chunk);
  float x[MagGeo<NW>::kQ];""", """  uint32_t client, chunk;
  mag_item_of(client, chunk);
  if (client >= a0.ws_stride_clients) return;
  float x[MagGeo<NW>::kQ];"""),
    ("fc_topk.hip", """  const fc_encode_job* jobs;   // batched encode: client blockIdx.y overrides g / packet / W
  uint64_t ws_stride;
  float* dense;             // fc_topk_encode_dense: also stream q = listed ? g : +0 (one client)
};""", """  const fc_encode_job* jobs;   // batched encode: client blockIdx.y overrides g / packet / W
  uint64_t ws_stride;
  float* dense;             // fc_topk_encode_dense: also stream q = listed ? g : +0 (one client)
  uint32_t ws_stride_clients;
};"""),
    ("fc_capi.hip", """  hipLaunchKernelGGL(k_compact_mag1, dim3(a.nchunks, m), dim3(kCBlock), 0, s, a);""",
     """  CompactArgs b = a;
  b.ws_stride_clients = m;
  const uint32_t il = m < (uint32_t)FC_MAG1_IL ? m : (uint32_t)FC_MAG1_IL;
  hipLaunchKernelGGL(k_compact_mag1, dim3(il, a.nchunks, (m + il - 1) / il), dim3(kCBlock), 0, s, b);"""),
]
