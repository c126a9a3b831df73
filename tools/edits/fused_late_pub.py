# A/B: k_fused_mag's chunk workgroups read fz_seq (their bracket tag) after issuing their
# gradient loads instead of before (the scalar load's wait no longer precedes the vector loads).
edits = [
    ("fc_topk.hip", """  TopkState* S = a0.W.st;
  const uint32_t pub = sload2(&S->fz_seq).x + 1u;   // not written by this launch
  if (blockIdx.x < nsamp) {
    if (threadIdx.x >= kBlock) return;""", """  TopkState* S = a0.W.st;
  if (blockIdx.x < nsamp) {
    if (threadIdx.x >= kBlock) return;
    const uint32_t pub = sload2(&S->fz_seq).x + 1u;   // not written by this launch"""),
    ("fc_topk.hip", """  const uint32_t* rec = &a0.W.pub[(blockIdx.x % kPubCopies) * kPubStride];
  const uint32_t tag = pub | 0x80000000u;
  typedef __attribute__((address_space(4))) const fc_rec4 fc_crec4;
  const bool try_s = !DENSE && chunk >= (uint32_t)FC_FUSED_SREC;
  fc_rec4 sr = {0u, 0u, 0u, 0u};
  if (try_s) sr = *(fc_crec4*)rec;
  mag_load<NW>(a0.g, chunk, a0.n, x);""", """  const uint32_t* rec = &a0.W.pub[(blockIdx.x % kPubCopies) * kPubStride];
  typedef __attribute__((address_space(4))) const fc_rec4 fc_crec4;
  const bool try_s = !DENSE && chunk >= (uint32_t)FC_FUSED_SREC;
  fc_rec4 sr = {0u, 0u, 0u, 0u};
  if (try_s) sr = *(fc_crec4*)rec;
  mag_load<NW>(a0.g, chunk, a0.n, x);
  const uint32_t tag = (sload2(&S->fz_seq).x + 1u) | 0x80000000u;   // after the loads issue"""),
]
