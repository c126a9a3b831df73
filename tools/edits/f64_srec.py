# A/B: k_fused64's later chunk workgroups (chunk >= 1024) read the bracket record with a scalar
# load issued before their gradient loads, as k_fused_mag<false>'s do since round 6.
edits = [
    ("fc_f64.hip", """  if (chunk < 1024u) __builtin_amdgcn_s_sleep(FC_F64_DELAY);   // the sample's loads first
  load64_chunk(a, chunk, x);
  if (threadIdx.x == 0) {
    const uint32_t* rec = &W.pub[(blockIdx.x % kPubCopies) * kPubStride];
    const uint32_t tag = pub | 0x80000000u;
    uint32_t it = 0;""", """  if (chunk < 1024u) __builtin_amdgcn_s_sleep(FC_F64_DELAY);   // the sample's loads first
  const uint32_t* rec = &W.pub[(blockIdx.x % kPubCopies) * kPubStride];
  const uint32_t tag = pub | 0x80000000u;
  typedef __attribute__((address_space(4))) const fc_rec4 fc_crec4;
  const bool try_s = chunk >= 1024u;
  fc_rec4 sr = {0u, 0u, 0u, 0u};
  if (try_s) sr = *(fc_crec4*)rec;
  load64_chunk(a, chunk, x);
  if (try_s && sr.w == tag) {
    compact64_body(a, chunk, x, sr.x, sr.y, sr.z, u.c);
    return;
  }
  if (threadIdx.x == 0) {
    uint32_t it = 0;"""),
]
