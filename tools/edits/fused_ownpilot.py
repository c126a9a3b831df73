# A/B: every sample workgroup of k_fused_mag computes the pilot window itself (loads the pilot
# segments, L2-resident after the first reader) instead of polling workgroup 0's published copy.
edits = [
    ("fc_topk.hip", "sample_body<kKeyMag, true>(a0.g, P, 0ull, 0ull, a0.W, a0.ib, a0.hdr, HI, blockIdx.x, nsamp, true, u.s, pub);",
     "sample_body<kKeyMag, false>(a0.g, P, 0ull, 0ull, a0.W, a0.ib, a0.hdr, HI, blockIdx.x, nsamp, false, u.s, pub);"),
]
