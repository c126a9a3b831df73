# A/B: k_fused_mag's sample workgroups compute the pilot window themselves when the pilot is
# two segments (n <= 32 M: P.segs == 2); above, they poll workgroup 0's published copy.
edits = [
    ("fc_topk.hip", "sample_body<kKeyMag, true>(a0.g, P, 0ull, 0ull, a0.W, a0.ib, a0.hdr, HI, blockIdx.x, nsamp, true, u.s, pub);",
     "sample_body<kKeyMag, false>(a0.g, P, 0ull, 0ull, a0.W, a0.ib, a0.hdr, HI, blockIdx.x, nsamp, P.segs > 2u, u.s, pub);"),
]
