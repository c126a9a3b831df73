# A/B: k_fused64's sample workgroups compute the pilot window themselves (as k_fused_mag's do
# since round 6) instead of polling workgroup 0's published copy.
edits = [
    ("fc_f64.hip", """    sample_body<kKeyMag, true, double>(a.g, P, 0ull, 0ull, W, ib, hdr, HI, blockIdx.x, nsamp,
                                       true, u.s, pub);""", """    sample_body<kKeyMag, false, double>(a.g, P, 0ull, 0ull, W, ib, hdr, HI, blockIdx.x, nsamp,
                                        false, u.s, pub);"""),
]
