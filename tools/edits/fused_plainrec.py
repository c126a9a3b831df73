# timing-only A/B: chunk workgroups past the first two resident rounds read the bracket record
# with one plain (cacheable) load instead of the sc1 poll (tests what the sc1 round trip costs;
# not correct in general: an XCD's L2 may hold a stale record)
edits = [
    ("fc_topk.hip", """    fc_rec4 r = ld16_agent(rec);
    while (r.w != tag && ++it < kSpinMax) {""", """    fc_rec4 r;
    if (chunk >= 2048u) r = *reinterpret_cast<const fc_rec4*>(rec);
    else r = ld16_agent(rec);
    while (r.w != tag && ++it < kSpinMax) {"""),
]
