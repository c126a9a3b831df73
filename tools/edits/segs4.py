# A/B: four sample segments per workgroup at every n (two up to 32 M before): half as many sample
# workgroups at 16 M (fewer flushes and ticket levels, twice the keys each), now that each one
# also ranks the pilot itself.
edits = [("fc_capi.hip", "  P.segs = n <= (32ull << 20) ? 2u : (uint32_t)kSampleSegs;", "  P.segs = (uint32_t)kSampleSegs;")]
