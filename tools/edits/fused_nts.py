# A/B: the lone fused packet encode writes its entries / candidates with non-temporal stores
edits = [("fc_topk.hip",
          "compact_mag_item<NW, MagShared, DENSE, true, !DENSE>(a0, mag_out(a0, 0u), chunk, st, x, u.m);",
          "compact_mag_item<NW, MagShared, DENSE, true, !DENSE, true>(a0, mag_out(a0, 0u), chunk, st, x, u.m);")]
