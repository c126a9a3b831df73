import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from openmsftl_amd import codec
from openmsftl_amd.compression import bitmask_words
n = 2000
for p in (0.3, 0.5):
    np.random.seed(1)
    key, pos, _, _ = codec.mt_state()
    want = np.random.binomial(1, p, (n,)).astype(np.uint8)
    R = codec.MtRound(n, 1, key, pos)
    got_w = R.binomial(0, p).cpu().numpy().view(np.uint32)
    got = np.unpackbits(got_w.view(np.uint8), bitorder="little")[:n]
    bad = np.nonzero(got != want)[0]
    print("p", p, "pos", pos, "bad", len(bad), "first", bad[:40].tolist())
    print("  bad mod 312:", sorted(set((bad % 312).tolist()))[:60])
