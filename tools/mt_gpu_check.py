import sys, time, numpy as np, torch
sys.path.insert(0, "/root/repo")
from openmsftl_amd import codec
from openmsftl_amd.compression import bitmask_words
for n, ps, seed, pre in [(100_003, [0.1, 0.7, 0.5], 3, 5), (1000, [0.3], 1, 0), (25_557_032, [0.1, 0.9], 11, 1),
                         (31, [0.5, 0.5, 0.0, 1.0], 2, 623)]:
    np.random.seed(seed); np.random.random_sample(pre)
    key, pos, hg, ga = codec.mt_state()
    want = [bitmask_words(np.random.binomial(1, p, (n,)), n, True) for p in ps]
    st_want = np.random.get_state()
    torch.cuda.synchronize(); t = time.time()
    R = codec.MtRound(n, len(ps), key, pos)
    got = [R.binomial(r, p).cpu().numpy().view(np.uint32) for r, p in enumerate(ps)]
    k2, p2, rd = R.end_state(); dt = time.time() - t
    ok = all((g == w).all() for g, w in zip(got, want))
    print(n, ps, "masks", ok, "state", (k2 == st_want[1]).all() and p2 == st_want[2], "redraw", rd, f"{dt*1e3:.1f} ms")
    if not ok:
        for g, w in zip(got, want):
            bad = np.nonzero(g != w)[0]
            print("  first bad word", bad[:5], len(bad))
n = 25_557_032
np.random.seed(0)
key, pos, hg, ga = codec.mt_state()
R = codec.MtRound(n, 8, key, pos)
out = torch.empty((n + 31)//32, dtype=torch.int32, device="cuda")
for r in range(8): R.binomial(r, 0.1, out)
torch.cuda.synchronize()
t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
t0.record()
R = codec.MtRound(n, 8, key, pos)
t1.record(); torch.cuda.synchronize(); print("begin 8 rows", t0.elapsed_time(t1), "ms")
t0.record()
for r in range(8): R.binomial(r, 0.1, out)
t1.record(); torch.cuda.synchronize(); print("per row 25.5M", t0.elapsed_time(t1)/8, "ms")
