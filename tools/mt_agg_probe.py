"""Where does a device-MT dropout round's time go?  Aggregator rates at 25.5 M (NumPy in/out):
'full', 'dropout-unbiased' (device MT draws), the same with the mask kernel replaced by a
precomputed mask (timing only), and the mask kernel alone."""
import sys, time, numpy as np, torch
sys.path.insert(0, "/root/repo")
from openmsftl_amd import Compression, codec
from openmsftl_amd.aggregation import Aggregator
n, M = 25_557_032, 32
rng = np.random.default_rng(0)
grads = [rng.standard_normal(n, dtype=np.float32) for _ in range(M)]
class Cl:
    def __init__(s, i, g, C): s.client_id, s.grad, s.C = i, g, C
def rate(cfg, reps=3):
    agg = Aggregator({"aggregation_scheme": "fed_avg"})
    C = Compression(cfg)
    best = 1e9
    for _ in range(reps):
        np.random.seed(1)
        t = time.perf_counter()
        agg.aggregate_grads([Cl(i, g, C) for i, g in enumerate(grads)])
        best = min(best, time.perf_counter() - t)
    return 4.0 * n * M / best / 1e9, best
print("full", rate({"compression_function": "full"}))
print("dropout-unbiased MT", rate({"compression_function": "dropout-unbiased", "dropout_p": 0.1}))
real = codec.MtRound.binomial
fixed = {}
def fake(self, row, p, out=None):
    if out is None:
        out = torch.empty((self.n + 31) // 32, dtype=torch.int32, device=self.dev)
    out.fill_(0x5555)
    self._mark()
    return out
codec.MtRound.binomial = fake
print("dropout-unbiased fake-mask", rate({"compression_function": "dropout-unbiased", "dropout_p": 0.1}))
codec.MtRound.binomial = real
np.random.seed(1)
key, pos, _, _ = codec.mt_state()
torch.cuda.synchronize()
t = time.perf_counter()
R = codec.MtRound(n, M, key, pos)
torch.cuda.synchronize()
t1 = time.perf_counter()
for r in range(M):
    R.binomial(r, 0.1)
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"begin {1e3*(t1-t):.2f} ms, {M} rows {1e3*(t2-t1):.2f} ms = {1e3*(t2-t1)/M:.3f} ms/row")
