import sys, os, json
sys.path.insert(0, os.getcwd())
import torch
from openmsftl_amd import _lib as L, codec
from openmsftl_amd.compression import kept_count
dev = torch.device("cuda", 0)
n = 134217728; k = kept_count(0.1, n)
import numpy as np
srng = np.random.default_rng(7)
scales = 10.0 ** srng.uniform(-4, -1, size=8)
grads = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1000 + i)).mul_(float(scales[i])) for i in range(8)]
pk = codec.encode_top_batch(grads, k)
for p in pk:
    h = p.header()
    print(json.dumps({"k": k, "n_entries": h.n_entries, "slack": round(h.n_entries / k - 1, 5), "n_cand": h.n_cand, "n_definite": h.n_definite}))
