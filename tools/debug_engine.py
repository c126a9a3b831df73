"""Debug helper: dump the encoder state after 1..6 engine passes for one input."""
import os, sys, struct
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openmsftl_amd import codec, _lib

FIELDS = ("err a_done b_done b1_hi b1_lo rr_hi rr_lo hi_none lo_all t_lo t_hi cand_on n_hi n_cand "
          "cand_over ent_over e_shift e_rank e_matched e_done e_src e_ticket e_small_n e_status").split()

def state(ws):
    raw = ws.buf[:256].cpu().numpy().tobytes()
    t, L64, pre = struct.unpack_from("<QQQ", raw, 0)
    vals = struct.unpack_from("<%dI" % len(FIELDS), raw, 24)
    d = dict(zip(FIELDS, vals)); d.update(ticket=hex(t), L64=hex(L64), e_prefix=hex(pre))
    return d

def run(g, k, passes):
    os.environ["FC_DEBUG_ENGINE_PASSES"] = str(passes)
    gt = torch.from_numpy(g).cuda()
    pkt = codec.encode_top(gt, k, check=False)
    torch.cuda.synchronize()
    ws = codec.Workspace.get(g.size, gt.device)
    h = pkt.header()
    return state(ws), h

if __name__ == "__main__":
    n, k = 70001, 7000
    g = np.full(n, 0.5, np.float32)
    for p in range(1, 7):
        st, h = run(g, k, p)
        print(p, {kk: st[kk] for kk in ("n_hi","n_cand","cand_over","e_shift","e_rank","e_matched","e_done","e_src","e_status","e_prefix","t_lo","t_hi","err")},
              "hdr:", h.status, h.n_entries, hex(h.thresh), flush=True)
