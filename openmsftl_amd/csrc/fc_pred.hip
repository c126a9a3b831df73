// fc_pred.hip — ballot-layout compaction for the predicates that are not |g| compares:
//   kSrcPhiloxKey  native rand-k (compression.py:39-45 with device keys): comp = key << IB | idx,
//                  key = Philox word >> 1; listed comp >= L64, candidates key in [t_lo, t_hi]
//   kSrcMaskBits   a host-drawn keep mask (rand parity mode's permutation, dropout's binomial)
//   kSrcBern       native dropout: keep iff Philox word < round(p * 2^32)
// (the mask codecs list a dropped inf / NaN as NaN: g * 0 = NaN, compression.py:52,59).
//
// Same geometry as k_compact_mag1 (one 512-thread workgroup per 8192-element chunk, element
// base + i*2048 + w*256 + j*64 + lane), so a group of 64 consecutive elements is one ballot,
// its count one scalar popcount, and a bitmap packet's two words ARE that ballot.  The Philox
// element map (fc_common.h) gives lane L of segment (i, w) one counter block whose four words
// are its groups j = 0..3: one Philox evaluation per 4 elements, no redundant rounds.  (The
// float4-layout kernel this replaces spent ~12 VALU per element on bit assembly and ran the
// mask encodes at 0.33-0.44 of the HBM roofline, rand-k at 0.21.)
//
// Native rand-k needs no sample: the keys are uniform, so the host places the bracket around
// the k-th key analytically (fc_capi.hip philox_bracket: +-8 binomial sigmas); k_setup_bracket
// writes it into the encoder state and zeroes the totals, the compaction lists and stages
// candidates, k_resolve bins them and picks T64 exactly (a bracket that misses -> RETRY).
#include "fc_state.h"

namespace fc {

enum PredSrc : int { kSrcPhiloxKey = 0, kSrcMaskBits = 1, kSrcBern = 2 };

struct PredShared {
  uint32_t gcnt[kMGroups / 4];                     // 4 group counts (bytes) per (i, w)
  uint32_t wcnt[8];                                // candidates per wave
  uint2 st[kStage + 4];                            // packed {chunk-local index, value bits}
  uint64_t cst[kCandSlot];                         // candidate comps, wave w at w * kCW
};

// Per-client bracket of an analytical (Philox-key) encode: state + static header.
struct SetupArgs {
  WsPtrs W;
  fc_packet_hdr* hdr;
  HdrInit HI;
  const fc_encode_job* jobs;       // batched: client blockIdx.x
  uint64_t ws_stride;
  uint32_t t_lo, t_hi, sbin, ib;
};

__global__ __launch_bounds__(64) void k_setup_bracket(SetupArgs a) {
  WsPtrs W = a.W;
  fc_packet_hdr* hdr = a.hdr;
  HdrInit HI = a.HI;
  if (a.jobs) {
    const fc_encode_job& J = a.jobs[blockIdx.x];
    hdr = J.hdr; HI.seed = J.seed; HI.offset = J.offset;
    W = ws_shift(W, (uint64_t)blockIdx.x * a.ws_stride);
  }
  TopkState* S = W.st;
  const int tid = threadIdx.x;
  S->shard_ent[tid] = 0u;
  S->shard_cnd[tid] = 0u;
  if (tid == 0) {
    S->t_lo = a.t_lo; S->t_hi = a.t_hi; S->sbin = a.sbin;
    S->L64 = (uint64_t)a.t_lo << a.ib;
    S->cand_on = 1u; S->n_cand = 0; S->cand_over = 0; S->ent_over = 0;
    write_hdr_static(hdr, HI);
    hdr->lower = (uint64_t)a.t_lo << a.ib;
  }
}

template <int SRC, int FMT>
__global__ __launch_bounds__(kCBlock, FC_MAG1_WAVES_PER_EU) void k_compact_pred(CompactArgs a0) {
  __shared__ __attribute__((aligned(16))) PredShared sh;
  constexpr int NW = kCWaves, NQ = MagGeo<NW>::kQ, NI = NQ / 4;
  static_assert(NQ == 16, "16 elements per lane");
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t chunk = blockIdx.x, client = blockIdx.y;
  const MagOut o = mag_out(a0, client);
  uint64_t seed = a0.seed, offset = a0.offset;
  fc_packet_hdr* hdr = a0.hdr;
  if (a0.jobs) {
    const fc_u32x4 so = sload4(&a0.jobs[client].seed);
    seed = ((uint64_t)so.y << 32) | so.x;
    offset = ((uint64_t)so.w << 32) | so.z;
  }
  float x[NQ];
  mag_load<NW>(o.g, chunk, a0.n, x);
  const uint32_t base = chunk * (uint32_t)kChunk;
  const uint32_t n32 = (uint32_t)a0.n;
  const uint32_t lbase = (uint32_t)(w * 256 + lane);
#define FC_LOC(q) (lbase + ((q) >> 2) * MagGeo<NW>::kIStride + ((q) & 3) * 64)
  if (SRC != kSrcPhiloxKey && a0.write_hdr && chunk == 0 && tid == 0)
    write_hdr_static(hdr, a0.HI);                  // mask pipelines: the header's one writer

  // ---- predicates: bit q of pb (listed), cb (candidate), nb (NaN stand-in) ---------------
  uint32_t Lk = 0, Li = 0, t_lo = 0, t_hi = 0, cand_on = 0;
  if (SRC == kSrcPhiloxKey) {
    const MagState st = mag_state(o.S);
    const bool none = st.L64 == kSelectNothing;
    Lk = none ? 0xffffffffu : (uint32_t)(st.L64 >> o.ib);
    Li = none ? 0xffffffffu : (uint32_t)(st.L64 & ((1ull << o.ib) - 1));
    t_lo = st.t_lo; t_hi = st.t_hi; cand_on = st.cand_on;
  }
  uint32_t pb = 0, cb = 0, nb = 0;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    uint4 r = make_uint4(0u, 0u, 0u, 0u);
    if (SRC != kSrcMaskBits)
      r = philox_seg(((uint64_t)base >> 8) + (uint32_t)(i * NW + w), (uint32_t)lane, seed, offset);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = i * 4 + j;
      const uint32_t e = base + FC_LOC(q);
      const bool valid = e < n32;
      const uint32_t word = j == 0 ? r.x : j == 1 ? r.y : j == 2 ? r.z : r.w;
      bool p, c = false, nf = false;
      if (SRC == kSrcPhiloxKey) {
        const uint32_t key = word >> 1;
        p = valid & ((key > Lk) | ((key == Lk) & (e >= Li)));
        c = valid & (cand_on != 0) & (key >= t_lo) & (key <= t_hi);
      } else {
        bool keep;
        if (SRC == kSrcMaskBits) keep = valid && ((a0.mask[e >> 5] >> (e & 31)) & 1u) != 0;
        else keep = (uint64_t)word < a0.bern_thr;
        nf = a0.nonfinite_keep && !keep && (__float_as_uint(x[q]) & 0x7fffffffu) >= 0x7f800000u;
        p = valid & (keep | nf);
        nf = nf & valid;
      }
      pb |= (uint32_t)p << q;
      cb |= (uint32_t)c << q;
      nb |= (uint32_t)nf << q;
    }
  }
  // ---- phase 1: group counts (scalar popcounts), every wave scans the 32 words itself -----
  uint32_t pk[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    pk[i] = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      pk[i] |= (uint32_t)__popcll(__ballot((pb >> (i * 4 + j)) & 1u)) << (8 * j);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NI; ++i) sh.gcnt[i * NW + w] = pk[i];
  }
  __syncthreads();
  const uint32_t word = lane < kMGroups / 4 ? sh.gcnt[lane] : 0u;
  const uint32_t sum4 = __builtin_amdgcn_sad_u8(word, 0u, 0u);
  const uint32_t incl = wave_incl_scan(sum4);
  const uint32_t tot_e = (uint32_t)__builtin_amdgcn_readlane((int)incl, kMGroups / 4 - 1);
  const uint32_t e0 = incl - sum4;
  const uint32_t qs1 = (uint32_t)__builtin_amdgcn_readlane((int)e0, 1 * NW);
  const uint32_t qs2 = (uint32_t)__builtin_amdgcn_readlane((int)e0, 2 * NW);
  const uint32_t qs3 = (uint32_t)__builtin_amdgcn_readlane((int)e0, 3 * NW);
  const uint32_t e1 = e0 + (word & 0xffu), e2 = e1 + ((word >> 8) & 0xffu);
  const uint32_t e3 = e2 + ((word >> 16) & 0xffu);
  const uint32_t o01 = e0 | (e1 << 16), o23 = e2 | (e3 << 16);
  auto goff_of = [&](int q) -> uint32_t {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + w);
    return (q & 1) ? v >> 16 : v & 0xffffu;
  };
  auto value = [&](int q) -> float {
    return ((nb >> q) & 1u) ? __uint_as_float(0x7fc00000u) : x[q];
  };
  // ---- phase 2: listed entries -> LDS stage (or straight to the slot); bitmap words -------
  const uint64_t slot = base;
  const bool staged = tot_e <= (uint32_t)kStage;   // block-uniform
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const bool p = (pb >> q) & 1u;
    const uint64_t m = __ballot(p);
    const uint32_t pos = prefix_count(m) + goff_of(q);
    if (FMT == FC_FMT_BITMAP && lane < 2)          // the group's two bitmap words
      a0.bitmap[(base + FC_LOC(q) - (uint32_t)lane) / 32 + (uint32_t)lane] = (uint32_t)(m >> (32 * lane));
    if (p) {
      if (staged) {
        sh.st[pos] = make_uint2(FC_LOC(q), __float_as_uint(value(q)));
      } else {
        if (FMT == FC_FMT_IDXVAL) o.idx[slot + pos] = (uint16_t)FC_LOC(q);
        o.val[slot + pos] = value(q);
      }
    }
  }
  // ---- candidates (rand-k): wave w's LDS sub-slot at a wave-uniform running count ---------
  constexpr int kCW = kCandSlot / NW;
  uint32_t wc = 0;
  if (SRC == kSrcPhiloxKey && cand_on) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool c = (cb >> q) & 1u;
      const uint64_t mc = __ballot(c);
      const uint32_t pos = wc + prefix_count(mc);
      if (c && pos < (uint32_t)kCW) {
        const uint32_t e = base + FC_LOC(q);
        sh.cst[w * kCW + pos] = comp_of(philox_word(e, seed, offset) >> 1, e, o.ib);
      }
      wc += (uint32_t)__popcll(mc);
    }
  }
  if (lane == 0) sh.wcnt[w] = wc;
#undef FC_LOC
  __syncthreads();
  uint32_t wn[NW], tot_c = 0;
  bool c_ovf = false;
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    wn[j] = sh.wcnt[j];
    tot_c += wn[j];
    c_ovf |= wn[j] > (uint32_t)kCW;
  }
  if (tid == 0) {
    o.cnt[chunk] = tot_e;
    if (FMT == FC_FMT_IDXVAL && o.qoff)
      o.qoff[chunk] = qs1 | ((uint64_t)qs2 << 16) | ((uint64_t)qs3 << 32) | ((uint64_t)tot_e << 48);
    if (SRC == kSrcPhiloxKey) {
      o.ccnt[chunk] = c_ovf ? max(tot_c, (uint32_t)kCandSlot + 1u) : tot_c;
      atomicAdd(&o.S->shard_ent[chunk % kShards], tot_e);
      if (tot_c) atomicAdd(&o.S->shard_cnd[chunk % kShards], tot_c);
    }
  }
  if (staged) {                                    // coalesced 16-B stores of the staged slot
    for (uint32_t t = 4 * tid; t < tot_e; t += 4 * kCBlock) {
      if (t + 4 <= tot_e) {
        const uint4 p0 = *reinterpret_cast<const uint4*>(&sh.st[t]);
        const uint4 p1 = *reinterpret_cast<const uint4*>(&sh.st[t + 2]);
        if (FMT == FC_FMT_IDXVAL)
          *reinterpret_cast<uint2*>(o.idx + slot + t) = make_uint2(p0.x | (p0.z << 16), p1.x | (p1.z << 16));
        *reinterpret_cast<uint4*>(o.val + slot + t) = make_uint4(p0.y, p0.w, p1.y, p1.w);
      } else {
        for (uint32_t u = t; u < tot_e; ++u) {
          if (FMT == FC_FMT_IDXVAL) o.idx[slot + u] = (uint16_t)sh.st[u].x;
          o.val[slot + u] = __uint_as_float(sh.st[u].y);
        }
      }
    }
  }
  if (SRC == kSrcPhiloxKey && tot_c && !c_ovf && tid < kCandSlot) {   // candidates out
    const uint32_t wj = (uint32_t)tid / kCW, p = (uint32_t)tid % kCW;
    uint32_t pre = 0, nj = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const uint32_t m = min(wn[j], (uint32_t)kCW);
      if ((uint32_t)j < wj) pre += m;
      if ((uint32_t)j == wj) nj = m;
    }
    if (p < nj) o.cand[(uint64_t)chunk * kCandSlot + pre + p] = sh.cst[tid];
  }
}

template __global__ void k_compact_pred<kSrcPhiloxKey, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact_pred<kSrcMaskBits, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact_pred<kSrcMaskBits, FC_FMT_BITMAP>(CompactArgs);
template __global__ void k_compact_pred<kSrcBern, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact_pred<kSrcBern, FC_FMT_BITMAP>(CompactArgs);

}  // namespace fc
