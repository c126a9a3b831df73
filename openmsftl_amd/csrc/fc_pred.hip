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

// Arguments of k_compact_pred: only what the pass reads (CompactArgs' header-init block and
// unused pointers, hoisted into SGPRs at entry, spilled ~180 SGPRs).  Mask pipelines write
// their static header with k_write_hdr after the pass.
struct PredArgs {
  const float* g;
  uint64_t n, seed, offset, bern_thr;
  const uint32_t* mask;
  uint16_t* idx;
  float* val;
  uint32_t* bitmap;
  uint32_t* cnt;
  uint64_t* qoff;
  TopkState* S;              // rand-k: encoder state (bracket, totals), candidate slots
  uint32_t* ccnt;
  uint64_t* cand;
  const fc_encode_job* jobs; // batched rand-k: client blockIdx.y
  uint64_t ws_stride;
  uint32_t ib, nonfinite_keep;
  uint32_t* chist;           // lone rand-k: the candidate histogram, binned here (one atomic per
                             // candidate; k_resolve<false> then needs no binning launch)
};

__global__ __launch_bounds__(64) void k_write_hdr(fc_packet_hdr* hdr, HdrInit HI) {
  if (threadIdx.x == 0) write_hdr_static(hdr, HI);
}

// FULL: the whole chunk is in range — non-temporal loads at immediate offsets and the host
// mask read as one 64-bit scalar load per group (its two words ARE the group's keep mask);
// the last, partial chunk clamps its addresses and reads the mask per lane.  (One body for
// both let hipcc merge the two load forms into per-lane 64-bit addresses without the NT hint.)
template <int SRC, int FMT, bool FULL>
__device__ __forceinline__ void pred_body(const PredArgs& a, uint32_t chunk, PredShared& sh) {
  // the packet / workspace pointers in the GLOBAL address space (fc_topk.hip MagOut: generic
  // ones, taken from the job table, made every store a flat_store that the next LDS wait waited on)
  FC_G uint16_t* const a_idx = (FC_G uint16_t*)a.idx;
  FC_G float* const a_val = (FC_G float*)a.val;
  FC_G uint32_t* const a_bitmap = (FC_G uint32_t*)a.bitmap;
  FC_G uint32_t* const a_cnt = (FC_G uint32_t*)a.cnt;
  FC_G uint64_t* const a_qoff = (FC_G uint64_t*)a.qoff;
  FC_G uint32_t* const a_ccnt = (FC_G uint32_t*)a.ccnt;
  FC_G uint64_t* const a_cand = (FC_G uint64_t*)a.cand;
  constexpr int NW = kCWaves, NQ = MagGeo<NW>::kQ, NI = NQ / 4;
  static_assert(NQ == 16, "16 elements per lane");
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);     // uniform: the readlane index below
  const uint32_t base = chunk * (uint32_t)kChunk;
  const uint32_t n32 = (uint32_t)a.n;
  const uint32_t lbase = (uint32_t)(w * 256 + lane);
  float x[NQ];
  {
    typedef __attribute__((address_space(1))) const float gf;
    if (FULL) {
      gf* gp = (gf*)a.g + base + lbase;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        x[q] = __builtin_nontemporal_load(gp + (q >> 2) * MagGeo<NW>::kIStride + (q & 3) * 64);
    } else {
      const uint32_t lastl = n32 - 1u - base;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        x[q] = ((gf*)a.g)[base + min(lbase + (q >> 2) * MagGeo<NW>::kIStride + (q & 3) * 64, lastl)];
    }
  }
#define FC_LOC(q) (lbase + ((q) >> 2) * MagGeo<NW>::kIStride + ((q) & 3) * 64)
  // ---- predicates: bit q of pb (listed), cb (candidate), nb (NaN stand-in) ---------------
  uint32_t Lk = 0, Li = 0, t_lo = 0, t_hi = 0, cand_on = 0, sbin = 0;
  if (SRC == kSrcPhiloxKey) {
    const MagState st = mag_state(a.S);
    const bool none = st.L64 == kSelectNothing;
    Lk = none ? 0xffffffffu : (uint32_t)(st.L64 >> a.ib);
    Li = none ? 0xffffffffu : (uint32_t)(st.L64 & ((1ull << a.ib) - 1));
    t_lo = st.t_lo; t_hi = st.t_hi; cand_on = st.cand_on; sbin = st.sbin;
  }
  const uint64_t seg0 = ((uint64_t)base >> 8) + (uint32_t)w;
  uint32_t pb = 0, cb = 0, nb = 0;
  auto preds = [&](int i) {
    uint4 r = make_uint4(0u, 0u, 0u, 0u);
    if (SRC != kSrcMaskBits) r = philox_seg(seg0 + (uint32_t)(i * NW), (uint32_t)lane, a.seed, a.offset);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = i * 4 + j;
      const uint32_t e = base + FC_LOC(q);
      const bool valid = FULL || e < n32;
      const uint32_t word = j == 0 ? r.x : j == 1 ? r.y : j == 2 ? r.z : r.w;
      bool p, c = false, nf = false;
      if (SRC == kSrcPhiloxKey) {
        const uint32_t key = word >> 1;
        p = valid & ((key > Lk) | ((key == Lk) & (e >= Li)));
        c = valid & (cand_on != 0) & (key >= t_lo) & (key <= t_hi);
      } else {
        bool keep;
        if (SRC == kSrcMaskBits) {
          if (FULL) {                                  // the group's 64 keep bits, scalar
            typedef __attribute__((address_space(4))) const uint64_t cu64;
            const uint32_t wu = (uint32_t)__builtin_amdgcn_readfirstlane(w);
            const uint64_t m64 = ((cu64*)a.mask)[(base >> 6) + (uint32_t)(i * 32 + j) + wu * 4u];
            keep = ((m64 >> lane) & 1ull) != 0;
          } else {
            keep = valid && ((a.mask[e >> 5] >> (e & 31)) & 1u) != 0;
          }
        } else {
          keep = (uint64_t)word < a.bern_thr;
        }
        nf = a.nonfinite_keep && !keep && (__float_as_uint(x[q]) & 0x7fffffffu) >= 0x7f800000u;
        p = valid & (keep | nf);
        nf = nf & valid;
      }
      pb |= (uint32_t)p << q;
      cb |= (uint32_t)c << q;
      nb |= (uint32_t)nf << q;
    }
  };
  if (SRC == kSrcPhiloxKey) {
    // one Philox block at a time (unrolled, hipcc interleaved the four and needed 89 VGPRs)
#pragma unroll 1
    for (int i = 0; i < NI; ++i) preds(i);
  } else {
#pragma unroll
    for (int i = 0; i < NI; ++i) preds(i);
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
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + wu);
    return (q & 1) ? v >> 16 : v & 0xffffu;
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
      a_bitmap[(base + FC_LOC(q) - (uint32_t)lane) / 32 + (uint32_t)lane] = (uint32_t)(m >> (32 * lane));
    const float v = ((nb >> q) & 1u) ? __uint_as_float(0x7fc00000u) : x[q];
    if (p) {
      if (staged) {
        sh.st[pos] = make_uint2(FC_LOC(q), __float_as_uint(v));
      } else {
        if (FMT == FC_FMT_IDXVAL) a_idx[slot + pos] = (uint16_t)FC_LOC(q);
        a_val[slot + pos] = v;
      }
    }
  }
  // ---- candidates (rand-k): wave w's LDS sub-slot at a wave-uniform running count; the key
  // is recomputed (one Philox block per segment that holds a candidate: rare); a lone encode
  // also bins them (a.chist) ---------------
  constexpr int kCW = kCandSlot / NW;
  uint32_t wc = 0;
  if (SRC == kSrcPhiloxKey && cand_on) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (!__any((cb >> (i * 4)) & 0xfu)) continue;   // uniform
      const uint4 r = philox_seg(seg0 + (uint32_t)(i * NW), (uint32_t)lane, a.seed, a.offset);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = i * 4 + j;
        const bool c = (cb >> q) & 1u;
        const uint64_t mc = __ballot(c);
        const uint32_t pos = wc + prefix_count(mc);
        const uint32_t word = j == 0 ? r.x : j == 1 ? r.y : j == 2 ? r.z : r.w;
        if (c && pos < (uint32_t)kCW) sh.cst[w * kCW + pos] = comp_of(word >> 1, base + FC_LOC(q), a.ib);
        if (c && a.chist) atomicAdd(&a.chist[((word >> 1) - t_lo) >> sbin], 1u);
        wc += (uint32_t)__popcll(mc);
      }
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
    a_cnt[chunk] = tot_e;
    if (FMT == FC_FMT_IDXVAL && a_qoff)
      a_qoff[chunk] = qs1 | ((uint64_t)qs2 << 16) | ((uint64_t)qs3 << 32) | ((uint64_t)tot_e << 48);
    if (SRC == kSrcPhiloxKey) {
      a_ccnt[chunk] = c_ovf ? max(tot_c, (uint32_t)kCandSlot + 1u) : tot_c;
      atomicAdd(&a.S->shard_ent[chunk % kShards], tot_e);
      if (tot_c) atomicAdd(&a.S->shard_cnd[chunk % kShards], tot_c);
    }
  }
  if (staged) {                                    // coalesced 16-B stores of the staged slot
    for (uint32_t t = 4 * tid; t < tot_e; t += 4 * kCBlock) {
      if (t + 4 <= tot_e) {
        const uint4 p0 = *reinterpret_cast<const uint4*>(&sh.st[t]);
        const uint4 p1 = *reinterpret_cast<const uint4*>(&sh.st[t + 2]);
        if (FMT == FC_FMT_IDXVAL)
          *(FC_G fc_u32x2*)(a_idx + slot + t) = fc_u32x2{p0.x | (p0.z << 16), p1.x | (p1.z << 16)};
        *(FC_G fc_u32x4*)(a_val + slot + t) = fc_u32x4{p0.y, p0.w, p1.y, p1.w};
      } else {
        for (uint32_t u = t; u < tot_e; ++u) {
          if (FMT == FC_FMT_IDXVAL) a_idx[slot + u] = (uint16_t)sh.st[u].x;
          a_val[slot + u] = __uint_as_float(sh.st[u].y);
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
    if (p < nj) a_cand[(uint64_t)chunk * kCandSlot + pre + p] = sh.cst[tid];
  }
}

// rand-k's occupancy (its Philox rounds, unrolled four at a time, once spilled 39 VGPRs)
constexpr int FC_PRED_PHILOX_WAVES = 8;
template <int SRC, int FMT>
__global__ __launch_bounds__(kCBlock, SRC == kSrcPhiloxKey ? FC_PRED_PHILOX_WAVES : FC_MAG1_WAVES_PER_EU) void k_compact_pred(PredArgs a) {
  __shared__ __attribute__((aligned(16))) PredShared sh;
  const uint32_t chunk = blockIdx.x;
  if (a.jobs) {                                    // batched rand-k: client blockIdx.y
    const uint32_t client = blockIdx.y;
    const fc_u32x8 v = sload8(&a.jobs[client]);    // {g, idx, val, cnt}
    a.g = as_ptr<const float>(v[0], v[1]); a.idx = as_ptr<uint16_t>(v[2], v[3]);
    a.val = as_ptr<float>(v[4], v[5]); a.cnt = as_ptr<uint32_t>(v[6], v[7]);
    const fc_u32x4 so = sload4(&a.jobs[client].seed);
    a.seed = ((uint64_t)so.y << 32) | so.x;
    a.offset = ((uint64_t)so.w << 32) | so.z;
    const fc_u32x2 qv = sload2(&a.jobs[client].qoff);
    a.qoff = as_ptr<uint64_t>(qv.x, qv.y);
    const uint64_t sh_b = (uint64_t)client * a.ws_stride;
    a.S = reinterpret_cast<TopkState*>(reinterpret_cast<char*>(a.S) + sh_b);
    a.ccnt = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.ccnt) + sh_b);
    a.cand = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(a.cand) + sh_b);
  }
  if ((uint64_t)chunk * kChunk + kChunk <= a.n)    // block-uniform
    pred_body<SRC, FMT, true>(a, chunk, sh);
  else
    pred_body<SRC, FMT, false>(a, chunk, sh);
}

template __global__ void k_compact_pred<kSrcPhiloxKey, FC_FMT_IDXVAL>(PredArgs);
template __global__ void k_compact_pred<kSrcMaskBits, FC_FMT_IDXVAL>(PredArgs);
template __global__ void k_compact_pred<kSrcMaskBits, FC_FMT_BITMAP>(PredArgs);
template __global__ void k_compact_pred<kSrcBern, FC_FMT_IDXVAL>(PredArgs);
template __global__ void k_compact_pred<kSrcBern, FC_FMT_BITMAP>(PredArgs);

}  // namespace fc
