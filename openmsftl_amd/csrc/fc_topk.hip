// fc_topk.hip — top-k / native rand-k encode for MI355X (gfx950).
//
// Replaces compression.py:31-45 (argsort(|g|)[::-1][:k] / permutation[:k]) with a
// streaming select whose only full read of g is ONE compaction launch:
//
//   k_sample_l1, k_sample_l2   stratified sample (<= 1 M keys, <1 % of g) -> two-level
//                              4096-bin histograms -> bracket [t_lo, t_hi] around the k-th key
//   k_compact                  one pass over g: every element with key >= t_lo is written
//                              (idx, val) in ascending index order (decoupled look-back over
//                              8192-element chunks); keys inside the bracket are also
//                              appended to a small candidate list; keys above t_hi counted
//   k_engine (x <= 6)          radix select (12-bit digits, LDS histograms) on the
//                              candidates -> exact composite threshold T64; finishes with an
//                              LDS bitonic sort once <= 2048 candidates remain
//
// Selection rule: comp = key << IB | idx is unique per element, the k
// largest comps are kept <=> argsort(|g|, stable)[::-1][:k] (highest index first in a tie),
// NaN above +inf.  The packet keeps every element with comp >= L64 (L64 <= T64); the decoder
// keeps comp >= T64.  fc_topk_encode_exact runs the same engine over g itself (no bracket).
#include "fc_state.h"

namespace fc {

template <int KM>
__device__ __forceinline__ uint4 keys4(const float4& x, uint64_t e, uint64_t seed,
                                       uint64_t off) {
  if (KM == kKeyMag) return make_uint4(mag_key(x.x), mag_key(x.y), mag_key(x.z), mag_key(x.w));
  const uint4 r = philox_block(e >> 2, seed, off);    // e is a multiple of 4
  return make_uint4(r.x >> 1, r.y >> 1, r.z >> 1, r.w >> 1);
}
template <int KM>
__device__ __forceinline__ uint32_t key1(float x, uint64_t i, uint64_t seed, uint64_t off) {
  if (KM == kKeyMag) return mag_key(x);
  return philox_word(i, seed, off) >> 1;
}
__device__ __forceinline__ uint32_t u4get(const uint4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// Find the bin holding the rank1-th largest element (1-based, descending bins) of an LDS
// histogram of kHistBins counts.  Result in s_out[0] = bin, s_out[1] = 1-based rank inside.
__device__ void find_rank_desc(const uint32_t* h, uint32_t rank1, uint32_t* s_tmp,
                               uint32_t* s_out) {
  const int t = threadIdx.x;
  constexpr int per = kHistBins / kBlock;   // 16 bins per thread, highest bins first
  const int top = kHistBins - 1 - per * t;
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < per; ++b) sum += h[top - b];
  __syncthreads();                          // callers may still be reading s_out
  if (t == 0) { s_out[0] = 0; s_out[1] = 1; }
  __syncthreads();
  const uint32_t excl = block_excl_scan(sum, s_tmp, nullptr);
  if (rank1 > excl && rank1 <= excl + sum) {
    uint32_t c = excl;
    for (int b = 0; b < per; ++b) {
      const uint32_t hb = h[top - b];
      if (rank1 <= c + hb) { s_out[0] = (uint32_t)(top - b); s_out[1] = rank1 - c; break; }
      c += hb;
    }
  }
  __syncthreads();
}

// --------------------------------------------------------------------------------------
// Sampling: level 1 (key >> 19, 4096 bins) and level 2 ((key >> 7) & 0xfff inside the two
// level-1 bins that hold the bracket ranks).
// --------------------------------------------------------------------------------------
template <int KM, int LEVEL>
__global__ __launch_bounds__(kBlock) void k_sample(const float* __restrict__ g, SamplePlan P,
                                                   uint64_t seed, uint64_t off, WsPtrs W,
                                                   uint32_t ib, fc_packet_hdr* hdr,
                                                   HdrInit HI) {
  __shared__ uint32_t ha[kHistBins];
  __shared__ uint32_t hb[LEVEL == 2 ? kHistBins : 1];
  __shared__ uint32_t s_tmp[8], s_out[4], s_flag;
  TopkState* S = W.st;
  const int tid = threadIdx.x;
  for (int b = tid; b < kHistBins; b += kBlock) { ha[b] = 0; if (LEVEL == 2) hb[b] = 0; }
  if (LEVEL == 1 && blockIdx.x == 0 && tid == 0) write_hdr_static(hdr, HI);
  uint32_t b1_hi = 0, b1_lo = 0, hi_none = 0, lo_all = 0;
  if (LEVEL == 2) { b1_hi = S->b1_hi; b1_lo = S->b1_lo; hi_none = S->hi_none; lo_all = S->lo_all; }
  __syncthreads();
  for (uint32_t s = blockIdx.x; s < P.nseg; s += gridDim.x) {
    const uint64_t st = seg_start(P, s);
    const uint64_t lim = P.full ? (st + 1024 < P.n ? st + 1024 : P.n) : st + 1024;
    const uint64_t e = st + (uint64_t)tid * 4;
    if (e < lim) {
      const float4 x = load4(g, e, lim);
      const uint4 kk = keys4<KM>(x, e, seed, off);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (e + j >= lim) break;
        const uint32_t key = u4get(kk, j);
        if (LEVEL == 1) {
          atomicAdd(&ha[key >> 19], 1u);
        } else {
          const uint32_t b1 = key >> 19, b2 = (key >> 7) & 0xfffu;
          if (!hi_none && b1 == b1_hi) atomicAdd(&ha[b2], 1u);
          if (!lo_all && b1 == b1_lo) atomicAdd(&hb[b2], 1u);
        }
      }
    }
  }
  __syncthreads();
  uint32_t* gha = LEVEL == 1 ? W.hist1 : W.hist2h;
  for (int b = tid; b < kHistBins; b += kBlock) {
    if (ha[b]) atomicAdd(&gha[b], ha[b]);
    if (LEVEL == 2 && hb[b]) atomicAdd(&W.hist2l[b], hb[b]);
  }
  uint32_t* done = LEVEL == 1 ? &S->a_done : &S->b_done;
  if (!last_block_arrive(done, gridDim.x, &s_flag)) return;
  // ---- last workgroup: resolve the bracket ranks ----
  for (int b = tid; b < kHistBins; b += kBlock) {
    ha[b] = ld_agent(&gha[b]); gha[b] = 0;
    if (LEVEL == 2) { hb[b] = ld_agent(&W.hist2l[b]); W.hist2l[b] = 0; }
  }
  __syncthreads();
  if (LEVEL == 1) {
    uint32_t bh = 0, rh = 1, bl = 0, rl = 1;
    if (!P.hi_none) { find_rank_desc(ha, (uint32_t)P.r_hi, s_tmp, s_out); bh = s_out[0]; rh = s_out[1]; }
    if (!P.lo_all) { find_rank_desc(ha, (uint32_t)P.r_lo, s_tmp, s_out); bl = s_out[0]; rl = s_out[1]; }
    if (tid == 0) {
      S->b1_hi = bh; S->rr_hi = rh; S->b1_lo = bl; S->rr_lo = rl;
      S->hi_none = P.hi_none; S->lo_all = P.lo_all; S->a_done = 0;
    }
  } else {
    uint32_t t_hi = 0xffffffffu, t_lo = 0u;
    if (!hi_none) {
      find_rank_desc(ha, S->rr_hi, s_tmp, s_out);
      t_hi = (b1_hi << 19) | (s_out[0] << 7) | 0x7fu;
    }
    if (!lo_all) {
      find_rank_desc(hb, S->rr_lo, s_tmp, s_out);
      t_lo = (b1_lo << 19) | (s_out[0] << 7);
    }
    if (tid == 0) {
      S->t_lo = t_lo; S->t_hi = t_hi; S->L64 = (uint64_t)t_lo << ib; S->cand_on = 1;
      S->n_hi = 0; S->n_cand = 0; S->cand_over = 0; S->ent_over = 0;
      S->e_done = 0; S->e_ticket = 0; S->e_small_n = 0; S->e_status = 0;
      S->b_done = 0;
      hdr->lower = (uint64_t)t_lo << ib;
    }
  }
}

// --------------------------------------------------------------------------------------
// k_compact: one pass over g, ordered stream compaction with decoupled look-back.
// --------------------------------------------------------------------------------------
enum Pred : int { kPredKey = 0, kPredMask = 1, kPredBern = 2 };

struct CompactArgs {
  const float* g;
  uint64_t n;
  uint32_t ib, nchunks;
  uint64_t seed, offset;
  const uint32_t* mask;     // kPredMask
  uint64_t bern_thr;        // kPredBern: keep iff word < thr
  uint32_t nonfinite_keep;  // dropout: dropped inf/NaN are listed as NaN (g * 0 == NaN)
  uint32_t write_hdr;       // first kernel of a mask pipeline writes the static header
  uint32_t* idx;
  float* val;
  uint32_t* bitmap;
  uint64_t cap;
  uint32_t* dir;
  fc_packet_hdr* hdr;
  WsPtrs W;
  HdrInit HI;
};

constexpr uint32_t kSpinLimit = 1u << 22;

template <int KM, int PRED, int FMT>
__global__ __launch_bounds__(kBlock) void k_compact(CompactArgs a) {
  __shared__ uint32_t s_wcnt[kVec * kWaves];
  __shared__ uint32_t s_bex, s_cnt_def, s_cnt_cand, s_cand_base;
  __shared__ uint64_t s_tk;
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  TopkState* S = a.W.st;
  if (tid == 0) {
    const uint64_t tk = atomicAdd((unsigned long long*)&S->ticket, 1ull);
    if ((uint32_t)tk == a.nchunks - 1)                    // every ticket handed out
      atomicExch((unsigned long long*)&S->ticket, ((tk >> 32) + 1) << 32);
    s_tk = tk; s_cnt_def = 0; s_cnt_cand = 0;
  }
  __syncthreads();
  const uint32_t chunk = (uint32_t)s_tk, epoch = (uint32_t)(s_tk >> 32);
  const uint64_t base = (uint64_t)chunk * kChunk;

  uint64_t L64 = 0;
  uint32_t t_lo = 0, t_hi = 0xffffffffu, cand_on = 0;
  if (PRED == kPredKey) { L64 = S->L64; t_lo = S->t_lo; t_hi = S->t_hi; cand_on = S->cand_on; }

  float4 x[kVec];
#pragma unroll
  for (int i = 0; i < kVec; ++i)
    x[i] = load4(a.g, base + (uint64_t)(i * 1024 + w * 256 + lane * 4), a.n);

  uint32_t pbits = 0, cbits = 0, ndef = 0;
#pragma unroll
  for (int i = 0; i < kVec; ++i) {
    const uint64_t e0 = base + (uint64_t)(i * 1024 + w * 256 + lane * 4);
    uint4 kk = make_uint4(0, 0, 0, 0);
    if (PRED == kPredKey) kk = keys4<KM>(x[i], e0, a.seed, a.offset);
    if (PRED == kPredBern) kk = philox_block(e0 >> 2, a.seed, a.offset);
    uint32_t mword = 0;
    if (PRED == kPredMask && e0 < a.n) mword = a.mask[e0 >> 5] >> (e0 & 31);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t e = e0 + j;
      const bool valid = e < a.n;
      bool p = false;
      if (PRED == kPredKey) {
        const uint32_t key = u4get(kk, j);
        p = valid && comp_of(key, (uint32_t)e, a.ib) >= L64;
        ndef += (valid && key > t_hi) ? 1u : 0u;
        if (valid && cand_on && key >= t_lo && key <= t_hi) cbits |= 1u << (i * 4 + j);
      } else {
        const bool keep = PRED == kPredMask ? ((mword >> j) & 1u) != 0
                                            : (uint64_t)u4get(kk, j) < a.bern_thr;
        const uint32_t ab = __float_as_uint(f4get(x[i], j)) & 0x7fffffffu;
        const bool nan_standin = a.nonfinite_keep && !keep && ab >= 0x7f800000u;  // g*0 = NaN
        p = valid && (keep || nan_standin);
        if (valid && nan_standin) cbits |= 1u << (i * 4 + j);   // listed as NaN, not as g
      }
      if (p) pbits |= 1u << (i * 4 + j);
    }
  }

  // per-iteration wave ballots -> ordered offsets
  uint32_t lane_excl[kVec];
#pragma unroll
  for (int i = 0; i < kVec; ++i) {
    const uint64_t m0 = __ballot((pbits >> (i * 4 + 0)) & 1u);
    const uint64_t m1 = __ballot((pbits >> (i * 4 + 1)) & 1u);
    const uint64_t m2 = __ballot((pbits >> (i * 4 + 2)) & 1u);
    const uint64_t m3 = __ballot((pbits >> (i * 4 + 3)) & 1u);
    lane_excl[i] = prefix_count(m0) + prefix_count(m1) + prefix_count(m2) + prefix_count(m3);
    if (lane == 0)
      s_wcnt[i * kWaves + w] = __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
    if (FMT == FC_FMT_BITMAP && lane < 8) {
      const int sh = lane * 8;
      const uint32_t word = spread4((uint32_t)(m0 >> sh)) | (spread4((uint32_t)(m1 >> sh)) << 1) |
                            (spread4((uint32_t)(m2 >> sh)) << 2) | (spread4((uint32_t)(m3 >> sh)) << 3);
      a.bitmap[(base + (uint64_t)(i * 1024 + w * 256)) / 32 + lane] = word;
    }
  }
  if (PRED == kPredKey) {
    if (ndef) atomicAdd(&s_cnt_def, ndef);
  }
  uint32_t my_cand_off = 0;
  const uint32_t ncand = PRED == kPredKey ? (uint32_t)__popc(cbits) : 0u;
  if (ncand) my_cand_off = atomicAdd(&s_cnt_cand, ncand);
  __syncthreads();

  if (w == 0) {
    // (i, w) exclusive scan of the 32 wave counts
    uint32_t v = lane < kVec * kWaves ? s_wcnt[lane] : 0u, inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane < kVec * kWaves) s_wcnt[lane] = inc - v;
    const uint32_t agg = __shfl(inc, 63, 64);
    // decoupled look-back
    uint64_t* status = a.W.status;
    uint32_t excl = 0;
    if (chunk == 0) {
      if (lane == 0) st_agent(&status[0], granule(epoch, kFlagInc, agg));
    } else {
      if (lane == 0) st_agent(&status[chunk], granule(epoch, kFlagAgg, agg));
      int64_t jw = (int64_t)chunk - 1;
      uint32_t spins = 0;
      const uint32_t ep = epoch & 0x3fffffffu;
      while (true) {
        const int64_t p = jw - lane;
        uint64_t s = granule(epoch, kFlagInc, 0);
        bool ready = true;
        if (p >= 0) {
          s = ld_agent(&status[p]);
          ready = g_epoch(s) == ep && g_flag(s) != 0;
        }
        while (!__all(ready)) {
          __builtin_amdgcn_s_sleep(1);
          if (!ready) {
            s = ld_agent(&status[p]);
            ready = g_epoch(s) == ep && g_flag(s) != 0;
          }
          if (++spins > kSpinLimit) {            // never expected: bounded for safety
            if (!ready) { s = granule(epoch, kFlagInc, 0); ready = true; atomicOr(&S->err, 1u); }
          }
        }
        const uint64_t incm = __ballot(g_flag(s) == kFlagInc);
        if (incm) {
          const int L = __ffsll((long long)incm) - 1;   // nearest inclusive predecessor
          excl += wave_sum(lane <= L ? g_val(s) : 0u);
          break;
        }
        excl += wave_sum(g_val(s));
        jw -= 64;
      }
      if (lane == 0) st_agent(&status[chunk], granule(epoch, kFlagInc, excl + agg));
    }
    if (lane == 0) {
      s_bex = excl;
      a.dir[chunk] = excl;
      if (chunk == a.nchunks - 1) {             // the ONLY writer of hdr in this launch
        if (a.write_hdr) write_hdr_static(a.hdr, a.HI);
        a.dir[a.nchunks] = excl + agg;
        a.hdr->n_entries = excl + agg;
        if ((uint64_t)excl + agg > a.cap) {
          a.hdr->status = FC_STATUS_OVERFLOW;
          if (PRED == kPredKey) atomicOr(&S->ent_over, 1u);
        }
      }
      if (PRED == kPredKey) {
        if (s_cnt_def) atomicAdd(&S->n_hi, s_cnt_def);
        if (s_cnt_cand) s_cand_base = atomicAdd(&S->n_cand, s_cnt_cand);
      }
    }
  }
  __syncthreads();

  // candidates (unordered; the engine is order-free because comps are unique)
  if (PRED == kPredKey && ncand) {
    uint64_t pos = (uint64_t)s_cand_base + my_cand_off;
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      const uint64_t e0 = base + (uint64_t)(i * 1024 + w * 256 + lane * 4);
      const uint4 kk = keys4<KM>(x[i], e0, a.seed, a.offset);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if ((cbits >> (i * 4 + j)) & 1u) {
          if (pos < a.W.cand_cap) a.W.cand[pos] = comp_of(u4get(kk, j), (uint32_t)(e0 + j), a.ib);
          else atomicOr(&S->cand_over, 1u);
          ++pos;
        }
      }
    }
  }

  // ordered entry writes
  const uint32_t bex = s_bex;
#pragma unroll
  for (int i = 0; i < kVec; ++i) {
    uint64_t pos = (uint64_t)bex + s_wcnt[i * kWaves + w] + lane_excl[i];
    const uint64_t e0 = base + (uint64_t)(i * 1024 + w * 256 + lane * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if ((pbits >> (i * 4 + j)) & 1u) {
        if (pos < a.cap) {
          float v = f4get(x[i], j);
          if (PRED != kPredKey && ((cbits >> (i * 4 + j)) & 1u)) v = __uint_as_float(0x7fc00000u);
          if (FMT == FC_FMT_IDXVAL) a.idx[pos] = (uint32_t)(e0 + j);
          a.val[pos] = v;
        }
        ++pos;
      }
    }
  }
}

// --------------------------------------------------------------------------------------
// k_engine: one radix / collect pass of the exact selection of the rank-th largest comp.
// --------------------------------------------------------------------------------------
struct EngineArgs {
  const float* g;           // src 2 (dense)
  uint64_t n;
  const uint32_t* idx;      // src 1 (packet entries)
  const float* val;
  uint32_t ib;
  uint32_t first;           // 1: initialise the state (every block computes it identically)
  uint32_t exact;           // 1: exact pipeline (engine runs BEFORE k_compact)
  uint64_t k;
  uint64_t seed, offset;
  fc_packet_hdr* hdr;
  WsPtrs W;
  HdrInit HI;
};

struct EngState {
  uint64_t prefix;
  uint32_t shift, rank, matched, done, src, status;
  uint64_t result;
};

__device__ __forceinline__ int clz64(uint64_t x) { return x ? __clzll((long long)x) : 64; }

// Every field is assigned on every path (a partially initialised state let hipcc fold the
// rank of the cand_over path into an undefined register — see DESIGN.md §Lessons).
template <int KM>
__device__ __forceinline__ EngState engine_init(const EngineArgs& a) {
  TopkState* S = a.W.st;
  const uint32_t top = 31 + a.ib;          // comps < 2^(31+IB)
  const uint32_t k32 = (uint32_t)a.k;
  if (a.exact) {
    const uint32_t done = (a.k == 0 || a.k >= a.n) ? 1u : 0u;
    const uint64_t res = a.k == 0 ? kSelectNothing : 0ull;
    return EngState{0ull, top, k32, (uint32_t)a.n, done, 2u, (uint32_t)FC_STATUS_OK, res};
  }
  const uint32_t n_hi = S->n_hi, n_cand = S->n_cand, t_lo = S->t_lo, t_hi = S->t_hi;
  const uint32_t n_ent = a.hdr->n_entries;
  const bool retry = S->ent_over != 0 || S->err != 0 || (uint64_t)n_hi + n_cand < a.k;
  if (a.k == 0)
    return EngState{0ull, top, 0u, 0u, 1u, 2u, (uint32_t)FC_STATUS_OK, kSelectNothing};
  if (retry)
    return EngState{0ull, top, k32, 0u, 1u, 2u, (uint32_t)FC_STATUS_RETRY_EXACT, 0ull};
  const bool use_entries = n_hi > a.k || S->cand_over != 0;   // the listed superset
  if (use_entries)
    return EngState{0ull, top, k32, n_ent, 0u, 1u, (uint32_t)FC_STATUS_OK, 0ull};
  const uint32_t rank = k32 - n_hi;
  if (rank == 0)
    return EngState{0ull, top, 0u, n_cand, 1u, 0u, (uint32_t)FC_STATUS_OK,
                    ((uint64_t)t_hi + 1) << a.ib};
  const uint64_t lo = (uint64_t)t_lo << a.ib;
  const uint64_t hi = ((uint64_t)t_hi << a.ib) | ((1ull << a.ib) - 1);
  const uint32_t sh = 64 - clz64(lo ^ hi);
  const uint64_t prefix = sh >= 64 ? 0ull : (lo >> sh) << sh;
  return EngState{prefix, sh, rank, n_cand, 0u, 0u, (uint32_t)FC_STATUS_OK, 0ull};
}

template <int KM>
__device__ __forceinline__ uint64_t engine_comp(const EngineArgs& a, uint32_t src, uint64_t i) {
  if (src == 0) return a.W.cand[i];
  if (src == 1) {
    const uint32_t id = a.idx[i];
    return comp_of(key1<KM>(a.val[i], id, a.seed, a.offset), id, a.ib);
  }
  return comp_of(key1<KM>(a.g[i], i, a.seed, a.offset), (uint32_t)i, a.ib);
}

template <int KM>
__global__ __launch_bounds__(kBlock) void k_engine(EngineArgs a) {
  __shared__ uint32_t h[kHistBins];            // reused as the bitonic buffer (16 KiB)
  __shared__ uint32_t s_tmp[8], s_out[4], s_flag, s_cnt, s_base;
  TopkState* S = a.W.st;
  const int tid = threadIdx.x;
  const EngState E0 = a.first ? engine_init<KM>(a)
                              : EngState{S->e_prefix, S->e_shift, S->e_rank, S->e_matched,
                                         S->e_done, S->e_src, S->e_status, S->e_prefix};
  EngState E = E0;
  if (!a.first && E.done) return;             // resolved by an earlier pass

  uint64_t cnt = E.src == 0 ? (uint64_t)min(S->n_cand, (uint32_t)a.W.cand_cap)
               : E.src == 1 ? (uint64_t)a.hdr->n_entries : a.n;
  const bool collect = !E.done && E.matched <= (uint32_t)kSmallCap;
  const uint32_t D = E.shift < (uint32_t)kHistBits ? E.shift : (uint32_t)kHistBits;
  if (!E.done) {
    for (int b = tid; b < kHistBins; b += kBlock) h[b] = 0;
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t hi_part = E.prefix >> E.shift;
    if (!collect) {
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < cnt; i += stride) {
        const uint64_t v = engine_comp<KM>(a, E.src, i);
        if ((v >> E.shift) == hi_part)
          atomicAdd(&h[(uint32_t)(v >> (E.shift - D)) & ((1u << D) - 1)], 1u);
      }
      __syncthreads();
      for (int b = tid; b < kHistBins; b += kBlock)
        if (h[b]) atomicAdd(&a.W.ehist[b], h[b]);
    } else {
      // gather the <= kSmallCap survivors (order free)
      uint32_t mine = 0;
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < cnt; i += stride) {
        const uint64_t v = engine_comp<KM>(a, E.src, i);
        mine += (v >> E.shift) == hi_part ? 1u : 0u;
      }
      uint32_t off = mine ? atomicAdd(&s_cnt, mine) : 0u;
      __syncthreads();
      if (tid == 0 && s_cnt) s_base = atomicAdd(&S->e_small_n, s_cnt);
      __syncthreads();
      if (mine) {
        uint32_t pos = s_base + off;
        for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < cnt; i += stride) {
          const uint64_t v = engine_comp<KM>(a, E.src, i);
          if ((v >> E.shift) == hi_part && pos < (uint32_t)kSmallCap) a.W.small[pos++] = v;
        }
      }
    }
  }
  if (!last_block_arrive(&S->e_ticket, gridDim.x, &s_flag)) return;

  // ---- last workgroup: advance the state ----
  if (!E.done) {
    if (!collect) {
      for (int b = tid; b < kHistBins; b += kBlock) { h[b] = ld_agent(&a.W.ehist[b]); a.W.ehist[b] = 0; }
      __syncthreads();
      find_rank_desc(h, E.rank, s_tmp, s_out);
      const uint32_t d = s_out[0];
      E.prefix |= (uint64_t)d << (E.shift - D);
      E.shift -= D;
      E.rank = s_out[1];
      E.matched = h[d];
      if (E.shift == 0) { E.done = 1; E.result = E.prefix; }
    } else {
      // bitonic sort (descending) of the survivors in LDS (as uint64 pairs in h[])
      uint64_t* sv = reinterpret_cast<uint64_t*>(h);
      const uint32_t m = E.matched;
      uint32_t P2 = 1;
      while (P2 < m) P2 <<= 1;
      for (uint32_t i = tid; i < P2; i += kBlock) sv[i] = i < m ? ld_agent(&a.W.small[i]) : 0ull;
      __syncthreads();
      for (uint32_t size = 2; size <= P2; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
          for (uint32_t t = tid; t < P2 / 2; t += kBlock) {
            const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
            const bool desc = (i & size) == 0;
            const uint64_t x = sv[i], y = sv[j];
            if ((x < y) == desc) { sv[i] = y; sv[j] = x; }
          }
          __syncthreads();
        }
      }
      if (E.rank >= 1 && E.rank <= m) E.result = sv[E.rank - 1];
      else E.status = FC_STATUS_TIMEOUT;   // inconsistent state: never expected
      E.done = 1;
      __syncthreads();
    }
  }
  if (tid == 0) {
    if (a.first && a.exact) write_hdr_static(a.hdr, a.HI);   // sole hdr writer of this launch
    S->e_prefix = E.prefix; S->e_shift = E.shift; S->e_rank = E.rank; S->e_matched = E.matched;
    S->e_done = E.done; S->e_src = E.src; S->e_status = E.status;
    S->e_ticket = 0; S->e_small_n = 0;
    if (E.done) {
      a.hdr->thresh = E.result;
      if (E.status != FC_STATUS_OK) a.hdr->status = E.status;
      if (!a.exact) {
        a.hdr->n_definite = S->n_hi; a.hdr->n_cand = S->n_cand;
        S->n_hi = 0; S->n_cand = 0; S->cand_over = 0; S->ent_over = 0;
      } else {
        // exact pipeline: k_compact runs next and lists exactly comp >= T64
        S->L64 = E.result; S->t_lo = (uint32_t)(E.result >> a.ib); S->t_hi = 0xffffffffu;
        S->cand_on = 0; S->n_hi = 0; S->n_cand = 0; S->cand_over = 0; S->ent_over = 0;
        a.hdr->lower = E.result;
      }
    }
  }
}

// --------------------------------------------------------------------------------------
// explicit instantiations used by fc_capi.hip
// --------------------------------------------------------------------------------------
template __global__ void k_sample<kKeyMag, 1>(const float*, SamplePlan, uint64_t, uint64_t, WsPtrs, uint32_t, fc_packet_hdr*, HdrInit);
template __global__ void k_sample<kKeyMag, 2>(const float*, SamplePlan, uint64_t, uint64_t, WsPtrs, uint32_t, fc_packet_hdr*, HdrInit);
template __global__ void k_sample<kKeyPhilox, 1>(const float*, SamplePlan, uint64_t, uint64_t, WsPtrs, uint32_t, fc_packet_hdr*, HdrInit);
template __global__ void k_sample<kKeyPhilox, 2>(const float*, SamplePlan, uint64_t, uint64_t, WsPtrs, uint32_t, fc_packet_hdr*, HdrInit);
template __global__ void k_compact<kKeyMag, kPredKey, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact<kKeyPhilox, kPredKey, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact<kKeyMag, kPredMask, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact<kKeyMag, kPredMask, FC_FMT_BITMAP>(CompactArgs);
template __global__ void k_compact<kKeyMag, kPredBern, FC_FMT_IDXVAL>(CompactArgs);
template __global__ void k_compact<kKeyMag, kPredBern, FC_FMT_BITMAP>(CompactArgs);
template __global__ void k_engine<kKeyMag>(EngineArgs);
template __global__ void k_engine<kKeyPhilox>(EngineArgs);

}  // namespace fc
