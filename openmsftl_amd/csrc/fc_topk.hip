// fc_topk.hip — top-k / native rand-k encode for MI355X (gfx950).
//
// Replaces compression.py:31-45 (argsort(|g|)[::-1][:k] / permutation[:k]).  Fast path =
// three stages, ONE streaming read of g (a lone client's sample and compaction share one
// launch, k_fused_mag):
//
//   k_sample1                 stratified sample (<= 2 M keys, < 2 % of g) -> one 4096-bin
//                             histogram whose fine window a pilot sub-sample places -> key
//                             bracket [t_lo, t_hi] around the k-th key (+-6 sigma of the
//                             sample quantile)
//   k_compact(_mag1)          one pass over g, one independent workgroup per 8192-element
//                             chunk: every element with key >= t_lo is written (idx, val) in
//                             ascending index order into the chunk's SLOT of the packet
//                             ([c*8192, c*8192 + cnt[c])) — no global scan, no look-back; keys
//                             inside the bracket ("candidates") also go to the chunk's
//                             candidate slot (k_fused_mag also bins them: 4096-bin histogram)
//   k_resolve                 candidate histogram (built here from the candidate slots unless
//                             k_fused_mag did) -> the bin holding rank r = k - #(key > t_hi);
//                             gather that bin's candidates; LDS rank / bitonic sort -> exact
//                             T64 (dense output: the same launch then zeroes the slack in q)
//
// Anything unusual (bracket missed, candidate list overflow, > 4096 survivors) sets
// FC_STATUS_RETRY_EXACT; fc_topk_encode_exact then runs k_engine (12-bit radix select over
// g, <= 6 passes) followed by the compaction with L64 = T64 (no slack).
//
// Selection rule: comp = key << IB | idx is unique per element; the k
// largest comps are kept <=> argsort(|g|, stable)[::-1][:k] (highest index first in a tie),
// NaN above +inf.  The packet lists every element with comp >= L64 (L64 <= T64); decoders
// keep comp >= T64.
#include <type_traits>

#include "fc_state.h"

namespace fc {

template <int KM>
__device__ __forceinline__ uint4 keys4(const float4& x, uint64_t e, uint64_t seed,
                                       uint64_t off) {
  if (KM == kKeyMag) return make_uint4(mag_key(x.x), mag_key(x.y), mag_key(x.z), mag_key(x.w));
  return make_uint4(philox_word(e, seed, off) >> 1, philox_word(e + 1, seed, off) >> 1,
                    philox_word(e + 2, seed, off) >> 1, philox_word(e + 3, seed, off) >> 1);
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
// histogram of kHistBins counts.  Result in s_out[0] = bin, s_out[1] = 1-based rank inside
// (bin 0, rank 1 when rank1 is outside [1, total]).  256-thread workgroup; s_tmp[8]: the block
// scan uses [0, 4), the owners [4, 8).  Thread t sums bins kHistBins-1-16t down 16; after the
// scan the thread whose range holds the rank publishes (t, prefix), and one wave reads that
// range's 16 bins one per lane and finds the bin with a 16-lane prefix sum and a ballot (the
// owner walking its 16 bins through LDS was 16 dependent reads, ~1 us on the bracket's chain).
__device__ __forceinline__ void rank_owner(uint32_t r, uint32_t excl, uint32_t sum, uint32_t total,
                                           uint32_t* s_own) {
  if (r >= 1 && r <= total && r > excl && r <= excl + sum) { s_own[0] = threadIdx.x; s_own[1] = excl; }
  if (threadIdx.x == 0 && !(r >= 1 && r <= total)) s_own[0] = 0xffffffffu;
}
__device__ __forceinline__ void rank_in_owner(const uint32_t* h, uint32_t r, const uint32_t* s_own,
                                              uint32_t* out) {
  constexpr int per = kHistBins / kBlock;
  const uint32_t lane = (uint32_t)lane_id();
  const uint32_t ot = s_own[0];
  if (ot == 0xffffffffu) {
    if (lane == 0) { out[0] = 0; out[1] = 1; }
    return;
  }
  const uint32_t oex = s_own[1];
  const int otop = kHistBins - 1 - per * (int)ot;
  const uint32_t hb = lane < (uint32_t)per ? h[otop - (int)lane] : 0u;
  const uint32_t inc = wave_incl_scan(hb);
  if (lane < (uint32_t)per && r > oex + inc - hb && r <= oex + inc) {   // exactly one lane
    out[0] = (uint32_t)(otop - (int)lane);
    out[1] = r - (oex + inc - hb);
  }
}
__device__ void find_rank_desc(const uint32_t* h, uint32_t rank1, uint32_t* s_tmp,
                               uint32_t* s_out) {
  const int t = threadIdx.x;
  constexpr int per = kHistBins / kBlock;   // 16 bins per thread, highest bins first
  const int top = kHistBins - 1 - per * t;
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < per; ++b) sum += h[top - b];
  uint32_t total;
  const uint32_t excl = block_excl_scan(sum, s_tmp, &total);   // ends on a barrier
  rank_owner(rank1, excl, sum, total, s_tmp + 4);
  __syncthreads();
  if (t < 64) rank_in_owner(h, rank1, s_tmp + 4, s_out);
  __syncthreads();
}

// Both ranks of find_rank_desc in one scan: s_out[0..1] for r1 (wave 0), s_out[2..3] for r2
// (wave 1).  256-thread workgroup.
__device__ void find_ranks_desc(const uint32_t* h, uint32_t r1, uint32_t r2, uint32_t* s_tmp,
                                uint32_t* s_out) {
  const int t = threadIdx.x;
  constexpr int per = kHistBins / kBlock;
  const int top = kHistBins - 1 - per * t;
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < per; ++b) sum += h[top - b];
  uint32_t total;
  const uint32_t excl = block_excl_scan(sum, s_tmp, &total);
  rank_owner(r1, excl, sum, total, s_tmp + 4);
  rank_owner(r2, excl, sum, total, s_tmp + 6);
  __syncthreads();
  if (t < 64) rank_in_owner(h, r1, s_tmp + 4, s_out);
  else if (t < 128) rank_in_owner(h, r2, s_tmp + 6, s_out + 2);
  __syncthreads();
}

// Descending bitonic sort of P2 (power of two) uint64 values in LDS (256 threads).
__device__ void bitonic_desc(uint64_t* sv, uint32_t P2) {
  for (uint32_t size = 2; size <= P2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < P2 / 2; t += blockDim.x) {
        const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
        const bool desc = (i & size) == 0;
        const uint64_t x = sv[i], y = sv[j];
        if ((x < y) == desc) { sv[i] = y; sv[j] = x; }
      }
      __syncthreads();
    }
  }
}

// --------------------------------------------------------------------------------------
// k_sample1: the bracket [t_lo, t_hi] around the k-th key in ONE launch.
//
// Every workgroup first reads the same small PILOT (kPilotSegs sample segments, <= 8 K keys,
// L2-resident after the first reader) and finds, in an LDS histogram of key >> 19, the
// level-1 bins holding the pilot ranks pr_hi / pr_lo (the sample bracket ranks scaled to the
// pilot, widened by 7 pilot sigmas).  That fixes the same key window [klo, khi] in every
// workgroup, so their histograms of the real sample (<= 1 M keys, 4 segments per workgroup)
// can share one 4096-bin layout without a second launch:
//   bins    0..1023  coarse, key >> 21, keys below the window
//   bins 1024..3071  fine, (key - klo) >> fs, the window (>= 256 key units per bin)
//   bins 3072..4095  coarse, key >> 21, keys above the window
// Bin order is key order, so the last workgroup reads the bracket ranks straight off the
// summed histogram.  A pilot that misjudges the window only coarsens the bracket (more
// candidates), it cannot make it wrong.  (Two launches — level 1 on key >> 19, level 2 on
// (key >> 7) & 0xfff — took 17.8 + 21.5 us per 128 M gradient.)
// --------------------------------------------------------------------------------------
constexpr int kSampleSegs = FC_SAMPLE_SEGS_PER_WG;
// Bounded in-kernel polls (k_fused_mag's bracket and window waits, ~0.25 us each): a bracket
// arrives in 14-30 us (~100 polls); 8192 polls (~2-4 ms) end a co-residency stall between two
// fused launches on two queues with a RETRY (the exact re-encode) instead of ~60 ms
// (tests/test_gpu_parity.py::test_fused_encodes_on_concurrent_streams_never_stall).
constexpr uint32_t kSpinMax = 1u << 13;
constexpr uint32_t kFineLo = 1024, kFineBins = 2048, kFineHi = kFineLo + kFineBins;
constexpr uint32_t kCoarseShift = 21;            // 0x7fffffff >> 21 = 1023

struct FineWin {
  uint32_t klo, khi, fs;
};
__device__ __forceinline__ uint32_t fine_bin(uint32_t key, const FineWin& F) {
  if (key > F.khi) return kFineHi + (key >> kCoarseShift);
  if (key >= F.klo) return kFineLo + ((key - F.klo) >> F.fs);
  return key >> kCoarseShift;
}
__device__ __forceinline__ uint32_t fine_lower(uint32_t b, const FineWin& F) {
  if (b >= kFineHi) return max(F.khi + 1u, (b - kFineHi) << kCoarseShift);
  if (b >= kFineLo) return F.klo + ((b - kFineLo) << F.fs);
  return b << kCoarseShift;
}
__device__ __forceinline__ uint32_t fine_upper(uint32_t b, const FineWin& F) {
  uint64_t u;
  if (b >= kFineHi) {
    u = ((uint64_t)(b - kFineHi + 1) << kCoarseShift) - 1;
  } else if (b >= kFineLo) {
    u = (uint64_t)F.klo + ((uint64_t)(b - kFineLo + 1) << F.fs) - 1;
    if (u > F.khi) u = F.khi;
  } else {
    u = ((uint64_t)(b + 1) << kCoarseShift) - 1;
    if (u + 1 > F.klo) u = F.klo - 1ull;            // klo > 0 whenever a key lands below it
  }
  return u > 0xffffffffull ? 0xffffffffu : (uint32_t)u;
}

// The fine window spanning level-1 (key >> 19) bins blo .. bhi.
__device__ __forceinline__ FineWin win_of(uint32_t blo, uint32_t bhi) {
  FineWin F;
  F.klo = blo << 19;
  F.khi = ((bhi + 1u) << 19) - 1u;
  F.fs = 0;
  while (((F.khi - F.klo) >> F.fs) >= kFineBins) ++F.fs;
  return F;
}

// Segment s of the sample: element range [e, lim) of this thread's float4.
// (n < 2^32: 32-bit bounds keep k_fused_mag's sample part inside 64 VGPRs)
__device__ __forceinline__ void seg_lane(const SamplePlan& P, uint32_t s, int tid, uint32_t& e,
                                         uint32_t& lim) {
  const uint64_t st = seg_start(P, s);
  lim = (uint32_t)(P.full ? (st + 1024 < P.n ? st + 1024 : P.n) : st + 1024);
  e = (uint32_t)st + (uint32_t)tid * 4u;
}

// gh[b] += h[b] for the non-empty bins of a 4096-bin LDS histogram (256 threads).  (Two bins
// per 64-bit atomic measured SLOWER: +10 us per lone encode, the last arriver's shard loads
// queued behind the 64-bit atomics, profiles/r04_ab_sample_chain.jsonl.)
__device__ __forceinline__ void flush_hist(uint32_t* gh, const uint32_t* h, uint32_t nb = kHistBins) {
  for (uint32_t b = threadIdx.x; b < nb; b += kBlock)
    if (h[b]) atomicAdd(&gh[b], h[b]);
}

// Sample loads: 4 consecutive elements of g as the float4 whose mag_key gives their keys.
// float32: the values themselves.  float64 (fc_topk_dense_f64's sampled path, fc_f64.hip): the
// 31-bit HIGH key of each double (|x| bits >> 32: exponent + 20 mantissa bits) as a float bit
// pattern, so mag_key of it is that high key (clamped at kNanKey: a non-decreasing map, which is
// all a bracket needs).  Through the GLOBAL address space: a batched launch takes g from the job
// table, and hipcc made the generic pointer's loads flat_loads, which count in lgkmcnt too, so
// the scalar loads between segments waited for each segment's data (4 serial round trips per
// sample group instead of one).
typedef __attribute__((address_space(1))) const float fc_gfloat;
typedef __attribute__((address_space(1))) const double fc_gdouble;
typedef double fc_d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const fc_d2v fc_gd2v;
__device__ __forceinline__ float4 load4_sample(const float* __restrict__ g0, uint64_t e, uint64_t n) {
  fc_gfloat* g = (fc_gfloat*)g0;
  if (e + 4 <= n) {
    const fc_f4v v = *(fc_gf4v*)(g + e);
    return make_float4(v.x, v.y, v.z, v.w);
  }
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e + 0 < n) r.x = g[e + 0];
  if (e + 1 < n) r.y = g[e + 1];
  if (e + 2 < n) r.z = g[e + 2];
  if (e + 3 < n) r.w = g[e + 3];
  return r;
}
__device__ __forceinline__ float hikey_f(double x) {
  return __uint_as_float((uint32_t)(((uint64_t)__double_as_longlong(x) & 0x7fffffffffffffffull) >> 32));
}
__device__ __forceinline__ float4 load4_sample(const double* __restrict__ g0, uint64_t e, uint64_t n) {
  fc_gdouble* g = (fc_gdouble*)g0;
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  if (e + 4 <= n) {
    const fc_d2v a = *(fc_gd2v*)(g + e);
    const fc_d2v b = *(fc_gd2v*)(g + e + 2);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (e + j < n) v[j] = g[e + j];
  }
  return make_float4(hikey_f(v[0]), hikey_f(v[1]), hikey_f(v[2]), hikey_f(v[3]));
}

// Pilot level-1 histogram (key >> 19) of the kPilotSegs pilot segments -> the window.
// own: this workgroup IS workgroup 0 (its segments xs / es / ls are the pilot, already loaded).
template <int KM, bool OWN_ONLY = false, typename T = float>
__device__ __forceinline__ FineWin pilot_window(const T* __restrict__ g, const SamplePlan& P,
                                                uint64_t seed, uint64_t off, uint32_t* h,
                                                uint32_t* s_tmp, uint32_t* s_out, bool own,
                                                const float4 (&xs)[kSampleSegs],
                                                const uint32_t (&es)[kSampleSegs],
                                                const uint32_t (&ls)[kSampleSegs]) {
  static_assert(kPilotSegs == kSampleSegs, "the pilot is workgroup 0's share of the sample");
  const int tid = threadIdx.x;
  float4 xp[kPilotSegs];
  uint32_t ep[kPilotSegs], lp[kPilotSegs];
#pragma unroll
  for (int q = 0; q < kPilotSegs; ++q) {
    if (OWN_ONLY || own) {
      xp[q] = xs[q]; ep[q] = es[q]; lp[q] = ls[q];
      continue;
    }
    ep[q] = lp[q] = 0;
    xp[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((uint32_t)q < P.np) {
      seg_lane(P, pilot_seg(P, (uint32_t)q), tid, ep[q], lp[q]);
      if (ep[q] < lp[q]) xp[q] = load4_sample(g, ep[q], lp[q]);
    }
  }
  __syncthreads();                                  // h zeroed by the caller
  FC_TR(20);
#pragma unroll
  for (int q = 0; q < kPilotSegs; ++q) {
    if (ep[q] < lp[q]) {
      const uint4 kk = keys4<KM>(xp[q], ep[q], seed, off);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ep[q] + j < lp[q]) atomicAdd(&h[u4get(kk, j) >> 19], 1u);
    }
  }
  __syncthreads();
  FC_TR(21);
  find_ranks_desc(h, (uint32_t)P.pr_hi, (uint32_t)P.pr_lo, s_tmp, s_out);
  FC_TR(22);
  return win_of(s_out[2], s_out[0]);
}

// One launch: grid (ceil(nseg / kSampleSegs), clients).  k_sample1 and (round 6) k_fused_mag
// have every workgroup compute the window itself (no in-kernel wait); the shared form (workgroup
// 0 publishes an sc1 payload the others poll; fc_topk_dense_f64_sampled's k_fused64) was
// measured faster in round 4, when 256 workgroups re-reading the same 32 KB pilot took ~7 us of
// loads, and 1-7 us slower in round 6 (profiles/r06_ab_fused_ownpilot.jsonl).
struct SampleShared {
  uint32_t h[kHistBins];                          // pilot histogram, then the sample's
  uint32_t s_tmp[8], s_out[4], s_flag, s_win[3];
};

// The body of k_sample1 for workgroup bid of nb (256 threads).  shared_pilot: a lone client's
// launch (workgroup 0 publishes the window).  pub != 0 (k_fused_mag): once the bracket is
// known, publish it to the compaction workgroups of the same launch (the kPubCopies bracket
// records of W.pub, tag pub | bit 31).
// SHARED_ONLY: the launch is a lone client's (the window always comes from workgroup 0's own
// segments): no second set of pilot registers (k_fused_mag runs in 64 VGPRs)
template <int KM, bool SHARED_ONLY = false, typename T = float, bool PRE = false>
__device__ __forceinline__ void sample_body(const T* __restrict__ g, const SamplePlan& P,
                                            uint64_t seed, uint64_t off, const WsPtrs& W,
                                            uint32_t ib, fc_packet_hdr* hdr, const HdrInit& HI,
                                            uint32_t bid, uint32_t nb, bool shared_pilot,
                                            SampleShared& sm, uint32_t pub) {
  uint32_t* h = sm.h;
  uint32_t* s_tmp = sm.s_tmp;
  uint32_t* s_out = sm.s_out;
  uint32_t* s_win = sm.s_win;
  TopkState* S = W.st;
  const int tid = threadIdx.x;
  FC_TR(0);
  // The sample is P.pstride groups of kSampleSegs segments (group v: segments v + q * pstride;
  // group 0 is the pilot).  Workgroup bid of nb takes groups bid, bid + nb, ... one after the
  // other into the same histogram: a batched launch gives each workgroup FC_SAMPLE_ROUNDS = 4
  // (a quarter of the workgroups, one window, one flush and one ticket per four groups; the
  // launch was occupancy-bound at ~17 us per workgroup: 64 x 128 M 190 -> 125 us, 64 x 16 M
  // 84 -> 59 us).  The sample, its window and so the bracket are unchanged.
  float4 xs[kSampleSegs];
  uint32_t es[kSampleSegs], ls[kSampleSegs];
  auto load_group = [&](uint32_t v) {
#pragma unroll
    for (int q = 0; q < kSampleSegs; ++q) {
      const uint32_t s = v + (uint32_t)q * P.pstride;
      es[q] = ls[q] = 0;
      xs[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((uint32_t)q < P.segs && s < P.nseg) {
        seg_lane(P, s, tid, es[q], ls[q]);
        if (es[q] < ls[q]) xs[q] = load4_sample(g, es[q], ls[q]);
      }
    }
  };
  // this workgroup's first group first (plain loads: ~2 us sooner than non-temporal here)
  load_group(bid);
  for (int b = tid; b < kHistBins; b += kBlock) h[b] = 0;
  FineWin F;
  if (SHARED_ONLY) shared_pilot = true;
  if (PRE) {
    // a batched launch: k_pilot (the previous launch) left this client's window in win_flag
    const uint32_t w = S->win_flag;
    F = win_of(w & 0xfffu, (w >> 12) & 0xfffu);
    if ((w >> 31) == 0u) { F.klo = 0; F.khi = 0xffffffffu; F.fs = 31; }   // (never expected)
  } else if (!shared_pilot || bid == 0) {
    F = pilot_window<KM, SHARED_ONLY, T>(g, P, seed, off, h, s_tmp, s_out, bid == 0, xs, es, ls);
    // publish the window as ONE sc1 word (its two level-1 bins, bit 31 = valid): the pollers'
    // load returns the payload itself (a flag then three payload loads was one more round trip);
    // kWinCopies copies on their own lines, workgroup b polls copy b % kWinCopies
    if (shared_pilot && tid < kWinCopies)
      st_agent(&W.pub[(kPubCopies + tid) * kPubStride], 0x80000000u | ((F.khi >> 19) << 12) | (F.klo >> 19));
    for (int b = tid; b < kHistBins; b += kBlock) h[b] = 0;   // find_ranks_desc ended on a barrier
  } else {
    if (tid == 0) {                               // relaxed sc1 poll (bounded) of the payload
      uint32_t it = 0, w;
      const uint32_t* wf = &W.pub[(kPubCopies + bid % kWinCopies) * kPubStride];
      while (((w = ld_agent(wf)) >> 31) == 0u && ++it < kSpinMax) __builtin_amdgcn_s_sleep(2);
      s_win[0] = w;
    }
    __syncthreads();
    const uint32_t w = s_win[0];
    F = win_of(w & 0xfffu, (w >> 12) & 0xfffu);
    if ((w >> 31) == 0u) {                        // timed out (never expected): make the resolve retry
      if (tid == 0) st_agent(&S->err, 1u);
      F.klo = 0; F.khi = 0xffffffffu; F.fs = 31;
    }
  }
  __syncthreads();
  FC_TR(2);
  // ---- this workgroup's share of the sample ----
  // (Binning one below-window key in four, the rest exactly, changed nothing: the batched
  // sample's ~20 us of group loads + binning run at ~6.4 TB/s of sample bytes, FC_TRACE,
  // profiles/r05_ab_sample_pilot_sub4.jsonl.)
  auto hist_group = [&](const float4 (&xg)[kSampleSegs], const uint32_t (&eg)[kSampleSegs],
                        const uint32_t (&lg)[kSampleSegs]) {
#pragma unroll
    for (int q = 0; q < kSampleSegs; ++q) {
      if (eg[q] < lg[q]) {
        const uint4 kk = keys4<KM>(xg[q], eg[q], seed, off);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (eg[q] + j < lg[q]) atomicAdd(&h[fine_bin(u4get(kk, j), F)], 1u);
      }
    }
  };
  if (PRE) {
    // no pilot registers: the next group's loads are in flight while this one is binned
    for (uint32_t v = bid;;) {
      const uint32_t vn = v + nb;
      float4 xn[kSampleSegs];
      uint32_t en[kSampleSegs], ln[kSampleSegs];
#pragma unroll
      for (int q = 0; q < kSampleSegs; ++q) {
        const uint32_t s = vn + (uint32_t)q * P.pstride;
        en[q] = ln[q] = 0;
        xn[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((uint32_t)q < P.segs && vn < P.pstride && s < P.nseg) {
          seg_lane(P, s, tid, en[q], ln[q]);
          if (en[q] < ln[q]) xn[q] = load4_sample(g, en[q], ln[q]);
        }
      }
      hist_group(xs, es, ls);
      if (vn >= P.pstride) break;
#pragma unroll
      for (int q = 0; q < kSampleSegs; ++q) { xs[q] = xn[q]; es[q] = en[q]; ls[q] = ln[q]; }
      v = vn;
    }
  } else {
    for (uint32_t v = bid;;) {
      hist_group(xs, es, ls);
      v += nb;
      if (SHARED_ONLY || v >= P.pstride) break;  // (k_fused_mag: one group per workgroup)
      load_group(v);
    }
  }
  __syncthreads();
  FC_TR(3);
  // histogram shards: one per 128 workgroups (<= kSampleShards): the last arriver's shard loads
  // are on the bracket's latency chain (a lone 16 M encode has 128 sample workgroups: one shard)
  const uint32_t nsh = min((uint32_t)kSampleShards, max(1u, nb / 128u));
  flush_hist(W.hist1 + (bid % nsh) * kHistBins, h);   // into this workgroup's shard
  FC_TR(4);
  if (!last_block_arrive_tree(W.tick, nb, bid, &sm.s_flag, 18)) return;
  FC_TR(5);
  // ---- last workgroup: the bracket (read + clear the histogram) ----
  // the compaction's shard totals are reset first: wave 0's wait for its histogram loads below
  // also drains these stores, so they precede the bracket's publication (pub) without a drain
  // of their own
  if (tid < kShards) { st_agent(&S->shard_ent[tid], 0u); st_agent(&S->shard_cnd[tid], 0u); }
  {
    // every load first (one round trip), then the clearing stores: a load and a store of the
    // same address issue in order, so interleaving them cost one round trip per bin (~45 us)
    constexpr int kPer = kHistBins / kBlock;
    uint32_t t[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) t[j] = 0;
#pragma unroll
    for (int sh = 0; sh < kSampleShards; ++sh)
      if ((uint32_t)sh < nsh)
#pragma unroll
      for (int j = 0; j < kPer; ++j) t[j] += ld_agent(&W.hist1[sh * kHistBins + j * kBlock + tid]);
#pragma unroll
    for (int j = 0; j < kPer; ++j) h[j * kBlock + tid] = t[j];
  }
  __syncthreads();
  FC_TR(7);
  find_ranks_desc(h, P.hi_none ? 1u : (uint32_t)P.r_hi, P.lo_all ? 1u : (uint32_t)P.r_lo, s_tmp, s_out);
  FC_TR(23);
  const uint32_t t_hi = P.hi_none ? 0xffffffffu : fine_upper(s_out[0], F);
  const uint32_t t_lo = P.lo_all ? 0u : fine_lower(s_out[2], F);
  const uint64_t span = (uint64_t)t_hi - t_lo;            // candidate keys: [t_lo, t_hi]
  uint32_t sb = 0;
  while ((span >> sb) >= (1ull << P.cbins_log2)) ++sb;
  // pub != 0 (k_fused_mag): the bracket to the compaction workgroups of this launch, one 16-B
  // record per line (tag = pub | bit 31, never the previous launch's tag nor the zeroed start)
  if (pub && tid < kPubCopies) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the shard resets: long since done)
    fc_rec4 r;
    r.x = t_lo; r.y = t_hi; r.z = sb; r.w = pub | 0x80000000u;
    st16_agent(&W.pub[tid * kPubStride], r);
  }
  if (tid == 0) {
    st_agent(&S->t_lo, t_lo); st_agent(&S->t_hi, t_hi); st_agent(&S->sbin, sb);
    st_agent(&S->L64, (uint64_t)t_lo << ib);
    st_agent(&S->cand_on, 1u);
    S->n_cand = 0; S->cand_over = 0; S->ent_over = 0;
                                   // (err: set by a timed-out wait, read and cleared by this
                                   // call's k_resolve)
    // the header's only writer in this launch: a static header written by workgroup 0 at its
    // start raced this store through another XCD's L2 (lower read back as 0).  Nothing in this
    // launch reads it (k_resolve does, after the kernel boundary).
    write_hdr_static(hdr, HI);
    hdr->lower = (uint64_t)t_lo << ib;
  }
  // every sample workgroup has read its window copy (before its ticket): clear them for the next
  // launch (plain stores, visible after this kernel's end-of-launch write-back)
  if (shared_pilot && tid < kWinCopies) W.pub[(kPubCopies + tid) * kPubStride] = 0u;
  // clear the shards for the next call last, with plain 16-B stores (their next use is an
  // atomic in the next launch, after this kernel's end-of-launch write-back)
  for (uint32_t i = tid; i < (uint32_t)kHistBins * nsh / 4; i += kBlock)
    reinterpret_cast<uint4*>(W.hist1)[i] = make_uint4(0u, 0u, 0u, 0u);
  FC_TR(6);
}

// k_pilot: a batched encode's fine windows, one workgroup per client (grid = clients): the
// pilot's level-1 histogram and ranks (pilot_window) once per client, left in the client's
// win_flag for k_sample1<KM, true> (the next launch).  Every batched k_sample1 workgroup used
// to compute its client's window itself: 16 x 128 copies of the same pilot at configs[2], each
// 4096 conflicting LDS atomics and a rank search (~9 us of each workgroup's ~50 us chain,
// FC_TRACE, profiles/r05_trace_batch_16M.json).
template <int KM>
__global__ __launch_bounds__(kBlock) void k_pilot(SamplePlan P, WsPtrs W, const fc_encode_job* jobs,
                                                  uint64_t ws_stride) {
  __shared__ uint32_t h[kHistBins];
  __shared__ uint32_t s_tmp[8], s_out[4];
  const fc_encode_job& J = jobs[blockIdx.x];
  const float* g = J.g;
  W = ws_shift(W, (uint64_t)blockIdx.x * ws_stride);
  for (int b = threadIdx.x; b < kHistBins; b += kBlock) h[b] = 0;
  float4 xs[kSampleSegs];
  uint32_t es[kSampleSegs], ls[kSampleSegs];
#pragma unroll
  for (int q = 0; q < kSampleSegs; ++q) { xs[q] = make_float4(0.f, 0.f, 0.f, 0.f); es[q] = ls[q] = 0; }
  const FineWin F = pilot_window<KM>(g, P, J.seed, J.offset, h, s_tmp, s_out, false, xs, es, ls);
  if (threadIdx.x == 0) W.st->win_flag = 0x80000000u | ((F.khi >> 19) << 12) | (F.klo >> 19);
}
template __global__ void k_pilot<kKeyMag>(SamplePlan, WsPtrs, const fc_encode_job*, uint64_t);

template <int KM, bool PRE = false>
__global__ __launch_bounds__(kBlock, 8) void k_sample1(const float* __restrict__ g, SamplePlan P,
                                                    uint64_t seed, uint64_t off, WsPtrs W,
                                                    uint32_t ib, fc_packet_hdr* hdr, HdrInit HI,
                                                    const fc_encode_job* jobs,
                                                    uint64_t ws_stride) {
  __shared__ SampleShared sm;
  if (jobs) {                                     // batched: client blockIdx.y
    const fc_encode_job& J = jobs[blockIdx.y];
    g = J.g; hdr = J.hdr; seed = J.seed; off = J.offset;
    HI.seed = seed; HI.offset = off;
    W = ws_shift(W, (uint64_t)blockIdx.y * ws_stride);
  }
  // every workgroup computes the pilot window itself, or (PRE: batched) reads the one k_pilot
  // left (no workgroup of this launch waits for another: safe beside any other kernel); only
  // k_fused_mag shares workgroup 0's window
  sample_body<KM, false, float, PRE>(g, P, seed, off, W, ib, hdr, HI, blockIdx.x, gridDim.x, false, sm, 0u);
}


// --------------------------------------------------------------------------------------
// Compaction (k_compact_mag1 here, k_compact_pred in fc_pred.hip): one independent 512-thread
// workgroup per 8192-element chunk (slotted packet, no global scan).  Listed entries are
// staged in LDS and leave as coalesced 16-B stores; candidates go to the chunk's candidate
// slot (k_resolve bins them).
// --------------------------------------------------------------------------------------
constexpr int kCBlock = 512;
constexpr int kCWaves = kCBlock / 64;            // 8
constexpr int kStage = 2048;                     // LDS-staged entries per chunk

struct CompactArgs {
  const float* g;
  uint64_t n;
  uint32_t ib, nchunks;
  uint64_t seed, offset;
  const uint32_t* mask;     // kSrcMaskBits (fc_pred.hip): host keep mask
  uint64_t bern_thr;        // kSrcBern: keep iff Philox word < thr
  uint32_t nonfinite_keep;  // dropout: dropped inf/NaN are listed as NaN (g * 0 == NaN)
  uint32_t write_hdr;       // mask pipelines (no earlier kernel) write the static header
  uint16_t* idx;            // chunk-local indices (ABI 3)
  float* val;
  uint32_t* bitmap;
  uint32_t* cnt;            // entries per chunk
  uint64_t* qoff;           // quarter offsets per chunk (include/fedcodec.h), may be null
  fc_packet_hdr* hdr;
  WsPtrs W;
  HdrInit HI;
  const fc_encode_job* jobs;   // batched encode: client blockIdx.y overrides g / packet / W
  uint64_t ws_stride;
  float* dense;             // fc_topk_encode_dense: also stream q = listed ? g : +0 (one client)
  uint32_t grid3;           // k_compact_mag1(_dense): 3-D grid (clients of a group, chunks, groups)
  uint32_t m;               // its clients (the last group may be partial)
};

// Per-client fields of a batched launch (jobs[blockIdx.y]); no-op for a single client.
template <typename Args>
__device__ __forceinline__ void apply_job(Args& a) {
  if (!a.jobs) return;
  const fc_encode_job& J = a.jobs[blockIdx.y];
  a.idx = J.idx; a.val = J.val; a.cnt = J.cnt; a.hdr = J.hdr;
  if constexpr (std::is_same<Args, CompactArgs>::value) a.qoff = J.qoff;
  a.seed = J.seed; a.offset = J.offset;
  a.W = ws_shift(a.W, (uint64_t)blockIdx.y * a.ws_stride);
}

// --------------------------------------------------------------------------------------
// k_compact_mag: the top-k (|g| key) compaction in ballot form.  Element layout
//     e = base + i*2048 + w*256 + j*64 + lane      (i < 4, w < 8, j < 4)
// makes every (i, w, j) "group" 64 consecutive elements held one per lane in lane order, so
// a group's listed elements are one 64-bit compare mask (SGPRs), its count one scalar
// popcount, and a lane's position in the chunk slot = group offset + mbcnt(mask).  In the
// common case ("fast" chunks: whole chunk in range, thresholds finite, no index tie-break
// inside the chunk) the predicate of an element is ONE v_cmp of |g| (abs modifier) against a
// float threshold: the k_compact float4 layout spent ~12 VALU per element on keys, validity,
// tie-breaks and bit-field assembly and was VALU-issue-bound (146 us at 128 M vs a ~114 us
// read+write roofline for the same bytes).
//   listed    comp >= L64  <=>  |g| !< T_list   (NaN: unordered -> listed, as key 0x7f800001)
//   candidate listed && key <= t_hi  <=>  |g| <= T_hi (NaN never, t_hi < +inf bits)
// Anything else (partial chunk, the chunk holding L64's index tie-break, thresholds at or
// above +inf bits) takes the exact integer predicate of k_compact, per element.
// Candidates (rare) are appended through an LDS counter: k_resolve does not need them ordered.
// --------------------------------------------------------------------------------------
constexpr int kMGroups = 4 * kCWaves * 4;          // 128 groups of 64 elements
constexpr int kMQ = 16;                            // groups per wave (512-thread workgroups)
// elements per lane for NW waves per chunk; chunk-element stride of the i index
template <int NW> struct MagGeo {
  static constexpr int kQ = kChunk / (NW * 64);    // 16 (NW = 8) or 32 (NW = 4)
  static constexpr int kIStride = NW * 256;        // e = i*kIStride + w*256 + j*64 + lane
  static constexpr int kThreads = NW * 64;
};

// Workgroup barrier without a memory fence on the vector-memory counter: each wave's LDS
// accesses are complete (lgkmcnt(0)) and the compiler may not move memory operations across
// it (__syncthreads() may also wait vmcnt(0) and drain loads kept in flight across it).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int STAGE, bool RAWBAR>
struct MagSharedT {
  static constexpr int kStageN = STAGE;
  uint32_t gcnt[kMGroups / 4];                     // 4 group counts (bytes, <= 64) per (i, w)
  uint32_t wcnt[8];                                // candidates per wave (may exceed its sub-slot)
  uint2 st[STAGE + 4];                             // packed {chunk-local index, value bits}
  uint64_t cst[kCandSlot];                         // candidate comps: wave w's sub-slot at w * kCW
  uint16_t cstb[kCandSlot];                        // their candidate-histogram bins (BIN)
  __device__ static void barrier() {
    if (RAWBAR) lds_barrier();
    else __syncthreads();
  }
};
typedef MagSharedT<kStage, false> MagShared;

// Block-uniform predicate parameters of one chunk.
struct MagPred {
  float T_list, T_hi;                              // fast: listed |g| !< T_list, cand |g| <= T_hi
  uint32_t cand_all;                               // fast: t_hi >= NaN key, every listed one
  uint32_t Lk, Li, t_lo, t_hi, cand_on, n32;       // exact (k_compact's integer form)
};

// FAST: one float compare per element.  Exact (!FAST): x[q] was replaced by the element's
// exact predicate bits (mag_exact_bits: bit 1 listed, bit 0 candidate) and the value is
// re-read from g when it is staged, so both paths hold the same 16 registers per lane.
template <bool FAST>
__device__ __forceinline__ bool mag_listed(const MagPred& P, float v) {
  if (FAST) return !(__builtin_fabsf(v) < P.T_list);
  return (__float_as_uint(v) >> 1) & 1u;
}
template <bool FAST>
__device__ __forceinline__ bool mag_cand(const MagPred& P, float v) {
  if (FAST) return !(__builtin_fabsf(v) < P.T_list) & ((__builtin_fabsf(v) <= P.T_hi) | (P.cand_all != 0));
  return __float_as_uint(v) & 1u;
}
// k_compact's exact integer predicates (listed: comp >= L64; candidate: key in [t_lo, t_hi])
// for element e0 + offset(q), written over x[q].
template <int NW>
__device__ __forceinline__ void mag_exact_bits(const MagPred& P, float (&x)[MagGeo<NW>::kQ],
                                               uint32_t e0) {
#pragma unroll
  for (int q = 0; q < MagGeo<NW>::kQ; ++q) {
    const uint32_t e = e0 + (q >> 2) * MagGeo<NW>::kIStride + (q & 3) * 64;
    const uint32_t key = mag_key(x[q]);
    const bool valid = e < P.n32;
    const bool p = valid & ((key > P.Lk) | ((key == P.Lk) & (e >= P.Li)));
    const bool c = valid & (P.cand_on != 0) & (key >= P.t_lo) & (key <= P.t_hi);
    x[q] = __uint_as_float(((uint32_t)p << 1) | (uint32_t)c);
  }
}

// Output / workspace pointers of one item (client), built when the item is compacted: the
// full CompactArgs of two items live across the loop spilled ~130 SGPRs.  The data pointers are
// GLOBAL-address-space: a batched launch reads them from the job table, and as generic pointers
// hipcc made every packet store a flat_store, which also counts in lgkmcnt, so each wave's next
// LDS read waited for its packet stores (and wave 0 for the chunk's counts) to complete.
struct MagOut {
  const FC_G float* g;
  FC_G uint16_t* idx;
  FC_G float* val;
  FC_G uint32_t* cnt;
  FC_G uint64_t* qoff;
  TopkState* S;
  FC_G uint32_t* ccnt;
  FC_G uint64_t* cand;
  uint32_t* chist;          // (atomics)
  uint32_t ib;
  FC_G float* dense;        // nullptr unless fc_topk_encode_dense
};

// PKT = false (the drop-in dense path, fc_topk_encode_dense): q is the product, the packet
// entries are not written (-6 B per listed element of HBM writes) except for a chunk whose
// candidates overflowed their slot (k_resolve re-reads that chunk's entries).
// NTS: the packet entries and candidates leave with non-temporal stores.  The batched pass
// (k_compact_mag1) writes GBs of packets that only the next kernels read back: plain stores left
// the L2s full of dirty lines that the following k_resolve waited behind (64 x 128 M: compaction
// 7.24 -> 7.04 ms, resolve 171 -> 140 us; 128 x 16 M: 1.98 -> 1.92 ms, 94 -> 84 us).  A lone
// encode keeps plain stores: its ~80 MB of entries stay in the Infinity Cache for the decode that
// usually follows (packet round trip at 128 M: 260 us plain, 294 us non-temporal;
// profiles/r04_ab_entry_nt_stores.jsonl).
template <bool FAST, typename SH, int NW, bool DENSE, bool BIN, bool PKT = true, bool NTS = false>
__device__ __forceinline__ void compact_mag_body(const MagOut& a, const MagPred& P,
                                                 float (&x)[MagGeo<NW>::kQ], SH& sh,
                                                 uint32_t chunk, uint32_t sbin) {
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);     // uniform: the readlane index below
  const uint32_t base = chunk * (uint32_t)kChunk;
  const uint32_t lbase = (uint32_t)(w * 256 + lane);
  constexpr int NQ = MagGeo<NW>::kQ, NI = NQ / 4;
#define FC_LOC(q) (lbase + ((q) >> 2) * MagGeo<NW>::kIStride + ((q) & 3) * 64)
  // ---- phase 1: group counts (scalar popcounts of the compare masks) ---------------------
  uint32_t pk[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    pk[i] = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      pk[i] |= (uint32_t)__popcll(__ballot(mag_listed<FAST>(P, x[i * 4 + j])))
               << (8 * j);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NI; ++i) sh.gcnt[i * NW + w] = pk[i];
  }
  SH::barrier();
  // recompute the predicates in phase 2 (one v_cmp each) instead of keeping 16 compare masks
  // live in SGPRs across the scan (that spilled 87 SGPRs)
#pragma unroll
  for (int q = 0; q < NQ; ++q) asm volatile("" : "+v"(x[q]));
  // every wave scans the 32 packed (i, w) words itself (no second barrier): lane L < 32 holds
  // word L = (i, w), in element order
  const uint32_t word = lane < kMGroups / 4 ? sh.gcnt[lane] : 0u;
  const uint32_t sum4 = __builtin_amdgcn_sad_u8(word, 0u, 0u);      // sum of the 4 counts
  const uint32_t incl = wave_incl_scan(sum4);
  const uint32_t tot_e = (uint32_t)__builtin_amdgcn_readlane((int)incl, kMGroups / 4 - 1);
  const uint32_t e0 = incl - sum4;
  // word L covers elements [256 L, 256 L + 256) of the chunk (i * NW + w = element / 256), so
  // quarter q (2048 elements) starts where word 8 q does
  const uint32_t qs1 = (uint32_t)__builtin_amdgcn_readlane((int)e0, 8);
  const uint32_t qs2 = (uint32_t)__builtin_amdgcn_readlane((int)e0, 16);
  const uint32_t qs3 = (uint32_t)__builtin_amdgcn_readlane((int)e0, 24);
  const uint32_t e1 = e0 + (word & 0xffu), e2 = e1 + ((word >> 8) & 0xffu);
  const uint32_t e3 = e2 + ((word >> 16) & 0xffu);
  const uint32_t o01 = e0 | (e1 << 16), o23 = e2 | (e3 << 16);
  // group q's slot offset, read from its holder lane where it is used (a precomputed array
  // is NQ live SGPRs: it spilled at NQ = 32)
  auto goff_of = [&](int q) -> uint32_t {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)((q & 2) ? o23 : o01), (q >> 2) * NW + wu);
    return (q & 1) ? v >> 16 : v & 0xffffu;
  };

  // ---- phase 2: listed entries -> LDS stage (or straight to the slot when dense) -----------
  const uint64_t slot = base;
  // fc_topk_encode_dense: the dense result q = zeros_like(g); q[listed] = g (compression.py:
  // 33-37) leaves with the same coalesced layout as the loads; the slack entries (listed,
  // comp < T64) are zeroed by k_resolve once it has T64
  auto dense_out = [&](int q, bool p) {
    if (!DENSE) return;                               // uniform
    const uint32_t e = base + FC_LOC(q);
    if (!FAST && e >= P.n32) return;                    // partial last chunk
    const float v = p ? (FAST ? x[q] : a.g[e]) : 0.0f;
    __builtin_nontemporal_store(v, a.dense + e);   // (sc1 / plain stores: 269 vs 192 us)
  };
  // entries straight to the chunk's slot (predicated stores): a chunk too dense for the LDS
  // stage, or (!PKT) one whose candidates overflowed
  auto direct_entries = [&](bool dense_too) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool p = mag_listed<FAST>(P, x[q]);
      const uint32_t pos = prefix_count(__ballot(p)) + goff_of(q);
      if (p) {
        a.idx[slot + pos] = (uint16_t)FC_LOC(q);
        a.val[slot + pos] = FAST ? x[q] : a.g[base + FC_LOC(q)];
      }
      if (dense_too) dense_out(q, p);
    }
  };
  if (!PKT) {                                           // dense only: q, no entries
#pragma unroll
    for (int q = 0; q < NQ; ++q) dense_out(q, mag_listed<FAST>(P, x[q]));
  } else if (tot_e <= (uint32_t)SH::kStageN) {          // block-uniform
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool p = mag_listed<FAST>(P, x[q]);
      const uint32_t pos = prefix_count(__ballot(p)) + goff_of(q);
      if (p) sh.st[pos] = make_uint2(FC_LOC(q), __float_as_uint(FAST ? x[q] : a.g[base + FC_LOC(q)]));
      dense_out(q, p);
    }
  } else {
    direct_entries(true);
  }
  // ---- candidates (key in [t_lo, t_hi]): wave w stages them in its own LDS sub-slot of kCW
  // at a wave-uniform running count: no atomic and no branch per group (a per-group LDS atomic
  // reservation cost ~14 % of the compaction at 16 M).  A wave past kCW marks the chunk
  // overflowed (the resolve re-reads its entries slot).  BIN (a lone client's fused launch):
  // the candidates also go into the candidate histogram, one global atomic each; batched
  // launches leave that to k_resolve, which reads them anyway (the atomics cost 5.7 % of this
  // pass at 128 M; the resolve's own binning adds a grid barrier, hidden behind the other
  // encode chain but not on a lone client's critical path).
  constexpr int kCW = kCandSlot / NW;
  uint32_t wc = 0;
  if (P.cand_on) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool c = mag_cand<FAST>(P, x[q]);
      const uint64_t mc = __ballot(c);
      if (mc == 0) continue;   // uniform: most groups hold no candidate (configs[2] -1.3 %,
                               // profiles/r06_ab_cand_skip.jsonl)
      const uint32_t pos = wc + prefix_count(mc);
      if (c) {
        const uint32_t e = base + FC_LOC(q);
        const uint32_t key = mag_key(FAST ? x[q] : a.g[e]);
        if (pos < (uint32_t)kCW) sh.cst[w * kCW + pos] = comp_of(key, e, a.ib);
        if (BIN) {
          const uint32_t bin = (key - P.t_lo) >> sbin;
          if (pos < (uint32_t)kCW) sh.cstb[w * kCW + pos] = (uint16_t)bin;
          else atomicAdd(&a.chist[bin], 1u);
        }
      }
      wc += (uint32_t)__popcll(mc);
    }
  }
  if (lane == 0) sh.wcnt[w] = wc;
#undef FC_LOC
  SH::barrier();
  uint32_t wn[NW], tot_c = 0;
  bool c_ovf = false;
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    wn[j] = sh.wcnt[j];
    tot_c += wn[j];
    c_ovf |= wn[j] > (uint32_t)kCW;
  }
  if (tid == 0) {
    TopkState* S = a.S;
    a.cnt[chunk] = tot_e;
    if (a.qoff) a.qoff[chunk] = qs1 | ((uint64_t)qs2 << 16) | ((uint64_t)qs3 << 32) | ((uint64_t)tot_e << 48);
    // a wave past its sub-slot: report more than the slot holds (k_resolve's overflow test)
    a.ccnt[chunk] = c_ovf ? max(tot_c, (uint32_t)kCandSlot + 1u) : tot_c;
    atomicAdd(&S->shard_ent[chunk % kShards], tot_e);
    if (tot_c) atomicAdd(&S->shard_cnd[chunk % kShards], tot_c);
  }
  if (!PKT && c_ovf) direct_entries(false);            // rare: the resolve reads them
  if (PKT && tot_e <= (uint32_t)SH::kStageN) {          // coalesced 16-B stores of the staged slot
    for (uint32_t t = 4 * tid; t < tot_e; t += 4 * MagGeo<NW>::kThreads) {
      if (t + 4 <= tot_e) {
        const uint4 p0 = *reinterpret_cast<const uint4*>(&sh.st[t]);
        const uint4 p1 = *reinterpret_cast<const uint4*>(&sh.st[t + 2]);
        fc_u32x2 iv;                                       // 4 chunk-local u16 indices
        iv.x = p0.x | (p0.z << 16); iv.y = p1.x | (p1.z << 16);
        fc_u32x4 vv;
        vv.x = p0.y; vv.y = p0.w; vv.z = p1.y; vv.w = p1.w;
        FC_G fc_u32x2* ip = (FC_G fc_u32x2*)(a.idx + slot + t);
        FC_G fc_u32x4* vp = (FC_G fc_u32x4*)(a.val + slot + t);
        if (NTS) {
          __builtin_nontemporal_store(iv, ip);
          __builtin_nontemporal_store(vv, vp);
        } else {
          *ip = iv;
          *vp = vv;
        }
      } else {
        for (uint32_t u = t; u < tot_e; ++u) {
          a.idx[slot + u] = (uint16_t)sh.st[u].x;
          a.val[slot + u] = __uint_as_float(sh.st[u].y);
        }
      }
    }
  }
  // staged candidates out: thread t < kCandSlot holds sub-slot entry (t / kCW, t % kCW); its
  // place in the chunk's candidate slot is the wave-major prefix
  if (tot_c && (BIN || !c_ovf) && tid < kCandSlot) {
    const uint32_t wj = (uint32_t)tid / kCW, p = (uint32_t)tid % kCW;
    uint32_t pre = 0, nj = 0;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const uint32_t m = min(wn[j], (uint32_t)kCW);
      if ((uint32_t)j < wj) pre += m;
      if ((uint32_t)j == wj) nj = m;
    }
    if (p < nj) {
      if (BIN) atomicAdd(&a.chist[sh.cstb[tid]], 1u);
      if (!c_ovf) {
        FC_G uint64_t* cp = &a.cand[(uint64_t)chunk * kCandSlot + pre + p];
        if (NTS) __builtin_nontemporal_store(sh.cst[tid], cp);
        else *cp = sh.cst[tid];
      }
    }
  }
}

// Per-client records (job table, encoder state) are read with SCALAR loads: no kernel of this
// launch writes them, but they sit behind generic pointers, so hipcc issued vector loads and
// waited for them (vmcnt(0)) in front of the gradient loads: one extra serialized HBM/L2
// latency per workgroup.  Reading through the scalar cache is fine (nothing here writes it).
__device__ __forceinline__ fc_u32x2 sload2(const void* p) {
  fc_u32x2 v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ fc_u32x4 sload4(const void* p) {
  fc_u32x4 v;
  asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ fc_u32x8 sload8(const void* p) {
  fc_u32x8 v;
  asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
template <typename T>
__device__ __forceinline__ T* as_ptr(uint32_t lo, uint32_t hi) {
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ const float* mag_g(const CompactArgs& a0, uint32_t client) {
  if (!a0.jobs) return a0.g;
  const fc_u32x2 v = sload2(&a0.jobs[client].g);
  return as_ptr<const float>(v.x, v.y);
}
__device__ __forceinline__ TopkState* mag_S(const CompactArgs& a0, uint32_t client) {
  return reinterpret_cast<TopkState*>(reinterpret_cast<char*>(a0.W.st) + (uint64_t)client * a0.ws_stride);
}
__device__ __forceinline__ MagOut mag_out(const CompactArgs& a0, uint32_t client) {
  MagOut o;
  const WsPtrs W = a0.jobs ? ws_shift(a0.W, (uint64_t)client * a0.ws_stride) : a0.W;
  const float* g = a0.g;
  uint16_t* idx = a0.idx;
  float* val = a0.val;
  uint32_t* cnt = a0.cnt;
  uint64_t* qoff = a0.qoff;
  if (a0.jobs) {                                // {g, idx, val, cnt} = first 32 B of the job
    const fc_u32x8 v = sload8(&a0.jobs[client]);
    g = as_ptr<const float>(v[0], v[1]); idx = as_ptr<uint16_t>(v[2], v[3]);
    val = as_ptr<float>(v[4], v[5]); cnt = as_ptr<uint32_t>(v[6], v[7]);
    const fc_u32x2 qv = sload2(&a0.jobs[client].qoff);
    qoff = as_ptr<uint64_t>(qv.x, qv.y);
  }
  o.g = (const FC_G float*)g; o.idx = (FC_G uint16_t*)idx; o.val = (FC_G float*)val;
  o.cnt = (FC_G uint32_t*)cnt; o.qoff = (FC_G uint64_t*)qoff;
  o.dense = (FC_G float*)(a0.jobs ? nullptr : a0.dense);
  o.S = W.st; o.ccnt = (FC_G uint32_t*)W.ccnt; o.cand = (FC_G uint64_t*)W.cand; o.chist = W.chist;
  o.ib = a0.ib;
  return o;
}

struct MagState {                                  // the encoder state k_compact_mag reads
  uint64_t L64;
  uint32_t t_lo, t_hi, cand_on, sbin;
};
static_assert(offsetof(TopkState, L64) == 8 && offsetof(TopkState, t_hi) == offsetof(TopkState, t_lo) + 4 &&
              offsetof(TopkState, sbin) == offsetof(TopkState, t_lo) + 8 &&
              offsetof(TopkState, cand_on) == offsetof(TopkState, t_lo) + 12 &&
              offsetof(TopkState, t_lo) % 4 == 0, "MagState scalar-load layout");
__device__ __forceinline__ MagState mag_state(const TopkState* S) {
  MagState m;
  const fc_u32x2 l = sload2(&S->L64);
  const fc_u32x4 t = sload4(&S->t_lo);
  m.L64 = ((uint64_t)l.y << 32) | l.x;
  m.t_lo = t.x; m.t_hi = t.y; m.sbin = t.z; m.cand_on = t.w;
  return m;
}

// The chunk's 16 elements per lane in the ballot layout; the last, partial chunk clamps its
// addresses (its values past n are never listed: exact path).  Non-temporal loads: plain ones
// stream this shape faster in isolation (5.77-5.84 against 5.53-5.55 TB/s,
// tools/shape_probe.hip) but are equal in the batched compaction and 15 % slower on the dense
// path, whose 512 MB of q stores then compete with the gradient for the caches
// (profiles/r02_ab_mag_load_kind.jsonl).
template <int NW>
__device__ __forceinline__ void mag_load(const float* g, uint32_t chunk, uint64_t n,
                                         float (&x)[MagGeo<NW>::kQ]) {
  constexpr int NQ = MagGeo<NW>::kQ, IS = MagGeo<NW>::kIStride;
  const uint32_t base = chunk * (uint32_t)kChunk;
  typedef __attribute__((address_space(1))) const float gf;
  const uint32_t l0 = (uint32_t)((threadIdx.x >> 6) * 256 + lane_id());
  if ((uint64_t)base + kChunk > n) {
    const uint32_t last = (uint32_t)(n - 1) - base;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      x[q] = ((gf*)g)[base + min(l0 + (q >> 2) * IS + (q & 3) * 64, last)];
    return;
  }
  gf* gp = (gf*)g + base + l0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) x[q] = __builtin_nontemporal_load(gp + (q >> 2) * IS + (q & 3) * 64);
}

// One workgroup per item (grid = (nchunks, clients)); <= 64 VGPRs, so 4 resident 512-thread
// workgroups per CU overlap one another's load latency.  (A persistent variant that kept the
// next item's loads in flight measured 1.3-2.5x SLOWER: hipcc spilled the second register set
// and loop-carried state)
template <int NW, typename SH, bool DENSE, bool BIN, bool PKT = true, bool NTS = false>
__device__ __forceinline__ void compact_mag_item(const CompactArgs& a0, const MagOut& o,
                                                 uint32_t chunk, const MagState& st,
                                                 float (&x)[MagGeo<NW>::kQ], SH& sh) {
  const int tid = threadIdx.x;
  const uint32_t base = chunk * (uint32_t)kChunk;
  const bool full = (uint64_t)base + kChunk <= a0.n;
  const bool none = st.L64 == kSelectNothing;
  MagPred P;
  P.t_lo = st.t_lo; P.t_hi = st.t_hi; P.cand_on = st.cand_on; P.n32 = (uint32_t)a0.n;
  P.Lk = none ? 0xffffffffu : (uint32_t)(st.L64 >> a0.ib);
  P.Li = none ? 0xffffffffu : (uint32_t)(st.L64 & ((1ull << a0.ib) - 1));
  // every element of the chunk is listed iff key >= Lk_eff when the tie-break index Li lies
  // outside the chunk
  const uint32_t Lk_eff = base >= P.Li ? P.Lk : P.Lk + 1u;
  const bool tie_inside = !none && base < P.Li && (uint64_t)base + kChunk > P.Li;
  const bool fast = full && !none && !tie_inside && Lk_eff <= 0x7f800000u;
  P.T_list = __uint_as_float(fast ? Lk_eff : 0u);
  // candidates: listed && key <= t_hi (t_hi >= the NaN key: every listed element)
  P.cand_all = P.t_hi >= 0x7f800001u;
  P.T_hi = __uint_as_float(P.cand_all ? 0x7f800000u : P.t_hi);
  if (fast) {
    compact_mag_body<true, SH, NW, DENSE, BIN, PKT, NTS>(o, P, x, sh, chunk, st.sbin);
  } else if (none) {                                       // k = 0: nothing listed
    SH::barrier();
    if (tid == 0) {
      o.cnt[chunk] = 0;
      if (o.qoff) o.qoff[chunk] = 0;
      o.ccnt[chunk] = 0;
    }
    if (DENSE)
      for (uint32_t i = (uint32_t)tid; i < (uint32_t)kChunk && (uint64_t)base + i < a0.n; i += blockDim.x)
        o.dense[base + i] = 0.0f;
  } else {                                                 // rare: exact integer predicate
    mag_exact_bits<NW>(P, x, base + (uint32_t)((tid >> 6) * 256 + lane_id()));
    compact_mag_body<false, SH, NW, DENSE, BIN, PKT, NTS>(o, P, x, sh, chunk, st.sbin);
  }
}

constexpr int FC_MAG1_WAVES_PER_EU = 8;
constexpr int FC_MAG1_IL = 64;
constexpr int FC_FUSED_SREC = 2048;       // first chunk of k_fused_mag<false> that tries the scalar record
// Dispatch order: workgroups are dispatched x-fastest, so the chunks of FC_MAG1_IL clients are
// interleaved (chunk-major within a group of clients): FC_MAG1_IL address streams are in
// flight at once instead of one.  Measured (tools/kbench.py --batch 64, 128 M floats): IL 1 / 4
// / 8 / 32 / 64 = 8.49 / 7.98 / 7.97 / 7.58 / 7.57 ms per 64-client launch.  Not the
// candidate-histogram atomics (dropping them changes nothing) and not address diversity
// (rotating each client's start chunk: 7.76 ms).  The grid says it directly (grid3: x = client
// in the group, y = chunk, z = group); a linear grid re-mapped with two integer divisions at
// every workgroup's start (~60 scalar instructions ahead of the first load) took 1.2 % longer
// at 64 x 128 M (profiles/r05_ab_compact_grid3d.jsonl) and is kept for > 65535 chunks (the
// grid's y limit).
__device__ __forceinline__ void mag_item_of(const CompactArgs& a0, uint32_t& client, uint32_t& chunk) {
  if (a0.grid3) {
    client = blockIdx.z * gridDim.x + blockIdx.x;
    chunk = blockIdx.y;
    return;
  }
  if (FC_MAG1_IL == 1) {
    client = blockIdx.y; chunk = blockIdx.x;
    return;
  }
  const uint32_t nch = gridDim.x, M = gridDim.y;
  const uint32_t L = blockIdx.y * nch + blockIdx.x;
  const uint32_t gsz = nch * (uint32_t)FC_MAG1_IL;
  const uint32_t g = L / gsz, r = L - g * gsz;
  const uint32_t Ig = min((uint32_t)FC_MAG1_IL, M - g * (uint32_t)FC_MAG1_IL);
  chunk = r / Ig;
  const uint32_t j = r - chunk * Ig;
  client = g * (uint32_t)FC_MAG1_IL + j;
}

template <int NW, bool DENSE = false, bool NTS = false>
__device__ __forceinline__ void compact_mag_wg(const CompactArgs& a0) {
  __shared__ __attribute__((aligned(16))) MagShared sh;
  uint32_t client, chunk;
  mag_item_of(a0, client, chunk);
  if (client >= a0.m) return;                            // a partial last group
  float x[MagGeo<NW>::kQ];
  mag_load<NW>(mag_g(a0, client), chunk, a0.n, x);       // g first, state behind it
  const MagState st = mag_state(mag_S(a0, client));
  compact_mag_item<NW, MagShared, DENSE, false, true, NTS>(a0, mag_out(a0, client), chunk, st, x, sh);
}
// 512 threads (8 waves x 16 elements per lane)
__global__ __launch_bounds__(kCBlock, FC_MAG1_WAVES_PER_EU) void k_compact_mag1(CompactArgs a0) {
  compact_mag_wg<8, false, true>(a0);
}
// the same pass that also streams the dense result q (fc_topk_encode_dense; one client)
__global__ __launch_bounds__(kCBlock, FC_MAG1_WAVES_PER_EU) void k_compact_mag1_dense(CompactArgs a0) {
  compact_mag_wg<8, true>(a0);
}
// (A 256-thread form, 4 waves x 32 elements per lane, measured equal at 128 VGPRs and slower
// with spills at 80-96: DESIGN.md §Lessons.)

// --------------------------------------------------------------------------------------
// k_fused_mag: a lone client's k_sample1 + k_compact_mag1(_dense) in ONE launch.
// Workgroups [0, nsamp) run the sample (256 of their 512 threads) and are dispatched first
// (workgroups leave the dispatcher in order); every other workgroup is one chunk.  A chunk's
// workgroup issues its loads, then waits (bounded relaxed sc1 poll of one of the kPubCopies
// 16-B bracket records, fc_state.h) until the sample's last workgroup has written them with the
// tag (fz_seq + 1) | bit 31, so the first resident round of chunk loads overlaps the sample's
// latency chain
// instead of following it in a second launch.  fz_seq only changes in the k_resolve that
// follows (stream order): every workgroup of this launch reads the same value.  The sample
// never waits on a chunk workgroup, so no wait can deadlock; a timed-out one (never expected)
// sets S->err, and the resolve reports RETRY (the caller re-encodes exactly).
// --------------------------------------------------------------------------------------
// The resolve's bin search (k_resolve<false>'s head) as one workgroup's work (256 threads): from
// the shard totals and the candidate histogram of a fused encode, the bin beta holding rank r =
// k - #(key > t_hi), the rank inside it and its count -> S->rb_*; rb_flags bit 0 = retry (the
// exact path), bit 1 = rank 0 (T64 = (t_hi + 1) << ib: every candidate is slack).  AGENT: the
// counters were written in this launch (coherent loads), else by an earlier one.
template <bool AGENT = false>
__device__ __forceinline__ void beta_body(const WsPtrs& W, uint64_t k, uint32_t* h, uint32_t* s_tmp,
                                          uint32_t* s_out, uint32_t* s_tot) {
  TopkState* S = W.st;
  const int tid = threadIdx.x;
  auto ld = [](const uint32_t* p) { return AGENT ? ld_agent(p) : *p; };
  uint32_t se = 0, sc = 0;
  if (tid < kShards) { se = ld(&S->shard_ent[tid]); sc = ld(&S->shard_cnd[tid]); }
  const uint32_t err = ld(&S->err);
#pragma unroll
  for (int j = 0; j < kHistBins / kBlock; ++j) h[j * kBlock + tid] = ld(&W.chist[j * kBlock + tid]);
  if (tid < 64) {
    se = wave_sum(se);
    sc = wave_sum(sc);
    if (tid == 0) { s_tot[0] = se; s_tot[1] = sc; }
  }
  __syncthreads();
  const uint32_t n_ent = s_tot[0], n_cand = s_tot[1];
  const uint32_t n_hi = n_ent - n_cand;
  const bool bad = err || n_cand > n_ent || (uint64_t)n_ent < k || (uint64_t)n_hi > k;
  const uint32_t rank = bad ? 0u : (uint32_t)(k - n_hi);
  bool retry = bad;
  uint32_t beta = 0xffffffffu, r_in = 1, cnt = 0;
  if (!retry && rank > 0) {
    find_rank_desc(h, rank, s_tmp, s_out);
    beta = s_out[0]; r_in = s_out[1]; cnt = h[beta];
    retry = cnt > (uint32_t)kSmallCap || cnt < r_in;
  }
  if (tid == 0) {
    S->rb_beta = beta; S->rb_rin = r_in; S->rb_cnt = cnt;
    S->rb_flags = (retry ? 1u : 0u) | (!retry && rank == 0 ? 2u : 0u);
    S->rb_nent = n_ent; S->rb_ncand = n_cand;
  }
}

union FusedShared {
  SampleShared s;
  MagShared m;
};

// Candidate binning inside the fused launch (one device-scope atomic per candidate into the
// candidate histogram), so the resolve needs no binning launch.  Both lone paths bin in-kernel
// since round 4: with the candidate histogram at its padded workspace offset (fc_state.h) the
// atomics cost the 128 M packet encode +2 us in the fused kernel and save 8 us of resolve
// (170 -> 165 us; 16 M: equal).  Round 3 had measured 197 vs 148 us — the histogram's lines
// then collided in HBM with another hot line (profiles/r04_ab_fused_bin.jsonl).  The dense
// path writes no packet entries (only an overflowed chunk's, which the resolve re-reads).
template <bool DENSE, int NW>
__device__ __forceinline__ void fused_mag_wg(const CompactArgs& a0, const SamplePlan& P,
                                             const HdrInit& HI, uint32_t nsamp) {
  __shared__ __attribute__((aligned(16))) FusedShared u;
  __shared__ MagState s_st;
  TopkState* S = a0.W.st;
  const uint32_t pub = sload2(&S->fz_seq).x + 1u;   // not written by this launch
  if (blockIdx.x < nsamp) {
    if (threadIdx.x >= kBlock) return;
    // every sample workgroup computes the pilot window itself from the pilot segments (L2-hits
    // after the first reader) instead of polling workgroup 0's published copy: the window is
    // ready ~1.5 us sooner (encode_decode 16 M 59.0 -> 58.0 us, dense 128 M 209 -> 202 us;
    // profiles/r06_ab_fused_ownpilot.jsonl)
    sample_body<kKeyMag, false>(a0.g, P, 0ull, 0ull, a0.W, a0.ib, a0.hdr, HI, blockIdx.x, nsamp, false, u.s, pub);
    return;
  }
  // (chunks in dispatch order: spreading the resident ones over 8 / 64 address streams, as
  // the batched pass interleaves clients, measured 147 -> 155 / 164 us for a 128 M packet)
  const uint32_t chunk = blockIdx.x - nsamp;
  float x[MagGeo<NW>::kQ];
  // the first resident round (chunk < 1024) starts its loads ~2.4 us late (s_sleep 90 x 64
  // clocks), so that the sample's loads are not queued behind 32 MB of chunk loads; those still
  // arrive long before the bracket (~14 us at 16 M).  16 M dense fused kernel 38.7 -> 37.6 us,
  // 128 M packet 140.5 -> 138 us (profiles/r05_ab_fused_publish_find_delay.jsonl)
  if (chunk < 1024u) __builtin_amdgcn_s_sleep(90);
  // Later resident rounds of the packet form (chunk >= FC_FUSED_SREC, long after the bracket
  // is out) read the record with a SCALAR load issued before their gradient loads: it has its
  // own queue, while the sc1 poll's load waits behind the wave's 16 vector loads, and a matching
  // tag skips the poll and its barrier.  A stale or unpublished copy (a compute unit's scalar
  // cache or an XCD's L2 holding the line from before the publication) only falls back to the
  // poll.  128 M encode 154.6 -> 147.8 us, encode_decode 246.6 -> 239.2 us on one box; the dense
  // form got 8 us SLOWER with it (138 spilled SGPRs there), so it keeps the poll
  // (profiles/r06_ab_fused_scalar_record.jsonl).
  const uint32_t* rec = &a0.W.pub[(blockIdx.x % kPubCopies) * kPubStride];
  const uint32_t tag = pub | 0x80000000u;
  typedef __attribute__((address_space(4))) const fc_rec4 fc_crec4;
  const bool try_s = !DENSE && chunk >= (uint32_t)FC_FUSED_SREC;
  fc_rec4 sr = {0u, 0u, 0u, 0u};
  if (try_s) sr = *(fc_crec4*)rec;
  mag_load<NW>(a0.g, chunk, a0.n, x);
  FC_TR(24);
  MagState st;
  if (try_s && sr.w == tag) {
    st.t_lo = sr.x; st.t_hi = sr.y; st.sbin = sr.z; st.cand_on = 1u;
    st.L64 = (uint64_t)sr.x << a0.ib;   // = the sample's L64
  } else {
  if (threadIdx.x == 0) {           // this workgroup's copy of the bracket record
    uint32_t it = 0;
    fc_rec4 r = ld16_agent(rec);
    while (r.w != tag && ++it < kSpinMax) {
      __builtin_amdgcn_s_sleep(4);
      r = ld16_agent(rec);
    }
    if (it >= kSpinMax) st_agent(&S->err, 1u);
    MagState m;
    m.t_lo = r.x; m.t_hi = r.y; m.sbin = r.z; m.cand_on = 1u;
    m.L64 = (uint64_t)r.x << a0.ib;   // = the sample's L64
    s_st = m;
  }
  __syncthreads();
  FC_TR(25);
  st = s_st;
  }
  compact_mag_item<NW, MagShared, DENSE, true, !DENSE>(a0, mag_out(a0, 0u), chunk, st, x, u.m);
  FC_TR(26);
}
template <bool DENSE>
__global__ __launch_bounds__(kCBlock, FC_MAG1_WAVES_PER_EU) void k_fused_mag(CompactArgs a0, SamplePlan P,
                                                                              HdrInit HI, uint32_t nsamp) {
  fused_mag_wg<DENSE, 8>(a0, P, HI, nsamp);
}
template __global__ void k_fused_mag<false>(CompactArgs, SamplePlan, HdrInit, uint32_t);
template __global__ void k_fused_mag<true>(CompactArgs, SamplePlan, HdrInit, uint32_t);

// --------------------------------------------------------------------------------------
// k_resolve<BIN>: exact T64 from the bracket's candidates, in launches whose workgroups never
// wait for each other (only last-arriver tickets):
//   k_resolve<true>  (when the compaction did not bin the candidates: batched, unfused, rand-k)
//     every workgroup bins its chunks' candidates (candidate slot, or the entries slot of a chunk
//     whose candidates overflowed it) into the 4096-bin candidate histogram; the last arriver
//     sums the shards, finds the bin beta holding rank r = k - #(key > t_hi) and stores it;
//   k_resolve<false> every workgroup gathers its candidates in bin beta into the small list
//     (beta from k_resolve<true>, or from the histogram k_fused_mag filled while it streamed);
//     the last arriver sorts the <= 4096 survivors in LDS, picks T64 and writes the header.
// fc_topk_encode_dense (a.dense, one client): the compaction wrote q = g at every LISTED
// element (comp >= L64); the slack (comp < T64) must go back to +0.  Bins are in key order, so a
// candidate binned below beta is below T64 whatever T64 is: every workgroup zeroes those of its
// range before its ticket, and the last arriver zeroes the entries of bin beta below T64 from
// the sorted list it holds (their comps carry the index).  No fix-up launch, no wait.
// Round 4 had one launch whose workgroups waited in-kernel for the bin (and, dense, for T64):
// safe only while every workgroup of a client was resident; two launches on two queues
// interleaved by the XCDs stalled each other to the spin bound (42-84 ms, ~1 step in 70).
// --------------------------------------------------------------------------------------
struct ResolveArgs {
  uint32_t ib, nchunks;
  uint64_t k;
  const uint16_t* idx;      // packet (for overflowed candidate slots), chunk-local
  const float* val;
  const uint32_t* cnt;
  uint64_t seed, offset;
  uint32_t key_mode;
  fc_packet_hdr* hdr;
  WsPtrs W;
  const fc_encode_job* jobs;   // batched encode (see CompactArgs)
  uint64_t ws_stride;
  float* dense;                // fc_topk_encode_dense: zero the slack of q (one client)
  uint32_t rbin;               // 1: k_resolve<true> binned the candidates (the compaction did
                               // not: batched, unfused and rand-k); 0: k_fused_mag did
};

// chunks per workgroup (their gather sizes live in LDS; the launches size the grid so that no
// workgroup gets more).  1024 keeps the workgroup at 36.9 KB of LDS = 4 per CU: at 2048 (41 KB,
// 3 per CU) a 64-client batch's 1024 workgroups did not fit one round.
constexpr int kResolveChunksMax = 1024;

template <bool BIN>
__global__ __launch_bounds__(kBlock) void k_resolve(ResolveArgs a0) {
  ResolveArgs a = a0;
  apply_job(a);
  __shared__ uint64_t sv[kSmallCap];                      // 32 KiB: histogram, then sort
  __shared__ uint32_t s_pre[kResolveChunksMax];           // per-chunk gather sizes
  __shared__ uint32_t s_tmp[8], s_out[4], s_flag, s_cnt, s_base, s_tot[2];
  __shared__ uint64_t s_T;
  uint32_t* h = reinterpret_cast<uint32_t*>(sv);          // 4096 bins = 16 KiB
  TopkState* S = a.W.st;
  const int tid = threadIdx.x;
  FC_TR(8);
  // ---- totals (sharded counters written by the compaction) and the bracket: one round of
  // independent loads ----
  uint32_t se = 0, sc = 0;
  if (tid < kShards) { se = S->shard_ent[tid]; sc = S->shard_cnd[tid]; }
  const uint32_t t_lo = S->t_lo, t_hi = S->t_hi, sbin = S->sbin, err = S->err;
  const bool rbin = a.rbin != 0;
  // this workgroup's chunk range and (<= one per thread, the usual case) its candidate counts,
  // in the same round of loads
  const uint32_t per = (a.nchunks + gridDim.x - 1) / gridDim.x;
  const uint32_t c0 = blockIdx.x * per;
  const uint32_t c1 = min(c0 + per, a.nchunks);
  const uint32_t nc = c1 > c0 ? c1 - c0 : 0u;
  const uint32_t cc_early = (nc <= (uint32_t)kBlock && (uint32_t)tid < nc) ? a.W.ccnt[c0 + tid] : 0u;
  // the gather's bin: the compaction's histogram (every workgroup reads it), or k_resolve<true>'s
  uint32_t hv[kHistBins / kBlock];
  const bool own_hist = !BIN && !rbin;
#pragma unroll
  for (int j = 0; j < kHistBins / kBlock; ++j) hv[j] = own_hist ? a.W.chist[j * kBlock + tid] : 0u;
  static_assert(kShards == 64, "shard totals: one wave");
  if (tid < 64) {
    se = wave_sum(se);
    sc = wave_sum(sc);
    if (tid == 0) {
      s_tot[0] = se; s_tot[1] = sc;
      if (!BIN && rbin) { s_out[0] = ld_agent(&S->rb_beta); s_out[1] = ld_agent(&S->rb_rin);
                          s_out[2] = ld_agent(&S->rb_cnt); }
    }
  }
#pragma unroll
  for (int j = 0; j < kHistBins / kBlock; ++j) h[j * kBlock + tid] = hv[j];
  __syncthreads();
  const uint32_t n_ent = s_tot[0], n_cand = s_tot[1];
  const uint32_t n_hi = n_ent - n_cand;                   // listed above the bracket
  const bool bad = err || n_cand > n_ent || (uint64_t)n_ent < a.k || (uint64_t)n_hi > a.k;
  const uint32_t rank = bad ? 0u : (uint32_t)(a.k - n_hi);
  bool retry = bad || per > (uint32_t)kResolveChunksMax;  // grid-uniform (exact path)
  uint32_t beta = 0, r_in = 1, cnt_beta = 0;
  if (!BIN && !retry && rank > 0) {
    if (own_hist) {
      find_rank_desc(h, rank, s_tmp, s_out);
      beta = s_out[0]; r_in = s_out[1]; cnt_beta = h[beta];
    } else {
      beta = s_out[0]; r_in = s_out[1]; cnt_beta = s_out[2];
    }
    retry = cnt_beta > (uint32_t)kSmallCap || cnt_beta < r_in;
    __syncthreads();
  }
  const bool binning = BIN && !retry && rank > 0;         // grid-uniform
  const bool walk = BIN ? binning : (!retry && (rank > 0 || a.dense));
  if (BIN && !binning) return;   // nothing to bin (the gather launch sees the same retry / rank)
  // ---- per-chunk gather sizes: the candidate slot, or (bit 31) the entries slot of a chunk
  // whose candidates overflowed their slot ----
  if (walk) {
    for (uint32_t lc = tid; lc < nc; lc += kBlock) {
      const uint32_t c = c0 + lc;
      const uint32_t cc = nc <= (uint32_t)kBlock ? cc_early : a.W.ccnt[c];
      s_pre[lc] = cc > (uint32_t)kCandSlot ? (a.cnt[c] | 0x80000000u) : cc;
    }
    __syncthreads();
  }
  FC_TR(10);
  // tpc threads (a power of two) share a chunk and read its candidates kGatherU per thread and
  // pass, with no search (a binary search over a prefix per candidate cost ~4 us at 128 M).
  // At least 4 per chunk, looping over the chunks in more passes: with one thread per chunk
  // (a batch's 1024 chunks per workgroup at 128 M) every load instruction touched 64 cache
  // lines 2 KB apart — 64 x 128 M resolve 281 -> 172 us, 64 x 16 M 61 -> 51 us.
  constexpr int kGatherU = 8;
  uint32_t tpc = 64;
  while (tpc > 4 && tpc * nc > (uint32_t)kBlock) tpc >>= 1;
  uint64_t v0[kGatherU];                                  // first pass, kept for the later ones
#pragma unroll
  for (int u = 0; u < kGatherU; ++u) v0[u] = ~0ull;
  // fn(v) for every pass of this thread over its candidates as comps (~0 = not a candidate:
  // an overflowed chunk's entry outside [t_lo, t_hi]); reuse: the first pass comes from v0
  auto for_cands = [&](bool reuse, auto&& fn) {
    const uint32_t cpr = (uint32_t)kBlock / tpc;
    for (uint32_t cb = 0; cb < nc; cb += cpr) {
      const uint32_t lc = cb + (uint32_t)tid / tpc, q = (uint32_t)tid % tpc;
      const uint32_t info = lc < nc ? s_pre[lc] : 0u;
      const uint32_t sz = info & 0x7fffffffu;
      const bool ovf = (info >> 31) != 0;
      const uint32_t c = c0 + lc;
      for (uint32_t r0 = q; r0 < sz; r0 += tpc * kGatherU) {
        const bool first = cb == 0 && r0 == q;
        uint64_t v[kGatherU];
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
          const uint32_t r = r0 + (uint32_t)u * tpc;
          v[u] = ~0ull;
          if (reuse && first) {
            v[u] = v0[u];
          } else if (r < sz) {
            if (!ovf) {
              v[u] = a.W.cand[(uint64_t)c * kCandSlot + r];
            } else {
              const uint64_t p = (uint64_t)c * kChunk + r;
              const uint32_t id = c * (uint32_t)kChunk + a.idx[p];
              const uint32_t key = a.key_mode == FC_KEY_PHILOX ? (philox_word(id, a.seed, a.offset) >> 1)
                                                               : mag_key(a.val[p]);
              v[u] = (key >= t_lo && key <= t_hi) ? comp_of(key, id, a.ib) : ~0ull;
            }
          }
        }
        if (first && !reuse) {
#pragma unroll
          for (int u = 0; u < kGatherU; ++u) v0[u] = v[u];
        }
        fn(v);
      }
    }
  };
  auto bin_of = [&](uint64_t v) { return (((uint32_t)(v >> a.ib)) - t_lo) >> sbin; };
  if constexpr (BIN) {
    // ---- the candidate histogram: every workgroup bins the candidates of its chunk range in
    // LDS and flushes the non-empty bins into one of kCandShards (2) shards (one shared
    // histogram: its queued same-address atomics cost the lone encode 3 us; 4 / 8 shards: the
    // last arriver's extra shard loads cost more, fc_state.h); the last arriver (two-level
    // ticket) sums the shards, finds the bin beta holding rank r and stores it for the gather
    // launch.  (The compaction used to add every candidate into the histogram with a global
    // atomic: 5.7 % of that pass at 128 M.) ----
    for_cands(false, [&](const uint64_t (&v)[kGatherU]) {
#pragma unroll
      for (int u = 0; u < kGatherU; ++u)
        if (v[u] != ~0ull) atomicAdd(&h[bin_of(v[u])], 1u);
    });
    __syncthreads();
    FC_TR(29);
    // only the bins the bracket's span uses (the sample sized sbin for 2^cbins_log2 of them:
    // a batched launch flushes fewer coalesced atomics per workgroup)
    const uint32_t nb = min((uint32_t)kHistBins, ((t_hi - t_lo) >> sbin) + 1u);
    flush_hist(a.W.chist + (blockIdx.x % kCandShards) * kHistBins, h, nb);   // this workgroup's shard
    FC_TR(27);
    if (!last_block_arrive_tree(a.W.tick + 2 * kTickWords, gridDim.x, blockIdx.x, &s_flag)) return;
    // the last arriver sums the shards (every load first, then the clearing stores: their next
    // use is the next call's atomics, after this launch), finds beta and stores it
    constexpr int kPer = kHistBins / kBlock;
    uint32_t t[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) t[j] = 0;
#pragma unroll
    for (int sh = 0; sh < kCandShards; ++sh)
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if ((uint32_t)(j * kBlock + tid) < nb) t[j] += ld_agent(&a.W.chist[sh * kHistBins + j * kBlock + tid]);
#pragma unroll
    for (int j = 0; j < kPer; ++j) h[j * kBlock + tid] = t[j];
    __syncthreads();
    find_rank_desc(h, rank, s_tmp, s_out);
    if (tid == 0) {
      st_agent(&S->rb_beta, s_out[0]); st_agent(&S->rb_rin, s_out[1]);
      st_agent(&S->rb_cnt, h[s_out[0]]);
    }
    for (int sh = 0; sh < kCandShards; ++sh)
      for (uint32_t b = tid; b < nb; b += kBlock) a.W.chist[sh * kHistBins + b] = 0u;
    FC_TR(28);
    return;
  } else {
    // ---- gather bin beta into the LDS list, then into the small list ----
    if (!retry && rank > 0) {
      if (tid == 0) s_cnt = 0;
      __syncthreads();
      for_cands(false, [&](const uint64_t (&v)[kGatherU]) {
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
          if (v[u] != ~0ull && bin_of(v[u]) == beta) {
            const uint32_t q = atomicAdd(&s_cnt, 1u);
            if (q < (uint32_t)kSmallCap) sv[q] = v[u];
          }
        }
      });
      __syncthreads();
      if (tid == 0 && s_cnt) s_base = atomicAdd(&S->small_n, min(s_cnt, (uint32_t)kSmallCap));
      __syncthreads();
      const uint32_t mine = min(s_cnt, (uint32_t)kSmallCap);
      for (uint32_t q = tid; q < mine; q += kBlock)
        if (s_base + q < (uint32_t)kSmallCap) st_agent(&a.W.small[s_base + q], sv[q]);
    }
    FC_TR(11);
    // dense: zero this range's candidates binned below beta (below T64 whatever it is); with
    // rank == 0 every candidate is slack
    const uint64_t imask = (1ull << a.ib) - 1;
    if (a.dense && walk) {
      const uint32_t below = rank > 0 ? beta : 0xffffffffu;
      for_cands(rank > 0, [&](const uint64_t (&v)[kGatherU]) {
#pragma unroll
        for (int u = 0; u < kGatherU; ++u)
          if (v[u] != ~0ull && bin_of(v[u]) < below) a.dense[v[u] & imask] = 0.0f;
      });
    }
    if (!last_block_arrive_tree(a.W.tick + kTickWords, gridDim.x, blockIdx.x, &s_flag, 16)) return;
    FC_TR(12);
    // ---- last workgroup: T64 = the r_in-th largest of bin beta, the header, the dense slack of
    // bin beta, self-cleaning ----
    uint64_t T = 0;
    uint32_t first_below = 0, list_n = 0;                 // sv[first_below, list_n): below T
    bool sorted = false;
    if (retry) {
      T = 0;
    } else if (a.k == 0) {
      T = kSelectNothing;
    } else if (rank == 0) {
      T = ((uint64_t)t_hi + 1) << a.ib;                   // exactly the definite set
    } else if (cnt_beta <= (uint32_t)kBlock) {
      // thread i ranks candidate i by counting the larger ones (comps are unique)
      uint64_t mine = 0;
      if ((uint32_t)tid < cnt_beta) { mine = ld_agent(&a.W.small[tid]); sv[tid] = mine; }
      __syncthreads();
      if ((uint32_t)tid < cnt_beta) {
        uint32_t larger = 0;
        for (uint32_t j = 0; j < cnt_beta; ++j) larger += sv[j] > mine ? 1u : 0u;
        if (larger == r_in - 1) s_T = mine;
      }
      __syncthreads();
      T = s_T;
      list_n = cnt_beta;
    } else {
      uint32_t P2 = 1;
      while (P2 < cnt_beta) P2 <<= 1;
      for (uint32_t i = tid; i < P2; i += kBlock) sv[i] = i < cnt_beta ? ld_agent(&a.W.small[i]) : 0ull;
      __syncthreads();
      bitonic_desc(sv, P2);
      T = sv[r_in - 1];
      first_below = r_in; list_n = cnt_beta; sorted = true;
    }
    // another launch's timed-out wait (sticky err: the sample's pilot poll) makes the call retry
    const bool other_err = ld_agent(&S->err) != 0u;
    const uint32_t status = retry || other_err ? (uint32_t)FC_STATUS_RETRY_EXACT : (uint32_t)FC_STATUS_OK;
    FC_TR(14);
    if (a.dense && status == FC_STATUS_OK && rank > 0) {
      for (uint32_t i = (sorted ? first_below : 0u) + tid; i < list_n; i += kBlock) {
        const uint64_t v = sv[i];
        if (v < T) a.dense[v & imask] = 0.0f;
      }
    }
    if (!rbin)                                            // the compaction's bins, for the next call
      for (int b = tid; b < kHistBins; b += kBlock) a.W.chist[b] = 0;
    if (tid == 0) {
      a.hdr->thresh = T;
      a.hdr->n_entries = n_ent;
      if (status != FC_STATUS_OK) a.hdr->status = status;
      a.hdr->n_definite = n_hi;
      a.hdr->n_cand = n_cand;
      S->small_n = 0; S->err = 0;
      S->fz_seq += 1u;               // k_fused_mag: the next launch publishes fz_seq + 1
    }
    FC_TR(15);
  }
}
template __global__ void k_resolve<true>(ResolveArgs);
template __global__ void k_resolve<false>(ResolveArgs);

// --------------------------------------------------------------------------------------
// k_beta: the head of k_resolve<false> alone, for a lone fused packet encode whose gather and
// finish run inside its decode (fc_topk_encode_decode -> k_decode_res): from the shard totals
// and the candidate histogram k_fused_mag filled, the bin beta holding rank r = k - #(key >
// t_hi), the rank inside it and its count -> S->rb_*; rb_flags bit 0 = retry (the exact path),
// bit 1 = rank 0 (T64 = (t_hi + 1) << ib: every candidate is slack).  One workgroup.
// --------------------------------------------------------------------------------------
// k_beta also closes what needs no decode: the header's counts, T64 and the status when no entry
// of bin beta is left to rank (rank 0: T64 = (t_hi + 1) << ib; retry: RETRY), and the state the
// fused launch leaves (candidate histogram cleared, err reset, fz_seq bumped) — so the decode's
// workgroups take no last-arriver ticket: the one that stores bin beta's last entry finishes T64.
__global__ __launch_bounds__(kBlock) void k_beta(ResolveArgs a) {
  __shared__ uint32_t h[kHistBins];
  __shared__ uint32_t s_tmp[8], s_out[4], s_tot[2];
  beta_body<false>(a.W, a.k, h, s_tmp, s_out, s_tot);
  TopkState* S = a.W.st;
  const int tid = threadIdx.x;
  for (int b = tid; b < kHistBins; b += kBlock) a.W.chist[b] = 0;    // read by beta_body (barrier)
  if (tid == 0) {
    const uint32_t flags = S->rb_flags, n_ent = S->rb_nent, n_cand = S->rb_ncand;
    a.hdr->n_entries = n_ent;
    a.hdr->n_definite = n_ent - n_cand;
    a.hdr->n_cand = n_cand;
    if (flags & 1u) { a.hdr->thresh = 0; a.hdr->status = FC_STATUS_RETRY_EXACT; }
    else if (flags & 2u) a.hdr->thresh = ((uint64_t)S->t_hi + 1) << a.ib;
    S->err = 0;
    S->small_n = 0; S->small_done = 0;
    S->fz_seq += 1u;               // k_fused_mag: the next launch publishes fz_seq + 1
  }
}


// --------------------------------------------------------------------------------------
// k_engine: exact pipeline — one 12-bit radix (or final LDS-sort) pass of the selection of
// the k-th largest comp over g itself.  Runs BEFORE the compaction (which then lists exactly
// comp >= T64).  Used for trivial k and whenever the sampled bracket reports RETRY.
// --------------------------------------------------------------------------------------
struct EngineArgs {
  const float* g;
  uint64_t n;
  uint32_t ib;
  uint32_t first;
  uint64_t k;
  uint64_t seed, offset;
  fc_packet_hdr* hdr;
  WsPtrs W;
  HdrInit HI;
};

struct EngState {
  uint64_t prefix;
  uint32_t shift, rank, matched, done, status;
  uint64_t result;
};

template <int KM>
__global__ __launch_bounds__(kBlock) void k_engine(EngineArgs a) {
  __shared__ uint64_t sv[kSmallCap];                      // 32 KiB, also the histogram
  __shared__ uint32_t s_tmp[8], s_out[4], s_flag, s_cnt, s_base;
  uint32_t* h = reinterpret_cast<uint32_t*>(sv);
  TopkState* S = a.W.st;
  const int tid = threadIdx.x;
  // every field assigned on every path (a partially initialised state once let hipcc fold
  // a rank into an undefined register: DESIGN.md §Lessons)
  const uint32_t top = 31 + a.ib;
  const EngState E0 =
      a.first ? EngState{0ull, top, (uint32_t)a.k, (uint32_t)a.n,
                         (a.k == 0 || a.k >= a.n) ? 1u : 0u, (uint32_t)FC_STATUS_OK,
                         a.k == 0 ? kSelectNothing : 0ull}
              : EngState{S->e_prefix, S->e_shift, S->e_rank, S->e_matched, S->e_done,
                         S->e_status, S->e_prefix};
  EngState E = E0;
  if (!a.first && E.done) return;                         // resolved by an earlier pass

  const bool collect = !E.done && E.matched <= (uint32_t)kSmallCap;
  const uint32_t D = E.shift < (uint32_t)kHistBits ? E.shift : (uint32_t)kHistBits;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t hi_part = E.prefix >> E.shift;
  if (!E.done) {
    for (int b = tid; b < kHistBins; b += kBlock) h[b] = 0;
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    if (!collect) {
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < a.n; i += stride) {
        const uint64_t v = comp_of(key1<KM>(a.g[i], i, a.seed, a.offset), (uint32_t)i, a.ib);
        if ((v >> E.shift) == hi_part)
          atomicAdd(&h[(uint32_t)(v >> (E.shift - D)) & ((1u << D) - 1)], 1u);
      }
      __syncthreads();
      for (int b = tid; b < kHistBins; b += kBlock)
        if (h[b]) atomicAdd(&a.W.ehist[b], h[b]);
    } else {
      uint32_t mine = 0;
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < a.n; i += stride) {
        const uint64_t v = comp_of(key1<KM>(a.g[i], i, a.seed, a.offset), (uint32_t)i, a.ib);
        mine += (v >> E.shift) == hi_part ? 1u : 0u;
      }
      const uint32_t off = mine ? atomicAdd(&s_cnt, mine) : 0u;
      __syncthreads();
      if (tid == 0 && s_cnt) s_base = atomicAdd(&S->small_n, s_cnt);
      __syncthreads();
      if (mine) {
        uint32_t pos = s_base + off;
        for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < a.n; i += stride) {
          const uint64_t v = comp_of(key1<KM>(a.g[i], i, a.seed, a.offset), (uint32_t)i, a.ib);
          if ((v >> E.shift) == hi_part && pos < (uint32_t)kSmallCap) st_agent(&a.W.small[pos++], v);
        }
      }
    }
  }
  if (!last_block_arrive_sc1(&S->e_ticket, gridDim.x, &s_flag)) return;

  // ---- last workgroup: advance the state ----
  if (!E.done) {
    if (!collect) {
      __syncthreads();
      load_clear_hist(a.W.ehist, h);
      __syncthreads();
      find_rank_desc(h, E.rank, s_tmp, s_out);
      const uint32_t d = s_out[0];
      E.prefix |= (uint64_t)d << (E.shift - D);
      E.shift -= D;
      E.rank = s_out[1];
      E.matched = h[d];
      if (E.shift == 0) { E.done = 1; E.result = E.prefix; }
    } else {
      const uint32_t m = E.matched;
      uint32_t P2 = 1;
      while (P2 < m) P2 <<= 1;
      __syncthreads();
      for (uint32_t i = tid; i < P2; i += kBlock) sv[i] = i < m ? ld_agent(&a.W.small[i]) : 0ull;
      __syncthreads();
      bitonic_desc(sv, P2);
      if (E.rank >= 1 && E.rank <= m) E.result = sv[E.rank - 1];
      else E.status = FC_STATUS_TIMEOUT;   // inconsistent state: never expected
      E.done = 1;
      __syncthreads();
    }
  }
  if (tid == 0) {
    if (a.first) write_hdr_static(a.hdr, a.HI);   // sole hdr writer of this launch
    S->e_prefix = E.prefix; S->e_shift = E.shift; S->e_rank = E.rank; S->e_matched = E.matched;
    S->e_done = E.done; S->e_status = E.status;
    S->e_ticket = 0; S->small_n = 0;
    if (E.done) {
      a.hdr->thresh = E.result;
      a.hdr->lower = E.result;
      a.hdr->n_entries = (uint32_t)a.k;           // exactly comp >= T64 gets listed
      if (E.status != FC_STATUS_OK) a.hdr->status = E.status;
      // k_compact runs next and lists exactly comp >= T64
      S->L64 = E.result; S->t_lo = (uint32_t)(E.result >> a.ib); S->t_hi = 0xffffffffu;
      S->cand_on = 0; S->sbin = 0; S->n_cand = 0; S->cand_over = 0; S->ent_over = 0;
    }
  }
}

// --------------------------------------------------------------------------------------
// explicit instantiations used by fc_capi.hip
// --------------------------------------------------------------------------------------
template __global__ void k_sample1<kKeyMag, false>(const float*, SamplePlan, uint64_t, uint64_t, WsPtrs, uint32_t, fc_packet_hdr*, HdrInit, const fc_encode_job*, uint64_t);
template __global__ void k_sample1<kKeyMag, true>(const float*, SamplePlan, uint64_t, uint64_t, WsPtrs, uint32_t, fc_packet_hdr*, HdrInit, const fc_encode_job*, uint64_t);
template __global__ void k_engine<kKeyMag>(EngineArgs);
template __global__ void k_engine<kKeyPhilox>(EngineArgs);

}  // namespace fc
