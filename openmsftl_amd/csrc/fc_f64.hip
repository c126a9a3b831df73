// fc_f64.hip — float64 gradients (MI355X, gfx950).
//
// The reference reaches the codec with float64 gradients after RandomGaussian with
// noise_scale == 0 (attack_models.py:105-106); G then takes that dtype (aggregation.py:61) and
// every codec and the FedAVG reduce compute in float64.  This file gives that path its own
// kernels (all HBM-bound, nothing here is a contraction):
//
//   k_engine64 + k_select_dense64   'top' / native 'rand' (compression.py:31-45): exact radix
//                                   select of the k-th largest comp = key64 << 32 | idx (95 bits,
//                                   <= 8 passes of 12 bits, an LDS sort once <= 2048 remain),
//                                   then one pass q = comp >= T ? g : +0.  Same tie rule as the
//                                   fp32 path (highest index first = stable argsort reversed).
//   k_mask_dense64                  'rand' (host permutation mask) and 'dropout-*': the
//                                   reference's exact float64 arithmetic, q = g * mask and
//                                   (g * mask) / p (compression.py:47-60; mask from the host or
//                                   native Philox Bernoulli, the same draws as the fp32 path).
//   k_wsum64 / k_div_scalar64       gar.py:44 when G or the weights are float64:
//                                   acc = +0; acc = fl64(acc + fl64(double(g_i) * w_i)) in row
//                                   order (no FMA), and np.mean's count division.
#include "fc_state.h"

namespace fc {

typedef unsigned __int128 u128;
constexpr int kSmallCap64 = 2048;            // collected comps sorted in LDS (32 KiB)
constexpr uint64_t kNanKey64 = 0x7ff0000000000001ull;   // every NaN above +inf

__device__ __forceinline__ uint64_t mag_key64(double x) {
  const uint64_t u = (uint64_t)__double_as_longlong(x) & 0x7fffffffffffffffull;
  return u > 0x7ff0000000000000ull ? kNanKey64 : u;
}
template <int KM>
__device__ __forceinline__ u128 comp64(const double* g, uint64_t i, uint64_t seed, uint64_t off) {
  const uint64_t key = KM == kKeyMag ? mag_key64(g[i]) : (uint64_t)(philox_word(i, seed, off) >> 1);
  return ((u128)key << 32) | (u128)(uint32_t)i;
}

// Engine state, in the encoder workspace's state block after TopkState.
struct Eng64State {
  uint64_t p_hi, p_lo;                       // resolved high bits of T (u128 as two halves)
  uint32_t shift, rank, matched, done, status, ticket, small_n;
  uint32_t gen;                              // k_resolve64: bumped once T is published
};
static_assert(sizeof(TopkState) + sizeof(Eng64State) <= 1024, "state block");
constexpr uint64_t kEng64Off = 768;
static_assert(sizeof(TopkState) <= kEng64Off, "Eng64State offset");

struct Engine64Args {
  const double* g;
  uint64_t n, k, seed, offset;
  uint32_t first, key_mode;
  Eng64State* E;
  uint32_t* hist;                            // 4096 bins (global)
  u128* small;                               // kSmallCap64 collected comps
};

__device__ __forceinline__ u128 u128_of(uint64_t hi, uint64_t lo) { return ((u128)hi << 64) | lo; }

// Descending bitonic sort of P2 (power of two) u128 values in LDS.
__device__ void bitonic_desc128(u128* sv, uint32_t P2) {
  for (uint32_t size = 2; size <= P2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < P2 / 2; t += blockDim.x) {
        const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
        const bool desc = (i & size) == 0;
        const u128 x = sv[i], y = sv[j];
        if ((x < y) == desc) { sv[i] = y; sv[j] = x; }
      }
      __syncthreads();
    }
  }
}

// Rank-from-the-top bin of an LDS histogram (256 threads): fc_topk.hip's find_rank_desc (one
// wave searches the owning thread's 16 bins).
__device__ __forceinline__ void find_rank_desc64(const uint32_t* h, uint32_t rank1, uint32_t* s_tmp,
                                                 uint32_t* s_out) {
  find_rank_desc(h, rank1, s_tmp, s_out);
}

// One radix pass (or the final collect + LDS sort) of the k-th largest 95-bit comp.
template <int KM>
__global__ __launch_bounds__(kBlock) void k_engine64(Engine64Args a) {
  __shared__ u128 sv[kSmallCap64];                          // 32 KiB, also the histogram
  __shared__ uint32_t s_tmp[8], s_out[4], s_flag, s_cnt, s_base;
  uint32_t* h = reinterpret_cast<uint32_t*>(sv);
  Eng64State* E = a.E;
  const int tid = threadIdx.x;
  uint64_t p_hi = 0, p_lo = 0;
  uint32_t shift = 96, rank = (uint32_t)a.k, matched = (uint32_t)a.n;
  uint32_t done = (a.k == 0 || a.k >= a.n) ? 1u : 0u, status = FC_STATUS_OK;
  if (!a.first) {
    p_hi = E->p_hi; p_lo = E->p_lo; shift = E->shift; rank = E->rank; matched = E->matched;
    done = E->done; status = E->status;
    if (done) return;                                       // resolved by an earlier pass
  }
  const u128 prefix = u128_of(p_hi, p_lo);
  const bool collect = !done && matched <= (uint32_t)kSmallCap64;
  const uint32_t D = shift < (uint32_t)kHistBits ? shift : (uint32_t)kHistBits;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const u128 hi_part = shift >= 128 ? (u128)0 : (prefix >> shift);
  auto match = [&](const u128& v) { return shift >= 128 ? true : (v >> shift) == hi_part; };
  if (!done) {
    for (int b = tid; b < kHistBins; b += kBlock) h[b] = 0;
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    if (!collect) {
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < a.n; i += stride) {
        const u128 v = comp64<KM>(a.g, i, a.seed, a.offset);
        if (match(v)) atomicAdd(&h[(uint32_t)(v >> (shift - D)) & ((1u << D) - 1)], 1u);
      }
      __syncthreads();
      for (int b = tid; b < kHistBins; b += kBlock)
        if (h[b]) atomicAdd(&a.hist[b], h[b]);
    } else {
      uint32_t mine = 0;
      for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < a.n; i += stride)
        mine += match(comp64<KM>(a.g, i, a.seed, a.offset)) ? 1u : 0u;
      const uint32_t off = mine ? atomicAdd(&s_cnt, mine) : 0u;
      __syncthreads();
      if (tid == 0 && s_cnt) s_base = atomicAdd(&E->small_n, s_cnt);
      __syncthreads();
      if (mine) {
        uint32_t pos = s_base + off;
        for (uint64_t i = (uint64_t)blockIdx.x * kBlock + tid; i < a.n; i += stride) {
          const u128 v = comp64<KM>(a.g, i, a.seed, a.offset);
          if (match(v) && pos < (uint32_t)kSmallCap64) {
            uint64_t* d = reinterpret_cast<uint64_t*>(&a.small[pos++]);
            st_agent(d, (uint64_t)v);
            st_agent(d + 1, (uint64_t)(v >> 64));
          }
        }
      }
    }
  }
  if (!last_block_arrive_sc1(&E->ticket, gridDim.x, &s_flag)) return;
  // ---- last workgroup: advance the state ----
  u128 result = prefix;
  if (!done) {
    if (!collect) {
      __syncthreads();
      load_clear_hist(a.hist, h);
      __syncthreads();
      find_rank_desc64(h, rank, s_tmp, s_out);
      const uint32_t d = s_out[0];
      result = prefix | ((u128)d << (shift - D));
      shift -= D;
      rank = s_out[1];
      matched = h[d];
      if (shift == 0) done = 1;
    } else {
      const uint32_t m = matched;
      uint32_t P2 = 1;
      while (P2 < m) P2 <<= 1;
      __syncthreads();
      for (uint32_t i = tid; i < P2; i += kBlock) {
        u128 v = 0;
        if (i < m) {
          const uint64_t* s = reinterpret_cast<const uint64_t*>(&a.small[i]);
          v = u128_of(ld_agent(s + 1), ld_agent(s));
        }
        sv[i] = v;
      }
      __syncthreads();
      bitonic_desc128(sv, P2);
      if (rank >= 1 && rank <= m) result = sv[rank - 1];
      else status = FC_STATUS_TIMEOUT;                         // inconsistent state: never expected
      done = 1;
      __syncthreads();
    }
  }
  if (tid == 0) {
    E->p_hi = (uint64_t)(result >> 64); E->p_lo = (uint64_t)result;
    E->shift = shift; E->rank = rank; E->matched = matched; E->done = done; E->status = status;
    E->ticket = 0; E->small_n = 0;
  }
}

// q = comp >= T ? g : +0 (compression.py:33-37: zeros_like, then the selected copies).
template <int KM>
__global__ __launch_bounds__(kBlock) void k_select_dense64(const double* __restrict__ g, uint64_t n,
                                                           uint64_t k, uint64_t seed, uint64_t off,
                                                           const Eng64State* E, double* out) {
  const bool none = k == 0, all = k >= n;
  const u128 T = u128_of(E->p_hi, E->p_lo);
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const bool keep = all || (!none && comp64<KM>(g, i, seed, off) >= T);
    out[i] = keep ? g[i] : 0.0;
  }
}

// The reference's NumPy runs on x86 (SSE2): an invalid operation on non-NaN operands (inf * 0,
// 0 / 0) yields the "default NaN" 0xFFF8000000000000, and a NaN operand propagates quieted.
// These helpers give the same bits (the GPU's own default NaN is 0x7FF8000000000000).
__device__ __forceinline__ double quiet(double x) {
  return __longlong_as_double(__double_as_longlong(x) | 0x0008000000000000ll);
}
constexpr long long kX86DefaultNaN = (long long)0xFFF8000000000000ull;
__device__ __forceinline__ double x86_mul(double a, double b) {
  if (a != a) return quiet(a);
  if (b != b) return quiet(b);
  const double r = __dmul_rn(a, b);
  return r != r ? __longlong_as_double(kX86DefaultNaN) : r;
}
__device__ __forceinline__ double x86_div(double a, double b) {
  if (a != a) return quiet(a);
  if (b != b) return quiet(b);
  const double r = __ddiv_rn(a, b);
  return r != r ? __longlong_as_double(kX86DefaultNaN) : r;
}

// Mask codecs on float64: bit i of the keep mask from the host (mask_bits) or from the same
// Philox Bernoulli words as the fp32 path (word < bern_thr).
//   mode 0 ('rand'):             q = keep ? g : +0                 (zeros_like + copies)
//   mode 1 ('dropout-biased'):   q = g * double(keep)              (compression.py:52)
//   mode 2 ('dropout-unbiased'): q = (g * double(keep)) / p        (compression.py:59-60)
// T = float: a float32 gradient promoted exactly (NumPy's float32 * int64 mask -> float64), so
// fp32 'dropout-*' also reproduces g * 0 = -0.0 for negative g and the x86 NaN rules.
// Thread = (256-element segment, lane): elements seg*256 + j*64 + lane, j = 0..3 — the four
// words of ONE Philox block (fc_common.h's element map), coalesced across the wave.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_mask_dense64(const T* __restrict__ g, uint64_t n,
                                                         const uint32_t* __restrict__ mask,
                                                         uint64_t bern_thr, uint64_t seed,
                                                         uint64_t off, int mode, double p,
                                                         double* out) {
  const uint64_t slots = (n + 255) / 256 * 64;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < slots; t += stride) {
    const uint64_t seg = t >> 6;
    const uint32_t lane = (uint32_t)(t & 63);
    uint4 r = make_uint4(0u, 0u, 0u, 0u);
    if (!mask) r = philox_seg(seg, lane, seed, off);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t i = seg * 256 + (uint64_t)j * 64 + lane;
      if (i >= n) break;
      const uint32_t word = j == 0 ? r.x : j == 1 ? r.y : j == 2 ? r.z : r.w;
      const bool keep = mask ? ((mask[i >> 5] >> (i & 31)) & 1u) != 0 : (uint64_t)word < bern_thr;
      const double x = (double)g[i];
      double q;
      if (mode == 0) {
        q = keep ? x : 0.0;
      } else {
        q = x86_mul(x, keep ? 1.0 : 0.0);
        if (mode == 2) q = x86_div(q, p);
      }
      out[i] = q;
    }
  }
}

// gar.py:44 with float64 arithmetic: out = fl64(... fl64(+0 + fl64(double(g_0) w_0)) ...), rows
// float32 (rows_f64 = 0, promoted exactly) or float64; acc_in continues the sum held in out.
__global__ __launch_bounds__(kBlock) void k_wsum64(const void* const* rows, int rows_f64,
                                                   const double* w, int m, uint64_t n,
                                                   double* out, int acc_in) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
    double acc = acc_in ? out[e] : 0.0;
    for (int r = 0; r < m; ++r) {
      const double x = rows_f64 ? static_cast<const double*>(rows[r])[e]
                                : (double)static_cast<const float*>(rows[r])[e];
      acc = __dadd_rn(acc, __dmul_rn(x, w[r]));
    }
    out[e] = acc;
  }
}

__global__ __launch_bounds__(kBlock) void k_div_scalar64(double* x, uint64_t n, double d) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride)
    x[e] = __ddiv_rn(x[e], d);
}

// --------------------------------------------------------------------------------------
// Sampled fast path for magnitude keys (fc_topk_dense_f64_sampled): the fp32 design on the
// 31-bit HIGH key hk(x) = (|x| bits) >> 32 of each double (exponent + 20 mantissa bits;
// key32 = mag_key of it, a non-decreasing map of the 95-bit comp = key64 << 32 | idx):
//   k_fused64     ONE launch: its first workgroups run k_sample1's stratified sample + pilot
//                 window over hk (sample_body<double>) -> bracket [t_lo, t_hi] of key32 around
//                 the k-th key, published to the others; each of those is a chunk of ONE
//                 streaming pass, 8N read + 8N written: q = key32 >= t_lo ? g : +0; definite
//                 (key32 > t_hi) and candidate counts into the sharded totals; each candidate's
//                 exact comp into its chunk's slot, its bin into the histogram
//   k_resolve64   rank r = k - #definite among the candidates: every workgroup finds the bin
//                 beta holding it (the histogram, from L2) and gathers its chunks' candidates
//                 in beta (a chunk whose candidates overflowed its slot is rescanned from
//                 g); the last arriver sorts them (<= 2048, LDS) and picks T, the exact k-th
//                 largest comp; a bracket that missed or a bin beta above 2048 -> RETRY.
//                 q[idx] = +0 for the slack: every workgroup zeroes its candidates binned
//                 below beta (below T whatever T is) in the gather pass, the last arriver the
//                 entries of bin beta below T.  No workgroup waits for another.
// The exact radix engine (<= 8 passes of 8N) stays the fallback and serves native rand-k.
// --------------------------------------------------------------------------------------
constexpr int kC64Slot = 128;                  // candidate comps per chunk (the 2 KB slot)
constexpr uint32_t kResolve64Grid = 256;       // k_resolve64 workgroups at most (co-resident)
constexpr uint64_t kHdr64Off = 896;            // the sample's scratch packet header
static_assert(kEng64Off + sizeof(Eng64State) <= kHdr64Off && kHdr64Off + sizeof(fc_packet_hdr) <= 1024,
              "state block layout");
static_assert(kC64Slot * sizeof(u128) == kCandSlot * sizeof(uint64_t), "candidate slot bytes");

__device__ __forceinline__ uint32_t key32_of(double x) { return mag_key(hikey_f(x)); }

struct Fast64Args {
  const double* g;
  uint64_t n, k;
  uint32_t nchunks, per;       // per: chunks per k_resolve64 workgroup
  TopkState* S;
  Eng64State* E;
  uint32_t* ccnt;              // candidates per chunk (may exceed kC64Slot: overflowed)
  u128* cand;                  // chunk c's candidate comps at [c * kC64Slot, ...)
  uint32_t* chist;             // 4096-bin candidate histogram (zero between calls)
  uint32_t* tick;              // two-level ticket (k_resolve64)
  u128* small;                 // bin beta's candidates (<= kSmallCap64)
  double* out;
  uint32_t* status;            // caller's device word: FC_STATUS_OK / RETRY_EXACT
};

constexpr int FC_F64_DELAY = 90;               // k_fused64's first-round chunks: s_sleep before loading

// One workgroup per 8192-element chunk: 16 double2 per thread, coalesced (element
// base + 2 (i * 256 + tid) + {0, 1}).
constexpr int kI64 = kChunk / (2 * kBlock);     // 16
__device__ __forceinline__ void load64_chunk(const Fast64Args& a, uint32_t chunk, fc_d2v (&x)[kI64]) {
  const uint32_t tid = threadIdx.x;
  const uint64_t base = (uint64_t)chunk * kChunk;
  if (base + kChunk <= a.n) {
    fc_gd2v* gp = (fc_gd2v*)(a.g + base) + tid;
#pragma unroll
    for (int i = 0; i < kI64; ++i) x[i] = __builtin_nontemporal_load(gp + i * kBlock);
  } else {
#pragma unroll
    for (int i = 0; i < kI64; ++i) {
      const uint64_t e = base + 2ull * (i * kBlock + tid);
      x[i].x = e < a.n ? a.g[e] : 0.0;
      x[i].y = e + 1 < a.n ? a.g[e + 1] : 0.0;
    }
  }
}

struct Compact64Shared {
  uint32_t cnt, red[kBlock / 64];
};

// q = key32 >= t_lo ? g : +0 for one loaded chunk; candidates to the chunk's slot and the
// histogram; the chunk's totals into the shards
__device__ __forceinline__ void compact64_body(const Fast64Args& a, uint32_t chunk,
                                               const fc_d2v (&x)[kI64], uint32_t t_lo,
                                               uint32_t t_hi, uint32_t sbin, Compact64Shared& sh) {
  const uint32_t tid = threadIdx.x;
  const uint64_t base = (uint64_t)chunk * kChunk;
  const bool full = base + kChunk <= a.n;
  if (tid == 0) sh.cnt = 0;
  lds_barrier();
  uint32_t listed = 0;
#pragma unroll
  for (int i = 0; i < kI64; ++i) {
    fc_d2v q;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t e = base + 2ull * (i * kBlock + tid) + h;
      const double v = h ? x[i].y : x[i].x;
      const uint32_t key = key32_of(v);
      const bool L = e < a.n && key >= t_lo;
      listed += L ? 1u : 0u;
      if (h) q.y = L ? v : 0.0; else q.x = L ? v : 0.0;
      if (L && key <= t_hi) {
        const uint32_t pos = atomicAdd(&sh.cnt, 1u);
        if (pos < (uint32_t)kC64Slot) {
          const uint64_t key64 = mag_key64(v);
          uint64_t* d = reinterpret_cast<uint64_t*>(&a.cand[(uint64_t)chunk * kC64Slot + pos]);
          d[0] = (key64 << 32) | (uint32_t)e;
          d[1] = key64 >> 32;
        }
        atomicAdd(&a.chist[(key - t_lo) >> sbin], 1u);
      }
    }
    if (full) {
      __builtin_nontemporal_store(q, (fc_d2v*)(a.out + base) + tid + i * kBlock);
    } else {
      const uint64_t e = base + 2ull * (i * kBlock + tid);
      if (e < a.n) a.out[e] = q.x;
      if (e + 1 < a.n) a.out[e + 1] = q.y;
    }
  }
  listed = wave_sum(listed);
  if ((tid & 63) == 0) sh.red[tid >> 6] = listed;
  __syncthreads();
  if (tid == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) tot += sh.red[w];
    if (chunk == 0) *a.status = (uint32_t)FC_STATUS_OK;   // this call's status (k_resolve64)
    a.ccnt[chunk] = sh.cnt;
    atomicAdd(&a.S->shard_ent[chunk % kShards], tot);
    if (sh.cnt) atomicAdd(&a.S->shard_cnd[chunk % kShards], sh.cnt);
  }
}

// k_fused64: k_fused_mag's form for float64 (round 5; before, k_sample64 and k_compact64 were
// two launches): workgroups [0, nsamp) run the sample over the high keys (workgroup 0's
// segments are the pilot, its window published in line-spread copies), every other one is a
// chunk that issues its loads, polls its copy of the 16-B bracket record (tag fz_seq + 1,
// bounded) and streams q.  The sample never waits for a chunk workgroup; a timed-out poll sets
// S->err and k_resolve64 reports RETRY.
union Fused64Shared {
  SampleShared s;
  Compact64Shared c;
};
__global__ __launch_bounds__(kBlock) void k_fused64(Fast64Args a, SamplePlan P, WsPtrs W,
                                                    uint32_t ib, fc_packet_hdr* hdr, HdrInit HI,
                                                    uint32_t nsamp) {
  __shared__ Fused64Shared u;
  __shared__ uint32_t s_b[3];
  const uint32_t pub = sload2(&a.S->fz_seq).x + 1u;      // not written by this launch
  if (blockIdx.x < nsamp) {
    sample_body<kKeyMag, true, double>(a.g, P, 0ull, 0ull, W, ib, hdr, HI, blockIdx.x, nsamp,
                                       true, u.s, pub);
    return;
  }
  const uint32_t chunk = blockIdx.x - nsamp;
  fc_d2v x[kI64];
  if (chunk < 1024u) __builtin_amdgcn_s_sleep(FC_F64_DELAY);   // the sample's loads first
  load64_chunk(a, chunk, x);
  if (threadIdx.x == 0) {
    const uint32_t* rec = &W.pub[(blockIdx.x % kPubCopies) * kPubStride];
    const uint32_t tag = pub | 0x80000000u;
    uint32_t it = 0;
    fc_rec4 r = ld16_agent(rec);
    while (r.w != tag && ++it < kSpinMax) {
      __builtin_amdgcn_s_sleep(4);
      r = ld16_agent(rec);
    }
    if (it >= kSpinMax) st_agent(&a.S->err, 1u);
    s_b[0] = r.x; s_b[1] = r.y; s_b[2] = r.z;
  }
  __syncthreads();
  compact64_body(a, chunk, x, s_b[0], s_b[1], s_b[2], u.c);
}

// fn(comp) for every candidate of this workgroup's chunk range: kTpc64 threads per chunk read
// its candidate slot; a chunk whose candidates overflowed the slot (a dense bracket region, a
// small n's wide bracket) is rescanned from g by the whole workgroup instead.
constexpr uint32_t kTpc64 = 16;
template <typename F>
__device__ __forceinline__ void for_cands64(const Fast64Args& a, uint32_t c0, uint32_t c1,
                                            uint32_t t_lo, uint32_t t_hi, F&& fn) {
  const uint32_t cpr = kBlock / kTpc64;
  for (uint32_t cb = c0; cb < c1; cb += cpr) {
    const uint32_t c = cb + threadIdx.x / kTpc64, q = threadIdx.x % kTpc64;
    uint32_t cnt = c < c1 ? a.ccnt[c] : 0u;
    if (cnt > (uint32_t)kC64Slot) cnt = 0;                 // rescanned below
    for (uint32_t r = q; r < cnt; r += kTpc64) {
      const uint64_t* s = reinterpret_cast<const uint64_t*>(&a.cand[(uint64_t)c * kC64Slot + r]);
      fn(u128_of(s[1], s[0]));
    }
  }
  for (uint32_t c = c0; c < c1; ++c) {
    if (a.ccnt[c] <= (uint32_t)kC64Slot) continue;         // (uniform)
    const uint64_t base = (uint64_t)c * kChunk;
    for (uint32_t r = threadIdx.x; r < (uint32_t)kChunk; r += kBlock) {
      const uint64_t e = base + r;
      if (e >= a.n) break;
      const double v = a.g[e];
      const uint32_t key = key32_of(v);
      if (key >= t_lo && key <= t_hi) fn(((u128)mag_key64(v) << 32) | (u128)(uint32_t)e);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_resolve64(Fast64Args a) {
  __shared__ u128 sv[kSmallCap64];                        // 32 KiB: histogram, then sort
  __shared__ uint32_t s_tmp[8], s_out[4], s_flag, s_cnt, s_base, s_tot[2];
  uint32_t* h = reinterpret_cast<uint32_t*>(sv);
  const int tid = threadIdx.x;
  TopkState* S = a.S;
  const uint32_t c0 = blockIdx.x * a.per, c1 = min(c0 + a.per, a.nchunks);
  uint32_t se = 0, sc = 0;
  if (tid < kShards) { se = S->shard_ent[tid]; sc = S->shard_cnd[tid]; }
  uint32_t hv[kHistBins / kBlock];
#pragma unroll
  for (int j = 0; j < kHistBins / kBlock; ++j) hv[j] = a.chist[j * kBlock + tid];
  const uint32_t t_lo = S->t_lo, t_hi = S->t_hi, sbin = S->sbin;
  if (tid < 64) {
    se = wave_sum(se);
    sc = wave_sum(sc);
    if (tid == 0) { s_tot[0] = se; s_tot[1] = sc; s_cnt = 0; }
  }
#pragma unroll
  for (int j = 0; j < kHistBins / kBlock; ++j) h[j * kBlock + tid] = hv[j];
  __syncthreads();
  const uint32_t n_ent = s_tot[0], n_cand = s_tot[1], n_hi = n_ent - n_cand;
  bool retry = n_cand > n_ent || (uint64_t)n_ent < a.k || (uint64_t)n_hi >= a.k;
  const uint32_t rank = retry ? 0u : (uint32_t)(a.k - n_hi);
  uint32_t beta = 0, r_in = 1, cnt_beta = 0;
  if (!retry) {
    find_rank_desc64(h, rank, s_tmp, s_out);
    beta = s_out[0]; r_in = s_out[1]; cnt_beta = h[beta];
    retry = cnt_beta > (uint32_t)kSmallCap64 || cnt_beta < r_in;
  }
  __syncthreads();                                        // h (sv) is reused below
  if (!retry) {
    // one pass: a candidate binned below beta is below T whatever T is (bins are in key order):
    // zeroed at once; bin beta's candidates go to the small list for the last arriver
    for_cands64(a, c0, c1, t_lo, t_hi, [&](const u128& v) {
      const uint32_t key = (uint32_t)(v >> 64);           // = key64 >> 32: key32 before the clamp
      const uint32_t k32 = key > 0x7f800000u ? kNanKey : key;
      const uint32_t b = (k32 - t_lo) >> sbin;
      if (b < beta) {
        a.out[(uint32_t)v] = 0.0;
      } else if (b == beta) {
        const uint32_t q = atomicAdd(&s_cnt, 1u);
        if (q < (uint32_t)kSmallCap64) sv[q] = v;
      }
    });
    __syncthreads();
    const uint32_t mine = min(s_cnt, (uint32_t)kSmallCap64);
    if (tid == 0 && mine) s_base = atomicAdd(&a.E->small_n, mine);
    __syncthreads();
    for (uint32_t q = tid; q < mine; q += kBlock) {
      if (s_base + q < (uint32_t)kSmallCap64) {
        uint64_t* d = reinterpret_cast<uint64_t*>(&a.small[s_base + q]);
        st_agent(d, (uint64_t)sv[q]);
        st_agent(d + 1, (uint64_t)(sv[q] >> 64));
      }
    }
  }
  // no workgroup waits for another: the last arriver finishes the call alone
  if (!last_block_arrive_tree(a.tick, gridDim.x, blockIdx.x, &s_flag)) return;
  // ---- last workgroup: T = the r_in-th largest of bin beta, the slack of bin beta, status,
  // self-cleaning ----
  const bool err = ld_agent(&S->err) != 0u;
  const uint32_t got = ld_agent(&a.E->small_n);
  retry = retry || err || got != cnt_beta;
  if (!retry) {
    uint32_t P2 = 1;
    while (P2 < cnt_beta) P2 <<= 1;
    for (uint32_t i = tid; i < P2; i += kBlock) {
      u128 v = 0;
      if (i < cnt_beta) {
        const uint64_t* s = reinterpret_cast<const uint64_t*>(&a.small[i]);
        v = u128_of(ld_agent(s + 1), ld_agent(s));
      }
      sv[i] = v;
    }
    __syncthreads();
    bitonic_desc128(sv, P2);
    // T = sv[r_in - 1]: the entries after it are the slack of bin beta
    for (uint32_t i = r_in + tid; i < cnt_beta; i += kBlock) a.out[(uint32_t)sv[i]] = 0.0;
  }
  for (int b = tid; b < kHistBins; b += kBlock) st_agent(&a.chist[b], 0u);
  if (tid == 0) {
    const uint32_t st = retry ? (uint32_t)FC_STATUS_RETRY_EXACT : (uint32_t)FC_STATUS_OK;
    a.E->small_n = 0;
    S->err = 0;
    S->fz_seq += 1u;                                      // k_fused64: the next launch's tag
    atomicMax(a.status, st);                              // (k_fused64 reset it to OK)
  }
}

template __global__ void k_engine64<kKeyMag>(Engine64Args);
template __global__ void k_engine64<kKeyPhilox>(Engine64Args);
template __global__ void k_select_dense64<kKeyMag>(const double*, uint64_t, uint64_t, uint64_t, uint64_t, const Eng64State*, double*);
template __global__ void k_select_dense64<kKeyPhilox>(const double*, uint64_t, uint64_t, uint64_t, uint64_t, const Eng64State*, double*);

}  // namespace fc
