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
  uint32_t shift, rank, matched, done, status, ticket, small_n, pad_;
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

// Rank-from-the-top bin of an LDS histogram (256 threads): see fc_topk.hip find_rank_desc.
__device__ void find_rank_desc64(const uint32_t* h, uint32_t rank1, uint32_t* s_tmp, uint32_t* s_out) {
  const int t = threadIdx.x;
  constexpr int per = kHistBins / kBlock;
  const int top = kHistBins - 1 - per * t;
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < per; ++b) sum += h[top - b];
  __syncthreads();
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

template __global__ void k_engine64<kKeyMag>(Engine64Args);
template __global__ void k_engine64<kKeyPhilox>(Engine64Args);
template __global__ void k_select_dense64<kKeyMag>(const double*, uint64_t, uint64_t, uint64_t, uint64_t, const Eng64State*, double*);
template __global__ void k_select_dense64<kKeyPhilox>(const double*, uint64_t, uint64_t, uint64_t, uint64_t, const Eng64State*, double*);

}  // namespace fc
