// fc_qsgd.hip — QSGD stochastic quantiser (the 'qsgd' codec of compression.py:62-74) for
// MI355X (gfx950).  SURVEY.md §8(f) row 2: the reference raises NotImplementedError and keeps
// the formula only as a comment, so this codec is opt-in and "parity unpinned" with respect to
// the reference; it is pinned to oracle/qsgd_oracle.py, which restates the comment:
//
//   s = 2^num_bits,  tau = 1 + min(sqrt(d)/s, d/s^2),  norm = ||g||_2
//   q_i = sign(g_i) * norm / (s * tau) * floor(s * |g_i| / norm + U_i),  U_i ~ U[0, 1)
//
// (Alistarh et al., "QSGD", NeurIPS 2017; the reference's comment divides by tau, so
// E[q] = g / tau.)  Exact arithmetic of this build, shared with the oracle:
//   norm  = sqrt(sum of g_i^2 in fp64), the sum in a fixed order (k_qsgd_norm), stored as a
//           double in the header's `p` field;
//   U_i   = h_i * 2^-16, h_i = 16-bit half (i & 1) of Philox word (i >> 1) of the LINEAR map
//           (counter block i >> 3: one Philox-4x32-10 block dithers 8 elements;
//           oracle/philox.py linear_words; not the segment map of philox_word);
//   l_i   = floor(fl32(fl32(|g_i| * c) + U_i))   in [0, s]; 0 when not finite;
//           c = fl32(fl64(s / norm)); when that overflows (a norm below s / FLT_MAX) the same
//           formula in fp64 with c = fl64(s / norm).  (The quantise pass was VALU-bound: a
//           per-element fp64 division and two Philox blocks per 8 elements took 176-183 us at
//           128 M; fp32 arithmetic and one block per 8 elements, see profiles/r04_*qsgd*);
//   code  = signbit(g_i) << (W - 1) | l_i,  W = 4 (bits <= 2), 8 (<= 6), 16 (<= 14) bits,
//           packed little-endian, 32 / W codes per uint32;
//   value = (float)(+-(norm / (s * tau)) * l_i)   (fp64 product, one rounding to fp32).
// Bytes: encode 8N (norm pass + quantise pass) + N W / 8; decode N W / 8 + 4N.
#include "fc_state.h"

namespace fc {

constexpr int kQsgdNormGrid = 1024;            // fixed: the fp64 sum order depends on it
constexpr int kQsgdElems = 8;                  // elements per thread per step (quant/decode)
constexpr int kQsgdNormUnroll = 2;             // float4 loads in flight per thread (norm pass)
// (Plain cache-allocating loads, so that a back-to-front quantise pass could re-read the norm
// pass's tail from the Infinity Cache, measured slower: norm 98 -> 145 us at 128 M, and the
// quantise no faster; profiles/r04_ab_qsgd.jsonl.)

__host__ __device__ inline int qsgd_width(int bits) { return bits <= 2 ? 4 : bits <= 6 ? 8 : 16; }

struct QsgdParams {                            // from the header (decode) or the encode args
  double norm, scale;                          // scale = norm / (s * tau)
  double s, c;                                 // c = s / norm
  float s32, c32;                              // fl32 of both (c32 = +inf: use the fp64 form)
  int width;
};

__device__ __forceinline__ double qsgd_tau(double d, double s) {
  const double a = sqrt(d) / s, b = d / (s * s);
  return 1.0 + (a < b ? a : b);
}

// ---- pass 1: ||g||_2 (fp64, fixed order), header -------------------------------------------
__global__ __launch_bounds__(kBlock) void k_qsgd_norm(const float* __restrict__ g, uint64_t n,
                                                      int bits, uint64_t seed, uint64_t offset,
                                                      double* partial, uint32_t* ticket,
                                                      fc_packet_hdr* hdr) {
  __shared__ double s_red[kBlock / 64];
  __shared__ uint32_t s_flag;
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  double acc = 0.0;
  const uint64_t n4 = n / 4, stride = (uint64_t)gridDim.x * kBlock;
  // kQsgdNormUnroll float4 loads in flight per thread, the additions in a fixed per-thread
  // order: 2 loads 89 us per 128 M pass, 1 or 4 loads 96-97 us, 2 loads on grids of 512 / 2048
  // workgroups 94 / 102 us (profiles/r05_ab_qsgd.jsonl)
  uint64_t q = (uint64_t)blockIdx.x * kBlock + tid;
  for (; q + (kQsgdNormUnroll - 1) * stride < n4; q += kQsgdNormUnroll * stride) {
    float4 v[kQsgdNormUnroll];
#pragma unroll
    for (int u = 0; u < kQsgdNormUnroll; ++u) v[u] = load4_full(g + 4 * (q + u * stride));
#pragma unroll
    for (int u = 0; u < kQsgdNormUnroll; ++u) {
      acc += (double)v[u].x * v[u].x; acc += (double)v[u].y * v[u].y;
      acc += (double)v[u].z * v[u].z; acc += (double)v[u].w * v[u].w;
    }
  }
  for (; q < n4; q += stride) {
    const float4 v = load4_full(g + 4 * q);
    acc += (double)v.x * v.x; acc += (double)v.y * v.y;
    acc += (double)v.z * v.z; acc += (double)v.w * v.w;
  }
  if (blockIdx.x == 0 && tid < (int)(n - 4 * n4)) {            // tail (< 4 elements)
    const double t = g[4 * n4 + tid];
    acc += t * t;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) s_red[w] = acc;
  __syncthreads();
  if (tid == 0) {
    double b = 0.0;
    for (int i = 0; i < kBlock / 64; ++i) b += s_red[i];
    st_agent(reinterpret_cast<uint64_t*>(&partial[blockIdx.x]), (uint64_t)__double_as_longlong(b));
  }
  if (!last_block_arrive_sc1(ticket, gridDim.x, &s_flag)) return;
  // ---- last workgroup: fixed-order sum of the partials, header --------------------------
  double t = 0.0;
  for (uint32_t i = (uint32_t)tid; i < gridDim.x; i += kBlock)
    t += __longlong_as_double((long long)ld_agent(reinterpret_cast<const uint64_t*>(&partial[i])));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  __syncthreads();
  if (lane == 0) s_red[w] = t;
  __syncthreads();
  if (tid == 0) {
    double sum = 0.0;
    for (int i = 0; i < kBlock / 64; ++i) sum += s_red[i];
    hdr->thresh = 0; hdr->lower = 0;
    hdr->n = (uint32_t)n; hdr->k = (uint32_t)bits; hdr->n_entries = (uint32_t)n;
    hdr->index_bits = 0; hdr->codec = FC_CODEC_QSGD; hdr->status = FC_STATUS_OK;
    hdr->n_definite = 0; hdr->n_cand = 0;
    hdr->seed = seed; hdr->offset = offset; hdr->p = sqrt(sum);
    hdr->chunk = 0; hdr->format = FC_FMT_QSGD; hdr->key_mode = FC_KEY_PHILOX;
    hdr->reserved[0] = hdr->reserved[1] = hdr->reserved[2] = 0;
    *ticket = 0;                                                  // for the next encode
  }
}

__device__ __forceinline__ QsgdParams qsgd_params(double norm, int bits, uint64_t n) {
  QsgdParams q;
  q.norm = norm;
  q.s = (double)(1u << bits);
  q.scale = norm / (q.s * qsgd_tau((double)n, q.s));
  q.c = norm != 0.0 ? q.s / norm : __longlong_as_double(0x7ff0000000000000ll);
  q.s32 = (float)q.s;
  q.c32 = (float)q.c;
  q.width = qsgd_width(bits);
  return q;
}

// h: the element's 16 dither bits.  F32: c32 is finite (uniform per launch).
// The level is floor(p + U) with p = fl32(|x| * c32) and the sum EXACT (in fp64: p's bits and
// U's 16 fraction bits span < 53 bits wherever p + U is near an integer), so a round-to-nearest
// sum can never push it to the next integer; and it is clamped to s, never dropped: the exact
// s|x|/||x|| + U is < s + 1, only the fp32 product may overshoot s (a one-hot gradient at
// bits = 14 used to lose its one element about once in 1024 encodes).
template <bool F32>
__device__ __forceinline__ uint32_t qsgd_code(float x, uint32_t h, const QsgdParams& q) {
  const double u = (double)h * (1.0 / 65536.0);                  // exact
  const double f = F32 ? floor((double)__fmul_rn(__builtin_fabsf(x), q.c32) + u)
                       : floor((double)__builtin_fabsf(x) * q.c + u);
  const uint32_t l = !(f >= 0.0) ? 0u : (f >= q.s ? (uint32_t)q.s : (uint32_t)f);   // NaN -> 0
  return ((__float_as_uint(x) >> 31) << (q.width - 1)) | l;
}
__device__ __forceinline__ float qsgd_value(uint32_t code, const QsgdParams& q) {
  const uint32_t l = code & ((1u << (q.width - 1)) - 1u);
  const double v = q.scale * (double)l;
  return (float)(((code >> (q.width - 1)) & 1u) ? -v : v);
}

// ---- pass 2: quantise; thread = 8 consecutive elements -> 8 codes ----------------------------
constexpr int kQsgdQuantUnroll = 1;            // groups per thread and pass, loads issued first
__device__ __forceinline__ void qsgd_load8(const float* __restrict__ g, uint64_t e, uint64_t n,
                                           float (&x)[8]) {
  if (e + 8 <= n) {
    const float4 a = load4_full(g + e), b = load4_full(g + e + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = e + j < n ? g[e + j] : 0.f;
  }
}
// The pass for one arithmetic form (F32: c32 finite, uniform per launch) and code width: one
// branch per launch instead of both forms and the width tests per element.  Each load
// instruction reads 1 KB contiguous per wave: 8 consecutive elements per lane as two 16-B
// halves 32 B apart read 128 us per 128 M pass, the wave-contiguous halves and one DPP swap
// 116 us.  (Measured and kept out: one quad per thread, each quad computing its group's Philox
// block: 140 us; 4 groups per thread and pass: 129 us; without Philox or without the code
// arithmetic the pass is 2-3 us shorter: it waits on memory, profiles/r05_ab_qsgd.jsonl.)
__device__ __forceinline__ float4 qsgd_load4(const float* __restrict__ g, uint64_t e, uint64_t n) {
  if (e + 4 <= n) return load4_full(g + e);
  float4 v;
  v.x = e < n ? g[e] : 0.f; v.y = e + 1 < n ? g[e + 1] : 0.f;
  v.z = e + 2 < n ? g[e + 2] : 0.f; v.w = e + 3 < n ? g[e + 3] : 0.f;
  return v;
}
__device__ __forceinline__ float qsgd_swap1(float v) {     // the value of lane ^ 1
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1,
                                                            0xf, 0xf, true));
}
template <bool F32, int W>
__device__ __forceinline__ void qsgd_quant_pass(const float* __restrict__ g, uint64_t n,
                                                uint64_t seed, uint64_t offset,
                                                const QsgdParams& q, uint32_t* codes) {
  const uint64_t groups = (n + kQsgdElems - 1) / kQsgdElems;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint32_t lane = threadIdx.x & 63u;
  // A wave covers 64 consecutive groups (512 elements) per pass and loads them as two 1 KB
  // contiguous 16-B-per-lane loads (lane l: elements 4l.. and 256 + 4l..); the lane pairs then
  // swap halves so that lane 2m holds group m and lane 2m + 1 group 32 + m.
  for (uint64_t w0 = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u); w0 < groups;
       w0 += kQsgdQuantUnroll * stride) {
    float4 lo[kQsgdQuantUnroll], hi[kQsgdQuantUnroll];
#pragma unroll
    for (int u = 0; u < kQsgdQuantUnroll; ++u) {
      const uint64_t e0 = (w0 + u * stride) * kQsgdElems;
      if (e0 < n) {
        lo[u] = qsgd_load4(g, e0 + 4 * lane, n);
        hi[u] = qsgd_load4(g, e0 + 256 + 4 * lane, n);
      }
    }
#pragma unroll
    for (int u = 0; u < kQsgdQuantUnroll; ++u) {
      const uint64_t b = w0 + u * stride;
      if (b >= groups) break;                                      // wave-uniform
      const bool odd = lane & 1u;
      const float4 give = odd ? lo[u] : hi[u];
      float4 got;
      got.x = qsgd_swap1(give.x); got.y = qsgd_swap1(give.y);
      got.z = qsgd_swap1(give.z); got.w = qsgd_swap1(give.w);
      const float4 a = odd ? got : lo[u], c = odd ? hi[u] : got;
      const float xs[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
      const uint64_t t = b + (lane >> 1) + (odd ? 32u : 0u);
      if (t >= groups) continue;
      const uint64_t e = t * kQsgdElems;
      const uint4 r0 = philox_block(e >> 3, seed, offset);     // 8 x 16 dither bits
      const uint32_t wd[4] = {r0.x, r0.y, r0.z, r0.w};
      uint32_t c8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t h = (wd[j >> 1] >> (16 * (j & 1))) & 0xffffu;
        c8[j] = e + j >= n ? 0u : qsgd_code<F32>(xs[j], h, q);
      }
      if (W == 4) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) v |= c8[j] << (4 * j);
        codes[t] = v;
      } else if (W == 8) {
        reinterpret_cast<uint2*>(codes)[t] = make_uint2(c8[0] | c8[1] << 8 | c8[2] << 16 | c8[3] << 24,
                                                        c8[4] | c8[5] << 8 | c8[6] << 16 | c8[7] << 24);
      } else {
        reinterpret_cast<uint4*>(codes)[t] = make_uint4(c8[0] | c8[1] << 16, c8[2] | c8[3] << 16,
                                                        c8[4] | c8[5] << 16, c8[6] | c8[7] << 16);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_qsgd_quant(const float* __restrict__ g, uint64_t n,
                                                       int bits, uint64_t seed, uint64_t offset,
                                                       const fc_packet_hdr* hdr, uint32_t* codes) {
  const QsgdParams q = qsgd_params(hdr->p, bits, n);
  const bool f32 = q.c32 != __builtin_inff();
  if (f32) {
    if (q.width == 4) qsgd_quant_pass<true, 4>(g, n, seed, offset, q, codes);
    else if (q.width == 8) qsgd_quant_pass<true, 8>(g, n, seed, offset, q, codes);
    else qsgd_quant_pass<true, 16>(g, n, seed, offset, q, codes);
  } else {
    if (q.width == 4) qsgd_quant_pass<false, 4>(g, n, seed, offset, q, codes);
    else if (q.width == 8) qsgd_quant_pass<false, 8>(g, n, seed, offset, q, codes);
    else qsgd_quant_pass<false, 16>(g, n, seed, offset, q, codes);
  }
}

// ---- decode (ACC: FedAVG over packets in row order, from +0 as np.sum) ----------------------
struct QsgdDecodeArgs {
  const fc_packet_view* views;   // ACC
  fc_packet_view one;            // !ACC
  int m, acc_in;
  uint64_t n;
  float* out;
};

// The 4 codes of quad qd (elements 4 qd .. 4 qd + 3): 16 / 32 / 64 bits at quad index qd of
// the packed words (W = 4 / 8 / 16; little-endian W-bit fields, so a quad is contiguous).
__device__ __forceinline__ void qsgd_unpack4(const uint32_t* codes, uint64_t qd, int width,
                                             uint32_t (&c)[4]) {
  if (width == 4) {
    typedef __attribute__((address_space(1))) const uint16_t gu16;
    const uint32_t v = ((gu16*)codes)[qd];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = (v >> (4 * j)) & 0xfu;
  } else if (width == 8) {
    typedef __attribute__((address_space(1))) const uint32_t gu;
    const uint32_t v = ((gu*)codes)[qd];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = (v >> (8 * j)) & 0xffu;
  } else {
    typedef __attribute__((address_space(1))) const fc_u32x2 gu2;
    const fc_u32x2 v = ((gu2*)codes)[qd];
    c[0] = v.x & 0xffffu; c[1] = v.x >> 16; c[2] = v.y & 0xffffu; c[3] = v.y >> 16;
  }
}

// Thread = one quad of 4 elements: its codes are one 2 / 4 / 8-B load and its 4 values one
// 16-B store, so every store instruction writes a contiguous 1 KB per wave.  (8 elements per
// thread wrote two 16-B halves 32 B apart per lane: 146 us per 128 M decode with plain stores,
// 239 us with non-temporal ones, which do not merge the halves.)  Each packet's scale and
// width are computed once per workgroup (the fold: into LDS, kQsgdFoldM packets per launch;
// the host splits a longer fold into continued launches), not per quad: re-reading the header
// and an fp64 divide + sqrt per quad made the lone decode VALU-latency-bound (121 us at 128 M).
// kQsgdDecUnroll quads per thread and pass, their code loads issued first.
constexpr int kQsgdFoldM = 512;
constexpr int kQsgdDecUnroll = 2;
struct QsgdPkt {
  const uint32_t* codes;
  double scale;
  float weight;
  int width;
};
__device__ __forceinline__ float qsgd_value2(uint32_t code, double scale, int width) {
  const uint32_t l = code & ((1u << (width - 1)) - 1u);
  const double v = scale * (double)l;
  return (float)(((code >> (width - 1)) & 1u) ? -v : v);
}
// The fold when every packet of the launch has code width W: lane = E = 128 / W consecutive
// elements, so each packet's codes are ONE 16-B load per lane and 1 KB contiguous per wave
// (the quad layout below reads 2 / 4 / 8 B per lane and packet: 675 us for 70 x 25.6 M 2-bit
// packets, 1.3 TB/s of codes).  D packets' loads are issued before their additions, which
// stay in row order per element (gar.py:44).  The E sums go out as E / 4 16-B stores per lane.
template <int W>
__device__ __forceinline__ void qsgd_fold_wide(const QsgdDecodeArgs& a, const QsgdPkt* pk, int M) {
  constexpr int E = 128 / W, D = W == 4 ? 4 : W == 8 ? 4 : 2;
  constexpr uint32_t mask = (1u << W) - 1u;
  const uint64_t n = a.n;
  const uint64_t words = (n + kQsgdElems - 1) / kQsgdElems * (uint64_t)(W / 4);   // code words
  const uint64_t tiles = (n + E - 1) / E;                                          // lane tiles
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kBlock + threadIdx.x; u < tiles; u += stride) {
    const uint64_t e0 = u * E;
    const bool full = e0 + E <= n;
    float acc[E];
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] = 0.f;
    if (a.acc_in) {
      if (full) {
#pragma unroll
        for (int j = 0; j < E; j += 4) {
          const fc_f4v v = *(const fc_gf4v*)(a.out + e0 + j);
          acc[j] = v.x; acc[j + 1] = v.y; acc[j + 2] = v.z; acc[j + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) if (e0 + j < n) acc[j] = a.out[e0 + j];
      }
    }
    const bool wfull = 4 * (u + 1) <= words;
    for (int m0 = 0; m0 < M; m0 += D) {
      fc_u32x4 c[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (m0 + d >= M) break;
        const uint32_t* cw = pk[m0 + d].codes;
        if (wfull) {
          c[d] = __builtin_nontemporal_load((const FC_G fc_u32x4*)cw + u);
        } else {
          uint32_t t[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) t[i] = 4 * u + i < words ? ((const FC_G uint32_t*)cw)[4 * u + i] : 0u;
          c[d] = fc_u32x4{t[0], t[1], t[2], t[3]};
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (m0 + d >= M) break;
        const QsgdPkt& p = pk[m0 + d];
        const uint32_t cw4[4] = {c[d].x, c[d].y, c[d].z, c[d].w};
#pragma unroll
        for (int j = 0; j < E; ++j) {
          const uint32_t code = (cw4[(j * W) >> 5] >> ((j * W) & 31)) & mask;
          const float v = qsgd_value2(code, p.scale, W);
          acc[j] = __fadd_rn(acc[j], __fmul_rn(v, p.weight));
        }
      }
    }
    if (full) {
#pragma unroll
      for (int j = 0; j < E; j += 4)
        *(FC_G fc_f4v*)(a.out + e0 + j) = fc_f4v{acc[j], acc[j + 1], acc[j + 2], acc[j + 3]};
    } else {
#pragma unroll
      for (int j = 0; j < E; ++j) if (e0 + j < n) a.out[e0 + j] = acc[j];
    }
  }
}

// Code widths 4 and 8 fold through per-packet tables: T_m[c] = fl(value(c) * w_m) for the
// 2^W codes c, built in LDS by the workgroup (the same two roundings the per-element form does,
// so the sums are bit-identical), then each element of each packet is one bit-field extract,
// one LDS read and one addition.  (With the fp64 value per element the fold was VALU-bound:
// 465 us for 70 x 25.6 M 2-bit packets, 270-285 us with the tables; 5-bit: 480 -> 415 us.)
// kQsgdTabFloats floats of tables: 256 packets at W = 4, 16 at W = 8 per batch; a longer fold
// rebuilds them per batch and tile.  D packets' code loads are issued together (loading the
// next D while adding, or D = 2 / 8: no faster, profiles/r05_ab_qsgd.jsonl).
constexpr int kQsgdTabFloats = 4096;
template <int W>
__device__ __forceinline__ void qsgd_fold_lut(const QsgdDecodeArgs& a, const QsgdPkt* pk, int M,
                                              float* s_tab) {
  constexpr int E = 128 / W, NT = 1 << W, B = kQsgdTabFloats / NT, D = 4;
  constexpr uint32_t mask = NT - 1u;
  const uint64_t n = a.n;
  const uint64_t words = (n + kQsgdElems - 1) / kQsgdElems * (uint64_t)(W / 4);
  const uint64_t tiles = (n + E - 1) / E;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t first = (uint64_t)blockIdx.x * kBlock;
  for (uint64_t ub = first; ub < tiles; ub += stride) {         // workgroup-uniform
    const uint64_t u = ub + threadIdx.x, e0 = u * E;
    const bool active = u < tiles, full = e0 + E <= n, wfull = 4 * (u + 1) <= words;
    float acc[E];
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] = 0.f;
    if (active && a.acc_in) {
      if (full) {
#pragma unroll
        for (int j = 0; j < E; j += 4) {
          const fc_f4v v = *(const fc_gf4v*)(a.out + e0 + j);
          acc[j] = v.x; acc[j + 1] = v.y; acc[j + 2] = v.z; acc[j + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) if (e0 + j < n) acc[j] = a.out[e0 + j];
      }
    }
    for (int mb = 0; mb < M; mb += B) {
      const int nb = M - mb < B ? M - mb : B;
      if (ub == first || M > B) {                               // (re)build this batch's tables
        __syncthreads();
        for (int i = threadIdx.x; i < nb * NT; i += kBlock) {
          const QsgdPkt& p = pk[mb + i / NT];
          s_tab[i] = __fmul_rn(qsgd_value2((uint32_t)(i % NT), p.scale, W), p.weight);
        }
        __syncthreads();
      }
      if (!active) continue;
      auto load_group = [&](int m0, fc_u32x4 (&c)[D]) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          if (m0 + d >= nb) break;
          const uint32_t* cw = pk[mb + m0 + d].codes;
          if (wfull) {
            c[d] = __builtin_nontemporal_load((const FC_G fc_u32x4*)cw + u);
          } else {
            uint32_t t[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) t[i] = 4 * u + i < words ? ((const FC_G uint32_t*)cw)[4 * u + i] : 0u;
            c[d] = fc_u32x4{t[0], t[1], t[2], t[3]};
          }
        }
      };
      fc_u32x4 c[D];
      load_group(0, c);
      for (int m0 = 0; m0 < nb; m0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          if (m0 + d >= nb) break;
          const float* tab = s_tab + (m0 + d) * NT;
          const uint32_t cw4[4] = {c[d].x, c[d].y, c[d].z, c[d].w};
#pragma unroll
          for (int j = 0; j < E; ++j)
            acc[j] = __fadd_rn(acc[j], tab[(cw4[(j * W) >> 5] >> ((j * W) & 31)) & mask]);
        }
        if (m0 + D < nb) load_group(m0 + D, c);
      }
    }
    if (!active) continue;
    if (full) {
#pragma unroll
      for (int j = 0; j < E; j += 4)
        *(FC_G fc_f4v*)(a.out + e0 + j) = fc_f4v{acc[j], acc[j + 1], acc[j + 2], acc[j + 3]};
    } else {
#pragma unroll
      for (int j = 0; j < E; ++j) if (e0 + j < n) a.out[e0 + j] = acc[j];
    }
  }
}

template <bool ACC>
__global__ __launch_bounds__(kBlock) void k_qsgd_decode(QsgdDecodeArgs a) {
  const uint64_t n = a.n, quads = (n + 3) / 4;
  const int M = ACC ? a.m : 1;
  __shared__ QsgdPkt s_pk[ACC ? kQsgdFoldM : 1];
  __shared__ float s_tab[ACC ? kQsgdTabFloats : 1];
  QsgdPkt one;
  if (ACC) {
    const int w0 = qsgd_width((int)a.views[0].hdr->k);
    int same = 1;
    for (int m = threadIdx.x; m < M; m += kBlock) {
      const fc_packet_view& v = a.views[m];
      const QsgdParams q = qsgd_params(v.hdr->p, (int)v.hdr->k, n);
      s_pk[m] = QsgdPkt{static_cast<const uint32_t*>(v.idx), q.scale, v.weight, q.width};
      same &= q.width == w0;
    }
    if (__syncthreads_and(same)) {                     // one width in the launch: wide loads
      if (w0 == 4) qsgd_fold_lut<4>(a, s_pk, M, s_tab);
      else if (w0 == 8) qsgd_fold_lut<8>(a, s_pk, M, s_tab);
      else qsgd_fold_wide<16>(a, s_pk, M);
      return;
    }
  } else {
    const QsgdParams q = qsgd_params(a.one.hdr->p, (int)a.one.hdr->k, n);
    one = QsgdPkt{static_cast<const uint32_t*>(a.one.idx), q.scale, 1.0f, q.width};
  }
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t q0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x; q0 < quads;
       q0 += kQsgdDecUnroll * stride) {
    float acc[kQsgdDecUnroll][4];
#pragma unroll
    for (int u = 0; u < kQsgdDecUnroll; ++u) {
      const uint64_t qd = q0 + u * stride, e = qd * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[u][j] = 0.f;
      if (ACC && a.acc_in && qd < quads) {
        if (e + 4 <= n) {
          const fc_f4v v = *(fc_gf4v*)(a.out + e);
          acc[u][0] = v.x; acc[u][1] = v.y; acc[u][2] = v.z; acc[u][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) if (e + j < n) acc[u][j] = a.out[e + j];
        }
      }
    }
    for (int m = 0; m < M; ++m) {                                // rows in order (gar.py:44)
      const QsgdPkt& p = ACC ? s_pk[m] : one;
      uint32_t c[kQsgdDecUnroll][4];
#pragma unroll
      for (int u = 0; u < kQsgdDecUnroll; ++u)
        if (q0 + u * stride < quads) qsgd_unpack4(p.codes, q0 + u * stride, p.width, c[u]);
#pragma unroll
      for (int u = 0; u < kQsgdDecUnroll; ++u) {
        if (q0 + u * stride >= quads) break;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = qsgd_value2(c[u][j], p.scale, p.width);
          acc[u][j] = ACC ? __fadd_rn(acc[u][j], __fmul_rn(d, p.weight)) : d;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kQsgdDecUnroll; ++u) {
      const uint64_t qd = q0 + u * stride, e = qd * 4;
      if (qd >= quads) break;
      if (e + 4 <= n) {
        __builtin_nontemporal_store(fc_f4v{acc[u][0], acc[u][1], acc[u][2], acc[u][3]},
                                    reinterpret_cast<fc_f4v*>(a.out + e));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) if (e + j < n) a.out[e + j] = acc[u][j];
      }
    }
  }
}

template __global__ void k_qsgd_decode<true>(QsgdDecodeArgs);
template __global__ void k_qsgd_decode<false>(QsgdDecodeArgs);

}  // namespace fc
