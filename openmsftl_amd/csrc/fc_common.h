// fc_common.h — shared device helpers for the MI355X (gfx950) gradient codec.
//
// Geometry: every streaming kernel works on CHUNKs of 8192 fp32 elements (32 KiB) with a
// 256-thread workgroup (4 waves of 64).  Inside a chunk, element e is owned by
//     iteration i = e / 1024, wave w = (e / 256) % 4, lane l = (e / 4) % 64, slot j = e % 4
// so each wave instruction moves 1 KiB contiguous (one float4 per lane) and the (i, w, l, j)
// order is exactly ascending index order — ballots + mbcnt give ordered compaction offsets
// with no block-wide scan per element.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fc {

constexpr int kBlock = 256;                 // threads per workgroup
constexpr int kWaves = kBlock / 64;
constexpr int kVec = 8;                     // float4 per thread per chunk
constexpr int kChunk = kBlock * 4 * kVec;   // 8192 elements
constexpr int kChunkWords = kChunk / 32;    // bitmap words per chunk (256)
constexpr int kHistBits = 12;
constexpr int kHistBins = 1 << kHistBits;   // 4096
constexpr int kSmallCap = 4096;             // exact-finish list (LDS bitonic, 32 KiB)
constexpr int kEngineGrid = 256;            // radix-engine workgroups (one per CU)
constexpr int kEnginePasses = 6;            // ceil(63 / 12): enough for any comp width
constexpr int FC_RESOLVE_GRID = 256;
constexpr int kResolveGrid = FC_RESOLVE_GRID;           // k_resolve workgroups
constexpr int FC_RESOLVE_GRID_BATCH = 16;
constexpr int kResolveGridBatch = FC_RESOLVE_GRID_BATCH;   // k_resolve workgroups per client (batched encode;
                                                          // 16 vs 64: configs[2] +2.1 %, configs[3] +0.2 %)
constexpr int kSlots = kVec * kWaves;       // 32 (i, w) slots per chunk
constexpr int kCandSlot = 256;              // candidate slot per chunk (overflow: re-read entries)
constexpr int kShards = 64;                 // sharded k_compact totals

constexpr uint32_t kNanKey = 0x7f800001u;   // every NaN sorts above +inf
constexpr uint64_t kSelectNothing = 1ull << 63;

template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B record hand-off (one lane's dwordx4, 16-B aligned: one transaction each way): the
// agent-scope (sc1) forms of a vector store and a load; the load waits for its data.
typedef uint32_t fc_rec4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_agent(uint32_t* p, fc_rec4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ fc_rec4 ld16_agent(const uint32_t* p) {
  fc_rec4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// ---- keys ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mag_key(float x) {
  uint32_t u = __float_as_uint(x) & 0x7fffffffu;
  return u > 0x7f800000u ? kNanKey : u;
}
__device__ __forceinline__ uint64_t comp_of(uint32_t key, uint32_t idx, uint32_t ib) {
  return ((uint64_t)key << ib) | idx;
}

// ---- Philox4x32-10 (Salmon et al. SC'11); KAT-pinned by oracle/philox.py -------------
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    // one 32 x 32 -> 64 multiply per product (v_mad_u64_u32) instead of mul_lo + mul_hi: the
    // integer multiplies are quarter-rate and set the cost of every Philox-driven pass
    const uint64_t p0 = (uint64_t)c.x * 0xD2511F53ull, p1 = (uint64_t)c.z * 0xCD9E8D57ull;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
  }
  return c;
}
// counter block b: (lo32 b, hi32 b, lo32 offset, hi32 offset), key = seed
__device__ __forceinline__ uint4 philox_block(uint64_t b, uint64_t seed, uint64_t offset) {
  return philox4x32_10(make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)offset,
                                  (uint32_t)(offset >> 32)),
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}
// The codec's element -> word map (native rand-k keys, Bernoulli dropout masks):
//     element i  ->  block ((i >> 8) << 6) | (i & 63),  word (i >> 6) & 3
// The four words of a block go to elements 64 apart, so in the ballot layout (element
// seg*256 + j*64 + lane) lane L computes ONE block per 256-element segment and holds the
// words of its four groups j (oracle/philox.py element_words).  (QSGD keeps its own linear
// map, block i >> 2, for 8 consecutive elements per thread.)
__device__ __forceinline__ uint4 philox_seg(uint64_t seg, uint32_t lane, uint64_t seed,
                                            uint64_t offset) {
  return philox_block((seg << 6) | lane, seed, offset);
}
__device__ __forceinline__ uint32_t philox_word(uint64_t i, uint64_t seed, uint64_t offset) {
  const uint4 r = philox_seg(i >> 8, (uint32_t)(i & 63), seed, offset);
  const uint32_t s = (uint32_t)(i >> 6) & 3u;
  return s == 0 ? r.x : s == 1 ? r.y : s == 2 ? r.z : r.w;
}

// Key source: MAG = |g| bit pattern (top-k); PHILOX = random word (native rand-k).
enum KeyMode : int { kKeyMag = 0, kKeyPhilox = 1 };

// ---- wave helpers --------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint32_t prefix_count(uint64_t mask) {   // popc(mask & lanemask_lt)
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP (GFX9 row_shr / row_bcast):
// 6 fused adds, no LDS.  Lanes whose DPP source is out of range add 0.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}
__device__ __forceinline__ uint32_t lane63(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// float4 load of elements [e, e+4) with zero fill past n (16-B aligned base required)
__device__ __forceinline__ float4 load4(const float* __restrict__ g, uint64_t e, uint64_t n) {
  if (e + 4 <= n) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(g + e));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e + 0 < n) r.x = g[e + 0];
  if (e + 1 < n) r.y = g[e + 1];
  if (e + 2 < n) r.z = g[e + 2];
  if (e + 3 < n) r.w = g[e + 3];
  return r;
}
// float4 load of [e, e+4) with zero fill past n, default cache policy (latency-bound reads:
// the sample, where non-temporal loads measured ~2 us slower)
__device__ __forceinline__ float4 load4_plain(const float* __restrict__ g, uint64_t e, uint64_t n) {
  if (e + 4 <= n) return *reinterpret_cast<const float4*>(g + e);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e + 0 < n) r.x = g[e + 0];
  if (e + 1 < n) r.y = g[e + 1];
  if (e + 2 < n) r.z = g[e + 2];
  if (e + 3 < n) r.w = g[e + 3];
  return r;
}
typedef uint32_t fc_u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t fc_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t fc_u32x8 __attribute__((ext_vector_type(8)));
// Unconditional float4 load through the GLOBAL address space.  Pointers that come out of
// memory (batched job tables) are generic to the compiler, and a generic load is a flat_load
// that also counts in lgkmcnt; a per-element bounds branch between loads made hipcc wait for
// each one (4 serial HBM latencies per chunk).  Callers check bounds once per chunk.
typedef float fc_f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const fc_f4v fc_gf4v;
// GLOBAL address space for pointers that come out of memory (job tables, row / view arrays):
// as generic pointers their loads and stores are flat_ ops, which also count in lgkmcnt, so the
// next scalar-load or LDS wait waits for them too
#define FC_G __attribute__((address_space(1)))
__device__ __forceinline__ float4 load4_full(const float* p) {
  const fc_f4v v = __builtin_nontemporal_load((fc_gf4v*)p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float f4get(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
__device__ __forceinline__ void f4set(float4& v, int j, float x) {
  if (j == 0) v.x = x; else if (j == 1) v.y = x; else if (j == 2) v.z = x; else v.w = x;
}

// h[0..4096) = gh[0..4096) (sc1 loads), then gh = 0 — every load issued before any clearing
// store (a load and a store of one address issue in order: interleaved, each bin cost a round
// trip).  256-thread workgroup; the caller synchronises before reading h.
__device__ __forceinline__ void load_clear_hist(uint32_t* gh, uint32_t* h) {
  constexpr int kPer = 4096 / 256;
  uint32_t v[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) v[j] = ld_agent(&gh[j * 256 + threadIdx.x]);
#pragma unroll
  for (int j = 0; j < kPer; ++j) h[j * 256 + threadIdx.x] = v[j];
#pragma unroll
  for (int j = 0; j < kPer; ++j) st_agent(&gh[j * 256 + threadIdx.x], 0u);
}

// Spread the 8 bits of x to bits 0,4,8,...,28 (bitmap assembly from 4 ballots).
__device__ __forceinline__ uint32_t spread4(uint32_t x) {
  x &= 0xffu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  x = (x | (x << 3)) & 0x11111111u;
  return x;
}

// Exclusive block scan of one value per thread (256 threads).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp,
                                                    uint32_t* total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v);          // DPP: 6 fused adds, no LDS round trips
  if (lane == 63) s_tmp[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    const uint32_t s = s_tmp[i];
    if (i < w) base += s;
    tot += s;
  }
  __syncthreads();
  if (total) *total = tot;
  return base + inc - v;
}

// ---- diagnostic phase timestamps (FC_TRACE builds only; tools/trace_probe.py) ----------
// FC_TR(slot): thread 0 of the workgroup records s_memrealtime (100 MHz) at trace[block*32+slot].
#ifdef FC_TRACE
__device__ uint64_t g_fc_trace[1 << 16];
#define FC_TR(slot)                                                                          \
  do {                                                                                      \
    if (threadIdx.x == 0)                                                                   \
      g_fc_trace[((blockIdx.x + blockIdx.y * gridDim.x) * 32u + (slot)) & 0xffffu] =        \
          __builtin_amdgcn_s_memrealtime();                                                 \
  } while (0)
#else
#define FC_TR(slot) do {} while (0)
#endif

// Last-arriver ticket for payloads written ONLY by agent-scope atomics or sc1 stores and
// read ONLY by sc1 loads / atomics (MI355X_MICROARCH.md §visibility, "Hand-offs measured
// with sc1 loads": every storing wave drains, barrier, one lane adds; the workgroup whose
// add returned nblocks-1 loads after a barrier).  No L2 write-back fence needed.
__device__ __forceinline__ bool last_block_arrive_sc1(uint32_t* counter, uint32_t nblocks,
                                                      uint32_t* s_flag, int tr = -1) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tr >= 0) FC_TR(tr);
  if (threadIdx.x == 0) *s_flag = (atomicAdd(counter, 1u) == nblocks - 1) ? 1u : 0u;
  if (tr >= 0) FC_TR(tr + 1);
  __syncthreads();
  return *s_flag != 0;
}

// Two-level last-arriver ticket over nblocks workgroups (bid = this workgroup's index among
// them): the workgroups count into G <= 16 group counters on separate 256-B lines, the last of
// each group into one top counter.  Same-address atomics queue at ~35 ns each (256 workgroups
// on ONE counter took ~9 us, FC_TRACE); this keeps every queue at <= 16.  Payload rules are
// those of last_block_arrive_sc1 (sc1 stores drained before the first add; sc1 loads after).
// Each group's last arriver and the top's reset their counters: self-cleaning.
__device__ __forceinline__ bool last_block_arrive_tree(uint32_t* tick, uint32_t nblocks,
                                                       uint32_t bid, uint32_t* s_flag,
                                                       int tr = -1) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tr >= 0) FC_TR(tr);
  if (threadIdx.x == 0) {
    constexpr uint32_t kG = 16, kS = 64;             // fc_state.h kTickGroups / kTickStride
    const uint32_t G = nblocks < kG ? nblocks : kG;
    const uint32_t g = bid % G;
    const uint32_t gsize = nblocks / G + (g < nblocks % G ? 1u : 0u);
    bool last = false;
    if (atomicAdd(&tick[g * kS], 1u) == gsize - 1) {
      st_agent(&tick[g * kS], 0u);
      last = atomicAdd(&tick[kG * kS], 1u) == G - 1;
      if (last) st_agent(&tick[kG * kS], 0u);
    }
    *s_flag = last ? 1u : 0u;
  }
  if (tr >= 0) FC_TR(tr + 1);
  __syncthreads();
  return *s_flag != 0;
}

// Workgroup "last arriver" ticket (MI355X_MICROARCH.md §visibility valid producer form):
// every storing wave drains, barrier, lane 0 releases at agent scope, drains, then adds.
// Returns true in every thread of the last-arriving workgroup, after an agent acquire.
__device__ __forceinline__ bool last_block_arrive(uint32_t* counter, uint32_t nblocks,
                                                  uint32_t* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = atomicAdd(counter, 1u);
    const bool last = (t == nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *s_flag = last ? 1u : 0u;
  }
  __syncthreads();
  return *s_flag != 0;
}

}  // namespace fc
