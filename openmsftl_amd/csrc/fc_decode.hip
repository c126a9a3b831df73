// fc_decode.hip — packet decode and bit-exact FedAVG accumulation for MI355X (gfx950).
//
// k_decode<FMT, ACC, OutT>: one workgroup per 8192-element chunk.  For each packet (client,
// in G's row order) the chunk's slot entries [c*8192, c*8192 + cnt[c]) are expanded:
//   FC_FMT_IDXVAL : entries scattered into an LDS tile + LDS presence bitmap (keeps only
//                   comp >= T64, the sampled-bracket slack is dropped here)
//   FC_FMT_BITMAP : the chunk's 256 bitmap words are prefix-counted in LDS and every lane
//                   fetches its own kept values from the packet
// then each lane owns the same (i, w, lane, j) element layout as the encoder and either
// writes the dense result (ACC = false; compression.py:33-37 / 52 / 60) or folds it into a
// register accumulator exactly as gar.py:44 does on the dense G:
//   acc = +0;  acc = fl(acc + fl(w_i * d_i))  for i in row order  (no FMA: __fmul_rn /
//   __fadd_rn; NumPy's axis-0 add.reduce starts from +0, so the sum is never -0)
// so the FedAVG of M packets reads each packet once and writes the aggregate once.
#include <type_traits>

#include "fc_state.h"

namespace fc {

struct PktCache {
  const void* idx;          // uint16 chunk-local indices (FC_FMT_IDXVAL)
  const float* val;
  const uint32_t* bitmap;
  const uint32_t* cnt;
  uint64_t thresh, seed, offset;
  double p;
  uint32_t ib, codec, key_mode;
  float w;
};

__device__ __forceinline__ PktCache load_pkt(const fc_packet_view& v) {
  PktCache c;
  c.idx = v.idx; c.val = v.val; c.bitmap = v.bitmap; c.cnt = v.cnt; c.w = v.weight;
  const fc_packet_hdr* h = v.hdr;
  c.thresh = h->thresh; c.seed = h->seed; c.offset = h->offset; c.p = h->p;
  c.ib = h->index_bits; c.codec = h->codec; c.key_mode = h->key_mode;
  return c;
}

// Value the reference stores for a kept coordinate (compression.py:36/44/52/60) — f32 path.
__device__ __forceinline__ float kept_f32(float v, const PktCache& c) {
  if (c.codec == FC_CODEC_DROPOUT_UNBIASED) return (float)((double)v / c.p);  // fl32(fl64/p)
  return v;
}
__device__ __forceinline__ double kept_f64(float v, const PktCache& c) {
  if (c.codec == FC_CODEC_DROPOUT_UNBIASED) return (double)v / c.p;
  return (double)v;
}
// Value of a dropped coordinate: +0 (zeros_like), except 0/p = NaN for unbiased p == 0.
__device__ __forceinline__ float dropped_f32(const PktCache& c) {
  return (c.codec == FC_CODEC_DROPOUT_UNBIASED && c.p == 0.0) ? __uint_as_float(0x7fc00000u) : 0.0f;
}

__device__ __forceinline__ bool entry_kept(const PktCache& c, uint32_t id, float v) {
  if (c.thresh == 0) return true;
  const uint32_t key = c.key_mode == FC_KEY_PHILOX ? (philox_word(id, c.seed, c.offset) >> 1)
                                                   : mag_key(v);
  return comp_of(key, id, c.ib) >= c.thresh;
}

// Dense fp32 results leave with non-temporal 16-B stores (written once, read by the next
// kernel or D2H; the fused dense encode measured NT at 192 us against 269 for plain / sc1)
template <typename OutT>
__device__ __forceinline__ void store_out(OutT* out, uint64_t e, uint64_t n, const float4& v) {
  if (e + 4 <= n) {
    if constexpr (sizeof(OutT) == 4) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(out + e));
      return;
    }
  }
  if (e + 0 < n) out[e + 0] = (OutT)v.x;
  if (e + 1 < n) out[e + 1] = (OutT)v.y;
  if (e + 2 < n) out[e + 2] = (OutT)v.z;
  if (e + 3 < n) out[e + 3] = (OutT)v.w;
}

struct DecodeArgs {
  const fc_packet_view* views;  // device array (ACC) — or nullptr with `one` filled
  fc_packet_view one;
  int m;                        // packets in this launch (<= kDecMaxM)
  int acc_in;                   // ACC: continue an earlier launch's sum held in `out`
  uint64_t n;
  void* out;
};

constexpr int kDBlock = 256;                   // decode workgroup (4 waves)
constexpr int kDVec = kChunk / (kDBlock * 4);  // 8 float4 per thread: e = i*1024 + w*256 + lane*4
constexpr int kDecR = 4;                       // slot entries per thread per item (1024 / chunk)
constexpr int FC_DEC_GROUP = 4;
constexpr int kDecGroup = FC_DEC_GROUP;        // items whose loads are issued together
constexpr int kDecMaxM = 64;                   // packets per launch (the host splits larger batches)
constexpr int FC_SPARSE_MAXM = 128;
// k_decode_sparse: packets per launch.  Every launch after the first re-reads and re-writes the
// 4N-byte aggregate, so a whole 128-client batch is folded in one launch (uint8 fold counts
// in cntC stay exact up to 255).
constexpr int kSparseMaxM = FC_SPARSE_MAXM;
static_assert(kSparseMaxM <= 255, "cntC counts are uint8");
constexpr int kDecBlocksPerCU = 4;

// Pointers read back from memory are generic (flat) to the compiler; loads through these
// casts are plain global loads with a scalar base.
typedef __attribute__((address_space(1))) const float gf32;
typedef __attribute__((address_space(1))) const uint32_t gu32;
typedef __attribute__((address_space(1))) const uint16_t gu16;   // chunk-local packet indices

// Per-packet record staged in LDS once per workgroup (no per-step header/view loads).
struct DecMeta {
  const void* idx;            // FC_FMT_IDXVAL: uint16 idx; FC_FMT_BITMAP: uint32 bitmap
  const float* val;
  const uint32_t* cnt;
  uint64_t seed, offset;      // rand-k (PHILOX) keys for the slack filter
  double p;                   // dropout-unbiased scale
  uint64_t thresh;
  float w;
  uint32_t flags;             // ib | codec << 8 | key_mode << 16
};

// One "item" = one packet's slot in one chunk: its entry count, first kDecR*512 entries and
// (bitmap format) the thread's bitmap word, all loaded with one round of independent loads.
struct DecItem {
  uint32_t id[kDecR];
  float v[kDecR];
  uint32_t bw, cnt;
};

// LDS-read values are VGPRs to the compiler; the meta record is wave-uniform, so move it to
// SGPRs (scalar base + 32-bit lane offset addressing, no 64-bit VGPR address per load).
__device__ __forceinline__ uint32_t uni32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)uni32((uint32_t)(x >> 32)) << 32) | uni32((uint32_t)x);
}
template <typename T>
__device__ __forceinline__ T* uni_ptr(T* p) { return (T*)uni64((uint64_t)p); }

__device__ __forceinline__ DecMeta uni_meta(const DecMeta& m) {
  DecMeta u;
  u.idx = uni_ptr(m.idx); u.val = uni_ptr(m.val); u.cnt = uni_ptr(m.cnt);
  u.seed = uni64(m.seed); u.offset = uni64(m.offset);
  u.p = __longlong_as_double((long long)uni64((uint64_t)__double_as_longlong(m.p)));
  u.thresh = uni64(m.thresh); u.w = __uint_as_float(uni32(__float_as_uint(m.w)));
  u.flags = uni32(m.flags);
  return u;
}

// Unconditional loads (inside the chunk's 8192-entry slot; entries past cnt are ignored):
// no divergent branch around them, so the compiler waits on exactly one ring slot
// (vmcnt(N)) while the other kDecDepth-1 items stay in flight.
template <int FMT>
__device__ __forceinline__ void dec_load(DecItem& it, const DecMeta& pm, uint32_t c, int tid) {
  const uint64_t lo = (uint64_t)c * kChunk;
  gf32* val = (gf32*)pm.val + lo;                 // chunk slot base (scalar)
  gu16* idx = (gu16*)pm.idx + lo;
  it.cnt = ((gu32*)pm.cnt)[c];
#pragma unroll
  for (int r = 0; r < kDecR; ++r) {
    const uint32_t e = (uint32_t)(tid + r * kDBlock);
    it.v[r] = val[e];
    if (FMT == FC_FMT_IDXVAL) it.id[r] = idx[e];                 // chunk-local
  }
  if (FMT == FC_FMT_BITMAP) it.bw = ((gu32*)pm.idx + (uint64_t)c * kChunkWords)[tid];
}

__device__ __forceinline__ PktCache meta_pkt(const DecMeta& pm) {
  PktCache c;
  c.idx = pm.idx; c.val = pm.val; c.bitmap = (const uint32_t*)pm.idx; c.cnt = pm.cnt; c.w = pm.w;
  c.thresh = pm.thresh;
  c.ib = pm.flags & 0xffu; c.codec = (pm.flags >> 8) & 0xffu; c.key_mode = pm.flags >> 16;
  c.seed = pm.seed; c.offset = pm.offset; c.p = pm.p;
  return c;
}

struct SparseMeta;
__device__ __forceinline__ PktCache meta_pkt_s(const SparseMeta& m);

// Persistent, software-pipelined decode.  Workgroup b owns chunks b, b + G, ...; for every
// chunk it walks the packets in G's row order (gar.py:44), one "item" (packet, chunk) at a
// time.  Items are taken kDecGroup at a time: the group's loads (entry count, first 1024
// entries, bitmap word) are issued together in straight-line code, then the items are
// expanded one by one, each waiting only for its own loads (exact vmcnt; a loop-carried
// register ring made the compiler fall back to near-vmcnt(0) waits).  Four resident
// workgroups per CU overlap one group's latency with the others' work.
// Per item: scatter into the LDS tile (+ presence bits), barrier, every lane folds its 32
// elements, barrier.
template <int FMT, bool ACC, bool OUT64>
__global__ __launch_bounds__(kDBlock, kDecBlocksPerCU) void k_decode(DecodeArgs a) {
  __shared__ __attribute__((aligned(16))) float tile[kChunk];   // IDXVAL scatter / BITMAP values
  __shared__ uint32_t bits[2][kChunkWords];                      // presence (double-buffered)
  __shared__ uint32_t wpre[kChunkWords];
  __shared__ DecMeta s_meta[ACC ? kDecMaxM : 1];
  __shared__ uint32_t s_tmp[8];
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t M = ACC ? (uint32_t)a.m : 1u;
  const uint32_t nch = (uint32_t)((a.n + kChunk - 1) / kChunk);
  const uint32_t G = gridDim.x;
  if (blockIdx.x >= nch) return;
  const uint32_t J = (nch - blockIdx.x + G - 1) / G;             // chunks of this workgroup
  const uint32_t T = J * M;                                      // items

  if (tid < (int)M) {
    const fc_packet_view v = ACC ? a.views[tid] : a.one;
    const fc_packet_hdr* h = v.hdr;
    DecMeta d;
    d.idx = FMT == FC_FMT_IDXVAL ? v.idx : v.bitmap; d.val = v.val; d.cnt = v.cnt;
    d.seed = h->seed; d.offset = h->offset; d.p = h->p;
    d.thresh = h->thresh; d.w = v.weight;
    d.flags = (h->index_bits & 0xffu) | ((h->codec & 0xffu) << 8) | (h->key_mode << 16);
    s_meta[tid] = d;
  }
  bits[0][tid] = 0; bits[1][tid] = 0;
  __syncthreads();

  float4 acc[ACC ? kDVec : 1];
  uint32_t lj = 0, lm = 0;                                       // load cursor (item -> j, m)
  uint32_t pj = 0, pm_i = 0;                                     // process cursor
  for (uint32_t t0 = 0; t0 < T; t0 += kDecGroup) {
    DecItem grp[kDecGroup];
#pragma unroll
    for (int d = 0; d < kDecGroup; ++d) {                        // past the end: re-load (ignored)
      const uint32_t c = blockIdx.x + min(lj, J - 1) * G;
      dec_load<FMT>(grp[d], uni_meta(s_meta[lm]), c, tid);
      if (++lm == M) { lm = 0; ++lj; }
    }
#pragma unroll
    for (int d = 0; d < kDecGroup; ++d) {
      const uint32_t t = t0 + d;
      if (t < T) {                                               // uniform
        const DecItem& cur = grp[d];
        const uint32_t c = blockIdx.x + pj * G;
        const uint64_t base = (uint64_t)c * kChunk;
        const uint32_t m = pm_i;
        const DecMeta pm = uni_meta(s_meta[m]);
        const PktCache pk = meta_pkt(pm);
        const uint32_t cntv = uni32(cur.cnt);
        uint32_t* bb = bits[t & 1];
        if (ACC && m == 0 && a.acc_in) {
#pragma unroll
          for (int i = 0; i < kDVec; ++i)
            acc[i] = load4(reinterpret_cast<const float*>(a.out),
                           base + (uint32_t)(i * 1024 + w * 256 + lane * 4), a.n);
        }
        // ---- expand into LDS ----------------------------------------------------------------
        if (FMT == FC_FMT_IDXVAL) {
          // fp32 outputs get fl32(fl64(g)/p) (compression.py:60) once per entry, here
          const bool scale = !OUT64 && pk.codec == FC_CODEC_DROPOUT_UNBIASED;   // uniform
          if ((pk.key_mode == FC_KEY_PHILOX && pk.thresh != 0) || scale) {
            for (int r = 0; r < kDecR; ++r) {          // rand-k slack filter / scaling: one
              const uint32_t e = (uint32_t)(tid + r * kDBlock);   // entry at a time (VGPRs)
              const uint32_t loc = cur.id[r];
              if (e < cntv && loc < (uint32_t)kChunk && entry_kept(pk, (uint32_t)base + loc, cur.v[r])) {
                tile[loc] = scale ? (float)((double)cur.v[r] / pk.p) : cur.v[r];
                atomicOr(&bb[loc >> 5], 1u << (loc & 31));
              }
            }
          } else {
#pragma unroll
            for (int r = 0; r < kDecR; ++r) {
              const uint32_t e = (uint32_t)(tid + r * kDBlock);
              const uint32_t loc = cur.id[r];
              const bool keep = pk.thresh == 0 ||
                                comp_of(mag_key(cur.v[r]), (uint32_t)base + loc, pk.ib) >= pk.thresh;
              if (e < cntv && loc < (uint32_t)kChunk && keep) {
                tile[loc] = cur.v[r];
                atomicOr(&bb[loc >> 5], 1u << (loc & 31));
              }
            }
          }
          if (cntv > (uint32_t)(kDecR * kDBlock)) {              // dense slot (uniform, rare)
            gf32* pval = (gf32*)pm.val + base;
            gu16* pidx = (gu16*)pm.idx + base;
            for (uint32_t e = (uint32_t)(kDecR * kDBlock + tid); e < cntv; e += kDBlock) {
              const uint32_t loc = pidx[e];
              const uint32_t id = (uint32_t)base + loc;
              const float v = pval[e];
              if (loc < (uint32_t)kChunk && entry_kept(pk, id, v)) {
                tile[loc] = scale ? (float)((double)v / pk.p) : v;
                atomicOr(&bb[loc >> 5], 1u << (loc & 31));
              }
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);                  // vmcnt(0): none left pending
          }
        } else {
          bb[tid] = cur.bw;
          const bool scale = !OUT64 && pk.codec == FC_CODEC_DROPOUT_UNBIASED;   // uniform
          if (scale) {
#pragma unroll
            for (int r = 0; r < kDecR; ++r) {
              const uint32_t e = (uint32_t)(tid + r * kDBlock);
              if (e < cntv) tile[e] = (float)((double)cur.v[r] / pk.p);  // compression.py:60
            }
          } else {
#pragma unroll
            for (int r = 0; r < kDecR; ++r) {
              const uint32_t e = (uint32_t)(tid + r * kDBlock);
              if (e < cntv) tile[e] = cur.v[r];
            }
          }
          if (cntv > (uint32_t)(kDecR * kDBlock)) {
            gf32* pval = (gf32*)pm.val + base;
            for (uint32_t e = (uint32_t)(kDecR * kDBlock + tid); e < cntv; e += kDBlock)
              tile[e] = scale ? (float)((double)pval[e] / pk.p) : pval[e];
            __builtin_amdgcn_s_waitcnt(0x0F70);                  // vmcnt(0)
          }
          wpre[tid] = block_excl_scan(__popc(cur.bw), s_tmp, nullptr);
        }
        __syncthreads();
        // ---- every lane folds its own 32 elements ------------------------------------------
        const float dz = dropped_f32(pk);
        const bool unb = pk.codec == FC_CODEC_DROPOUT_UNBIASED;
#pragma unroll
        for (int i = 0; i < kDVec; ++i) {
          const uint32_t loc0 = (uint32_t)(i * 1024 + w * 256 + lane * 4);
          const uint32_t q = loc0 >> 5, sh = loc0 & 31;
          const uint32_t wq = bb[q];
          const uint32_t nib = (wq >> sh) & 0xfu;
          float raw[4];
          if (FMT == FC_FMT_IDXVAL) {
            const float4 tv = *reinterpret_cast<const float4*>(&tile[loc0]);
            raw[0] = tv.x; raw[1] = tv.y; raw[2] = tv.z; raw[3] = tv.w;
          } else {
            const uint32_t r0 = wpre[q] + __popc(wq & ((1u << sh) - 1u));
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              raw[jj] = ((nib >> jj) & 1u) ? tile[r0 + __popc(nib & ((1u << jj) - 1u))] : 0.f;
          }
          const uint64_t eo = base + loc0;
          if (OUT64) {   // fp64 result (dropout, compression.py:52/60): divide here, per element
            double* o = reinterpret_cast<double*>(a.out);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              if (eo + jj < a.n)
                o[eo + jj] = ((nib >> jj) & 1u) ? (unb ? (double)raw[jj] / pk.p : (double)raw[jj])
                                                : (double)dz;
            continue;
          }
          // fp32 paths: the tile already holds the kept value (fl32(fl64(g)/p) applied once
          // per entry at scatter time, not per element here)
          const float4 dv = make_float4((nib & 1u) ? raw[0] : dz, (nib & 2u) ? raw[1] : dz,
                                        (nib & 4u) ? raw[2] : dz, (nib & 8u) ? raw[3] : dz);
          if (ACC) {
            const float4 cw = make_float4(__fmul_rn(dv.x, pk.w), __fmul_rn(dv.y, pk.w),
                                          __fmul_rn(dv.z, pk.w), __fmul_rn(dv.w, pk.w));
            if (m == 0 && !a.acc_in) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);   // np.sum: +0 start
            acc[i] = make_float4(__fadd_rn(acc[i].x, cw.x), __fadd_rn(acc[i].y, cw.y),
                                 __fadd_rn(acc[i].z, cw.z), __fadd_rn(acc[i].w, cw.w));
          } else {
            store_out(reinterpret_cast<float*>(a.out), eo, a.n, dv);   // single packet: done
          }
        }
        __syncthreads();                                         // tile / wpre free again
        if (FMT == FC_FMT_IDXVAL) bb[tid] = 0;                   // for item t + 2
        if (ACC && m + 1 == M) {                                 // chunk done: write the sum
#pragma unroll
          for (int i = 0; i < kDVec; ++i)
            store_out(reinterpret_cast<float*>(a.out),
                      base + (uint64_t)(i * 1024 + w * 256 + lane * 4), a.n, acc[i]);
        }
        if (++pm_i == M) { pm_i = 0; ++pj; }
      }
    }
  }
}

// --------------------------------------------------------------------------------------
// k_decode_sparse<ACC>: FC_FMT_IDXVAL packets, fp32 result.  The chunk's result lives in an
// LDS tile; each packet's kept entries are folded into it in G's row order:
//     tile[loc] = fl(tile[loc] + fl(w * v))            (ACC; __fmul_rn / __fadd_rn)
//     tile[loc] = v                                     (!ACC, single packet: the dense decode)
// so the work per packet is proportional to its entries (k), not to N: k_decode<ACC> folded
// all 8192 elements of the chunk per packet and was VALU/LDS-bound at ~38 us per 128 M packet.
//
// gar.py:44 is np.sum(G * w[:, None], axis=0): NumPy's axis-0 add.reduce starts from +0 and
// adds the rows in order (probed: tests/test_oracle_golden.py::test_numpy_axis0_sum_order),
// so the dense sum is s = fl(...fl(fl(+0 + t_0) + t_1)...).  Such a sum is never -0 (+0 + -0
// == +0, and nonzero terms never cancel to -0 under RN), so skipping a dropped coordinate's
// term d_i = fl(dz * w_i) is exact whenever d_i is +-0: the tile starts at +0 and only kept
// entries are folded.  The exception is d_i == NaN (w_i = +-inf / NaN, or dropout-unbiased
// with p == 0, where dz = 0/0): every element such a "poisoning" packet did not fold is NaN
// (cntC counts their folds).  The result is exactly the dense sum of gar.py:44 over G.
//
// Loads: every item (packet, chunk) reads its first 1024 slot entries with addresses clamped
// to the slot's count (lanes past it re-read entry 0: no extra HBM traffic, no divergent
// branch, exact vmcnt waits); the counts are loaded one group of items ahead.
// --------------------------------------------------------------------------------------
constexpr int kSBlock = 256;
constexpr int kSR = 4;                         // entries per thread per item (1024 per item)
constexpr int FC_SGROUP = 4;
constexpr int kSGroup = FC_SGROUP;             // items whose loads are issued together
constexpr int kSBlocksPerCU = 3;               // 47 KB LDS per workgroup (4 per CU with the
                                               // poison counts dropped measured no faster)

struct SparseMeta {
  const void* idx;            // uint16 chunk-local indices
  const float* val;
  const uint32_t* cnt;
  uint64_t seed, offset;
  double p;
  uint64_t thresh;
  float w;
  uint32_t flags;             // ib | codec << 8 | key_mode << 16
};

__device__ __forceinline__ PktCache meta_pkt_s(const SparseMeta& pm) {
  PktCache c;
  c.idx = pm.idx; c.val = pm.val; c.bitmap = nullptr; c.cnt = pm.cnt; c.w = pm.w;
  c.thresh = pm.thresh;
  c.ib = pm.flags & 0xffu; c.codec = (pm.flags >> 8) & 0xffu; c.key_mode = (pm.flags >> 16) & 0xffu;
  c.seed = pm.seed; c.offset = pm.offset; c.p = pm.p;
  return c;
}

template <bool ACC>
__global__ __launch_bounds__(kSBlock, kSBlocksPerCU) void k_decode_sparse(DecodeArgs a) {
  __shared__ __attribute__((aligned(16))) float tile[kChunk];
  __shared__ __attribute__((aligned(16))) uint8_t cntC[ACC ? kChunk : 16];   // poisoning folds
  __shared__ SparseMeta s_meta[ACC ? kSparseMaxM : 1];
  __shared__ uint32_t s_nC;
  const int tid = threadIdx.x;
  const uint32_t M = ACC ? (uint32_t)a.m : 1u;
  const uint32_t nch = (uint32_t)((a.n + kChunk - 1) / kChunk);
  const uint32_t G = gridDim.x;
  if (blockIdx.x >= nch) return;
  const uint32_t J = (nch - blockIdx.x + G - 1) / G;             // chunks of this workgroup
  const uint32_t T = J * M;                                      // items (chunk-major)

  if (tid == 0) s_nC = 0;
  __syncthreads();
  if (tid < (int)M) {
    const fc_packet_view v = ACC ? a.views[tid] : a.one;
    const fc_packet_hdr* h = v.hdr;
    SparseMeta d;
    d.idx = v.idx; d.val = v.val; d.cnt = v.cnt;
    d.seed = h->seed; d.offset = h->offset; d.p = h->p;
    d.thresh = h->thresh; d.w = v.weight;
    d.flags = (h->index_bits & 0xffu) | ((h->codec & 0xffu) << 8) | (h->key_mode << 16);
    // a packet whose dropped term fl(dz * w) is NaN poisons what it does not fold (bit 24)
    const float dz = (h->codec == FC_CODEC_DROPOUT_UNBIASED && h->p == 0.0) ? __uint_as_float(0x7fc00000u) : 0.0f;
    const bool poison = __fmul_rn(dz, v.weight) != __fmul_rn(dz, v.weight);
    d.flags |= (uint32_t)poison << 24;
    s_meta[tid] = d;
    if (poison) atomicAdd(&s_nC, 1u);
  }
  __syncthreads();
  const uint32_t nC = s_nC;

  // ---- per-chunk tile init / write-out (each thread owns elements tid*4 + i*1024) ----------
  auto init_tile = [&](uint32_t c) {
    const uint64_t base = (uint64_t)c * kChunk;
    float dz = 0.0f;                                             // np.sum's +0 start
    if (!ACC) dz = dropped_f32(meta_pkt_s(s_meta[0]));
#pragma unroll
    for (int i = 0; i < kChunk / (kSBlock * 4); ++i) {
      const uint32_t loc = (uint32_t)(i * 1024 + tid * 4);
      float4 v = make_float4(dz, dz, dz, dz);
      if (ACC && a.acc_in) v = load4(reinterpret_cast<const float*>(a.out), base + loc, a.n);
      *reinterpret_cast<float4*>(&tile[loc]) = v;
      if (ACC && nC) *reinterpret_cast<uint32_t*>(&cntC[loc]) = 0u;
    }
  };
  auto write_tile = [&](uint32_t c) {
    const uint64_t base = (uint64_t)c * kChunk;
    float* out = reinterpret_cast<float*>(a.out);
#pragma unroll
    for (int i = 0; i < kChunk / (kSBlock * 4); ++i) {
      const uint32_t loc = (uint32_t)(i * 1024 + tid * 4);
      float4 v = *reinterpret_cast<const float4*>(&tile[loc]);
      if (ACC && nC) {                                           // poisoning packets
        const uint32_t k4 = *reinterpret_cast<const uint32_t*>(&cntC[loc]);
        auto fix = [&](float x, uint32_t kc) { return kc < nC ? __uint_as_float(0x7fc00000u) : x; };
        v = make_float4(fix(v.x, k4 & 0xffu), fix(v.y, (k4 >> 8) & 0xffu),
                        fix(v.z, (k4 >> 16) & 0xffu), fix(v.w, k4 >> 24));
      }
      store_out(out, base + loc, a.n, v);
    }
  };

  // ---- item loads: counts one group ahead, entries clamped to the count -------------------
  // Items are walked with incremental (chunk j, packet m) cursors (no per-item div/mod);
  // past the end the cursor repeats the last item (loaded, ignored).
  uint32_t cj = 0, cm = 0;                                       // next item to count-load
  auto next_item = [&](uint32_t& m, uint32_t& c) {
    const bool in = cj < J;
    m = in ? cm : M - 1;
    c = blockIdx.x + (in ? cj : J - 1) * G;
    if (in && ++cm == M) { cm = 0; ++cj; }
  };
  auto load_cnt = [&](uint32_t m, uint32_t c) -> uint32_t {     // uniform value, vector load
    return ((gu32*)uni_ptr(s_meta[m].cnt))[c];
  };
  // Two-slot software pipeline (loads issued in the order C0 C1 E0 | C2 E1 P0 | C3 E2 P1 ...,
  // C = slot counts of a group of items, E = its entries, P = its fold): the entries of group
  // g+1 are in flight while group g is folded, and every wait is a partial vmcnt (E_g is older
  // than C_{g+2} and E_{g+1}).  Slots alternate by group parity, so nothing loaded is copied.
  uint32_t gm[2][kSGroup], gc[2][kSGroup], cntg[2][kSGroup];
  uint32_t ids_[2][kSGroup][kSR];
  float vs_[2][kSGroup][kSR];
  uint32_t cn_[2][kSGroup], im_[2][kSGroup], ic_[2][kSGroup];
  auto issue_cnt = [&](int sl) {
#pragma unroll
    for (int d = 0; d < kSGroup; ++d) {
      next_item(gm[sl][d], gc[sl][d]);
      cntg[sl][d] = load_cnt(gm[sl][d], gc[sl][d]);
    }
  };
  auto issue_ent = [&](int sl) {
#pragma unroll
    for (int d = 0; d < kSGroup; ++d) {
      im_[sl][d] = gm[sl][d]; ic_[sl][d] = gc[sl][d];
      const SparseMeta& pm = s_meta[im_[sl][d]];
      const uint64_t lo = (uint64_t)ic_[sl][d] * kChunk;
      gf32* val = (gf32*)uni_ptr(pm.val) + lo;
      gu16* idx = (gu16*)uni_ptr(pm.idx) + lo;
      cn_[sl][d] = uni32(cntg[sl][d]);
      const uint32_t last = cn_[sl][d] ? cn_[sl][d] - 1 : 0u;
#pragma unroll
      for (int r = 0; r < kSR; ++r) {
        const uint32_t e = min((uint32_t)(tid + r * kSBlock), last);
        vs_[sl][d][r] = val[e];
        ids_[sl][d][r] = idx[e];
      }
    }
  };
  auto process = [&](int sl, uint32_t t0) {
    auto& ids = ids_[sl];
    auto& vs = vs_[sl];
    auto& cn = cn_[sl];
    auto& im = im_[sl];
    auto& ic = ic_[sl];
#pragma unroll
    for (int d = 0; d < kSGroup; ++d) {
      const uint32_t t = t0 + d;
      if (t >= T) break;                                         // uniform
      const uint32_t m = im[d];
      const uint32_t c = ic[d];
      const uint64_t base = (uint64_t)c * kChunk;
      const SparseMeta pm = s_meta[m];
      const float w = __uint_as_float(uni32(__float_as_uint(pm.w)));
      const uint64_t thresh = uni64(pm.thresh);
      const uint32_t flags = uni32(pm.flags);
      const uint32_t ib = flags & 0xffu, codec = (flags >> 8) & 0xffu;
      const uint32_t key_mode = (flags >> 16) & 0xffu, poison = flags >> 24;
      const bool scale = codec == FC_CODEC_DROPOUT_UNBIASED;     // fl32(fl64(g)/p), :60
      const bool generic = scale || (key_mode == FC_KEY_PHILOX && thresh != 0);
      auto fold = [&](uint32_t loc, float v) {                   // chunk-local index
        if (loc >= (uint32_t)kChunk) return;
        if (ACC) {
          const float term = __fmul_rn(v, w);
          const float s2 = __fadd_rn(tile[loc], term);
          tile[loc] = s2;
          if (poison) cntC[loc] = (uint8_t)(cntC[loc] + 1u);
        } else {
          tile[loc] = v;
        }
      };
      if (!generic) {                                            // top-k / dropout-biased
        // a packet's locations are distinct: all tile reads first, then all writes (one LDS
        // round trip per item, not one per entry)
        uint32_t loc[kSR];
        bool ok[kSR];
        float tv[kSR];
#pragma unroll
        for (int r = 0; r < kSR; ++r) {
          const uint32_t e = (uint32_t)(tid + r * kSBlock);
          loc[r] = ids[d][r];
          const bool keep = thresh == 0 || comp_of(mag_key(vs[d][r]), (uint32_t)base + loc[r], ib) >= thresh;
          ok[r] = e < cn[d] && keep && loc[r] < (uint32_t)kChunk;
          tv[r] = 0.f;
          if (ACC && ok[r]) tv[r] = tile[loc[r]];
        }
#pragma unroll
        for (int r = 0; r < kSR; ++r) {
          if (!ok[r]) continue;
          if (ACC) {
            const float s2 = __fadd_rn(tv[r], __fmul_rn(vs[d][r], w));
            tile[loc[r]] = s2;
            if (poison) cntC[loc[r]] = (uint8_t)(cntC[loc[r]] + 1u);
          } else {
            tile[loc[r]] = vs[d][r];
          }
        }
      } else {
        const PktCache pk = meta_pkt_s(pm);
        for (int r = 0; r < kSR; ++r) {
          const uint32_t e = (uint32_t)(tid + r * kSBlock);
          const uint32_t lc = ids[d][r];
          const float v = vs[d][r];
          if (e < cn[d] && entry_kept(pk, (uint32_t)base + lc, v)) fold(lc, scale ? (float)((double)v / pk.p) : v);
        }
      }
      if (cn[d] > (uint32_t)(kSR * kSBlock)) {                   // dense slot (uniform, rare)
        const PktCache pk = meta_pkt_s(pm);
        gf32* pval = (gf32*)uni_ptr(pm.val) + base;
        gu16* pidx = (gu16*)uni_ptr(pm.idx) + base;
        for (uint32_t e = (uint32_t)(kSR * kSBlock + tid); e < cn[d]; e += kSBlock) {
          const uint32_t lc = pidx[e];
          const float v = pval[e];
          if (entry_kept(pk, (uint32_t)base + lc, v)) fold(lc, scale ? (float)((double)v / pk.p) : v);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);                      // vmcnt(0): none left pending
      }
      __syncthreads();                                           // packet m folded
      if (m + 1 == M) {                                          // chunk done
        write_tile(c);
        const uint32_t cnext = c + G;
        if (t + 1 < T) {
          __syncthreads();                                       // write-out read the tile
          init_tile(cnext);
          __syncthreads();
        }
      }
    }
  };
  issue_cnt(0);
  issue_cnt(1);
  issue_ent(0);
  init_tile(blockIdx.x);
  __syncthreads();
  for (uint32_t t0 = 0; t0 < T; t0 += 2 * kSGroup) {
    issue_cnt(0);
    issue_ent(1);
    process(0, t0);
    if (t0 + kSGroup >= T) break;                                 // uniform
    issue_cnt(1);
    issue_ent(0);
    process(1, t0 + kSGroup);
  }
}

// --------------------------------------------------------------------------------------
// k_fold_q: the FedAVG fold of FC_FMT_IDXVAL packets (aggregation.py:61-63 + gar.py:44) with
// quarter ownership.  One workgroup of 4 waves per chunk; wave q owns quarter q (2048 elements,
// an 8 KB LDS tile) and folds every packet's entries of that quarter in G's row order,
//     tile[loc] = fl(tile[loc] + fl(w * v))           (__fmul_rn / __fadd_rn, no FMA)
// with NO barrier: the quarter's entries are the slot range [qoff_q, qoff_q+1) the encoder
// recorded (include/fedcodec.h), a packet's locations are distinct, and one wave's LDS
// operations execute in order.  (k_decode_sparse<true> shared one tile among the 4 waves and
// paid a workgroup barrier per (packet, chunk): 2.73 ms per 128 packets of 128 M.)
// The chunk's quarter offsets of all M packets are loaded once, one packet per lane, and read
// back with readlane; entries are loaded in groups of kQGroup items, two groups in flight.
// +0 start, skipped dropped coordinates and NaN-poisoning packets: see k_decode_sparse.
// --------------------------------------------------------------------------------------
constexpr int kQBlock = 256;
constexpr int kQuarter = kChunk / 4;
constexpr int FC_QR = 4;
constexpr int kQR = FC_QR;                      // entry rounds (x64 lanes) loaded per item: 256
                                                // entries (a quarter holds ~205 at f = 0.1; the
                                                // rare longer item folds its rest in a tail
                                                // loop: 4 rounds + tail 17.7 us/packet against
                                                // 5 rounds 19.9, 5 + tail 18.6)
constexpr int FC_QG = 3;
constexpr int kQGroup = FC_QG;                  // items per load group
constexpr int FC_QTAIL = 8;
// FC_QTAIL > kQR: an item holding more than kQR * 64 entries folds the rest in a tail loop
// right after its rounds; only a quarter above FC_QTAIL * 64 entries takes the slow body
constexpr int kQTail = FC_QTAIL > FC_QR ? FC_QTAIL : FC_QR;

static_assert(kSparseMaxM <= 128, "k_fold_q reads the quarter offsets of <= 128 packets "
                                   "(lanes 0..63 and 64..127)");

struct QMeta {
  const void* idx;                              // uint16 chunk-local indices
  const float* val;
  const void* qoff;                             // quarter offsets, or the counts (kQNoQoff)
  const fc_packet_hdr* hdr;
  uint64_t thresh;
  float w;
  uint32_t flags;                               // ib | codec << 8 | key_mode << 16 | poison << 24
};                                              //    | kQNoQoff
// a view without quarter offsets (the encoders may be given qoff = NULL): QMeta::qoff holds the
// per-chunk counts instead, and the chunk's offsets word becomes kQWhole | cnt — every quarter
// then scans the whole slot range [0, cnt) (slow body, loc filter), so the fold stays correct
constexpr uint32_t kQNoQoff = 1u << 25;
constexpr uint64_t kQWhole = 1ull << 63;        // never set in real offsets (cnt <= 8192)

// One entry of a packet folded into the quarter tile with the full per-entry rules (the slow
// body): rand-k (Philox keys) slack filter, dropout-unbiased fl32(fl64(v)/p) scaling.
template <bool DEC>
__device__ __forceinline__ void fold_q_entry(const PktCache& pk, float w, float* qt,
                                             uint32_t qbase, uint32_t id, float v) {
  if (!entry_kept(pk, id, v)) return;
  const float x = pk.codec == FC_CODEC_DROPOUT_UNBIASED ? (float)((double)v / pk.p) : v;
  const uint32_t loc = id - qbase;
  if (loc < (uint32_t)kQuarter) qt[loc] = DEC ? x : __fadd_rn(qt[loc], __fmul_rn(x, w));
}

// DEC: the dense decode of ONE packet with the same quarter-owned waves (no workgroup barrier
// per chunk): the tile starts at the packet's dropped value (+0, or NaN for dropout-unbiased
// with p = 0) and every kept entry is ASSIGNED, tile[loc] = v (-0.0 kept), instead of folded.
template <bool ACC_IN, bool DEC = false>
__global__ __launch_bounds__(kQBlock, 4) void k_fold_q(DecodeArgs a) {
  __shared__ __attribute__((aligned(16))) float tile[kChunk];
  __shared__ QMeta s_meta[kSparseMaxM];
  __shared__ uint32_t s_mark[4][kQuarter / 32];   // poisoning packets: kept-location bits
  __shared__ uint32_t s_slow;
  const int tid = threadIdx.x, lane = lane_id();
  // wave-uniform to the compiler (tid >> 6 is not): every range derived from q stays scalar and
  // the entry loads take a scalar base + 32-bit lane offset instead of per-lane 64-bit
  // addresses (fewer VALU per entry: the fold is issue-bound, not byte-bound)
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t M = (uint32_t)a.m;
  const uint32_t c = blockIdx.x;
  const uint64_t base = (uint64_t)c * kChunk;
  const uint32_t qbase = (uint32_t)base + (uint32_t)(q * kQuarter);
  if (tid == 0) s_slow = 0;
  s_mark[q][lane] = 0u;
  __syncthreads();
  if (tid < (int)M) {
    const fc_packet_view v = DEC ? a.one : a.views[tid];
    const fc_packet_hdr* h = v.hdr;
    QMeta d;
    d.idx = v.idx; d.val = v.val; d.hdr = h;
    d.qoff = v.qoff ? (const void*)v.qoff : (const void*)v.cnt;
    d.thresh = h->thresh; d.w = v.weight;
    const uint32_t codec = h->codec, key_mode = h->key_mode;
    const float dz = (codec == FC_CODEC_DROPOUT_UNBIASED && h->p == 0.0) ? __uint_as_float(0x7fc00000u) : 0.0f;
    const bool poison = __fmul_rn(dz, v.weight) != __fmul_rn(dz, v.weight);
    // the fast body's float form of comp >= T64 needs T64's key below +inf bits (k = 0's
    // kSelectNothing and an inf / NaN k-th element take the per-entry rules)
    const bool generic = codec == FC_CODEC_DROPOUT_UNBIASED || (key_mode == FC_KEY_PHILOX && d.thresh != 0) ||
                         (d.thresh >> (h->index_bits & 0xffu)) >= 0x7f800000ull;
    d.flags = (h->index_bits & 0xffu) | ((codec & 0xffu) << 8) | ((key_mode & 0xffu) << 16) |
              ((uint32_t)poison << 24) | (v.qoff ? 0u : kQNoQoff);
    s_meta[tid] = d;
    if (poison || generic) atomicOr(&s_slow, 1u);
  }
  __syncthreads();                              // the only workgroup barriers
  const bool slow = s_slow != 0;
  // this chunk's quarter offsets of packets lane and lane + 64
  // (a per-lane pointer: each lane reads a different packet's array)
  typedef __attribute__((address_space(1))) const uint64_t gu64;
  typedef __attribute__((address_space(1))) const uint32_t gu32c;
  auto qload = [&](uint32_t m) -> uint64_t {
    const QMeta& pm = s_meta[m];
    if (pm.flags & kQNoQoff) return kQWhole | ((gu32c*)pm.qoff)[c];
    return ((gu64*)pm.qoff)[c];
  };
  const uint64_t qo0 = (uint32_t)lane < M ? qload((uint32_t)lane) : 0ull;
  const uint64_t qo1 = (uint32_t)lane + 64 < M ? qload((uint32_t)lane + 64) : 0ull;
  // a quarter holding more than kQR * 64 entries in any packet sends this wave to the slow
  // body too: the fast body has no tail loop (a load loop inside the pipeline made the
  // compiler wait vmcnt(0) for the other slot's loads)
  auto qcount = [&](uint64_t v) -> uint32_t {
    if (v & kQWhole) return kQuarter + 1u;                  // whole-chunk scan: slow body
    const uint32_t st = q == 0 ? 0u : (uint32_t)(v >> (16 * (q - 1))) & 0xffffu;
    const uint32_t en = q == 3 ? (uint32_t)(v >> 48) : (uint32_t)(v >> (16 * q)) & 0xffffu;
    return en - st;
  };
  const bool dense_q = __any(qcount(qo0) > (uint32_t)(kQTail * 64) || qcount(qo1) > (uint32_t)(kQTail * 64));
  auto range = [&](uint32_t m, uint32_t& st, uint32_t& en) {   // uniform
    const uint64_t src = m < 64 ? qo0 : qo1;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)src, (int)(m & 63));
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(src >> 32), (int)(m & 63));
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    st = q == 0 ? 0u : (uint32_t)(v >> (16 * (q - 1))) & 0xffffu;
    en = q == 3 ? (uint32_t)(v >> 48) : (uint32_t)(v >> (16 * q)) & 0xffffu;
    if (v & kQWhole) { st = 0u; en = lo & 0xffffu; }      // no qoff: the whole slot range
  };
  // ---- tile init: +0 (np.sum's start) or the partial sum being continued ----
  float* qt = tile + q * kQuarter;
  float dz0 = 0.f;                                  // DEC: the dropped coordinates' value
  if (DEC) {
    const fc_packet_hdr* h = (const fc_packet_hdr*)uni_ptr(s_meta[0].hdr);
    if (h->codec == FC_CODEC_DROPOUT_UNBIASED && h->p == 0.0) dz0 = __uint_as_float(0x7fc00000u);
  }
#pragma unroll
  for (int i = 0; i < kQuarter / 256; ++i) {
    const uint32_t loc = (uint32_t)(i * 256 + lane * 4);
    float4 v = make_float4(dz0, dz0, dz0, dz0);
    if (ACC_IN) v = load4(reinterpret_cast<const float*>(a.out), (uint64_t)qbase + loc, a.n);
    *reinterpret_cast<float4*>(&qt[loc]) = v;
  }
  if (slow || dense_q) {
    // ---- slow body (a launch holding rand-k Philox, dropout-unbiased or NaN-poisoning
    // packets, or a quarter with more than kQR * 64 entries): item by item, every rule per
    // entry ----
    for (uint32_t m = 0; m < M; ++m) {
      uint32_t st, en;
      range(m, st, en);
      const QMeta& pm = s_meta[m];
      const fc_packet_hdr* h = (const fc_packet_hdr*)uni_ptr(pm.hdr);
      PktCache pk;
      pk.thresh = uni64(pm.thresh); pk.ib = uni32(pm.flags) & 0xffu;
      pk.codec = (uni32(pm.flags) >> 8) & 0xffu; pk.key_mode = (uni32(pm.flags) >> 16) & 0xffu;
      pk.seed = h->seed; pk.offset = h->offset; pk.p = h->p;
      const float w = __uint_as_float(uni32(__float_as_uint(pm.w)));
      gu16* pidx = (gu16*)uni_ptr(pm.idx) + base;
      gf32* pval = (gf32*)uni_ptr(pm.val) + base;
      if (!DEC && ((uni32(pm.flags) >> 24) & 1u)) {   // poisoning: NaN where this packet folds nothing
        for (uint32_t e = st + lane; e < en; e += 64) {
          const uint32_t id = (uint32_t)base + pidx[e];
          const uint32_t loc = id - qbase;
          if (loc < (uint32_t)kQuarter && entry_kept(pk, id, pval[e]))
            atomicOr(&s_mark[q][loc >> 5], 1u << (loc & 31));
        }
        const uint32_t bits = s_mark[q][lane];
        for (int b = 0; b < 32; ++b)
          if (!((bits >> b) & 1u)) qt[lane * 32 + b] = __uint_as_float(0x7fc00000u);
        s_mark[q][lane] = 0u;
      }
      for (uint32_t e = st + lane; e < en; e += 64)
        fold_q_entry<DEC>(pk, w, qt, qbase, (uint32_t)base + pidx[e], pval[e]);
    }
  } else {
    // ---- fast body: top-k / mask-selected packets; two register slots of kQGroup items, the
    // loads of one group in flight while the other is folded (every wait a partial vmcnt).
    // Per entry: loc = lc & 2047 (lc - q * 2048 for an entry of this quarter), one count
    // compare and comp >= T64 in float form:
    //     comp >= T64  <=>  !(|v| <= Tf)  ||  (|v| == Tf && lc >= Ti - chunk base)
    // (Tf = T64's key as a float; NaN is unordered -> kept, its key is above every finite T).
    // Lanes past the item's end re-read its last entry and fold into a dummy slot; every tile
    // read is masked into the quarter.  (Round 2's form — 64-bit comps and a branch per read —
    // spent 34 VALU lane-ops per entry.  A uint8-index packet, ABI 4 with 64-B segment rows,
    // cut the packet bytes 16 % and made this fold 7-9 % SLOWER: the segment of each entry
    // costs VALU, and the fold is issue-bound — branch exp/abi4-u8-index,
    // profiles/r03_ab_abi4_u8_index.jsonl.)
    uint32_t ids_[2][kQGroup][kQR];
    float vs_[2][kQGroup][kQR];
    uint32_t qn_[2][kQGroup];                                   // the item's entries (uniform)
    auto issue = [&](int sl, uint32_t m0) {
#pragma unroll
      for (int d = 0; d < kQGroup; ++d) {
        const uint32_t m = min(m0 + (uint32_t)d, M - 1);          // past the end: re-load (ignored)
        uint32_t st, en;
        range(m, st, en);
        qn_[sl][d] = en - st;
        const QMeta& pm = s_meta[m];
        gf32* val = (gf32*)uni_ptr(pm.val) + base + st;
        gu16* idx = (gu16*)uni_ptr(pm.idx) + base + st;
        // lanes past the item's end re-read its last entry (one address, no extra traffic:
        // unclamped loads of the next entries cost +25 % bytes, 19.4 against 17.6 us/packet)
        const uint32_t last = en > st ? en - st - 1u : 0u;
#pragma unroll
        for (int r = 0; r < kQR; ++r) {
          const uint32_t e = min((uint32_t)(lane + r * 64), last);
          vs_[sl][d][r] = val[e];
          ids_[sl][d][r] = idx[e];
        }
      }
    };
    auto process = [&](int sl, uint32_t m0) {
#pragma unroll
      for (int d = 0; d < kQGroup; ++d) {
        const uint32_t m = m0 + (uint32_t)d;
        if (m >= M) break;                                        // uniform
        const QMeta& pm = s_meta[m];
        const float w = __uint_as_float(uni32(__float_as_uint(pm.w)));
        const uint64_t thresh = uni64(pm.thresh);
        const uint32_t ib = uni32(pm.flags) & 0xffu;
        const float Tf = __uint_as_float((uint32_t)(thresh >> ib));
        const uint32_t Ti = (uint32_t)(thresh & ((1ull << ib) - 1ull));
        const uint32_t b32 = (uint32_t)base;
        const uint32_t Tr = Ti <= b32 ? 0u : min(Ti - b32, (uint32_t)kChunk);   // tie cut in the chunk
        const uint32_t qn = qn_[sl][d];
        const int lim = (int)qn - lane;                           // entries left for this lane
        // branch-free: a lane whose entry is not folded (past the item's end, or slack below
        // T64) reads and writes its own dummy slot in s_mark (used only by slow-body waves)
        // instead of an exec-mask branch around every tile access
        float* slot[kQR];
        float tv[kQR];
        float* dummy = reinterpret_cast<float*>(&s_mark[q][lane]);
#pragma unroll
        for (int r = 0; r < kQR; ++r) {                           // all tile reads, then writes
          const uint32_t lc = ids_[sl][d][r];                     // chunk-local
          const float v = vs_[sl][d][r];
          const float av = __builtin_fabsf(v);
          const bool ok = (lim > r * 64) & (!(av <= Tf) | ((av == Tf) & (lc >= Tr)));
          slot[r] = ok ? qt + (lc & (uint32_t)(kQuarter - 1)) : dummy;
          tv[r] = DEC ? 0.f : *slot[r];
        }
#pragma unroll
        for (int r = 0; r < kQR; ++r)
          *slot[r] = DEC ? vs_[sl][d][r] : __fadd_rn(tv[r], __fmul_rn(vs_[sl][d][r], w));
        if (kQTail > kQR && qn > (uint32_t)(kQR * 64)) {          // rare, uniform: the rest
          uint32_t st, en;
          range(m, st, en);
          gf32* val = (gf32*)uni_ptr(pm.val) + base;
          gu16* idx = (gu16*)uni_ptr(pm.idx) + base;
          for (uint32_t e = st + (uint32_t)(kQR * 64) + lane; e < en; e += 64) {
            const uint32_t lc = idx[e];
            const float v = val[e];
            const float av = __builtin_fabsf(v);
            const uint32_t l2 = lc & (uint32_t)(kQuarter - 1);
            if (!(av <= Tf) | ((av == Tf) & (lc >= Tr)))
              qt[l2] = DEC ? v : __fadd_rn(qt[l2], __fmul_rn(v, w));
          }
        }
      }
    };
    issue(0, 0);
    for (uint32_t m0 = 0; m0 < M; m0 += 2 * kQGroup) {
      issue(1, m0 + kQGroup);
      process(0, m0);
      if (m0 + kQGroup >= M) break;                                // uniform
      issue(0, m0 + 2 * kQGroup);
      process(1, m0 + kQGroup);
    }
  }
  // ---- write the quarter out ----
  float* out = reinterpret_cast<float*>(a.out);
#pragma unroll
  for (int i = 0; i < kQuarter / 256; ++i) {
    const uint32_t loc = (uint32_t)(i * 256 + lane * 4);
    store_out(out, (uint64_t)qbase + loc, a.n, *reinterpret_cast<const float4*>(&qt[loc]));
  }
}

// --------------------------------------------------------------------------------------
// k_decode_res: the dense decode of a lone fused packet encode that also finishes its resolve
// (fc_topk_encode_decode), so no gather launch sits between encode and decode.  k_beta has
// placed the bin beta of the candidate histogram that holds rank r (and closed the header and the
// state when bin beta needs no ranking); every entry the packet lists is, by its key, definite
// (above the bracket: kept), a candidate binned above beta (kept), below beta (slack: below T64
// whatever T64 is) or in bin beta.  The quarter-owned waves of k_fold_q<false, true> assign the
// kept entries into their tile; a bin-beta entry goes to the small list (comp + value bits) and
// its location is NOT written by this workgroup.  The workgroup that stores bin beta's last entry
// (k_beta counted them: a counter, not a ticket in every workgroup) ranks the list, writes T64
// and stores each bin-beta location once: its value if comp >= T64, else +0.  Every output byte
// thus has one writer in the launch.
// --------------------------------------------------------------------------------------
struct DecResArgs {
  const uint16_t* idx;
  const float* val;
  const uint64_t* qoff;
  fc_packet_hdr* hdr;
  float* out;
  uint64_t n;
  uint32_t ib, pad_;
  WsPtrs W;
};

__global__ __launch_bounds__(kQBlock, 4) void k_decode_res(DecResArgs a) {
  __shared__ __attribute__((aligned(16))) float tile[kChunk];    // the finisher: its sort list
  __shared__ uint32_t s_skip[4][kQuarter / 32];                 // bin-beta locations per quarter
  __shared__ uint32_t s_fin[4];                                 // per wave: it holds the finisher
  __shared__ uint64_t s_T;
  const int tid = threadIdx.x, lane = lane_id();
  const int q = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t c = blockIdx.x;
  const uint64_t base = (uint64_t)c * kChunk;
  const uint32_t qbase = (uint32_t)base + (uint32_t)(q * kQuarter);
  // the quarter offsets with the state: one round trip for both (the offsets used to be loaded
  // only after the flags were known and a workgroup barrier)
  const uint64_t qo = a.qoff[c];
  TopkState* S = a.W.st;
  const uint32_t t_lo = S->t_lo, t_hi = S->t_hi, sbin = S->sbin;
  const uint32_t beta = S->rb_beta, flags = S->rb_flags, cnt = S->rb_cnt;
  const bool gather = (flags & 3u) == 0;                         // not retry, not rank 0
  // every wave owns its quarter of the tile, its skip bits and its finisher flag: no barrier
  // before the entries (a wave's LDS stores land in program order)
  float* qt = tile + q * kQuarter;
#pragma unroll
  for (int i = 0; i < kQuarter / 256; ++i)
    *reinterpret_cast<float4*>(&qt[i * 256 + lane * 4]) = make_float4(0.f, 0.f, 0.f, 0.f);
  s_skip[q][lane] = 0u;
  if (lane == 0) s_fin[q] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  bool finisher = false;
  if (!(flags & 1u)) {
    const uint32_t st = q == 0 ? 0u : (uint32_t)(qo >> (16 * (q - 1))) & 0xffffu;
    const uint32_t en = q == 3 ? (uint32_t)(qo >> 48) : (uint32_t)(qo >> (16 * q)) & 0xffffu;
    gu16* pidx = (gu16*)a.idx + base;
    gf32* pval = (gf32*)a.val + base;
    for (uint32_t e = st + (uint32_t)lane; e < en; e += 64) {
      const uint32_t lc = pidx[e];
      const float v = pval[e];
      const uint32_t key = mag_key(v);
      const uint32_t loc = lc & (uint32_t)(kQuarter - 1);
      const uint32_t bin = (key - t_lo) >> sbin;                // meaningful for candidates
      const bool cand = key <= t_hi;
      if (!cand || bin > beta) {                                 // beta = ~0 (rank 0): none
        qt[loc] = v;
      } else if (bin == beta && gather) {
        const uint32_t pos = atomicAdd(&S->small_n, 1u);        // < cnt <= kSmallCap (k_beta)
        st_agent(&a.W.small[pos], comp_of(key, (uint32_t)base + lc, a.ib));
        st_agent(&a.W.smallv[pos], __float_as_uint(v));
        atomicOr(&s_skip[q][loc >> 5], 1u << (loc & 31));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the entry is stored ...
        if (atomicAdd(&S->small_done, 1u) == cnt - 1u) finisher = true;   // ... then counted
      }
    }
  }
  if (finisher) s_fin[q] = 1u;
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  float* out = a.out;
#pragma unroll
  for (int i = 0; i < kQuarter / 256; ++i) {
    const uint32_t loc = (uint32_t)(i * 256 + lane * 4);
    const float4 v = *reinterpret_cast<const float4*>(&qt[loc]);
    const uint32_t skip = (s_skip[q][loc >> 5] >> (loc & 31)) & 0xfu;
    const uint64_t e = (uint64_t)qbase + loc;
    if (!skip) {
      store_out(out, e, a.n, v);
    } else {                                                     // rare: leave bin beta's locations
      if (!(skip & 1u) && e + 0 < a.n) out[e + 0] = v.x;
      if (!(skip & 2u) && e + 1 < a.n) out[e + 1] = v.y;
      if (!(skip & 4u) && e + 2 < a.n) out[e + 2] = v.z;
      if (!(skip & 8u) && e + 3 < a.n) out[e + 3] = v.w;
    }
  }
  if (!gather) return;                                           // uniform
  __syncthreads();
  if (!(s_fin[0] | s_fin[1] | s_fin[2] | s_fin[3])) return;
  // ---- the finisher: T64 = the r_in-th largest of bin beta, its locations, the header ----
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  uint64_t* sv = reinterpret_cast<uint64_t*>(tile);               // 4096 comps
  const uint32_t r_in = S->rb_rin;
  uint64_t T;
  if (cnt <= (uint32_t)kQBlock) {
    uint64_t mine = 0;
    if ((uint32_t)tid < cnt) { mine = ld_agent(&a.W.small[tid]); sv[tid] = mine; }
    __syncthreads();
    if ((uint32_t)tid < cnt) {
      uint32_t larger = 0;
      for (uint32_t j = 0; j < cnt; ++j) larger += sv[j] > mine ? 1u : 0u;
      if (larger == r_in - 1) s_T = mine;
    }
    __syncthreads();
    T = s_T;
  } else {
    uint32_t P2 = 1;
    while (P2 < cnt) P2 <<= 1;
    for (uint32_t i = tid; i < P2; i += kQBlock) sv[i] = i < cnt ? ld_agent(&a.W.small[i]) : 0ull;
    __syncthreads();
    bitonic_desc(sv, P2);
    T = sv[r_in - 1];
  }
  const uint64_t imask = (1ull << a.ib) - 1;
  for (uint32_t i = tid; i < cnt; i += kQBlock) {
    const uint64_t comp = ld_agent(&a.W.small[i]);
    const uint32_t vb = ld_agent(&a.W.smallv[i]);
    out[comp & imask] = comp >= T ? __uint_as_float(vb) : 0.0f;
  }
  if (tid == 0) {
    a.hdr->thresh = T;
    S->small_n = 0; S->small_done = 0;
  }
}

// Dense FedAVG over M row pointers (gar.py:44 with 'full' rows): one float4 per thread.
// acc_in: continue the row-order sum already in `out` (rows streamed in groups).
__global__ __launch_bounds__(kBlock) void k_wsum(const float* const* rows, const float* w,
                                                 int m, uint64_t n, float* out, int acc_in) {
  const uint64_t nq = (n + 3) / 4;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += stride) {
    const uint64_t e = q * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (acc_in) {
      if (e + 4 <= n) {
        acc = *reinterpret_cast<const float4*>(out + e);
      } else {
        acc.x = e + 0 < n ? out[e + 0] : 0.f;
        acc.y = e + 1 < n ? out[e + 1] : 0.f;
        acc.z = e + 2 < n ? out[e + 2] : 0.f;
      }
    }
    for (int r = 0; r < m; ++r) {
      const FC_G float* row = (const FC_G float*)rows[r];   // (global: rows come from memory)
      float4 x;
      if (((uintptr_t)row & 15) == 0) {        // rows of an (M, N) G with N % 4 != 0 are not
        if (e + 4 <= n) {                       // 16-B aligned: wave-uniform scalar fallback
          const fc_f4v v = __builtin_nontemporal_load((fc_gf4v*)(row + e));
          x = make_float4(v.x, v.y, v.z, v.w);
        } else {
          x.x = e + 0 < n ? row[e + 0] : 0.f;
          x.y = e + 1 < n ? row[e + 1] : 0.f;
          x.z = e + 2 < n ? row[e + 2] : 0.f;
          x.w = 0.f;
        }
      } else {
        x.x = e + 0 < n ? row[e + 0] : 0.f;
        x.y = e + 1 < n ? row[e + 1] : 0.f;
        x.z = e + 2 < n ? row[e + 2] : 0.f;
        x.w = e + 3 < n ? row[e + 3] : 0.f;
      }
      const float wr = w[r];
      const float4 cw = make_float4(__fmul_rn(x.x, wr), __fmul_rn(x.y, wr),
                                    __fmul_rn(x.z, wr), __fmul_rn(x.w, wr));
      acc = make_float4(__fadd_rn(acc.x, cw.x), __fadd_rn(acc.y, cw.y),      // from +0 (np.sum)
                        __fadd_rn(acc.z, cw.z), __fadd_rn(acc.w, cw.w));
    }
    store_out(out, e, n, acc);
  }
}

// Cluster mean (aggregation.py:91 np.mean(G[s:e], axis=0)): x = fl(x / d) in place, x the
// +0-started row-order sum of the cluster (k_decode_sparse / k_wsum with weights 1).
__global__ __launch_bounds__(kBlock) void k_div_scalar(float* x, uint64_t n, float d) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * 4;
  for (uint64_t e = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4; e < n; e += stride) {
    if (e + 4 <= n) {
      float4 v = *reinterpret_cast<float4*>(x + e);
      v = make_float4(__fdiv_rn(v.x, d), __fdiv_rn(v.y, d), __fdiv_rn(v.z, d), __fdiv_rn(v.w, d));
      *reinterpret_cast<float4*>(x + e) = v;
    } else {
      for (uint64_t i = e; i < n; ++i) x[i] = __fdiv_rn(x[i], d);
    }
  }
}

// Flat-layout staging (model_helper.py:11-13 flatten_params; client.py:52-53
// grad = current_weights - flatten_params): parameter p (grid.y) of `count` tensors is copied
// to flat[off_p, off_p + size_p) and, when `grad` is set, grad = fl32(flat_old - flat_new)
// (np.float32 subtraction) with flat updated in place to the new weights.  scatter = 1 runs
// the inverse (dist_weights_to_model / dist_grads_to_model, model_helper.py:16-35).
__global__ __launch_bounds__(kBlock) void k_flat_stage(const float* const* params, const uint64_t* offs,
                                                       float* flat, float* grad, int scatter) {
  const uint32_t p = blockIdx.y;
  const uint64_t off = offs[p], size = offs[p + 1] - off;
  float* prm = const_cast<float*>(params[p]);
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < size; i += (uint64_t)gridDim.x * kBlock) {
    if (scatter) {
      prm[i] = flat[off + i];
    } else {
      const float nw = prm[i];
      if (grad) grad[off + i] = __fsub_rn(flat[off + i], nw);
      flat[off + i] = nw;
    }
  }
}

template __global__ void k_decode<FC_FMT_IDXVAL, false, false>(DecodeArgs);
template __global__ void k_decode<FC_FMT_IDXVAL, false, true>(DecodeArgs);
template __global__ void k_decode<FC_FMT_BITMAP, false, false>(DecodeArgs);
template __global__ void k_decode<FC_FMT_BITMAP, false, true>(DecodeArgs);
template __global__ void k_fold_q<false>(DecodeArgs);
template __global__ void k_fold_q<true>(DecodeArgs);
template __global__ void k_fold_q<false, true>(DecodeArgs);
template __global__ void k_decode_sparse<false>(DecodeArgs);
template __global__ void k_decode<FC_FMT_BITMAP, true, false>(DecodeArgs);

}  // namespace fc
