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
//   acc = fl(w_0 * d_0);  acc = fl(acc + fl(w_i * d_i))   (no FMA: __fmul_rn / __fadd_rn)
// so the FedAVG of M packets reads each packet once and writes the aggregate once.
#include "fc_state.h"

namespace fc {

struct PktCache {
  const uint32_t* idx;
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

template <typename OutT>
__device__ __forceinline__ void store_out(OutT* out, uint64_t e, uint64_t n, const float4& v) {
  if (e + 4 <= n) {
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<float4*>(out + e) = v;
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
  int m;
  uint64_t n;
  void* out;
};

template <int FMT, bool ACC, bool OUT64>
__global__ __launch_bounds__(kBlock) void k_decode(DecodeArgs a) {
  __shared__ __attribute__((aligned(16))) float tile[FMT == FC_FMT_IDXVAL ? kChunk : 4];
  __shared__ uint32_t bits[kChunkWords];
  __shared__ uint32_t wpre[kChunkWords];
  __shared__ uint32_t s_tmp[8];
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t c = blockIdx.x;
  const uint64_t base = (uint64_t)c * kChunk;

  float4 acc[kVec];
  double4 out64[OUT64 ? kVec : 1];
  (void)out64;

  for (int m = 0; m < a.m; ++m) {
    const PktCache pk = load_pkt(ACC ? a.views[m] : a.one);
    const uint32_t lo = c * (uint32_t)kChunk, hi = lo + pk.cnt[c];   // chunk c's slot
    __syncthreads();                                     // previous packet fully consumed
    if (FMT == FC_FMT_IDXVAL) {
      bits[tid] = 0;
      __syncthreads();
      for (uint32_t e = lo + tid; e < hi; e += kBlock) {
        const uint32_t id = pk.idx[e];
        const float v = pk.val[e];
        const uint32_t loc = id - (uint32_t)base;
        if (loc < (uint32_t)kChunk && entry_kept(pk, id, v)) {
          tile[loc] = v;
          atomicOr(&bits[loc >> 5], 1u << (loc & 31));
        }
      }
    } else {
      const uint32_t wd = pk.bitmap[(uint64_t)c * kChunkWords + tid];
      bits[tid] = wd;
      wpre[tid] = block_excl_scan(__popc(wd), s_tmp, nullptr);
    }
    __syncthreads();
    const float dz = dropped_f32(pk);
#pragma unroll
    for (int i = 0; i < kVec; ++i) {
      const uint32_t loc0 = (uint32_t)(i * 1024 + w * 256 + lane * 4);
      const uint32_t q = loc0 >> 5, sh = loc0 & 31;
      const uint32_t wq = bits[q];
      const uint32_t nib = (wq >> sh) & 0xfu;
      float4 d;
      if (FMT == FC_FMT_IDXVAL) {
        const float4 t = *reinterpret_cast<const float4*>(&tile[loc0]);
        d.x = (nib & 1u) ? kept_f32(t.x, pk) : dz;
        d.y = (nib & 2u) ? kept_f32(t.y, pk) : dz;
        d.z = (nib & 4u) ? kept_f32(t.z, pk) : dz;
        d.w = (nib & 8u) ? kept_f32(t.w, pk) : dz;
        if (OUT64) {
          out64[i].x = (nib & 1u) ? kept_f64(t.x, pk) : (double)dz;
          out64[i].y = (nib & 2u) ? kept_f64(t.y, pk) : (double)dz;
          out64[i].z = (nib & 4u) ? kept_f64(t.z, pk) : (double)dz;
          out64[i].w = (nib & 8u) ? kept_f64(t.w, pk) : (double)dz;
        }
      } else {
        uint32_t r = lo + wpre[q] + __popc(wq & ((1u << sh) - 1u));
        float raw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) raw[j] = ((nib >> j) & 1u) ? pk.val[r + __popc(nib & ((1u << j) - 1u))] : 0.f;
        d.x = (nib & 1u) ? kept_f32(raw[0], pk) : dz;
        d.y = (nib & 2u) ? kept_f32(raw[1], pk) : dz;
        d.z = (nib & 4u) ? kept_f32(raw[2], pk) : dz;
        d.w = (nib & 8u) ? kept_f32(raw[3], pk) : dz;
        if (OUT64) {
          out64[i].x = (nib & 1u) ? kept_f64(raw[0], pk) : (double)dz;
          out64[i].y = (nib & 2u) ? kept_f64(raw[1], pk) : (double)dz;
          out64[i].z = (nib & 4u) ? kept_f64(raw[2], pk) : (double)dz;
          out64[i].w = (nib & 8u) ? kept_f64(raw[3], pk) : (double)dz;
        }
      }
      if (ACC) {
        const float4 cw = make_float4(__fmul_rn(d.x, pk.w), __fmul_rn(d.y, pk.w),
                                      __fmul_rn(d.z, pk.w), __fmul_rn(d.w, pk.w));
        if (m == 0) acc[i] = cw;
        else acc[i] = make_float4(__fadd_rn(acc[i].x, cw.x), __fadd_rn(acc[i].y, cw.y),
                                  __fadd_rn(acc[i].z, cw.z), __fadd_rn(acc[i].w, cw.w));
      } else {
        acc[i] = d;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kVec; ++i) {
    const uint64_t e = base + (uint64_t)(i * 1024 + w * 256 + lane * 4);
    if (OUT64) {
      double* o = reinterpret_cast<double*>(a.out);
      if (e + 0 < a.n) o[e + 0] = out64[i].x;
      if (e + 1 < a.n) o[e + 1] = out64[i].y;
      if (e + 2 < a.n) o[e + 2] = out64[i].z;
      if (e + 3 < a.n) o[e + 3] = out64[i].w;
    } else {
      store_out(reinterpret_cast<float*>(a.out), e, a.n, acc[i]);
    }
  }
}

// Dense FedAVG over M row pointers (gar.py:44 with 'full' rows): one float4 per thread.
__global__ __launch_bounds__(kBlock) void k_wsum(const float* const* rows, const float* w,
                                                 int m, uint64_t n, float* out) {
  const uint64_t nq = (n + 3) / 4;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += stride) {
    const uint64_t e = q * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < m; ++r) {
      const float* row = rows[r];
      float4 x;
      if (((uintptr_t)row & 15) == 0) {        // rows of an (M, N) G with N % 4 != 0 are not
        x = load4(row, e, n);                   // 16-B aligned: wave-uniform scalar fallback
      } else {
        x.x = e + 0 < n ? row[e + 0] : 0.f;
        x.y = e + 1 < n ? row[e + 1] : 0.f;
        x.z = e + 2 < n ? row[e + 2] : 0.f;
        x.w = e + 3 < n ? row[e + 3] : 0.f;
      }
      const float wr = w[r];
      const float4 cw = make_float4(__fmul_rn(x.x, wr), __fmul_rn(x.y, wr),
                                    __fmul_rn(x.z, wr), __fmul_rn(x.w, wr));
      if (r == 0) acc = cw;
      else acc = make_float4(__fadd_rn(acc.x, cw.x), __fadd_rn(acc.y, cw.y),
                             __fadd_rn(acc.z, cw.z), __fadd_rn(acc.w, cw.w));
    }
    store_out(out, e, n, acc);
  }
}

template __global__ void k_decode<FC_FMT_IDXVAL, false, false>(DecodeArgs);
template __global__ void k_decode<FC_FMT_IDXVAL, false, true>(DecodeArgs);
template __global__ void k_decode<FC_FMT_BITMAP, false, false>(DecodeArgs);
template __global__ void k_decode<FC_FMT_BITMAP, false, true>(DecodeArgs);
template __global__ void k_decode<FC_FMT_IDXVAL, true, false>(DecodeArgs);
template __global__ void k_decode<FC_FMT_BITMAP, true, false>(DecodeArgs);

}  // namespace fc
