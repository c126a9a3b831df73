// shape_probe.hip — achievable HBM rate of the top-k encode's access shape under different
// kernel structures: every 8192-float chunk is read (32 KiB) and ~7.1 KB of its packet slot is
// written (f = 0.1: ~893 entries x 8 B), 16384 chunks x 8 gradients-worth of launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/shape_probe tools/shape_probe.hip && tools/shape_probe
// Variants (all move the same bytes):
//   slot1_nt4   one 512-thread workgroup per chunk, 16 x 4-B non-temporal loads per lane in the
//               ballot layout (k_compact_mag1's shape)
//   slot1_ld4   the same with plain loads
//   slot1_x4    one workgroup per chunk, 4 x 16-B loads per lane
//   slot2_nt4   two chunks per workgroup, both chunks' loads issued up front
//   pers_nt4    persistent (4 workgroups per CU): the next chunk's loads in flight while the
//               current one is reduced and written
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kChunk = 8192, kWr4 = 447;   // float4 written per chunk

template <bool NT>
__device__ __forceinline__ void load16(const float* g, size_t base, float (&x)[16]) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float* p = g + base + w * 256 + lane;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float* a = p + (q >> 2) * 2048 + (q & 3) * 64;
    x[q] = NT ? __builtin_nontemporal_load(a) : *a;
  }
}
__device__ __forceinline__ void write_slot(float4* o, size_t chunk, float s) {
  for (int t = threadIdx.x; t < kWr4; t += 512) o[chunk * 2048 + t] = make_float4(s, s, s, s);
}
__device__ __forceinline__ float sum16(const float (&x)[16]) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += x[q];
  return s;
}

template <bool NT>
__global__ __launch_bounds__(512) void k_slot1(const float* g, float4* o) {
  float x[16];
  load16<NT>(g, (size_t)blockIdx.x * kChunk, x);
  write_slot(o, blockIdx.x, sum16(x));
}
typedef float fx4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512) void k_slot1_x4(const fx4* g, float4* o) {
  const size_t base = (size_t)blockIdx.x * 2048;
  fx4 x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = __builtin_nontemporal_load(g + base + i * 512 + threadIdx.x);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += x[i].x + x[i].y + x[i].z + x[i].w;
  write_slot(o, blockIdx.x, s);
}
__global__ __launch_bounds__(512) void k_slot2(const float* g, float4* o) {
  float x[16], y[16];
  load16<true>(g, (size_t)(2 * blockIdx.x) * kChunk, x);
  load16<true>(g, (size_t)(2 * blockIdx.x + 1) * kChunk, y);
  write_slot(o, 2 * blockIdx.x, sum16(x));
  write_slot(o, 2 * blockIdx.x + 1, sum16(y));
}
__global__ __launch_bounds__(512) void k_pers(const float* g, float4* o, int nch) {
  float x[16], y[16];
  int c = blockIdx.x;
  if (c >= nch) return;
  load16<true>(g, (size_t)c * kChunk, x);
  for (;;) {
    const int c2 = c + gridDim.x;
    if (c2 < nch) load16<true>(g, (size_t)c2 * kChunk, y);
    write_slot(o, c, sum16(x));
    if (c2 >= nch) break;
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q] = y[q];
    c = c2;
  }
}

int main() {
  const int nch = 16384 * 8;                       // 8 x 128 M floats = 4 GiB read
  const size_t n = (size_t)nch * kChunk;
  float* g; float4* o;
  CK(hipMalloc(&g, n * 4)); CK(hipMalloc(&o, n * 4));
  CK(hipMemset(g, 0x3c, n * 4));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const double bytes = n * 4.0 + (double)nch * kWr4 * 16;
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int it = 0; it < 5; ++it) launch();
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    const double us = 1e3 * ms / 5;
    printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  for (int rep = 0; rep < 2; ++rep) {
    timeit("slot1_nt4", [&] { hipLaunchKernelGGL(k_slot1<true>, dim3(nch), dim3(512), 0, 0, g, o); });
    timeit("slot1_ld4", [&] { hipLaunchKernelGGL(k_slot1<false>, dim3(nch), dim3(512), 0, 0, g, o); });
    timeit("slot1_x4", [&] { hipLaunchKernelGGL(k_slot1_x4, dim3(nch), dim3(512), 0, 0, (const fx4*)g, o); });
    timeit("slot2_nt4", [&] { hipLaunchKernelGGL(k_slot2, dim3(nch / 2), dim3(512), 0, 0, g, o); });
    for (int grid : {1024, 2048})  {
      char nm[32]; snprintf(nm, sizeof nm, "pers_nt4_g%d", grid);
      timeit(nm, [&] { hipLaunchKernelGGL(k_pers, dim3(grid), dim3(512), 0, 0, g, o, nch); });
    }
  }
  return 0;
}
