// pmc_calib.hip — known-byte-count kernels to calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for
// the access shapes of k_compact_mag1 (MI355X_MICROARCH.md §HBM: "Other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libpmc_calib.so tools/pmc_calib.hip
// Driven by tools/pmc_calib.py under `rocprofv3 --pmc FETCH_SIZE` (and a WRITE_SIZE pass).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((address_space(1))) const float gf;

// k_compact_mag1's read: 512-thread workgroups, 8192 floats each, element
// base + i*2048 + w*256 + j*64 + lane (i, j < 4): 4 B per lane, one 256-B segment per wave
// instruction, non-temporal.  One float per workgroup is written (negligible).
__global__ __launch_bounds__(512) void k_read4_nt(const float* g, float* sink) {
  const uint32_t base = blockIdx.x * 8192u + (threadIdx.x >> 6) * 256u + (threadIdx.x & 63u);
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += __builtin_nontemporal_load((gf*)g + base + (q >> 2) * 2048 + (q & 3) * 64);
  if (s == 1234.5f) sink[blockIdx.x] = s;       // keeps the loads; never taken for randn data
}

// The guide's calibrated shape for comparison: 16 B per lane, coalesced.
__global__ __launch_bounds__(256) void k_read16(const float4* g, float* sink) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const float4 v = g[i];
  if (v.x + v.y + v.z + v.w == 1234.5f) sink[blockIdx.x] = v.x;
}

// k_compact_mag1's packet stores: 16 B per lane (uint4), coalesced.
__global__ __launch_bounds__(256) void k_write16(uint4* out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// k_compact_mag1's packet index stores since ABI 3: 8 B per lane (4 uint16 indices), coalesced.
__global__ __launch_bounds__(256) void k_write8(uint2* out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  out[i] = make_uint2((uint32_t)i, 1u);
}

// k_compact_mag1_dense's q stores: 4 B per lane in the read layout, non-temporal.
__global__ __launch_bounds__(512) void k_write4_nt(float* out) {
  const uint32_t base = blockIdx.x * 8192u + (threadIdx.x >> 6) * 256u + (threadIdx.x & 63u);
#pragma unroll
  for (int q = 0; q < 16; ++q) __builtin_nontemporal_store(1.0f, out + base + (q >> 2) * 2048 + (q & 3) * 64);
}

extern "C" int pmc_calib_run(int which, void* buf, uint64_t nfloats, void* sink) {
  switch (which) {
    case 0: hipLaunchKernelGGL(k_read4_nt, dim3((uint32_t)(nfloats / 8192)), dim3(512), 0, 0, (const float*)buf, (float*)sink); break;
    case 1: hipLaunchKernelGGL(k_read16, dim3((uint32_t)(nfloats / 1024)), dim3(256), 0, 0, (const float4*)buf, (float*)sink); break;
    case 2: hipLaunchKernelGGL(k_write16, dim3((uint32_t)(nfloats / 1024)), dim3(256), 0, 0, (uint4*)buf); break;
    case 3: hipLaunchKernelGGL(k_write4_nt, dim3((uint32_t)(nfloats / 8192)), dim3(512), 0, 0, (float*)buf); break;
    case 4: hipLaunchKernelGGL(k_write8, dim3((uint32_t)(nfloats / 512)), dim3(256), 0, 0, (uint2*)buf); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
