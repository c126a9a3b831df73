// coherence_probe.hip — which intra-launch read forms see other workgroups' atomics?
// 1024 workgroups each atomicAdd 1 to 16 counters, then the last arriver (release/acquire
// ticket) reads the counters three ways.  The counters are zeroed before each trial by
// (Z0) hipMemset, (Z1) a plain-store kernel, (Z2) an atomicExch kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_add(unsigned* cnt, unsigned* done, unsigned* out) {
  __shared__ unsigned s_last;
  if (threadIdx.x < 16) atomicAdd(&cnt[threadIdx.x * 32], 1u);   // one line per counter
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = atomicAdd(done, 1u);
    s_last = t == gridDim.x - 1;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x < 16) {
    unsigned* c = &cnt[threadIdx.x * 32];
    out[threadIdx.x] = ld_agent(c);
    out[16 + threadIdx.x] = *(volatile unsigned*)c;
    out[32 + threadIdx.x] = atomicAdd(c, 0u);
  }
  if (threadIdx.x == 0) *done = 0;
}
__global__ void k_zero_plain(unsigned* cnt) { if (threadIdx.x < 16) cnt[threadIdx.x * 32] = 0; }
__global__ void k_zero_atomic(unsigned* cnt) { if (threadIdx.x < 16) atomicExch(&cnt[threadIdx.x * 32], 0u); }
__global__ void k_read_plain(const unsigned* cnt, unsigned* sink) {   // pull lines into L2s
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = cnt[threadIdx.x * 32];
}

int main() {
  unsigned *cnt, *done, *out, *sink;
  hipMalloc(&cnt, 16 * 32 * 4); hipMalloc(&done, 4); hipMalloc(&out, 48 * 4);
  hipMalloc(&sink, 1024 * 16 * 4);
  hipMemset(done, 0, 4);
  const int trials = 200;
  int bad[3][3] = {{0}};
  for (int z = 0; z < 3; ++z) {
    for (int t = 0; t < trials; ++t) {
      if (z == 0) hipMemset(cnt, 0, 16 * 32 * 4);
      if (z == 1) hipLaunchKernelGGL(k_zero_plain, 1, 64, 0, 0, cnt);
      if (z == 2) hipLaunchKernelGGL(k_zero_atomic, 1, 64, 0, 0, cnt);
      if (t & 1) hipLaunchKernelGGL(k_read_plain, 1024, 64, 0, 0, cnt, sink);
      hipLaunchKernelGGL(k_add, 1024, 256, 0, 0, cnt, done, out);
      unsigned h[48];
      hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
      for (int m = 0; m < 3; ++m)
        for (int i = 0; i < 16; ++i)
          if (h[m * 16 + i] != 1024) { bad[z][m]++; break; }
    }
  }
  const char* zn[3] = {"memset", "plain-zero kernel", "atomicExch-zero kernel"};
  const char* mn[3] = {"ld_agent(sc1)", "plain volatile", "atomicAdd(0)"};
  for (int z = 0; z < 3; ++z)
    for (int m = 0; m < 3; ++m)
      printf("zero=%-22s read=%-16s stale trials: %d / %d\n", zn[z], mn[m], bad[z][m], trials);
  return 0;
}
