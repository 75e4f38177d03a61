// Probe: cost of a lone wave's SoA dword stores vs quad-transposed dwordx4 stores (gfx950).
// hipcc --offload-arch=gfx950 -O3 -o store_probe store_probe.hip && ./store_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint64_t now() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int MODE>
__global__ void __launch_bounds__(64) probe(float* out, int n, uint64_t* cyc, float seed) {
  const int lane = threadIdx.x, e = blockIdx.x * 64 + lane;
  float w[40];
#pragma unroll
  for (int k = 0; k < 40; k++) w[k] = seed * (k + 1) + e;
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t0 = now();
  __builtin_amdgcn_sched_barrier(0);
  if (MODE == 0) {  // SoA, one dword per lane per word
#pragma unroll
    for (int k = 0; k < 40; k++) out[(size_t)k * n + e] = w[k];
  } else if (MODE == 1) {  // quad transpose via shuffles, dwordx4 per lane
    const int q = lane & 3, e0 = e - q;
#pragma unroll
    for (int kb = 0; kb < 40; kb += 4) {
      float4 v;
      // lane q gets word kb+q of lanes e0..e0+3
      float x0 = __shfl(w[kb + q], (lane & ~3) + 0, 64);
      float x1 = __shfl(w[kb + q], (lane & ~3) + 1, 64);
      float x2 = __shfl(w[kb + q], (lane & ~3) + 2, 64);
      float x3 = __shfl(w[kb + q], (lane & ~3) + 3, 64);
      v = make_float4(x0, x1, x2, x3);
      *reinterpret_cast<float4*>(out + (size_t)(kb + q) * n + e0) = v;
    }
  } else {  // same count of dword stores but AoS (one lane writes 40 consecutive words)
#pragma unroll
    for (int k = 0; k < 40; k += 4)
      *reinterpret_cast<float4*>(out + (size_t)e * 40 + k) = make_float4(w[k], w[k + 1], w[k + 2], w[k + 3]);
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t1 = now();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int n = 4096, nb = n / 64;
  float* out;
  uint64_t* cyc;
  hipMalloc(&out, sizeof(float) * 40 * n);
  hipMalloc(&cyc, sizeof(uint64_t) * nb);
  uint64_t h[64];
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(nb), dim3(64), 0, 0, out, n, cyc, 1.5f);
      if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(nb), dim3(64), 0, 0, out, n, cyc, 1.5f);
      if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(nb), dim3(64), 0, 0, out, n, cyc, 1.5f);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      uint64_t s = 0, mx = 0;
      for (int i = 0; i < nb; i++) { s += h[i]; mx = h[i] > mx ? h[i] : mx; }
      printf("mode %d rep %d: mean %llu cycles/wave (s_memtime units), max %llu, kernel %.2f us\n", mode, rep,
             (unsigned long long)(s / nb), (unsigned long long)mx, ms * 1000);
    }
  }
  return 0;
}
