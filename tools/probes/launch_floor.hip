// Launch-floor probe (diagnostic, never part of the product): how long does a launch of the
// contacts-off kernel's shape take when the waves do (a) nothing, (b) load the 37 state words of
// their env and store them back, (c) (b) with a dependent chain of N FMAs between load and store.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o mujoco_playground_amd/csrc/build/libprobe_floor.so tools/probes/launch_floor.hip
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(192, 1) k_empty(float* s, int n) {}

// ILP independent dependent-FMA chains of N steps each, fully unrolled (no loop branch)
template <int N, int ILP>
__global__ void __launch_bounds__(192, 1) k_chain(float* s, int n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  if (wave != 0 || e >= n) return;
  float v[37];
#pragma unroll
  for (int i = 0; i < 37; i++) v[i] = s[(size_t)i * n + e];
  float x[ILP];
#pragma unroll
  for (int c = 0; c < ILP; c++) x[c] = v[c];
#pragma unroll
  for (int k = 0; k < N; k++)
#pragma unroll
    for (int c = 0; c < ILP; c++) x[c] = fmaf(x[c], 0.999f, 1e-7f);
#pragma unroll
  for (int c = 0; c < ILP; c++) v[c] = x[c];
#pragma unroll
  for (int i = 0; i < 37; i++) s[(size_t)i * n + e] = v[i];
}

extern "C" int probe_launch(int which, float* s, int n, int reps, hipStream_t st) {
  const dim3 g((n + 63) / 64), b(192);
  for (int r = 0; r < reps; r++) {
    switch (which) {
      case 0: hipLaunchKernelGGL(k_empty, g, b, 0, st, s, n); break;
      case 1: hipLaunchKernelGGL((k_chain<0, 1>), g, b, 0, st, s, n); break;
      case 2: hipLaunchKernelGGL((k_chain<1000, 1>), g, b, 0, st, s, n); break;
      case 3: hipLaunchKernelGGL((k_chain<500, 2>), g, b, 0, st, s, n); break;
      case 4: hipLaunchKernelGGL((k_chain<250, 4>), g, b, 0, st, s, n); break;
      default: hipLaunchKernelGGL((k_chain<2000, 1>), g, b, 0, st, s, n); break;
    }
  }
  return (int)hipGetLastError();
}
