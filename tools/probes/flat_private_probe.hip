// Minimal reproducer: a C++ conditional whose operands are all
// lvalues -- two fields of a private struct and an LDS element -- is itself an lvalue, so clang
// emits a select of POINTERS (private vs LDS, through a generic pointer) and one load. Inside a
// __noinline__ device function the struct then stays a private alloca and the load is a flat load
// of a private address. Run on gfx950 (ROCm 7.2), that load returned the NEIGHBOURING field in the
// dynamics wave built as a called function (C.tran_m instead of C.tran_w: the contact regulariser's
// `qslot_tran`). This probe compares four variants per lane:
//   sel_ref_inline  : the lvalue conditional, inlined
//   sel_ref_noinline: the lvalue conditional in a __noinline__ function (the failing shape)
//   sel_val_noinline: the same with value operands (the fix in ackphys_quad.inc)
//   expected        : computed on the host
//     hipcc --offload-arch=gfx950 -O3 tools/probes/flat_private_probe.hip -o tools/probes/flat_private_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

struct Chain {
  float a[3], b[3];
  float w, m, mu;  // like QChain's tran_w, tran_m, mu_m: adjacent private floats
};

__device__ __forceinline__ void fill(Chain& C, int q) {
  for (int k = 0; k < 3; k++) {
    C.a[k] = 0.1f * (q + k);
    C.b[k] = 0.2f * (q - k);
  }
  C.w = 0.35f + 0.01f * q;  // W_TRAN-like
  C.m = 0.099f + 0.001f * q;  // MESH_TRAN-like
  C.mu = 1.0f;
}
template <bool VAL>
__device__ __forceinline__ float pick(const Chain& C, int t, const float* x) {
  if constexpr (VAL) {
    const float w = C.w, m = C.m;
    return t < 2 ? w : (t < 4 ? m : x[(t - 4) * 11 * 64 + 9 * 64 + (threadIdx.x & 63)]);
  } else {
    return t < 2 ? C.w : (t < 4 ? C.m : x[(t - 4) * 11 * 64 + 9 * 64 + (threadIdx.x & 63)]);  // an lvalue: select of pointers
  }
}
// slots visited as the kernels' FOR_QSLOTS does (a wave-uniform bit mask, loop not unrolled); the
// result of slot t is written to its row of `rows` (LDS), read back for the return value
__device__ __noinline__ void keep(Chain* c) { asm volatile("" ::"v"(c) : "memory"); }
template <bool VAL>
__device__ __forceinline__ float body(int t, int q, float* x, uint32_t wact) {
  Chain C;
  fill(C, q);
  keep(&C);  // C's address escapes: it stays in private memory (as QChain did in the noinline build)
  float s = 0.0f;
#pragma unroll 1
  for (uint32_t m = wact; m; m &= m - 1) {
    const int u = __builtin_ctz(m);
    s += pick<VAL>(C, u, x) * (u == t ? 1.0f : 0.0f);
  }
  return s;
}
template <bool VAL>
__device__ __noinline__ float body_noinline(int t, int q, float* x, uint32_t wact) { return body<VAL>(t, q, x, wact); }
__device__ __forceinline__ float body_inline(int t, int q, float* x, uint32_t wact) { return body<false>(t, q, x, wact); }

__global__ void probe(float* out, uint32_t wact) {
  __shared__ float x[4 * 11 * 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 4 * 11 * 64; i += 64) x[i] = 100.0f + i / 64;
  __syncthreads();
  const int t = lane & 7, q = lane & 3;
  out[4 * lane + 0] = body_inline(t, q, x, wact);
  out[4 * lane + 1] = body_noinline<false>(t, q, x, wact);
  out[4 * lane + 2] = body_noinline<true>(t, q, x, wact);
  // slot t's row 9 of the extras holds 100 + (t - 4) * 11 + 9
  out[4 * lane + 3] = t < 2 ? 0.35f + 0.01f * q : (t < 4 ? 0.099f + 0.001f * q : 100.0f + (t - 4) * 11 + 9);
}

int main() {
  float* d;
  float h[256];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 0xFFu);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad[3] = {0, 0, 0};
  for (int l = 0; l < 64; l++)
    for (int v = 0; v < 3; v++) bad[v] += h[4 * l + v] != h[4 * l + 3];
  printf("lanes wrong of 64: sel_ref_inline %d, sel_ref_noinline %d, sel_val_noinline %d\n", bad[0], bad[1], bad[2]);
  for (int l = 0; l < 8; l++)
    printf("lane %d (t %d): inline %.4f noinline %.4f value-noinline %.4f expected %.4f\n", l, l & 7, h[4 * l],
           h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  hipFree(d);
  return 0;
}
