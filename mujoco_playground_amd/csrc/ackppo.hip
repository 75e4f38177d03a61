// ackppo.hip -- on-device PPO learner kernels for gfx950 (C-ABI: include/ackppo.h).
//
// Restates stable-baselines3 2.7.0 PPO('MlpPolicy') as src/rl/train.py:99-128 configures it
// (hyper-parameters: the rl_logs/ppo checkpoints' data file). Network: 79-64-64 tanh actor and critic MLPs.
//
// Mapping:
//  * ackppo_act: 16 envs per 256-lane workgroup; weights staged in LDS (W1 transposed, both
//    layers XOR-swizzled), both layers as 16x16 f32 MFMA tiles (v_mfma_f32_16x16x4_f32; wave w
//    owns unit tiles 2w, 2w+1 of the 128 actor|critic units), heads + sampling on wave 0.
//  * ackppo_value / ackppo_bootstrap: the same kernel without the sampling (value only) or
//    without the policy step (bootstrap only), so every value of a rollout -- per step, the
//    TimeLimit bootstrap and the last values -- comes from one arithmetic path.
//  * ackppo_grad: one 256-lane workgroup per 32-sample tile. Forward layers, the W2^T backward
//    and the weight-gradient sums over the tile (kept in the MFMA accumulators across tiles)
//    are f32 MFMA tiles; heads, loss gradient and d2 on the VALU; every activation / delta
//    lives in LDS tiles [unit][sample]. Each workgroup writes one partial gradient row.
//    ackppo_reduce sums the rows (coalesced over parameters); ackppo_adam applies the global
//    norm clip and the Adam step; ackppo_epoch runs a whole epoch of minibatches in one host
//    call. No host round trip inside an update.
#include <dlfcn.h>

#include <chrono>
#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>
#include <string.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/ackppo.h"
#include "ackppo_math.inc"

#define PP_UNROLL_STR "unroll 2"

#ifdef PP_STAMPS
__device__ unsigned long long* g_pp_stamps;
#define PSTAMP(k)                                                                              \
  do {                                                                                         \
    unsigned long long _t;                                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");               \
    if (threadIdx.x == 0) g_pp_stamps[(size_t)(k)*gridDim.x + blockIdx.x] = _t;                 \
  } while (0)
// the 100 MHz constant clock (workgroup start / end across the grid: the kernel's timeline)
#define PRSTAMP(k)                                                                             \
  do {                                                                                         \
    unsigned long long _t;                                                                     \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");           \
    if (threadIdx.x == 0) g_pp_stamps[(size_t)(k)*gridDim.x + blockIdx.x] = _t;                 \
  } while (0)
#else
#define PSTAMP(k) \
  do {            \
  } while (0)
#define PRSTAMP(k) \
  do {             \
  } while (0)
#endif

namespace pp {

constexpr int NOBS = ACKPPO_NOBS, NA = ACKPPO_NACT, H = ACKPPO_HIDDEN, P = ACKPPO_NPARAM;
struct Net {
  int w1, b1, w2, b2;
};
constexpr Net ACTOR{ACKPPO_OFF_PI_W1, ACKPPO_OFF_PI_B1, ACKPPO_OFF_PI_W2, ACKPPO_OFF_PI_B2};
constexpr Net CRITIC{ACKPPO_OFF_VF_W1, ACKPPO_OFF_VF_B1, ACKPPO_OFF_VF_W2, ACKPPO_OFF_VF_B2};

using ppm::fexp;
using ppm::ftanh;
using ppm::gauss_term;
using ppm::f4v;   // f32 MFMA 16x16x4 (exact f32 products, a k-ordered fmaf chain; ackppo_math.inc)
using ppm::mfma4;

// Sum over the wave, the same rounded value in every lane. Symmetric pairings only (every step adds
// a lane's value and its partner's, so both end with the same bits): xor 1 and xor 2 inside quads,
// the 8-lane and 16-lane mirrors (DPP row_half_mirror / row_mirror), then row pairs and wave halves
// by permlane16 / permlane32 swaps. (As xor shuffles each step was a ds_bpermute round trip through
// LDS, ~120 cycles: the gradient launch's four loss sums took ~3.4k cycles at the end of every
// workgroup.) Every lane of the wave must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// v + (v of lane ^ 16) and v + (v of lane ^ 32), as the xor-shuffle sums give them bit for bit (one
// swap and one add; the add is commutative, so the odd row's lanes round the same sum)
__device__ __forceinline__ float sum_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_f<0x141>(v);  // row_half_mirror: lane i <-> 7 - i of each 8
  v += dpp_f<0x140>(v);  // row_mirror: lane i <-> 15 - i of each 16
  return sum_xor32(sum_xor16(v));  // row pairs, then the wave halves
}
// LDS written by some lanes of this wave, read by others: order the accesses (one wave's LDS
// operations execute in order) and keep the compiler from moving them across
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace pp

using namespace pp;

// ------------------------------------------------------------------ rollout kernels

struct ActArgs {
  const float* params;
  const float* obs;
  int n;
  int64_t env_offset;
  uint64_t seed;
  uint32_t step;
  int deterministic;
  float* obs_rows;
  float* action;
  float* env_action;
  float* log_prob;
  float* value;
  // previous rollout step's TimeLimit bootstrap (ackppo_act_boot; tobs == nullptr: none)
  const float* tobs;
  const float* reward;
  const uint8_t* term;
  const uint8_t* trunc;
  float gamma;
  float* reward_out;
  float* done_out;
};


extern "C" __global__ void __launch_bounds__(256) ackppo_gae_kernel(const float* rew, const float* val,
                                                                    const float* starts, const float* last_val,
                                                                    const float* last_done, int T, int n, float gamma,
                                                                    float lam, float* adv, float* ret) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float last = 0.0f;
  float next_v = last_val[e], next_nt = 1.0f - last_done[e];
  for (int t = T - 1; t >= 0; t--) {
    const size_t s = (size_t)t * n + e;
    const float v = val[s];
    const float delta = rew[s] + gamma * next_v * next_nt - v;
    last = delta + gamma * lam * next_nt * last;
    adv[s] = last;
    ret[s] = last + v;
    next_v = v;
    next_nt = 1.0f - starts[s];
  }
}

// one 1024-lane workgroup per minibatch: the gathered advantages stay in registers (ADV_CACHE per
// lane; larger minibatches re-gather the rest) for the two double-precision passes (mean, then
// the unbiased variance about it), each reduced with wave shuffles and one LDS word per wave
constexpr int ADV_THREADS = 1024, ADV_CACHE = 8;
__device__ __forceinline__ double block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // red is reused between calls
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < ADV_THREADS / 64; i++) t += red[i];
  return t;
}
extern "C" __global__ void __launch_bounds__(ADV_THREADS) ackppo_adv_stats_kernel(const float* adv, const int32_t* idx,
                                                                                  int n_idx, int batch, int normalize,
                                                                                  float* stats) {
  __shared__ double red[ADV_THREADS / 64];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int lo = m * batch, hi = min(lo + batch, n_idx), cnt = hi - lo;
  if (!normalize || cnt <= 1) {
    if (tid == 0) { stats[2 * m] = 0.0f; stats[2 * m + 1] = 1.0f; }
    return;
  }
  float v[ADV_CACHE];
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < ADV_CACHE; c++) {
    const int i = lo + tid + c * ADV_THREADS;
    v[c] = i < hi ? adv[idx[i]] : 0.0f;
    s += v[c];
  }
  for (int i = lo + tid + ADV_CACHE * ADV_THREADS; i < hi; i += ADV_THREADS) s += adv[idx[i]];
  const double mean = block_sum_d(s, red) / cnt;
  double q = 0.0;
#pragma unroll
  for (int c = 0; c < ADV_CACHE; c++) {
    const double d = (double)v[c] - mean;
    q += (lo + tid + c * ADV_THREADS < hi) ? d * d : 0.0;
  }
  for (int i = lo + tid + ADV_CACHE * ADV_THREADS; i < hi; i += ADV_THREADS) {
    const double d = adv[idx[i]] - mean;
    q += d * d;
  }
  const double var = block_sum_d(q, red) / (cnt - 1);
  if (tid == 0) {
    const float sd = (float)sqrt(var);
    stats[2 * m] = (float)mean;
    stats[2 * m + 1] = 1.0f / (sd + 1e-8f);
  }
}

// Data-parallel form of the same statistics (a world minibatch m is the union of every rank's
// minibatch m): phase 0 writes this rank's (count, sum) into moments[0..1][m]; after the host
// all-reduces those rows, phase 1 writes the squared deviations about the GLOBAL mean into
// moments[2][m]; after the second all-reduce, ackppo_adv_finalize forms the stats. The sums are
// the single-rank kernel's, so world 1 reproduces ackppo_adv_stats bit for bit.
// blockIdx.y = epoch e of an all-epoch launch (ackppo_train): idx rows [e][n_idx], moment rows
// [3][E][nmb] (E = gridDim.y; E = 1 is the per-epoch layout [3][nmb]).
extern "C" __global__ void __launch_bounds__(ADV_THREADS) ackppo_adv_moments_kernel(const float* adv,
                                                                                    const int32_t* idx, int n_idx,
                                                                                    int batch, int phase, int nmb,
                                                                                    double* moments) {
  __shared__ double red[ADV_THREADS / 64];
  const int m = blockIdx.x, tid = threadIdx.x, NM = nmb * gridDim.y, j = blockIdx.y * nmb + m;
  idx += (size_t)blockIdx.y * n_idx;
  const int lo = m * batch, hi = min(lo + batch, n_idx), cnt = hi - lo;
  if (phase == 0) {
    double s = 0.0;
    for (int i = lo + tid; i < hi; i += ADV_THREADS) s += adv[idx[i]];
    // same per-lane order as ackppo_adv_stats_kernel: cached slots then the rest, all ascending
    const double tot = block_sum_d(s, red);
    if (tid == 0) {
      moments[j] = (double)cnt;
      moments[NM + j] = tot;
      moments[2 * NM + j] = 0.0;
    }
  } else {
    const double n = moments[j];
    const double mean = n > 0.0 ? moments[NM + j] / n : 0.0;
    double q = 0.0;
    for (int i = lo + tid; i < hi; i += ADV_THREADS) {
      const double d = (double)adv[idx[i]] - mean;
      q += d * d;
    }
    const double tot = block_sum_d(q, red);
    if (tid == 0) moments[2 * NM + j] = tot;
  }
}
extern "C" __global__ void __launch_bounds__(256) ackppo_adv_finalize_kernel(const double* moments, int nmb,
                                                                             int normalize, float* stats) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= nmb) return;
  const double n = moments[m];
  if (!normalize || n <= 1.0) {
    stats[2 * m] = 0.0f;
    stats[2 * m + 1] = 1.0f;
    return;
  }
  const double mean = moments[nmb + m] / n;
  const float sd = (float)sqrt(moments[2 * nmb + m] / (n - 1.0));
  stats[2 * m] = (float)mean;
  stats[2 * m + 1] = 1.0f / (sd + 1e-8f);
}

// ------------------------------------------------------------------ update kernels

struct GradArgs {
  const float* params;
  const float* obs_rows;
  const float* actions;
  const float* old_logp;
  const float* adv;
  const float* ret;
  const int32_t* idx;
  int batch;
  const float* stats;
  float clip, ent_coef, vf_coef;
  float* gpart;
  float* lpart;
  const float* wimg;  // ackppo_grad1i: the weight image (ackppo_train_desc::weight_image)
};

// ---- Adam (torch.optim.Adam after clip_grad_norm_). Two global-norm orders: grad_norm256 (the
// C-ABI ackppo_adam: every 256-thread workgroup sums scale * grad itself, thread t: float4
// j = t + 256 k ascending, x^2 + y^2 + z^2 + w^2 each; wave shuffles; the four wave sums in order)
// and the blocked order of the update kernels (norm_block_sq / norm_from_blocks below).
struct AdamK {
  float scale, coef, b1, b2, eps, step_size, bc2_sqrt, lsmin;
};
__device__ __forceinline__ float grad_norm256(const float* __restrict__ g, float scale, float* red) {
  static_assert(P % 4 == 0, "float4 parameter vector");
  const int tid = threadIdx.x;
  constexpr int NJ = (P / 4 + 255) / 256;
  float4 v[NJ];  // every load in flight at once (a rolled loop waited for each L2 round trip in turn)
#pragma unroll
  for (int i = 0; i < NJ; i++) {
    const int j = tid + 256 * i;
    v[i] = j < P / 4 ? reinterpret_cast<const float4*>(g)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float ss = 0.0f;
#pragma unroll
  for (int i = 0; i < NJ; i++) {
    const float x = v[i].x * scale, y = v[i].y * scale, z = v[i].z * scale, w = v[i].w * scale;
    ss = fmaf(x, x, ss);
    ss = fmaf(y, y, ss);
    ss = fmaf(z, z, ss);
    ss = fmaf(w, w, ss);
  }
  ss = wave_sum(ss);
  __syncthreads();  // red may be in use
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  return sqrtf((red[0] + red[1]) + (red[2] + red[3]));
}
// The blocked order (ackppo_reduce_norm_kernel, ackppo_adam_blocked_kernel; ackppo_train and
// ackppo_epoch): norm block b (128 parameters, b < NB_N) contributes S_b = wave_sum of (scale g)^2
// over parameters 128 b + lane plus the same over 128 b + 64 + lane; the norm is the square root of
// a 256-lane tree over S_0 .. S_{NB_N - 1} (wave sums, then (w0 + w1) + (w2 + w3)). Each workgroup
// forms its own S_b in the reduction; the Adam launch after it reads all of them.
constexpr int NB_P = 128, NB_N = (P + NB_P - 1) / NB_P;
static_assert(NB_N <= 256, "one 256-lane tree over the norm blocks");
// S_b of norm block b from threads 0-127 (thread t: parameter 128 b + t, gv its gradient; red: 2
// floats of LDS); the value is returned to every thread
__device__ __forceinline__ float norm_block_sq(float gv, float scale, int b, float* red) {
  const int t = threadIdx.x;
  const bool in = t < NB_P && NB_P * b + t < P;
  const float x = in ? gv * scale : 0.0f;
  const float s = wave_sum(x * x);
  __syncthreads();  // red may be in use
  if (t < NB_P && (t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  return red[0] + red[1];
}
// the norm from the blocks' S_b (sq[b * stride], b < NB_N: visible to this workgroup), on threads 0-255 (red: 4
// floats of LDS); every thread of the workgroup gets it
__device__ __forceinline__ float norm_from_blocks(const float* sq, int stride, float* red) {
  const int t = threadIdx.x;
  float v = t < NB_N ? sq[(size_t)t * stride] : 0.0f;
  v = wave_sum(v);
  __syncthreads();
  if (t < 256 && (t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  return sqrtf((red[0] + red[1]) + (red[2] + red[3]));
}
__device__ __forceinline__ AdamK adam_k(float norm, float scale, float max_norm, float b1, float b2, float eps,
                                        float step_size, float bc2_sqrt, float lsmin) {
  return AdamK{scale, fminf(max_norm / (norm + 1e-6f), 1.0f), b1, b2, eps, step_size, bc2_sqrt, lsmin};  // clip_grad_norm_
}
// the opt-in entropy floor: log_std held at or above lsmin after its Adam step (-inf: untouched, bit for bit)
__device__ __forceinline__ float ls_floor(const AdamK& k, float ls) { return k.lsmin > -INFINITY ? fmaxf(ls, k.lsmin) : ls; }
__device__ __forceinline__ void adam_elem(const AdamK& k, float p, float g, float m, float v, float& pn, float& mn,
                                          float& vn) {
  // no fma contraction: the fused (staging) and unfused (ackppo_adam_kernel) instances must round
  // alike wherever the compiler inlines them
#pragma clang fp contract(off)
  const float gi = g * k.scale * k.coef;
  mn = m + (1.0f - k.b1) * (gi - m);                 // exp_avg.lerp_(grad, 1 - beta1)
  vn = v * k.b2 + (1.0f - k.b2) * gi * gi;           // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  pn = p - k.step_size * (mn / (sqrtf(vn) / k.bc2_sqrt + k.eps));
}

// ---- staged policy weights (ackppo_act's LDS map, floats): the first layers transposed ([k][unit],
// so a lane's 16 units are 4 contiguous 16-B reads), the second layers row-major.
// W1T: [80][128] = [k][actor|critic unit], W2: [unit][k] row-major per net. Both are XOR-swizzled
// (w1t_at / w2_at) so the MFMA operand reads -- 16 consecutive units x 4 consecutive k per wave --
// hit 64 distinct LDS banks (W1T, layer-2 W2 reads) or at most 4 lanes per bank (W2^T reads).
constexpr int W_W1T = 0, W_W2_A = 80 * 2 * H, W_W2_C = W_W2_A + H * H;
// W1T also XORs the unit index with (k >> 2) & 15: the staging writes, whose lanes hold
// consecutive k of one unit, then spread over 16 banks instead of one (the reads stay
// conflict-free: within a 16-unit block the extra XOR only permutes the units)
__device__ __forceinline__ int w1t_at(int k, int c) {
  return W_W1T + k * 2 * H + (c ^ (16 * (k & 3)) ^ ((k >> 2) & 15));
}
__device__ __forceinline__ int w2_at(int u, int k) { return u * H + (k ^ (4 * (u & 15))); }
constexpr int W_B1_A = W_W2_C + H * H, W_B2_A = W_B1_A + H, W_B1_C = W_B2_A + H, W_B2_C = W_B1_C + H;
constexpr int W_AW = W_B2_C + H, W_AB = W_AW + 2 * H, W_CW = W_AB + 4, W_CB = W_CW + H, W_LS = W_CB + 4;
constexpr int W_TOTAL = W_LS + 4;
constexpr int GRAD_THREADS = 256;
constexpr int GRAD_MAX_BLOCKS = 256;  // partial gradient rows (one per 32-sample tile) at most

__device__ __forceinline__ void stage_grad_weights(const float* __restrict__ p, float* w) {
  // Every global load of the staging is issued before the first LDS write (W1, W2 as 16-B loads,
  // the short vectors as words), so a workgroup pays one memory latency instead of one per
  // phase. First layers transposed (k row 79 = 0) and swizzled, second layers swizzled. (A
  // conflict-free LDS -> LDS transpose through a scratch tile measured slower: 14.4k -> 20.2k
  // cycles per workgroup.)
  static_assert(ACKPPO_OFF_PI_W1 % 4 == 0 && ACKPPO_OFF_VF_W1 % 4 == 0 && (H * NOBS) % 4 == 0, "16-B W1 staging");
  static_assert(ACKPPO_OFF_PI_W2 % 4 == 0 && ACKPPO_OFF_VF_W2 % 4 == 0, "16-B W2 loads");
  constexpr int N1 = H * NOBS / 4, IT1 = (2 * N1 + GRAD_THREADS - 1) / GRAD_THREADS;  // float4 per net, 10 per thread
  constexpr int IT2 = H * H / 4 / GRAD_THREADS;
  const int tid = threadIdx.x;
  float4 v[IT1], va[IT2], vc[IT2];
#pragma unroll
  for (int j = 0; j < IT1; j++) {
    const int i = tid + j * GRAD_THREADS, net = i >= N1;
    if (i < 2 * N1) v[j] = reinterpret_cast<const float4*>(p + (net ? ACKPPO_OFF_VF_W1 : ACKPPO_OFF_PI_W1))[i - net * N1];
  }
#pragma unroll
  for (int j = 0; j < IT2; j++) {
    va[j] = reinterpret_cast<const float4*>(p + ACKPPO_OFF_PI_W2)[tid + j * GRAD_THREADS];
    vc[j] = reinterpret_cast<const float4*>(p + ACKPPO_OFF_VF_W2)[tid + j * GRAD_THREADS];
  }
  // short vectors: thread t < 64 takes entry t of the 7 64-vectors; threads 64-68 the scalars
  constexpr int VSRC[7] = {ACKPPO_OFF_PI_B1, ACKPPO_OFF_PI_B2, ACKPPO_OFF_VF_B1, ACKPPO_OFF_VF_B2,
                           ACKPPO_OFF_ACT_W, ACKPPO_OFF_ACT_W + H, ACKPPO_OFF_VAL_W};
  constexpr int VDST[7] = {W_B1_A, W_B2_A, W_B1_C, W_B2_C, W_AW, W_AW + H, W_CW};
  float vs[7];
  if (tid < H) {
#pragma unroll
    for (int j = 0; j < 7; j++) vs[j] = p[VSRC[j] + tid];
  }
  const int sc = tid - H;  // 0: act_b[0], 1: act_b[1], 2: log_std[0], 3: log_std[1], 4: val_b
  const bool has_sc = sc >= 0 && sc < 5;
  const float vsc = has_sc ? p[sc < 2 ? ACKPPO_OFF_ACT_B + sc : (sc < 4 ? ACKPPO_OFF_LOG_STD + sc - 2 : ACKPPO_OFF_VAL_B)]
                           : 0.0f;
#pragma unroll
  for (int j = 0; j < IT1; j++) {
    const int i = tid + j * GRAD_THREADS, net = i >= N1;
    if (i < 2 * N1) {
      const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int r = 4 * (i - net * N1) + c, u = r / NOBS, k = r - u * NOBS;
        w[w1t_at(k, net * H + u)] = e[c];
      }
    }
  }
  if (tid < 2 * H) w[w1t_at(NOBS, tid)] = 0.0f;
#pragma unroll
  for (int j = 0; j < IT2; j++) {
    const int i = 4 * (tid + j * GRAD_THREADS), u = i / H, k = i - u * H;  // 4 k of one row
    const float ea[4] = {va[j].x, va[j].y, va[j].z, va[j].w}, ec[4] = {vc[j].x, vc[j].y, vc[j].z, vc[j].w};
#pragma unroll
    for (int c = 0; c < 4; c++) {
      w[W_W2_A + w2_at(u, k + c)] = ea[c];
      w[W_W2_C + w2_at(u, k + c)] = ec[c];
    }
  }
  if (tid < H) {
#pragma unroll
    for (int j = 0; j < 7; j++) w[VDST[j] + tid] = vs[j];
  }
  if (has_sc) w[sc < 2 ? W_AB + sc : (sc < 4 ? W_LS + sc - 2 : W_CB)] = vsc;
}

// ---- ackppo_grad: one net per workgroup. Workgroup 2 t + net takes the actor (net 0) or the critic
// (net 1) of 32-sample tile t. Its LDS (one net's weights, the tile and its activations, ~78 KB) lets
// TWO workgroups share a CU, so one workgroup's barrier waits and memory latencies hide under the
// other's MFMA / VALU work (round 3's two-net workgroup filled a CU's LDS alone: 4 waves per CU, one
// per SIMD; 26.6 -> 23.8 us per 8192-sample minibatch). Wave w owns unit tile w (16 units) of its
// net in every product, for both 16-sample halves of the tile. D1 overwrites H1 in place once the
// W2 gradient has read H1 (two barriers), which is what brings the footprint under 80 KB.
namespace g1 {
constexpr int T = 32, LDP = 36;  // samples per tile, padded tile row (floats)
// weights: W1T [80][64] = [k][unit], XOR-swizzled as w1t_at (64-wide rows: the 16-bank groups of
// the four k of an MFMA read stay distinct); W2 [unit][k] swizzled as w2_at
constexpr int W1T = 0, W2 = W1T + 80 * H, B1 = W2 + H * H, B2 = B1 + H;
constexpr int HW = B2 + H;            // heads: actor [2][64] (critic [1][64])
constexpr int HB = HW + 2 * H;        // actor: b[2], log_std[2] (critic: b[1])
constexpr int WEND = HB + 4;
// the tile regions start at TBASE = WEND rounded up to whole 64-lane float4 rounds (ACKPPO_WIMAGE):
// the weight image's LDS-DMA copies (grad1i) write whole rounds, and their padding must not land in
// a tile that another wave is already filling (the first tile's X is written before the barrier)
constexpr int TBASE = (WEND + 255) / 256 * 256;
constexpr int X = TBASE, H1 = X + 80 * LDP, H2 = H1 + H * LDP, D2 = H2 + H * LDP;  // D1 overwrites H1
constexpr int GA = D2 + H * LDP;      // actor: gmu [2][LDP], glog [2][LDP]; critic: gv [LDP]
constexpr int TOTAL1 = GA + 4 * LDP;
constexpr int TSZ = TOTAL1 - TBASE;  // one tile's region (X .. GA)
// NT tiles per workgroup: 512 threads, the two tiles' waves share one staged copy of the net's
// weights and one partial row (half the rows for the reduction), one workgroup per CU (measured
// against one 256-thread tile per workgroup, two workgroups per CU: 18.9 vs 19.9 us, round 4)
constexpr int NT = 2;
static_assert(NT == 1 || NT == 2, "one or two tiles per workgroup");
constexpr int TOTAL = TBASE + NT * TSZ;
static_assert(NT == 2 ? TOTAL * 4 <= 160 * 1024 : TOTAL * 4 * 2 <= 160 * 1024,
              "two one-net grad workgroups (or one two-tile workgroup) per CU's 160 KiB LDS");
// NT == 2: the end-of-kernel exchange of the halves' accumulators fits a tile region
static_assert(22 * 256 <= TSZ && 16 * 256 <= TSZ, "accumulator exchange");
__device__ __forceinline__ int w1t(int k, int u) { return W1T + k * H + (u ^ (16 * (k & 3)) ^ ((k >> 2) & 15)); }
__device__ __forceinline__ int w2(int u, int k) { return W2 + w2_at(u, k); }
constexpr int MAX_TILES = GRAD_MAX_BLOCKS;  // partial rows: one per tile (both nets' workgroups write it)
// the weight image (ackppo_train_desc::weight_image): net n's LDS weight block [0, WEND) at
// n * WIMG, padded to whole 64-lane rounds of float4 copies
constexpr int WIMG = ACKPPO_WIMAGE;
static_assert(WEND <= WIMG && WIMG % 256 == 0 && WIMG - WEND < 256 && WIMG == TBASE,
              "weight image: WEND in whole 64-lane float4 rounds, the tiles after them");
static_assert(WIMG <= TOTAL, "the image copy's padding lands inside the workgroup's LDS");
// image position of parameter p (-1: a pad word); the inverse of stage_net's LDS map
__device__ __forceinline__ int wimg_index(int p) {
  constexpr int NW1 = H * NOBS, NW2 = H * H;
  if (p < ACKPPO_OFF_PI_W1) return p < 2 ? HB + 2 + p : -1;  // log_std
  if (p >= ACKPPO_OFF_ACT_W) {
    if (p < ACKPPO_OFF_ACT_B) return HW + (p - ACKPPO_OFF_ACT_W);
    if (p < ACKPPO_OFF_ACT_B + 2) return HB + (p - ACKPPO_OFF_ACT_B);
    if (p < ACKPPO_OFF_VAL_W) return -1;
    if (p < ACKPPO_OFF_VAL_B) return WIMG + HW + (p - ACKPPO_OFF_VAL_W);
    return p == ACKPPO_OFF_VAL_B ? WIMG + HB : -1;
  }
  const int net = p >= ACKPPO_OFF_VF_W1 ? 1 : 0;
  const int r = p - (net ? ACKPPO_OFF_VF_W1 : ACKPPO_OFF_PI_W1);  // within [W1][b1][W2][b2]
  const int base = net * WIMG;
  if (r < NW1) return base + w1t(r % NOBS, r / NOBS);
  if (r < NW1 + H) return base + B1 + (r - NW1);
  if (r < NW1 + H + NW2) return base + w2((r - NW1 - H) / H, (r - NW1 - H) % H);
  return base + B2 + (r - NW1 - H - NW2);
}
}  // namespace g1

// LDS weight layout of the grad kernel ackppo_grad1 (g1: W1T swizzled, W2 swizzled)
struct L1 {
  static __device__ __forceinline__ void w1(float* w, int u, int k, float x) { w[g1::w1t(k, u)] = x; }
  static __device__ __forceinline__ void w2(float* w, int u, int k, float x) { w[g1::w2(u, k)] = x; }
  static constexpr int B1 = g1::B1, B2 = g1::B2, HW = g1::HW, HB = g1::HB;
};
template <class LY = L1, int NTHR = GRAD_THREADS>
__device__ __forceinline__ void stage_net(const float* __restrict__ params, float* w, int net) {
  // all global loads first (one latency), then the LDS writes: W1 (float4 rows of 79 inputs)
  // transposed and swizzled, W2 swizzled, the short vectors
  constexpr int N1 = H * NOBS / 4, IT1 = (N1 + NTHR - 1) / NTHR, IT2 = H * H / 4 / NTHR;
  static_assert(H * H / 4 % NTHR == 0, "whole W2 float4 rounds");
  const int tid = threadIdx.x;
  const int o1 = net ? ACKPPO_OFF_VF_W1 : ACKPPO_OFF_PI_W1, o2 = net ? ACKPPO_OFF_VF_W2 : ACKPPO_OFF_PI_W2;
  float4 v[IT1], v2[IT2];
#pragma unroll
  for (int j = 0; j < IT1; j++) {
    const int i = tid + j * NTHR;
    if (i < N1) v[j] = *reinterpret_cast<const float4*>(params + o1 + 4 * i);
  }
#pragma unroll
  for (int j = 0; j < IT2; j++) v2[j] = *reinterpret_cast<const float4*>(params + o2 + 4 * (tid + j * NTHR));
  __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the scatter (one memory latency)
  // short vectors: threads 0-63 b1, b2 and the head rows; 64-67 the head biases / log_std
  float b1 = 0.f, b2 = 0.f, hw0 = 0.f, hw1 = 0.f, hs = 0.f;
  if (tid < H) {
    b1 = params[(net ? ACKPPO_OFF_VF_B1 : ACKPPO_OFF_PI_B1) + tid];
    b2 = params[(net ? ACKPPO_OFF_VF_B2 : ACKPPO_OFF_PI_B2) + tid];
    hw0 = params[(net ? ACKPPO_OFF_VAL_W : ACKPPO_OFF_ACT_W) + tid];
    if (!net) hw1 = params[ACKPPO_OFF_ACT_W + H + tid];
  }
  const int sc = tid - H;  // actor: 0, 1 action_net.bias, 2, 3 log_std; critic: 0 value_net.bias
  const bool has_sc = sc >= 0 && sc < (net ? 1 : 4);
  if (has_sc)
    hs = params[net ? ACKPPO_OFF_VAL_B : (sc < 2 ? ACKPPO_OFF_ACT_B + sc : ACKPPO_OFF_LOG_STD + sc - 2)];
#pragma unroll
  for (int j = 0; j < IT1; j++) {
    const int i = tid + j * NTHR;
    if (i < N1) {
      const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int r = 4 * i + c, u = r / NOBS, kk = r - u * NOBS;
        LY::w1(w, u, kk, e[c]);
      }
    }
  }
  if (tid < H) LY::w1(w, tid, NOBS, 0.0f);  // input 79: the zero pad of the 80-deep layer-1 product
#pragma unroll
  for (int j = 0; j < IT2; j++) {
    const int i = 4 * (tid + j * NTHR), u = i / H, kk = i - u * H;
    const float e[4] = {v2[j].x, v2[j].y, v2[j].z, v2[j].w};
#pragma unroll
    for (int c = 0; c < 4; c++) LY::w2(w, u, kk + c, e[c]);
  }
  if (tid < H) {
    w[LY::B1 + tid] = b1;
    w[LY::B2 + tid] = b2;
    w[LY::HW + tid] = hw0;
    w[LY::HW + H + tid] = hw1;
  }
  if (has_sc) w[LY::HB + sc] = hs;
}

// ackppo_grad1i's staging: the net's weight image copied into LDS by LDS-DMA (global_load_lds,
// 16 B per lane: lane l of a wave writes float4 (base + l), the image already in the LDS layout) --
// no registers, no transposing writes. The copies land behind the tile loop's first barrier.
template <int NTHR>
__device__ __forceinline__ void stage_image(const float* __restrict__ img, float* w) {
  constexpr int N4 = g1::WIMG / 4;
  static_assert(N4 % 64 == 0, "whole 64-lane rounds");
  const int tid = threadIdx.x, wbase = tid & ~63;
#pragma unroll
  for (int j = 0; j < (N4 + NTHR - 1) / NTHR; j++) {
    const int i0 = j * NTHR + wbase;  // wave-uniform: the round's LDS base
    if (i0 < N4)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(img + 4 * (i0 + (tid & 63))),
                                       (__attribute__((address_space(3))) void*)(w + 4 * i0), 16, 0, 0);
  }
}
// the weight image of both nets from the parameters (once per ackppo_train call; every Adam step
// then keeps it in step): stage_net's LDS map, written to HBM, pad words zero
extern "C" __global__ void __launch_bounds__(GRAD_THREADS) ackppo_wimage_kernel(const float* params, float* img) {
  const int net = blockIdx.x;
  float* w = img + net * g1::WIMG;
  for (int i = threadIdx.x; i < g1::WIMG; i += GRAD_THREADS) w[i] = 0.0f;
  __syncthreads();
  stage_net<L1>(params, w, net);
}

__device__ __forceinline__ float row_sum_t(const float* a) {  // 32 samples of one LDS tile row
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < g1::T; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(a + i);
    s += (v.x + v.y) + (v.z + v.w);
  }
  return s;
}
__device__ __forceinline__ float row_dot_t(const float* a, const float* b) {
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < g1::T; i += 4) {
    const float4 u = *reinterpret_cast<const float4*>(a + i), v = *reinterpret_cast<const float4*>(b + i);
    s = fmaf(u.x, v.x, s);
    s = fmaf(u.y, v.y, s);
    s = fmaf(u.z, v.z, s);
    s = fmaf(u.w, v.w, s);
  }
  return s;
}

// vector gradient items of the one-net workgroup: actor i < 64 b1 (D1 rows), < 128 b2 (D2 rows),
// < 256 action_net.weight (gmu[d] . H2 rows), 256-257 its bias, 258-259 log_std; critic i < 64 b1,
// < 128 b2, < 192 value_net.weight (gv . H2 rows), 192 its bias
constexpr int G1_NVA = 260, G1_NVC = 193;
__device__ __forceinline__ float vec_item_g1(const float* tl, int net, int i) {
  using namespace g1;
  if (i < 64) return row_sum_t(tl + H1 + i * LDP);  // after D1 replaced H1
  if (i < 128) return row_sum_t(tl + D2 + (i - 64) * LDP);
  if (net == 0) {
    if (i < 256) return row_dot_t(tl + GA + ((i - 128) >> 6) * LDP, tl + H2 + ((i - 128) & 63) * LDP);
    return row_sum_t(tl + GA + (i < 258 ? i - 256 : 2 + i - 258) * LDP);
  }
  if (i < 192) return row_dot_t(tl + GA, tl + H2 + (i - 128) * LDP);
  return row_sum_t(tl + GA);
}
__device__ __forceinline__ int vec_offset_g1(int net, int i) {
  if (i < 64) return (net ? ACKPPO_OFF_VF_B1 : ACKPPO_OFF_PI_B1) + i;
  if (i < 128) return (net ? ACKPPO_OFF_VF_B2 : ACKPPO_OFF_PI_B2) + i - 64;
  if (net == 0) {
    if (i < 256) return ACKPPO_OFF_ACT_W + (i - 128);
    return i < 258 ? ACKPPO_OFF_ACT_B + i - 256 : ACKPPO_OFF_LOG_STD + i - 258;
  }
  return i < 192 ? ACKPPO_OFF_VAL_W + (i - 128) : ACKPPO_OFF_VAL_B;
}

// the workgroup's loss sums into its loss row (threads 0-3: sum tid of the four)
__device__ __forceinline__ void loss_row(const GradArgs& A, int row, int net, float s) {
  const int tid = threadIdx.x;
  float* lp = A.lpart + (size_t)row * ACKPPO_NLOSS;
  if (net == 0) {
    lp[tid == 0 ? 0 : tid + 1] = s;  // policy loss, clipped count, approx-kl sum, samples
    if (tid == 0) lp[5] = lp[6] = lp[7] = 0.0f;
  } else if (tid == 0) {
    lp[1] = s;  // value loss sum
  }
}
namespace g1 {
constexpr int LS_SLOT = 22 * GRAD_THREADS;  // a half's four waves' loss sums, after its hand-over words
static_assert(LS_SLOT + 16 <= TSZ, "loss sums in the hand-over region");
}  // namespace g1
template <bool IMG = false>
__device__ __forceinline__ void grad1(const GradArgs& A) {
  using namespace g1;
  PRSTAMP(13);
  PSTAMP(0);
  extern __shared__ float tl[];
  constexpr int NTHR = GRAD_THREADS * NT;
  const int tid = threadIdx.x, lane = tid & 63;
  // NT == 2: waves 0-3 take tile 2 g of tile group g, waves 4-7 tile 2 g + 1 (half = 1); htid is
  // the thread's index within its half (every per-tile role below is the 256-thread one)
  const int wave8 = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = NT == 1 ? 0 : wave8 >> 2, wave = wave8 & 3, htid = tid & (GRAD_THREADS - 1);
  const int net = blockIdx.x & 1, grp0 = blockIdx.x >> 1, gstride = gridDim.x >> 1;
  float* w = tl;
  const float invB = 1.0f / (float)A.batch;
  const int ntiles = (A.batch + T - 1) / T, ngrp = (ntiles + NT - 1) / NT;
  const int li = lane & 15, lk = lane >> 4;
  const int ub = 16 * wave;  // the wave's unit tile
  // heads' lane roles: wave w, samples 8 w + (lane & 7); actor lanes (d = (lane >> 3) & 1, quarter
  // q = lane >> 4 of the 64 inputs), critic lanes (eighth q = lane >> 3)
  const int hs = 8 * wave + (lane & 7);
  // the minibatch's advantage moments, read first (the actor heads read them in the loop, where the
  // load sat on the heads phase's critical path)
  const float adv_mean = A.stats[0], adv_inv_sd = A.stats[1];
  float xg[10];
  float hin[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // a tile's gathers: the observation rows (X) and the heads' per-sample inputs (hin), each behind its
  // sample-index load
  auto row_idx = [&](int tile) __attribute__((always_inline)) {
    const int s0 = tile * T, nvalid = max(0, min(T, A.batch - s0));
    return A.idx[nvalid > 0 ? s0 + min(htid >> 3, nvalid - 1) : 0];
  };
  auto gather_x = [&](int tile, int ir) __attribute__((always_inline)) {
    // unconditional loads from valid addresses (a clamped sample and input), zeros selected after:
    // conditional loads compile to exec-masked branches that wait for each load in turn. A tile
    // past the batch (the second half of a last, odd group) has nvalid = 0: sample 0's rows, all zeroed
    const int s0 = tile * T, nvalid = max(0, min(T, A.batch - s0));
    const int r = htid >> 3, q = htid & 7;
    const float* row = A.obs_rows + (size_t)ir * NOBS;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const int k = q * 10 + i;
      const float v = row[min(k, NOBS - 1)];
      xg[i] = (r < nvalid && k < NOBS) ? v : 0.0f;
    }
  };
  // the heads' per-sample inputs, unmasked (a clamped sample past the batch reads valid rows): the
  // heads zero them for invalid samples where they use them, so nothing waits for these loads
  // before then (selects right behind the loads had each wave wait out the index and the row
  // latencies before layer 1)
  auto head_idx = [&](int tile) __attribute__((always_inline)) {
    const int s0 = tile * T, nvalid = max(0, min(T, A.batch - s0));
    return A.idx[nvalid > 0 ? s0 + min(hs, nvalid - 1) : 0];
  };
  // (straight-line: the critic loads the actor's three words too and never reads them -- with a
  // branch per net the two paths' registers were merged by copies that waited for the loads)
  auto gather_h = [&](int sidx) __attribute__((always_inline)) {
    hin[0] = *(net ? A.ret + sidx : A.actions + 2 * (size_t)sidx);
    hin[1] = A.actions[2 * (size_t)sidx + 1];
    hin[2] = A.old_logp[sidx];
    hin[3] = A.adv[sidx];
  };
  auto loads = [&](int tile) __attribute__((always_inline)) {
    gather_x(tile, row_idx(tile));
  };

  int hx = 0;  // grad1i: the first tile's heads sample index (loaded with the rows' index)
  if constexpr (IMG) {
    // the first tile's sample indices, then the weight image's LDS-DMA copies (no registers), then the
    // rows those indices address: the two dependent gathers run under the copies instead of after them
    // (vmcnt retires in issue order, so the gathers' addresses wait only for the older index loads)
    // (the heads' inputs are gathered in the loop: they are needed only after both layers)
    int ir = 0;
    if (grp0 < ngrp) {
      ir = row_idx(NT * grp0 + half);
      hx = head_idx(NT * grp0 + half);
    }
    stage_image<NTHR>(A.wimg + net * WIMG, w);
    if (grp0 < ngrp) gather_x(NT * grp0 + half, ir);
    // the LDS-DMA copies count in vmcnt, not lgkmcnt: drain them before the first barrier makes the
    // block visible to the other waves (on gfx950 neither the barrier nor a workgroup fence waits)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (grp0 < ngrp) {  // the first tile's X into its (DMA-free) tile region now: xg dies here
      float* tb0 = tl + half * TSZ;
      const int r = htid >> 3, q = htid & 7;
#pragma unroll
      for (int i = 0; i < 10; i++) tb0[X + (q * 10 + i) * LDP + r] = xg[i];
    }
  } else {
    stage_net<L1, NTHR>(A.params, w, net);
  }

  f4v gw1[5], gw2[4];
#pragma unroll
  for (int j = 0; j < 5; j++) gw1[j] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int j = 0; j < 4; j++) gw2[j] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
  float accv[2] = {0.0f, 0.0f};  // vector items tid and tid + 256 (vec_item_g1)
  float la = 0.0f, lb = 0.0f, lc = 0.0f, ln = 0.0f;

  for (int grp = grp0; grp < ngrp; grp += gstride) {  // the same trip count in both halves (barriers)
    const int tile = NT * grp + half;
    // an opaque zero per tile: every LDS address below depends on it, so none is hoisted out of the
    // tile loop (the hoisted swizzled addresses filled the register file and spilled)
    int zo = 0;
    asm volatile("" : "+v"(zo));
    float* tb = tl + zo + half * TSZ;
    const float* wb = tl + zo;
    const int s0 = tile * T, nvalid = max(0, min(T, A.batch - s0));
    __syncthreads();  // the previous tile's LDS reads are done (and the weights staged)
    int sidx = hx;  // grad1i's first tile: X in LDS already, the heads' index loaded with the rows'
    if (!(IMG && grp == grp0)) {
      loads(tile);
      const int r = htid >> 3, q = htid & 7;
#pragma unroll
      for (int i = 0; i < 10; i++) tb[X + (q * 10 + i) * LDP + r] = xg[i];
      sidx = head_idx(tile);
    }
    gather_h(sidx);  // one load site: hin stays in flight through both layers
    __syncthreads();
    PSTAMP(1);
    {  // layer 1: H1 [64 x 32] = tanh(W1 X + b1)
      f4v a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      // software-pipelined by blocks of KB k-steps: block b + 1's operand reads are issued before
      // block b's MFMAs, so the LDS latency hides under them (left to the scheduler, each k-step
      // read its X pair into the same two registers and waited for it)
      constexpr int KB = 5, NBK = 20 / KB;
      float bias[4];  // read with the first operands (the epilogue waited for each in turn)
#pragma unroll
      for (int r = 0; r < 4; r++) bias[r] = wb[B1 + ub + 4 * lk + r];
      float wa[2][KB], xa[2][KB], xb[2][KB];
      auto ld1 = [&](int b, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < KB; s++) {
          const int k = 4 * (b * KB + s) + lk;
          wa[buf][s] = wb[w1t(k, ub + li)];
          xa[buf][s] = tb[X + k * LDP + li];
          xb[buf][s] = tb[X + k * LDP + 16 + li];
        }
      };
      ld1(0, 0);
#pragma unroll
      for (int b = 0; b < NBK; b++) {
        if (b + 1 < NBK) ld1(b + 1, (b + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < KB; s++) {
          a0 = mfma4(wa[b & 1][s], xa[b & 1][s], a0);
          a1 = mfma4(wa[b & 1][s], xb[b & 1][s], a1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int u = ub + 4 * lk + r;
        const float bb = bias[r];
        tb[H1 + u * LDP + li] = ftanh(a0[r] + bb);
        tb[H1 + u * LDP + 16 + li] = ftanh(a1[r] + bb);
      }
    }
    __syncthreads();
    PSTAMP(2);
    {  // layer 2: H2 [64 x 32] = tanh(W2 H1 + b2)
      f4v a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      constexpr int KB = 4, NBK = H / 4 / KB;  // pipelined as layer 1
      float bias[4];
#pragma unroll
      for (int r = 0; r < 4; r++) bias[r] = wb[B2 + ub + 4 * lk + r];
      float wa[2][KB], xa[2][KB], xb[2][KB];
      auto ld2 = [&](int b, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < KB; s++) {
          const int k = 4 * (b * KB + s) + lk;
          wa[buf][s] = wb[w2(ub + li, k)];
          xa[buf][s] = tb[H1 + k * LDP + li];
          xb[buf][s] = tb[H1 + k * LDP + 16 + li];
        }
      };
      ld2(0, 0);
#pragma unroll
      for (int b = 0; b < NBK; b++) {
        if (b + 1 < NBK) ld2(b + 1, (b + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < KB; s++) {
          a0 = mfma4(wa[b & 1][s], xa[b & 1][s], a0);
          a1 = mfma4(wa[b & 1][s], xb[b & 1][s], a1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int u = ub + 4 * lk + r;
        const float bb = bias[r];
        tb[H2 + u * LDP + li] = ftanh(a0[r] + bb);
        tb[H2 + u * LDP + 16 + li] = ftanh(a1[r] + bb);
      }
    }
    __syncthreads();
    PSTAMP(3);
    const bool hvalid = hs < nvalid;
#pragma unroll
    for (int i = 0; i < 4; i++) hin[i] = hvalid ? hin[i] : 0.0f;
    if (net == 0) {  // actor heads: mu[d] of sample hs, a 16-term quarter per lane, butterflies over q
      const int d = (lane >> 3) & 1, q = lane >> 4;
      float m = 0.0f;
#pragma unroll
      for (int j = 0; j < 16; j++) {  // k order rotated by 2q: the four quarters' H2 reads hit distinct banks
        const int k = 16 * q + ((j + 2 * q) & 15);
        m = fmaf(wb[HW + d * H + k], tb[H2 + k * LDP + hs], m);
      }
      m = sum_xor32(sum_xor16(m));  // = m + m^16, then + ^32 (the xor-shuffle sums, bit for bit)
      m += wb[HB + d];
      const float mo = dpp_f<0x128>(m);  // the other dimension's mean: lane ^ 8 (row_ror 8)
      const float mu0 = d ? mo : m, mu1 = d ? m : mo;
      const float ls0 = wb[HB + 2], ls1 = wb[HB + 3];
      const float logp = gauss_term(hin[0], mu0, ls0) + gauss_term(hin[1], mu1, ls1);
      const float lr = logp - hin[2];
      const float r = fexp(lr);
      const float adv = (hin[3] - adv_mean) * adv_inv_sd;
      const float rc = fminf(fmaxf(r, 1.0f - A.clip), 1.0f + A.clip);
      const float l1 = adv * r, l2 = adv * rc;
      // d(-min(l1, l2))/dlogp: through l1 when it is the minimum (ties: torch.min splits the
      // gradient and the clamp passes it, so the sum is the full l1 gradient), else 0
      const float glogp = hvalid ? ((l1 <= l2) ? -adv * r * invB : 0.0f) : 0.0f;
      if (q == 0) {
        const float ls = d ? ls1 : ls0, mu = d ? mu1 : mu0, ad = d ? hin[1] : hin[0];
        const float inv_var = fexp(-2.0f * ls);
        const float dv = ad - mu;
        tb[GA + d * LDP + hs] = glogp * dv * inv_var;
        tb[GA + (2 + d) * LDP + hs] = glogp * (dv * dv * inv_var - 1.0f);
        if (d == 0 && hvalid) {
          la += -fminf(l1, l2);
          lb += (fabsf(r - 1.0f) > A.clip) ? 1.0f : 0.0f;
          lc += (r - 1.0f) - lr;
          ln += 1.0f;
        }
      }
    } else {  // critic head: V of sample hs, an 8-term eighth per lane
      const int q = lane >> 3;
      float v = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; j++) {  // k order rotated by 2q: the eight groups' H2 reads hit distinct banks
        const int k = 8 * q + ((j + 2 * q) & 7);
        v = fmaf(wb[HW + k], tb[H2 + k * LDP + hs], v);
      }
      v += dpp_f<0x128>(v);         // + lane ^ 8 (row_ror 8)
      v = sum_xor32(sum_xor16(v));  // + ^16, + ^32
      v += wb[HB];
      if (q == 0) {
        const float R = hin[0];
        tb[GA + hs] = hvalid ? A.vf_coef * 2.0f * (v - R) * invB : 0.0f;
        if (hvalid) la += (R - v) * (R - v);
      }
    }
    __syncthreads();
    PSTAMP(4);
    {  // D2 = dL/dH2 (1 - H2^2): thread (unit tid >> 2, samples 8 (tid & 3) ...)
      const int u = htid >> 2, c0 = 8 * (htid & 3);
      const float ha = wb[HW + u], hb = net ? 0.0f : wb[HW + H + u];
#pragma unroll
      for (int c = c0; c < c0 + 8; c += 4) {
        const float4 h2 = *reinterpret_cast<const float4*>(tb + H2 + u * LDP + c);
        const float4 g0 = *reinterpret_cast<const float4*>(tb + GA + c);
        float4 dh;
        if (net == 0) {
          const float4 g1v = *reinterpret_cast<const float4*>(tb + GA + LDP + c);
          dh = make_float4(g0.x * ha + g1v.x * hb, g0.y * ha + g1v.y * hb, g0.z * ha + g1v.z * hb, g0.w * ha + g1v.w * hb);
        } else {
          dh = make_float4(g0.x * ha, g0.y * ha, g0.z * ha, g0.w * ha);
        }
        *reinterpret_cast<float4*>(tb + D2 + u * LDP + c) =
            make_float4(dh.x * (1.0f - h2.x * h2.x), dh.y * (1.0f - h2.y * h2.y), dh.z * (1.0f - h2.z * h2.z),
                        dh.w * (1.0f - h2.w * h2.w));
      }
    }
    __syncthreads();
    PSTAMP(5);
    f4v d1a = {0.f, 0.f, 0.f, 0.f}, d1b = {0.f, 0.f, 0.f, 0.f};
    {  // W2^T D2 for the wave's layer-1 units, and gW2 [64 x 64] += D2 H1^T (rows = the wave's units)
      {  // pipelined as the forward layers
        constexpr int KB = 4, NBK = H / 4 / KB;
        float wt[2][KB], da[2][KB], db[2][KB];
        auto ldb = [&](int b, int buf) __attribute__((always_inline)) {
#pragma unroll
          for (int s = 0; s < KB; s++) {
            const int k = 4 * (b * KB + s) + lk;  // layer-2 unit
            wt[buf][s] = wb[w2(k, ub + li)];
            da[buf][s] = tb[D2 + k * LDP + li];
            db[buf][s] = tb[D2 + k * LDP + 16 + li];
          }
        };
        ldb(0, 0);
#pragma unroll
        for (int b = 0; b < NBK; b++) {
          if (b + 1 < NBK) ldb(b + 1, (b + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 0; s < KB; s++) {
            d1a = mfma4(wt[b & 1][s], da[b & 1][s], d1a);
            d1b = mfma4(wt[b & 1][s], db[b & 1][s], d1b);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // scheduling regions: bounded register pressure
#pragma unroll
      for (int q0 = 0; q0 < T; q0 += 4) {
        const int q = q0 + lk;  // sample
        const float a = tb[D2 + (ub + li) * LDP + q];
#pragma unroll
        for (int j = 0; j < 4; j++) gw2[j] = mfma4(a, tb[H1 + (16 * j + li) * LDP + q], gw2[j]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // vector items read before D1 replaces H1 (vec_item_g1): b2 and the heads
#pragma unroll
    for (int bb = 0; bb < 2; bb++) {
      const int i = htid + bb * GRAD_THREADS;
      if (i >= 64 && i < (net ? G1_NVC : G1_NVA)) accv[bb] += vec_item_g1(tb, net, i);
    }
    __syncthreads();  // every read of H1 (gW2) and H2 is done: D1 may replace H1
    PSTAMP(6);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int u = ub + 4 * lk + r;
      const float h1a = tb[H1 + u * LDP + li], h1b = tb[H1 + u * LDP + 16 + li];
      tb[H1 + u * LDP + li] = d1a[r] * (1.0f - h1a * h1a);
      tb[H1 + u * LDP + 16 + li] = d1b[r] * (1.0f - h1b * h1b);
    }
    __syncthreads();
    PSTAMP(7);
    // gW1 [64 x 80] += D1 X^T (rows = the wave's units); b1 = the row sums of D1
#pragma unroll
    for (int q0 = 0; q0 < T; q0 += 4) {
      const int q = q0 + lk;
      const float a = tb[H1 + (ub + li) * LDP + q];
#pragma unroll
      for (int j = 0; j < 5; j++) gw1[j] = mfma4(a, tb[X + (16 * j + li) * LDP + q], gw1[j]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (htid < H) accv[0] += vec_item_g1(tb, net, htid);
  }
  PSTAMP(8);
  // this workgroup's net's share of partial row grp0: its weight gradients and vector items
  const int row = grp0;
  float* g = A.gpart + (size_t)row * P;
  const int ow1 = net ? ACKPPO_OFF_VF_W1 : ACKPPO_OFF_PI_W1, ow2 = net ? ACKPPO_OFF_VF_W2 : ACKPPO_OFF_PI_W2;
  bool st_w1 = true, st_w2 = true;
  // loss sums: per wave here, then the waves in order through LDS (with NT == 2, behind the
  // hand-over's two barriers: a barrier after the partial-row stores waited for those stores)
  la = wave_sum(la);
  lb = wave_sum(lb);
  lc = wave_sum(lc);
  ln = wave_sum(ln);
  if constexpr (NT == 2) {
    // the halves' sums combined through LDS, tile 2 g's first: half 1 hands over gW1 and the vector
    // items (into its tile region) and stores the combined gW2; half 0 hands over gW2 and stores
    // the combined gW1 and vector items
    __syncthreads();  // every tile read is done
    PSTAMP(9);
    float* xo = tl + TBASE + half * TSZ;  // this half's hand-over region, [component][256]
    const float* xi = tl + TBASE + (1 - half) * TSZ;
    if (lane == 0) {
      float* ls = xo + LS_SLOT + 4 * wave;
      ls[0] = la;
      ls[1] = lb;
      ls[2] = lc;
      ls[3] = ln;
    }
    if (half == 1) {
#pragma unroll
      for (int j = 0; j < 5; j++)
#pragma unroll
        for (int r = 0; r < 4; r++) xo[(4 * j + r) * GRAD_THREADS + htid] = gw1[j][r];
      xo[20 * GRAD_THREADS + htid] = accv[0];
      xo[21 * GRAD_THREADS + htid] = accv[1];
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int r = 0; r < 4; r++) xo[(4 * j + r) * GRAD_THREADS + htid] = gw2[j][r];
    }
    __syncthreads();
    PSTAMP(10);
    if (half == 0) {
#pragma unroll
      for (int j = 0; j < 5; j++)
#pragma unroll
        for (int r = 0; r < 4; r++) gw1[j][r] = gw1[j][r] + xi[(4 * j + r) * GRAD_THREADS + htid];
      accv[0] = accv[0] + xi[20 * GRAD_THREADS + htid];
      accv[1] = accv[1] + xi[21 * GRAD_THREADS + htid];
      st_w2 = false;
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int r = 0; r < 4; r++) gw2[j][r] = xi[(4 * j + r) * GRAD_THREADS + htid] + gw2[j][r];
      st_w1 = false;
    }
  }
  if constexpr (NT == 2) {
    if (tid < 4) {
      const float* ls = tl + TBASE + LS_SLOT;
      const float s = ((ls[tid] + ls[4 + tid]) + (ls[8 + tid] + ls[12 + tid])) +
                      ((ls[TSZ + tid] + ls[TSZ + 4 + tid]) + (ls[TSZ + 8 + tid] + ls[TSZ + 12 + tid]));
      loss_row(A, row, net, s);
    }
  }
  if (st_w1) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int u = ub + 4 * lk + r;
#pragma unroll
      for (int j = 0; j < 5; j++)
        if (16 * j + li < NOBS) g[ow1 + u * NOBS + 16 * j + li] = gw1[j][r];
    }
#pragma unroll
    for (int bb = 0; bb < 2; bb++) {
      const int i = htid + bb * GRAD_THREADS;
      if (i < (net ? G1_NVC : G1_NVA)) g[vec_offset_g1(net, i)] = accv[bb];
    }
  }
  if (st_w2) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int u = ub + 4 * lk + r;
#pragma unroll
      for (int j = 0; j < 4; j++) g[ow2 + u * H + 16 * j + li] = gw2[j][r];
    }
  }
  PSTAMP(11);
  if constexpr (NT == 1) {
    __syncthreads();  // the tile is done
    if (lane == 0) {
      tl[X + 4 * wave8 + 0] = la;
      tl[X + 4 * wave8 + 1] = lb;
      tl[X + 4 * wave8 + 2] = lc;
      tl[X + 4 * wave8 + 3] = ln;
    }
    __syncthreads();
    PSTAMP(12);
    if (tid < 4) loss_row(A, row, net, (tl[X + tid] + tl[X + 4 + tid]) + (tl[X + 8 + tid] + tl[X + 12 + tid]));
  }
  PSTAMP(15);
  PRSTAMP(14);
}
extern "C" __global__ void __launch_bounds__(GRAD_THREADS * g1::NT, 2 / g1::NT) ackppo_grad1_kernel(GradArgs A) {
  grad1<false>(A);
}
extern "C" __global__ void __launch_bounds__(GRAD_THREADS * g1::NT, 2 / g1::NT) ackppo_grad1i_kernel(GradArgs A) {
  grad1<true>(A);
}

// ---- ackppo_act: MFMA policy tile. 16 envs per 256-lane workgroup (4096 envs = 256 workgroups,
// one per CU): the weights are staged as in ackppo_grad (transposed / swizzled), X [80][16],
// H1 / H2 [128 units][16 envs] in LDS; wave w computes unit tiles 2w, 2w + 1 of both layers as
// 16x16 f32 MFMA tiles (k-ordered fmaf chains, like the grad kernel's forward pass); wave 0 then
// evaluates the heads (lanes (env, output): mu0, mu1, value) and samples the actions.
constexpr int AE = 16;  // envs per workgroup
constexpr int A_X = W_TOTAL, A_H1 = A_X + 80 * AE, A_H2 = A_H1 + 2 * H * AE, A_TOTAL = A_H2 + 2 * H * AE;
constexpr size_t ACT_LDS = (size_t)A_TOTAL * sizeof(float);

// layers 1-2 of both nets and the three heads for the 16 envs of X (already in LDS): returns, in
// wave 0, lane (env li, output lk) = mu0 / mu1 / value
__device__ __forceinline__ float act_forward(float* tl, const float* w, int wave, int lane) {
  const int li = lane & 15, lk = lane >> 4;
  const int nid = wave >> 1, ub0 = 32 * (wave & 1);
  {  // layer 1: [128 x 16] = W1T^T [128 x 80] . X [80 x 16]
    f4v acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll  // k0 compile-time: the W1T swizzle folds to an immediate XOR per read
    for (int k0 = 0; k0 < 80; k0 += 4) {
      const int k = k0 + lk;
      const float b = tl[A_X + k * AE + li];
      acc0 = mfma4(w[w1t_at(k, nid * H + ub0 + li)], b, acc0);
      acc1 = mfma4(w[w1t_at(k, nid * H + ub0 + 16 + li)], b, acc1);
    }
    const float* bias = w + (nid ? W_B1_C : W_B1_A);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int u = ub0 + 4 * lk + r;
      tl[A_H1 + (nid * H + u) * AE + li] = ftanh(acc0[r] + bias[u]);
      tl[A_H1 + (nid * H + u + 16) * AE + li] = ftanh(acc1[r] + bias[u + 16]);
    }
  }
  __syncthreads();
  {  // layer 2 per net: [64 x 16] = W2 [64 x 64] . H1 [64 x 16]
    const float* W2 = w + (nid ? W_W2_C : W_W2_A);
    const float* h1 = tl + A_H1 + nid * H * AE;
    f4v acc0 = {0.0f, 0.0f, 0.0f, 0.0f}, acc1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int k0 = 0; k0 < H; k0 += 4) {
      const int k = k0 + lk;
      const float b = h1[k * AE + li];
      acc0 = mfma4(W2[w2_at(ub0 + li, k)], b, acc0);
      acc1 = mfma4(W2[w2_at(ub0 + 16 + li, k)], b, acc1);
    }
    const float* bias = w + (nid ? W_B2_C : W_B2_A);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int u = ub0 + 4 * lk + r;
      tl[A_H2 + (nid * H + u) * AE + li] = ftanh(acc0[r] + bias[u]);
      tl[A_H2 + (nid * H + u + 16) * AE + li] = ftanh(acc1[r] + bias[u + 16]);
    }
  }
  __syncthreads();
  // heads: lane (env li, output lk): 0 mu0, 1 mu1 (actor H2 rows 0-63), 2 value (critic rows 64-127)
  float v = 0.0f;
  if (wave == 0) {
    const int wo = lk == 0 ? W_AW : (lk == 1 ? W_AW + H : W_CW);
    const float* h2 = tl + A_H2 + (lk == 2 ? H * AE : 0);
#pragma unroll 8
    for (int j = 0; j < H; j++) v = fmaf(w[wo + j], h2[j * AE + li], v);
    v += lk == 0 ? w[W_AB] : (lk == 1 ? w[W_AB + 1] : w[W_CB]);
  }
  return v;
}
__device__ __forceinline__ void act_load_x(float* tl, const float* soa, int n, int e0, int nv, int tid) {
  // X [k][env] from an SoA observation (row 79 and padding envs zero)
  const int e = tid & 15;
#pragma unroll
  for (int k = tid >> 4; k < 80; k += 16) tl[A_X + k * AE + e] = (k < NOBS && e < nv) ? soa[(size_t)k * n + e0 + e] : 0.0f;
}

extern "C" __global__ void __launch_bounds__(GRAD_THREADS) ackppo_act_kernel(ActArgs A) {
  extern __shared__ float tl[];
  float* w = tl;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lk = lane >> 4;
  const int e0 = blockIdx.x * AE, nv = min(AE, A.n - e0);
  stage_grad_weights(A.params, w);
  if (A.tobs) {
    // the previous step's TimeLimit bootstrap (ackppo_bootstrap's semantics): the critic on the
    // terminal observations, only in workgroups holding a truncated-not-terminated env (rare)
    const int eb = e0 + (tid & 15);
    const bool mine = tid < AE && (tid & 15) < nv;
    const bool te = mine && A.term[eb] != 0, tr = mine && A.trunc[eb] != 0;
    const bool boot = tr && !te;
    float vb = 0.0f;
    if (__syncthreads_or(boot)) {
      act_load_x(tl, A.tobs, A.n, e0, nv, tid);
      __syncthreads();
      const float v = act_forward(tl, w, wave, lane);
      vb = __shfl(v, (tid & 15) + 32, 64);  // wave 0: value of env tid & 15
      __syncthreads();                      // X is reloaded below
    }
    if (mine) {
      float r = A.reward[eb];
      if (boot) r = fmaf(A.gamma, vb, r);
      A.reward_out[eb] = r;
      A.done_out[eb] = (te || tr) ? 1.0f : 0.0f;
    }
  }
  if (!A.obs) return;  // ackppo_bootstrap: the bootstrap alone (the same critic path as ackppo_act_boot)
  act_load_x(tl, A.obs, A.n, e0, nv, tid);
  __syncthreads();
  if (A.obs_rows) {  // rollout-buffer rows [env][79]: one contiguous block of nv * 79 words
    for (int i = tid; i < nv * NOBS; i += GRAD_THREADS) {
      const int e = i / NOBS, k = i - e * NOBS;
      A.obs_rows[(size_t)e0 * NOBS + i] = tl[A_X + k * AE + e];
    }
  }
  const float v = act_forward(tl, w, wave, lane);
  if (wave != 0) return;
  const float mu1 = __shfl(v, li + 16, 64), val = __shfl(v, li + 32, 64);
  if (lk != 0 || li >= nv) return;
  const int e = e0 + li;
  if (!A.env_action) {  // ackppo_value: the critic alone (the same path as the rollout's values)
    A.value[e] = val;
    return;
  }
  const float mu[NA] = {v, mu1};
  float a[NA];
  const float lp = ppm::sample_action(mu, w[W_LS], w[W_LS + 1], A.deterministic != 0, A.env_offset + e, A.step, A.seed,
                                      a);
  if (A.action) {
    A.action[2 * (size_t)e] = a[0];
    A.action[2 * (size_t)e + 1] = a[1];
  }
  A.env_action[2 * (size_t)e] = fminf(fmaxf(a[0], -1.0f), 1.0f);
  A.env_action[2 * (size_t)e + 1] = fminf(fmaxf(a[1], -1.0f), 1.0f);
  if (A.log_prob) A.log_prob[e] = lp;
  if (A.value) A.value[e] = val;
}

// ---- ackppo_permutation: out[i] = pi(i), a keyed pseudo-random bijection of [0, n) -- a
// 4-round balanced Feistel network on 2*half >= bits(n - 1) bits (round function: a
// multiply-xorshift hash of the right half and the round key), cycle-walked until the value
// falls in [0, n) (bijective on [0, n) because the network is bijective on [0, 2^(2 half));
// 2^(2 half) < 4n, so a walk takes < 4 network passes on average). One thread per index.
__device__ __forceinline__ uint32_t perm_hash(uint32_t x, uint32_t k) {
  x = (x ^ k) * 0x9E3779B1u;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  return x ^ (x >> 16);
}
__device__ __forceinline__ uint32_t perm_at(uint32_t i, int n, int half, const uint32_t keys[4]) {
  const uint32_t mask = (1u << half) - 1u;
  uint32_t x = i;
  do {
    uint32_t L = x >> half, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t t = L ^ (perm_hash(R, keys[r]) & mask);
      L = R;
      R = t;
    }
    x = (L << half) | R;
  } while (x >= (uint32_t)n);
  return x;
}
// the round keys of (seed, epoch): splitmix64 of seed ^ golden * (epoch + 1)
__host__ __device__ inline void perm_keys(uint64_t seed, uint32_t epoch, uint32_t k[4]) {
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * ((uint64_t)epoch + 1));
  for (int r = 0; r < 4; r++) {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t y = z;
    y = (y ^ (y >> 30)) * 0xBF58476D1CE4E5B9ull;
    y = (y ^ (y >> 27)) * 0x94D049BB133111EBull;
    k[r] = (uint32_t)(y ^ (y >> 31));
  }
}
__host__ __device__ inline int perm_half(int n) {
  int bits = 1;
  while ((1u << bits) < (uint32_t)n) bits++;
  return (bits + 1) / 2;
}
extern "C" __global__ void __launch_bounds__(256) ackppo_perm_kernel(int n, int half, uint32_t k0, uint32_t k1,
                                                                     uint32_t k2, uint32_t k3, int32_t* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t keys[4] = {k0, k1, k2, k3};
  out[i] = (int32_t)perm_at((uint32_t)i, n, half, keys);
}

// Every epoch's shuffle and minibatch advantage statistics of one ackppo_train call in ONE launch
// (the advantages do not change during the call): workgroup (m, e) computes positions
// [m B, (m + 1) B) of epoch e's permutation (the Feistel map above, keys of epoch epoch0 + e),
// writes them to perm[e][.], gathers the advantages and forms minibatch m's statistics with
// ackppo_adv_stats_kernel's arithmetic (the same bits). Replaces 2 launches per epoch.
extern "C" __global__ void __launch_bounds__(ADV_THREADS) ackppo_perm_stats_kernel(const float* adv, int n, int batch,
                                                                                   uint64_t seed, uint32_t epoch0,
                                                                                   int normalize, int32_t* perm,
                                                                                   float* stats) {
  __shared__ double red[ADV_THREADS / 64];
  const int m = blockIdx.x, e = blockIdx.y, tid = threadIdx.x, nmb = gridDim.x;
  uint32_t keys[4];
  perm_keys(seed, epoch0 + (uint32_t)e, keys);
  const int half = perm_half(n);
  int32_t* out = perm + (size_t)e * n;
  float* st = stats + 2 * ((size_t)e * nmb + m);
  const int lo = m * batch, hi = min(lo + batch, n), cnt = hi - lo;
  float v[ADV_CACHE];
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < ADV_CACHE; c++) {
    const int i = lo + tid + c * ADV_THREADS;
    v[c] = 0.0f;
    if (i < hi) {
      const uint32_t x = perm_at((uint32_t)i, n, half, keys);
      out[i] = (int32_t)x;
      v[c] = adv[x];
    }
    s += v[c];
  }
  for (int i = lo + tid + ADV_CACHE * ADV_THREADS; i < hi; i += ADV_THREADS) {
    const uint32_t x = perm_at((uint32_t)i, n, half, keys);
    out[i] = (int32_t)x;
    s += adv[x];
  }
  if (!normalize || cnt <= 1) {
    if (tid == 0) { st[0] = 0.0f; st[1] = 1.0f; }
    return;
  }
  const double mean = block_sum_d(s, red) / cnt;
  double q = 0.0;
#pragma unroll
  for (int c = 0; c < ADV_CACHE; c++) {
    const double d = (double)v[c] - mean;
    q += (lo + tid + c * ADV_THREADS < hi) ? d * d : 0.0;
  }
  for (int i = lo + tid + ADV_CACHE * ADV_THREADS; i < hi; i += ADV_THREADS) {
    const double d = adv[out[i]] - mean;  // this thread's own write above
    q += d * d;
  }
  const double var = block_sum_d(q, red) / (cnt - 1);
  if (tid == 0) {
    const float sd = (float)sqrt(var);
    st[0] = (float)mean;
    st[1] = 1.0f / (sd + 1e-8f);
  }
}

// The data-parallel form of ackppo_perm_stats_kernel: workgroup (m, e) writes positions
// [m B, (m + 1) B) of epoch e's shuffle and this rank's (count, sum) of minibatch m's advantages
// into moments[0..1][e][m] (ackppo_adv_moments_kernel phase 0's arithmetic, the same bits); one
// all-reduce then covers every epoch's first moments.
extern "C" __global__ void __launch_bounds__(ADV_THREADS) ackppo_perm_moments_kernel(const float* adv, int n, int batch,
                                                                                     uint64_t seed, uint32_t epoch0,
                                                                                     int32_t* perm, double* moments) {
  __shared__ double red[ADV_THREADS / 64];
  const int m = blockIdx.x, e = blockIdx.y, tid = threadIdx.x, nmb = gridDim.x, NM = nmb * gridDim.y;
  const int j = e * nmb + m;
  uint32_t keys[4];
  perm_keys(seed, epoch0 + (uint32_t)e, keys);
  const int half = perm_half(n);
  int32_t* out = perm + (size_t)e * n;
  const int lo = m * batch, hi = min(lo + batch, n), cnt = hi - lo;
  double s = 0.0;
  for (int i = lo + tid; i < hi; i += ADV_THREADS) {
    const uint32_t x = perm_at((uint32_t)i, n, half, keys);
    out[i] = (int32_t)x;
    s += adv[x];
  }
  const double tot = block_sum_d(s, red);
  if (tid == 0) {
    moments[j] = (double)cnt;
    moments[NM + j] = tot;
    moments[2 * NM + j] = 0.0;
  }
}

// The reduction of the partial rows (the C-ABI ackppo_reduce): no atomics, no scratch. A
// 1024-thread block owns 64 consecutive parameters; its 16 waves each sum every 16th partial row of
// them (every row load in flight at once), the 16 sums are combined through LDS; block 0 also
// reduces the loss rows. (It replaced a two-launch form, row groups in place then the group sums;
// 2- and 4-parameter vector loads per lane measured slower, round 4.) The caller-owned partial rows
// are the only buffer, so concurrent learners on other streams or devices share nothing.
constexpr int R1_P = 64, R1_G = 16;  // parameters per block, row groups
extern "C" __global__ void __launch_bounds__(1024) ackppo_reduce1_kernel(const float* gpart, int nblk,
                                                                        const float* lpart, float ent_coef,
                                                                        float* grad, float* loss, int accumulate) {
  // a block owns R1_P consecutive parameters: lane pl of wave g loads its one from every 16th row
  __shared__ float red[R1_G][R1_P + 1];
  __shared__ float lred[256];
  const int tid = threadIdx.x, pl = tid & (R1_P - 1), g = tid / R1_P;
  const int vidx = blockIdx.x * R1_P + pl;  // parameter index
  const bool vok = vidx < P;
  // all R1_K of this thread's rows in flight at once (one memory latency, not four), then summed in
  // blocks of 4 rows into acc[0..3] while a whole block of 4 remains, the tail rows into acc[0]
  constexpr int R1_K = GRAD_MAX_BLOCKS / R1_G;
  static_assert(R1_K % 4 == 0, "row blocks of four");
  float x[R1_K];
#pragma unroll
  for (int k = 0; k < R1_K; k++) {
    const int b = g + k * R1_G;
    x[k] = (vok && b < nblk) ? gpart[(size_t)b * P + vidx] : 0.0f;
  }
  int nmain = 0;  // blocks j with g + 4 R1_G j + 3 R1_G < nblk (a prefix)
#pragma unroll
  for (int j = 0; j < R1_K / 4; j++) nmain += (g + 4 * R1_G * j + 3 * R1_G < nblk) ? 1 : 0;
  {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < R1_K / 4; j++)
      if (j < nmain) {
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] += x[4 * j + i];
      }
#pragma unroll
    for (int k = 0; k < R1_K; k++)
      if (k >= 4 * nmain) acc[0] += x[k];  // rows past nblk are 0.0f: adding them changes nothing
    red[g][pl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();
  const int pidx = blockIdx.x * R1_P + tid;
  if (tid < R1_P && pidx < P) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < R1_G; k++) s += red[k][tid];
    if (pidx == ACKPPO_OFF_LOG_STD || pidx == ACKPPO_OFF_LOG_STD + 1) s -= ent_coef;
    grad[pidx] = s;
  }
  if (blockIdx.x == 0) {  // loss rows (32 block-strided groups x 8 slots, then an LDS tree), on the block's first 256 threads
    static_assert(ACKPPO_NLOSS == 8, "loss row layout");
    const int slot = tid & 7, grp = tid >> 3;
    float s = 0.0f;
    if (tid < 256)
      for (int b = grp; b < nblk; b += 32) s += lpart[(size_t)b * ACKPPO_NLOSS + slot];
    if (tid < 256) lred[tid] = s;
    __syncthreads();
    for (int o = 128; o >= 8; o >>= 1) {
      if (tid < o) lred[tid] += lred[tid + o];
      __syncthreads();
    }
    if (tid < ACKPPO_NLOSS) loss[tid] = (accumulate ? loss[tid] : 0.0f) + lred[tid];
  }
}

// clip_grad_norm_ + Adam over the whole vector (the C-ABI ackppo_adam): 256-thread workgroups, each
// forming the global norm itself (grad_norm256) and updating 256 float4 of parameters in place
extern "C" __global__ void __launch_bounds__(256) ackppo_adam_kernel(float* params, const float* grad, float* m,
                                                                     float* v, float scale, float max_norm, float b1,
                                                                     float b2, float eps, float step_size,
                                                                     float bc2_sqrt, float* norm_out, float lsmin) {
  __shared__ float red[4];
  // this thread's parameter and moments are loaded before the norm (their latency hides under it)
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int jc = j < P / 4 ? j : P / 4 - 1;
  const float4 pv = reinterpret_cast<const float4*>(params)[jc];
  const float4 mv = reinterpret_cast<const float4*>(m)[jc], vv = reinterpret_cast<const float4*>(v)[jc];
  const float norm = grad_norm256(grad, scale, red);
  const AdamK k = adam_k(norm, scale, max_norm, b1, b2, eps, step_size, bc2_sqrt, lsmin);
  if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = norm;
  if (j >= P / 4) return;
  const float4 gv = reinterpret_cast<const float4*>(grad)[j];
  float4 pn, mn, vn;
  adam_elem(k, pv.x, gv.x, mv.x, vv.x, pn.x, mn.x, vn.x);
  adam_elem(k, pv.y, gv.y, mv.y, vv.y, pn.y, mn.y, vn.y);
  adam_elem(k, pv.z, gv.z, mv.z, vv.z, pn.z, mn.z, vn.z);
  adam_elem(k, pv.w, gv.w, mv.w, vv.w, pn.w, mn.w, vn.w);
  static_assert(ACKPPO_OFF_LOG_STD == 0, "log_std in the first float4");
  if (j == 0) {
    pn.x = ls_floor(k, pn.x);
    pn.y = ls_floor(k, pn.y);
  }
  reinterpret_cast<float4*>(params)[j] = pn;
  reinterpret_cast<float4*>(m)[j] = mn;
  reinterpret_cast<float4*>(v)[j] = vn;
}

// ---- the update kernels of ackppo_train / ackppo_epoch: the reduction also forms each norm
// block's S_b (norm_block_sq), so the Adam launch after it reads 147 words for the global norm
// instead of re-reading the whole gradient. Workgroup b owns norm block b: parameters 128 b ..
// 128 b + 127 (147 workgroups for 18 764 parameters); S_b goes to row 0, column 128 b of the
// partial rows, which only workgroup b reads (and the next gradient launch rewrites).
struct UpdArgs {
  float* gpart;  // partial rows [nblk][P] (ackppo_grad); row 0 column 128 b: S_b after the reduction
  int nblk;
  const float* lpart;
  float ent_coef;
  float* grad;
  float* loss;
  int accumulate;
  int sq;  // ackppo_reduce_norm_kernel: write S_b (0: the data-parallel path forms them after its all-reduce)
  float* params;
  float* m;
  float* v;
  float scale, max_norm, b1, b2, eps, step_size, bc2_sqrt, lsmin;
  float* norm_out;
  float* wimg;  // optional weight image kept in step (ackppo_train_desc::weight_image)
};
// Adam on norm block b's parameters once every S_b is visible: threads 0-127 own parameter 128 b + t
// (gv its gradient, pv / mv / vv loaded earlier), threads 0-255 form the norm
__device__ __forceinline__ void adam_block_update(const UpdArgs& A, int b, float gv, float pv, float mv, float vv,
                                                  float* nred) {
  const int t = threadIdx.x, p = b * NB_P + t;
  const float norm = norm_from_blocks(A.gpart, NB_P, nred);
  const AdamK k = adam_k(norm, A.scale, A.max_norm, A.b1, A.b2, A.eps, A.step_size, A.bc2_sqrt, A.lsmin);
  if (b == 0 && t == 0 && A.norm_out) A.norm_out[0] = norm;
  if (t >= NB_P || p >= P) return;
  float pn, mn, vn;
  adam_elem(k, pv, gv, mv, vv, pn, mn, vn);
  static_assert(ACKPPO_OFF_LOG_STD == 0, "log_std first");
  if (p < 2) pn = ls_floor(k, pn);
  A.params[p] = pn;
  A.m[p] = mn;
  A.v[p] = vn;
  if (A.wimg) {  // the new parameter into the weight image as well (ackppo_grad1i stages from it)
    const int ix = g1::wimg_index(p);
    if (ix >= 0) A.wimg[ix] = pn;
  }
}
// the partial rows reduced (8 row groups x 128 parameters; rows g, g + 8, ... in blocks of four as
// ackppo_reduce1_kernel) into grad, the loss rows on workgroup 0, and S_b
constexpr int RA_G = 8;
constexpr int RA_THREADS = RA_G * NB_P;
// RKV: the row slots a thread loads (RK = GRAD_MAX_BLOCKS / RA_G in general; RK / 2 when nblk <= 128, the
// bench's 8192-sample minibatch). Every load is issued unconditionally from a clamped row and column
// and masked after (guarded loads were one exec-mask branch each); with RKV < RK the slots past RKV
// are the zeros the RK form adds to acc[0], so one + 0.0f stands for them (a -0.0 sum becomes +0.0
// there too): the same bits either way.
template <int RKV>
__device__ __forceinline__ float reduce_rows(const UpdArgs& A, float (*red)[NB_P + 1], float* lred) {
  const int tid = threadIdx.x, b = blockIdx.x;
  const int pidx = b * NB_P + tid;  // threads 0-127: the parameter this thread finishes
  const bool own = tid < NB_P && pidx < P;
  constexpr int RK = GRAD_MAX_BLOCKS / RA_G;
  static_assert(RK % 4 == 0 && RKV % 4 == 0 && RKV <= RK, "row blocks of four");
  static_assert(P % 4 == 0 && NB_P % 4 == 0, "whole 16-B vectors per row and block");
  {
    const int pl = tid & (NB_P - 1), g = __builtin_amdgcn_readfirstlane(tid / NB_P);  // g: wave-uniform
    const int pcol = b * NB_P + pl;
    const float* col = A.gpart + min(pcol, P - 1);
    float x[RKV];
#pragma unroll
    for (int k = 0; k < RKV; k++) x[k] = col[(size_t)min(g + k * RA_G, A.nblk - 1) * P];
#pragma unroll
    for (int k = 0; k < RKV; k++) x[k] = (pcol < P && g + k * RA_G < A.nblk) ? x[k] : 0.0f;
    int nmain = 0;
#pragma unroll
    for (int j = 0; j < RK / 4; j++) nmain += (g + 4 * RA_G * j + 3 * RA_G < A.nblk) ? 1 : 0;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < RKV / 4; j++)
      if (j < nmain) {
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] += x[4 * j + i];
      }
#pragma unroll
    for (int k = 0; k < RKV; k++)
      if (k >= 4 * nmain) acc[0] += x[k];
    if constexpr (RKV < RK) acc[0] += 0.0f;
    red[g][pl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();
  float gv = 0.0f;
  if (own) {
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < RA_G; k++) s += red[k][tid];
    if (pidx == ACKPPO_OFF_LOG_STD || pidx == ACKPPO_OFF_LOG_STD + 1) s -= A.ent_coef;
    A.grad[pidx] = s;
    gv = s;
  }
  if (b == 0) {  // loss rows: as ackppo_reduce1_kernel
    const int slot = tid & 7, grp = tid >> 3;
    float s = 0.0f;
    if (tid < 256)
      for (int r = grp; r < A.nblk; r += 32) s += A.lpart[(size_t)r * ACKPPO_NLOSS + slot];
    if (tid < 256) lred[tid] = s;
    __syncthreads();
    for (int o = 128; o >= 8; o >>= 1) {
      if (tid < o) lred[tid] += lred[tid + o];
      __syncthreads();
    }
    if (tid < ACKPPO_NLOSS) A.loss[tid] = (A.accumulate ? A.loss[tid] : 0.0f) + lred[tid];
  }
  return gv;
}
template <int RKV>
__device__ __forceinline__ void reduce_norm(const UpdArgs& A) {
  __shared__ float red[RA_G][NB_P + 1];
  __shared__ float lred[256];
  __shared__ float nred[2];
  const int tid = threadIdx.x, b = blockIdx.x;
  const float gv = reduce_rows<RKV>(A, red, lred);
  if (!A.sq) return;
  const float sb = norm_block_sq(gv, A.scale, b, nred);  // every row read above is done (barriers)
  if (tid == 0) A.gpart[(size_t)b * NB_P] = sb;
}
extern "C" __global__ void __launch_bounds__(RA_THREADS) ackppo_reduce_norm_kernel(UpdArgs A) {
  reduce_norm<GRAD_MAX_BLOCKS / RA_G>(A);
}
extern "C" __global__ void __launch_bounds__(RA_THREADS) ackppo_reduce_norm128_kernel(UpdArgs A) {  // nblk <= 128
  reduce_norm<GRAD_MAX_BLOCKS / RA_G / 2>(A);
}
// the reduction launch for U.nblk partial rows
void reduce_norm_launch(const UpdArgs& U, hipStream_t st) {
  if (U.nblk <= GRAD_MAX_BLOCKS / 2)
    hipLaunchKernelGGL(ackppo_reduce_norm128_kernel, dim3(NB_N), dim3(RA_THREADS), 0, st, U);
  else
    hipLaunchKernelGGL(ackppo_reduce_norm_kernel, dim3(NB_N), dim3(RA_THREADS), 0, st, U);
}
// S_b of the gradient as it is now (the data-parallel path: after its all-reduce)
extern "C" __global__ void __launch_bounds__(NB_P) ackppo_norm_blocks_kernel(UpdArgs A) {
  __shared__ float nred[2];
  const int t = threadIdx.x, b = blockIdx.x, p = b * NB_P + t;
  const float sb = norm_block_sq(p < P ? A.grad[p] : 0.0f, A.scale, b, nred);
  if (t == 0) A.gpart[(size_t)b * NB_P] = sb;
}
// clip_grad_norm_ + Adam with the blocked norm: workgroup b updates norm block b's parameters
extern "C" __global__ void __launch_bounds__(256) ackppo_adam_blocked_kernel(UpdArgs A) {
  __shared__ float nred[4];
  const int t = threadIdx.x, b = blockIdx.x, p = b * NB_P + t;
  const bool own = t < NB_P && p < P;
  float gv = 0.0f, pv = 0.0f, mv = 0.0f, vv = 0.0f;
  if (own) {  // issued before the norm: their latency hides under it
    gv = A.grad[p];
    pv = A.params[p];
    mv = A.m[p];
    vv = A.v[p];
  }
  adam_block_update(A, b, gv, pv, mv, vv, nred);
}

// ------------------------------------------------------------------ C-ABI

namespace {
thread_local char g_err[256] = "";
int fail(int code, const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return code;
}
int launched(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return ACKPPO_EHIP;
  }
  return ACKPPO_OK;
}
#ifndef AK_GRAD1_LDS_PAD  // diagnostic builds: extra LDS per workgroup (e.g. one workgroup per CU)
#define AK_GRAD1_LDS_PAD 0
#endif
constexpr size_t GRAD_LDS = (size_t)g1::TOTAL * sizeof(float) + AK_GRAD1_LDS_PAD;
// hipFuncSetAttribute is applied per device: flags indexed by the caller's current device
constexpr int MAX_DEV = 64;
bool g_grad_attr[MAX_DEV] = {};
bool g_policy_attr[MAX_DEV] = {};
int current_device() {
  int d = 0;
  return (hipGetDevice(&d) == hipSuccess && d >= 0 && d < MAX_DEV) ? d : -1;
}
bool policy_lds_ready() {
  const int dev = current_device();
  if (dev < 0) return false;
  if (g_policy_attr[dev]) return true;
  if (hipFuncSetAttribute((const void*)ackppo_act_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ACT_LDS) !=
      hipSuccess)
    return false;
  g_policy_attr[dev] = true;
  return true;
}
bool g_grad1i_attr[MAX_DEV] = {};
// ackppo_grad's launch: two workgroups (actor, critic) per partial row; with A.wimg, the variant that
// stages the weight image (ackppo_train)
int grad_launch(const GradArgs& A, void* stream) {
  const int dev = current_device();
  if (dev < 0) return fail(ACKPPO_EHIP, "ackppo_grad: no usable current device");
  const bool img = A.wimg != nullptr;
  bool& ready = img ? g_grad1i_attr[dev] : g_grad_attr[dev];
  if (!ready) {
    const void* kern = img ? (const void*)ackppo_grad1i_kernel : (const void*)ackppo_grad1_kernel;
    if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRAD_LDS) != hipSuccess)
      return fail(ACKPPO_EHIP, "ackppo_grad: cannot reserve the grad kernel's LDS footprint");
    ready = true;
  }
  const int nblk = ackppo_grad_blocks(A.batch);
  hipLaunchKernelGGL(img ? ackppo_grad1i_kernel : ackppo_grad1_kernel, dim3(2 * nblk),
                       dim3(GRAD_THREADS * g1::NT),
                       GRAD_LDS, (hipStream_t)stream, A);
  return launched("ackppo_grad");
}
}  // namespace

extern "C" {

const char* ackppo_last_error(void) { return g_err; }
#ifdef PP_STAMPS
int ackppo_diag_set_stamps(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_pp_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -3;
}
#endif

int ackppo_act(const float* params, const float* obs_soa, int n_env, int64_t env_offset, uint64_t seed, uint32_t step,
               int deterministic, float* obs_rows, float* action, float* env_action, float* log_prob, float* value,
               void* stream) {
  if (!params || !obs_soa || !env_action || n_env < 0) return fail(ACKPPO_EINVAL, "ackppo_act: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  ActArgs A{params, obs_soa, n_env, env_offset, seed, step, deterministic, obs_rows, action, env_action, log_prob, value,
            nullptr, nullptr, nullptr, nullptr, 0.0f, nullptr, nullptr};
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_act: cannot reserve the policy LDS tile");
  hipLaunchKernelGGL(ackppo_act_kernel, dim3((n_env + AE - 1) / AE), dim3(GRAD_THREADS), ACT_LDS, (hipStream_t)stream,
                     A);
  return launched("ackppo_act");
}

int ackppo_act_boot(const float* params, const float* obs_soa, int n_env, int64_t env_offset, uint64_t seed,
                    uint32_t step, int deterministic, float* obs_rows, float* action, float* env_action,
                    float* log_prob, float* value, const float* terminal_obs_soa, const float* reward,
                    const uint8_t* term, const uint8_t* trunc, float gamma, float* reward_out, float* done_out,
                    void* stream) {
  if (!params || !obs_soa || !env_action || n_env < 0 || !terminal_obs_soa || !reward || !term || !trunc ||
      !reward_out || !done_out)
    return fail(ACKPPO_EINVAL, "ackppo_act_boot: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  ActArgs A{params,  obs_soa,          n_env,  env_offset, seed, step,  deterministic, obs_rows,   action, env_action,
            log_prob, value, terminal_obs_soa, reward, term,       trunc, gamma, reward_out,    done_out};
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_act_boot: cannot reserve the policy LDS tile");
  hipLaunchKernelGGL(ackppo_act_kernel, dim3((n_env + AE - 1) / AE), dim3(GRAD_THREADS), ACT_LDS, (hipStream_t)stream,
                     A);
  return launched("ackppo_act_boot");
}

int ackppo_value(const float* params, const float* obs_soa, int n_env, float* value, void* stream) {
  if (!params || !obs_soa || !value || n_env < 0) return fail(ACKPPO_EINVAL, "ackppo_value: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_value: cannot reserve the policy LDS tile");
  // the act kernel without sampling: the same critic arithmetic as the rollout's per-step values
  ActArgs A{params,  obs_soa, n_env,   0,       0,       0,       1,      nullptr, nullptr, nullptr,
            nullptr, value,   nullptr, nullptr, nullptr, nullptr, 0.0f, nullptr, nullptr};
  hipLaunchKernelGGL(ackppo_act_kernel, dim3((n_env + AE - 1) / AE), dim3(GRAD_THREADS), ACT_LDS, (hipStream_t)stream,
                     A);
  return launched("ackppo_value");
}

int ackppo_bootstrap(const float* params, const float* terminal_obs_soa, const float* reward, const uint8_t* term,
                     const uint8_t* trunc, int n_env, float gamma, float* reward_out, float* done_out, void* stream) {
  if (!params || !terminal_obs_soa || !reward || !term || !trunc || !reward_out || !done_out || n_env < 0)
    return fail(ACKPPO_EINVAL, "ackppo_bootstrap: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_bootstrap: cannot reserve the policy LDS tile");
  // the act kernel's bootstrap part alone (obs == nullptr): bit-identical to ackppo_act_boot's
  ActArgs A{params,  nullptr,          n_env,  0,    0,     0,     1,          nullptr, nullptr, nullptr,
            nullptr, nullptr, terminal_obs_soa, reward, term, trunc, gamma, reward_out, done_out};
  hipLaunchKernelGGL(ackppo_act_kernel, dim3((n_env + AE - 1) / AE), dim3(GRAD_THREADS), ACT_LDS, (hipStream_t)stream,
                     A);
  return launched("ackppo_bootstrap");
}

int ackppo_gae(const float* rewards, const float* values, const float* episode_starts, const float* last_values,
               const float* last_dones, int T, int n_env, float gamma, float gae_lambda, float* advantages,
               float* returns, void* stream) {
  if (!rewards || !values || !episode_starts || !last_values || !last_dones || !advantages || !returns || T < 0 ||
      n_env < 0)
    return fail(ACKPPO_EINVAL, "ackppo_gae: bad arguments");
  if (T == 0 || n_env == 0) return ACKPPO_OK;
  hipLaunchKernelGGL(ackppo_gae_kernel, dim3((n_env + 255) / 256), dim3(256), 0, (hipStream_t)stream, rewards, values,
                     episode_starts, last_values, last_dones, T, n_env, gamma, gae_lambda, advantages, returns);
  return launched("ackppo_gae");
}

int ackppo_permutation(int n, uint64_t seed, uint32_t epoch, int32_t* out, void* stream) {
  if (!out || n < 0 || n > (1 << 30)) return fail(ACKPPO_EINVAL, "ackppo_permutation: bad arguments");
  if (n == 0) return ACKPPO_OK;
  const int half = perm_half(n);
  uint32_t k[4];
  perm_keys(seed, epoch, k);  // round keys: splitmix64 of (seed, epoch)
  hipLaunchKernelGGL(ackppo_perm_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, half, k[0], k[1],
                     k[2], k[3], out);
  return launched("ackppo_permutation");
}

int ackppo_adv_stats(const float* advantages, const int32_t* idx, int n_idx, int batch, int normalize, float* stats,
                     void* stream) {
  if (!advantages || !idx || !stats || n_idx < 0 || batch <= 0) return fail(ACKPPO_EINVAL, "ackppo_adv_stats: bad arguments");
  const int nmb = (n_idx + batch - 1) / batch;
  if (nmb == 0) return ACKPPO_OK;
  hipLaunchKernelGGL(ackppo_adv_stats_kernel, dim3(nmb), dim3(ADV_THREADS), 0, (hipStream_t)stream, advantages, idx, n_idx,
                     batch, normalize, stats);
  return launched("ackppo_adv_stats");
}

int ackppo_adv_moments(const float* advantages, const int32_t* idx, int n_idx, int batch, int phase, double* moments,
                       void* stream) {
  if (!advantages || !idx || !moments || n_idx < 0 || batch <= 0 || (phase != 0 && phase != 1))
    return fail(ACKPPO_EINVAL, "ackppo_adv_moments: bad arguments");
  const int nmb = (n_idx + batch - 1) / batch;
  if (nmb == 0) return ACKPPO_OK;
  hipLaunchKernelGGL(ackppo_adv_moments_kernel, dim3(nmb), dim3(ADV_THREADS), 0, (hipStream_t)stream, advantages, idx,
                     n_idx, batch, phase, nmb, moments);
  return launched("ackppo_adv_moments");
}

int ackppo_adv_finalize(const double* moments, int nmb, int normalize, float* stats, void* stream) {
  if (!moments || !stats || nmb < 0) return fail(ACKPPO_EINVAL, "ackppo_adv_finalize: bad arguments");
  if (nmb == 0) return ACKPPO_OK;
  hipLaunchKernelGGL(ackppo_adv_finalize_kernel, dim3((nmb + 255) / 256), dim3(256), 0, (hipStream_t)stream, moments,
                     nmb, normalize, stats);
  return launched("ackppo_adv_finalize");
}

int ackppo_grad(const float* params, const float* obs_rows, const float* actions, const float* old_log_prob,
                const float* advantages, const float* returns, const int32_t* idx, int batch, const float* stats,
                float clip_range, float ent_coef, float vf_coef, float* grad_partial, float* loss_partial,
                void* stream) {
  if (!params || !obs_rows || !actions || !old_log_prob || !advantages || !returns || !idx || !stats ||
      !grad_partial || !loss_partial || batch <= 0)
    return fail(ACKPPO_EINVAL, "ackppo_grad: bad arguments");
  const int dev = current_device();
  if (dev < 0) return fail(ACKPPO_EHIP, "ackppo_grad: no usable current device");
  GradArgs A{params, obs_rows, actions, old_log_prob, advantages, returns, idx, batch, stats, clip_range, ent_coef,
             vf_coef, grad_partial, loss_partial};
  return grad_launch(A, stream);
}

int ackppo_grad_blocks(int batch) {
  if (batch <= 0) return 0;
  const int tiles = (batch + g1::T - 1) / g1::T;
  const int rows = (tiles + g1::NT - 1) / g1::NT;  // one partial row per tile group
  return rows < GRAD_MAX_BLOCKS ? rows : GRAD_MAX_BLOCKS;
}

namespace {
int reduce_launch(float* grad_partial, const float* loss_partial, int nblk, float ent_coef, float* grad,
                  float* loss, int accumulate, void* stream) {
  hipLaunchKernelGGL(ackppo_reduce1_kernel, dim3((P + R1_P - 1) / R1_P), dim3(R1_P * R1_G), 0, (hipStream_t)stream,
                     grad_partial, nblk, loss_partial, ent_coef, grad, loss, accumulate);
  return launched("ackppo_reduce");
}
}  // namespace

int ackppo_reduce(float* grad_partial, const float* loss_partial, int nblk, float ent_coef, float* grad,
                  float* loss, void* stream) {
  if (!grad_partial || !loss_partial || !grad || !loss || nblk <= 0 || nblk > GRAD_MAX_BLOCKS)
    return fail(ACKPPO_EINVAL, "ackppo_reduce: bad arguments (nblk: 1..ackppo_grad_blocks(batch))");
  return reduce_launch(grad_partial, loss_partial, nblk, ent_coef, grad, loss, 0, stream);
}

namespace {
int adam_launch(float* params, const float* grad, float* exp_avg, float* exp_avg_sq, float grad_scale,
                float max_grad_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt,
                float* grad_norm_out, float lsmin, void* stream) {
  if (!params || !grad || !exp_avg || !exp_avg_sq) return fail(ACKPPO_EINVAL, "ackppo_adam: bad arguments");
  hipLaunchKernelGGL(ackppo_adam_kernel, dim3((P / 4 + 255) / 256), dim3(256), 0, (hipStream_t)stream, params, grad,
                     exp_avg, exp_avg_sq, grad_scale, max_grad_norm, beta1, beta2, eps, step_size, bc2_sqrt,
                     grad_norm_out, lsmin);
  return launched("ackppo_adam");
}
// torch's bias corrections of Adam step t, in float64 as the host path
void adam_scalars(double lr, double beta1, double beta2, double t, float& step_size, float& bc2_sqrt) {
  step_size = (float)(lr / (1.0 - pow(beta1, t)));
  bc2_sqrt = (float)sqrt(1.0 - pow(beta2, t));
}
// one minibatch's reduction and Adam step (ackppo_epoch / ackppo_train, single rank): two launches,
// the norm from the reduction's block sums
int reduce_adam_launch(UpdArgs& U, void* stream) {
  U.sq = 1;
  reduce_norm_launch(U, (hipStream_t)stream);
  if (const int rc = launched("ackppo_reduce_norm")) return rc;
  hipLaunchKernelGGL(ackppo_adam_blocked_kernel, dim3(NB_N), dim3(256), 0, (hipStream_t)stream, U);
  return launched("ackppo_adam_blocked");
}
}  // namespace

int ackppo_adam(float* params, const float* grad, float* exp_avg, float* exp_avg_sq, float grad_scale,
                float max_grad_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt,
                float* grad_norm_out, void* stream) {
  return adam_launch(params, grad, exp_avg, exp_avg_sq, grad_scale, max_grad_norm, beta1, beta2, eps, step_size,
                     bc2_sqrt, grad_norm_out, -INFINITY, stream);
}

int ackppo_epoch(float* params, const float* obs_rows, const float* actions, const float* old_log_prob,
                 const float* advantages, const float* returns, const int32_t* idx, int n_idx, int batch,
                 const float* stats, float clip_range, float ent_coef, float vf_coef, float max_grad_norm,
                 double learning_rate, double beta1, double beta2, float eps, int64_t adam_step0,
                 float* grad_partial, float* loss_partial, float* grad, float* loss_acc, float* exp_avg,
                 float* exp_avg_sq, float* grad_norm_out, void* stream) {
  if (!params || !obs_rows || !actions || !old_log_prob || !advantages || !returns || !idx || !stats ||
      !grad_partial || !loss_partial || !grad || !loss_acc || !exp_avg || !exp_avg_sq || n_idx < 0 || batch <= 0 ||
      adam_step0 < 0)
    return fail(ACKPPO_EINVAL, "ackppo_epoch: bad arguments");
  const int nmb = (n_idx + batch - 1) / batch;
  UpdArgs U{grad_partial, 0, loss_partial, ent_coef, grad, loss_acc, 1, 1, params, exp_avg, exp_avg_sq,
            1.0f, max_grad_norm, (float)beta1, (float)beta2, eps, 0.0f, 0.0f, -INFINITY, grad_norm_out, nullptr};
  for (int m = 0; m < nmb; m++) {
    const int nb = n_idx - m * batch < batch ? n_idx - m * batch : batch;
    int rc = ackppo_grad(params, obs_rows, actions, old_log_prob, advantages, returns, idx + (size_t)m * batch, nb,
                         stats + 2 * m, clip_range, ent_coef, vf_coef, grad_partial, loss_partial, stream);
    if (rc) return rc;
    U.nblk = ackppo_grad_blocks(nb);
    adam_scalars(learning_rate, beta1, beta2, (double)(adam_step0 + m + 1), U.step_size, U.bc2_sqrt);
    if ((rc = reduce_adam_launch(U, stream))) return rc;
  }
  return ACKPPO_OK;
}


int ackppo_train(const ackppo_train_desc* d, void* stream) {
  if (!d || !d->obs_rows || !d->actions || !d->old_log_prob || !d->advantages || !d->returns || !d->params ||
      !d->exp_avg || !d->exp_avg_sq || !d->perm || !d->stats || !d->grad_partial || !d->loss_partial || !d->grad ||
      !d->loss_acc || d->n_idx < 0 || d->batch <= 0 || d->n_epochs < 0 || d->adam_step0 < 0 || d->world < 1)
    return fail(ACKPPO_EINVAL, "ackppo_train: bad arguments");
  // the data-parallel sequence whenever there is a hook (world 1 with a hook: its collectives reduce
  // over one rank -- the same path, timed on one GPU)
  const bool dp = d->allreduce != nullptr;
  if ((d->world > 1 && !dp) || (dp && !d->moments))
    return fail(ACKPPO_EINVAL, "ackppo_train: world > 1 needs an all-reduce hook, a hook needs the moments buffer");
  float* wimg = d->weight_image;
  const int S = d->n_idx, B = d->batch, nmb = (S + B - 1) / B;
  // the moments layout a hook uses: [3][n_epochs][nmb] with the all-epoch buffers, else [3][nmb];
  // the caller states the buffer's size, so a buffer sized for the per-epoch layout is refused, not
  // overrun
  const int64_t need_moments = 3 * (int64_t)nmb * ((d->perm_epochs && d->stats_epochs) ? d->n_epochs : 1);
  if (dp && d->moments_count < need_moments)
    return fail(ACKPPO_EINVAL, "ackppo_train: moments_count smaller than the hook's moments layout needs");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(d->loss_acc, 0, ACKPPO_NLOSS * sizeof(float), st) != hipSuccess)
    return fail(ACKPPO_EHIP, "ackppo_train: hipMemsetAsync(loss_acc)");
  if (S == 0 || d->n_epochs == 0) return ACKPPO_OK;
  if (wimg) {  // the image of the parameters as they are now; each Adam step below keeps it current
    hipLaunchKernelGGL(ackppo_wimage_kernel, dim3(2), dim3(GRAD_THREADS), 0, st, d->params, wimg);
    if (const int rc0 = launched("ackppo_train: weight image")) return rc0;
  }
  int rc;
  auto coll = [&](void* buf, int64_t count, int dtype, const char* what) -> int {
    g_err[0] = 0;
    const int r = d->allreduce(buf, count, dtype, d->allreduce_user, stream);
    if (r) {
      char why[sizeof g_err];
      snprintf(why, sizeof why, "%s", g_err);  // the hook's own message, if it left one
      snprintf(g_err, sizeof g_err, "ackppo_train: %s all-reduce failed (%d) %s", what, r, why);
      return ACKPPO_EHIP;
    }
    return ACKPPO_OK;
  };
  // with the per-call buffers: every epoch's shuffle and statistics at the start (the advantages do
  // not change during the call) -- single rank one launch; data-parallel the shuffles and first
  // moments in one launch, 2 all-reduces for all epochs (not 2 per epoch), deviations, finalize
  const bool all_epochs = d->perm_epochs && d->stats_epochs;
  if (all_epochs) {
    if (S > (1 << 30)) return fail(ACKPPO_EINVAL, "ackppo_train: n_idx too large for the shuffle");
    const dim3 grid(nmb, d->n_epochs);
    if (!dp) {
      hipLaunchKernelGGL(ackppo_perm_stats_kernel, grid, dim3(ADV_THREADS), 0, st, d->advantages, S, B, d->perm_key,
                         d->perm_epoch0, d->normalize_advantage, d->perm_epochs, d->stats_epochs);
      if ((rc = launched("ackppo_train: shuffles and statistics"))) return rc;
    } else {
      const int NM = nmb * d->n_epochs;
      double* mom = d->moments;
      hipLaunchKernelGGL(ackppo_perm_moments_kernel, grid, dim3(ADV_THREADS), 0, st, d->advantages, S, B, d->perm_key,
                         d->perm_epoch0, d->perm_epochs, mom);
      if ((rc = launched("ackppo_train: shuffles and moments"))) return rc;
      if ((rc = coll(mom, 2 * (int64_t)NM, ACKPPO_F64, "advantage count/sum"))) return rc;
      hipLaunchKernelGGL(ackppo_adv_moments_kernel, grid, dim3(ADV_THREADS), 0, st, d->advantages, d->perm_epochs, S,
                         B, 1, nmb, mom);
      if ((rc = launched("ackppo_train: advantage deviations"))) return rc;
      if ((rc = coll(mom + 2 * NM, NM, ACKPPO_F64, "advantage deviation"))) return rc;
      if ((rc = ackppo_adv_finalize(mom, NM, d->normalize_advantage, d->stats_epochs, stream))) return rc;
    }
  }
  UpdArgs U{d->grad_partial, 0, d->loss_partial, d->ent_coef, d->grad, d->loss_acc, 1, 1, d->params, d->exp_avg,
            d->exp_avg_sq, 1.0f / (float)d->world, d->max_grad_norm, (float)d->beta1, (float)d->beta2, d->eps, 0.0f,
            0.0f, d->log_std_min, d->grad_norm_out, wimg};
  for (int ep = 0; ep < d->n_epochs; ep++) {
    const int32_t* perm = all_epochs ? d->perm_epochs + (size_t)ep * S : d->perm;
    const float* stats = all_epochs ? d->stats_epochs + (size_t)ep * nmb * 2 : d->stats;
    if (!all_epochs && !dp) {
      if ((rc = ackppo_permutation(S, d->perm_key, d->perm_epoch0 + (uint32_t)ep, d->perm, stream))) return rc;
      if ((rc = ackppo_adv_stats(d->advantages, d->perm, S, B, d->normalize_advantage, d->stats, stream))) return rc;
    } else if (dp && !all_epochs) {
      if ((rc = ackppo_permutation(S, d->perm_key, d->perm_epoch0 + (uint32_t)ep, d->perm, stream))) return rc;
      double* mom = d->moments;
      if ((rc = ackppo_adv_moments(d->advantages, d->perm, S, B, 0, mom, stream))) return rc;
      if ((rc = coll(mom, 2 * (int64_t)nmb, ACKPPO_F64, "advantage count/sum"))) return rc;
      if ((rc = ackppo_adv_moments(d->advantages, d->perm, S, B, 1, mom, stream))) return rc;
      if ((rc = coll(mom + 2 * nmb, nmb, ACKPPO_F64, "advantage deviation"))) return rc;
      if ((rc = ackppo_adv_finalize(mom, nmb, d->normalize_advantage, d->stats, stream))) return rc;
    }
    for (int m = 0; m < nmb; m++) {
      const int nb = S - m * B < B ? S - m * B : B;
      GradArgs A{d->params, d->obs_rows, d->actions, d->old_log_prob, d->advantages, d->returns, perm + (size_t)m * B,
                 nb, stats + 2 * m, d->clip_range, d->ent_coef, d->vf_coef, d->grad_partial, d->loss_partial, wimg};
      if ((rc = grad_launch(A, stream))) return rc;
      U.nblk = ackppo_grad_blocks(nb);
      adam_scalars(d->learning_rate, d->beta1, d->beta2, (double)(d->adam_step0 + (int64_t)ep * nmb + m + 1),
                   U.step_size, U.bc2_sqrt);
      // single rank: the reduction (with the norm blocks' sums), the Adam step; data-parallel: the
      // reduction, the gradient's all-reduce, the norm blocks' sums, the Adam step (the same order)
      if (!dp) {
        if ((rc = reduce_adam_launch(U, stream))) return rc;
      } else {
        U.sq = 0;
        reduce_norm_launch(U, st);
        if ((rc = launched("ackppo_train: reduction"))) return rc;
        if ((rc = coll(d->grad, ACKPPO_NPARAM, ACKPPO_F32, "gradient"))) return rc;
        hipLaunchKernelGGL(ackppo_norm_blocks_kernel, dim3(NB_N), dim3(NB_P), 0, st, U);
        hipLaunchKernelGGL(ackppo_adam_blocked_kernel, dim3(NB_N), dim3(256), 0, st, U);
        if ((rc = launched("ackppo_train: Adam step"))) return rc;
      }
    }
  }
  return ACKPPO_OK;
}

// ---- native RCCL: the process's own librccl.so.1 (torch's, when it is loaded), opened at run time
namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclAllReduce) allreduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
  decltype(&ncclCommGetAsyncError) async_err = nullptr;
  bool ok = false;
};
Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    // only the RCCL already in the process (torch's): a second copy, built against another HIP
    // runtime, must never be loaded beside it (its communicators would not be torch's either)
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) return x;
    x.get_id = (decltype(x.get_id))dlsym(h, "ncclGetUniqueId");
    x.init = (decltype(x.init))dlsym(h, "ncclCommInitRank");
    x.allreduce = (decltype(x.allreduce))dlsym(h, "ncclAllReduce");
    x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
    x.errstr = (decltype(x.errstr))dlsym(h, "ncclGetErrorString");
    x.async_err = (decltype(x.async_err))dlsym(h, "ncclCommGetAsyncError");
    x.ok = x.get_id && x.init && x.allreduce && x.destroy && x.errstr && x.async_err;
    return x;
  }();
  return r;
}
int rccl_fail(const char* what, ncclResult_t r) {
  snprintf(g_err, sizeof g_err, "%s: %s", what, rccl().errstr ? rccl().errstr(r) : "RCCL error");
  return ACKPPO_EHIP;
}
// A non-blocking communicator (ncclConfig_t::blocking = 0, e.g. one torch built with
// TORCH_NCCL_USE_COMM_NONBLOCKING) may return ncclInProgress from an enqueue: the call is then
// still being issued, and ncclCommGetAsyncError reports ncclInProgress until it is done. Poll it
// (bounded: 60 s of host time, then an error -- never a silent success).
ncclResult_t rccl_settle(ncclComm_t comm, ncclResult_t r) {
  if (r != ncclInProgress) return r;
  const auto t0 = std::chrono::steady_clock::now();
  while (r == ncclInProgress) {
    if (rccl().async_err(comm, &r) != ncclSuccess) return ncclInternalError;
    if (r == ncclInProgress && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return ncclInProgress;
  }
  return r;
}
}  // namespace

int ackppo_rccl_unique_id(void* id128) {
  if (!id128) return fail(ACKPPO_EINVAL, "ackppo_rccl_unique_id: bad arguments");
  if (!rccl().ok) return fail(ACKPPO_EHIP, "ackppo_rccl_unique_id: no librccl.so.1 loaded in this process (import torch first)");
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
  ncclUniqueId id;
  const ncclResult_t r = rccl().get_id(&id);
  if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
  memcpy(id128, &id, sizeof id);
  return ACKPPO_OK;
}

int ackppo_rccl_init(const void* id128, int nranks, int rank, void** comm) {
  if (!id128 || !comm || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(ACKPPO_EINVAL, "ackppo_rccl_init: bad arguments");
  if (!rccl().ok) return fail(ACKPPO_EHIP, "ackppo_rccl_init: no librccl.so.1 loaded in this process (import torch first)");
  ncclUniqueId id;
  memcpy(&id, id128, sizeof id);
  ncclComm_t c = nullptr;
  const ncclResult_t r = rccl().init(&c, nranks, id, rank);
  if (r != ncclSuccess) return rccl_fail("ncclCommInitRank", r);  // a blocking communicator (no config)
  *comm = c;
  return ACKPPO_OK;
}

int ackppo_rccl_allreduce(void* buf, int64_t count, int dtype, void* comm, void* stream) {
  if (!buf || !comm || count < 0 || (dtype != ACKPPO_F32 && dtype != ACKPPO_F64))
    return fail(ACKPPO_EINVAL, "ackppo_rccl_allreduce: bad arguments");
  if (!rccl().ok) return fail(ACKPPO_EHIP, "ackppo_rccl_allreduce: no librccl.so.1 loaded in this process");
  const ncclResult_t r = rccl_settle(
      (ncclComm_t)comm, rccl().allreduce(buf, buf, (size_t)count, dtype == ACKPPO_F32 ? ncclFloat32 : ncclFloat64,
                                         ncclSum, (ncclComm_t)comm, (hipStream_t)stream));
  return r == ncclSuccess ? ACKPPO_OK : rccl_fail("ncclAllReduce", r);
}

int ackppo_rccl_destroy(void* comm) {
  if (!comm) return ACKPPO_OK;
  if (!rccl().ok) return fail(ACKPPO_EHIP, "ackppo_rccl_destroy: no librccl.so.1 loaded in this process");
  const ncclResult_t r = rccl().destroy((ncclComm_t)comm);
  return r == ncclSuccess ? ACKPPO_OK : rccl_fail("ncclCommDestroy", r);
}

int ackppo_rccl_library(char* path, int size) {
  if (!path || size <= 0) return fail(ACKPPO_EINVAL, "ackppo_rccl_library: bad arguments");
  path[0] = 0;
  if (!rccl().ok) return fail(ACKPPO_EHIP, "ackppo_rccl_library: no librccl.so.1 loaded in this process");
  Dl_info info;
  if (!dladdr((void*)rccl().allreduce, &info) || !info.dli_fname)
    return fail(ACKPPO_EHIP, "ackppo_rccl_library: dladdr failed");
  snprintf(path, (size_t)size, "%s", info.dli_fname);
  return ACKPPO_OK;
}

}  // extern "C"
