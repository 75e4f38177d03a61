// ackppo.hip -- on-device PPO learner kernels for gfx950 (C-ABI: include/ackppo.h).
//
// Restates stable-baselines3 2.7.0 PPO('MlpPolicy') as src/rl/train.py:99-128 configures it
// (hyper-parameters: the rl_logs/ppo checkpoints' data file). Network: 79-64-64 tanh actor and critic MLPs.
//
// Mapping:
//  * rollout (ackppo_act / ackppo_value / ackppo_bootstrap): one lane per env, 64-lane
//    workgroups; weights are read with wave-uniform addresses (scalar loads through the
//    constant cache, FMA with an SGPR operand), hidden activations live in a per-lane LDS
//    column so the unit loop stays rolled.
//  * update (ackppo_grad): one 256-lane workgroup per 64-sample tile, lane = sample. Waves 0-1
//    run the actor, waves 2-3 the critic, each on half of the hidden units: forward, loss
//    gradient, backward to the hidden layers, all activations/deltas staged in LDS tiles
//    [unit][sample]. All four waves then form
//    the weight gradients (sums over the tile of outer products) as 4x4 register blocks fed
//    by 16-B LDS reads along the sample axis, and write the tile's partial gradient row.
//    ackppo_reduce sums the rows (coalesced over parameters); ackppo_adam applies the global
//    norm clip and the Adam step. The whole minibatch is 3 launches, no host round trip.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/ackppo.h"

#ifndef PP_UNROLL
#define PP_UNROLL 2
#endif
#define PP_STR2(x) #x
#define PP_STR(x) PP_STR2(x)
#define PP_UNROLL_STR PP_STR(unroll PP_UNROLL)

namespace pp {

constexpr int NOBS = ACKPPO_NOBS, NA = ACKPPO_NACT, H = ACKPPO_HIDDEN, P = ACKPPO_NPARAM;
constexpr int TILE = ACKPPO_TILE;
constexpr int LDP = 68;  // LDS row stride of the grad tiles: 16-B aligned rows, 4-bank skew per row
constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;
constexpr float TWO_PI = 6.28318530717958647692f;

struct Net {
  int w1, b1, w2, b2;
};
constexpr Net ACTOR{ACKPPO_OFF_PI_W1, ACKPPO_OFF_PI_B1, ACKPPO_OFF_PI_W2, ACKPPO_OFF_PI_B2};
constexpr Net CRITIC{ACKPPO_OFF_VF_W1, ACKPPO_OFF_VF_B1, ACKPPO_OFF_VF_W2, ACKPPO_OFF_VF_B2};

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// out[j] = tanh(b[j] + W[j,:] . x) for the 64 units, written to an LDS column (stride cs).
// W/b addresses are wave-uniform: scalar loads, x stays in VGPRs.
template <int IN>
__device__ __forceinline__ void dense_tanh(const float* __restrict__ W, const float* __restrict__ b,
                                           const float (&x)[IN], float* col, int cs) {
_Pragma(PP_UNROLL_STR)
  for (int j = 0; j < H; j++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < IN; k++) acc = fmaf(W[j * IN + k], x[k], acc);
    col[j * cs] = tanhf(acc + b[j]);
  }
}

template <int N>
__device__ __forceinline__ void load_col(const float* col, int cs, float (&h)[N]) {
#pragma unroll
  for (int k = 0; k < N; k++) h[k] = col[k * cs];
}

// trunk of one net: x -> h2 (registers); h1 and h2 also left in LDS columns c1 / c2
__device__ __forceinline__ void trunk(const float* __restrict__ p, const Net net, const float (&x)[NOBS], float* c1,
                                      float* c2, int cs, float (&h)[H]) {
  dense_tanh<NOBS>(p + net.w1, p + net.b1, x, c1, cs);
  load_col(c1, cs, h);
  dense_tanh<H>(p + net.w2, p + net.b2, h, c2, cs);
  load_col(c2, cs, h);
}

__device__ __forceinline__ float critic_head(const float* __restrict__ p, const float (&h)[H]) {
  float v = 0.0f;
#pragma unroll
  for (int j = 0; j < H; j++) v = fmaf(p[ACKPPO_OFF_VAL_W + j], h[j], v);
  return v + p[ACKPPO_OFF_VAL_B];
}

__device__ __forceinline__ void actor_head(const float* __restrict__ p, const float (&h)[H], float mu[NA]) {
#pragma unroll
  for (int d = 0; d < NA; d++) {
    float m = 0.0f;
#pragma unroll
    for (int j = 0; j < H; j++) m = fmaf(p[ACKPPO_OFF_ACT_W + d * H + j], h[j], m);
    mu[d] = m + p[ACKPPO_OFF_ACT_B + d];
  }
}

// torch.distributions.Normal.log_prob summed over the action dims (SB3 DiagGaussianDistribution)
__device__ __forceinline__ float gauss_logp(const float a[NA], const float mu[NA], const float* __restrict__ p) {
  float lp = 0.0f;
#pragma unroll
  for (int d = 0; d < NA; d++) {
    const float sigma = expf(p[ACKPPO_OFF_LOG_STD + d]);
    const float dv = a[d] - mu[d];
    lp += -(dv * dv) / (2.0f * sigma * sigma) - logf(sigma) - LOG_SQRT_2PI;
  }
  return lp;
}

__device__ __forceinline__ void load_obs_soa(const float* obs, int n, int e, float (&x)[NOBS]) {
#pragma unroll
  for (int k = 0; k < NOBS; k++) x[k] = obs[(size_t)k * n + e];
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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
};

// Policy tile: 64 envs (lane = env) x 4 waves. The whole parameter vector is staged in LDS once
// per workgroup (wide coalesced loads) and read back with wave-uniform addresses (LDS broadcast).
// Waves split the hidden units: wave w computes units [32w, 32w+32) of the concatenated
// actor|critic layers (waves 0-1 actor, 2-3 critic), activations exchanged through LDS tiles
// H1/H2 [128 units][64 envs].
constexpr int PT_ENVS = 64, PT_THREADS = 256;
struct PolicyLds {
  float w[P];
  float h1[2 * H * PT_ENVS];
  float h2[2 * H * PT_ENVS];
};

__device__ __forceinline__ void stage_params(const float* __restrict__ p, float* w) {
  const float4* src = reinterpret_cast<const float4*>(p);
  float4* dst = reinterpret_cast<float4*>(w);
#pragma unroll 4
  for (int i = threadIdx.x; i < P / 4; i += PT_THREADS) dst[i] = src[i];
}

// trunks of both nets for the tile; leaves H2 in LDS (caller syncs after)
__device__ __forceinline__ void policy_trunks(PolicyLds& L, const float (&x)[NOBS], int lane, int wave,
                                              bool actor, bool critic) {
  const bool mine = (wave < 2) ? actor : critic;
  const Net net = (wave < 2) ? ACTOR : CRITIC;
  const int u0 = (wave & 1) * 32;   // first unit of this wave within its net
  const int hrow = (wave >> 1) * H;  // actor rows 0..63, critic rows 64..127
  if (mine) {
    const float* W1 = L.w + net.w1;
    const float* b1 = L.w + net.b1;
_Pragma(PP_UNROLL_STR)
    for (int u = u0; u < u0 + 32; u++) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < NOBS; k++) acc = fmaf(W1[u * NOBS + k], x[k], acc);
      L.h1[(hrow + u) * PT_ENVS + lane] = tanhf(acc + b1[u]);
    }
  }
  __syncthreads();
  if (mine) {
    float h[H];
#pragma unroll
    for (int k = 0; k < H; k++) h[k] = L.h1[(hrow + k) * PT_ENVS + lane];
    const float* W2 = L.w + net.w2;
    const float* b2 = L.w + net.b2;
_Pragma(PP_UNROLL_STR)
    for (int u = u0; u < u0 + 32; u++) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < H; k++) acc = fmaf(W2[u * H + k], h[k], acc);
      L.h2[(hrow + u) * PT_ENVS + lane] = tanhf(acc + b2[u]);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float tile_value(const PolicyLds& L, int lane) {
  float v = 0.0f;
#pragma unroll 8
  for (int j = 0; j < H; j++) v = fmaf(L.w[ACKPPO_OFF_VAL_W + j], L.h2[(H + j) * PT_ENVS + lane], v);
  return v + L.w[ACKPPO_OFF_VAL_B];
}

__device__ __forceinline__ void tile_mu(const PolicyLds& L, int lane, float mu[NA]) {
#pragma unroll
  for (int d = 0; d < NA; d++) {
    float m = 0.0f;
#pragma unroll 8
    for (int j = 0; j < H; j++) m = fmaf(L.w[ACKPPO_OFF_ACT_W + d * H + j], L.h2[j * PT_ENVS + lane], m);
    mu[d] = m + L.w[ACKPPO_OFF_ACT_B + d];
  }
}

extern "C" __global__ void __launch_bounds__(PT_THREADS) ackppo_act_kernel(ActArgs A) {
  extern __shared__ float lds_raw[];
  PolicyLds& L = *reinterpret_cast<PolicyLds*>(lds_raw);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int e = blockIdx.x * PT_ENVS + lane;
  const bool valid = e < A.n;
  const int ec = valid ? e : A.n - 1;  // padding lanes recompute the last env, write nothing
  stage_params(A.params, L.w);
  float x[NOBS];
  load_obs_soa(A.obs, A.n, ec, x);
  __syncthreads();
  if (A.obs_rows && valid && wave >= 2) {  // waves 2/3 copy the observation row (half each)
    const int k0 = wave == 2 ? 0 : 40, k1 = wave == 2 ? 40 : NOBS;
#pragma unroll
    for (int k = 0; k < NOBS; k++)
      if (k >= k0 && k < k1) A.obs_rows[(size_t)e * NOBS + k] = x[k];
  }
  policy_trunks(L, x, lane, wave, true, A.value != nullptr);
  if (!valid) return;
  if (wave == 2 && A.value) A.value[e] = tile_value(L, lane);
  if (wave != 0) return;
  const float* p = L.w;
  float mu[NA], a[NA];
  tile_mu(L, lane, mu);
  if (A.deterministic) {
    a[0] = mu[0];
    a[1] = mu[1];
  } else {
    uint32_t c[4] = {(uint32_t)(A.env_offset + e), A.step, 2u, 0u};
    philox(c, (uint32_t)A.seed, (uint32_t)(A.seed >> 32));
    const float u1 = (float)((c[0] >> 8) + 1u) * (1.0f / 16777216.0f);  // (0, 1]
    const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);         // [0, 1)
    const float r = sqrtf(-2.0f * logf(u1));
    const float z[NA] = {r * cosf(TWO_PI * u2), r * sinf(TWO_PI * u2)};
#pragma unroll
    for (int d = 0; d < NA; d++) a[d] = mu[d] + expf(p[ACKPPO_OFF_LOG_STD + d]) * z[d];
  }
  if (A.action) {
    A.action[2 * (size_t)e] = a[0];
    A.action[2 * (size_t)e + 1] = a[1];
  }
  A.env_action[2 * (size_t)e] = fminf(fmaxf(a[0], -1.0f), 1.0f);
  A.env_action[2 * (size_t)e + 1] = fminf(fmaxf(a[1], -1.0f), 1.0f);
  if (A.log_prob) A.log_prob[e] = gauss_logp(a, mu, p);
}

extern "C" __global__ void __launch_bounds__(PT_THREADS) ackppo_value_kernel(const float* params, const float* obs,
                                                                             int n, float* value) {
  extern __shared__ float lds_raw[];
  PolicyLds& L = *reinterpret_cast<PolicyLds*>(lds_raw);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int e = blockIdx.x * PT_ENVS + lane;
  const int ec = e < n ? e : n - 1;
  stage_params(params, L.w);
  float x[NOBS];
  load_obs_soa(obs, n, ec, x);
  __syncthreads();
  policy_trunks(L, x, lane, wave, false, true);
  if (e < n && wave == 2) value[e] = tile_value(L, lane);
}

// bootstrap: only tiles holding a truncated (not terminated) env run the critic
extern "C" __global__ void __launch_bounds__(PT_THREADS) ackppo_bootstrap_kernel(const float* params, const float* tobs,
                                                                                 const float* reward,
                                                                                 const uint8_t* term,
                                                                                 const uint8_t* trunc, int n,
                                                                                 float gamma, float* reward_out,
                                                                                 float* done_out) {
  extern __shared__ float lds_raw[];
  PolicyLds& L = *reinterpret_cast<PolicyLds*>(lds_raw);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int e = blockIdx.x * PT_ENVS + lane;
  const bool valid = e < n;
  const int ec = valid ? e : n - 1;
  const bool te = term[ec] != 0, tr = trunc[ec] != 0;
  const bool boot = valid && tr && !te;  // TimeLimit.truncated = truncated and not terminated
  if (__syncthreads_or(boot)) {
    stage_params(params, L.w);
    float x[NOBS];
    load_obs_soa(tobs, n, ec, x);
    __syncthreads();
    policy_trunks(L, x, lane, wave, false, true);
  }
  if (valid && wave == 2) {
    float r = reward[e];
    if (boot) r += gamma * tile_value(L, lane);
    reward_out[e] = r;
    done_out[e] = (te || tr) ? 1.0f : 0.0f;
  }
}

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

extern "C" __global__ void __launch_bounds__(256) ackppo_adv_stats_kernel(const float* adv, const int32_t* idx,
                                                                          int n_idx, int batch, int normalize,
                                                                          float* stats) {
  __shared__ double red[256];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int lo = m * batch, hi = min(lo + batch, n_idx), cnt = hi - lo;
  if (!normalize || cnt <= 1) {
    if (tid == 0) { stats[2 * m] = 0.0f; stats[2 * m + 1] = 1.0f; }
    return;
  }
  double s = 0.0;
#pragma unroll 8
  for (int i = lo + tid; i < hi; i += 256) s += adv[idx[i]];
  red[tid] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const double mean = red[0] / cnt;
  __syncthreads();
  double q = 0.0;
#pragma unroll 8
  for (int i = lo + tid; i < hi; i += 256) {
    const double d = adv[idx[i]] - mean;
    q += d * d;
  }
  red[tid] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    const float sd = (float)sqrt(red[0] / (cnt - 1));
    stats[2 * m] = (float)mean;
    stats[2 * m + 1] = 1.0f / (sd + 1e-8f);
  }
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
};

// LDS map of one tile (floats, rows of LDP): X [80 rows], then per net h1, h2, d2, d1 [64 rows each],
// then gmu [2], glog [2], gv [1] rows.
constexpr int T_X = 0, T_NET = 80 * LDP, NET_SZ = 4 * H * LDP;
constexpr int T_H1 = 0, T_H2 = H * LDP, T_D2 = 2 * H * LDP, T_D1 = 3 * H * LDP;
constexpr int T_VEC = T_NET + 2 * NET_SZ;
constexpr int T_GMU = T_VEC, T_GLOG = T_VEC + 2 * LDP, T_GV = T_VEC + 4 * LDP;
constexpr int T_TOTAL = T_VEC + 5 * LDP;
static_assert(T_TOTAL * 4 <= 160 * 1024, "grad tile exceeds the 160 KiB LDS of a CU");
constexpr int GRAD_THREADS = 256;

// sum over the tile's samples of a[ra][s] * b[rb][s] for a 4x4 block of rows (16-B LDS reads)
__device__ __forceinline__ void outer4x4(const float* a, const float* b, float acc[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = 0.0f;
#pragma unroll 4
  for (int s = 0; s < TILE; s += 4) {
    float4 av[4], bv[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      av[i] = *reinterpret_cast<const float4*>(a + i * LDP + s);
      bv[i] = *reinterpret_cast<const float4*>(b + i * LDP + s);
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        acc[i][j] = fmaf(av[i].x, bv[j].x, acc[i][j]);
        acc[i][j] = fmaf(av[i].y, bv[j].y, acc[i][j]);
        acc[i][j] = fmaf(av[i].z, bv[j].z, acc[i][j]);
        acc[i][j] = fmaf(av[i].w, bv[j].w, acc[i][j]);
      }
  }
}

__device__ __forceinline__ float row_sum(const float* a) {
  float s = 0.0f;
#pragma unroll 4
  for (int i = 0; i < TILE; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(a + i);
    s += (v.x + v.y) + (v.z + v.w);
  }
  return s;
}

__device__ __forceinline__ float row_dot(const float* a, const float* b) {
  float s = 0.0f;
#pragma unroll 4
  for (int i = 0; i < TILE; i += 4) {
    const float4 u = *reinterpret_cast<const float4*>(a + i), v = *reinterpret_cast<const float4*>(b + i);
    s = fmaf(u.x, v.x, s);
    s = fmaf(u.y, v.y, s);
    s = fmaf(u.z, v.z, s);
    s = fmaf(u.w, v.w, s);
  }
  return s;
}

extern "C" __global__ void __launch_bounds__(GRAD_THREADS) ackppo_grad_kernel(GradArgs A) {
  extern __shared__ float tl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar weight loads below
  const int blk = blockIdx.x;
  const int s0 = blk * TILE;
  const int nvalid = min(TILE, A.batch - s0);
  const float* __restrict__ p = A.params;

  // cooperative gather of the tile's observation rows into X [k][s] (zero rows for padding):
  // thread t copies a quarter row (20 words) with all its loads in flight at once
  {
    const int s = tid >> 2, q = tid & 3;
    const bool ok = s < nvalid;
    const float* row = A.obs_rows + (size_t)(ok ? A.idx[s0 + s] : 0) * NOBS;
    float v[20];
#pragma unroll
    for (int i = 0; i < 20; i++) {
      const int k = q * 20 + i;
      v[i] = (ok && k < NOBS) ? row[k] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 20; i++) tl[T_X + (q * 20 + i) * LDP + s] = v[i];
  }
  __syncthreads();

  // ---- per-sample forward / loss gradient / backward. lane = sample; wave w works on net
  // (w >> 1) (0 actor, 1 critic) and on units [32 (w & 1), +32) of each of its layers.
  const bool valid = lane < nvalid;
  const int sidx = valid ? A.idx[s0 + lane] : 0;
  const int nid = wave >> 1, u0 = (wave & 1) * 32;
  const Net net = nid == 0 ? ACTOR : CRITIC;
  float* nt = tl + T_NET + nid * NET_SZ;
  const float invB = 1.0f / (float)A.batch;
  {  // layer 1
    float x[NOBS];
    load_col(tl + T_X + lane, LDP, x);
    const float* W1 = p + net.w1;
_Pragma(PP_UNROLL_STR)
    for (int u = u0; u < u0 + 32; u++) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < NOBS; k++) acc = fmaf(W1[u * NOBS + k], x[k], acc);
      nt[T_H1 + u * LDP + lane] = tanhf(acc + p[net.b1 + u]);
    }
  }
  __syncthreads();
  {  // layer 2
    float h[H];
    load_col(nt + T_H1 + lane, LDP, h);
    const float* W2 = p + net.w2;
_Pragma(PP_UNROLL_STR)
    for (int u = u0; u < u0 + 32; u++) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < H; k++) acc = fmaf(W2[u * H + k], h[k], acc);
      nt[T_H2 + u * LDP + lane] = tanhf(acc + p[net.b2 + u]);
    }
  }
  __syncthreads();
  // heads and the loss gradient w.r.t. their outputs (waves 0 and 2)
  float loss_a = 0.0f, loss_b = 0.0f, loss_c = 0.0f;
  if (wave == 0) {
    float h[H], mu[NA], a[NA];
    load_col(nt + T_H2 + lane, LDP, h);
    actor_head(p, h, mu);
    a[0] = A.actions[2 * (size_t)sidx];
    a[1] = A.actions[2 * (size_t)sidx + 1];
    const float logp = gauss_logp(a, mu, p);
    const float lr = logp - A.old_logp[sidx];
    const float r = expf(lr);
    const float adv = (A.adv[sidx] - A.stats[0]) * A.stats[1];
    const float rc = fminf(fmaxf(r, 1.0f - A.clip), 1.0f + A.clip);
    const float l1 = adv * r, l2 = adv * rc;
    // d(-min(l1, l2))/dlogp: through l1 when it is the minimum (ties: torch.min splits the
    // gradient and the clamp passes it, so the sum is the full l1 gradient), else 0
    const float glogp = valid ? ((l1 <= l2) ? -adv * r * invB : 0.0f) : 0.0f;
#pragma unroll
    for (int d = 0; d < NA; d++) {
      const float sigma = expf(p[ACKPPO_OFF_LOG_STD + d]);
      const float dv = a[d] - mu[d];
      tl[T_GMU + d * LDP + lane] = glogp * dv / (sigma * sigma);
      tl[T_GLOG + d * LDP + lane] = glogp * (dv * dv / (sigma * sigma) - 1.0f);
    }
    if (valid) {
      loss_a = -fminf(l1, l2);
      loss_b = (fabsf(r - 1.0f) > A.clip) ? 1.0f : 0.0f;
      loss_c = (r - 1.0f) - lr;
    }
  } else if (wave == 2) {
    float h[H];
    load_col(nt + T_H2 + lane, LDP, h);
    const float v = critic_head(p, h);
    const float R = A.ret[sidx];
    tl[T_GV + lane] = valid ? A.vf_coef * 2.0f * (v - R) * invB : 0.0f;
    if (valid) loss_a = (R - v) * (R - v);
  }
  __syncthreads();
  // d2[u] = (dL/dh2[u]) (1 - h2[u]^2) for this wave's units
  if (nid == 0) {
    const float g0 = tl[T_GMU + lane], g1 = tl[T_GMU + LDP + lane];
#pragma unroll 4
    for (int u = u0; u < u0 + 32; u++) {
      const float hu = nt[T_H2 + u * LDP + lane];
      nt[T_D2 + u * LDP + lane] = (g0 * p[ACKPPO_OFF_ACT_W + u] + g1 * p[ACKPPO_OFF_ACT_W + H + u]) * (1.0f - hu * hu);
    }
  } else {
    const float gv = tl[T_GV + lane];
#pragma unroll 4
    for (int u = u0; u < u0 + 32; u++) {
      const float hu = nt[T_H2 + u * LDP + lane];
      nt[T_D2 + u * LDP + lane] = gv * p[ACKPPO_OFF_VAL_W + u] * (1.0f - hu * hu);
    }
  }
  __syncthreads();
  {  // d1[k] = (sum_j d2[j] W2[j][k]) (1 - h1[k]^2) for this wave's k in [u0, u0+32)
    float d1[32];
#pragma unroll
    for (int k = 0; k < 32; k++) d1[k] = 0.0f;
    const float* W2 = p + net.w2 + u0;
_Pragma(PP_UNROLL_STR)
    for (int j = 0; j < H; j++) {
      const float dj = nt[T_D2 + j * LDP + lane];
#pragma unroll
      for (int k = 0; k < 32; k++) d1[k] = fmaf(dj, W2[j * H + k], d1[k]);
    }
#pragma unroll
    for (int k = 0; k < 32; k++) {
      const float hk = nt[T_H1 + (u0 + k) * LDP + lane];
      nt[T_D1 + (u0 + k) * LDP + lane] = d1[k] * (1.0f - hk * hk);
    }
  }
  // loss statistics of the tile (waves 0 and 2 hold them)
  if (wave == 0 || wave == 2) {
    loss_a = wave_sum(loss_a);
    loss_b = wave_sum(loss_b);
    loss_c = wave_sum(loss_c);
    if (lane == 0) {
      float* lp = A.lpart + (size_t)blk * ACKPPO_NLOSS;
      if (wave == 0) {
        lp[0] = loss_a;
        lp[2] = loss_b;
        lp[3] = loss_c;
        lp[4] = (float)nvalid;
        lp[5] = lp[6] = lp[7] = 0.0f;
      } else {
        lp[1] = loss_a;
      }
    }
  }
  __syncthreads();

  // ---- weight gradients: sums over the tile of outer products (all waves, both nets)
  float* g = A.gpart + (size_t)blk * P;
  // layer 1: [64 units][79 inputs] per net as 4x4 blocks (16 x 20 blocks per net)
  for (int b = tid; b < 2 * 16 * 20; b += GRAD_THREADS) {
    const int nn = b / 320, r = b - nn * 320, jb = r / 20, kb = r - jb * 20;
    const float* net_t = tl + T_NET + nn * NET_SZ;
    float acc[4][4];
    outer4x4(net_t + T_D1 + 4 * jb * LDP, tl + T_X + 4 * kb * LDP, acc);
    const int w1 = nn == 0 ? ACKPPO_OFF_PI_W1 : ACKPPO_OFF_VF_W1;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (4 * kb + j < NOBS) g[w1 + (4 * jb + i) * NOBS + 4 * kb + j] = acc[i][j];
  }
  // layer 2: [64][64] per net (16 x 16 blocks per net)
  for (int b = tid; b < 2 * 16 * 16; b += GRAD_THREADS) {
    const int nn = b / 256, r = b - nn * 256, jb = r / 16, kb = r - jb * 16;
    const float* net_t = tl + T_NET + nn * NET_SZ;
    float acc[4][4];
    outer4x4(net_t + T_D2 + 4 * jb * LDP, net_t + T_H1 + 4 * kb * LDP, acc);
    const int w2 = nn == 0 ? ACKPPO_OFF_PI_W2 : ACKPPO_OFF_VF_W2;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) g[w2 + (4 * jb + i) * H + 4 * kb + j] = acc[i][j];
  }
  // biases, heads, log_std
  const float* an = tl + T_NET;
  const float* cn = tl + T_NET + NET_SZ;
  for (int i = tid; i < 453; i += GRAD_THREADS) {
    if (i < 64) g[ACKPPO_OFF_PI_B1 + i] = row_sum(an + T_D1 + i * LDP);
    else if (i < 128) g[ACKPPO_OFF_PI_B2 + i - 64] = row_sum(an + T_D2 + (i - 64) * LDP);
    else if (i < 192) g[ACKPPO_OFF_VF_B1 + i - 128] = row_sum(cn + T_D1 + (i - 128) * LDP);
    else if (i < 256) g[ACKPPO_OFF_VF_B2 + i - 192] = row_sum(cn + T_D2 + (i - 192) * LDP);
    else if (i < 384) {
      const int d = (i - 256) >> 6, j = (i - 256) & 63;
      g[ACKPPO_OFF_ACT_W + d * H + j] = row_dot(tl + T_GMU + d * LDP, an + T_H2 + j * LDP);
    } else if (i < 386) g[ACKPPO_OFF_ACT_B + i - 384] = row_sum(tl + T_GMU + (i - 384) * LDP);
    else if (i < 450) g[ACKPPO_OFF_VAL_W + i - 386] = row_dot(tl + T_GV, cn + T_H2 + (i - 386) * LDP);
    else if (i == 450) g[ACKPPO_OFF_VAL_B] = row_sum(tl + T_GV);
    else g[ACKPPO_OFF_LOG_STD + i - 451] = row_sum(tl + T_GLOG + (i - 451) * LDP);
  }
}

extern "C" __global__ void __launch_bounds__(256) ackppo_reduce_kernel(const float* gpart, const float* lpart, int nblk,
                                                                       float ent_coef, float* grad, float* loss) {
  const int pidx = blockIdx.x * 256 + threadIdx.x;
  if (pidx < P) {
    // 8 independent partial sums keep 8 row loads in flight per thread
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int b = 0;
    for (; b + 8 <= nblk; b += 8) {
#pragma unroll
      for (int i = 0; i < 8; i++) acc[i] += gpart[(size_t)(b + i) * P + pidx];
    }
    for (; b < nblk; b++) acc[0] += gpart[(size_t)b * P + pidx];
    float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    if (pidx == ACKPPO_OFF_LOG_STD || pidx == ACKPPO_OFF_LOG_STD + 1) s -= ent_coef;
    grad[pidx] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x < ACKPPO_NLOSS) {
    float s = 0.0f;
    for (int b = 0; b < nblk; b++) s += lpart[(size_t)b * ACKPPO_NLOSS + threadIdx.x];
    loss[threadIdx.x] = s;
  }
}

extern "C" __global__ void __launch_bounds__(256) ackppo_adam_kernel(float* params, const float* grad, float* m,
                                                                     float* v, float scale, float max_norm, float b1,
                                                                     float b2, float eps, float step_size,
                                                                     float bc2_sqrt, float* norm_out) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  // every block forms the global norm itself (75 KB from L2) instead of a second launch
  float ss = 0.0f;
#pragma unroll 8
  for (int i = tid; i < P; i += 256) {
    const float gi = grad[i] * scale;
    ss = fmaf(gi, gi, ss);
  }
  red[tid] = ss;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float norm = sqrtf(red[0]);
  const float coef = fminf(max_norm / (norm + 1e-6f), 1.0f);  // torch clip_grad_norm_
  if (blockIdx.x == 0 && tid == 0 && norm_out) norm_out[0] = norm;
  const int i = blockIdx.x * 256 + tid;
  if (i >= P) return;
  const float gi = grad[i] * scale * coef;
  const float mi = m[i] + (1.0f - b1) * (gi - m[i]);  // exp_avg.lerp_(grad, 1 - beta1)
  const float vi = v[i] * b2 + (1.0f - b2) * gi * gi;  // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  m[i] = mi;
  v[i] = vi;
  params[i] -= step_size * (mi / (sqrtf(vi) / bc2_sqrt + eps));
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
constexpr size_t GRAD_LDS = (size_t)T_TOTAL * sizeof(float);
bool g_grad_attr = false;
bool g_policy_attr = false;
bool policy_lds_ready() {
  if (g_policy_attr) return true;
  const void* ks[3] = {(const void*)ackppo_act_kernel, (const void*)ackppo_value_kernel,
                       (const void*)ackppo_bootstrap_kernel};
  for (const void* k : ks)
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(PolicyLds)) != hipSuccess)
      return false;
  g_policy_attr = true;
  return true;
}
}  // namespace

extern "C" {

const char* ackppo_last_error(void) { return g_err; }

int ackppo_act(const float* params, const float* obs_soa, int n_env, int64_t env_offset, uint64_t seed, uint32_t step,
               int deterministic, float* obs_rows, float* action, float* env_action, float* log_prob, float* value,
               void* stream) {
  if (!params || !obs_soa || !env_action || n_env < 0) return fail(ACKPPO_EINVAL, "ackppo_act: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  ActArgs A{params, obs_soa, n_env, env_offset, seed, step, deterministic, obs_rows, action, env_action, log_prob, value};
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_act: cannot reserve the policy LDS tile");
  hipLaunchKernelGGL(ackppo_act_kernel, dim3((n_env + PT_ENVS - 1) / PT_ENVS), dim3(PT_THREADS), sizeof(PolicyLds),
                     (hipStream_t)stream, A);
  return launched("ackppo_act");
}

int ackppo_value(const float* params, const float* obs_soa, int n_env, float* value, void* stream) {
  if (!params || !obs_soa || !value || n_env < 0) return fail(ACKPPO_EINVAL, "ackppo_value: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_value: cannot reserve the policy LDS tile");
  hipLaunchKernelGGL(ackppo_value_kernel, dim3((n_env + PT_ENVS - 1) / PT_ENVS), dim3(PT_THREADS), sizeof(PolicyLds),
                     (hipStream_t)stream, params, obs_soa, n_env, value);
  return launched("ackppo_value");
}

int ackppo_bootstrap(const float* params, const float* terminal_obs_soa, const float* reward, const uint8_t* term,
                     const uint8_t* trunc, int n_env, float gamma, float* reward_out, float* done_out, void* stream) {
  if (!params || !terminal_obs_soa || !reward || !term || !trunc || !reward_out || !done_out || n_env < 0)
    return fail(ACKPPO_EINVAL, "ackppo_bootstrap: bad arguments");
  if (n_env == 0) return ACKPPO_OK;
  if (!policy_lds_ready()) return fail(ACKPPO_EHIP, "ackppo_bootstrap: cannot reserve the policy LDS tile");
  hipLaunchKernelGGL(ackppo_bootstrap_kernel, dim3((n_env + PT_ENVS - 1) / PT_ENVS), dim3(PT_THREADS),
                     sizeof(PolicyLds), (hipStream_t)stream, params, terminal_obs_soa, reward, term, trunc, n_env,
                     gamma, reward_out, done_out);
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

int ackppo_adv_stats(const float* advantages, const int32_t* idx, int n_idx, int batch, int normalize, float* stats,
                     void* stream) {
  if (!advantages || !idx || !stats || n_idx < 0 || batch <= 0) return fail(ACKPPO_EINVAL, "ackppo_adv_stats: bad arguments");
  const int nmb = (n_idx + batch - 1) / batch;
  if (nmb == 0) return ACKPPO_OK;
  hipLaunchKernelGGL(ackppo_adv_stats_kernel, dim3(nmb), dim3(256), 0, (hipStream_t)stream, advantages, idx, n_idx,
                     batch, normalize, stats);
  return launched("ackppo_adv_stats");
}

int ackppo_grad(const float* params, const float* obs_rows, const float* actions, const float* old_log_prob,
                const float* advantages, const float* returns, const int32_t* idx, int batch, const float* stats,
                float clip_range, float ent_coef, float vf_coef, float* grad_partial, float* loss_partial,
                void* stream) {
  if (!params || !obs_rows || !actions || !old_log_prob || !advantages || !returns || !idx || !stats ||
      !grad_partial || !loss_partial || batch <= 0)
    return fail(ACKPPO_EINVAL, "ackppo_grad: bad arguments");
  if (!g_grad_attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)ackppo_grad_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRAD_LDS);
    if (e != hipSuccess) return fail(ACKPPO_EHIP, "ackppo_grad: cannot reserve the 159 KiB LDS tile");
    g_grad_attr = true;
  }
  GradArgs A{params, obs_rows, actions, old_log_prob, advantages, returns, idx, batch, stats, clip_range, ent_coef,
             vf_coef, grad_partial, loss_partial};
  hipLaunchKernelGGL(ackppo_grad_kernel, dim3((batch + TILE - 1) / TILE), dim3(GRAD_THREADS), GRAD_LDS,
                     (hipStream_t)stream, A);
  return launched("ackppo_grad");
}

int ackppo_reduce(const float* grad_partial, const float* loss_partial, int nblk, float ent_coef, float* grad,
                  float* loss, void* stream) {
  if (!grad_partial || !loss_partial || !grad || !loss || nblk <= 0) return fail(ACKPPO_EINVAL, "ackppo_reduce: bad arguments");
  hipLaunchKernelGGL(ackppo_reduce_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, grad_partial,
                     loss_partial, nblk, ent_coef, grad, loss);
  return launched("ackppo_reduce");
}

int ackppo_adam(float* params, const float* grad, float* exp_avg, float* exp_avg_sq, float grad_scale,
                float max_grad_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt,
                float* grad_norm_out, void* stream) {
  if (!params || !grad || !exp_avg || !exp_avg_sq) return fail(ACKPPO_EINVAL, "ackppo_adam: bad arguments");
  hipLaunchKernelGGL(ackppo_adam_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, params, grad,
                     exp_avg, exp_avg_sq, grad_scale, max_grad_norm, beta1, beta2, eps, step_size, bc2_sqrt,
                     grad_norm_out);
  return launched("ackppo_adam");
}

}  // extern "C"
