// ackphys_step.hip -- MI355X (gfx950) batched physics step for ackermann_robot_v2.
//
// One wavefront lane per environment. Each lane runs the whole reference step for its env
// (src/rl/envs/ackermann_env.py:187-229):
//   controller (f64, src/core/controller.py:98-140) -> checkPos/Vel -> kinematics -> lidar /
//   odometry / obs / reward (pre-integration, ackermann_env.py:231-312) -> composite inertia +
//   Newton-Euler bias in CHASSIS-FRAME coordinates -> passive + actuators -> plane-cylinder and
//   plane-convex contacts -> equality / friction-loss / limit / pyramidal-contact rows ->
//   primal Newton solve (exact piecewise-quadratic line search) -> implicit-damping Euler ->
//   auto-reset with Philox goals (ackermann_env.py:143-185).
//
// Layout: state/obs are SoA [word][N] so every global access is lane-contiguous (coalesced);
// actions are AoS [N][2] (8 B per lane, also contiguous). Per-contact-slot scratch lives in
// LDS as [slot][field][lane] (bank-conflict-free, wave-uniform slot loops).
//
// Coordinates: u = (v_b, w_b, qdot_hinges) with v_b = R^T v_world. In u every CoM is fixed in
// the chassis frame and every wheel/steer inertia is isotropic (checked by codegen.py), so the
// 12x12 mass matrix is constant except the two front spin-axis couplings. The constraint
// problem is the same convex program as MuJoCo's (cost is invariant under u = T q, T orthogonal).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ackphys_model_gen.h"
#include "ackphys_scene_gen.h"

// Diagnostic build only (-DAK_STAMPS): per-wave s_memtime phase stamps, never in the product.
#ifdef AK_STAMPS
// layout: [AK_NSTAMP][blocks] phase stamps, [blocks][64] Newton iteration counts, [5][blocks] Newton phases
#define AK_NSTAMP 24
__device__ unsigned long long* g_stamps;
// slot dump of env 0 (quad kernels; tools/probes/quad_slot_probe.py): [4 lanes][QSN_MAX][AK_SLOTF]
// then qacc_smooth[12], qacc[12]
#define AK_SLOTF 40
#define AK_QSN_MAX 12
__device__ float* g_dump;
// The stamps are kept in LDS (one row per wave) and written out when the wave leaves its role
// function: a global store per stamp would add a pointer load and a vmcnt(0) wait to every stamp.
__shared__ unsigned long long ak_stamp_lds[4][AK_NSTAMP];
#define STAMP(k)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    unsigned long long _t;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");          \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    if ((threadIdx.x & 63) == 0) ak_stamp_lds[threadIdx.x >> 6][k] = _t;                  \
  } while (0)
struct StampScope {
  bool on;
  // four-wave workgroups (the fused PPO rollout: dynamics waves 0-1, observation waves 2-3) flush
  // waves 0 and 2 only: the stamp rows are per workgroup
  __device__ explicit StampScope(bool on_ = true) : on(on_ && !(blockDim.x == 256 && ((threadIdx.x >> 6) & 1))) {
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < AK_NSTAMP; k++) ak_stamp_lds[threadIdx.x >> 6][k] = 0;
  }
  __device__ ~StampScope() {
    if (on && (threadIdx.x & 63) == 0)
      for (int k = 0; k < AK_NSTAMP; k++)
        if (const unsigned long long v = ak_stamp_lds[threadIdx.x >> 6][k]) g_stamps[(size_t)k * gridDim.x + blockIdx.x] = v;
  }
};
#define STAMP_SCOPE StampScope _stamp_scope;
// loop-top clocks of the multi-step kernels (tools/probes/step_clock.py): rows AK_NSTAMP + 69 .. 72 hold
// the shader clock and the 100 MHz real-time counter at the loop top of the first and the last step
// (thread 0 of each workgroup)
#define LOOP_CLOCK(k, last)                                                                              \
  do {                                                                                                   \
    if (((k) == 0 || (k) == (last)) && threadIdx.x == 0) {                                               \
      unsigned long long _c, _r;                                                                         \
      asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(_c), "=s"(_r)::"memory"); \
      const size_t _o = (k) == 0 ? 0 : 2;                                                                \
      g_stamps[(AK_NSTAMP + 69 + _o) * (size_t)gridDim.x + blockIdx.x] = _c;                             \
      g_stamps[(AK_NSTAMP + 70 + _o) * (size_t)gridDim.x + blockIdx.x] = _r;                             \
    }                                                                                                    \
  } while (0)
// per-step roles of a multi-step kernel: flushed unless Args::stamp_skip (the PPO rollout keeps one step's)
#define STAMP_SCOPE_A(A) StampScope _stamp_scope(!(A).stamp_skip);
// Newton-phase accumulators (diag build): NT_MARK(ph) adds the cycles since the previous mark to phase ph
#define NT_DECL unsigned long long _nt_acc[5] = {0, 0, 0, 0, 0}, _nt_last = 0;
#define NT_NOW(v)                                                                \
  do {                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                           \
  } while (0)
#define NT_START NT_NOW(_nt_last)
#define NT_MARK(ph)                 \
  do {                              \
    unsigned long long _t;          \
    NT_NOW(_t);                     \
    _nt_acc[ph] += _t - _nt_last;   \
    _nt_last = _t;                  \
  } while (0)
#define NT_FLUSH                                                                                              \
  do {                                                                                                        \
    if ((threadIdx.x & 63) == 0)                                                                              \
      for (int _p = 0; _p < 5; _p++)                                                                          \
        g_stamps[(AK_NSTAMP + 64 + _p) * (size_t)gridDim.x + blockIdx.x] = _nt_acc[_p];                              \
  } while (0)
#else
#define NT_DECL
#define NT_START
#define NT_MARK(ph)
#define NT_FLUSH
#define STAMP_SCOPE
#define STAMP_SCOPE_A(A)
#define LOOP_CLOCK(k, last) \
  do {                      \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#endif

namespace ak {
using namespace apg;

constexpr int NV = 12;
constexpr int NSTATE = 44;
constexpr int NOBS = 79;
constexpr int ST_QPOS = 0, ST_QVEL = 13, ST_WARM = 25, ST_GOAL = 37, ST_REF = 39, ST_STEP = 42, ST_EPIS = 43;
constexpr uint32_t F_CONTACTS = 1u, F_AUTORESET = 2u, F_POSTSTEP_OBS = 4u;
constexpr int NSLOT = 24;        // 4 wheels x 4 + 2 meshes x 4 contact slots
constexpr int NF = 13;           // Pb[3], D, jar[4], jp[4], active
constexpr int NSCAL = 11;        // eq(1) + frictionloss(6) + limits(4)
constexpr int MAXIT = 12;        // Newton iterations cap (MuJoCo: 100; converges in 1-4 here)
constexpr int LSIT = 12;         // line-search iterations cap
constexpr float MINVAL = 1e-15f;

// env parameters: AckermannRobotEnv.__init__ kwargs (ackermann_env.py:51-60)
struct EnvParams {
  int max_episode_steps;
  float goal_distance_threshold, collision_threshold, max_linear_velocity, max_angular_velocity;
  // opt-in task variants (NOT the reference; default off = ackermann_env.py exactly): action_repeat
  // mj_steps per env step with the same ctrl (obs/reward at the last one's pre-integration pose),
  // nohit_clear: a rangefinder reading -1 (no hit) is no obstacle for the collision test
  int action_repeat = 1;
  int nohit_clear = 0;
  // goal_cells > 0 (obstacle scene only): goals at the centres of the spawn-connected free maze
  // cells within goal_cells breadth-first steps (scene1::FREE_XY / FREE_LE), not 2-8 m away
  int goal_cells = 0;
};
// the collision test's reading of one ray: with nohit_clear a -1 (no hit) reading is +inf
// the quad kernels compile the variant only into their VAR instantiations (the host launches those
// whenever a variant field is set); the lane kernels read the fields at run time
template <bool VAR>
__device__ __forceinline__ EnvParams var_prm(const EnvParams& p) {
  EnvParams r = p;
  if (!VAR) { r.action_repeat = 1; r.nohit_clear = 0; }
  return r;
}
__device__ __forceinline__ float coll_reading(float v, const EnvParams& prm) {
  return (prm.nohit_clear && v < 0.0f) ? 3.0e38f : v;
}
// min_lidar / collision from the minimum of the collision readings (ackermann_env.py:279-284)
__device__ __forceinline__ void coll_result(float minl, const EnvParams& prm, float& min_lidar, bool& coll) {
  coll = minl < prm.collision_threshold;
  min_lidar = (prm.nohit_clear && minl >= 3.0e38f) ? -1.0f : minl;
}

struct Args {
  const float* action;
  float* state;
  float* obs;
  float* reward;
  uint8_t* term;
  uint8_t* trunc;
  float* tobs;
  float* info;
  float* ep;  // [4][N] running return, running length, completed-return sum, completed episodes
  EnvParams prm;
  int n;
  uint32_t flags;
  uint64_t seed;
  int64_t env_offset;
  int epw;  // lane kernel: envs per 64-lane wave (lanes >= epw idle)
  int ksteps = 1;    // rollout kernels: consecutive steps per launch (action k at action + 2kN)
  int per_step = 0;  // rollout kernels: step k's outputs in slice k of obs/reward/term/trunc/tobs/info
  // lane rollout kernels: LDS mirror of the state words ([NSTATE][64 PW]) between the steps of a
  // launch: sm_in = this step reads its state there (not HBM), sm_out = the dynamics wave leaves
  // the post-step state there instead of storing it (every step but the launch's last)
  float* sm = nullptr;       // the mirror this step reads (sm_in)
  float* sm_next = nullptr;  // the mirror the next step reads, written by this step (sm_out); double
                             // buffered, so the dynamics wave can write it before barrier 1
  int sm_in = 0, sm_out = 0;
  // contacts-off rollout kernel: the prep wave computes step k + 1's controller output (a function of
  // the action alone) during step k from next_action into nctrl (LDS [3][64]); read when sm_in
  const float* next_action = nullptr;
  float* nctrl = nullptr;
  // quad rollout kernels: where step k's observation wave writes step k + 1's controller output
  // (the other half of a step-parity double buffer, so it can be written before barrier 1)
  float* nctrl_out = nullptr;
#ifdef AK_STAMPS
  int stamp_skip = 0;  // diagnostic build: this role call's stamps are not flushed
#endif
};

// Args of step k of a rollout launch: the k-th action row and, with per_step, the k-th output slices
__device__ __forceinline__ Args step_args(const Args& A, int k) {
  Args B = A;
  const size_t n = (size_t)A.n, kk = (size_t)k;
  B.action = A.action + kk * 2 * n;
  if (A.per_step) {
    B.obs = A.obs + kk * NOBS * n;
    B.reward = A.reward + kk * n;
    B.term = A.term + kk * n;
    B.trunc = A.trunc + kk * n;
    if (A.tobs) B.tobs = A.tobs + kk * NOBS * n;
    if (A.info) B.info = A.info + kk * 4 * n;
  }
  return B;
}

// ------------------------------------------------------------------ SoA buffer access
// Every per-env array is [rows][n] (or [n] / [n][2]). Accesses go through a buffer descriptor
// (SGPRs) with ONE per-lane byte offset (4e) and a scalar row offset (4kn): no per-lane 64-bit
// address per word, which the compiler otherwise hoists to the kernel start and keeps alive (spilled)
// until the stores at the end. Out-of-range / NULL (num_records 0) accesses are dropped by hardware.
struct Soa {
  __amdgpu_buffer_rsrc_t r;
  uint32_t row;  // bytes per row
};
__device__ __forceinline__ Soa soa(const void* base, uint32_t rows, uint32_t n, uint32_t esize = 4) {
  Soa b;
  b.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, base ? (int)(rows * n * esize) : 0,
                                          0x00020000);
  b.row = n * esize;
  return b;
}
__device__ __forceinline__ float ldf(const Soa& b, int k, uint32_t vo) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, vo, k * b.row, 0));
}
__device__ __forceinline__ void stf(const Soa& b, int k, uint32_t vo, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), b.r, vo, k * b.row, 0);
}
__device__ __forceinline__ void stb(const Soa& b, uint32_t vo_byte, uint8_t v) {
  __builtin_amdgcn_raw_buffer_store_b8(v, b.r, vo_byte, 0, 0);
}
// row index that differs between lanes (quad kernel: each lane owns different rays): fold the
// row offset into the per-lane VGPR offset so the scalar offset stays uniform (no waterfall)
__device__ __forceinline__ void stf_lane_row(const Soa& b, int k, uint32_t vo, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), b.r, vo + (uint32_t)k * b.row, 0, 0);
}

// terminal observation of auto-resetting lanes: copy the 79 words this lane just wrote to `obs`
// into `tobs` (before the reset overwrites them). The common step never enters this (wave-uniform
// test), so the observation stores stay single, unconditional and uniform-descriptor.
__device__ __forceinline__ void copy_terminal_obs(const Soa& obs, const Soa& tobs, uint32_t vo, bool mine) {
  if (__builtin_amdgcn_ballot_w64(mine) == 0ull) return;
  __builtin_amdgcn_s_waitcnt(0);  // this lane's obs stores have landed
  __threadfence();
  if (mine) {
#pragma unroll 8
    for (int k = 0; k < NOBS; k++) stf(tobs, k, vo, ldf(obs, k, vo));
  }
}

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ float sq(float x) { return x * x; }
__device__ __forceinline__ void cross(float r[3], const float a[3], const float b[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ float dot(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ bool is_bad(float x) { return !(fabsf(x) <= 1e10f); }  // NaN or huge

// Reciprocal / division / square-root helpers (and the Cholesky pivots): the hardware 1-ulp
// v_rcp / v_rsq / v_sqrt forms. With SLP vectorisation on they made the register allocation worse
// (36.7 -> 37.9 us/step contacts off); in the no-SLP build they measure faster (nc kernel 9.05 ->
// 8.75 us, contacts on 69.2 -> 68.7 us; tools/variant_sweep.sh) and every parity test holds.
// An argument that is a compile-time constant once inlined (model constants: the constant blocks
// of the mass matrix and of its factors, impedance and regulariser terms) takes the correctly
// rounded form, which the compiler folds; the hardware builtins are opaque to constant folding and
// otherwise run (or, in a rollout kernel's step loop, are hoisted and held in registers) per step.
#define AK_HW_OR_FOLD(x, folded, hw) (__builtin_constant_p(x) ? (folded) : (hw))
__device__ __forceinline__ float frcp(float x) { return AK_HW_OR_FOLD(x, 1.0f / x, __builtin_amdgcn_rcpf(x)); }
__device__ __forceinline__ float fdiv(float a, float b) {
  return AK_HW_OR_FOLD(b, a * (1.0f / b), a * __builtin_amdgcn_rcpf(b));
}
__device__ __forceinline__ float frsq(float x) { return AK_HW_OR_FOLD(x, 1.0f / sqrtf(x), __builtin_amdgcn_rsqf(x)); }
__device__ __forceinline__ float fsqrt(float x) { return AK_HW_OR_FOLD(x, sqrtf(x), __builtin_amdgcn_sqrtf(x)); }
#define AK_PIVOT_RSQ(x) frsq(x)
// sin / cos: the kernels' arguments are steer angles (|x| < ~0.7) and half rotation angles of one
// step (|x| << 1), so when every lane's |x| <= pi/4 the wave takes the Cephes minimax polynomials of
// that interval (the ones sincosf itself uses after its range reduction); otherwise sincosf.
__device__ __forceinline__ void fsincos(float x, float& s, float& c) {
  if (__builtin_amdgcn_ballot_w64(!(fabsf(x) <= 0.785398163f)) == 0ull) {
    const float z = x * x;
    s = fmaf(x * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), x);
    c = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
             fmaf(-0.5f, z, 1.0f));
    return;
  }
  sincosf(x, &s, &c);
}
// wrap to [-pi, pi] (atan2(sin a, cos a) of the reference) for |a| <= 3 pi
__device__ __forceinline__ float wrap_pi(float a) {
  return fmaf(__builtin_rintf(a * 0.159154943091895336f), -6.28318530717958648f, a);
}

// Philox4x32-10 (Random123); identical to oracle/ackphys_oracle.c
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// ------------------------------------------------------------------ controller (f64)
// BicycleController.cmd_vel_to_controls + apply_cmd_vel, controller.py:98-140, evaluated in
// float64 exactly like the reference (its thresholds 1e-6 / 1e-5 sit on f64 values).
template <bool BF = false>  // BF: branch-free form (same values), chosen per kernel by measurement
__device__ __forceinline__ void controller(float a0f, float a1f, float max_lin, float max_ang, float ctrl[3], bool& bad) {
  // np.clip on the float32 action, then action * max_velocity: float32 x Python float stays
  // float32 under NumPy 2 promotion (ackermann_env.py:190-194); controller works in float64.
  // Restated without the f64 atan/tan round trip: with y = L om / den, delta = clip(atan(y), +-35 deg)
  // and tan(delta) = y inside the clip (tan(35 deg) outside), |delta| < 1e-6 <=> |y| < 1e-6 (to 3e-19),
  // R = L / tan(delta) is finite (|R| > 0.28 > eps) unless |tan(delta)| <= eps -- the reference's
  // 0 * inf = NaN path, which zeroes ctrl -- so v (R -+ T/2) / R = v (1 -+ tan(delta) T / 2L).
  a0f = a0f < -1.0f ? -1.0f : (a0f > 1.0f ? 1.0f : a0f);
  a1f = a1f < -1.0f ? -1.0f : (a1f > 1.0f ? 1.0f : a1f);
  const double L = 0.20, T = 0.174, rw = 0.0325, eps = 1e-5;
  const double TAN_LIM = 0.70020753820970977;  // tan(35 deg) (controller.py:112)
  const double v = (double)(a0f * max_lin), om = (double)(a1f * max_ang);
  double y = 0.0, vl = v, vr = v;
  if constexpr (BF) {
    // both sides evaluated and selected (no basic-block boundaries, so the scheduler can interleave
    // the f64 chain with the kinematics); a zero denominator only arises when om == 0, whose y is 0.
    // Measured: contacts-on quad kernel 68.2 -> 66.5 us; the obstacle kernel 73.8 -> 74.9 us and
    // the lane kernels even, so only the flat-scene quad kernel uses it.
    const double den = fabs(v) > eps ? v : (double)((om > 0) - (om < 0)) * eps;
    y = fabs(om) < 1e-6 ? 0.0 : (L * om) / den;
    const double t = fabs(y) > TAN_LIM ? copysign(TAN_LIM, y) : y;
    const double k = fabs(t) > eps ? t * (T / (2.0 * L)) : __builtin_nan("");
    const bool straight = fabs(y) < 1e-6;
    vl = straight ? v : v * (1.0 - k);
    vr = straight ? v : v * (1.0 + k);
  } else {
    if (!(fabs(om) < 1e-6)) {
      const double den = fabs(v) > eps ? v : (double)((om > 0) - (om < 0)) * eps;
      y = (L * om) / den;
    }
    if (!(fabs(y) < 1e-6)) {
      const double t = fabs(y) > TAN_LIM ? copysign(TAN_LIM, y) : y;
      const double k = fabs(t) > eps ? t * (T / (2.0 * L)) : __builtin_nan("");
      vl = v * (1.0 - k);
      vr = v * (1.0 + k);
    }
  }
  const double wl = vl * (1.0 / rw), wr = vr * (1.0 / rw);
  const float c0 = fminf(fmaxf(atanf((float)y), -0.61f), 0.61f);  // clip(delta, +-0.61)
  double c1 = (wl != wl) ? wl : (wl < -50 ? -50 : (wl > 50 ? 50 : wl));
  double c2 = (wr != wr) ? wr : (wr < -50 ? -50 : (wr > 50 ? 50 : wr));
  bad = (c0 != c0) || !(fabs(c1) <= 1e10) || !(fabs(c2) <= 1e10);
  ctrl[0] = bad ? 0.0f : c0; ctrl[1] = bad ? 0.0f : (float)c1; ctrl[2] = bad ? 0.0f : (float)c2;  // MuJoCo zeroes bad ctrl
}

// ------------------------------------------------------------------ kinematics
__device__ __forceinline__ void quat_R(const float q[4], float R[9]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
__device__ __forceinline__ void normq(float q[4]) {
  float n = fsqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else { float inv = frcp(n); q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv; }
}
// rotate v about unit axis s by angle (Rodrigues): the steer rotation of front-wheel frames
__device__ __forceinline__ void rot_axis(float r[3], const float s[3], const float v[3], float c, float sn) {
  float sxv[3];
  cross(sxv, s, v);
  float sv = dot(s, v) * (1 - c);
#pragma unroll
  for (int k = 0; k < 3; k++) r[k] = v[k] * c + sxv[k] * sn + s[k] * sv;
}

// ------------------------------------------------------------------ observation + reward
// _get_observation / _calculate_reward (ackermann_env.py:231-312) on the PRE-integration pose
// (mj_step's sensors and xpos/xquat come from its mj_forward). Lidar: rays are horizontal in
// the chassis frame at RAY_Z and every robot geom lies below that plane (codegen.py proves it),
// so only the floor can be hit: mj_ray's plane test with the 40x40 rectangle, cutoff clamp.
struct ObsOut { float minl, dist, reward; bool term, coll; };

__device__ __forceinline__ ObsOut observe_head(const float p[3], const float q[4], const float R[9], float gx, float gy,
                               const float ref[3], float out8[7], const EnvParams& prm) {
  // odometry (odometry.py:62-103, 154-170)
  float x = p[0] - ref[0], y = p[1] - ref[1];
  float yaw = atan2f(2 * (q[0] * q[3] + q[1] * q[2]), 1 - 2 * (q[2] * q[2] + q[3] * q[3]));
  float dx = gx - x, dy = gy - y;
  float dist = sqrtf(dx * dx + dy * dy);
  float ang = atan2f(dy, dx) - yaw;
  ang = wrap_pi(ang);
  out8[0] = x; out8[1] = y; out8[2] = yaw; out8[3] = dx; out8[4] = dy; out8[5] = dist; out8[6] = ang;
  ObsOut o;
  o.dist = dist;
  o.term = dist < prm.goal_distance_threshold;
  return o;
}

// Every rangefinder site sits at RAY_R * (its direction) + RAY_Z e_z in the chassis frame (sites at
// R_z(5i deg) (r, 0, 0), rays along the site x-axis: ackermann_robot_v2.xml:83-86), so a ray's world
// origin is the pose constant (cx, cy, c0) plus RAY_R times its world direction: per ray, three
// two-term dot products instead of six three-term ones.
constexpr float RAY_R = RAY_ORG[0][0];
constexpr bool rays_radial() {
  for (int i = 0; i < 72; i++) {
    const float ex = RAY_ORG[i][0] - RAY_R * RAY_DIR[i][0], ey = RAY_ORG[i][1] - RAY_R * RAY_DIR[i][1];
    if (ex > 1e-8f || ex < -1e-8f || ey > 1e-8f || ey < -1e-8f) return false;
  }
  return RAY_DIR[0][0] == 1.0f && RAY_DIR[0][1] == 0.0f;
}
static_assert(rays_radial(), "rangefinder sites must lie on a circle around the z axis, rays pointing outwards");
struct RayFrame {
  float cx, cy, c0;  // world position of the ring centre at RAY_Z
  float r0, r1, r3, r4, r6, r7;  // the chassis rotation's columns x, y
};
__device__ __forceinline__ RayFrame ray_frame(const float p[3], const float R[9]) {
  return RayFrame{p[0] + R[2] * RAY_Z, p[1] + R[5] * RAY_Z, p[2] + R[8] * RAY_Z, R[0], R[1], R[3], R[4], R[6], R[7]};
}
// chassis-frame direction (dxb, dyb, 0) -> mj_ray's plane test against the finite floor rectangle;
// distance from the site (t), clamped to the cutoff, -1 for no hit. The site sits RAY_R out along
// the ray from the ring centre C, so the plane is met sd = -C_z / d_z from C and t = sd - RAY_R
// from the site. The hit test combines its terms with a non-short-circuit &: with && the compiler
// sank the hit-point arithmetic under a per-ray branch (32 s_cbranch per 32 rays, ~27 VALU per ray
// when the rays can hit); this form is branch-free at ~16 VALU per ray (tools: a 32-ray kernel
// compiled both ways, 1009 -> 639 VALU).
__device__ __forceinline__ float ray_floor_f(const RayFrame& F, float dxb, float dyb) {
  const float dz = F.r6 * dxb + F.r7 * dyb;
  const float ux = F.r0 * dxb + F.r1 * dyb, uy = F.r3 * dxb + F.r4 * dyb;
  const float sd = -F.c0 * __builtin_amdgcn_rcpf(dz);  // hardware reciprocal: 1 ulp, within the obs parity
  const float hx = fmaf(sd, ux, F.cx), hy = fmaf(sd, uy, F.cy);
  const float t = sd - RAY_R;
  bool inside;
  if constexpr (FLOOR_SIZE[0] == FLOOR_SIZE[1]) inside = fmaxf(fabsf(hx), fabsf(hy)) <= FLOOR_SIZE[0];
  else inside = (fabsf(hx) <= FLOOR_SIZE[0]) & (fabsf(hy) <= FLOOR_SIZE[1]);
  const bool hit = (dz <= -MINVAL) & (t >= 0.0f) & inside;
  return hit ? fminf(t, RAY_CUTOFF) : -1.0f;
}
// The ring's bounding test (mj_ray culls geoms by their extent before the exact test; this culls
// the 72 floor tests at once, and is exact: it only reports "every ray misses" when every ray's own
// test above returns -1). All rays lie in the chassis plane z = RAY_Z, so a ray's world direction d
// has |d_z| <= A = |(R20, R21)| and |d_xy| >= sqrt(1 - A^2). Ring below the floor (centre height
// C_z < 0): a downward ray starts at C_z + RAY_R d_z < 0 and meets the plane behind it (t < 0); an
// upward one fails d_z <= -MINVAL. Ring above: a downward ray meets the plane at s = C_z / |d_z| >=
// C_z / A from the centre, horizontally s |d_xy| from the centre's foot point, which must be within
// |C_xy| + |FLOOR_SIZE| for a hit on the floor rectangle. The margins (1e-4 relative below, 0.2 %
// and 1 m above) dwarf the f32 rounding of the per-ray tests; the transition band is cast in full.
// Why it matters: on the flat floor most readings are -1 (a level robot's rays never reach the
// floor within its 40 m extent), and casting 62 rays is ~2.3k of the observation waves' cycles.
__device__ __forceinline__ bool floor_rays_all_miss(const float p[3], const float R[9]) {
  const float cz = p[2] + R[8] * RAY_Z;
  if (cz < -1e-4f * (1.0f + fabsf(p[2]))) return true;
  const float a2 = R[6] * R[6] + R[7] * R[7];
  const float reach = fabsf(p[0] + R[2] * RAY_Z) + fabsf(p[1] + R[5] * RAY_Z) +
                      sqrtf(FLOOR_SIZE[0] * FLOOR_SIZE[0] + FLOOR_SIZE[1] * FLOOR_SIZE[1]) + 1.0f;
  return cz > 0.0f && cz * cz * (1.0f - a2) > 1.002f * a2 * reach * reach;
}

// ------------------------------------------------------------------ impedance / reference
// x^p: small integer powers (solimp's default power 2 in both models) as products -- powf is the
// device library's general routine (~150 instructions, not folded for a constant exponent)
__device__ __forceinline__ float fpow(float x, float p) {
  if (p == 1.0f) return x;
  if (p == 2.0f) return x * x;
  if (p == 3.0f) return x * x * x;
  return powf(x, p);
}
__device__ __forceinline__ float impedance_p(float pos, float d0, float dmax, float width, float mid, float pw) {
  // getimpedance: solimp (d0, dmax, width, mid, power), margin 0
  float x = fabsf(pos) * (1.0f / width);
  if (x >= 1.0f) return dmax;
  float y;
  if (pw == 1.0f) y = x;
  else if (x <= mid) y = fpow(x, pw) / fpow(mid, pw - 1.0f);
  else y = 1.0f - fpow(1.0f - x, pw) / fpow(1.0f - mid, pw - 1.0f);
  float imp = d0 + y * (dmax - d0);
  return fminf(fmaxf(imp, 0.0001f), 0.9999f);
}
// joint / dof / equality rows
__device__ __forceinline__ float impedance(float pos) {
  return impedance_p(pos, SOLIMP[0], SOLIMP[1], SOLIMP[2], SOLIMP[3], SOLIMP[4]);
}
// K, B from solref (refsafe: timeconst >= 2*dt)
__device__ __forceinline__ void ref_kb_p(float sr0, float sr1, float dmax, float& K, float& B) {
  const float tc = sr0 > 2.0f * DT ? sr0 : 2.0f * DT;
  const float dr = sr1;
  K = frcp(dmax * dmax * tc * tc * dr * dr);
  B = fdiv(2.0f, dmax * tc);
}
__device__ __forceinline__ void ref_kb(float& K, float& B) { ref_kb_p(SOLREF[0], SOLREF[1], SOLIMP[1], K, B); }

#include "ackphys_scene.inc"

// writes the 79 observation words of one env to dst (stride n); returns reward/term/etc.
struct NoPreMin {
  __device__ __forceinline__ float operator()() const { return 3.0e38f; }
};
// RFIRST > 10: rays 10 .. RFIRST-1 were cast (and stored) by another wave, whose minimum reading
// `premin()` returns once it is available
template <int SC, int RFIRST = 10, class PreMin = NoPreMin>
__device__ __forceinline__ ObsOut observe(const float p[3], const float q[4], const float R[9], float gx, float gy,
                          const float ref[3], const Soa& dst, uint32_t vo, const EnvParams& prm,
                          const PreMin& premin = PreMin{}) {
  float head[7];
  ObsOut o = observe_head(p, q, R, gx, gy, ref, head, prm);
  STAMP(11);
  // rays 10..71 are observed; obs[0:10] alias sensordata[76] = ray 71 (name-lookup aliasing,
  // ackermann_env.py:131-141); the min over the 72 aliased readings is the min over rays 10..71.
  float minl = 3.0e38f, v71 = -1.0f;
  const RayFrame F = ray_frame(p, R);
  if (SC == 0 && __builtin_amdgcn_ballot_w64(!floor_rays_all_miss(p, R)) == 0ull) {
#pragma unroll
    for (int i = RFIRST; i < 72; i++) stf(dst, i, vo, -1.0f);
    minl = coll_reading(-1.0f, prm);
  } else {
#pragma unroll
    for (int i = RFIRST; i < 72; i++) {
      float v;
      if constexpr (SC == 0) v = ray_floor_f(F, RAY_DIR[i][0], RAY_DIR[i][1]);
      else v = ray_scene<SC>(F, RAY_DIR[i][0], RAY_DIR[i][1]);
      stf(dst, i, vo, v);
      minl = fminf(minl, coll_reading(v, prm));
      v71 = v;
    }
  }
  STAMP(12);
#pragma unroll
  for (int i = 0; i < 10; i++) stf(dst, i, vo, v71);
#pragma unroll
  for (int k = 0; k < 7; k++) stf(dst, 72 + k, vo, head[k]);
  if constexpr (RFIRST > 10) minl = fminf(minl, premin());
  coll_result(minl, prm, o.minl, o.coll);
  float r = 0.0f;
  r -= o.dist * 0.1f;
  if (o.term) r += 100.0f;
  if (o.coll) r -= 50.0f;
  r -= 0.01f;
  o.reward = r;
  return o;
}

// ------------------------------------------------------------------ structured factorisation
// The Hessians of this model are sparse with a fixed structure: a hinge couples only to the free
// joint's dofs (wheel / steer inertia about the chassis; contact rows of its own wheel) and to the
// other hinge of its wheel (steer <-> spin) or the steer equality (steer L <-> steer R). With the
// hinges eliminated first (rear spins, front spins, front steers), then the free joint's linear and
// angular dofs, the Cholesky factor has no fill outside the 6x6 free-joint block. The patterns
// below are derived at compile time; skipped terms are structural zeros (0 * finite), so results
// equal the dense factorisation up to the reordering's rounding.
struct SymPat { bool nz[NV][NV]; };
// Every kernel factors structured (measured against the dense kind 3 in rounds 1-2: contacts on
// 69.3 vs 70.0 us per step, obstacles 73.9 vs 76.3 us; the lane kernel faster structured too).
constexpr int ORD[NV] = {W_SPIN_DOF[0], W_SPIN_DOF[1], W_SPIN_DOF[2], W_SPIN_DOF[3], W_STEER_DOF[2],
                         W_STEER_DOF[3], 0, 1, 2, 3, 4, 5};
static_assert(W_STEER_DOF[0] < 0 && W_STEER_DOF[1] < 0 && W_STEER_DOF[2] >= 6 && W_STEER_DOF[3] >= 6,
              "factorisation order assumes rear wheels without steering and two steered front wheels");
constexpr bool ord_is_perm() {
  bool seen[NV] = {};
  for (int i = 0; i < NV; i++) {
    if (ORD[i] < 0 || ORD[i] >= NV || seen[ORD[i]]) return false;
    seen[ORD[i]] = true;
  }
  return true;
}
static_assert(ord_is_perm(), "ORD must be a permutation of the dofs");
// kind 0: mass matrix (a0, implicit Euler); 1: + scalar rows (equality, friction loss, limits);
// 2: + contact rows (every wheel / plate contact couples the free joint and its wheel's hinges)
constexpr SymPat make_pat(int kind) {
  SymPat p{};
  auto set = [&p](int a, int b) { p.nz[a][b] = true; p.nz[b][a] = true; };
  for (int i = 0; i < NV; i++) set(i, i);
  for (int a = 3; a < 6; a++)
    for (int b = 0; b < 6; b++) set(a, b);  // I_O and m [c]x
  for (int w = 0; w < 4; w++) {
    for (int a = 3; a < 6; a++) {
      set(W_SPIN_DOF[w], a);
      if (W_STEER_DOF[w] >= 0) set(W_STEER_DOF[w], a);
    }
    if (W_STEER_DOF[w] >= 0) set(W_SPIN_DOF[w], W_STEER_DOF[w]);
  }
  if (kind >= 1) set(EQ_DOF1, EQ_DOF2);
  if (kind >= 2) {
    for (int a = 0; a < 6; a++)
      for (int b = 0; b < 6; b++) set(a, b);
    for (int w = 0; w < 4; w++)
      for (int a = 0; a < 6; a++) {
        set(W_SPIN_DOF[w], a);
        if (W_STEER_DOF[w] >= 0) set(W_STEER_DOF[w], a);
      }
  }
  return p;
}
// pattern of the factor in elimination order (lower triangle, with fill)
constexpr SymPat make_lpat(int kind) {
  const SymPat p = make_pat(kind);
  SymPat l{};
  for (int i = 0; i < NV; i++)
    for (int j = 0; j <= i; j++) l.nz[i][j] = p.nz[ORD[i]][ORD[j]];
  for (int k = 0; k < NV; k++)
    for (int i = k + 1; i < NV; i++)
      if (l.nz[i][k])
        for (int j = k + 1; j <= i; j++)
          if (l.nz[j][k]) l.nz[i][j] = true;
  return l;
}
constexpr SymPat PAT[3] = {make_pat(0), make_pat(1), make_pat(2)};
constexpr SymPat LPAT[3] = {make_lpat(0), make_lpat(1), make_lpat(2)};
constexpr bool no_fill(int kind) {  // the order creates no fill outside the free-joint block
  for (int i = 0; i < NV; i++)
    for (int j = 0; j < i; j++)
      if (LPAT[kind].nz[i][j] && !PAT[kind].nz[ORD[i]][ORD[j]] && (ORD[i] >= 6 || ORD[j] >= 6)) return false;
  return true;
}
static_assert(no_fill(0) && no_fill(1) && no_fill(2), "hinge-first order must not fill hinge rows");

// In-place structured Cholesky: entry (i, j) of the factor in elimination order is stored in the
// natural lower-triangle slot of dofs (ORD i, ORD j), the diagonal as 1/L_jj. H holds the lower
// triangle in natural order and is read only where PAT[KIND] is set (fill slots start from 0).
#define AK_F(A, i, j) A[ORD[i] > ORD[j] ? ORD[i] : ORD[j]][ORD[i] > ORD[j] ? ORD[j] : ORD[i]]
template <int KIND>
__device__ __forceinline__ void chol_sp(float H[NV][NV]) {
#pragma unroll
  for (int j = 0; j < NV; j++) {
    float s = AK_F(H, j, j);
#pragma unroll
    for (int k = 0; k < j; k++)
      if (LPAT[KIND].nz[j][k]) s -= AK_F(H, j, k) * AK_F(H, j, k);
    const float inv = AK_PIVOT_RSQ(fmaxf(s, 1e-30f));
    AK_F(H, j, j) = inv;
#pragma unroll
    for (int i = j + 1; i < NV; i++) {
      if (!LPAT[KIND].nz[i][j]) continue;
      float t = PAT[KIND].nz[ORD[i]][ORD[j]] ? AK_F(H, i, j) : 0.0f;
#pragma unroll
      for (int k = 0; k < j; k++)
        if (LPAT[KIND].nz[i][k] && LPAT[KIND].nz[j][k]) t -= AK_F(H, i, k) * AK_F(H, j, k);
      AK_F(H, i, j) = t * inv;
    }
  }
}
// x <- H^-1 x with H factored by chol_sp<KIND>; x in natural dof order
template <int KIND>
__device__ __forceinline__ void chol_sp_solve(const float H[NV][NV], float x[NV]) {
  float y[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) {
    float s = x[ORD[i]];
#pragma unroll
    for (int k = 0; k < i; k++)
      if (LPAT[KIND].nz[i][k]) s -= AK_F(H, i, k) * y[k];
    y[i] = s * AK_F(H, i, i);
  }
#pragma unroll
  for (int i = NV - 1; i >= 0; i--) {
    float s = y[i];
#pragma unroll
    for (int k = i + 1; k < NV; k++)
      if (LPAT[KIND].nz[k][i]) s -= AK_F(H, k, i) * y[k];
    y[i] = s * AK_F(H, i, i);
  }
#pragma unroll
  for (int i = 0; i < NV; i++) x[ORD[i]] = y[i];
}
// y = M x over the mass matrix's structural nonzeros (zero terms skipped, natural summation order).
// Entries that fold to a compile-time 0 (zero components of the model's constant axes and offsets)
// are skipped too: IEEE keeps 0 * x (x may be inf), so the compiler emitted those multiplies; for
// finite x a +-0 term never changes a sum that starts at +0.
template <int KIND = 0>
__device__ __forceinline__ void symv_M(const float M[NV][NV], const float x[NV], float y[NV]) {
#pragma unroll
  for (int i = 0; i < NV; i++) {
    float s = 0;
#pragma unroll
    for (int j = 0; j < NV; j++)
      if (PAT[KIND].nz[i][j]) {
        const float m = j <= i ? M[i][j] : M[j][i];
        if (!(__builtin_constant_p(m) && m == 0.0f)) s += m * x[j];
      }
    y[i] = s;
  }
}

// ------------------------------------------------------------------ mass matrix (u coords)
// Lower triangle. Constant except the front spin couplings (axis a(delta) in chassis frame).
__device__ __forceinline__ void build_M(float M[NV][NV], const float sa[2][3]) {
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int j = 0; j < NV; j++) M[i][j] = 0.0f;
  M[0][0] = M[1][1] = M[2][2] = M_TOT;
  // M_{w v} = m [c]x  (lower block rows 3..5, cols 0..2)
  const float cx = C_TOT[0], cy = C_TOT[1], cz = C_TOT[2];
  M[3][1] = -M_TOT * cz; M[3][2] = M_TOT * cy;
  M[4][0] = M_TOT * cz; M[4][2] = -M_TOT * cx;
  M[5][0] = -M_TOT * cy; M[5][1] = M_TOT * cx;
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b <= a; b++) M[3 + a][3 + b] = I_O[a][b];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const int ds = W_SPIN_DOF[w];
    if (W_STEER_DOF[w] < 0) {
#pragma unroll
      for (int k = 0; k < 3; k++) M[ds][3 + k] = W_I[w] * W_SPIN_AXIS[w][k];
      M[ds][ds] = W_I[w] + ARMATURE[ds];
    } else {
      const int st = W_STEER_DOF[w], s = w - 2;
#pragma unroll
      for (int k = 0; k < 3; k++) M[st][3 + k] = (S_I[s] + W_I[w]) * S_AXIS[s][k];
      M[st][st] = S_I[s] + W_I[w] + ARMATURE[st];
#pragma unroll
      for (int k = 0; k < 3; k++) M[ds][3 + k] = W_I[w] * sa[s][k];
      M[ds][st] = W_I[w] * dot(S_AXIS[s], sa[s]);
      M[ds][ds] = W_I[w] + ARMATURE[ds];
    }
  }
}

// ------------------------------------------------------------------ bias forces (RNE, u coords)
// qfrc_bias = Coriolis/centrifugal/gyroscopic + gravity, Newton-Euler per body in the chassis
// frame with zero generalised acceleration (MuJoCo mj_rne with flg_acc = 0).
__device__ __forceinline__ void bias(const float u[NV], const float R[9], const float sa[2][3], float b[NV]) {
  const float w[3] = {u[3], u[4], u[5]};
  // gravity in the chassis frame
  const float g[3] = {R[0] * GRAV[0] + R[3] * GRAV[1] + R[6] * GRAV[2], R[1] * GRAV[0] + R[4] * GRAV[1] + R[7] * GRAV[2],
                      R[2] * GRAV[0] + R[5] * GRAV[1] + R[8] * GRAV[2]};
#pragma unroll
  for (int i = 0; i < NV; i++) b[i] = 0.0f;
  // chassis group
  {
    float wxr[3], a[3], f[3], Iw[3], gy[3], rxf[3];
    cross(wxr, w, C_G);
    cross(a, w, wxr);
#pragma unroll
    for (int k = 0; k < 3; k++) f[k] = M_G * (a[k] - g[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) Iw[k] = I_G[k][0] * w[0] + I_G[k][1] * w[1] + I_G[k][2] * w[2];
    cross(gy, w, Iw);
    cross(rxf, C_G, f);
#pragma unroll
    for (int k = 0; k < 3; k++) { b[k] += f[k]; b[3 + k] += rxf[k] + gy[k]; }
  }
#pragma unroll
  for (int wi = 0; wi < 4; wi++) {
    const float* r = W_ANCHOR[wi];
    float wxr[3], a[3], f[3], rxf[3];
    cross(wxr, w, r);
    cross(a, w, wxr);
    const float ms = W_M[wi] + (W_STEER_DOF[wi] >= 0 ? S_M[wi - 2 < 0 ? 0 : wi - 2] : 0.0f);
#pragma unroll
    for (int k = 0; k < 3; k++) f[k] = ms * (a[k] - g[k]);
    cross(rxf, r, f);
    float tau[3];
    const int ds = W_SPIN_DOF[wi];
    if (W_STEER_DOF[wi] < 0) {
      // alpha = w x a qdot ; isotropic: no gyroscopic torque
      float wxa[3];
      cross(wxa, w, W_SPIN_AXIS[wi]);
#pragma unroll
      for (int k = 0; k < 3; k++) tau[k] = W_I[wi] * wxa[k] * u[ds];
      b[ds] += dot(W_SPIN_AXIS[wi], tau);
    } else {
      const int st = W_STEER_DOF[wi], s = wi - 2;
      const float* sax = S_AXIS[s];
      const float* ax = sa[s];
      float wxs[3], ws[3], wsxa[3];
      cross(wxs, w, sax);
#pragma unroll
      for (int k = 0; k < 3; k++) ws[k] = w[k] + sax[k] * u[st];
      cross(wsxa, ws, ax);
      float ts[3], tw[3];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        ts[k] = S_I[s] * wxs[k] * u[st];
        tw[k] = W_I[wi] * (wxs[k] * u[st] + wsxa[k] * u[ds]);
        tau[k] = ts[k] + tw[k];
      }
      b[st] += dot(sax, tau);
      b[ds] += dot(ax, tw);
    }
#pragma unroll
    for (int k = 0; k < 3; k++) { b[k] += f[k]; b[3 + k] += rxf[k] + tau[k]; }
  }
}

// ------------------------------------------------------------------ contact slots in LDS
struct Slots {
  float* base;     // [NSLOT][NF][64] for this block; lane offset applied
  uint32_t lmask;  // this lane's active contact slots
  uint32_t wmask;  // OR over the wave (uniform): loops visit only these slots
  __device__ __forceinline__ float& at(int s, int f) const { return base[(s * NF + f) * 64]; }
  __device__ __forceinline__ bool on(int s) const { return (lmask >> s) & 1u; }
};
// iterate the wave-uniform set bits of m (slot indices), skipping lanes where the slot is off
#define FOR_SLOTS(S, m, s)                  \
  for (uint32_t _m = (m); _m; _m &= _m - 1) \
    if (const int s = __builtin_ctz(_m); !(S).on(s)) { } else

// chain geometry: contact point P (chassis frame) -> jacobian rows G[dir][8] for the 3 frame
// directions; columns 0..5 = v_b, w_b; col 6/7 = chain hinge dofs (see dof6/dof7).
template <int CH>
struct Chain {
  static constexpr bool wheel = CH < 4;
  static constexpr bool front = CH == 2 || CH == 3;
  static constexpr int dof6 = !wheel ? -1 : (front ? W_STEER_DOF[CH] : W_SPIN_DOF[CH]);
  static constexpr int dof7 = front ? W_SPIN_DOF[CH] : -1;
};

template <int CH>
__device__ __forceinline__ void jac_rows(const float P[3], const float dirs[3][3], const float sa[2][3],
                                         float G[3][8]) {
  float c6[3] = {0, 0, 0}, c7[3] = {0, 0, 0};
  if constexpr (Chain<CH>::wheel) {
    float rel[3] = {P[0] - W_ANCHOR[CH][0], P[1] - W_ANCHOR[CH][1], P[2] - W_ANCHOR[CH][2]};
    if constexpr (Chain<CH>::front) {
      cross(c6, S_AXIS[CH - 2], rel);
      cross(c7, sa[CH - 2], rel);
    } else {
      cross(c6, W_SPIN_AXIS[CH], rel);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const float* db = dirs[d];
    float pxd[3];
    cross(pxd, P, db);
    G[d][0] = db[0]; G[d][1] = db[1]; G[d][2] = db[2];
    G[d][3] = pxd[0]; G[d][4] = pxd[1]; G[d][5] = pxd[2];
    G[d][6] = dot(c6, db);
    G[d][7] = dot(c7, db);
  }
}

template <int CH>
__device__ __forceinline__ float row_dot(const float J[8], const float x[NV]) {
  float s = J[0] * x[0] + J[1] * x[1] + J[2] * x[2] + J[3] * x[3] + J[4] * x[4] + J[5] * x[5];
  if constexpr (Chain<CH>::dof6 >= 0) s += J[6] * x[Chain<CH>::dof6];
  if constexpr (Chain<CH>::dof7 >= 0) s += J[7] * x[Chain<CH>::dof7];
  return s;
}
template <int CH>
__device__ __forceinline__ void row_axpy(const float J[8], float f, float g[NV]) {
#pragma unroll
  for (int k = 0; k < 6; k++) g[k] += f * J[k];
  if constexpr (Chain<CH>::dof6 >= 0) g[Chain<CH>::dof6] += f * J[6];
  if constexpr (Chain<CH>::dof7 >= 0) g[Chain<CH>::dof7] += f * J[7];
}
template <int CH>
__device__ __forceinline__ void row_outer(const float J[8], float Dv, float H[NV][NV]) {
  constexpr int idx[8] = {0, 1, 2, 3, 4, 5, Chain<CH>::dof6, Chain<CH>::dof7};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (idx[i] < 0) continue;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (idx[j] < 0 || idx[j] > idx[i]) continue;
      H[idx[i]][idx[j]] += Dv * J[i] * J[j];
    }
  }
}
__device__ __forceinline__ void pyr_row(const float G[3][8], int r, float mu, float J[8]) {
  // rows: (k=0,s=-1), (k=0,s=+1), (k=1,s=-1), (k=1,s=+1): J = Jn + s*mu*Jt_k
  const int k = 1 + (r >> 1);
  const float s = (r & 1) ? mu : -mu;
#pragma unroll
  for (int i = 0; i < 8; i++) J[i] = G[0][i] + s * G[k][i];
}

template <int CH>
__device__ __forceinline__ float chain_mu() {
  if constexpr (CH < 4) return MU_WHEEL;
  else return MESH_MU[CH - 4];
}

// scalar rows (single/two-dof jacobians): 0 eq, 1..6 friction loss on dofs 6..11, 7..10 limits
__device__ __forceinline__ void scal_dofs(int r, int& d1, float& c1, int& d2) {
  d2 = -1;
  if (r == 0) { d1 = EQ_DOF1; c1 = 1.0f; d2 = EQ_DOF2; }
  else if (r <= 6) { d1 = 5 + r; c1 = 1.0f; }
  else { d1 = LIM_DOF[(r - 7) >> 1]; c1 = ((r - 7) & 1) ? -1.0f : 1.0f; }
}

// ------------------------------------------------------------------ the per-env step
struct Solver {
  float M[NV][NV];           // mass matrix (lower)
  float a0[NV];              // qacc_smooth
  float fs[NV];              // qfrc_smooth
};

// row cost derivative bookkeeping for the line search
__device__ __forceinline__ void ls_row(float x, float jp, float D, int type, float Rfl, float fl, float& g, float& h) {
  if (type == 0) { g += D * x * jp; h += D * jp * jp; }
  else if (type == 1) {
    if (x <= -Rfl) g -= fl * jp;
    else if (x >= Rfl) g += fl * jp;
    else { g += D * x * jp; h += D * jp * jp; }
  } else if (x < 0.0f) { g += D * x * jp; h += D * jp * jp; }
}

// pairwise sum (independent adds: ILP for a lone wave, whose dependent VALU chain issues every 4+ cycles)
template <int N>
__device__ __forceinline__ float tsum(const float (&v)[N]) {
  float t[N];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = v[i];
#pragma unroll
  for (int w = 1; w < N; w *= 2)
#pragma unroll
    for (int i = 0; i + w < N; i += 2 * w) t[i] += t[i + w];
  return t[0];
}

// line-search derivative phi'(al) / phi''(al) contributions of the scalar rows (equality,
// frictionloss Huber, limits), branchless; only rows with (r & MASK) == sel (the quad kernel
// splits them over its 4 lanes)
template <int MASK>
__device__ __forceinline__ void scal_ls(float al, const float sj[NSCAL], const float sjp[NSCAL], const float sD[NSCAL],
                                        const float sRfl[NSCAL], const float sfl[NSCAL], const bool sact[NSCAL], int sel,
                                        float& g, float& h) {
  float gs[NSCAL], hs[NSCAL];
#pragma unroll
  for (int r = 0; r < NSCAL; r++) {
    const float jp = sjp[r], x = fmaf(al, jp, sj[r]);
    bool quad;
    float lin = 0.0f;
    if (r == 0) quad = true;
    else if (r <= 6) {
      quad = x > -sRfl[r] && x < sRfl[r];
      lin = x <= -sRfl[r] ? -sfl[r] : sfl[r];
    } else quad = x < 0.0f;
    const bool on = sact[r] && ((r & MASK) == sel);
    const float Djp = sD[r] * jp;
    gs[r] = on ? (quad ? Djp * x : lin * jp) : 0.0f;
    hs[r] = (on && quad) ? Djp * jp : 0.0f;
  }
  g += tsum(gs);
  h += tsum(hs);
}

// f32 noise scale of phi'(alpha) (sum of the magnitudes of its terms at alpha = 0): the line
// search accepts |phi'| below 1e-5 of it -- at the optimum the Newton direction is rounding
// noise and a purely relative test (1e-4 |phi'(0)|) can never be met
template <int MASK>
__device__ __forceinline__ float scal_noise(const float sj[NSCAL], const float sjp[NSCAL], const float sD[NSCAL],
                                            const float sRfl[NSCAL], const float sfl[NSCAL], const bool sact[NSCAL],
                                            int sel) {
  float t[NSCAL];
#pragma unroll
  for (int r = 0; r < NSCAL; r++) {
    const float x = sj[r], jp = sjp[r];
    bool quad;
    if (r == 0) quad = true;
    else if (r <= 6) quad = x > -sRfl[r] && x < sRfl[r];
    else quad = x < 0.0f;
    const bool on = sact[r] && ((r & MASK) == sel);
    const bool lin = r >= 1 && r <= 6 && !quad;
    t[r] = on ? (quad ? sD[r] * (fabsf(x * jp) + jp * jp) : (lin ? sfl[r] * fabsf(jp) : 0.0f)) : 0.0f;
  }
  return tsum(t);
}

template <int CH>
__device__ __forceinline__ void slot_loop_hess(const Slots& S, const float dirs[3][3], const float sa[2][3],
                                               float H[NV][NV], float grad[NV]) {
  constexpr int s0 = CH < 4 ? CH * 4 : 16 + (CH - 4) * 4;
  const float mu = chain_mu<CH>();
  FOR_SLOTS(S, S.wmask & (15u << s0), s) {
    float P[3] = {S.at(s, 0), S.at(s, 1), S.at(s, 2)};
    float D = S.at(s, 3);
    float G[3][8];
    jac_rows<CH>(P, dirs, sa, G);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float jar = S.at(s, 4 + r);
      if (jar < 0.0f) {
        float J[8];
        pyr_row(G, r, mu, J);
        row_outer<CH>(J, D, H);
        row_axpy<CH>(J, D * jar, grad);  // grad -= f J with f = -D jar
      }
    }
  }
}

template <int CH>
__device__ __forceinline__ void slot_loop_jp(const Slots& S, const float dirs[3][3], const float sa[2][3],
                                             const float p[NV]) {
  constexpr int s0 = CH < 4 ? CH * 4 : 16 + (CH - 4) * 4;
  const float mu = chain_mu<CH>();
  FOR_SLOTS(S, S.wmask & (15u << s0), s) {
    float P[3] = {S.at(s, 0), S.at(s, 1), S.at(s, 2)};
    float G[3][8];
    jac_rows<CH>(P, dirs, sa, G);
    float gn = row_dot<CH>(G[0], p), g1 = row_dot<CH>(G[1], p), g2 = row_dot<CH>(G[2], p);
    S.at(s, 8) = gn - mu * g1;
    S.at(s, 9) = gn + mu * g1;
    S.at(s, 10) = gn - mu * g2;
    S.at(s, 11) = gn + mu * g2;
  }
}

// jar init: jar = J a - aref, with aref = -B (J u) - K imp pos
template <int CH>
__device__ __forceinline__ void slot_loop_init(const Slots& S, const float dirs[3][3], const float sa[2][3],
                                               const float a[NV], const float u[NV], float K, float B) {
  constexpr int s0 = CH < 4 ? CH * 4 : 16 + (CH - 4) * 4;
  const float mu = chain_mu<CH>();
  FOR_SLOTS(S, S.wmask & (15u << s0), s) {
    float P[3] = {S.at(s, 0), S.at(s, 1), S.at(s, 2)};
    float dist = S.at(s, 3);  // holds dist until replaced by D
    float G[3][8];
    jac_rows<CH>(P, dirs, sa, G);
    float an = row_dot<CH>(G[0], a), a1 = row_dot<CH>(G[1], a), a2 = row_dot<CH>(G[2], a);
    float vn = row_dot<CH>(G[0], u), v1 = row_dot<CH>(G[1], u), v2 = row_dot<CH>(G[2], u);
    float imp = impedance(dist);
    float ja[4] = {an - mu * a1, an + mu * a1, an - mu * a2, an + mu * a2};
    float jv[4] = {vn - mu * v1, vn + mu * v1, vn - mu * v2, vn + mu * v2};
#pragma unroll
    for (int r = 0; r < 4; r++) S.at(s, 4 + r) = ja[r] + B * jv[r] + K * imp * dist;
    // pyramidal regulariser shared by the 4 edges:
    // R = (1-imp)/imp * tran*(1+mu^2) * 2 mu^2 / impratio   (see oracle make_constraint)
    float tran = CH < 4 ? W_TRAN[CH < 4 ? CH : 0] : MESH_TRAN[CH >= 4 ? CH - 4 : 0];
    float Rr = fmaxf(MINVAL, fdiv(1.0f - imp, imp) * tran * (1.0f + mu * mu) * (2.0f * mu * mu / IMPRATIO));
    S.at(s, 3) = frcp(Rr);
  }
}

// constraint force accumulation qfrc_c += J^T f at the current jar
template <int CH>
__device__ __forceinline__ void slot_loop_force(const Slots& S, const float dirs[3][3], const float sa[2][3],
                                                float fc[NV]) {
  constexpr int s0 = CH < 4 ? CH * 4 : 16 + (CH - 4) * 4;
  const float mu = chain_mu<CH>();
  FOR_SLOTS(S, S.wmask & (15u << s0), s) {
    float P[3] = {S.at(s, 0), S.at(s, 1), S.at(s, 2)};
    float D = S.at(s, 3);
    float G[3][8];
    jac_rows<CH>(P, dirs, sa, G);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float jar = S.at(s, 4 + r);
      if (jar < 0.0f) {
        float J[8];
        pyr_row(G, r, mu, J);
        row_axpy<CH>(J, -D * jar, fc);
      }
    }
  }
}


// plane-cylinder for wheel W: writes up to 4 slots (mjc_PlaneCylinder restatement)
template <int W>
__device__ __forceinline__ uint32_t wheel_contacts(const Slots& S, const float p[3], const float R[9], const float cyl_b[3]) {
  constexpr int s0 = W * 4;
  float c[3], axis[3];
  const float* an = W_ANCHOR[W];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c[k] = p[k] + R[3 * k] * an[0] + R[3 * k + 1] * an[1] + R[3 * k + 2] * an[2];
    axis[k] = R[3 * k] * cyl_b[0] + R[3 * k + 1] * cyl_b[1] + R[3 * k + 2] * cyl_b[2];
  }
  float prjaxis = axis[2];
  if (prjaxis > 0) { axis[0] = -axis[0]; axis[1] = -axis[1]; axis[2] = -axis[2]; prjaxis = -prjaxis; }
  float dist0 = c[2];
  float vec[3] = {axis[0] * prjaxis, axis[1] * prjaxis, axis[2] * prjaxis - 1.0f};
  float len2 = dot(vec, vec), prjvec;
  if (len2 >= MINVAL * MINVAL) {
    float sc = CYL_R * frsq(len2);
    vec[0] *= sc; vec[1] *= sc; vec[2] *= sc;
    prjvec = vec[2];
  } else {  // disk parallel to the plane (measure zero): any in-plane radius
    vec[0] = R[0] * CYL_R; vec[1] = R[3] * CYL_R; vec[2] = R[6] * CYL_R;
    prjvec = 0.0f;
  }
#pragma unroll
  for (int k = 0; k < 3; k++) axis[k] *= CYL_H;
  prjaxis *= CYL_H;
  float dpos[4][3], dd[4];
  bool act[4] = {false, false, false, false};
  float d1 = dist0 + prjaxis + prjvec;
  if (d1 <= 0.0f) {
    act[0] = true; dd[0] = d1;
#pragma unroll
    for (int k = 0; k < 3; k++) dpos[0][k] = c[k] + vec[k] + axis[k];
    float d2 = dist0 - prjaxis + prjvec;
    if (d2 <= 0.0f) {
      act[1] = true; dd[1] = d2;
#pragma unroll
      for (int k = 0; k < 3; k++) dpos[1][k] = c[k] + vec[k] - axis[k];
    }
    if (dist0 + prjaxis - prjvec <= 0.0f) {
      float v1[3];
      cross(v1, vec, axis);
      float nv1 = fsqrt(dot(v1, v1));
      float sc = nv1 < MINVAL ? 0.0f : CYL_R * 0.8660254037844386f * frcp(nv1);
      float d3 = dist0 + prjaxis - 0.5f * prjvec;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        float sg = t == 0 ? -1.0f : 1.0f;
        act[2 + t] = true; dd[2 + t] = d3;
#pragma unroll
        for (int k = 0; k < 3; k++) dpos[2 + t][k] = c[k] + axis[k] - 0.5f * vec[k] + sg * sc * v1[k];
      }
    }
  }
  uint32_t bits = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    // included in the constraint set only if dist < margin - gap = 0
    bool on = act[t] && dd[t] < 0.0f;
    if (on) {
      bits |= 1u << (s0 + t);
      // midpoint contact position, then chassis-frame point relative to the chassis origin
      float w[3] = {dpos[t][0] - p[0], dpos[t][1] - p[1], dpos[t][2] - 0.5f * dd[t] - p[2]};
      S.at(s0 + t, 0) = R[0] * w[0] + R[3] * w[1] + R[6] * w[2];
      S.at(s0 + t, 1) = R[1] * w[0] + R[4] * w[1] + R[7] * w[2];
      S.at(s0 + t, 2) = R[2] * w[0] + R[5] * w[1] + R[8] * w[2];
      S.at(s0 + t, 3) = dd[t];
    }
  }
  return bits;
}

// plane vs convex hull of welded mesh K: support vertex + up to 3 spread vertices
template <int K>
__device__ __forceinline__ uint32_t mesh_contacts(const Slots& S, const float p[3], const float R[9]) {
  constexpr int s0 = 16 + K * 4;
  // conservative lower bound on the hull's height (chassis-frame AABB)
  float zc = p[2], ext = 0.0f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    float cen = 0.5f * (HULL_LO[K][k] + HULL_HI[K][k]), half = 0.5f * (HULL_HI[K][k] - HULL_LO[K][k]);
    zc += R[6 + k] * cen;
    ext += fabsf(R[6 + k]) * half;
  }
  if (zc - ext > 0.0f) return 0;
  int best = 0;
  float bz = 3.0e38f;
  for (int i = 0; i < HULL_N[K]; i++) {
    float z = p[2] + R[6] * HULL[K][i][0] + R[7] * HULL[K][i][1] + R[8] * HULL[K][i][2];
    if (z < bz) { bz = z; best = i; }
  }
  if (bz > 0.0f) return 0;
  int sel[4] = {best, -1, -1, -1};
  int nsel = 1;
  for (int it = 0; it < 3; it++) {
    int pick = -1;
    float pickd = 1e-12f;
    for (int i = 0; i < HULL_N[K]; i++) {
      float z = p[2] + R[6] * HULL[K][i][0] + R[7] * HULL[K][i][1] + R[8] * HULL[K][i][2];
      if (z > 0.0f) continue;
      float dmin = 3.0e38f;
      for (int s = 0; s < nsel; s++) {
        float e0 = HULL[K][i][0] - HULL[K][sel[s]][0], e1 = HULL[K][i][1] - HULL[K][sel[s]][1],
              e2 = HULL[K][i][2] - HULL[K][sel[s]][2];
        dmin = fminf(dmin, e0 * e0 + e1 * e1 + e2 * e2);
      }
      if (dmin > pickd) { pickd = dmin; pick = i; }
    }
    if (pick < 0) break;
    sel[nsel++] = pick;
  }
  uint32_t bits = 0;
  for (int t = 0; t < nsel; t++) {
    int i = sel[t];
    float z = p[2] + R[6] * HULL[K][i][0] + R[7] * HULL[K][i][1] + R[8] * HULL[K][i][2];
    if (!(z < 0.0f)) continue;
    // P_b = h - n_b*dist/2, n_b = R^T e_z
    S.at(s0 + t, 0) = HULL[K][i][0] - R[6] * 0.5f * z;
    S.at(s0 + t, 1) = HULL[K][i][1] - R[7] * 0.5f * z;
    S.at(s0 + t, 2) = HULL[K][i][2] - R[8] * 0.5f * z;
    S.at(s0 + t, 3) = z;
    bits |= 1u << (s0 + t);
  }
  return bits;
}

#define FOR_CHAINS(F, ...) \
  F<0>(__VA_ARGS__);       \
  F<1>(__VA_ARGS__);       \
  F<2>(__VA_ARGS__);       \
  F<3>(__VA_ARGS__);       \
  F<4>(__VA_ARGS__);       \
  F<5>(__VA_ARGS__)

struct StepResult {
  float qacc[NV];  // u coords
  float acce[NV];  // implicit-damping Euler acceleration, u coords
  bool bad;
};

// mj_Euler + mj_advance: qvel += h acc (u coords -> world linear), positions (free joint: quaternion
// exponential in the body frame, then normalise), qacc_warmstart <- qacc (back to q coords).
// R is the pre-integration chassis rotation the u coordinates are expressed in.
__device__ __forceinline__ void euler_advance(const float u[NV], const StepResult& res, const float R[9],
                                              float qpos[13], float qvel[NV], float warm[NV]) {
  float vb[3];
#pragma unroll
  for (int k = 0; k < 3; k++) vb[k] = u[k] + DT * res.acce[k];
#pragma unroll
  for (int k = 0; k < 3; k++) qvel[k] = R[3 * k] * vb[0] + R[3 * k + 1] * vb[1] + R[3 * k + 2] * vb[2];
#pragma unroll
  for (int i = 3; i < NV; i++) qvel[i] = u[i] + DT * res.acce[i];
#pragma unroll
  for (int k = 0; k < 3; k++) qpos[k] += DT * qvel[k];
  {
    const float w[3] = {qvel[3], qvel[4], qvel[5]};
    const float wn = fsqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    float ang = DT * wn;
    float ax[3];
    if (wn < MINVAL) { ax[0] = 1; ax[1] = 0; ax[2] = 0; ang = 0; }
    else { const float iw = frcp(wn); ax[0] = w[0] * iw; ax[1] = w[1] * iw; ax[2] = w[2] * iw; }
    float s, c;
    fsincos(0.5f * ang, s, c);
    const float qr[4] = {c, ax[0] * s, ax[1] * s, ax[2] * s};
    float qq[4] = {qpos[3], qpos[4], qpos[5], qpos[6]};
    normq(qq);
    qpos[3] = qq[0] * qr[0] - qq[1] * qr[1] - qq[2] * qr[2] - qq[3] * qr[3];
    qpos[4] = qq[0] * qr[1] + qq[1] * qr[0] + qq[2] * qr[3] - qq[3] * qr[2];
    qpos[5] = qq[0] * qr[2] - qq[1] * qr[3] + qq[2] * qr[0] + qq[3] * qr[1];
    qpos[6] = qq[0] * qr[3] + qq[1] * qr[2] - qq[2] * qr[1] + qq[3] * qr[0];
  }
#pragma unroll
  for (int j = 7; j < 13; j++) qpos[j] += DT * qvel[j - 1];
#pragma unroll
  for (int k = 0; k < 3; k++) warm[k] = R[3 * k] * res.qacc[0] + R[3 * k + 1] * res.qacc[1] + R[3 * k + 2] * res.qacc[2];
#pragma unroll
  for (int i = 3; i < NV; i++) warm[i] = res.qacc[i];
}

// chassis-frame velocities / warmstart (u coordinates) of the loaded state
__device__ __forceinline__ void to_u(const float qpos[13], const float qvel[NV], const float warm[NV], float R[9],
                                     float u[NV], float wu[NV]) {
  float q[4] = {qpos[3], qpos[4], qpos[5], qpos[6]};
  normq(q);
  quat_R(q, R);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    u[k] = R[k] * qvel[0] + R[3 + k] * qvel[1] + R[6 + k] * qvel[2];
    wu[k] = R[k] * warm[0] + R[3 + k] * warm[1] + R[6 + k] * warm[2];
  }
#pragma unroll
  for (int i = 3; i < NV; i++) { u[i] = qvel[i]; wu[i] = warm[i]; }
}
__device__ __forceinline__ void reset_to_qpos0(float qpos[13], float qvel[NV], float warm[NV], float ctrl[3]) {
#pragma unroll
  for (int i = 0; i < 13; i++) qpos[i] = QPOS0[i];
#pragma unroll
  for (int i = 0; i < NV; i++) { qvel[i] = 0.0f; warm[i] = 0.0f; }
  ctrl[0] = ctrl[1] = ctrl[2] = 0.0f;
}

// Pose the observation is taken at. Default: the pre-integration pose (mj_step's sensors and x*
// arrays). F_POSTSTEP_OBS: render_mode="human" (ackermann_env.py:202-207) runs mj_forward after
// mj_step, so obs/reward see the integrated pose.
__device__ __forceinline__ void obs_pose(uint32_t flags, const float qpos[13], float p[3], float q[4], float R[9]) {
  if (flags & F_POSTSTEP_OBS) {
#pragma unroll
    for (int k = 0; k < 3; k++) p[k] = qpos[k];
#pragma unroll
    for (int k = 0; k < 4; k++) q[k] = qpos[3 + k];
    normq(q);
    quat_R(q, R);
  }
}

// Scalar constraint rows (equality, dof friction loss, joint limits) of one env: their reference
// accelerations aref (jar = J a - aref), D = 1/R, the Huber width R floss and floss, and which
// rows exist. They read only hinge positions and hinge speeds (u = qvel there), so the lane
// kernels' observation wave computes them beside the dynamics wave (see step_split).
struct ScalRows {
  float aref[NSCAL], D[NSCAL], Rfl[NSCAL], fl[NSCAL];
  bool act[NSCAL];
  float eqc2;  // equality row J = e_EQ_DOF1 + eqc2 e_EQ_DOF2
};
static_assert(EQ_DOF1 >= 6 && EQ_DOF2 >= 6, "equality between hinge dofs");
__device__ __forceinline__ void scalar_rows(const float qpos[13], const float u[NV], ScalRows& r_) {
  float K, B;
  ref_kb(K, B);
  {
    // equality (polycoef), pos and diagApprox
    const float dif = qpos[EQ_QPOS2] - QPOS0[EQ_QPOS2];
    const float cpos = EQ_POLY[0] + dif * (EQ_POLY[1] + dif * (EQ_POLY[2] + dif * (EQ_POLY[3] + dif * EQ_POLY[4])));
    const float cvel = EQ_POLY[1] + dif * (2 * EQ_POLY[2] + dif * (3 * EQ_POLY[3] + dif * 4 * EQ_POLY[4]));
    r_.eqc2 = -cvel;
    const float pos = qpos[EQ_QPOS1] - QPOS0[EQ_QPOS1] - cpos;
    const float imp = impedance(pos);
    const float diag = DOF_INVW[EQ_DOF1] + DOF_INVW[EQ_DOF2];
    const float Rr = fmaxf(MINVAL, fdiv(1 - imp, imp) * diag);
    r_.D[0] = frcp(Rr); r_.Rfl[0] = 0; r_.fl[0] = 0; r_.act[0] = true;
    const float jv = u[EQ_DOF1] + r_.eqc2 * u[EQ_DOF2];
    r_.aref[0] = -B * jv - K * imp * pos;
  }
#pragma unroll
  for (int r = 1; r <= 6; r++) {
    const int d = 5 + r;
    const float imp = impedance(0.0f);
    const float Rr = fmaxf(MINVAL, fdiv(1 - imp, imp) * DOF_INVW[d]);
    r_.D[r] = frcp(Rr); r_.fl[r] = FRICTIONLOSS[d]; r_.Rfl[r] = Rr * FRICTIONLOSS[d];
    r_.act[r] = FRICTIONLOSS[d] > 0.0f;
    r_.aref[r] = -B * u[d];
  }
#pragma unroll
  for (int r = 7; r < NSCAL; r++) {
    const int l = (r - 7) >> 1, side = ((r - 7) & 1) ? 1 : -1;
    const float q = qpos[LIM_QPOS[l]];
    const float dist = side * (LIM_RANGE[l][side > 0 ? 1 : 0] - q);
    r_.act[r] = dist < 0.0f;
    const float imp = impedance(dist);
    const float Rr = fmaxf(MINVAL, fdiv(1 - imp, imp) * DOF_INVW[LIM_DOF[l]]);
    r_.D[r] = frcp(Rr); r_.fl[r] = 0; r_.Rfl[r] = 0;
    const float jv = -side * u[LIM_DOF[l]];
    r_.aref[r] = -B * jv - K * imp * dist;
  }
}
// the state-dependent words of ScalRows through LDS ([word][slot], conflict-free): aref 0..10,
// D of the equality and the limits, the limits' existence bits, eqc2; the rest is constant
constexpr int XCH_ROWS = NSCAL + 1 + (NSCAL - 7) + 1 + 1;  // + ctrl 3
constexpr int XCH_WORDS = XCH_ROWS + 3;
__device__ __forceinline__ void xch_put(float* x, int slot, int stride, const ScalRows& r, const float ctrl[3]) {
  int w = 0;
#pragma unroll
  for (int k = 0; k < NSCAL; k++) x[(w++) * stride + slot] = r.aref[k];
  x[(w++) * stride + slot] = r.D[0];
  uint32_t bits = 0;
#pragma unroll
  for (int k = 7; k < NSCAL; k++) {
    x[(w++) * stride + slot] = r.D[k];
    bits |= (r.act[k] ? 1u : 0u) << k;
  }
  x[(w++) * stride + slot] = __uint_as_float(bits);
  x[(w++) * stride + slot] = r.eqc2;
#pragma unroll
  for (int k = 0; k < 3; k++) x[(w++) * stride + slot] = ctrl[k];
}
__device__ __forceinline__ void xch_get(const float* x, int slot, int stride, ScalRows& r, float ctrl[3]) {
  int w = 0;
#pragma unroll
  for (int k = 0; k < NSCAL; k++) r.aref[k] = x[(w++) * stride + slot];
  r.D[0] = x[(w++) * stride + slot];
  r.Rfl[0] = 0; r.fl[0] = 0; r.act[0] = true;
#pragma unroll
  for (int k = 1; k <= 6; k++) {  // friction loss: constants (impedance at pos 0)
    const int d = 5 + k;
    const float imp = impedance(0.0f);
    const float Rr = fmaxf(MINVAL, fdiv(1 - imp, imp) * DOF_INVW[d]);
    r.D[k] = frcp(Rr); r.fl[k] = FRICTIONLOSS[d]; r.Rfl[k] = Rr * FRICTIONLOSS[d];
    r.act[k] = FRICTIONLOSS[d] > 0.0f;
  }
#pragma unroll
  for (int k = 7; k < NSCAL; k++) { r.D[k] = x[(w++) * stride + slot]; r.fl[k] = 0; r.Rfl[k] = 0; }
  const uint32_t bits = __float_as_uint(x[(w++) * stride + slot]);
#pragma unroll
  for (int k = 7; k < NSCAL; k++) r.act[k] = (bits >> k) & 1u;
  r.eqc2 = x[(w++) * stride + slot];
#pragma unroll
  for (int k = 0; k < 3; k++) ctrl[k] = x[(w++) * stride + slot];
}

// The implicit-Euler factor chol(M + h diag(damping)) depends on the steer angles alone (M is
// constant but for the front spin axes), so the prep wave computes it beside the solve and hands
// its structural nonzeros over (float4 per lane: 16-byte LDS reads, conflict-free).
constexpr int eu_words(int kind = 0) {
  int n = 0;
  for (int i = 0; i < NV; i++)
    for (int j = 0; j <= i; j++) n += LPAT[kind].nz[i][j] ? 1 : 0;
  return n;
}
constexpr int EU_VEC = (eu_words() + 3) / 4;
// chol(M) (EU = false: qacc_smooth) or chol(M + h diag(damping)) (EU: implicit Euler) at the
// front steer angles d2, d3
template <bool EU>
__device__ __forceinline__ void mass_factor(float d2, float d3, float L[NV][NV]) {
  float sa[2][3];
#pragma unroll
  for (int s = 0; s < 2; s++) {
    float c, sn;
    fsincos(s == 0 ? d2 : d3, sn, c);
    rot_axis(sa[s], S_AXIS[s], W_SPIN_AXIS[2 + s], c, sn);
  }
  build_M(L, sa);
  if constexpr (EU) {
#pragma unroll
    for (int i = 0; i < NV; i++) L[i][i] += DT * DAMPING[i];
  }
  chol_sp<0>(L);
}
__device__ __forceinline__ void euler_factor(const float qpos[13], float L[NV][NV]) {
  mass_factor<true>(qpos[W_STEER_QPOS[2]], qpos[W_STEER_QPOS[3]], L);
}
template <int KIND = 0, int NVEC = EU_VEC>
__device__ __forceinline__ void eu_put(float* x, int lane, const float L[NV][NV]) {
  float w[4 * NVEC];
  int n = 0;
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int j = 0; j <= i; j++)
      if (LPAT[KIND].nz[i][j]) w[n++] = AK_F(L, i, j);
#pragma unroll
  for (int k = n; k < 4 * NVEC; k++) w[k] = 0.0f;
  float4* x4 = reinterpret_cast<float4*>(x);
#pragma unroll
  for (int v = 0; v < NVEC; v++) x4[v * 64 + lane] = make_float4(w[4 * v], w[4 * v + 1], w[4 * v + 2], w[4 * v + 3]);
}
template <int KIND = 0, int NVEC = EU_VEC>
__device__ __forceinline__ void eu_get(const float* x, int lane, float L[NV][NV]) {
  float w[4 * NVEC];
  const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll
  for (int v = 0; v < NVEC; v++) {
    const float4 t = x4[v * 64 + lane];
    w[4 * v] = t.x; w[4 * v + 1] = t.y; w[4 * v + 2] = t.z; w[4 * v + 3] = t.w;
  }
  int n = 0;
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int j = 0; j <= i; j++)
      if (LPAT[KIND].nz[i][j]) AK_F(L, i, j) = w[n++];
}

// H of the piece whose quadratic rows are qmask, lower triangle, as dyn_post builds it
__device__ __forceinline__ void piece_hessian(const float M[NV][NV], uint32_t qmask, const float sD[NSCAL], float eqc2,
                                              float H[NV][NV]) {
#pragma unroll
  for (int i = 0; i < NV; i++)
#pragma unroll
    for (int j = 0; j < NV; j++) H[i][j] = (j <= i) ? M[i][j] : 0.0f;
#pragma unroll
  for (int r = 0; r < NSCAL; r++) {
    if (!((qmask >> r) & 1u)) continue;
    int d1, d2;
    float c1;
    scal_dofs(r, d1, c1, d2);
    H[d1][d1] += sD[r] * c1 * c1;
    if (d2 >= 0) {
      H[d2][d2] += sD[r] * eqc2 * eqc2;
      if (d2 > d1) H[d2][d1] += sD[r] * c1 * eqc2;
      else H[d1][d2] += sD[r] * c1 * eqc2;
    }
  }
}
// where the dynamics wave finds the prep wave's Euler factor (XEU): LDS words, flag, lane
struct EuHand {
  const float* x;
  int* flag;
  int lane;
};

// forward dynamics, first part (no control): steer-dependent axes, mass matrix, bias, passive
struct DynPre {
  float sa[2][3], cyl[2][3];
  Solver sv;  // M; fs = -bias - damping (actuator forces added in dyn_post)
};
__device__ __forceinline__ void dyn_pre(const float qpos[13], const float u[NV], const float R[9], DynPre& P) {
  // front steer angles -> spin / cylinder axes in the chassis frame
#pragma unroll
  for (int s = 0; s < 2; s++) {
    float d = qpos[W_STEER_QPOS[2 + s]];
    float c, sn;
    fsincos(d, sn, c);
    rot_axis(P.sa[s], S_AXIS[s], W_SPIN_AXIS[2 + s], c, sn);
    rot_axis(P.cyl[s], S_AXIS[s], W_CYL_AXIS[2 + s], c, sn);
  }
  STAMP(2);
  build_M(P.sv.M, P.sa);
  float b[NV];
  bias(u, R, P.sa, b);
  // passive damping (mj_passive)
#pragma unroll
  for (int i = 0; i < NV; i++) P.sv.fs[i] = -b[i] - DAMPING[i] * u[i];
}

// forward dynamics, second part: actuators, qacc_smooth, constraints and solve, Euler force
// XEU / XM: the Euler / mass-matrix factor comes from another wave (eh / mh), see step_split
template <int NC, bool XEU = false, bool XM = false>  // NC = 1: contacts off
__device__ __forceinline__ void dyn_post(Slots& S, DynPre& P, const float qpos[13], const float u[NV],
                                         const float warm_u[NV], const float R[9], const float ctrl[3], uint32_t flags,
                                         const ScalRows& sr, StepResult& out, EuHand eh = EuHand{},
                                         EuHand mh = EuHand{}) {
  float(&sa)[2][3] = P.sa;
  float(&cyl)[2][3] = P.cyl;
  Solver& sv = P.sv;
  (void)sa;
  {  // actuators (mj_fwdActuation)
    float c0 = ctrl[0];
    if (ACT_CTRLLIMITED[0]) c0 = fminf(fmaxf(c0, ACT_CTRLRANGE[0][0]), ACT_CTRLRANGE[0][1]);
    float f0 = ACT_GAIN[0] * c0 + ACT_BIAS1[0] * qpos[ACT_STEER_QPOS] + ACT_BIAS2[0] * u[ACT_STEER_DOF];
    if (ACT_FORCELIMITED[0]) f0 = fminf(fmaxf(f0, ACT_FORCERANGE[0][0]), ACT_FORCERANGE[0][1]);
    sv.fs[ACT_STEER_DOF] += f0;
    float c1 = ctrl[1], c2 = ctrl[2];
    if (ACT_CTRLLIMITED[1]) c1 = fminf(fmaxf(c1, ACT_CTRLRANGE[1][0]), ACT_CTRLRANGE[1][1]);
    if (ACT_CTRLLIMITED[2]) c2 = fminf(fmaxf(c2, ACT_CTRLRANGE[2][0]), ACT_CTRLRANGE[2][1]);
    float f1 = ACT_GAIN[1] * c1 + ACT_BIAS2[1] * u[ACT_RL_DOF];
    float f2 = ACT_GAIN[2] * c2 + ACT_BIAS2[2] * u[ACT_RR_DOF];
    if (ACT_FORCELIMITED[1]) f1 = fminf(fmaxf(f1, ACT_FORCERANGE[1][0]), ACT_FORCERANGE[1][1]);
    if (ACT_FORCELIMITED[2]) f2 = fminf(fmaxf(f2, ACT_FORCERANGE[2][0]), ACT_FORCERANGE[2][1]);
    sv.fs[ACT_RL_DOF] += f1;
    sv.fs[ACT_RR_DOF] += f2;
  }
  // qacc_smooth = M^-1 fs
  float L[NV][NV];
  if constexpr (XM) {  // factored by the observation wave (same steer angles)
    while (__hip_atomic_load(mh.flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
    eu_get(mh.x, mh.lane, L);
  } else {
#pragma unroll
    for (int i = 0; i < NV; i++)
#pragma unroll
      for (int j = 0; j < NV; j++) L[i][j] = sv.M[i][j];
    chol_sp<0>(L);
  }
#pragma unroll
  for (int i = 0; i < NV; i++) sv.a0[i] = sv.fs[i];
  chol_sp_solve<0>(L, sv.a0);

  STAMP(3);
  // contacts
  S.lmask = 0u;
  if (!NC && (flags & F_CONTACTS)) {
    const float rear_cyl[3] = {W_CYL_AXIS[0][0], W_CYL_AXIS[0][1], W_CYL_AXIS[0][2]};
    const float rear_cyl1[3] = {W_CYL_AXIS[1][0], W_CYL_AXIS[1][1], W_CYL_AXIS[1][2]};
    S.lmask |= wheel_contacts<0>(S, qpos, R, rear_cyl);
    S.lmask |= wheel_contacts<1>(S, qpos, R, rear_cyl1);
    S.lmask |= wheel_contacts<2>(S, qpos, R, cyl[0]);
    S.lmask |= wheel_contacts<3>(S, qpos, R, cyl[1]);
    S.lmask |= mesh_contacts<0>(S, qpos, R);
    S.lmask |= mesh_contacts<1>(S, qpos, R);
  }
  // wave-uniform union of active slots (24 ballots -> SGPR mask)
  S.wmask = 0u;
  if constexpr (!NC) {
#pragma unroll
    for (int b = 0; b < NSLOT; b++)
      if (__ballot((S.lmask >> b) & 1u)) S.wmask |= 1u << b;
  }
  const uint32_t wm = NC ? 0u : S.wmask;  // compile-time 0 without contacts: every slot loop folds away
  // contact frame directions in the chassis frame: n = e_z, t1 = e_y, t2 = -e_x (mju_makeFrame)
  float dirs[3][3] = {{R[6], R[7], R[8]}, {R[3], R[4], R[5]}, {-R[0], -R[1], -R[2]}};

  STAMP(4);
  float K, B;
  ref_kb(K, B);
  // scalar rows: jar, D, type, R*floss
  float sj[NSCAL], sD[NSCAL], sRfl[NSCAL], sfl[NSCAL], sjp[NSCAL];
  bool sact[NSCAL];
  const float eqc2 = sr.eqc2;
#pragma unroll
  for (int r = 0; r < NSCAL; r++) {
    sj[r] = sr.aref[r];  // holds aref for now
    sD[r] = sr.D[r];
    sRfl[r] = sr.Rfl[r];
    sfl[r] = sr.fl[r];
    sact[r] = sr.act[r];
  }
  // aref of scalar rows is in sj; jar(a) = J a - aref

  // warmstart: the cheaper of qacc_warmstart and qacc_smooth (cost = gauss + constraint)
  auto scal_J_dot = [&](int r, const float x[NV]) __attribute__((always_inline)) -> float {
    if (r == 0) return x[EQ_DOF1] + eqc2 * x[EQ_DOF2];
    if (r <= 6) return x[5 + r];
    int l = (r - 7) >> 1;
    float c = ((r - 7) & 1) ? -1.0f : 1.0f;
    return c * x[LIM_DOF[l]];
  };
  auto scal_cost = [&](int r, float x) __attribute__((always_inline)) -> float {
    if (!sact[r]) return 0.0f;
    if (r == 0) return 0.5f * sD[r] * x * x;
    if (r <= 6) {
      if (x <= -sRfl[r]) return -sfl[r] * x - 0.5f * sRfl[r] * sfl[r];
      if (x >= sRfl[r]) return sfl[r] * x - 0.5f * sRfl[r] * sfl[r];
      return 0.5f * sD[r] * x * x;
    }
    return x < 0.0f ? 0.5f * sD[r] * x * x : 0.0f;
  };
  float cost_w = 0.0f, cost_s = 0.0f;
  {
    float dw[NV], Mdw[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) dw[i] = warm_u[i] - sv.a0[i];
    symv_M<0>(sv.M, dw, Mdw);
#pragma unroll
    for (int i = 0; i < NV; i++) cost_w += 0.5f * dw[i] * Mdw[i];
#pragma unroll
    for (int r = 0; r < NSCAL; r++) {
      cost_w += scal_cost(r, scal_J_dot(r, warm_u) - sj[r]);
      cost_s += scal_cost(r, scal_J_dot(r, sv.a0) - sj[r]);
    }
  }
  // contact rows: need jar at both candidates. Initialise slots at warm and at a0 (cheap).
  // slot field 4..7 temporarily = J a_w - aref ; we evaluate cost then re-init for the chosen.
  if constexpr (!NC) { FOR_CHAINS(slot_loop_init, S, dirs, sa, warm_u, u, K, B); }
  float cw_c = 0.0f;
  FOR_SLOTS(S, wm, s) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      float x = S.at(s, 4 + r);
      if (x < 0.0f) cw_c += 0.5f * S.at(s, 3) * x * x;
    }
  }
  cost_w += cw_c;
  // jar at a0 = jar_w + J (a0 - warm): use the Jp machinery with p = a0 - warm
  float a[NV];
  {
    float dpa[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) dpa[i] = sv.a0[i] - warm_u[i];
    if constexpr (!NC) { FOR_CHAINS(slot_loop_jp, S, dirs, sa, dpa); }
    float cs_c = 0.0f;
    FOR_SLOTS(S, wm, s) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float x = S.at(s, 4 + r) + S.at(s, 8 + r);
        if (x < 0.0f) cs_c += 0.5f * S.at(s, 3) * x * x;
      }
    }
    cost_s += cs_c;
    // Newton start. MuJoCo takes the cheaper of qacc_warmstart and qacc_smooth; the contacts-off
    // kernel starts from qacc_warmstart : the cost is strictly convex (M > 0), so
    // both starts reach the same unique minimiser -- the parity tests hold it to the oracle, which
    // applies MuJoCo's rule -- and on the benchmark workload the oracle's rule picks qacc_smooth
    // for 85 % of env-steps, from where Newton needs one more iteration (wave max 3 vs 2). With
    // contacts (stiff, ill-conditioned in f32) the f32 solve's last digits depend on the start, so
    // the contact kernels keep MuJoCo's rule.
    const bool use_w = NC ? true : cost_w < cost_s;
#pragma unroll
    for (int i = 0; i < NV; i++) a[i] = use_w ? warm_u[i] : sv.a0[i];
    if (!use_w) {
      FOR_SLOTS(S, wm, s) {
#pragma unroll
        for (int r = 0; r < 4; r++) S.at(s, 4 + r) += S.at(s, 8 + r);
      }
    }
  }
  // Predicted active set (contacts-off kernel). Within a fixed set of row states the cost is
  // quadratic, so ONE Newton step from any point on that piece lands on its minimiser, and if the
  // rows there are in the assumed states that minimiser is the optimum (strict convexity). The
  // states are predicted at qacc_smooth moved onto the steering equality (the servo drives one
  // steer, the equality the other), each friction-loss row as its own one-dof problem: its
  // saturated force floss moves x by floss * invweight, so the row ends in the quadratic zone iff
  // |x_p| <= R floss + floss invweight. The f64 probe (tools/probes/active_set_probe.py) finds the
  // exact final states this way for 99.84 % of env-steps on the benchmark workload (the misses:
  // steer pairs the equality does not hold together); a miss continues with Newton from the
  // piece's minimiser, which is a start as good as any.
  bool exact = false;
#ifdef AK_STAMPS
  int diag_pair = 0;  // diag build: 1 = this lane's one-dof steer guess was inconsistent (9-pair search)
#endif
  if constexpr (NC) {
    float ap[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) ap[i] = sv.a0[i];
    {  // minimal diagonal-mass-norm move of the two steer accelerations onto J_eq a = 0
      const float m1 = sv.M[EQ_DOF1][EQ_DOF1], m2 = sv.M[EQ_DOF2][EQ_DOF2];
      const float je = ap[EQ_DOF1] + eqc2 * ap[EQ_DOF2];
      const float lam = je * frcp(1.0f / m1 + eqc2 * eqc2 / m2);
      ap[EQ_DOF1] -= lam / m1;
      ap[EQ_DOF2] -= lam * eqc2 / m2;
    }
    int pst[NSCAL];  // predicted state: friction loss -1 / 0 (quadratic) / +1, limit 1 = active
#pragma unroll
    for (int r = 0; r < NSCAL; r++) {
      const float xp = scal_J_dot(r, ap) - sj[r];
      if (r == 0) pst[r] = 0;
      else if (r <= 6) {
        const float thr = sRfl[r] + sfl[r] * DOF_INVW[5 + r];
        pst[r] = xp < -thr ? -1 : (xp > thr ? 1 : 0);
      } else pst[r] = xp < 0.0f ? 1 : 0;
    }
    {  // the steer pair (friction-loss rows of the two steers, joined by the equality row): their
       // states from the exact two-dof sub-problem at qacc_smooth (diagonal masses, equality and
       // both Huber rows), solved on the one-dof guess first and, in waves where that guess is
       // inconsistent for some lane, over all 9 state pairs (probe: 100 % of 35 840 env-steps)
      constexpr int r1 = EQ_DOF1 - 5, r2 = EQ_DOF2 - 5;
      static_assert(r1 >= 1 && r1 <= 6 && r2 >= 1 && r2 <= 6, "equality joins two hinge dofs with friction-loss rows");
      const float m1 = sv.M[EQ_DOF1][EQ_DOF1], m2 = sv.M[EQ_DOF2][EQ_DOF2], De = sD[0], ae = sj[0], c = eqc2;
      const float b1 = m1 * sv.a0[EQ_DOF1] + De * ae, b2 = m2 * sv.a0[EQ_DOF2] + De * c * ae;
      const float h11 = m1 + De, h22 = m2 + De * c * c, h12 = De * c;
      auto consistent = [&](int s1, int s2) __attribute__((always_inline)) -> bool {
        const bool q1 = sact[r1] && s1 == 0, q2 = sact[r2] && s2 == 0;
        const float H11 = h11 + (q1 ? sD[r1] : 0.0f), H22 = h22 + (q2 ? sD[r2] : 0.0f);
        const float B1 = b1 + (q1 ? sD[r1] * sj[r1] : -(float)s1 * sfl[r1]);
        const float B2 = b2 + (q2 ? sD[r2] * sj[r2] : -(float)s2 * sfl[r2]);
        const float idet = frcp(H11 * H22 - h12 * h12);
        const float x1 = (B1 * H22 - h12 * B2) * idet - sj[r1], x2 = (H11 * B2 - h12 * B1) * idet - sj[r2];
        const int t1 = x1 <= -sRfl[r1] ? -1 : (x1 >= sRfl[r1] ? 1 : 0);
        const int t2 = x2 <= -sRfl[r2] ? -1 : (x2 >= sRfl[r2] ? 1 : 0);
        return t1 == s1 && t2 == s2;
      };
      bool ok = consistent(pst[r1], pst[r2]);
#ifdef AK_STAMPS
      diag_pair = ok ? 0 : 1;
#endif
      if (__builtin_amdgcn_ballot_w64(!ok) != 0ull) {
#pragma unroll 1
        for (int k = 0; k < 9; k++) {
          const int s1 = k / 3 - 1, s2 = k % 3 - 1;
          if (!ok && consistent(s1, s2)) {
            ok = true;
            pst[r1] = s1;
            pst[r2] = s2;
          }
        }
      }
    }
    // one Newton step from qacc_smooth on the predicted piece (gradient of that piece at a0)
#pragma unroll
    for (int i = 0; i < NV; i++) a[i] = sv.a0[i];
#pragma unroll
    for (int r = 0; r < NSCAL; r++) sj[r] = scal_J_dot(r, a) - sj[r];
    float H[NV][NV], grad[NV];
    uint32_t qmask = 0u;  // the piece's quadratic rows
#pragma unroll
    for (int i = 0; i < NV; i++) grad[i] = 0.0f;
#pragma unroll
    for (int r = 0; r < NSCAL; r++) {
      if (!sact[r]) continue;
      int d1, d2;
      float c1;
      scal_dofs(r, d1, c1, d2);
      const bool quad = (r == 0) || (r <= 6 ? pst[r] == 0 : pst[r] == 1);
      const float f = quad ? -sD[r] * sj[r] : (r <= 6 ? -(float)pst[r] * sfl[r] : 0.0f);
      grad[d1] -= f * c1;
      if (d2 >= 0) grad[d2] -= f * eqc2;
      if (quad) qmask |= 1u << r;
    }
    piece_hessian(sv.M, qmask, sD, eqc2, H);
    chol_sp<1>(H);
    float pdir[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) pdir[i] = -grad[i];
    chol_sp_solve<1>(H, pdir);
#pragma unroll
    for (int i = 0; i < NV; i++) a[i] += pdir[i];
    int changed = 0;
#pragma unroll
    for (int r = 0; r < NSCAL; r++) {
      const float x = sj[r] + scal_J_dot(r, pdir);
      sj[r] = x;
      if (sact[r] && r > 0) {
        const int s1 = r <= 6 ? (x <= -sRfl[r] ? -1 : (x >= sRfl[r] ? 1 : 0)) : (x < 0.0f ? 1 : 0);
        changed += s1 != pst[r];
      }
    }
    exact = changed == 0;
  } else {
    // scalar jar at a
#pragma unroll
    for (int r = 0; r < NSCAL; r++) sj[r] = scal_J_dot(r, a) - sj[r];
  }

  STAMP(5);
  // ---------------- Newton iterations
  // Converged when the previous step was a full (alpha = 1) Newton step that changed no row
  // state -- within a fixed active set the cost is quadratic, so that step was exact -- or when
  // the gradient is at the f32 noise floor of its two cancelling parts (rows flickering at a
  // region boundary), or after MAXIT iterations.
  int it_done = MAXIT, why = 4;
  NT_DECL
  NT_START;
  // wave-uniform skip when every lane is already exact (the predicted piece): otherwise the
  // loop's invariant set-up, which the compiler hoists ahead of the first exit test, still runs
  if (__builtin_amdgcn_ballot_w64(!exact) == 0ull) { it_done = 0; why = 1; }
  else
#pragma unroll 1
  for (int it = 0; it < MAXIT; it++) {
    if (exact) { it_done = it; if (why != 2) why = 1; break; }
    float H[NV][NV], grad[NV];
    float gscale = 0.0f;
    {
      float da[NV];
#pragma unroll
      for (int i = 0; i < NV; i++) da[i] = a[i] - sv.a0[i];
      symv_M<0>(sv.M, da, grad);
#pragma unroll
      for (int i = 0; i < NV; i++) gscale = fmaxf(gscale, fabsf(grad[i]));
    }
#pragma unroll
    for (int i = 0; i < NV; i++)
#pragma unroll
      for (int j = 0; j < NV; j++) H[i][j] = (j <= i) ? sv.M[i][j] : 0.0f;
    // scalar rows
#pragma unroll
    for (int r = 0; r < NSCAL; r++) {
      if (!sact[r]) continue;
      int d1, d2;
      float c1;
      scal_dofs(r, d1, c1, d2);
      float x = sj[r];
      float f;
      bool quad;
      if (r == 0) { f = -sD[r] * x; quad = true; }
      else if (r <= 6) {
        if (x <= -sRfl[r]) { f = sfl[r]; quad = false; }
        else if (x >= sRfl[r]) { f = -sfl[r]; quad = false; }
        else { f = -sD[r] * x; quad = true; }
      } else { quad = x < 0.0f; f = quad ? -sD[r] * x : 0.0f; }
      grad[d1] -= f * c1;
      if (d2 >= 0) grad[d2] -= f * eqc2;
      if (quad) {
        H[d1][d1] += sD[r] * c1 * c1;
        if (d2 >= 0) {
          H[d2][d2] += sD[r] * eqc2 * eqc2;
          if (d2 > d1) H[d2][d1] += sD[r] * c1 * eqc2;
          else H[d1][d2] += sD[r] * c1 * eqc2;
        }
      }
    }
    if constexpr (!NC) { FOR_CHAINS(slot_loop_hess, S, dirs, sa, H, grad); }
    (void)gscale;
    NT_MARK(0);
    if (wm) chol_sp<2>(H);  // wave-uniform: contact rows present in some lane
    else chol_sp<1>(H);
    float pdir[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) pdir[i] = -grad[i];
    if (wm) chol_sp_solve<2>(H, pdir);
    else chol_sp_solve<1>(H, pdir);
    NT_MARK(1);
    // Jp for all rows
    if constexpr (!NC) { FOR_CHAINS(slot_loop_jp, S, dirs, sa, pdir); }
#pragma unroll
    for (int r = 0; r < NSCAL; r++) sjp[r] = scal_J_dot(r, pdir);
    // exact line search on the piecewise-linear derivative phi'(alpha)
    float Mp[NV];
    symv_M<0>(sv.M, pdir, Mp);
    float pMp = 0.0f, pg0 = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; i++) { pMp += pdir[i] * Mp[i]; pg0 += Mp[i] * (a[i] - sv.a0[i]); }
    auto dphi = [&](float al, float& g, float& h) __attribute__((always_inline)) {
      g = fmaf(al, pMp, pg0);
      h = pMp;
      scal_ls<0>(al, sj, sjp, sD, sRfl, sfl, sact, 0, g, h);
      FOR_SLOTS(S, wm, s) {
        float D = S.at(s, 3);
#pragma unroll
        for (int r = 0; r < 4; r++) {
          float jp = S.at(s, 8 + r);
          float x = S.at(s, 4 + r) + al * jp;
          if (x < 0.0f) { g += D * x * jp; h += D * jp * jp; }
        }
      }
    };
    // phi'(0) = grad . p (no row pass needed); try the full Newton step first
    float g0 = 0.0f;
#pragma unroll
    for (int i = 0; i < NV; i++) g0 += grad[i] * pdir[i];
    if (!(g0 < 0.0f)) { it_done = it; why = 3; break; }  // no descent left: optimum to f32 precision
    float ns = fabsf(pg0) + fabsf(pMp) + scal_noise<0>(sj, sjp, sD, sRfl, sfl, sact, 0);
    FOR_SLOTS(S, wm, s) {
      const float D = S.at(s, 3);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float x = S.at(s, 4 + r), jp = S.at(s, 8 + r);
        if (x < 0.0f) ns += D * (fabsf(x * jp) + jp * jp);
      }
    }
    const float gtol = fmaxf(1e-4f * fabsf(g0), 1e-5f * ns);
    NT_MARK(2);
    float lo = 0.0f, hi = 3.0e38f, al = 1.0f;
    bool full = false;
#pragma unroll 1
    for (int k = 0; k < LSIT; k++) {
      float g, h;
      dphi(al, g, h);
      if (fabsf(g) <= gtol) { full = (k == 0); break; }
      if (g < 0.0f) lo = al; else hi = al;
      float nal = al - g * __builtin_amdgcn_rcpf(h);  // a proposal inside the bracket: 1-ulp rcp suffices
      if (!(nal > lo && nal < hi)) nal = (hi < 3.0e38f) ? 0.5f * (lo + hi) : 2.0f * al;
      bool tiny = fabsf(nal - al) <= 1e-6f * al;
      al = nal;
      if (tiny) break;
    }
    NT_MARK(3);
    // move, count row-state changes; "still" = the update is below f32 resolution of a
    int changed = 0;
    bool still = true;
#pragma unroll
    for (int i = 0; i < NV; i++) {
      float d = al * pdir[i];
      still = still && fabsf(d) <= 2e-6f * fmaxf(fabsf(a[i]), 1.0f);
      a[i] += d;
    }
#pragma unroll
    for (int r = 0; r < NSCAL; r++) {
      float x0 = sj[r], x1 = sj[r] + al * sjp[r];
      if (sact[r] && r > 0) {
        if (r <= 6) changed += ((x0 <= -sRfl[r]) != (x1 <= -sRfl[r])) + ((x0 >= sRfl[r]) != (x1 >= sRfl[r]));
        else changed += (x0 < 0.0f) != (x1 < 0.0f);
      }
      sj[r] = x1;
    }
    FOR_SLOTS(S, wm, s) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float x0 = S.at(s, 4 + r), x1 = x0 + al * S.at(s, 8 + r);
        changed += (x0 < 0.0f) != (x1 < 0.0f);
        S.at(s, 4 + r) = x1;
      }
    }
    exact = (full && changed == 0) || still;
    if (still && !(full && changed == 0)) why = 2;
#ifdef AK_TRACE
    if (threadIdx.x == 0 && blockIdx.x == 0)
      printf("[trace] it %d al %.7g full %d changed %d still %d g0 %.6g gtol %.6g ns %.6g pMp %.6g pg0 %.6g |p|inf %.6g\n", it, al,
             (int)full, changed, (int)still, g0, gtol, ns, pMp, pg0,
             fmaxf(fmaxf(fabsf(pdir[6]), fabsf(pdir[8])), fmaxf(fabsf(pdir[0]), fabsf(pdir[3]))));
#endif
    NT_MARK(4);
  }
  STAMP(6);
  NT_FLUSH;
#ifdef AK_STAMPS
  g_stamps[AK_NSTAMP * (size_t)gridDim.x + blockIdx.x * 64 + (threadIdx.x & 63)] =
      (unsigned long long)(it_done * 8 + why) + ((unsigned long long)diag_pair << 16) + ((unsigned long long)!exact << 17);
#else
  (void)it_done;
  (void)why;
#endif
#pragma unroll
  for (int i = 0; i < NV; i++) out.qacc[i] = a[i];
  // qfrc_constraint = J^T f at the solution
  float fc[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) fc[i] = 0.0f;
#pragma unroll
  for (int r = 0; r < NSCAL; r++) {
    if (!sact[r]) continue;
    int d1, d2;
    float c1;
    scal_dofs(r, d1, c1, d2);
    float x = sj[r], f;
    if (r == 0) f = -sD[r] * x;
    else if (r <= 6) f = (x <= -sRfl[r]) ? sfl[r] : ((x >= sRfl[r]) ? -sfl[r] : -sD[r] * x);
    else f = x < 0.0f ? -sD[r] * x : 0.0f;
    fc[d1] += f * c1;
    if (d2 >= 0) fc[d2] += f * eqc2;
  }
  if constexpr (!NC) { FOR_CHAINS(slot_loop_force, S, dirs, sa, fc); }
  // implicit damping Euler: (M + h diag(B)) acc = fs + fc
  if constexpr (XEU) {  // factored by the prep wave (same steer angles): wait for its flag
    STAMP(17);
    while (__hip_atomic_load(eh.flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
    STAMP(18);
    eu_get(eh.x, eh.lane, L);
  } else {
#pragma unroll
    for (int i = 0; i < NV; i++)
#pragma unroll
      for (int j = 0; j < NV; j++) L[i][j] = (j <= i) ? sv.M[i][j] : 0.0f;
#pragma unroll
    for (int i = 0; i < NV; i++) L[i][i] += DT * DAMPING[i];
    chol_sp<0>(L);
  }
#pragma unroll
  for (int i = 0; i < NV; i++) out.acce[i] = sv.fs[i] + fc[i];
  chol_sp_solve<0>(L, out.acce);
  bool bad = false;
#pragma unroll
  for (int i = 0; i < NV; i++) bad |= is_bad(a[i]);
  out.bad = bad;
  STAMP(7);
}

// forward dynamics + constraint solve for one env (state in registers), u coordinates
template <int NC>
__device__ __forceinline__ void dynamics(Slots& S, const float qpos[13], const float u[NV], const float warm_u[NV],
                                         const float R[9], const float ctrl[3], uint32_t flags, StepResult& out) {
  DynPre P;
  dyn_pre(qpos, u, R, P);
  ScalRows sr;
  scalar_rows(qpos, u, sr);
  dyn_post<NC>(S, P, qpos, u, warm_u, R, ctrl, flags, sr, out);
}

// ------------------------------------------------------------------ state I/O helpers
template <int SC>
__device__ __forceinline__ void reset_pose(float qpos[13], float qvel[NV], float warm[NV]) {
  // SimpleMapSpawner.load_random_environment: qpos0 with chassis at (0,0,0.1), identity quat
  // (the obstacle scene spawns at its own free cell, Scene<1>)
#pragma unroll
  for (int i = 0; i < 13; i++) qpos[i] = QPOS0[i];
  qpos[0] = Scene<SC>::SPX; qpos[1] = Scene<SC>::SPY; qpos[2] = Scene<SC>::SPZ;
  qpos[3] = 1.0f; qpos[4] = 0.0f; qpos[5] = 0.0f; qpos[6] = 0.0f;
#pragma unroll
  for (int i = 0; i < NV; i++) { qvel[i] = 0.0f; warm[i] = 0.0f; }
}

// goal = robot_start_position + (d cos th, d sin th) (ackermann_env.py:167-172) in the odometry
// frame, where the start position is (0, 0) whatever the spawn point (odometry.py:62-103).
// Opt-in maze task (obstacle scene, prm.goal_cells > 0): the centre of free cell
// floor(u * FREE_LE[d]) of the breadth-first list, u from the same Philox word, integer arithmetic
// (the oracle draws the same cell), minus the spawn (odometry frame: the reset pose is identity)
template <int SC>
__device__ __forceinline__ void goal_sample(uint64_t seed, int64_t genv, uint32_t episode, const EnvParams& prm,
                                            float& gx, float& gy) {
  uint32_t c[4] = {(uint32_t)genv, episode, 0u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  if constexpr (SC == 1) {
    if (prm.goal_cells > 0) {
      using namespace scene1;
      const uint32_t nle = (uint32_t)FREE_LE[prm.goal_cells < FREE_MAXD ? prm.goal_cells : FREE_MAXD];
      const uint32_t i = (uint32_t)(((uint64_t)(c[0] >> 8) * nle) >> 24);
      gx = FREE_XY[i][0] - SPAWN[0];
      gy = FREE_XY[i][1] - SPAWN[1];
      return;
    }
  }
  float d = 2.0f + 6.0f * u01(c[0]);
  float th = 6.283185307179586f * u01(c[1]);
  gx = d * cosf(th);
  gy = d * sinf(th);
}

// reset env e: writes state words + observation
template <int SC>
__device__ __forceinline__ void reset_env(const Soa& state, const Soa& obs, uint32_t vo, uint64_t seed, int64_t genv,
                                          uint32_t episode, const EnvParams& prm, float* smw = nullptr,
                                          int sms = 0) {
  float qpos[13], qvel[NV], warm[NV];
  reset_pose<SC>(qpos, qvel, warm);
  float gx, gy;
  goal_sample<SC>(seed, genv, episode, prm, gx, gy);
  float q[4] = {qpos[3], qpos[4], qpos[5], qpos[6]};
  normq(q);
  float R[9];
  quat_R(q, R);
  float ref[3] = {qpos[0], qpos[1], qpos[2]};  // odometry reference = chassis xpos at reset
#pragma unroll
  for (int i = 0; i < 13; i++) stf(state, ST_QPOS + i, vo, qpos[i]);
#pragma unroll
  for (int i = 0; i < NV; i++) {
    stf(state, ST_QVEL + i, vo, 0.0f);
    stf(state, ST_WARM + i, vo, 0.0f);
  }
  stf(state, ST_GOAL, vo, gx);
  stf(state, ST_GOAL + 1, vo, gy);
#pragma unroll
  for (int k = 0; k < 3; k++) stf(state, ST_REF + k, vo, ref[k]);
  stf(state, ST_STEP, vo, __uint_as_float(0u));
  stf(state, ST_EPIS, vo, __uint_as_float(episode));
  if (smw) {  // rollout: the same words into the LDS state mirror for the launch's next step
#pragma unroll
    for (int i = 0; i < 13; i++) smw[(ST_QPOS + i) * sms] = qpos[i];
#pragma unroll
    for (int i = 0; i < NV; i++) { smw[(ST_QVEL + i) * sms] = 0.0f; smw[(ST_WARM + i) * sms] = 0.0f; }
    smw[ST_GOAL * sms] = gx;
    smw[(ST_GOAL + 1) * sms] = gy;
#pragma unroll
    for (int k = 0; k < 3; k++) smw[(ST_REF + k) * sms] = ref[k];
    smw[ST_STEP * sms] = __uint_as_float(0u);
    smw[ST_EPIS * sms] = __uint_as_float(episode);
  }
  observe<SC>(qpos, q, R, gx, gy, ref, obs, vo, prm);
}

}  // namespace ak

#include "ackphys_quad.inc"
#include "ackphys_ppo.inc"

// ====================================================================== kernels
using namespace ak;

// The whole step of one env on one lane, observation included (F_POSTSTEP_OBS: obs/reward need the
// integrated pose, so nothing can run beside the dynamics).
__device__ __forceinline__ void step_serial(const Args& A, float* lds, int lane, int e) {
  STAMP_SCOPE
  const int n = A.n;
  STAMP(0);
  Slots S{lds + lane};
  const uint32_t vo = 4u * (uint32_t)e;
  const Soa st = soa(A.state, NSTATE, n);
  float qpos[13], qvel[NV], warm[NV];
#pragma unroll
  for (int i = 0; i < 13; i++) qpos[i] = ldf(st, ST_QPOS + i, vo);
#pragma unroll
  for (int i = 0; i < NV; i++) qvel[i] = ldf(st, ST_QVEL + i, vo);
#pragma unroll
  for (int i = 0; i < NV; i++) warm[i] = ldf(st, ST_WARM + i, vo);
  const float gx = ldf(st, ST_GOAL, vo), gy = ldf(st, ST_GOAL + 1, vo);
  const float ref[3] = {ldf(st, ST_REF, vo), ldf(st, ST_REF + 1, vo), ldf(st, ST_REF + 2, vo)};
  uint32_t step = __float_as_uint(ldf(st, ST_STEP, vo));
  uint32_t episode = __float_as_uint(ldf(st, ST_EPIS, vo));
  const Soa act = soa(A.action, 2, n);
  const float a0 = ldf(act, 0, 2 * vo), a1 = ldf(act, 0, 2 * vo + 4);

  // controller -> ctrl (float64, reference thresholds)
  float ctrl[3];
  bool badctrl;
  controller(a0, a1, A.prm.max_linear_velocity, A.prm.max_angular_velocity, ctrl, badctrl);
  STAMP(1);

  // mj_checkPos / mj_checkVel: bad state -> mj_resetData (qpos0, zero velocity/warmstart/ctrl)
  bool bad_state = false;
#pragma unroll
  for (int i = 0; i < 13; i++) bad_state |= is_bad(qpos[i]);
#pragma unroll
  for (int i = 0; i < NV; i++) bad_state |= is_bad(qvel[i]);
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    if (bad_state) {
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = QPOS0[i];
#pragma unroll
      for (int i = 0; i < NV; i++) { qvel[i] = 0.0f; warm[i] = 0.0f; }
      ctrl[0] = ctrl[1] = ctrl[2] = 0.0f;
    }
    // kinematics (pre-integration)
    float q[4] = {qpos[3], qpos[4], qpos[5], qpos[6]};
    normq(q);
    float R[9];
    quat_R(q, R);
    // u = (R^T v, w, hinges)
    float u[NV], wu[NV];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      u[k] = R[k] * qvel[0] + R[3 + k] * qvel[1] + R[6 + k] * qvel[2];
      wu[k] = R[k] * warm[0] + R[3 + k] * warm[1] + R[6 + k] * warm[2];
    }
#pragma unroll
    for (int i = 3; i < NV; i++) { u[i] = qvel[i]; wu[i] = warm[i]; }
    StepResult res;
    dynamics<0>(S, qpos, u, wu, R, ctrl, A.flags, res);
    if (res.bad && pass == 0) { bad_state = true; continue; }

    STAMP(8);
    float p[3] = {qpos[0], qpos[1], qpos[2]};
    euler_advance(u, res, R, qpos, qvel, warm);
    obs_pose(A.flags, qpos, p, q, R);
    const uint32_t nstep = step + 1;
    const bool trunc = nstep >= (uint32_t)A.prm.max_episode_steps;
    float head[7];
    ObsOut oh = observe_head(p, q, R, gx, gy, ref, head, A.prm);
    const bool done_pre = oh.term || trunc;
    const bool autoreset = (A.flags & F_AUTORESET) && done_pre;
    const Soa obs = soa(A.obs, NOBS, n);
    ObsOut o = observe<0>(p, q, R, gx, gy, ref, obs, vo, A.prm);
    if (A.tobs) copy_terminal_obs(obs, soa(A.tobs, NOBS, n), vo, autoreset);
    stf(soa(A.reward, 1, n), 0, vo, o.reward);
    stb(soa(A.term, 1, n, 1), (uint32_t)e, o.term ? 1 : 0);
    stb(soa(A.trunc, 1, n, 1), (uint32_t)e, trunc ? 1 : 0);
    if (A.ep) {
      // Monitor-wrapper episode bookkeeping (train.py:70): r/l of finished episodes
      const Soa ep = soa(A.ep, 4, n);
      float ret = ldf(ep, 0, vo) + o.reward, len = ldf(ep, 1, vo) + 1.0f;
      if (o.term || trunc) {
        stf(ep, 2, vo, ldf(ep, 2, vo) + ret);
        stf(ep, 3, vo, ldf(ep, 3, vo) + 1.0f);
        ret = 0.0f;
        len = 0.0f;
      }
      stf(ep, 0, vo, ret);
      stf(ep, 1, vo, len);
    }
    if (A.info) {
      const Soa inf = soa(A.info, 4, n);
      stf(inf, 0, vo, o.minl);
      stf(inf, 1, vo, o.coll ? 1.0f : 0.0f);
      stf(inf, 2, vo, o.dist);
      stf(inf, 3, vo, bad_state ? 1.0f : 0.0f);
    }

    STAMP(9);
    if (autoreset) {
      reset_env<0>(st, obs, vo, A.seed, A.env_offset + e, episode + 1, A.prm);
      return;
    }
#pragma unroll
    for (int i = 0; i < 13; i++) stf(st, ST_QPOS + i, vo, qpos[i]);
#pragma unroll
    for (int i = 0; i < NV; i++) stf(st, ST_QVEL + i, vo, qvel[i]);
#pragma unroll
    for (int i = 0; i < NV; i++) stf(st, ST_WARM + i, vo, warm[i]);
    stf(st, ST_STEP, vo, __uint_as_float(nstep));
    STAMP(10);
    return;
  }
}

// Wave-specialised step (default flags): a 128-lane workgroup holds 64 envs twice. Wave 0 runs the
// dynamics (controller, Newton, Euler) and writes the state; wave 1, on another SIMD of the CU, runs
// the observation of the same envs -- odometry, the 72 rays, reward, done flags, Monitor stats --
// which mj_step takes at the PRE-integration pose (a10-a13), so it needs nothing from wave 0 except
// in two places, exchanged through LDS at two barriers:
//   barrier 1: wave 0 -> wave 1 "this env's dynamics blew up" (mj_checkAcc -> mj_resetData: the
//              step is redone from qpos0, so its observation is taken at qpos0 too; rare);
//   barrier 2: wave 1 -> wave 0 "auto-reset this env" (term from the goal distance, trunc), after
//              wave 1 has written obs, so wave 0's reset observation lands last.
// The observation leaves the critical path (~20 % of the serial step).
// true if some env of the workgroup (npair dynamics waves x 64) was redone: the same answer in
// every wave, so the conditional barrier 2 is workgroup-uniform
__device__ __forceinline__ bool any_redo(const uint8_t* sh_bad, int lane, int npair) {
  bool r = false;
  for (int w = 0; w < npair; w++) r |= sh_bad[w * 64 + lane] != 0;
  return r;
}

// The lane kernels' helper waves, each measured faster than without it: a third
// "prep" wave computes the controller and the scalar rows (LDS + flag), factors M + h diag(damping)
// for the Euler solve (flag 2) and casts rays 10 .. PREP_RAYS-1; the observation wave factors M for
// qacc_smooth (flag 3) before its observation. (Measured and dropped, rounds 2-3: the prep wave
// factoring the typical predicted piece, 4.52 -> 4.79-4.97 us per step; the observation wave
// computing the bias forces, 4.52 -> 5.03 us.)
constexpr int PREP_RAYS = 40;
constexpr int XEU_OFF = (XCH_WORDS + 1) * 64;  // float offset of the Euler factor words in xch
constexpr int XM_OFF = XEU_OFF + 4 * EU_VEC * 64;  // ... and of the mass-matrix factor
constexpr int XCH_FLOATS = XM_OFF + 4 * EU_VEC * 64;

template <int NC>
__device__ __forceinline__ void step_dyn_wave(const Args& A, float* lds, float* xch, int* xflag, uint8_t* sh_bad,
                                              const uint8_t* sh_reset, int lane, int e, bool valid, int slot,
                                              int npair) {
  STAMP_SCOPE_A(A)
  const int n = A.n;
  Slots S{lds + lane};
  const uint32_t vo = 4u * (uint32_t)e;
  const Soa st = soa(A.state, NSTATE, n);
  float qpos[13], qvel[NV], warm[NV];
  bool redo = false, bad_state = false;
  uint32_t step = 0, episode = 0;
  float R[9], u[NV], wu[NV], ctrl[3] = {0.0f, 0.0f, 0.0f};
  DynPre P;
  if (lane == 0) { xflag[0] = 0; xflag[1] = 0; xflag[2] = 0; xflag[3] = 0; xflag[4] = 0; }
  __syncthreads();  // barrier 0: the exchange flags are clear before the prep wave can raise them
  const int sms = 64 * npair;  // word stride of the LDS state mirrors
  float* const smw = A.sm ? A.sm + slot : nullptr;
  float* const smn = A.sm_next ? A.sm_next + slot : nullptr;
  if (valid) {
    STAMP(0);
    if (A.sm_in) {
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = smw[(ST_QPOS + i) * sms];
#pragma unroll
      for (int i = 0; i < NV; i++) qvel[i] = smw[(ST_QVEL + i) * sms];
#pragma unroll
      for (int i = 0; i < NV; i++) warm[i] = smw[(ST_WARM + i) * sms];
      step = __float_as_uint(smw[ST_STEP * sms]);
      episode = __float_as_uint(smw[ST_EPIS * sms]);
    } else {
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = ldf(st, ST_QPOS + i, vo);
#pragma unroll
      for (int i = 0; i < NV; i++) qvel[i] = ldf(st, ST_QVEL + i, vo);
#pragma unroll
      for (int i = 0; i < NV; i++) warm[i] = ldf(st, ST_WARM + i, vo);
      step = __float_as_uint(ldf(st, ST_STEP, vo));
      episode = __float_as_uint(ldf(st, ST_EPIS, vo));
      if (A.sm_out) {  // first step of a rollout launch: the words only a reset changes, into both mirrors
#pragma unroll
        for (int k = 0; k < 5; k++) {
          const float v = ldf(st, ST_GOAL + k, vo);
          smw[(ST_GOAL + k) * sms] = v;
          smn[(ST_GOAL + k) * sms] = v;
        }
        smw[ST_EPIS * sms] = __uint_as_float(episode);
        smn[ST_EPIS * sms] = __uint_as_float(episode);
      }
    }
    STAMP(1);
#pragma unroll
    for (int i = 0; i < 13; i++) bad_state |= is_bad(qpos[i]);
#pragma unroll
    for (int i = 0; i < NV; i++) bad_state |= is_bad(qvel[i]);
    if (bad_state) reset_to_qpos0(qpos, qvel, warm, ctrl);  // mj_checkPos / mj_checkVel -> mj_resetData
    to_u(qpos, qvel, warm, R, u, wu);
    dyn_pre(qpos, u, R, P);
  }
  ScalRows sr;
  {
    // the prep wave has put this env's controller output and scalar rows into LDS (computed from
    // the loaded state; an env reset for a bad state computes its own at qpos0): wait for its flag
    STAMP(20);
    while (__hip_atomic_load(xflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
    STAMP(15);
    float xc[3];
    xch_get(xch, slot, 64, sr, xc);
    if (bad_state) scalar_rows(qpos, u, sr);
    else {
      ctrl[0] = xc[0]; ctrl[1] = xc[1]; ctrl[2] = xc[2];
    }
  }
  if (valid) {
    StepResult res;
    dyn_post<NC, true, true>(S, P, qpos, u, wu, R, ctrl, A.flags, sr, res, EuHand{xch + XEU_OFF, xflag + 2, lane},
                             EuHand{xch + XM_OFF, xflag + 3, lane});
    if (res.bad) {  // mj_checkAcc: mj_resetData and the step redone from qpos0 (rare)
      bad_state = redo = true;
      reset_to_qpos0(qpos, qvel, warm, ctrl);
      to_u(qpos, qvel, warm, R, u, wu);
      dynamics<NC>(S, qpos, u, wu, R, ctrl, A.flags, res);
    }
    euler_advance(u, res, R, qpos, qvel, warm);
    if (A.sm_out) {  // rollout, not the launch's last step: the next step reads the state from LDS
#pragma unroll
      for (int i = 0; i < 13; i++) smn[(ST_QPOS + i) * sms] = qpos[i];
#pragma unroll
      for (int i = 0; i < NV; i++) smn[(ST_QVEL + i) * sms] = qvel[i];
#pragma unroll
      for (int i = 0; i < NV; i++) smn[(ST_WARM + i) * sms] = warm[i];
      smn[ST_STEP * sms] = __uint_as_float(step + 1);
    }
    STAMP(8);
  }
  sh_bad[slot] = redo ? 1 : 0;
  __syncthreads();  // 1: wave 1 has written obs and the auto-reset decisions; it learns the redos
  // 2 (only when some env of the workgroup was redone; every wave reads the same bytes): wave 1
  // has re-observed the redone envs at qpos0 and revised their auto-reset decisions
  if (__builtin_amdgcn_ballot_w64(any_redo(sh_bad, lane, npair)) != 0ull) __syncthreads();
  if (!valid) return;
  STAMP(9);
  if (sh_reset[slot]) {
    reset_env<0>(st, soa(A.obs, NOBS, n), vo, A.seed, A.env_offset + e, episode + 1, A.prm, A.sm_out ? smn : nullptr,
                 sms);
    if (A.sm_out) {  // the reset words into the other mirror too (goal, odometry reference, episode live on)
#pragma unroll
      for (int w = 0; w < NSTATE; w++) smw[w * sms] = smn[w * sms];
    }
    return;
  }
  if (A.sm_out) return;  // the state is in the next step's LDS mirror
#pragma unroll
  for (int i = 0; i < 13; i++) stf(st, ST_QPOS + i, vo, qpos[i]);
#pragma unroll
  for (int i = 0; i < NV; i++) stf(st, ST_QVEL + i, vo, qvel[i]);
#pragma unroll
  for (int i = 0; i < NV; i++) stf(st, ST_WARM + i, vo, warm[i]);
  stf(st, ST_STEP, vo, __uint_as_float(step + 1));
  STAMP(10);
}

__device__ __forceinline__ void step_obs_wave(const Args& A, float* xch, int* xflag, const uint8_t* sh_bad,
                                              uint8_t* sh_reset, int lane, int e, bool valid, int slot, int npair) {
  STAMP_SCOPE_A(A)
  __syncthreads();  // barrier 0 (see step_dyn_wave)
  const int n = A.n;
  const uint32_t vo = 4u * (uint32_t)e;
  const Soa st = soa(A.state, NSTATE, n);
  const Soa obs = soa(A.obs, NOBS, n);
  float qpos[13];
  float gx = 0.0f, gy = 0.0f, ref[3] = {0.0f, 0.0f, 0.0f};
  uint32_t step = 0;
  bool bad_state = false;
  float ep0 = 0.0f, ep1 = 0.0f, ep2 = 0.0f, ep3 = 0.0f;
  const Soa ep = soa(A.ep, 4, n);
  float qvel[NV];
  if (valid) {
    // rollout steps after a launch's first read the LDS state mirror instead (same words)
    if (A.sm_in) {
      const float* smr = A.sm + slot;
      const int sms = 64 * npair;
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = smr[(ST_QPOS + i) * sms];
#pragma unroll
      for (int i = 0; i < NV; i++) qvel[i] = smr[(ST_QVEL + i) * sms];
      gx = smr[ST_GOAL * sms];
      gy = smr[(ST_GOAL + 1) * sms];
#pragma unroll
      for (int k = 0; k < 3; k++) ref[k] = smr[(ST_REF + k) * sms];
      step = __float_as_uint(smr[ST_STEP * sms]);
    } else {
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = ldf(st, ST_QPOS + i, vo);
#pragma unroll
      for (int i = 0; i < NV; i++) qvel[i] = ldf(st, ST_QVEL + i, vo);
      gx = ldf(st, ST_GOAL, vo);
      gy = ldf(st, ST_GOAL + 1, vo);
#pragma unroll
      for (int k = 0; k < 3; k++) ref[k] = ldf(st, ST_REF + k, vo);
      step = __float_as_uint(ldf(st, ST_STEP, vo));
    }
    if (A.ep) { ep0 = ldf(ep, 0, vo); ep1 = ldf(ep, 1, vo); ep2 = ldf(ep, 2, vo); ep3 = ldf(ep, 3, vo); }
    // mj_checkPos / mj_checkVel on the loaded state (the same test as wave 0's)
#pragma unroll
    for (int i = 0; i < 13; i++) bad_state |= is_bad(qpos[i]);
#pragma unroll
    for (int i = 0; i < NV; i++) bad_state |= is_bad(qvel[i]);
  }
  {  // chol(M) for the dynamics wave's qacc_smooth, at qpos0 for a reset state
    if (valid) {
      float L[NV][NV];
      mass_factor<false>(bad_state ? QPOS0[W_STEER_QPOS[2]] : qpos[W_STEER_QPOS[2]],
                         bad_state ? QPOS0[W_STEER_QPOS[3]] : qpos[W_STEER_QPOS[3]], L);
      eu_put(xch + XM_OFF, lane, L);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(xflag + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const uint32_t nstep = step + 1;
  const bool trunc = nstep >= (uint32_t)A.prm.max_episode_steps;
  ObsOut o{};
  bool redo = false, autoreset = false;
#pragma unroll 1
  for (int pass = 0; pass < 2; pass++) {
    if (bad_state || redo) {
#pragma unroll
      for (int i = 0; i < 7; i++) qpos[i] = QPOS0[i];
    }
    if (valid && (pass == 0 || redo)) {
      float p[3] = {qpos[0], qpos[1], qpos[2]};
      float q[4] = {qpos[3], qpos[4], qpos[5], qpos[6]};
      normq(q);
      float R[9];
      quat_R(q, R);
      if (pass == 0) {
        o = observe<0, PREP_RAYS>(p, q, R, gx, gy, ref, obs, vo, A.prm, [&]() __attribute__((always_inline)) {
          // the prep wave's rays: written to obs and their minimum to LDS before it raised flag 1
          while (__hip_atomic_load(xflag + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
            __builtin_amdgcn_s_sleep(1);
          STAMP(19);
          return xch[XCH_WORDS * 64 + lane];
        });
      } else {
        o = observe<0>(p, q, R, gx, gy, ref, obs, vo, A.prm);  // redone env: every ray at qpos0
      }
      stf(soa(A.reward, 1, n), 0, vo, o.reward);
      stb(soa(A.term, 1, n, 1), (uint32_t)e, o.term ? 1 : 0);
      stb(soa(A.trunc, 1, n, 1), (uint32_t)e, trunc ? 1 : 0);
      if (A.info) {
        const Soa inf = soa(A.info, 4, n);
        stf(inf, 0, vo, o.minl);
        stf(inf, 1, vo, o.coll ? 1.0f : 0.0f);
        stf(inf, 2, vo, o.dist);
        stf(inf, 3, vo, (bad_state || redo) ? 1.0f : 0.0f);
      }
      autoreset = (A.flags & F_AUTORESET) && (o.term || trunc);
    }
    // terminal obs before wave 0 may overwrite obs with the reset observation
    if (A.tobs) copy_terminal_obs(obs, soa(A.tobs, NOBS, n), vo, autoreset && (pass == 0 || redo));
    sh_reset[slot] = autoreset ? 1 : 0;
    __syncthreads();  // pass 0: barrier 1; pass 1: barrier 2 (see step_dyn_wave)
    if (pass == 1) break;
    if (__builtin_amdgcn_ballot_w64(any_redo(sh_bad, lane, npair)) == 0ull) break;
    redo = valid && sh_bad[slot];
  }
  if (valid && A.ep) {
    // Monitor-wrapper episode bookkeeping (train.py:70): r/l of finished episodes
    float ret = ep0 + o.reward, len = ep1 + 1.0f;
    if (o.term || trunc) {
      stf(ep, 2, vo, ep2 + ret);
      stf(ep, 3, vo, ep3 + 1.0f);
      ret = 0.0f;
      len = 0.0f;
    }
    stf(ep, 0, vo, ret);
    stf(ep, 1, vo, len);
  }
}

// F_POSTSTEP_OBS (render_mode="human"): one lane per env runs the whole step
extern "C" __global__ void __launch_bounds__(64, 1) ackphys_step_serial_kernel(Args A) {
  __shared__ float lds[NSLOT * NF * 64];
  const int lane = threadIdx.x;
  const int e = blockIdx.x * A.epw + lane;
  if (lane >= A.epw || e >= A.n) return;
  step_serial(A, lds, lane, e);
}

// Prep wave: the controller (float64) and the scalar constraint rows of the same 64 envs,
// off the dynamics wave's critical path -- they need only the action and the hinge positions and
// speeds. Handed over through LDS and a workgroup-scope release / acquire flag (no barrier: the
// observation wave must not wait for it). Then the implicit-Euler factor, which the
// dynamics wave needs only after its solve (flag 2), and (PREP_RAYS) rangefinders for the
// observation wave (flag 1); the wave joins barriers 1 and 2 and exits.
template <int NC>
__device__ __forceinline__ void step_prep_wave(const Args& A, float* xch, int* xflag, const uint8_t* sh_bad, int lane,
                                               int e, bool valid) {
  STAMP_SCOPE_A(A)
  __syncthreads();  // barrier 0 (see step_dyn_wave)
  const int n = A.n;
  const uint32_t vo = 4u * (uint32_t)e;
  const Soa st = soa(A.state, NSTATE, n);
  float qpos[13];
  bool bad = false;
  ScalRows sr;
  if (valid) {
    float qvel[NV];
    if (A.sm_in) {  // rollout: LDS state mirror (one wave pair)
      const float* smr = A.sm + lane;
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = smr[(ST_QPOS + i) * 64];
#pragma unroll
      for (int i = 0; i < NV; i++) qvel[i] = smr[(ST_QVEL + i) * 64];
    } else {
#pragma unroll
      for (int i = 0; i < 13; i++) qpos[i] = ldf(st, ST_QPOS + i, vo);
#pragma unroll
      for (int i = 0; i < NV; i++) qvel[i] = ldf(st, ST_QVEL + i, vo);
    }
    float ctrl[3];
    if (A.nctrl && A.sm_in) {  // rollout: computed during the previous step
#pragma unroll
      for (int j = 0; j < 3; j++) ctrl[j] = A.nctrl[j * 64 + lane];
      STAMP(21);
    } else {
      const Soa act = soa(A.action, 2, n);
      const float a0 = ldf(act, 0, 2 * vo), a1 = ldf(act, 0, 2 * vo + 4);
      bool badctrl;
      STAMP(21);
      controller(a0, a1, A.prm.max_linear_velocity, A.prm.max_angular_velocity, ctrl, badctrl);
    }
    STAMP(22);
    scalar_rows(qpos, qvel, sr);  // hinge dofs only: u = qvel there
    STAMP(23);
    xch_put(xch, lane, 64, sr, ctrl);
    // mj_checkPos / mj_checkVel (the dynamics wave's test): a reset state is factored / observed at qpos0
#pragma unroll
    for (int i = 0; i < 13; i++) bad |= is_bad(qpos[i]);
#pragma unroll
    for (int i = 0; i < NV; i++) bad |= is_bad(qvel[i]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // every lane's exchange words before the flag
  if (lane == 0) __hip_atomic_store(xflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  STAMP(13);
  if (valid && bad) {
#pragma unroll
    for (int i = 0; i < 13; i++) qpos[i] = QPOS0[i];
  }
  {
    if (valid) {
      float L[NV][NV];
      euler_factor(qpos, L);
      eu_put(xch + XEU_OFF, lane, L);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(xflag + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    STAMP(16);
  }
  {
    // rangefinders 10 .. PREP_RAYS-1 of the observation (taken at the pre-integration pose, or at
    // qpos0 for a state mj_checkPos/Vel resets): stored here, their minimum handed to wave 1
    float mn = 3.0e38f;
    if (valid) {
      const float p[3] = {qpos[0], qpos[1], qpos[2]};
      float q[4] = {qpos[3], qpos[4], qpos[5], qpos[6]};
      normq(q);
      float R[9];
      quat_R(q, R);
      const Soa obs = soa(A.obs, NOBS, n);
      const RayFrame F = ray_frame(p, R);
      if (__builtin_amdgcn_ballot_w64(!floor_rays_all_miss(p, R)) == 0ull) {
#pragma unroll
        for (int i = 10; i < PREP_RAYS; i++) stf(obs, i, vo, -1.0f);
        mn = coll_reading(-1.0f, A.prm);
      } else {
#pragma unroll
        for (int i = 10; i < PREP_RAYS; i++) {
          const float v = ray_floor_f(F, RAY_DIR[i][0], RAY_DIR[i][1]);
          stf(obs, i, vo, v);
          mn = fminf(mn, coll_reading(v, A.prm));
        }
      }
    }
    xch[XCH_WORDS * 64 + lane] = mn;
    __builtin_amdgcn_s_waitcnt(0);  // the observation rows are written (wave 1 may copy them as terminal obs)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(xflag + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    STAMP(14);
  }
  if (A.next_action && valid) {  // rollout: the next step's controller, off that step's critical path
    const Soa act = soa(A.next_action, 2, n);
    const float a0 = ldf(act, 0, 2 * vo), a1 = ldf(act, 0, 2 * vo + 4);
    float c[3];
    bool badctrl;
    controller(a0, a1, A.prm.max_linear_velocity, A.prm.max_angular_velocity, c, badctrl);
#pragma unroll
    for (int j = 0; j < 3; j++) A.nctrl[j * 64 + lane] = c[j];
  }
  __syncthreads();                                                           // barrier 1
  if (__builtin_amdgcn_ballot_w64(any_redo(sh_bad, lane, 1)) != 0ull) __syncthreads();  // barrier 2
}

// PW wave pairs per workgroup: waves 0..PW-1 run the dynamics of envs [64 w, 64 w + 64) of the
// block, waves PW..2PW-1 their observations (2 PW waves on the CU's 4 SIMDs); a third wave
// (PW = 1) prepares the controller and scalar rows
template <int NC, int PW>
__device__ __forceinline__ void step_split(const Args& A) {
  static_assert(PW == 1, "the prep wave serves one dynamics wave");
  __shared__ float lds[NC ? 1 : NSLOT * NF * 64];
  __shared__ __attribute__((aligned(16))) float xch[XCH_FLOATS];
  __shared__ int xflag[5];
  __shared__ uint8_t sh_bad[64 * PW], sh_reset[64 * PW];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int pair = wave % PW, slot = pair * 64 + lane;
  const int e = blockIdx.x * (A.epw * PW) + pair * A.epw + lane;
  const bool valid = lane < A.epw && e < A.n;
  if (wave < PW) step_dyn_wave<NC>(A, lds, xch, xflag, sh_bad, sh_reset, lane, e, valid, slot, PW);
  else if (wave < 2 * PW) step_obs_wave(A, xch, xflag, sh_bad, sh_reset, lane, e, valid, slot, PW);
  else step_prep_wave<NC>(A, xch, xflag, sh_bad, lane, blockIdx.x * A.epw + lane, lane < A.epw && blockIdx.x * A.epw + lane < A.n);
}
constexpr int LANE_THREADS = 64 * 3;  // dynamics, observation and prep wave
extern "C" __global__ void __launch_bounds__(LANE_THREADS, 1) ackphys_step_kernel(Args A) {
  step_split<0, 1>(A);
}
// contacts off (BASELINE configs[1]): the contact machinery is compiled out
extern "C" __global__ void __launch_bounds__(LANE_THREADS, 1) ackphys_step_nc_kernel(Args A) {
  step_split<1, 1>(A);
}

// Rollout kernels (ackphys_rollout): A.ksteps consecutive steps of the same envs in one launch,
// each one exactly the single-step kernel's work with its own action row and output slices. The
// state goes through HBM (L1/L2 hits) between steps as between launches; what a step costs less is
// the launch: dispatch, wave start-up and the drain of the whole grid. Step k + 1's prep and
// observation waves load the state the dynamics wave stored in step k: with the prep wave that
// store precedes barrier 0 of step k + 1, which the loading waves pass first (same CU, so the
// workgroup-scope fence of the barrier suffices). Between steps the state lives in an LDS mirror
// (double-buffered), not HBM; only the launch's last step stores it.
template <int NC, int PW>
__device__ __forceinline__ void rollout_split(const Args& A) {
  __shared__ float sm[2][NSTATE * 64 * PW];
  __shared__ float nctrl[3 * 64];
#pragma unroll 1
  for (int k = 0; k < A.ksteps; k++) {
    Args B = step_args(A, k);
    B.sm = sm[k & 1];
    B.sm_next = sm[(k + 1) & 1];
    B.sm_in = k > 0;
    B.sm_out = k + 1 < A.ksteps;
    B.nctrl = nctrl;
    B.next_action = k + 1 < A.ksteps ? A.action + (size_t)(k + 1) * 2 * A.n : nullptr;
#ifdef AK_STAMPS  // the stamps kept are a mid-rollout step's (state into the LDS mirror, not HBM)
    B.stamp_skip = A.ksteps > 1 && k != A.ksteps - 2;
#endif
    step_split<NC, PW>(B);
  }
}
extern "C" __global__ void __launch_bounds__(LANE_THREADS, 1) ackphys_rollout_nc_kernel(Args A) {
  rollout_split<1, 1>(A);
}
extern "C" __global__ void __launch_bounds__(LANE_THREADS, 1) ackphys_rollout_kernel(Args A) {
  rollout_split<0, 1>(A);
}

template <int SC>
__device__ __forceinline__ void reset_body(const uint8_t* mask, float* state, float* obs, int n, uint64_t seed,
                                           int64_t env_offset, const EnvParams& prm) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  if (mask && !mask[e]) return;
  const Soa st = soa(state, NSTATE, n), ob = soa(obs, NOBS, n);
  const uint32_t vo = 4u * (uint32_t)e;
  const uint32_t episode = __float_as_uint(ldf(st, ST_EPIS, vo)) + 1u;
  reset_env<SC>(st, ob, vo, seed, env_offset + e, episode, prm);
}
extern "C" __global__ void __launch_bounds__(256) ackphys_reset_kernel(const uint8_t* mask, float* state, float* obs,
                                                                       int n, uint64_t seed, int64_t env_offset,
                                                                       EnvParams prm) {
  reset_body<0>(mask, state, obs, n, seed, env_offset, prm);
}
extern "C" __global__ void __launch_bounds__(256) ackphys_reset_obst_kernel(const uint8_t* mask, float* state,
                                                                            float* obs, int n, uint64_t seed,
                                                                            int64_t env_offset, EnvParams prm) {
  reset_body<1>(mask, state, obs, n, seed, env_offset, prm);
}

extern "C" __global__ void __launch_bounds__(256) ackphys_actions_kernel(float* actions, int n, int k_steps,
                                                                         uint64_t seed, uint32_t step0, int64_t env_offset) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  for (int k = 0; k < k_steps; k++) {
    uint32_t c[4] = {(uint32_t)(env_offset + e), step0 + (uint32_t)k, 1u, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float2 v = make_float2(2.0f * u01(c[0]) - 1.0f, 2.0f * u01(c[1]) - 1.0f);
    reinterpret_cast<float2*>(actions)[(size_t)k * n + e] = v;
  }
}

// ====================================================================== C-ABI (include/ackphys.h)
#include "../../include/ackphys.h"
#include "../../include/ackphys_model.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct ackphys_ctx {
  int n_env;
  int device;
  int64_t env_offset;
  ak::EnvParams prm;
  int variant;  // ACKPHYS_VARIANT_LANE (1 lane/env) or ACKPHYS_VARIANT_QUAD (4 lanes/env)
  int scene;    // 0: ackermann_robot_v2 (floor only); 1: obstacle scene (floor + boxes)
  float* pimg = nullptr;  // ackphys_ppo_rollout: the policy's weight image (allocated at the first call)
};

static thread_local char g_err[512];
static int fail(int code, const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return code;
}
static int hipfail(hipError_t e, const char* where) {
  snprintf(g_err, sizeof g_err, "%s: %s", where, hipGetErrorString(e));
  return ACKPHYS_EHIP;
}

// Switches the calling thread to the context's device only when it differs, and restores the
// caller's device on return (torch keeps its own notion of the current device).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

static uint64_t fnv1a64(const unsigned char* p, size_t n) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 0x100000001B3ull; }
  return h;
}

extern "C" {

const char* ackphys_last_error(void) { return g_err; }
#ifdef AK_STAMPS
int ackphys_diag_set_stamps(void* buf) {
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf));
  return e == hipSuccess ? 0 : hipfail(e, "hipMemcpyToSymbol");
}
int ackphys_diag_set_dump(void* buf) {
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_dump), &buf, sizeof(buf));
  return e == hipSuccess ? 0 : hipfail(e, "hipMemcpyToSymbol");
}
#endif

const char* ackphys_version(void) {
  return "ackphys 0.3 (gfx950; step kernels: lane-per-env, quad-per-env; scenes: v2 floor, obstacles)";
}
uint64_t ackphys_model_fnv(void) { return apg::MODEL_FNV; }

int ackphys_create(const void* model_blob, size_t nbytes, int n_env, int device, ackphys_t** out) {
  if (!out) return fail(ACKPHYS_EINVAL, "out is NULL");
  *out = nullptr;
  if (!model_blob || nbytes < sizeof(apm_model_t)) return fail(ACKPHYS_EMODEL, "model blob missing or too small");
  const apm_model_t* m = (const apm_model_t*)model_blob;
  if (m->magic != APM_MAGIC || m->version != APM_VERSION || m->nbytes != nbytes)
    return fail(ACKPHYS_EMODEL, "model blob: bad magic/version/size");
  const uint64_t h = fnv1a64((const unsigned char*)model_blob, nbytes);
  int scene = -1;
  if (h == apg::MODEL_FNV) scene = 0;
  else if (h == apg::scene1::SCENE_FNV) scene = 1;
  if (scene < 0)
    return fail(ACKPHYS_EMODEL, "model blob does not match a model these kernels were specialised on "
                                "(regenerate with python -m mujoco_playground_amd.model.build and rebuild)");
  if (n_env <= 0) return fail(ACKPHYS_EINVAL, "n_env must be positive");
  // buffer descriptors address [79][N] float arrays with 31-bit byte ranges
  if (n_env > ACKPHYS_MAX_ENVS) return fail(ACKPHYS_EINVAL, "n_env exceeds ACKPHYS_MAX_ENVS");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hipfail(e, "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return fail(ACKPHYS_EINVAL, "device index out of range");
  ackphys_ctx* c = new ackphys_ctx;
  c->n_env = n_env;
  c->device = device;
  c->env_offset = 0;
  c->prm = ak::EnvParams{1000, 0.5f, 0.15f, 1.0f, 1.0f};  // AckermannRobotEnv defaults
  c->variant = ACKPHYS_VARIANT_AUTO;
  c->scene = scene;
  *out = c;
  return ACKPHYS_OK;
}

int ackphys_destroy(ackphys_t* ctx) {
  if (ctx && ctx->pimg) {
    DeviceGuard dg(ctx->device);
    (void)hipFree(ctx->pimg);
  }
  delete ctx;
  return ACKPHYS_OK;
}

int ackphys_set_env_params(ackphys_t* ctx, const ackphys_env_params* p) {
  if (!ctx || !p) return fail(ACKPHYS_EINVAL, "ackphys_set_env_params: NULL argument");
  if (p->max_episode_steps <= 0) return fail(ACKPHYS_EINVAL, "max_episode_steps must be positive");
  if (p->action_repeat < 1 || p->action_repeat > 1000) return fail(ACKPHYS_EINVAL, "action_repeat must be in [1, 1000]");
  if (p->goal_cells < 0) return fail(ACKPHYS_EINVAL, "goal_cells must be >= 0");
  if (p->goal_cells > 0 && ctx->scene != 1) return fail(ACKPHYS_EINVAL, "goal_cells needs the obstacle scene (maze cells)");
  ctx->prm = ak::EnvParams{p->max_episode_steps, (float)p->goal_distance_threshold, (float)p->collision_threshold,
                           (float)p->max_linear_velocity, (float)p->max_angular_velocity, p->action_repeat,
                           p->nohit_clear ? 1 : 0, p->goal_cells};
  return ACKPHYS_OK;
}

int ackphys_set_variant(ackphys_t* ctx, int variant) {
  if (!ctx) return fail(ACKPHYS_EINVAL, "ctx is NULL");
  if (variant != ACKPHYS_VARIANT_LANE && variant != ACKPHYS_VARIANT_QUAD && variant != ACKPHYS_VARIANT_AUTO &&
      variant != ACKPHYS_VARIANT_LANE16)
    return fail(ACKPHYS_EINVAL, "bad variant");
  ctx->variant = variant;
  return ACKPHYS_OK;
}

int ackphys_set_env_offset(ackphys_t* ctx, int64_t off) {
  if (!ctx) return fail(ACKPHYS_EINVAL, "ctx is NULL");
  ctx->env_offset = off;
  return ACKPHYS_OK;
}

// One launch of a.ksteps steps: the rollout kernels when ksteps > 1 (the post-step-observation mode
// has none: its K single-step launches run back to back on the stream, same results).
static int launch_steps(ackphys_t* ctx, ak::Args a, uint32_t flags, void* stream);

int ackphys_step(ackphys_t* ctx, const float* action, float* state, float* obs, float* reward, uint8_t* term,
                 uint8_t* trunc, float* terminal_obs, float* info, float* episode, uint32_t flags, uint64_t seed,
                 void* stream) {
  if (!ctx || !action || !state || !obs || !reward || !term || !trunc)
    return fail(ACKPHYS_EINVAL, "ackphys_step: NULL argument");
  DeviceGuard dg(ctx->device);
  if (dg.err != hipSuccess) return hipfail(dg.err, "hipSetDevice");
  ak::Args a{action, state, obs, reward, term, trunc, terminal_obs, info, episode, ctx->prm, ctx->n_env, flags, seed,
             ctx->env_offset, 64};
  return launch_steps(ctx, a, flags, stream);
}

int ackphys_rollout(ackphys_t* ctx, int k_steps, const float* actions, float* state, float* obs, float* reward,
                    uint8_t* term, uint8_t* trunc, float* terminal_obs, float* info, float* episode, uint32_t flags,
                    uint64_t seed, int per_step_outputs, void* stream) {
  if (!ctx || !actions || !state || !obs || !reward || !term || !trunc)
    return fail(ACKPHYS_EINVAL, "ackphys_rollout: NULL argument");
  if (k_steps <= 0) return fail(ACKPHYS_EINVAL, "ackphys_rollout: k_steps must be positive");
  DeviceGuard dg(ctx->device);
  if (dg.err != hipSuccess) return hipfail(dg.err, "hipSetDevice");
  ak::Args a{actions, state, obs, reward, term, trunc, terminal_obs, info, episode, ctx->prm, ctx->n_env, flags, seed,
             ctx->env_offset, 64};
  a.ksteps = k_steps;
  a.per_step = per_step_outputs ? 1 : 0;
  if (flags & ACKPHYS_POSTSTEP_OBS) {
    const size_t n = (size_t)ctx->n_env;
    for (int k = 0; k < k_steps; k++) {
      ak::Args b = a;
      b.ksteps = 1;
      b.per_step = 0;
      b.action = actions + (size_t)k * 2 * n;
      if (a.per_step) {
        b.obs = obs + (size_t)k * ACKPHYS_NOBS * n;
        b.reward = reward + (size_t)k * n;
        b.term = term + (size_t)k * n;
        b.trunc = trunc + (size_t)k * n;
        if (terminal_obs) b.tobs = terminal_obs + (size_t)k * ACKPHYS_NOBS * n;
        if (info) b.info = info + (size_t)k * 4 * n;
      }
      const int rc = launch_steps(ctx, b, flags, stream);
      if (rc) return rc;
    }
    return ACKPHYS_OK;
  }
  return launch_steps(ctx, a, flags, stream);
}

// Envs per quad wave. Per-step launches: 16 (a step lasts as long as the slowest wave, and more
// waves with fewer envs measured slower). Rollout launches: 8, i.e. 512 workgroups, two or more
// per CU, all four SIMDs busy, and each wave's per-step Newton maximum taken over 8 envs instead
// of 16: contacts on 39.6 -> 37.2 us per step (tools/quad_epw_sweep.sh). The obstacle scene's
// slot LDS (94 KB at a 64-lane stride) allows one workgroup per CU, so its 8-env rollout kernel
// lays the slots out at a 32-lane stride (47 KB; ackphys_rollout_obst8_kernel); at 16 envs per
// wave and 94 KB, 8 envs had measured 84 us. Since round 3 both scenes' kernels run split quads (8
// lanes per env, QSlots in ackphys_quad.inc): at most 8 envs per wave, per-step launches included.
// ACKPHYS_QUAD_EPW overrides (experiments; <= 8).
static int quad_epw(bool multi, int scene) {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("ACKPHYS_QUAD_EPW");
    v = s ? atoi(s) : 0;
    if (v < 0 || v > 16) v = 0;
  }
  (void)multi;
  (void)scene;
  return v ? (v < 8 ? v : 8) : 8;
}

static int launch_steps(ackphys_t* ctx, ak::Args a, uint32_t flags, void* stream) {
  hipError_t e;
  const bool multi = a.ksteps > 1;
  // AUTO: with contacts the quad mapping wins (contact rows dominate and split 4 ways); without
  // contacts the replicated serial core dominates and one lane per env is marginally faster.
  const bool quad = ctx->variant == ACKPHYS_VARIANT_QUAD ||
                    (ctx->variant == ACKPHYS_VARIANT_AUTO && (flags & ACKPHYS_CONTACTS));
  if (ctx->prm.action_repeat > 1 && (!(quad || ctx->scene == 1) || (flags & ACKPHYS_POSTSTEP_OBS)))
    return fail(ACKPHYS_EINVAL, "action_repeat > 1 runs on the quad mapping with pre-integration observations");
  // the task variant on the quad mapping runs in dedicated rollout kernels (K = 1 for a step)
  if ((ctx->prm.action_repeat > 1 || ctx->prm.nohit_clear) && (quad || ctx->scene == 1) &&
      !(flags & ACKPHYS_POSTSTEP_OBS)) {
    if (ctx->scene == 1 && ctx->variant != ACKPHYS_VARIANT_QUAD && ctx->variant != ACKPHYS_VARIANT_AUTO)
      return fail(ACKPHYS_EINVAL, "the obstacle scene runs on the quad mapping (variant AUTO or QUAD)");
    a.epw = quad_epw(true, ctx->scene);
    if (a.epw > 8) a.epw = 8;  // the 32-lane slot stride / split quads hold 8 envs per wave
    const int blocks = (ctx->n_env + a.epw - 1) / a.epw;
    hipLaunchKernelGGL(ctx->scene == 1 ? ackphys_rollout_obst8_var_kernel : ackphys_rollout_quad_var_kernel,
                       dim3(blocks), dim3(128), 0, (hipStream_t)stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return hipfail(e, "ackphys_rollout_var launch");
    return ACKPHYS_OK;
  }
  if (ctx->scene == 1) {  // the obstacle scene is specialised on the quad mapping only
    if (ctx->variant != ACKPHYS_VARIANT_QUAD && ctx->variant != ACKPHYS_VARIANT_AUTO)
      return fail(ACKPHYS_EINVAL, "the obstacle scene runs on the quad mapping (variant AUTO or QUAD)");
    a.epw = (flags & ACKPHYS_POSTSTEP_OBS) ? 16 : quad_epw(multi, ctx->scene);
    int blocks = (ctx->n_env + a.epw - 1) / a.epw;
    if (flags & ACKPHYS_POSTSTEP_OBS)
      hipLaunchKernelGGL(ackphys_step_obst_serial_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(!multi ? ackphys_step_obst_kernel : ackphys_rollout_obst8_kernel,
                         dim3(blocks), dim3(128), 0, (hipStream_t)stream, a);
  } else if (quad) {
    a.epw = (flags & ACKPHYS_POSTSTEP_OBS) ? 16 : quad_epw(multi, ctx->scene);
    int blocks = (ctx->n_env + a.epw - 1) / a.epw;
    if (flags & ACKPHYS_POSTSTEP_OBS)
      hipLaunchKernelGGL(ackphys_step_quad_serial_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(multi ? ackphys_rollout_quad_kernel : ackphys_step_quad_kernel, dim3(blocks), dim3(128), 0,
                         (hipStream_t)stream, a);
  } else {
    a.epw = ctx->variant == ACKPHYS_VARIANT_LANE16 ? 16 : 64;
    int blocks = (ctx->n_env + a.epw - 1) / a.epw;
    if (flags & ACKPHYS_POSTSTEP_OBS)
      hipLaunchKernelGGL(ackphys_step_serial_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, a);
    else if (flags & ACKPHYS_CONTACTS)
      hipLaunchKernelGGL(multi ? ackphys_rollout_kernel : ackphys_step_kernel, dim3(blocks),
                         dim3(LANE_THREADS), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(multi ? ackphys_rollout_nc_kernel : ackphys_step_nc_kernel, dim3(blocks), dim3(LANE_THREADS),
                         0, (hipStream_t)stream, a);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hipfail(e, "ackphys_step_kernel launch");
  return ACKPHYS_OK;
}

int ackphys_reset(ackphys_t* ctx, const uint8_t* mask, uint64_t seed, float* state, float* obs, void* stream) {
  if (!ctx || !state || !obs) return fail(ACKPHYS_EINVAL, "ackphys_reset: NULL argument");
  DeviceGuard dg(ctx->device);
  if (dg.err != hipSuccess) return hipfail(dg.err, "hipSetDevice");
  hipError_t e;
  int blocks = (ctx->n_env + 255) / 256;
  if (ctx->scene == 1)
    hipLaunchKernelGGL(ackphys_reset_obst_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, mask, state, obs,
                       ctx->n_env, seed, ctx->env_offset, ctx->prm);
  else
    hipLaunchKernelGGL(ackphys_reset_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, mask, state, obs,
                       ctx->n_env, seed, ctx->env_offset, ctx->prm);
  e = hipGetLastError();
  if (e != hipSuccess) return hipfail(e, "ackphys_reset_kernel launch");
  return ACKPHYS_OK;
}

int ackphys_ppo_rollout(ackphys_t* ctx, const float* params, int n_steps, uint32_t step0, uint64_t policy_seed,
                        int deterministic, float gamma, float* state, float* obs, float* reward, uint8_t* term,
                        uint8_t* trunc, float* terminal_obs, float* episode, float* obs_rows, float* actions,
                        float* log_prob, float* value, float* rollout_reward, float* episode_starts, float* last_dones,
                        float* last_values, uint32_t flags, uint64_t seed, void* stream) {
  if (!ctx || !params || !state || !obs || !reward || !term || !trunc || !obs_rows || !actions || !log_prob ||
      !value || !rollout_reward || !episode_starts || !last_dones || !last_values)
    return fail(ACKPHYS_EINVAL, "ackphys_ppo_rollout: NULL argument");
  if (n_steps <= 0) return fail(ACKPHYS_EINVAL, "ackphys_ppo_rollout: n_steps must be positive");
  if (!(flags & ACKPHYS_CONTACTS) || !(flags & ACKPHYS_AUTORESET) || (flags & ACKPHYS_POSTSTEP_OBS))
    return fail(ACKPHYS_EINVAL, "ackphys_ppo_rollout: needs ACKPHYS_CONTACTS | ACKPHYS_AUTORESET (no POSTSTEP_OBS)");
  if (ctx->variant != ACKPHYS_VARIANT_AUTO && ctx->variant != ACKPHYS_VARIANT_QUAD)
    return fail(ACKPHYS_EINVAL, "ackphys_ppo_rollout: runs on the quad mapping (variant AUTO or QUAD)");
  DeviceGuard dg(ctx->device);
  if (dg.err != hipSuccess) return hipfail(dg.err, "hipSetDevice");
  ak::Args a{nullptr, state, obs, reward, term, trunc, terminal_obs, nullptr, episode, ctx->prm, ctx->n_env, flags,
             seed, ctx->env_offset, ak::PPO_PE};
  if (!ctx->pimg) {
    const hipError_t me = hipMalloc(&ctx->pimg, sizeof(float) * ak::PIMG_N);
    if (me != hipSuccess) {
      ctx->pimg = nullptr;
      return hipfail(me, "ackphys_ppo_rollout: weight image");
    }
  }
  // the weights as the policy's MFMA operands, from this call's parameters (they change every update)
  hipLaunchKernelGGL(ak::ackphys_policy_image_kernel, dim3((ak::PIMG_N + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     params, ctx->pimg);
  ak::PpoArgs P{params, policy_seed, step0, deterministic, gamma, n_steps, obs_rows, actions, log_prob, value,
                rollout_reward, episode_starts, last_dones, last_values, ctx->pimg};
  const int blocks = (ctx->n_env + ak::PPO_PE - 1) / ak::PPO_PE;
  const bool var = ctx->prm.action_repeat > 1 || ctx->prm.nohit_clear;
  hipLaunchKernelGGL(ctx->scene == 1 ? (var ? ackphys_ppo_rollout_obst8_var_kernel : ackphys_ppo_rollout_obst8_kernel)
                                     : (var ? ackphys_ppo_rollout_quad_var_kernel : ackphys_ppo_rollout_quad_kernel),
                     dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, P);  // 16 envs, 4 waves (ppo_rollout)
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hipfail(e, "ackphys_ppo_rollout launch");
  return ACKPHYS_OK;
}

int ackphys_random_actions(ackphys_t* ctx, float* actions, int k_steps, uint64_t seed, uint32_t step0, void* stream) {
  if (!ctx || !actions || k_steps <= 0) return fail(ACKPHYS_EINVAL, "ackphys_random_actions: bad argument");
  DeviceGuard dg(ctx->device);
  if (dg.err != hipSuccess) return hipfail(dg.err, "hipSetDevice");
  hipError_t e;
  int blocks = (ctx->n_env + 255) / 256;
  hipLaunchKernelGGL(ackphys_actions_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, actions, ctx->n_env,
                     k_steps, seed, step0, ctx->env_offset);
  e = hipGetLastError();
  if (e != hipSuccess) return hipfail(e, "ackphys_actions_kernel launch");
  return ACKPHYS_OK;
}

}  // extern "C"
