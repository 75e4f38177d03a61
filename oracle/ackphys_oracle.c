/* ackphys_oracle.c -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
 *
 * Float64 CPU restatement of the reference's per-env hot path:
 *   AckermannRobotEnv.step (src/rl/envs/ackermann_env.py:187-229)
 *     -> BicycleController.apply_cmd_vel (src/core/controller.py:98-140)
 *     -> mujoco.mj_step (ackermann_env.py:200)            [MuJoCo C engine, NOT vendored]
 *     -> _get_observation / _calculate_reward (ackermann_env.py:231-312)
 *        with Odometry.calculate_odom (src/core/odometry.py:62-103,154-170)
 *   AckermannRobotEnv.reset (ackermann_env.py:143-185) + SimpleMapSpawner
 *     (src/rl/envs/simple_map_spawner.py:22-54).
 *
 * mj_step is restated from MuJoCo's published algorithms (>= 3.1; the reference pins only
 * `mujoco>=3.0.0`, requirements.txt:4) as generic routines over the compiled-model blob
 * (include/ackphys_model.h): mj_kinematics, mj_comPos, mj_crb, mj_comVel, mj_rne,
 * mj_passive, mj_fwdActuation, mj_collision (plane-cylinder, plane-convex), mj_makeConstraint
 * (joint equality, dof friction loss, joint limits, pyramidal contacts), mj_makeImpedance,
 * the primal Newton solver, mj_Euler with implicit dof damping, mj_ray rangefinders.
 * PHYSICS PARITY IS UNPINNED: mujoco is not installed anywhere in this image and the
 * reference has no physics fixtures. Controller/obs/reward are pinned by
 * golden vectors generated from the reference's own Python (tests/golden/).
 *
 * The product (mujoco_playground_amd/csrc, HIP) never includes, links or calls this file.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/ackphys_model.h"
#include "ackphys_oracle.h"

/* stage markers for the FLOP-counting build (oracle/flops/fd.hpp, `make flops`); no-ops here.
 * 1 controller, 2 kinematics, 3 mass matrix, 4 collision, 5 sensors (rays), 6 velocity/bias/
 * actuation, 7 qacc_smooth, 8 constraint rows, 9 Newton solver, 10 Euler, 11 obs/reward, 12 reset */
#ifndef OR_STAGE
#define OR_STAGE(k) ((void)0)
#endif

#define mjMINVAL 1e-15
#define mjMINIMP 0.0001
#define mjMAXIMP 0.9999
#define mjMAXVAL 1e10
#define OR_MAXCON 64
#define OR_MAXEFC 320
#define NSTATE 44
#define NOBS 79

/* state layout (float words per env), shared with the HIP product */
#define ST_QPOS 0
#define ST_QVEL 13
#define ST_WARM 25
#define ST_GOAL 37
#define ST_REF 39
#define ST_STEP 42
#define ST_EPIS 43

#define FLAG_CONTACTS 1u
#define FLAG_AUTORESET 2u
#define FLAG_POSTSTEP_OBS 4u /* render_mode="human": mj_forward after mj_step (ackermann_env.py:202-207) */

/* controller constants: controller.py:85-86 */
#define CTL_WHEEL_R 0.0325
#define CTL_WHEELBASE 0.20
#define CTL_TRACK 0.174

#define OR_MAXFEAT 96
/* convex-hull features (geom frame) for the box-convex separating-axis test */
typedef struct {
  int nf, ne;
  double fn[OR_MAXFEAT][3]; /* unique outward face normals */
  double ed[OR_MAXFEAT][3]; /* unique edge directions (up to sign) */
} or_hullfeat;

struct or_ctx {
  const apm_model_t* m;
  or_hullfeat hf[APM_MAXMESH];
  const float* mesh_vert;
  const int32_t* mesh_face;
  const float* hull_vert;
  void* blob;
  double tolerance;
  int maxiter;
  int env_offset;
  /* AckermannRobotEnv.__init__ kwargs (ackermann_env.py:51-60) */
  int max_steps;
  double goal_thresh, coll_thresh, max_lin, max_ang;
  /* opt-in task variants (NOT the reference; 1 / 0 = ackermann_env.py): mj_steps per env step,
     rangefinder -1 readings ignored by the collision test (include/ackphys.h) */
  int action_repeat, nohit_clear;
  /* opt-in maze goals (goal_cells > 0, obstacle scene): the box-free cells of the box lattice
     4-connected to the spawn cell, by breadth-first distance (free_d), centres free_xy */
  int goal_cells, nfree;
  double free_xy[256][2];
  int free_d[256];
  /* resolved ids (reference looks these up by name) */
  int chassis_body, act_steer, act_rl, act_rr;
  int lidar_adr[72];
};

typedef struct {
  double pos[3], frame[9], dist, friction[5], solref[2], solimp[5], includemargin;
  int dim, geom1, geom2;
} or_contact;

typedef struct {
  /* state */
  double qpos[APM_MAXQ], qvel[APM_MAXDOF], qacc_warmstart[APM_MAXDOF], ctrl[APM_MAXU];
  /* position-dependent */
  double xpos[APM_MAXBODY][3], xquat[APM_MAXBODY][4], xmat[APM_MAXBODY][9];
  double xipos[APM_MAXBODY][3], ximat[APM_MAXBODY][9];
  double xanchor[APM_MAXJNT][3], xaxis[APM_MAXJNT][3];
  double geom_xpos[APM_MAXGEOM][3], geom_xmat[APM_MAXGEOM][9];
  double site_xpos[APM_MAXSITE][3], site_xmat[APM_MAXSITE][9];
  double subtree_com[APM_MAXBODY][3], subtree_mass[APM_MAXBODY];
  double cinert[APM_MAXBODY][36], cdof[APM_MAXDOF][6];
  double qM[APM_MAXDOF * APM_MAXDOF];
  /* velocity-dependent */
  double cvel[APM_MAXBODY][6], cdof_dot[APM_MAXDOF][6];
  double qfrc_bias[APM_MAXDOF], qfrc_passive[APM_MAXDOF], qfrc_actuator[APM_MAXDOF];
  double actuator_force[APM_MAXU];
  double qfrc_smooth[APM_MAXDOF], qacc_smooth[APM_MAXDOF];
  double qacc[APM_MAXDOF], qfrc_constraint[APM_MAXDOF];
  double sensordata[APM_MAXSENSOR];
  /* contacts / constraints */
  int ncon;
  or_contact con[OR_MAXCON];
  int nefc;
  int efc_type[OR_MAXEFC]; /* 0 eq, 1 friction, 2 limit, 3 contact */
  double efc_J[OR_MAXEFC][APM_MAXDOF];
  double efc_pos[OR_MAXEFC], efc_margin[OR_MAXEFC], efc_floss[OR_MAXEFC];
  double efc_diag[OR_MAXEFC], efc_R[OR_MAXEFC], efc_D[OR_MAXEFC], efc_aref[OR_MAXEFC];
  double efc_vel[OR_MAXEFC], efc_force[OR_MAXEFC];
  int efc_conid[OR_MAXEFC];
  int solver_niter;
  int bad_state, bad_ctrl;
} or_data;

static __thread char g_err[256];
static void set_err(const char* s) { snprintf(g_err, sizeof(g_err), "%s", s); }
const char* or_last_error(void) { return g_err; }
int or_model_struct_size(void) { return (int)sizeof(apm_model_t); }

/* ------------------------------------------------------------------ small linear algebra */

static void quat2mat(double res[9], const double q[4]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  res[0] = 1 - 2 * (y * y + z * z); res[1] = 2 * (x * y - w * z); res[2] = 2 * (x * z + w * y);
  res[3] = 2 * (x * y + w * z); res[4] = 1 - 2 * (x * x + z * z); res[5] = 2 * (y * z - w * x);
  res[6] = 2 * (x * z - w * y); res[7] = 2 * (y * z + w * x); res[8] = 1 - 2 * (x * x + y * y);
}
static void mulquat(double r[4], const double a[4], const double b[4]) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof t);
}
static double normalize4(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < mjMINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else { q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n; }
  return n;
}
static double normalize3(double v[3]) {
  double n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (n < mjMINVAL) { v[0] = 1; v[1] = v[2] = 0; }
  else { v[0] /= n; v[1] /= n; v[2] /= n; }
  return n;
}
static void mulmatvec3(double r[3], const double M[9], const double v[3]) {
  double t[3] = {M[0] * v[0] + M[1] * v[1] + M[2] * v[2], M[3] * v[0] + M[4] * v[1] + M[5] * v[2],
                 M[6] * v[0] + M[7] * v[1] + M[8] * v[2]};
  memcpy(r, t, sizeof t);
}
static void mulmatTvec3(double r[3], const double M[9], const double v[3]) {
  double t[3] = {M[0] * v[0] + M[3] * v[1] + M[6] * v[2], M[1] * v[0] + M[4] * v[1] + M[7] * v[2],
                 M[2] * v[0] + M[5] * v[1] + M[8] * v[2]};
  memcpy(r, t, sizeof t);
}
static void mulmat3(double r[9], const double A[9], const double B[9]) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(r, t, sizeof t);
}
static void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof t);
}
static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* spatial algebra, motion/force vectors ordered (angular, linear) as MuJoCo's cdof/cvel */
static void cross_motion(double r[6], const double v[6], const double u[6]) {
  double a[3], b[3], c[3];
  cross3(a, v, u);           /* w x u_ang */
  cross3(b, v, u + 3);       /* w x u_lin */
  cross3(c, v + 3, u);       /* v_lin x u_ang */
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static void cross_force(double r[6], const double v[6], const double f[6]) {
  double a[3], b[3], c[3];
  cross3(a, v, f);           /* w x f_ang */
  cross3(b, v + 3, f + 3);   /* v_lin x f_lin */
  cross3(c, v, f + 3);       /* w x f_lin */
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
static void mul6(double r[6], const double I[36], const double v[6]) {
  for (int i = 0; i < 6; i++) {
    double s = 0;
    for (int j = 0; j < 6; j++) s += I[6 * i + j] * v[j];
    r[i] = s;
  }
}

/* dense Cholesky (lower) in place; returns 0 on success */
static int cholesky(double* A, int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (s <= 0) return -1;
    s = sqrt(s);
    A[j * n + j] = s;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / s;
    }
  }
  return 0;
}
static void chol_solve(const double* L, int n, double* x) {
  for (int i = 0; i < n; i++) {
    double s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

/* ------------------------------------------------------------------ Philox4x32-10 (Random123) */

static void philox4x32_10(uint32_t ctr[4], const uint32_t key_in[2]) {
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ ctr[1] ^ k0, n1 = lo1, n2 = hi0 ^ ctr[3] ^ k1, n3 = lo0;
    ctr[0] = n0; ctr[1] = n1; ctr[2] = n2; ctr[3] = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
/* exported for tests: out[4] = philox(counter, key) */
void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  philox4x32_10(c, key);
  memcpy(out, c, sizeof c);
}
static double u01(uint32_t x) { return (double)(x >> 8) * (1.0 / 16777216.0); }

/* ------------------------------------------------------------------ convex hull features
   Faces = supporting planes through 3 hull vertices (all vertices on one side); edges = vertex
   pairs lying on >= 2 distinct face planes. Brute force, once per context (36 vertices here). */
static void feat_add(double (*arr)[3], int* n, const double v[3], int sign_free) {
  for (int i = 0; i < *n; i++) {
    double dd = dot3(arr[i], v);
    if (dd > 1 - 1e-9 || (sign_free && dd < -1 + 1e-9)) return;
  }
  if (*n < OR_MAXFEAT) { memcpy(arr[*n], v, sizeof(double) * 3); (*n)++; }
}
static void hull_features(const float* hv, int n, or_hullfeat* f) {
  f->nf = f->ne = 0;
  double scale = 0;
  for (int i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) scale = fmax(scale, fabs((double)hv[3 * i + k]));
  const double tol = 1e-9 * (scale > 0 ? scale : 1);
#define HV(i, k) ((double)hv[3 * (i) + (k)])
  for (int i = 0; i < n; i++)
    for (int j = i + 1; j < n; j++)
      for (int k = j + 1; k < n; k++) {
        double e1[3] = {HV(j, 0) - HV(i, 0), HV(j, 1) - HV(i, 1), HV(j, 2) - HV(i, 2)};
        double e2[3] = {HV(k, 0) - HV(i, 0), HV(k, 1) - HV(i, 1), HV(k, 2) - HV(i, 2)};
        double nn[3];
        cross3(nn, e1, e2);
        double len = sqrt(dot3(nn, nn));
        if (len < 1e-12 * scale * scale) continue;
        for (int t = 0; t < 3; t++) nn[t] /= len;
        double off = nn[0] * HV(i, 0) + nn[1] * HV(i, 1) + nn[2] * HV(i, 2);
        int above = 0, below = 0;
        for (int v = 0; v < n; v++) {
          double sd = nn[0] * HV(v, 0) + nn[1] * HV(v, 1) + nn[2] * HV(v, 2) - off;
          if (sd > tol) above++;
          else if (sd < -tol) below++;
        }
        if (above && below) continue;
        if (above) for (int t = 0; t < 3; t++) nn[t] = -nn[t];
        feat_add(f->fn, &f->nf, nn, 0);
      }
  double off[OR_MAXFEAT];
  for (int a = 0; a < f->nf; a++) {
    off[a] = -1e300;
    for (int v = 0; v < n; v++) off[a] = fmax(off[a], f->fn[a][0] * HV(v, 0) + f->fn[a][1] * HV(v, 1) + f->fn[a][2] * HV(v, 2));
  }
  for (int i = 0; i < n; i++)
    for (int j = i + 1; j < n; j++) {
      double e[3] = {HV(j, 0) - HV(i, 0), HV(j, 1) - HV(i, 1), HV(j, 2) - HV(i, 2)};
      double len = sqrt(dot3(e, e));
      if (len < tol) continue;
      int on = 0;
      for (int a = 0; a < f->nf; a++) {
        double si = f->fn[a][0] * HV(i, 0) + f->fn[a][1] * HV(i, 1) + f->fn[a][2] * HV(i, 2) - off[a];
        double sj = f->fn[a][0] * HV(j, 0) + f->fn[a][1] * HV(j, 1) + f->fn[a][2] * HV(j, 2) - off[a];
        if (fabs(si) < tol && fabs(sj) < tol) on++;
      }
      if (on < 2) continue;
      for (int t = 0; t < 3; t++) e[t] /= len;
      feat_add(f->ed, &f->ne, e, 1);
    }
#undef HV
}
int or_hull_features(const or_ctx* c, int mesh, double* fn, double* ed, int* nf, int* ne) {
  if (mesh < 0 || mesh >= c->m->nmesh) return -1;
  const or_hullfeat* f = &c->hf[mesh];
  memcpy(fn, f->fn, sizeof(double) * 3 * f->nf);
  memcpy(ed, f->ed, sizeof(double) * 3 * f->ne);
  *nf = f->nf;
  *ne = f->ne;
  return 0;
}

/* ------------------------------------------------------------------ model setup */
static int find_actuator(const apm_model_t* m, int jnt) {
  for (int i = 0; i < m->nu; i++)
    if (m->actuator_trnid[i] == jnt) return i;
  return -1;
}

int or_create(const void* blob, size_t nbytes, or_ctx** out) {
  if (!blob || nbytes < sizeof(apm_model_t)) { set_err("blob too small"); return -1; }
  const apm_model_t* hm = (const apm_model_t*)blob;
  if (hm->magic != APM_MAGIC || hm->version != APM_VERSION) { set_err("bad blob magic/version"); return -2; }
  if (hm->nbytes != nbytes || hm->hdr_bytes != sizeof(apm_model_t)) { set_err("blob size mismatch"); return -3; }
  or_ctx* c = (or_ctx*)calloc(1, sizeof(or_ctx));
  c->blob = malloc(nbytes);
  memcpy(c->blob, blob, nbytes);
  c->m = (const apm_model_t*)c->blob;
  const char* tail = (const char*)c->blob + sizeof(apm_model_t);
  c->mesh_vert = (const float*)tail;
  c->mesh_face = (const int32_t*)(tail + 12 * (size_t)c->m->nmeshvert);
  c->hull_vert = (const float*)(tail + 12 * (size_t)c->m->nmeshvert + 12 * (size_t)c->m->nmeshface);
  for (int k = 0; k < c->m->nmesh; k++)
    hull_features(c->hull_vert + 3 * c->m->mesh_hulladr[k], c->m->mesh_hullnum[k], &c->hf[k]);
  c->tolerance = 1e-12; /* tighter than MuJoCo's 1e-8: the oracle targets the exact optimum */
  c->maxiter = c->m->iterations;
  c->chassis_body = c->m->jnt_bodyid[0]; /* the free joint's body ("chassis") */
  c->max_steps = 1000; c->goal_thresh = 0.5; c->coll_thresh = 0.15; c->max_lin = 1.0; c->max_ang = 1.0;
  c->action_repeat = 1; c->nohit_clear = 0; c->goal_cells = 0; c->nfree = 0;
  /* BicycleController actuator lookup by name (controller.py:94-96): steering servo on the
     first limited hinge, rear drives on the first two hinges -- resolved by trnid order. */
  c->act_steer = 0; c->act_rl = 1; c->act_rr = 2;
  (void)find_actuator;
  /* lidar addresses, with the reference's name-lookup aliasing (ackermann_env.py:131-141):
     "lidar-{i}" for i<10 does not exist (names are zero-padded "lidar-0i"), mj_name2id
     returns -1 and sensor_adr[-1] is the LAST sensor's address. */
  int last = c->m->nsensor - 1;
  int nlid = 0;
  for (int s = 0; s < c->m->nsensor; s++)
    if (c->m->sensor_type[s] == APM_SENS_RANGEFINDER) nlid++;
  if (nlid != 72) { set_err("expected 72 rangefinders"); free(c->blob); free(c); return -4; }
  int first_lidar = c->m->nsensor - 72;
  for (int i = 0; i < 72; i++)
    c->lidar_adr[i] = (i < 10) ? c->m->sensor_adr[last] : c->m->sensor_adr[first_lidar + i];
  *out = c;
  return 0;
}

void or_destroy(or_ctx* c) {
  if (!c) return;
  free(c->blob);
  free(c);
}

void or_set_solver(or_ctx* c, double tolerance, int maxiter) { c->tolerance = tolerance; c->maxiter = maxiter; }
void or_set_env_offset(or_ctx* c, int off) { c->env_offset = off; }
void or_set_env_params(or_ctx* c, int max_steps, double goal, double coll, double max_lin, double max_ang) {
  c->max_steps = max_steps; c->goal_thresh = goal; c->coll_thresh = coll; c->max_lin = max_lin; c->max_ang = max_ang;
}
void or_set_env_variant(or_ctx* c, int action_repeat, int nohit_clear) {
  c->action_repeat = action_repeat < 1 ? 1 : action_repeat;
  c->nohit_clear = nohit_clear != 0;
}

/* Free maze cells of the world's static boxes: the lattice origin is the boxes' lowest corner and
   its pitch the smallest box footprint; a cell is free when no box overlaps its interior; cells
   4-connected to the spawn's cell are listed in breadth-first order, sorted by (distance, row,
   column), the spawn cell left out. Returns the count, 0 when the world has no boxes, -1 on a
   lattice the tables cannot hold. */
static int free_cells(or_ctx* c) {
  const apm_model_t* m = c->m;
  double x0 = 1e300, y0 = 1e300, x1 = -1e300, y1 = -1e300, cell = 1e300;
  int nb = 0;
  /* static (world-welded) boxes; their bodies sit at the world origin unrotated (model/codegen.py
     checks that for the scene), so geom_pos + body_pos is the world centre */
#define OR_STATIC_BOX(g) (m->geom_type[g] == APM_GEOM_BOX && m->body_weldid[m->geom_bodyid[g]] == 0)
#define OR_BOX_C(g, k) (m->geom_pos[g][k] + m->body_pos[m->geom_bodyid[g]][k])
  for (int g = 0; g < m->ngeom; g++) {
    if (!OR_STATIC_BOX(g)) continue;
    nb++;
    x0 = fmin(x0, OR_BOX_C(g, 0) - m->geom_size[g][0]); x1 = fmax(x1, OR_BOX_C(g, 0) + m->geom_size[g][0]);
    y0 = fmin(y0, OR_BOX_C(g, 1) - m->geom_size[g][1]); y1 = fmax(y1, OR_BOX_C(g, 1) + m->geom_size[g][1]);
    cell = fmin(cell, 2 * fmin(m->geom_size[g][0], m->geom_size[g][1]));
  }
  if (!nb) return 0;
  const int nx = (int)ceil((x1 - x0) / cell - 1e-9), ny = (int)ceil((y1 - y0) / cell - 1e-9);
  if (nx * ny > 256) return -1;
  int occ[256] = {0}, dist[256], queue[256];
  for (int g = 0; g < m->ngeom; g++) {
    if (!OR_STATIC_BOX(g)) continue;
    for (int iy = 0; iy < ny; iy++)
      for (int ix = 0; ix < nx; ix++) {
        const double cx = x0 + ix * cell, cy = y0 + iy * cell, e = 1e-6;
        if (OR_BOX_C(g, 0) - m->geom_size[g][0] < cx + cell - e && OR_BOX_C(g, 0) + m->geom_size[g][0] > cx + e &&
            OR_BOX_C(g, 1) - m->geom_size[g][1] < cy + cell - e && OR_BOX_C(g, 1) + m->geom_size[g][1] > cy + e)
          occ[iy * nx + ix] = 1;
      }
  }
#undef OR_STATIC_BOX
#undef OR_BOX_C
  const int sx = (int)floor((m->spawn[0] - x0) / cell), sy = (int)floor((m->spawn[1] - y0) / cell);
  if (sx < 0 || sx >= nx || sy < 0 || sy >= ny || occ[sy * nx + sx]) return -1;
  for (int i = 0; i < nx * ny; i++) dist[i] = -1;
  int head = 0, tail = 0;
  dist[sy * nx + sx] = 0;
  queue[tail++] = sy * nx + sx;
  while (head < tail) {
    const int q = queue[head++], qx = q % nx, qy = q / nx;
    const int nbr[4][2] = {{qx + 1, qy}, {qx - 1, qy}, {qx, qy + 1}, {qx, qy - 1}};
    for (int k = 0; k < 4; k++) {
      const int ax = nbr[k][0], ay = nbr[k][1];
      if (ax < 0 || ax >= nx || ay < 0 || ay >= ny || occ[ay * nx + ax] || dist[ay * nx + ax] >= 0) continue;
      dist[ay * nx + ax] = dist[q] + 1;
      queue[tail++] = ay * nx + ax;
    }
  }
  int n = 0;
  for (int d = 1; d <= nx * ny; d++)  /* by distance, then row-major (row, column) */
    for (int i = 0; i < nx * ny; i++)
      if (dist[i] == d) {
        c->free_xy[n][0] = x0 + (i % nx + 0.5) * cell;
        c->free_xy[n][1] = y0 + (i / nx + 0.5) * cell;
        c->free_d[n++] = d;
      }
  return n;
}
int or_set_goal_cells(or_ctx* c, int goal_cells) {
  if (goal_cells <= 0) { c->goal_cells = 0; return 0; }
  const int n = free_cells(c);
  if (n <= 0) { set_err("goal_cells needs a world of static boxes with a free spawn cell"); return -1; }
  c->nfree = n;
  c->goal_cells = goal_cells;
  return 0;
}

/* ------------------------------------------------------------------ mj_kinematics */

static void kinematics(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  d->xpos[0][0] = d->xpos[0][1] = d->xpos[0][2] = 0;
  d->xquat[0][0] = 1; d->xquat[0][1] = d->xquat[0][2] = d->xquat[0][3] = 0;
  quat2mat(d->xmat[0], d->xquat[0]);
  memcpy(d->xipos[0], d->xpos[0], sizeof(double) * 3);
  memcpy(d->ximat[0], d->xmat[0], sizeof(double) * 9);
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parentid[i];
    int ja = m->body_jntadr[i], jn = m->body_jntnum[i];
    double pos[3], quat[4];
    if (jn == 1 && m->jnt_type[ja] == APM_JNT_FREE) {
      int a = m->jnt_qposadr[ja];
      memcpy(pos, d->qpos + a, sizeof pos);
      memcpy(quat, d->qpos + a + 3, sizeof quat);
      normalize4(quat);
      memcpy(d->xanchor[ja], pos, sizeof pos);
      d->xaxis[ja][0] = 0; d->xaxis[ja][1] = 0; d->xaxis[ja][2] = 1;
    } else {
      mulmatvec3(pos, d->xmat[p], m->body_pos[i]);
      pos[0] += d->xpos[p][0]; pos[1] += d->xpos[p][1]; pos[2] += d->xpos[p][2];
      mulquat(quat, d->xquat[p], m->body_quat[i]);
      for (int j = ja; j < ja + jn; j++) {
        double mat[9], qloc[4];
        quat2mat(mat, quat);
        mulmatvec3(d->xaxis[j], mat, m->jnt_axis[j]);
        mulmatvec3(d->xanchor[j], mat, m->jnt_pos[j]);
        for (int k = 0; k < 3; k++) d->xanchor[j][k] += pos[k];
        int qa = m->jnt_qposadr[j];
        double ang = d->qpos[qa] - m->qpos0[qa];
        double s = sin(0.5 * ang);
        qloc[0] = cos(0.5 * ang);
        qloc[1] = m->jnt_axis[j][0] * s; qloc[2] = m->jnt_axis[j][1] * s; qloc[3] = m->jnt_axis[j][2] * s;
        mulquat(quat, quat, qloc);
        normalize4(quat);
        quat2mat(mat, quat);
        double off[3];
        mulmatvec3(off, mat, m->jnt_pos[j]);
        for (int k = 0; k < 3; k++) pos[k] = d->xanchor[j][k] - off[k];
      }
      normalize4(quat);
    }
    memcpy(d->xpos[i], pos, sizeof pos);
    memcpy(d->xquat[i], quat, sizeof quat);
    quat2mat(d->xmat[i], quat);
    double t[3], im[9];
    mulmatvec3(t, d->xmat[i], m->body_ipos[i]);
    for (int k = 0; k < 3; k++) d->xipos[i][k] = d->xpos[i][k] + t[k];
    quat2mat(im, m->body_iquat[i]);
    mulmat3(d->ximat[i], d->xmat[i], im);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    double t[3], gm[9];
    mulmatvec3(t, d->xmat[b], m->geom_pos[g]);
    for (int k = 0; k < 3; k++) d->geom_xpos[g][k] = d->xpos[b][k] + t[k];
    quat2mat(gm, m->geom_quat[g]);
    mulmat3(d->geom_xmat[g], d->xmat[b], gm);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    double t[3], sm[9];
    mulmatvec3(t, d->xmat[b], m->site_pos[s]);
    for (int k = 0; k < 3; k++) d->site_xpos[s][k] = d->xpos[b][k] + t[k];
    quat2mat(sm, m->site_quat[s]);
    mulmat3(d->site_xmat[s], d->xmat[b], sm);
  }
}

/* ------------------------------------------------------------------ mj_comPos */

static void com_pos(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  for (int i = 0; i < m->nbody; i++) {
    d->subtree_mass[i] = m->body_mass[i];
    for (int k = 0; k < 3; k++) d->subtree_com[i][k] = m->body_mass[i] * d->xipos[i][k];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    d->subtree_mass[p] += d->subtree_mass[i];
    for (int k = 0; k < 3; k++) d->subtree_com[p][k] += d->subtree_com[i][k];
  }
  for (int i = 0; i < m->nbody; i++) {
    if (d->subtree_mass[i] < mjMINVAL)
      memcpy(d->subtree_com[i], d->xipos[i], sizeof(double) * 3);
    else
      for (int k = 0; k < 3; k++) d->subtree_com[i][k] /= d->subtree_mass[i];
  }
  /* com-based spatial inertia of each body about subtree_com[rootid] */
  for (int i = 1; i < m->nbody; i++) {
    const double* O = d->subtree_com[m->body_rootid[i]];
    double mass = m->body_mass[i], cc[3], Iw[9], tmp[9];
    for (int k = 0; k < 3; k++) cc[k] = d->xipos[i][k] - O[k];
    /* Iw = ximat diag(I) ximat^T */
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) tmp[3 * a + b] = d->ximat[i][3 * a + b] * m->body_inertia[i][b];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++)
        Iw[3 * a + b] = tmp[3 * a] * d->ximat[i][3 * b] + tmp[3 * a + 1] * d->ximat[i][3 * b + 1] +
                        tmp[3 * a + 2] * d->ximat[i][3 * b + 2];
    double* I6 = d->cinert[i];
    memset(I6, 0, sizeof(double) * 36);
    double cx[9] = {0, -cc[2], cc[1], cc[2], 0, -cc[0], -cc[1], cc[0], 0};
    double c2 = dot3(cc, cc);
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        /* I_O = Iw + m(|c|^2 1 - c c^T) */
        I6[6 * a + b] = Iw[3 * a + b] + mass * ((a == b ? c2 : 0) - cc[a] * cc[b]);
        I6[6 * a + 3 + b] = mass * cx[3 * a + b];
        I6[6 * (3 + a) + b] = -mass * cx[3 * a + b];
        I6[6 * (3 + a) + 3 + b] = (a == b) ? mass : 0;
      }
  }
  /* cdof */
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    const double* O = d->subtree_com[m->body_rootid[b]];
    if (m->jnt_type[j] == APM_JNT_FREE) {
      for (int k = 0; k < 3; k++) {
        double* cd = d->cdof[da + k];
        memset(cd, 0, sizeof(double) * 6);
        cd[3 + k] = 1;
      }
      double off[3] = {O[0] - d->xpos[b][0], O[1] - d->xpos[b][1], O[2] - d->xpos[b][2]};
      for (int k = 0; k < 3; k++) {
        double ax[3] = {d->xmat[b][k], d->xmat[b][3 + k], d->xmat[b][6 + k]};
        double* cd = d->cdof[da + 3 + k];
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(cd + 3, ax, off);
      }
    } else {
      double off[3] = {O[0] - d->xanchor[j][0], O[1] - d->xanchor[j][1], O[2] - d->xanchor[j][2]};
      double* cd = d->cdof[da];
      memcpy(cd, d->xaxis[j], sizeof(double) * 3);
      cross3(cd + 3, d->xaxis[j], off);
    }
  }
}

/* ------------------------------------------------------------------ mj_crb (dense qM) */

static void crb(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  int nv = m->nv;
  double crbi[APM_MAXBODY][36];
  memcpy(crbi, d->cinert, sizeof(double) * 36 * m->nbody);
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 36; k++) crbi[p][k] += crbi[i][k];
  }
  memset(d->qM, 0, sizeof(double) * nv * nv);
  for (int i = 0; i < nv; i++) {
    double buf[6];
    mul6(buf, crbi[m->dof_bodyid[i]], d->cdof[i]);
    int j = i;
    while (j >= 0) {
      double s = 0;
      for (int k = 0; k < 6; k++) s += d->cdof[j][k] * buf[k];
      d->qM[i * nv + j] = s;
      d->qM[j * nv + i] = s;
      j = m->dof_parentid[j];
    }
    d->qM[i * nv + i] += m->dof_armature[i];
  }
}

/* ------------------------------------------------------------------ mj_comVel + mj_rne */

static void com_vel(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  memset(d->cvel[0], 0, sizeof(double) * 6);
  for (int i = 1; i < m->nbody; i++) {
    double cvel[6];
    memcpy(cvel, d->cvel[m->body_parentid[i]], sizeof cvel);
    for (int j = m->body_jntadr[i]; j < m->body_jntadr[i] + m->body_jntnum[i]; j++) {
      int da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == APM_JNT_FREE) {
        for (int k = 0; k < 3; k++) {
          memset(d->cdof_dot[da + k], 0, sizeof(double) * 6);
          for (int t = 0; t < 6; t++) cvel[t] += d->cdof[da + k][t] * d->qvel[da + k];
        }
        for (int k = 3; k < 6; k++) cross_motion(d->cdof_dot[da + k], cvel, d->cdof[da + k]);
        for (int k = 3; k < 6; k++)
          for (int t = 0; t < 6; t++) cvel[t] += d->cdof[da + k][t] * d->qvel[da + k];
      } else {
        cross_motion(d->cdof_dot[da], cvel, d->cdof[da]);
        for (int t = 0; t < 6; t++) cvel[t] += d->cdof[da][t] * d->qvel[da];
      }
    }
    memcpy(d->cvel[i], cvel, sizeof cvel);
  }
}

static void rne(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  double cacc[APM_MAXBODY][6], cfrc[APM_MAXBODY][6];
  memset(cacc[0], 0, sizeof(double) * 6);
  cacc[0][3] = -m->gravity[0]; cacc[0][4] = -m->gravity[1]; cacc[0][5] = -m->gravity[2];
  for (int i = 1; i < m->nbody; i++) {
    memcpy(cacc[i], cacc[m->body_parentid[i]], sizeof(double) * 6);
    for (int k = m->body_dofadr[i]; k < m->body_dofadr[i] + m->body_dofnum[i]; k++)
      for (int t = 0; t < 6; t++) cacc[i][t] += d->cdof_dot[k][t] * d->qvel[k];
    double a[6], mv[6], cf[6];
    mul6(a, d->cinert[i], cacc[i]);
    mul6(mv, d->cinert[i], d->cvel[i]);
    cross_force(cf, d->cvel[i], mv);
    for (int t = 0; t < 6; t++) cfrc[i][t] = a[t] + cf[t];
  }
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int t = 0; t < 6; t++) cfrc[p][t] += cfrc[i][t];
  }
  for (int k = 0; k < m->nv; k++) {
    double s = 0;
    for (int t = 0; t < 6; t++) s += d->cdof[k][t] * cfrc[m->dof_bodyid[k]][t];
    d->qfrc_bias[k] = s;
  }
}

/* ------------------------------------------------------------------ passive + actuation */

static void passive(const or_ctx* c, or_data* d) {
  for (int i = 0; i < c->m->nv; i++) d->qfrc_passive[i] = -c->m->dof_damping[i] * d->qvel[i];
}

static void actuation(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  memset(d->qfrc_actuator, 0, sizeof(double) * m->nv);
  for (int i = 0; i < m->nu; i++) {
    double ctrl = d->ctrl[i];
    if (m->actuator_ctrllimited[i]) {
      if (ctrl < m->actuator_ctrlrange[i][0]) ctrl = m->actuator_ctrlrange[i][0];
      if (ctrl > m->actuator_ctrlrange[i][1]) ctrl = m->actuator_ctrlrange[i][1];
    }
    int j = m->actuator_trnid[i];
    double gear = m->actuator_gear[i];
    double len = gear * d->qpos[m->jnt_qposadr[j]];
    double vel = gear * d->qvel[m->jnt_dofadr[j]];
    double f = m->actuator_gainprm[i][0] * ctrl + m->actuator_biasprm[i][0] +
               m->actuator_biasprm[i][1] * len + m->actuator_biasprm[i][2] * vel;
    if (m->actuator_forcelimited[i]) {
      if (f < m->actuator_forcerange[i][0]) f = m->actuator_forcerange[i][0];
      if (f > m->actuator_forcerange[i][1]) f = m->actuator_forcerange[i][1];
    }
    d->actuator_force[i] = f;
    d->qfrc_actuator[m->jnt_dofadr[j]] += gear * f;
  }
}

/* ------------------------------------------------------------------ collision */

static void make_frame(double frame[9]) {
  /* mju_makeFrame: normal in frame[0:3]; y = (0,1,0) if |n_y| < 0.5 else (0,0,1) */
  double* y = frame + 3;
  if (fabs(frame[1]) < 0.5) { y[0] = 0; y[1] = 1; y[2] = 0; }
  else { y[0] = 0; y[1] = 0; y[2] = 1; }
  double dd = dot3(frame, y);
  for (int k = 0; k < 3; k++) y[k] -= dd * frame[k];
  normalize3(y);
  cross3(frame + 6, frame, y);
}

static void mix_params(const apm_model_t* m, int g1, int g2, or_contact* con) {
  con->dim = m->geom_condim[g1] > m->geom_condim[g2] ? m->geom_condim[g1] : m->geom_condim[g2];
  /* mixed geom friction (slide, spin, roll) -> contact 5-vector (slide, slide, spin, roll, roll) */
  double fr[3];
  for (int k = 0; k < 3; k++) fr[k] = fmax(m->geom_friction[g1][k], m->geom_friction[g2][k]);
  con->friction[0] = fr[0]; con->friction[1] = fr[0]; con->friction[2] = fr[1];
  con->friction[3] = fr[2]; con->friction[4] = fr[2];
  double s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2];
  double mix = (s1 < mjMINVAL && s2 < mjMINVAL) ? 0.5 : (s1 < mjMINVAL ? 0 : (s2 < mjMINVAL ? 1 : s1 / (s1 + s2)));
  for (int k = 0; k < 2; k++)
    con->solref[k] = (m->geom_solref[g1][0] > 0 && m->geom_solref[g2][0] > 0)
                         ? mix * m->geom_solref[g1][k] + (1 - mix) * m->geom_solref[g2][k]
                         : fmin(m->geom_solref[g1][k], m->geom_solref[g2][k]);
  for (int k = 0; k < 5; k++) con->solimp[k] = mix * m->geom_solimp[g1][k] + (1 - mix) * m->geom_solimp[g2][k];
  double margin = fmax(m->geom_margin[g1], m->geom_margin[g2]);
  double gap = fmax(m->geom_gap[g1], m->geom_gap[g2]);
  con->includemargin = margin - gap;
}

/* mjc_PlaneCylinder [ext]: up to 2 rim points of the near cap ... + 2 cap "triangle" points */
static int plane_cylinder(const or_data* d, const apm_model_t* m, int g1, int g2, double margin, or_contact* con) {
  const double *mat1 = d->geom_xmat[g1], *mat2 = d->geom_xmat[g2];
  const double *pos1 = d->geom_xpos[g1], *pos2 = d->geom_xpos[g2];
  const double* size = m->geom_size[g2];
  double normal[3] = {mat1[2], mat1[5], mat1[8]};
  double axis[3] = {mat2[2], mat2[5], mat2[8]};
  double prjaxis = dot3(normal, axis);
  if (prjaxis > 0) { axis[0] = -axis[0]; axis[1] = -axis[1]; axis[2] = -axis[2]; prjaxis = -prjaxis; }
  double dif[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  double dist0 = dot3(dif, normal);
  /* vec: radial direction pointing towards the plane, length = radius */
  double vec[3] = {axis[0] * prjaxis - normal[0], axis[1] * prjaxis - normal[1], axis[2] * prjaxis - normal[2]};
  double len2 = dot3(vec, vec), prjvec;
  if (len2 >= mjMINVAL * mjMINVAL) {
    double s = size[0] / sqrt(len2);
    vec[0] *= s; vec[1] *= s; vec[2] *= s;
    prjvec = dot3(vec, normal);
  } else {
    vec[0] = mat2[0] * size[0]; vec[1] = mat2[3] * size[0]; vec[2] = mat2[6] * size[0];
    prjvec = 0;
  }
  for (int k = 0; k < 3; k++) axis[k] *= size[1];
  prjaxis *= size[1];
  int cnt = 0;
  double dd = dist0 + prjaxis + prjvec;
  if (dd > margin) return 0;
  for (int side = 0; side < 2; side++) {
    double sg = side == 0 ? 1.0 : -1.0;
    dd = dist0 + sg * prjaxis + prjvec;
    if (dd <= margin) {
      or_contact* cc = con + cnt++;
      cc->dist = dd;
      for (int k = 0; k < 3; k++) cc->pos[k] = pos2[k] + vec[k] + sg * axis[k] - normal[k] * dd * 0.5;
      memcpy(cc->frame, normal, sizeof normal);
    }
  }
  /* cap "triangle" points: the near cap is entirely within margin -> add the two rim points at
     +-120 deg from the nearest one */
  if (dist0 + prjaxis - prjvec <= margin) {
    double vec1[3];
    cross3(vec1, vec, axis);
    normalize3(vec1);
    double r32 = size[0] * sqrt(3.0) / 2;
    for (int k = 0; k < 3; k++) vec1[k] *= r32;
    dd = dist0 + prjaxis - 0.5 * prjvec;
    for (int s = -1; s <= 1; s += 2) {
      or_contact* cc = con + cnt++;
      cc->dist = dd;
      for (int k = 0; k < 3; k++) cc->pos[k] = pos2[k] + axis[k] - 0.5 * vec[k] + s * vec1[k] - normal[k] * dd * 0.5;
      memcpy(cc->frame, normal, sizeof normal);
    }
  }
  return cnt;
}

/* plane vs convex hull: support vertex + up to 3 more hull vertices within margin, chosen
   greedily for maximal spread (restated, confidence L -- see DESIGN.md) */
static int plane_convex(const or_ctx* c, const or_data* d, int g1, int g2, double margin, or_contact* con) {
  const apm_model_t* m = c->m;
  const double *mat1 = d->geom_xmat[g1], *pos1 = d->geom_xpos[g1];
  const double *mat2 = d->geom_xmat[g2], *pos2 = d->geom_xpos[g2];
  double normal[3] = {mat1[2], mat1[5], mat1[8]};
  int mid = m->geom_dataid[g2];
  const float* hv = c->hull_vert + 3 * m->mesh_hulladr[mid];
  int nh = m->mesh_hullnum[mid];
  double wp[64][3], dist[64];
  int best = -1;
  for (int i = 0; i < nh && i < 64; i++) {
    double v[3] = {hv[3 * i], hv[3 * i + 1], hv[3 * i + 2]}, w[3];
    mulmatvec3(w, mat2, v);
    for (int k = 0; k < 3; k++) wp[i][k] = w[k] + pos2[k];
    double df[3] = {wp[i][0] - pos1[0], wp[i][1] - pos1[1], wp[i][2] - pos1[2]};
    dist[i] = dot3(normal, df);
    if (best < 0 || dist[i] < dist[best]) best = i;
  }
  if (best < 0 || dist[best] > margin) return 0;
  int sel[4] = {best, -1, -1, -1}, nsel = 1;
  while (nsel < 4) {
    int pick = -1;
    double pickd = 1e-12;
    for (int i = 0; i < nh; i++) {
      if (dist[i] > margin) continue;
      double dmin = 1e300;
      for (int s = 0; s < nsel; s++) {
        double e[3] = {wp[i][0] - wp[sel[s]][0], wp[i][1] - wp[sel[s]][1], wp[i][2] - wp[sel[s]][2]};
        double dd = dot3(e, e);
        if (dd < dmin) dmin = dd;
      }
      if (dmin > pickd) { pickd = dmin; pick = i; }
    }
    if (pick < 0) break;
    sel[nsel++] = pick;
  }
  for (int s = 0; s < nsel; s++) {
    or_contact* cc = con + s;
    cc->dist = dist[sel[s]];
    for (int k = 0; k < 3; k++) cc->pos[k] = wp[sel[s]][k] - normal[k] * cc->dist * 0.5;
    memcpy(cc->frame, normal, sizeof normal);
  }
  return nsel;
}

/* ---------------- box vs convex geoms (obstacle scene)
   MuJoCo routes box-cylinder and box-mesh pairs to its general convex collider, which returns
   ONE contact per pair (multiccd off) at its estimate of the minimum translation [ext]. This
   restatement computes that minimum translation by a separating-axis test over a fixed
   candidate set with exact support functions:
     box-mesh:     box axes, hull face normals, hull edge dirs x box axes (complete for polytopes);
     cylinder-box: box axes, cylinder axis, cylinder axis x box axes, and for each box axis
                   whose edges come within the cylinder's bounding radius, the best direction
                   perpendicular to that axis (edge-rim contacts; 1-D search, see edge_family).
   dist = the largest separation over the set (<= 0: penetration), normal from geom1 to geom2
   (MuJoCo pair order: cylinder(5) < box(6) < mesh(7)); the contact point is the robot geom's
   deepest point moved half the penetration back (the witness midpoint). Support points that are
   not unique (face/edge parallel to the separating plane) average the candidates within 1 um. */
#define OR_TIE 1e-6
#define OR_KINK_TOL 5e-7
/* the kink snap below is a deliberate departure from mj_collision (whose general convex collider
   has no such rule): it exists because the kernel's f32 edge search is rounding-limited at the
   kink. or_set_kink_snap(0) turns it off so tests can bound what the snap changes (normal, depth:
   tests/test_obstacle_scene.py::test_kink_snap_changes_only_the_tie) */
static int g_kink_snap = 1;
void or_set_kink_snap(int on) { g_kink_snap = on != 0; }
static void box_frame(const or_data* d, const apm_model_t* m, int g, double c[3], double A[3][3], double h[3]) {
  for (int k = 0; k < 3; k++) {
    c[k] = d->geom_xpos[g][k];
    h[k] = m->geom_size[g][k];
    for (int t = 0; t < 3; t++) A[k][t] = d->geom_xmat[g][3 * t + k]; /* A[k] = k-th box axis (world) */
  }
}
static double box_radius(const double A[3][3], const double h[3], const double n[3]) {
  return h[0] * fabs(dot3(A[0], n)) + h[1] * fabs(dot3(A[1], n)) + h[2] * fabs(dot3(A[2], n));
}
/* separation of geom2's interval [lo2, hi2] from geom1's [lo1, hi1] along +-n; keeps the best */
static int sat_axis(const double n[3], double lo1, double hi1, double lo2, double hi2, double* best, double nb[3]) {
  double s1 = lo2 - hi1, s2 = lo1 - hi2;
  double sep = s1 >= s2 ? s1 : s2;
  if (sep > *best) {
    *best = sep;
    double sg = s1 >= s2 ? 1.0 : -1.0;
    nb[0] = sg * n[0]; nb[1] = sg * n[1]; nb[2] = sg * n[2];
  }
  return sep > 0;
}
static double cyl_extent(const double a[3], double r, double h, const double n[3]) {
  double an = dot3(a, n);
  return h * fabs(an) + r * sqrt(fmax(0.0, 1.0 - an * an));
}
/* box (geom1) vs convex mesh (geom2) */
static int box_convex(const or_ctx* c, const or_data* d, int gb, int gm, or_contact* con) {
  const apm_model_t* m = c->m;
  double bc[3], A[3][3], bh[3];
  box_frame(d, m, gb, bc, A, bh);
  int mid = m->geom_dataid[gm];
  const float* hv = c->hull_vert + 3 * m->mesh_hulladr[mid];
  int nh = m->mesh_hullnum[mid];
  const double* R = d->geom_xmat[gm];
  double w[64][3];
  for (int i = 0; i < nh && i < 64; i++) {
    double v[3] = {hv[3 * i], hv[3 * i + 1], hv[3 * i + 2]};
    mulmatvec3(w[i], R, v);
    for (int k = 0; k < 3; k++) w[i][k] += d->geom_xpos[gm][k];
  }
  const or_hullfeat* f = &c->hf[mid];
  double best = -1e300, nb[3] = {0, 0, 1};
  int nax = 3 + f->nf + 3 * f->ne;
  for (int a = 0; a < nax; a++) {
    double n[3];
    if (a < 3) { memcpy(n, A[a], sizeof n); }
    else if (a < 3 + f->nf) { mulmatvec3(n, R, f->fn[a - 3]); }
    else {
      int e = (a - 3 - f->nf) / 3, k = (a - 3 - f->nf) % 3;
      double ew[3];
      mulmatvec3(ew, R, f->ed[e]);
      cross3(n, ew, A[k]);
      double len = sqrt(dot3(n, n));
      if (len < 1e-6) continue;
      for (int t = 0; t < 3; t++) n[t] /= len;
    }
    double lo = 1e300, hi = -1e300;
    for (int i = 0; i < nh; i++) {
      double pr = dot3(w[i], n);
      lo = fmin(lo, pr);
      hi = fmax(hi, pr);
    }
    double cb = dot3(bc, n), rb = box_radius(A, bh, n);
    if (sat_axis(n, cb - rb, cb + rb, lo, hi, &best, nb)) return 0;
  }
  /* witness: the hull's deepest point into the box (support along -nb), ties averaged */
  double mn = 1e300;
  for (int i = 0; i < nh; i++) mn = fmin(mn, dot3(w[i], nb));
  double wp[3] = {0, 0, 0};
  int cnt = 0;
  for (int i = 0; i < nh; i++)
    if (dot3(w[i], nb) <= mn + OR_TIE) { for (int k = 0; k < 3; k++) wp[k] += w[i][k]; cnt++; }
  con->dist = best;
  for (int k = 0; k < 3; k++) con->pos[k] = wp[k] / cnt - 0.5 * best * nb[k];
  memcpy(con->frame, nb, sizeof nb);
  return 1;
}
/* cylinder (geom1) vs box (geom2) */
static double cyl_box_sep(const double cc[3], const double a[3], double r, double h, const double bc[3],
                          const double A[3][3], const double bh[3], const double n[3], double* sgn) {
  double cn = dot3(cc, n), ce = cyl_extent(a, r, h, n);
  double cb = dot3(bc, n), rb = box_radius(A, bh, n);
  double s1 = (cb - rb) - (cn + ce), s2 = (cn - ce) - (cb + rb);
  *sgn = s1 >= s2 ? 1.0 : -1.0;
  return s1 >= s2 ? s1 : s2;
}
/* separation maximised over the directions perpendicular to box axis k (box-edge vs cap-rim
   contacts): 32 samples of the half circle, then 24 ternary-search rounds around the best */
static void edge_family(const double cc[3], const double a[3], double r, double h, const double bc[3],
                        const double A[3][3], const double bh[3], int k, double n_out[3]) {
  const double* u = A[(k + 1) % 3];
  const double* w = A[(k + 2) % 3];
  double sg, bestv = -1e300, bphi = 0;
  for (int i = 0; i < 32; i++) {
    double phi = M_PI * i / 32.0, n[3];
    for (int t = 0; t < 3; t++) n[t] = cos(phi) * u[t] + sin(phi) * w[t];
    double v = cyl_box_sep(cc, a, r, h, bc, A, bh, n, &sg);
    if (v > bestv) { bestv = v; bphi = phi; }
  }
  double lo = bphi - M_PI / 32.0, hi = bphi + M_PI / 32.0;
  for (int it = 0; it < 24; it++) {
    double m1 = lo + (hi - lo) / 3.0, m2 = hi - (hi - lo) / 3.0, n1[3], n2[3];
    for (int t = 0; t < 3; t++) {
      n1[t] = cos(m1) * u[t] + sin(m1) * w[t];
      n2[t] = cos(m2) * u[t] + sin(m2) * w[t];
    }
    if (cyl_box_sep(cc, a, r, h, bc, A, bh, n1, &sg) < cyl_box_sep(cc, a, r, h, bc, A, bh, n2, &sg)) lo = m1;
    else hi = m2;
  }
  double phi = 0.5 * (lo + hi);
  for (int t = 0; t < 3; t++) n_out[t] = cos(phi) * u[t] + sin(phi) * w[t];
  /* the family's kink: the cylinder extent h|a.n| + r sqrt(1 - (a.n)^2) has a corner at a.n = 0
     (n = +-a x A[k], a wheel rim against a box edge) where the separation peaks; the search above
     only brackets it, so snap to it when it is as good to within OR_KINK_TOL (the kernel's f32
     search is rounding-limited there; both apply this rule, ackphys_scene.inc cb_edge_family) */
  double nk[3];
  cross3(nk, a, A[k]);
  double len = sqrt(dot3(nk, nk));
  if (g_kink_snap && len >= 1e-6) {
    double il = (dot3(nk, n_out) < 0 ? -1.0 : 1.0) / len;
    for (int t = 0; t < 3; t++) nk[t] *= il;
    if (cyl_box_sep(cc, a, r, h, bc, A, bh, nk, &sg) >= cyl_box_sep(cc, a, r, h, bc, A, bh, n_out, &sg) - OR_KINK_TOL)
      memcpy(n_out, nk, sizeof nk);
  }
}
/* can an edge of the box parallel to axis k come within rb of point c? */
static int edge_reach(const double c[3], const double bc[3], const double A[3][3], const double bh[3], int k, double rb) {
  int i1 = (k + 1) % 3, i2 = (k + 2) % 3;
  double d[3] = {c[0] - bc[0], c[1] - bc[1], c[2] - bc[2]};
  double lk = dot3(d, A[k]), l1 = dot3(d, A[i1]), l2 = dot3(d, A[i2]);
  double ek = fmax(0.0, fabs(lk) - bh[k]);
  for (int e = 0; e < 4; e++) {
    double o1 = (e & 1) ? bh[i1] : -bh[i1], o2 = (e & 2) ? bh[i2] : -bh[i2];
    if (ek * ek + (l1 - o1) * (l1 - o1) + (l2 - o2) * (l2 - o2) <= rb * rb) return 1;
  }
  return 0;
}
static int cylinder_box(const or_data* d, const apm_model_t* m, int gc, int gb, or_contact* con) {
  double bc[3], A[3][3], bh[3];
  box_frame(d, m, gb, bc, A, bh);
  const double* cc = d->geom_xpos[gc];
  double a[3] = {d->geom_xmat[gc][2], d->geom_xmat[gc][5], d->geom_xmat[gc][8]};
  double r = m->geom_size[gc][0], h = m->geom_size[gc][1];
  double rbnd = sqrt(r * r + h * h);
  double best = -1e300, nb[3] = {0, 0, 1};
  for (int ax = 0; ax < 10; ax++) {
    double n[3];
    if (ax < 3) memcpy(n, A[ax], sizeof n);
    else if (ax == 3) memcpy(n, a, sizeof n);
    else if (ax < 7) {
      cross3(n, a, A[ax - 4]);
      double len = sqrt(dot3(n, n));
      if (len < 1e-6) continue;
      for (int t = 0; t < 3; t++) n[t] /= len;
    } else {
      if (!edge_reach(cc, bc, A, bh, ax - 7, rbnd)) continue;
      edge_family(cc, a, r, h, bc, A, bh, ax - 7, n);
    }
    double cn = dot3(cc, n), ce = cyl_extent(a, r, h, n);
    double cb = dot3(bc, n), rb = box_radius(A, bh, n);
    if (sat_axis(n, cn - ce, cn + ce, cb - rb, cb + rb, &best, nb)) return 0;
  }
  /* witness: the cylinder's deepest point into the box (support along +nb), ties averaged */
  double an = dot3(a, nb);
  double sg = (2 * h * fabs(an) < OR_TIE) ? 0.0 : (an > 0 ? 1.0 : -1.0);
  double rad[3] = {nb[0] - an * a[0], nb[1] - an * a[1], nb[2] - an * a[2]};
  double rl = sqrt(dot3(rad, rad));
  double rs = (r * rl < OR_TIE) ? 0.0 : r / rl;
  con->dist = best;
  for (int t = 0; t < 3; t++) con->pos[t] = cc[t] + sg * h * a[t] + rs * rad[t] + 0.5 * best * nb[t];
  memcpy(con->frame, nb, sizeof nb);
  return 1;
}

static void collision(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  d->ncon = 0;
  for (int g1 = 0; g1 < m->ngeom; g1++)
    for (int g2 = g1 + 1; g2 < m->ngeom; g2++) {
      int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
      int w1 = m->body_weldid[b1], w2 = m->body_weldid[b2];
      if (w1 == w2) continue;
      int pw1 = m->body_weldid[m->body_parentid[w1]], pw2 = m->body_weldid[m->body_parentid[w2]];
      if (w1 && w2 && (w1 == pw2 || w2 == pw1)) continue; /* filterparent */
      if (!((m->geom_contype[g1] & m->geom_conaffinity[g2]) || (m->geom_contype[g2] & m->geom_conaffinity[g1])))
        continue;
      int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
      int ga = g1, gb = g2;
      if (t1 > t2) { ga = g2; gb = g1; int t = t1; t1 = t2; t2 = t; }
      double margin = fmax(m->geom_margin[ga], m->geom_margin[gb]);
      /* broadphase: bounding spheres (planes unbounded) */
      if (t1 != APM_GEOM_PLANE) {
        double df[3] = {d->geom_xpos[ga][0] - d->geom_xpos[gb][0], d->geom_xpos[ga][1] - d->geom_xpos[gb][1],
                        d->geom_xpos[ga][2] - d->geom_xpos[gb][2]};
        double rr = m->geom_rbound[ga] + m->geom_rbound[gb] + margin;
        if (dot3(df, df) > rr * rr) continue;
      }
      or_contact tmp[8];
      int n = 0;
      if (t1 == APM_GEOM_PLANE && t2 == APM_GEOM_CYLINDER) n = plane_cylinder(d, m, ga, gb, margin, tmp);
      else if (t1 == APM_GEOM_PLANE && t2 == APM_GEOM_MESH) n = plane_convex(c, d, ga, gb, margin, tmp);
      else if (t1 == APM_GEOM_CYLINDER && t2 == APM_GEOM_BOX) n = cylinder_box(d, m, ga, gb, tmp);
      else if (t1 == APM_GEOM_BOX && t2 == APM_GEOM_MESH) n = box_convex(c, d, ga, gb, tmp);
      else continue; /* pair types not present in this model class */
      for (int k = 0; k < n && d->ncon < OR_MAXCON; k++) {
        or_contact* cc = d->con + d->ncon++;
        *cc = tmp[k];
        cc->geom1 = ga; cc->geom2 = gb;
        mix_params(m, ga, gb, cc);
        make_frame(cc->frame);
      }
    }
}

/* ------------------------------------------------------------------ jacobians */

/* translational jacobian of a world point attached to body (mj_jac) */
static void jac_point(const or_ctx* c, const or_data* d, int body, const double pt[3], double jacp[3][APM_MAXDOF]) {
  const apm_model_t* m = c->m;
  memset(jacp, 0, sizeof(double) * 3 * APM_MAXDOF);
  int b = body;
  while (b > 0 && m->body_dofnum[b] == 0) b = m->body_parentid[b];
  if (b == 0) return;
  const double* O = d->subtree_com[m->body_rootid[body]];
  double off[3] = {pt[0] - O[0], pt[1] - O[1], pt[2] - O[2]};
  int j = m->body_dofadr[b] + m->body_dofnum[b] - 1;
  while (j >= 0) {
    const double* cd = d->cdof[j];
    double t[3];
    cross3(t, cd, off);
    for (int k = 0; k < 3; k++) jacp[k][j] = cd[3 + k] + t[k];
    j = m->dof_parentid[j];
  }
}

/* ------------------------------------------------------------------ constraints */

static double power_sigmoid(double x, double mid, double p) {
  if (p == 1) return x;
  if (x <= mid) return pow(x, p) / pow(mid, p - 1);
  return 1 - pow(1 - x, p) / pow(1 - mid, p - 1);
}
static double impedance(const double solimp[5], double pos, double margin) {
  double d0 = fmin(fmax(solimp[0], mjMINIMP), mjMAXIMP);
  double dmax = fmin(fmax(solimp[1], mjMINIMP), mjMAXIMP);
  double width = solimp[2], mid = solimp[3], power = solimp[4];
  if (d0 == dmax || width <= mjMINVAL) return 0.5 * (d0 + dmax);
  double x = fabs(pos - margin) / width;
  if (x >= 1) return dmax;
  double y = power_sigmoid(x, mid, power);
  double imp = d0 + y * (dmax - d0);
  return fmin(fmax(imp, mjMINIMP), mjMAXIMP);
}

static void add_row(or_data* d, int type, const double* J, int nv, double pos, double margin, double floss,
                    double diag, const double solref[2], const double solimp[5], double timestep, int conid,
                    double rscale) {
  int i = d->nefc++;
  d->efc_type[i] = type;
  memcpy(d->efc_J[i], J, sizeof(double) * nv);
  d->efc_pos[i] = pos;
  d->efc_margin[i] = margin;
  d->efc_floss[i] = floss;
  d->efc_diag[i] = diag;
  d->efc_conid[i] = conid;
  double imp = impedance(solimp, pos, margin);
  double dmax = fmin(fmax(solimp[1], mjMINIMP), mjMAXIMP);
  double K, B;
  if (solref[0] > 0) {
    double tc = fmax(solref[0], 2 * timestep); /* refsafe */
    double dr = solref[1];
    K = 1.0 / fmax(mjMINVAL, dmax * dmax * tc * tc * dr * dr);
    B = 2.0 / fmax(mjMINVAL, dmax * tc);
  } else {
    K = -solref[0] / (dmax * dmax);
    B = -solref[1] / dmax;
  }
  d->efc_R[i] = fmax(mjMINVAL, (1 - imp) * diag * rscale / imp);
  d->efc_D[i] = 1.0 / d->efc_R[i];
  double vel = 0;
  for (int k = 0; k < nv; k++) vel += J[k] * d->qvel[k];
  d->efc_vel[i] = vel;
  d->efc_aref[i] = -B * vel - K * imp * (pos - margin);
}

static void make_constraint(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  int nv = m->nv;
  double dt = m->timestep;
  double J[APM_MAXDOF];
  d->nefc = 0;
  /* equality (joint) */
  for (int e = 0; e < m->neq; e++) {
    int j1 = m->eq_obj1id[e], j2 = m->eq_obj2id[e];
    const double* pc = m->eq_polycoef[e];
    memset(J, 0, sizeof J);
    int q1 = m->jnt_qposadr[j1], v1 = m->jnt_dofadr[j1];
    double pos, diag;
    if (j2 < 0) {
      pos = d->qpos[q1] - pc[0];
      J[v1] = 1;
      diag = m->dof_invweight0[v1];
    } else {
      int q2 = m->jnt_qposadr[j2], v2 = m->jnt_dofadr[j2];
      double dif = d->qpos[q2] - m->qpos0[q2];
      double cpos = pc[0] + dif * (pc[1] + dif * (pc[2] + dif * (pc[3] + dif * pc[4])));
      double cvel = pc[1] + dif * (2 * pc[2] + dif * (3 * pc[3] + dif * 4 * pc[4]));
      pos = d->qpos[q1] - m->qpos0[q1] - cpos;
      J[v1] = 1;
      J[v2] = -cvel;
      diag = m->dof_invweight0[v1] + m->dof_invweight0[v2];
    }
    add_row(d, 0, J, nv, pos, 0, 0, diag, m->eq_solref[e], m->eq_solimp[e], dt, -1, 1.0);
  }
  /* dof friction loss */
  for (int i = 0; i < nv; i++) {
    if (m->dof_frictionloss[i] <= 0) continue;
    memset(J, 0, sizeof J);
    J[i] = 1;
    add_row(d, 1, J, nv, 0, 0, m->dof_frictionloss[i], m->dof_invweight0[i], m->dof_solref[i], m->dof_solimp[i], dt,
            -1, 1.0);
  }
  /* joint limits (hinge) */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j] || m->jnt_type[j] != APM_JNT_HINGE) continue;
    double q = d->qpos[m->jnt_qposadr[j]];
    for (int side = -1; side <= 1; side += 2) {
      double dist = side * (m->jnt_range[j][(side + 1) / 2] - q);
      if (dist < m->jnt_margin[j]) {
        memset(J, 0, sizeof J);
        J[m->jnt_dofadr[j]] = -side;
        add_row(d, 2, J, nv, dist, m->jnt_margin[j], 0, m->dof_invweight0[m->jnt_dofadr[j]], m->jnt_solref[j],
                m->jnt_solimp[j], dt, -1, 1.0);
      }
    }
  }
  /* contacts: pyramidal cone */
  for (int ci = 0; ci < d->ncon; ci++) {
    or_contact* con = d->con + ci;
    if (!(con->dist < con->includemargin)) continue;
    int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
    double jp1[3][APM_MAXDOF], jp2[3][APM_MAXDOF], jd[3][APM_MAXDOF];
    jac_point(c, d, b1, con->pos, jp1);
    jac_point(c, d, b2, con->pos, jp2);
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < nv; i++) jd[k][i] = jp2[k][i] - jp1[k][i];
    double Jc[3][APM_MAXDOF];
    for (int r = 0; r < 3; r++)
      for (int i = 0; i < nv; i++)
        Jc[r][i] = con->frame[3 * r] * jd[0][i] + con->frame[3 * r + 1] * jd[1][i] + con->frame[3 * r + 2] * jd[2][i];
    double tran = m->body_invweight0[b1][0] + m->body_invweight0[b2][0];
    if (con->dim == 1) {
      add_row(d, 3, Jc[0], nv, con->dist, con->includemargin, 0, tran, con->solref, con->solimp, dt, ci, 1.0);
      continue;
    }
    /* condim 3: 4 pyramid edges J_n +- mu_k J_tk; all edges share one regulariser:
       R = (1-imp)/imp * tran*(1+mu0^2) * 2*mu0^2/impratio  [ext, MJX constraint.py] */
    double mu0 = con->friction[0];
    double diag = tran + mu0 * mu0 * tran;
    double rscale = 2 * mu0 * mu0 / c->m->impratio;
    for (int k = 0; k < con->dim - 1 && k < 2; k++)
      for (int s = -1; s <= 1; s += 2) {
        for (int i = 0; i < nv; i++) J[i] = Jc[0][i] + (s > 0 ? 1 : -1) * con->friction[k] * Jc[1 + k][i];
        add_row(d, 3, J, nv, con->dist, con->includemargin, 0, diag, con->solref, con->solimp, dt, ci, rscale);
      }
  }
}

/* ------------------------------------------------------------------ Newton solver */

/* constraint cost + forces at jar; returns cost; quad[i] = 1 if row in quadratic region */
static double constraint_eval(const or_data* d, const double* jar, double* force, int* quad) {
  double cost = 0;
  for (int i = 0; i < d->nefc; i++) {
    double x = jar[i], D = d->efc_D[i], R = d->efc_R[i];
    int t = d->efc_type[i];
    double f = 0;
    int q = 0;
    if (t == 0) { f = -D * x; cost += 0.5 * D * x * x; q = 1; }
    else if (t == 1) {
      double fl = d->efc_floss[i];
      if (x <= -R * fl) { f = fl; cost += -fl * x - 0.5 * R * fl * fl; }
      else if (x >= R * fl) { f = -fl; cost += fl * x - 0.5 * R * fl * fl; }
      else { f = -D * x; cost += 0.5 * D * x * x; q = 1; }
    } else {
      if (x < 0) { f = -D * x; cost += 0.5 * D * x * x; q = 1; }
    }
    if (force) force[i] = f;
    if (quad) quad[i] = q;
  }
  return cost;
}

static double total_cost(const or_ctx* c, const or_data* d, const double* a, double* jar_out) {
  int nv = c->m->nv;
  double jar[OR_MAXEFC], da[APM_MAXDOF], g = 0;
  for (int i = 0; i < nv; i++) da[i] = a[i] - d->qacc_smooth[i];
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) g += 0.5 * da[i] * d->qM[i * nv + j] * da[j];
  for (int r = 0; r < d->nefc; r++) {
    double s = 0;
    for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * a[i];
    jar[r] = s - d->efc_aref[r];
  }
  if (jar_out) memcpy(jar_out, jar, sizeof(double) * d->nefc);
  return g + constraint_eval(d, jar, NULL, NULL);
}

/* derivative of one row's cost at x = jar + alpha*Jp, times Jp; and curvature */
static void row_deriv(const or_data* d, int i, double x, double jp, double* g, double* h) {
  double D = d->efc_D[i], R = d->efc_R[i];
  int t = d->efc_type[i];
  if (t == 0) { *g += D * x * jp; *h += D * jp * jp; }
  else if (t == 1) {
    double fl = d->efc_floss[i];
    if (x <= -R * fl) *g += -fl * jp;
    else if (x >= R * fl) *g += fl * jp;
    else { *g += D * x * jp; *h += D * jp * jp; }
  } else if (x < 0) { *g += D * x * jp; *h += D * jp * jp; }
}

static int cmpd(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}

/* exact minimiser of the convex piecewise-quadratic phi(alpha) along p, alpha >= 0 */
static double line_search(const or_ctx* c, const or_data* d, const double* a, const double* p, const double* jar) {
  int nv = c->m->nv;
  double Mp[APM_MAXDOF], Jp[OR_MAXEFC];
  double pMp = 0, pg0 = 0;
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int j = 0; j < nv; j++) s += d->qM[i * nv + j] * p[j];
    Mp[i] = s;
  }
  for (int i = 0; i < nv; i++) { pMp += p[i] * Mp[i]; pg0 += Mp[i] * (a[i] - d->qacc_smooth[i]); }
  for (int r = 0; r < d->nefc; r++) {
    double s = 0;
    for (int i = 0; i < nv; i++) s += d->efc_J[r][i] * p[i];
    Jp[r] = s;
  }
  /* breakpoints */
  double bp[2 * OR_MAXEFC + 1];
  int nb = 0;
  for (int r = 0; r < d->nefc; r++) {
    if (Jp[r] == 0) continue;
    int t = d->efc_type[r];
    if (t == 2 || t == 3) {
      double al = -jar[r] / Jp[r];
      if (al > 0) bp[nb++] = al;
    } else if (t == 1) {
      double th = d->efc_R[r] * d->efc_floss[r];
      double a1 = (-th - jar[r]) / Jp[r], a2 = (th - jar[r]) / Jp[r];
      if (a1 > 0) bp[nb++] = a1;
      if (a2 > 0) bp[nb++] = a2;
    }
  }
  qsort(bp, nb, sizeof(double), cmpd);
  double lo = 0;
  for (int k = 0; k <= nb; k++) {
    double hi = (k < nb) ? bp[k] : 1e300;
    if (hi <= lo) continue;
    /* region sample point: midpoint (or lo+1 on the last, unbounded piece) */
    double mid = (k < nb) ? 0.5 * (lo + hi) : lo + 1.0;
    /* phi'(alpha) = c0 + c1*alpha on this piece */
    double g = 0, h = 0;
    for (int r = 0; r < d->nefc; r++) {
      double gg = 0, hh = 0;
      row_deriv(d, r, jar[r] + mid * Jp[r], Jp[r], &gg, &hh);
      /* gg = s'(x)*Jp evaluated at mid; linear part: s'(x) = D*x on quad pieces */
      h += hh;
      g += gg - hh * mid; /* constant part of the derivative on this piece */
    }
    double c1 = pMp + h, c0 = pg0 + g;
    double root = (c1 > 0) ? -c0 / c1 : (c0 < 0 ? 1e300 : lo);
    if (root <= lo) return lo;
    if (root < hi) return root;
    lo = hi;
  }
  return lo;
}

static void solve_newton(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  int nv = m->nv, nefc = d->nefc;
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  double a[APM_MAXDOF], jar[OR_MAXEFC], force[OR_MAXEFC];
  int quad[OR_MAXEFC];
  /* warmstart: pick the cheaper of qacc_warmstart and qacc_smooth */
  double cw = total_cost(c, d, d->qacc_warmstart, NULL);
  double cs = total_cost(c, d, d->qacc_smooth, NULL);
  memcpy(a, cw < cs ? d->qacc_warmstart : d->qacc_smooth, sizeof(double) * nv);
  d->solver_niter = 0;
  if (nefc == 0) {
    memcpy(d->qacc, d->qacc_smooth, sizeof(double) * nv);
    memset(d->qfrc_constraint, 0, sizeof(double) * nv);
    return;
  }
  double cost = total_cost(c, d, a, jar);
  for (int iter = 0; iter < c->maxiter; iter++) {
    constraint_eval(d, jar, force, quad);
    double grad[APM_MAXDOF], H[APM_MAXDOF * APM_MAXDOF], p[APM_MAXDOF];
    for (int i = 0; i < nv; i++) {
      double s = 0;
      for (int j = 0; j < nv; j++) s += d->qM[i * nv + j] * (a[j] - d->qacc_smooth[j]);
      for (int r = 0; r < nefc; r++) s -= d->efc_J[r][i] * force[r];
      grad[i] = s;
    }
    memcpy(H, d->qM, sizeof(double) * nv * nv);
    for (int r = 0; r < nefc; r++) {
      if (!quad[r]) continue;
      for (int i = 0; i < nv; i++) {
        if (d->efc_J[r][i] == 0) continue;
        for (int j = 0; j < nv; j++) H[i * nv + j] += d->efc_D[r] * d->efc_J[r][i] * d->efc_J[r][j];
      }
    }
    if (cholesky(H, nv)) break;
    for (int i = 0; i < nv; i++) p[i] = -grad[i];
    chol_solve(H, nv, p);
    double alpha = line_search(c, d, a, p, jar);
    d->solver_niter = iter + 1;
    if (alpha == 0) break;
    for (int i = 0; i < nv; i++) a[i] += alpha * p[i];
    double newcost = total_cost(c, d, a, jar);
    double improvement = scale * (cost - newcost);
    cost = newcost;
    /* gradient at the new point */
    constraint_eval(d, jar, force, quad);
    double gn = 0;
    for (int i = 0; i < nv; i++) {
      double s = 0;
      for (int j = 0; j < nv; j++) s += d->qM[i * nv + j] * (a[j] - d->qacc_smooth[j]);
      for (int r = 0; r < nefc; r++) s -= d->efc_J[r][i] * force[r];
      gn += s * s;
    }
    double gradient = scale * sqrt(gn);
    if (improvement < c->tolerance || gradient < c->tolerance) break;
  }
  constraint_eval(d, jar, force, quad);
  memcpy(d->qacc, a, sizeof(double) * nv);
  memcpy(d->efc_force, force, sizeof(double) * nefc);
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int r = 0; r < nefc; r++) s += d->efc_J[r][i] * force[r];
    d->qfrc_constraint[i] = s;
  }
}

/* ------------------------------------------------------------------ ray casting (mj_ray) */

static double ray_quad(double a, double b, double c, double x[2]) {
  double det = b * b - a * c;
  if (det < mjMINVAL) { x[0] = x[1] = -1; return -1; }
  det = sqrt(det);
  x[0] = (-b - det) / a;
  x[1] = (-b + det) / a;
  if (x[0] >= 0) return x[0];
  if (x[1] >= 0) return x[1];
  return -1;
}
static void ray_map(const double pos[3], const double mat[9], const double pnt[3], const double vec[3], double lp[3],
                    double lv[3]) {
  double dif[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]};
  mulmatTvec3(lp, mat, dif);
  mulmatTvec3(lv, mat, vec);
}
static double ray_sphere_bound(const double pos[3], double r2, const double pnt[3], const double vec[3]) {
  double dif[3] = {pnt[0] - pos[0], pnt[1] - pos[1], pnt[2] - pos[2]}, x[2];
  return ray_quad(dot3(vec, vec), dot3(vec, dif), dot3(dif, dif) - r2, x);
}
static double ray_plane(const double pos[3], const double mat[9], const double size[3], const double pnt[3],
                        const double vec[3]) {
  double lp[3], lv[3];
  ray_map(pos, mat, pnt, vec, lp, lv);
  if (lv[2] > -mjMINVAL) return -1;
  double x = -lp[2] / lv[2];
  if (x < 0) return -1;
  double p0 = lp[0] + x * lv[0], p1 = lp[1] + x * lv[1];
  if ((size[0] <= 0 || fabs(p0) <= size[0]) && (size[1] <= 0 || fabs(p1) <= size[1])) return x;
  return -1;
}
static double ray_cylinder(const double pos[3], const double mat[9], const double size[3], const double pnt[3],
                           const double vec[3]) {
  if (ray_sphere_bound(pos, size[0] * size[0] + size[1] * size[1], pnt, vec) < 0) return -1;
  double lp[3], lv[3], x = -1;
  ray_map(pos, mat, pnt, vec, lp, lv);
  for (int side = -1; side <= 1; side += 2) {
    if (lv[2] != 0) {
      double sol = (side * size[1] - lp[2]) / lv[2];
      if (sol >= 0) {
        double p0 = lp[0] + sol * lv[0], p1 = lp[1] + sol * lv[1];
        if (p0 * p0 + p1 * p1 <= size[0] * size[0] && (x < 0 || sol < x)) x = sol;
      }
    }
  }
  double xx[2];
  ray_quad(lv[0] * lv[0] + lv[1] * lv[1], lv[0] * lp[0] + lv[1] * lp[1], lp[0] * lp[0] + lp[1] * lp[1] - size[0] * size[0],
           xx);
  for (int i = 0; i < 2; i++)
    if (xx[i] >= 0 && fabs(lp[2] + xx[i] * lv[2]) <= size[1] && (x < 0 || xx[i] < x)) x = xx[i];
  return x;
}
/* ray vs box: nearest face-plane crossing x >= 0 whose point lies on the face (entry distance
   from outside, exit distance from inside) */
static double ray_box(const double pos[3], const double mat[9], const double size[3], const double pnt[3],
                      const double vec[3]) {
  if (ray_sphere_bound(pos, dot3(size, size), pnt, vec) < 0) return -1;
  double lp[3], lv[3], x = -1;
  ray_map(pos, mat, pnt, vec, lp, lv);
  for (int i = 0; i < 3; i++) {
    if (fabs(lv[i]) < mjMINVAL) continue;
    for (int side = -1; side <= 1; side += 2) {
      double sol = (side * size[i] - lp[i]) / lv[i];
      if (sol < 0) continue;
      int in = 1;
      for (int j = 0; j < 3; j++)
        if (j != i && fabs(lp[j] + sol * lv[j]) > size[j]) in = 0;
      if (in && (x < 0 || sol < x)) x = sol;
    }
  }
  return x;
}
/* ray vs triangle (a,b,c): Moller-Trumbore in the mesh frame; nearest x >= 0 or -1 */
static double ray_triangle(const double a[3], const double b[3], const double cc[3], const double lp[3],
                           const double lv[3]) {
  double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {cc[0] - a[0], cc[1] - a[1], cc[2] - a[2]};
  double pv[3], tv[3], qv[3];
  cross3(pv, lv, e2);
  double det = dot3(e1, pv);
  if (fabs(det) < mjMINVAL) return -1;
  double inv = 1.0 / det;
  tv[0] = lp[0] - a[0]; tv[1] = lp[1] - a[1]; tv[2] = lp[2] - a[2];
  double u = dot3(tv, pv) * inv;
  if (u < 0 || u > 1) return -1;
  cross3(qv, tv, e1);
  double v = dot3(lv, qv) * inv;
  if (v < 0 || u + v > 1) return -1;
  double x = dot3(e2, qv) * inv;
  return x >= 0 ? x : -1;
}
static double ray_mesh(const or_ctx* c, const or_data* d, int g, const double pnt[3], const double vec[3]) {
  const apm_model_t* m = c->m;
  if (ray_sphere_bound(d->geom_xpos[g], m->geom_rbound[g] * m->geom_rbound[g], pnt, vec) < 0) return -1;
  double lp[3], lv[3], x = -1;
  ray_map(d->geom_xpos[g], d->geom_xmat[g], pnt, vec, lp, lv);
  int mid = m->geom_dataid[g];
  /* mesh AABB slab test in the mesh frame (pure prefilter: the result is unchanged) */
  {
    double tmin = 0, tmax = 1e300;
    for (int k = 0; k < 3; k++) {
      double lo = m->mesh_aabb[mid][k] - m->mesh_aabb[mid][3 + k], hi = m->mesh_aabb[mid][k] + m->mesh_aabb[mid][3 + k];
      if (fabs(lv[k]) < mjMINVAL) {
        if (lp[k] < lo || lp[k] > hi) return -1;
      } else {
        double t1 = (lo - lp[k]) / lv[k], t2 = (hi - lp[k]) / lv[k];
        if (t1 > t2) { double t = t1; t1 = t2; t2 = t; }
        if (t1 > tmin) tmin = t1;
        if (t2 < tmax) tmax = t2;
        if (tmin > tmax) return -1;
      }
    }
  }
  const float* V = c->mesh_vert + 3 * m->mesh_vertadr[mid];
  const int32_t* F = c->mesh_face + 3 * m->mesh_faceadr[mid];
  for (int f = 0; f < m->mesh_facenum[mid]; f++) {
    double tri[3][3];
    for (int k = 0; k < 3; k++)
      for (int t = 0; t < 3; t++) tri[k][t] = V[3 * F[3 * f + k] + t];
    double s = ray_triangle(tri[0], tri[1], tri[2], lp, lv);
    if (s >= 0 && (x < 0 || s < x)) x = s;
  }
  return x;
}
static double mj_ray(const or_ctx* c, const or_data* d, const double pnt[3], const double vec[3], int bodyexclude) {
  const apm_model_t* m = c->m;
  double dist = -1;
  for (int g = 0; g < m->ngeom; g++) {
    if (m->geom_bodyid[g] == bodyexclude) continue;
    if (m->geom_rgba[g][3] == 0) continue;
    double nd;
    switch (m->geom_type[g]) {
      case APM_GEOM_PLANE: nd = ray_plane(d->geom_xpos[g], d->geom_xmat[g], m->geom_size[g], pnt, vec); break;
      case APM_GEOM_CYLINDER: nd = ray_cylinder(d->geom_xpos[g], d->geom_xmat[g], m->geom_size[g], pnt, vec); break;
      case APM_GEOM_BOX: nd = ray_box(d->geom_xpos[g], d->geom_xmat[g], m->geom_size[g], pnt, vec); break;
      case APM_GEOM_MESH: nd = ray_mesh(c, d, g, pnt, vec); break;
      default: nd = -1;
    }
    if (nd >= 0 && (nd < dist || dist < 0)) dist = nd;
  }
  return dist;
}

static void sensors(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  for (int s = 0; s < m->nsensor; s++) {
    double v = 0;
    int o = m->sensor_objid[s];
    switch (m->sensor_type[s]) {
      case APM_SENS_JOINTPOS: v = d->qpos[m->jnt_qposadr[o]]; break;
      case APM_SENS_JOINTVEL: v = d->qvel[m->jnt_dofadr[o]]; break;
      case APM_SENS_RANGEFINDER: {
        double dir[3] = {d->site_xmat[o][2], d->site_xmat[o][5], d->site_xmat[o][8]};
        v = mj_ray(c, d, d->site_xpos[o], dir, m->site_bodyid[o]);
        break;
      }
    }
    /* cutoff: rangefinder data are "positive": clamp above only, -1 (no hit) preserved */
    if (m->sensor_cutoff[s] > 0) {
      if (m->sensor_type[s] == APM_SENS_RANGEFINDER) v = fmin(v, m->sensor_cutoff[s]);
      else v = fmin(fmax(v, -m->sensor_cutoff[s]), m->sensor_cutoff[s]);
    }
    d->sensordata[m->sensor_adr[s]] = v;
  }
}

/* ------------------------------------------------------------------ mj_forward / mj_step */

static int is_bad(double x) { return isnan(x) || fabs(x) > mjMAXVAL; }

static void reset_data(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  memcpy(d->qpos, m->qpos0, sizeof(double) * m->nq);
  memset(d->qvel, 0, sizeof(double) * m->nv);
  memset(d->qacc_warmstart, 0, sizeof(double) * m->nv);
  memset(d->ctrl, 0, sizeof(double) * m->nu);
}

static void forward(const or_ctx* c, or_data* d, uint32_t flags) {
  const apm_model_t* m = c->m;
  OR_STAGE(2);
  kinematics(c, d);
  com_pos(c, d);
  OR_STAGE(3);
  crb(c, d);
  OR_STAGE(4);
  if (flags & FLAG_CONTACTS) collision(c, d);
  else d->ncon = 0;
  OR_STAGE(5);
  sensors(c, d); /* positional + velocity sensors (joint sensors read qpos/qvel directly) */
  OR_STAGE(6);
  com_vel(c, d);
  rne(c, d);
  passive(c, d);
  actuation(c, d);
  OR_STAGE(7);
  int nv = m->nv;
  for (int i = 0; i < nv; i++) d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i];
  double L[APM_MAXDOF * APM_MAXDOF];
  memcpy(L, d->qM, sizeof(double) * nv * nv);
  cholesky(L, nv);
  memcpy(d->qacc_smooth, d->qfrc_smooth, sizeof(double) * nv);
  chol_solve(L, nv, d->qacc_smooth);
  OR_STAGE(8);
  make_constraint(c, d);
  OR_STAGE(9);
  solve_newton(c, d);
  OR_STAGE(0);
}

static void integrate_pos(const or_ctx* c, double* qpos, const double* qvel, double h) {
  const apm_model_t* m = c->m;
  for (int j = 0; j < m->njnt; j++) {
    int pa = m->jnt_qposadr[j], va = m->jnt_dofadr[j];
    if (m->jnt_type[j] == APM_JNT_FREE) {
      for (int k = 0; k < 3; k++) qpos[pa + k] += h * qvel[va + k];
      /* mju_quatIntegrate: q <- normalize(q) * exp(h*w/2), w in the local frame */
      double w[3] = {qvel[va + 3], qvel[va + 4], qvel[va + 5]};
      double ang = h * normalize3(w);
      double qr[4] = {cos(0.5 * ang), w[0] * sin(0.5 * ang), w[1] * sin(0.5 * ang), w[2] * sin(0.5 * ang)};
      double* q = qpos + pa + 3;
      normalize4(q);
      mulquat(q, q, qr);
    } else {
      qpos[pa] += h * qvel[va];
    }
  }
}

static void euler(const or_ctx* c, or_data* d) {
  const apm_model_t* m = c->m;
  int nv = m->nv;
  double h = m->timestep, MhB[APM_MAXDOF * APM_MAXDOF], qacc[APM_MAXDOF];
  memcpy(MhB, d->qM, sizeof(double) * nv * nv);
  int dmp = 0;
  for (int i = 0; i < nv; i++)
    if (m->dof_damping[i] > 0) dmp = 1;
  if (dmp) {
    for (int i = 0; i < nv; i++) MhB[i * nv + i] += h * m->dof_damping[i];
    cholesky(MhB, nv);
    for (int i = 0; i < nv; i++) qacc[i] = d->qfrc_smooth[i] + d->qfrc_constraint[i];
    chol_solve(MhB, nv, qacc);
  } else {
    memcpy(qacc, d->qacc, sizeof(double) * nv);
  }
  for (int i = 0; i < nv; i++) d->qvel[i] += h * qacc[i];
  integrate_pos(c, d->qpos, d->qvel, h);
  memcpy(d->qacc_warmstart, d->qacc, sizeof(double) * nv);
}

static void mj_step(const or_ctx* c, or_data* d, uint32_t flags) {
  const apm_model_t* m = c->m;
  d->bad_state = 0;
  for (int i = 0; i < m->nq; i++)
    if (is_bad(d->qpos[i])) d->bad_state = 1;
  for (int i = 0; i < m->nv; i++)
    if (is_bad(d->qvel[i])) d->bad_state = 1;
  if (d->bad_state) reset_data(c, d);
  forward(c, d, flags);
  int bad = 0;
  for (int i = 0; i < m->nv; i++)
    if (is_bad(d->qacc[i])) bad = 1;
  if (bad) {
    d->bad_state = 1;
    reset_data(c, d);
    forward(c, d, flags);
  }
  OR_STAGE(10);
  euler(c, d);
  OR_STAGE(0);
}

/* ------------------------------------------------------------------ env glue */

/* BicycleController.cmd_vel_to_controls + apply_cmd_vel (controller.py:98-140); ctrl[3] */
void or_controller2(const float action[2], double max_lin, double max_ang, double ctrl[3]) {
  /* np.clip of the float32 action; action[i] * python float stays float32 (NumPy 2 promotion) */
  float a0 = action[0], a1 = action[1];
  a0 = a0 < -1.0f ? -1.0f : (a0 > 1.0f ? 1.0f : a0);
  a1 = a1 < -1.0f ? -1.0f : (a1 > 1.0f ? 1.0f : a1);
  volatile float lx = a0 * (float)max_lin, az = a1 * (float)max_ang;
  double v = (double)lx, omega = (double)az, eps = 1e-5, delta;
  if (fabs(omega) < 1e-6) delta = 0.0;
  else {
    double den = fabs(v) > eps ? v : ((omega > 0) - (omega < 0)) * eps;
    delta = atan((CTL_WHEELBASE * omega) / den);
  }
  double lim = 35.0 * (M_PI / 180.0); /* np.deg2rad(35) */
  if (delta < -lim) delta = -lim;
  if (delta > lim) delta = lim;
  double vl, vr;
  if (fabs(delta) < 1e-6) vl = vr = v;
  else {
    double t = tan(delta);
    double R = fabs(t) > eps ? CTL_WHEELBASE / t : INFINITY;
    double wt = fabs(R) > eps ? v / R : 0.0;
    vl = wt * (R - CTL_TRACK / 2.0);  /* 0 * inf -> NaN when R is infinite (as in the reference) */
    vr = wt * (R + CTL_TRACK / 2.0);
  }
  double wl = vl / CTL_WHEEL_R, wr = vr / CTL_WHEEL_R;
  double c0 = delta < -0.61 ? -0.61 : (delta > 0.61 ? 0.61 : delta);
  double c1 = isnan(wl) ? wl : (wl < -50 ? -50 : (wl > 50 ? 50 : wl));
  double c2 = isnan(wr) ? wr : (wr < -50 ? -50 : (wr > 50 ? 50 : wr));
  ctrl[0] = c0; ctrl[1] = c1; ctrl[2] = c2;
}

void or_controller(const float action[2], double ctrl[3]) { or_controller2(action, 1.0, 1.0, ctrl); }

/* odometry yaw (odometry.py:154-170) */
static double quat_yaw(const double q[4]) {
  return atan2(2 * (q[0] * q[3] + q[1] * q[2]), 1 - 2 * (q[2] * q[2] + q[3] * q[3]));
}

/* _get_observation + _calculate_reward on the current forward data (pre-integration) */
static void observe(const or_ctx* c, const or_data* d, const double goal[2], const double ref[3], double obs[NOBS],
                    double* reward, int* term, double info[3]) {
  const double* xp = d->xpos[c->chassis_body];
  double pos[3] = {xp[0] - ref[0], xp[1] - ref[1], xp[2] - ref[2]};
  double yaw = quat_yaw(d->xquat[c->chassis_body]);
  for (int i = 0; i < 72; i++) obs[i] = (float)d->sensordata[c->lidar_adr[i]];
  obs[72] = (float)pos[0];
  obs[73] = (float)pos[1];
  obs[74] = (float)yaw;
  double gx = goal[0] - pos[0], gy = goal[1] - pos[1];
  double dist = sqrt(gx * gx + gy * gy);
  double ang = atan2(gy, gx) - yaw;
  ang = atan2(sin(ang), cos(ang));
  obs[75] = (float)gx; obs[76] = (float)gy; obs[77] = (float)dist; obs[78] = (float)ang;
  double minl = 1e300;
  for (int i = 0; i < 72; i++) {
    double v = d->sensordata[c->lidar_adr[i]];
    if (c->nohit_clear && v < 0) continue; /* variant: a no-hit reading is no obstacle */
    if (v < minl) minl = v;
  }
  int coll = minl < c->coll_thresh;
  if (c->nohit_clear && minl == 1e300) minl = -1.0;
  int t = dist < c->goal_thresh;
  double r = 0.0;
  r -= dist * 0.1;
  if (t) r += 100.0;
  if (coll) r -= 50.0;
  r -= 0.01;
  *reward = r;
  *term = t;
  if (info) { info[0] = minl; info[1] = coll; info[2] = dist; }
}

static void load_state(const or_ctx* c, or_data* d, const double* st) {
  memset(d, 0, sizeof(*d));
  memcpy(d->qpos, st + ST_QPOS, sizeof(double) * c->m->nq);
  memcpy(d->qvel, st + ST_QVEL, sizeof(double) * c->m->nv);
  memcpy(d->qacc_warmstart, st + ST_WARM, sizeof(double) * c->m->nv);
}
static void store_state(const or_ctx* c, const or_data* d, double* st) {
  memcpy(st + ST_QPOS, d->qpos, sizeof(double) * c->m->nq);
  memcpy(st + ST_QVEL, d->qvel, sizeof(double) * c->m->nv);
  memcpy(st + ST_WARM, d->qacc_warmstart, sizeof(double) * c->m->nv);
}

/* reset one env (a14): spawner pose, zero velocity/warmstart, Philox goal, mj_forward, obs */
static void env_reset(const or_ctx* c, or_data* d, double* st, int env, uint64_t seed, double obs[NOBS]) {
  const apm_model_t* m = c->m;
  double episode = st[ST_EPIS] + 1;
  memset(d, 0, sizeof(*d));
  memcpy(d->qpos, m->qpos0, sizeof(double) * m->nq);
  /* simple_map_spawner.py:43 (robot_pos=[0,0,0.1]); the obstacle scene's spawn is its own */
  d->qpos[0] = m->spawn[0]; d->qpos[1] = m->spawn[1]; d->qpos[2] = m->spawn[2];
  d->qpos[3] = 1; d->qpos[4] = 0; d->qpos[5] = 0; d->qpos[6] = 0; /* :50 */
  /* mj_forward (simple_map_spawner.py:52): only its position stage feeds the env state / obs */
  kinematics(c, d);
  com_pos(c, d);
  sensors(c, d);
  uint32_t ctr[4] = {(uint32_t)(env + c->env_offset), (uint32_t)episode, 0u, 0u};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  philox4x32_10(ctr, key);
  double dd = 2.0 + 6.0 * u01(ctr[0]);
  double th = 2.0 * M_PI * u01(ctr[1]);
  /* goal = robot_start_position + offset (ackermann_env.py:167-172), in the odometry frame:
     robot_start_position is the odometry position at reset, i.e. (0, 0) (odometry.py:62-103
     measures from the reset pose), whatever the spawn point */
  st[ST_GOAL] = dd * cos(th);
  st[ST_GOAL + 1] = dd * sin(th);
  if (c->goal_cells > 0) { /* opt-in maze task: free cell floor(u * #cells within goal_cells) */
    uint32_t nle = 0;
    for (int i = 0; i < c->nfree; i++) nle += c->free_d[i] <= c->goal_cells;
    const uint32_t i = (uint32_t)(((uint64_t)(ctr[0] >> 8) * nle) >> 24);
    st[ST_GOAL] = c->free_xy[i][0] - m->spawn[0];
    st[ST_GOAL + 1] = c->free_xy[i][1] - m->spawn[1];
  }
  memcpy(st + ST_REF, d->xpos[c->chassis_body], sizeof(double) * 3);
  st[ST_STEP] = 0;
  st[ST_EPIS] = episode;
  store_state(c, d, st);
  double r;
  int t;
  observe(c, d, st + ST_GOAL, st + ST_REF, obs, &r, &t, NULL);
}

/* one env step (a1): state in/out [44], action [2] (float32 as the Gym Box dtype) */
static void env_step(const or_ctx* c, or_data* d, double* st, const float* action, uint32_t flags, int env,
                     uint64_t seed, double obs[NOBS], double* reward, uint8_t* term, uint8_t* trunc,
                     double* terminal_obs, double info[4]) {
  load_state(c, d, st);
  double ctrl[3];
  OR_STAGE(1);
  or_controller2(action, c->max_lin, c->max_ang, ctrl);
  OR_STAGE(0);
  d->bad_ctrl = 0;
  for (int k = 0; k < 3; k++)
    if (is_bad(ctrl[k])) d->bad_ctrl = 1;
  if (d->bad_ctrl) ctrl[0] = ctrl[1] = ctrl[2] = 0; /* MuJoCo zeroes ctrl on bad values [ext] */
  d->ctrl[c->act_steer] = ctrl[0];
  d->ctrl[c->act_rl] = ctrl[1];
  d->ctrl[c->act_rr] = ctrl[2];
  /* action_repeat mj_steps with the same ctrl (1 = the reference); the observation below comes from
     the last one's forward pass (its pre-integration pose), as after a single mj_step */
  for (int s = 0; s < c->action_repeat; s++) mj_step(c, d, flags);
  if (flags & FLAG_POSTSTEP_OBS) { /* mj_forward's position stage on the integrated state feeds the obs */
    kinematics(c, d);
    com_pos(c, d);
    sensors(c, d);
  }
  int t;
  double inf3[3];
  OR_STAGE(11);
  observe(c, d, st + ST_GOAL, st + ST_REF, obs, reward, &t, inf3);
  OR_STAGE(0);
  store_state(c, d, st);
  st[ST_STEP] += 1;
  int tr = st[ST_STEP] >= c->max_steps;
  *term = (uint8_t)t;
  *trunc = (uint8_t)tr;
  if (info) { info[0] = inf3[0]; info[1] = inf3[1]; info[2] = inf3[2]; info[3] = d->bad_state; }
  if ((flags & FLAG_AUTORESET) && (t || tr)) {
    if (terminal_obs) memcpy(terminal_obs, obs, sizeof(double) * NOBS);
    OR_STAGE(12);
    env_reset(c, d, st, env, seed, obs);
    OR_STAGE(0);
  }
}

/* golden-vector entry: _get_observation/_calculate_reward from raw mjData fields */
int or_observe_raw(const or_ctx* c, const double xpos[3], const double xquat[4], const double* sensordata,
                   const double goal[2], const double ref[3], double obs[NOBS], double* reward, int* term,
                   double info[3]) {
  or_data* d = (or_data*)calloc(1, sizeof(or_data));
  memcpy(d->xpos[c->chassis_body], xpos, sizeof(double) * 3);
  memcpy(d->xquat[c->chassis_body], xquat, sizeof(double) * 4);
  memcpy(d->sensordata, sensordata, sizeof(double) * c->m->nsensordata);
  observe(c, d, goal, ref, obs, reward, term, info);
  free(d);
  return 0;
}

/* ------------------------------------------------------------------ exported batch API */

/* states [n][44] (f64, in/out), actions [n][2] f32, obs [n][79], reward [n], term/trunc [n],
   terminal_obs [n][79] (nullable), info [n][4] (nullable). OpenMP over envs. */
int or_step_batch(const or_ctx* c, int n, double* states, const float* actions, uint32_t flags, uint64_t seed,
                  double* obs, double* reward, uint8_t* term, uint8_t* trunc, double* terminal_obs, double* info,
                  int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
#endif
    or_data* d = (or_data*)malloc(sizeof(or_data));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int e = 0; e < n; e++)
      env_step(c, d, states + (size_t)e * NSTATE, actions + 2 * (size_t)e, flags, e, seed, obs + (size_t)e * NOBS,
               reward + e, term + e, trunc + e, terminal_obs ? terminal_obs + (size_t)e * NOBS : NULL,
               info ? info + 4 * (size_t)e : NULL);
    free(d);
#ifdef _OPENMP
  }
#endif
  return 0;
}

int or_reset_batch(const or_ctx* c, int n, const uint8_t* mask, uint64_t seed, double* states, double* obs) {
  or_data* d = (or_data*)malloc(sizeof(or_data));
  for (int e = 0; e < n; e++)
    if (!mask || mask[e]) env_reset(c, d, states + (size_t)e * NSTATE, e, seed, obs + (size_t)e * NOBS);
  free(d);
  return 0;
}

/* diagnostics for tests: one forward+step of a single env, dumping intermediate quantities.
   out layout (doubles): see oracle/oracle.py DIAG_FIELDS. */
int or_step_diag(const or_ctx* c, const double* st_in, const double* ctrl_in, uint32_t flags, double* out) {
  or_data* d = (or_data*)calloc(1, sizeof(or_data));
  const apm_model_t* m = c->m;
  load_state(c, d, st_in);
  memcpy(d->ctrl, ctrl_in, sizeof(double) * m->nu);
  d->bad_state = 0;
  forward(c, d, flags);
  int nv = m->nv, o = 0;
  memcpy(out + o, d->qM, sizeof(double) * nv * nv); o += nv * nv;
  memcpy(out + o, d->qfrc_bias, sizeof(double) * nv); o += nv;
  memcpy(out + o, d->qfrc_passive, sizeof(double) * nv); o += nv;
  memcpy(out + o, d->qfrc_actuator, sizeof(double) * nv); o += nv;
  memcpy(out + o, d->qacc_smooth, sizeof(double) * nv); o += nv;
  memcpy(out + o, d->qacc, sizeof(double) * nv); o += nv;
  memcpy(out + o, d->qfrc_constraint, sizeof(double) * nv); o += nv;
  out[o++] = d->ncon;
  out[o++] = d->nefc;
  out[o++] = d->solver_niter;
  for (int k = 0; k < 32; k++) {
    if (k < d->ncon) {
      memcpy(out + o, d->con[k].pos, sizeof(double) * 3);
      out[o + 3] = d->con[k].dist;
      out[o + 4] = d->con[k].geom2;
    } else memset(out + o, 0, sizeof(double) * 5);
    o += 5;
  }
  memcpy(out + o, d->sensordata, sizeof(double) * m->nsensordata); o += m->nsensordata;
  memcpy(out + o, d->xpos[c->chassis_body], sizeof(double) * 3); o += 3;
  memcpy(out + o, d->xquat[c->chassis_body], sizeof(double) * 4); o += 4;
  memcpy(out + o, d->subtree_com[c->chassis_body], sizeof(double) * 3); o += 3;
  /* efc rows */
  for (int r = 0; r < 96; r++) {
    if (r < d->nefc) {
      out[o] = d->efc_type[r]; out[o + 1] = d->efc_pos[r]; out[o + 2] = d->efc_R[r];
      out[o + 3] = d->efc_aref[r]; out[o + 4] = d->efc_force[r]; out[o + 5] = d->efc_diag[r];
    } else memset(out + o, 0, sizeof(double) * 6);
    o += 6;
  }
  /* efc jacobian rows */
  for (int r = 0; r < 96; r++) {
    if (r < d->nefc) memcpy(out + o, d->efc_J[r], sizeof(double) * nv);
    else memset(out + o, 0, sizeof(double) * nv);
    o += nv;
  }
  euler(c, d);
  memcpy(out + o, d->qpos, sizeof(double) * m->nq); o += m->nq;
  memcpy(out + o, d->qvel, sizeof(double) * nv); o += nv;
  free(d);
  return o;
}

/* test export: the contacts mj_collision produces at qpos (mj_kinematics first); per contact
   out[16] = geom1, geom2, dist, pos[3], frame[9], dim. Returns the number of contacts. */
int or_contacts(const or_ctx* c, const double* qpos, double* out, int maxcon) {
  or_data* d = (or_data*)calloc(1, sizeof(or_data));
  memcpy(d->qpos, qpos, sizeof(double) * c->m->nq);
  kinematics(c, d);
  collision(c, d);
  int n = d->ncon < maxcon ? d->ncon : maxcon;
  for (int k = 0; k < n; k++) {
    const or_contact* cc = d->con + k;
    double* o = out + 16 * k;
    o[0] = cc->geom1; o[1] = cc->geom2; o[2] = cc->dist;
    memcpy(o + 3, cc->pos, sizeof(double) * 3);
    memcpy(o + 6, cc->frame, sizeof(double) * 9);
    o[15] = cc->dim;
  }
  free(d);
  return n;
}
/* test export: mj_ray from pnt along unit vec (no body excluded) */
double or_ray(const or_ctx* c, const double* qpos, const double pnt[3], const double vec[3]) {
  or_data* d = (or_data*)calloc(1, sizeof(or_data));
  memcpy(d->qpos, qpos, sizeof(double) * c->m->nq);
  kinematics(c, d);
  double r = mj_ray(c, d, pnt, vec, -1);
  free(d);
  return r;
}

/* ------------------------------------------------------------------ host twin of the C-ABI */

static float f32_of_u32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u32_of_f32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static void soa_to_row(const float* state, int n, int e, double st[NSTATE]) {
  for (int k = 0; k < NSTATE; k++) st[k] = state[(size_t)k * n + e];
  st[ST_STEP] = u32_of_f32(state[(size_t)ST_STEP * n + e]);
  st[ST_EPIS] = u32_of_f32(state[(size_t)ST_EPIS * n + e]);
}
static void row_to_soa(const double st[NSTATE], int n, int e, float* state) {
  for (int k = 0; k < NSTATE; k++) state[(size_t)k * n + e] = (float)st[k];
  state[(size_t)ST_STEP * n + e] = f32_of_u32((uint32_t)st[ST_STEP]);
  state[(size_t)ST_EPIS * n + e] = f32_of_u32((uint32_t)st[ST_EPIS]);
}

/* ackphys_step (include/ackphys.h) on host SoA buffers; episode stats as the kernel keeps them */
int ackphys_step_cpu(or_ctx* c, int n, const float* action, float* state, float* obs, float* reward,
                     uint8_t* term, uint8_t* trunc, float* terminal_obs, float* info, float* episode,
                     uint32_t flags, uint64_t seed, int nthreads) {
  if (!c || n < 0 || !action || !state || !obs || !reward || !term || !trunc) return -1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
#endif
    or_data* d = (or_data*)malloc(sizeof(or_data));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int e = 0; e < n; e++) {
      double st[NSTATE], o[NOBS], to[NOBS], inf[4], r;
      soa_to_row(state, n, e, st);
      env_step(c, d, st, action + 2 * (size_t)e, flags, e, seed, o, &r, term + e, trunc + e, to, inf);
      row_to_soa(st, n, e, state);
      const int done = term[e] || trunc[e];
      const double* src = ((flags & FLAG_AUTORESET) && done && terminal_obs) ? to : o;
      float* dst = ((flags & FLAG_AUTORESET) && done && terminal_obs) ? terminal_obs : obs;
      for (int k = 0; k < NOBS; k++) dst[(size_t)k * n + e] = (float)src[k];
      if ((flags & FLAG_AUTORESET) && done && terminal_obs)
        for (int k = 0; k < NOBS; k++) obs[(size_t)k * n + e] = (float)o[k];
      reward[e] = (float)r;
      if (info)
        for (int k = 0; k < 4; k++) info[(size_t)k * n + e] = (float)inf[k];
      if (episode) {
        float ret = episode[e] + (float)r, len = episode[(size_t)n + e] + 1.0f;
        if (done) {
          episode[2 * (size_t)n + e] += ret;
          episode[3 * (size_t)n + e] += 1.0f;
          ret = 0.0f;
          len = 0.0f;
        }
        episode[e] = ret;
        episode[(size_t)n + e] = len;
      }
    }
    free(d);
#ifdef _OPENMP
  }
#endif
  return 0;
}

int ackphys_reset_cpu(or_ctx* c, int n, const uint8_t* mask, uint64_t seed, float* state, float* obs) {
  if (!c || n < 0 || !state || !obs) return -1;
  or_data* d = (or_data*)malloc(sizeof(or_data));
  for (int e = 0; e < n; e++) {
    if (mask && !mask[e]) continue;
    double st[NSTATE], o[NOBS];
    soa_to_row(state, n, e, st);
    env_reset(c, d, st, e, seed, o);
    row_to_soa(st, n, e, state);
    for (int k = 0; k < NOBS; k++) obs[(size_t)k * n + e] = (float)o[k];
  }
  free(d);
  return 0;
}
