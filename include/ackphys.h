/* ackphys.h -- C-ABI of libackphys.so, the MI355X batched physics step for the
 * ackermann_robot_v2 environment.
 *
 * This is the drop-in boundary that replaces, for N environments at once, the reference's
 * per-env call chain (one Python env per process, src/rl/train.py:73-76):
 *
 *   AckermannRobotEnv.step(action)            src/rl/envs/ackermann_env.py:187-229
 *     BicycleController.apply_cmd_vel         src/core/controller.py:136-140 (98-134)
 *     mujoco.mj_step(model, data)             src/rl/envs/ackermann_env.py:200
 *     _get_observation / _calculate_reward    src/rl/envs/ackermann_env.py:231-312
 *   AckermannRobotEnv.reset()                 src/rl/envs/ackermann_env.py:143-185
 *     SimpleMapSpawner.load_random_environment src/rl/envs/simple_map_spawner.py:22-54
 *
 * Conventions
 *  - All array arguments are DEVICE pointers owned by the caller (torch tensors in the
 *    Python host layer); the library never allocates per call and never synchronises.
 *  - Work is enqueued on `stream` (a hipStream_t passed as void*; NULL = default stream).
 *  - Every entry point returns 0 on success or a negative ACKPHYS_E* code; the message is
 *    available from ackphys_last_error() (thread-local).
 *
 * Layouts (N = n_env given to ackphys_create; all float32 unless noted)
 *  state  [44][N]  word k of env e at state[k*N + e]:
 *           0-12 qpos (free joint xyz + quat wxyz, 6 hinges), 13-24 qvel, 25-36 qacc_warmstart,
 *           37-38 goal xy, 39-41 odometry reference xyz, 42 step_count (uint32 bits),
 *           43 episode counter (uint32 bits)
 *  action [N][2]   normalised (linear_x, angular_z) in [-1,1] (clipped like the reference)
 *  obs    [79][N]  72 lidar, x, y, yaw, dx, dy, dist, angle (ackermann_env.py:231-265)
 *  reward [N], term [N] (uint8), trunc [N] (uint8)
 *  terminal_obs [79][N] (nullable): observation before auto-reset, written for done envs
 *  info   [4][N]  (nullable): min_lidar, collision, goal_distance, bad_state
 *  episode [4][N] (nullable, in/out): Monitor-wrapper statistics (src/rl/train.py:70):
 *           running return, running length, sum of completed-episode returns, completed count
 */
#ifndef ACKPHYS_H
#define ACKPHYS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ackphys_ctx ackphys_t;

#define ACKPHYS_NSTATE 44
#define ACKPHYS_MAX_ENVS (1 << 22) /* per context (shard); more envs = more contexts */
#define ACKPHYS_NOBS 79

/* step flags */
#define ACKPHYS_CONTACTS 1u  /* 0 = MJCF <flag contact="disable"/> (BASELINE config 2) */
#define ACKPHYS_AUTORESET 2u /* SB3 VecEnv semantics: reset done envs inside the step */
/* obs/reward from the post-step pose: render_mode="human" runs mj_forward after mj_step
 * (ackermann_env.py:202-207). Default (flag clear): the pre-integration pose mj_step's sensors see. */
#define ACKPHYS_POSTSTEP_OBS 4u

/* error codes */
#define ACKPHYS_OK 0
#define ACKPHYS_EINVAL -1
#define ACKPHYS_EMODEL -2
#define ACKPHYS_EHIP -3

/* Create a context for n_env environments on HIP device `device`.
 * model_blob: the compiled model (include/ackphys_model.h), i.e. what the reference
 * builds with mujoco.MjModel.from_xml_path (simple_map_spawner.py:37). The library's kernels
 * are specialised on one model; a blob that does not match it is rejected (ACKPHYS_EMODEL). */
int ackphys_create(const void* model_blob, size_t nbytes, int n_env, int device, ackphys_t** out);
int ackphys_destroy(ackphys_t* ctx);

/* AckermannRobotEnv.__init__ keyword arguments (ackermann_env.py:51-60); defaults
 * 1000 / 0.5 / 0.15 / 1.0 / 1.0 are in effect until this is called. */
typedef struct ackphys_env_params {
  int32_t max_episode_steps;
  double goal_distance_threshold;
  double collision_threshold;
  double max_linear_velocity;
  double max_angular_velocity;
  /* Opt-in task variants, NOT the reference env (1 / 0 = ackermann_env.py exactly):
   * action_repeat: mj_steps per env step with the same ctrl (observation, reward and done at the
   *   last one's pre-integration pose; step_count and truncation count env steps; info bad_state
   *   reports the last mj_step's starting state, a NaN reset by an earlier one is not flagged);
   *   > 1 runs on the quad mapping (or the obstacle scene) with pre-integration observations;
   * nohit_clear: a rangefinder reading -1 (no hit) counts as no obstacle in the collision test
   *   (the reference's min over the readings makes every no-hit ray a collision,
   *   ackermann_env.py:279-284); info min_lidar is then the minimum over the hits, -1 if none;
 * goal_cells (obstacle scene only, 0 = the reference's goals 2-8 m away in a random direction,
 *   ackermann_env.py:167-172): > 0 draws each episode's goal at the centre of a box-free maze
 *   cell 4-connected to the spawn cell within goal_cells breadth-first steps of it (a maze task
 *   a policy can reach; the reference's goals mostly lie behind walls). */
  int32_t action_repeat;
  int32_t nohit_clear;
  int32_t goal_cells;
} ackphys_env_params;
int ackphys_set_env_params(ackphys_t* ctx, const ackphys_env_params* params);

/* Step-kernel mapping: ACKPHYS_VARIANT_QUAD runs each env's dynamics on 8 lanes of a wavefront
 * (two per wheel, each with half of the wheel's contact slots: Jacobian rows, Hessian/line-search
 * partials; the observation on 4 lanes, a quarter of the rays each; 8 envs per wave);
 * ACKPHYS_VARIANT_LANE runs each env on one lane; ACKPHYS_VARIANT_AUTO (default) picks QUAD when
 * contacts are enabled and LANE otherwise. Same results up to f32 summation order. */
#define ACKPHYS_VARIANT_LANE 0
#define ACKPHYS_VARIANT_QUAD 1
#define ACKPHYS_VARIANT_AUTO 2
#define ACKPHYS_VARIANT_LANE16 3 /* one lane per env, 16 envs per wave (4x the waves, shorter wave tails) */
int ackphys_set_variant(ackphys_t* ctx, int variant);

/* Global index of this context's env 0 (multi-GPU sharding: rank r passes r*n_env); it keys
 * the Philox streams for goals so a sharded run is identical to an unsharded one. */
int ackphys_set_env_offset(ackphys_t* ctx, int64_t env_offset);

/* One environment step for all N envs (replaces AckermannRobotEnv.step). */
int ackphys_step(ackphys_t* ctx, const float* action, float* state, float* obs, float* reward, uint8_t* term,
                 uint8_t* trunc, float* terminal_obs, float* info, float* episode, uint32_t flags, uint64_t seed,
                 void* stream);

/* k_steps consecutive steps of all N envs in ONE launch, for open-loop action sequences (the
 * random-ctrl benchmark configs, replayed action streams, scripted controllers): exactly
 * k_steps ackphys_step calls with actions[k] ([K][N][2]), same kernels' arithmetic, same
 * auto-reset and episode statistics. per_step_outputs = 0: obs/reward/term/trunc/terminal_obs/info
 * are the single-step shapes, overwritten by every step (left holding step K-1's); != 0: they are
 * [K][...] and step k writes slice k (a rollout buffer). With ACKPHYS_POSTSTEP_OBS the steps are
 * K single-step launches. Replaces a Python loop of env.step over a precomputed action array. */
int ackphys_rollout(ackphys_t* ctx, int k_steps, const float* actions, float* state, float* obs, float* reward,
                    uint8_t* term, uint8_t* trunc, float* terminal_obs, float* info, float* episode, uint32_t flags,
                    uint64_t seed, int per_step_outputs, void* stream);

/* Reset the envs whose mask byte is non-zero (mask NULL = all) (replaces
 * AckermannRobotEnv.reset): spawner pose, zero velocities, Philox(seed, env, episode) goal,
 * observation at the reset state. */
int ackphys_reset(ackphys_t* ctx, const uint8_t* mask, uint64_t seed, float* state, float* obs, void* stream);

/* Policy-in-the-loop PPO rollout of n_steps steps in ONE launch (BASELINE configs[3]): exactly the
 * per-step loop of stable-baselines3's collect_rollouts (src/rl/train.py:175-179) as libackppo runs
 * it -- ackppo_act (ackppo_act_boot) + ackphys_step with auto-reset + ackppo_bootstrap after the last
 * step + ackppo_value -- with the same results bit for bit. params: the flat policy vector of
 * include/ackppo.h; policy_seed / step0: the action noise's Philox key and the step counter of
 * rollout step 0 (step t uses step0 + t); deterministic != 0: actions = mean.
 * Sim buffers as for ackphys_step (in place, holding step n_steps-1's outputs afterwards; obs is
 * read as the observation of step 0 and left as the one after the last step); terminal_obs and
 * episode nullable. Rollout buffer (T = n_steps, N = n_env): obs_rows [T*N][79], actions [T*N][2]
 * (unclipped samples), log_prob / value / rollout_reward (with the TimeLimit bootstrap) /
 * episode_starts [T][N] (row 0 is the caller's: the previous rollout's last_dones), last_dones [N],
 * last_values [N]. Needs flags ACKPHYS_CONTACTS | ACKPHYS_AUTORESET (no ACKPHYS_POSTSTEP_OBS) and the
 * quad mapping (variant AUTO or QUAD). Replaces the reference's DummyVecEnv.step loop under SB3.
 * The first call on a context allocates a 72 KB device buffer it keeps (the policy's weights in the
 * kernel's operand order, rebuilt from params on the stream at every call; freed by
 * ackphys_destroy), so calls on one context must not run concurrently on different streams. */
int ackphys_ppo_rollout(ackphys_t* ctx, const float* params, int n_steps, uint32_t step0, uint64_t policy_seed,
                        int deterministic, float gamma, float* state, float* obs, float* reward, uint8_t* term,
                        uint8_t* trunc, float* terminal_obs, float* episode, float* obs_rows, float* actions,
                        float* log_prob, float* value, float* rollout_reward, float* episode_starts, float* last_dones,
                        float* last_values, uint32_t flags, uint64_t seed, void* stream);

/* Fill actions[K][N][2] with i.i.d. U[-1,1) from Philox4x32-10 keyed by seed, counter
 * (env_offset + env, step0 + k, 1, 0): the benchmark's synthetic "random ctrl" input. */
int ackphys_random_actions(ackphys_t* ctx, float* actions, int k_steps, uint64_t seed, uint32_t step0, void* stream);

/* FNV-1a 64 of the model blob the kernels were specialised on. */
uint64_t ackphys_model_fnv(void);
const char* ackphys_last_error(void);
const char* ackphys_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ACKPHYS_H */
