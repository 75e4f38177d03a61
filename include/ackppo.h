/* ackppo.h -- C-ABI of libackppo.so: the on-device PPO learner that consumes the batched
 * Ackermann env (BASELINE configs[3], "PPO rollout").
 *
 * It restates what the reference trains with (src/rl/train.py:99-128, 175-179; the stored
 * hyper-parameters in the rl_logs/ppo checkpoints' data file): stable-baselines3 2.7.0 PPO('MlpPolicy'), i.e.
 *   ActorCriticPolicy: separate 79-64-64 tanh MLPs for actor and critic, action_net 64->2,
 *   value_net 64->1, a state-independent log_std [2]; DiagGaussian actions, clipped to the
 *   action Box before env.step (stored unclipped); GAE(lambda) with the TimeLimit bootstrap
 *   (reward += gamma * V(terminal_obs) on truncation); per-minibatch advantage
 *   normalisation; loss = clipped surrogate + vf_coef * MSE(returns, V) - ent_coef * entropy;
 *   global grad-norm clipping (max_grad_norm); Adam (torch semantics, eps 1e-5).
 * SB3 is not installed here; the parity oracle is oracle/ppo_oracle.py (numpy float64),
 * itself cross-checked against torch autograd on the CPU (tests/test_ppo_oracle.py).
 *
 * Parameters live in ONE flat float32 vector: the SB3 state_dict tensors (policy.pth key
 * names, parameters() order), each starting at a multiple of 4 floats (ACKPPO_OFF_*); pad
 * words are zero. Gradients, Adam moments and gradient partials share the layout.
 *
 * Conventions (as include/ackphys.h): DEVICE pointers owned by the caller; work is enqueued
 * on `stream` (hipStream_t as void*, NULL = default); nothing allocates or synchronises;
 * 0 = success, negative = error (message via ackppo_last_error()).
 *
 * Sample index s = t * n_env + e for rollout step t and env e; every [T][N] buffer is laid
 * out that way, obs_rows is [T*N][79] (row per sample, gathered by minibatch index).
 */
#ifndef ACKPPO_H
#define ACKPPO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACKPPO_NOBS 79
#define ACKPPO_NACT 2
#define ACKPPO_HIDDEN 64
/* flat parameter layout (floats) -- policy.pth keys */
#define ACKPPO_OFF_LOG_STD 0      /* log_std                          [2]     */
#define ACKPPO_OFF_PI_W1 4        /* mlp_extractor.policy_net.0.weight [64][79] */
#define ACKPPO_OFF_PI_B1 5060     /* mlp_extractor.policy_net.0.bias   [64]    */
#define ACKPPO_OFF_PI_W2 5124     /* mlp_extractor.policy_net.2.weight [64][64] */
#define ACKPPO_OFF_PI_B2 9220     /* mlp_extractor.policy_net.2.bias   [64]    */
#define ACKPPO_OFF_VF_W1 9284     /* mlp_extractor.value_net.0.weight  [64][79] */
#define ACKPPO_OFF_VF_B1 14340    /* mlp_extractor.value_net.0.bias    [64]    */
#define ACKPPO_OFF_VF_W2 14404    /* mlp_extractor.value_net.2.weight  [64][64] */
#define ACKPPO_OFF_VF_B2 18500    /* mlp_extractor.value_net.2.bias    [64]    */
#define ACKPPO_OFF_ACT_W 18564    /* action_net.weight                 [2][64]  */
#define ACKPPO_OFF_ACT_B 18692    /* action_net.bias                   [2]     */
#define ACKPPO_OFF_VAL_W 18696    /* value_net.weight                  [1][64]  */
#define ACKPPO_OFF_VAL_B 18760    /* value_net.bias                    [1]     */
#define ACKPPO_NPARAM 18764
#define ACKPPO_NLOSS 8            /* loss partial words per workgroup (see ackppo_grad) */
#define ACKPPO_WIMAGE 9728        /* floats per net of ackppo_train_desc::weight_image */

#define ACKPPO_OK 0
#define ACKPPO_EINVAL -1
#define ACKPPO_EHIP -3

/* Rollout policy step (SB3 collect_rollouts: policy(obs) -> actions, values, log_probs):
 * obs_soa [79][n] (ackphys_step's obs buffer). Gaussian noise: Philox4x32-10, key = seed,
 * counter = (env_offset + e, step, 2, 0), Box-Muller on the first two words.
 * deterministic != 0: action = mean (predict(deterministic=True)).
 * Outputs: action [n][2] unclipped sample, env_action [n][2] clipped to [-1,1] (what env.step
 * receives), log_prob [n], value [n], obs_rows [n][79] copy of the observation (rollout
 * buffer rows). Every output except env_action may be NULL. */
int ackppo_act(const float* params, const float* obs_soa, int n_env, int64_t env_offset, uint64_t seed,
               uint32_t step, int deterministic, float* obs_rows, float* action, float* env_action,
               float* log_prob, float* value, void* stream);

/* ackppo_act for rollout step t + 1 fused with the TimeLimit bootstrap of step t (saves the
 * ackppo_bootstrap launch on every step but the last): the same outputs as ackppo_act, plus
 * exactly ackppo_bootstrap's reward_out / done_out for the previous step's terminal_obs_soa,
 * reward, term, trunc (read before this launch overwrites nothing they hold). */
int ackppo_act_boot(const float* params, const float* obs_soa, int n_env, int64_t env_offset, uint64_t seed,
                    uint32_t step, int deterministic, float* obs_rows, float* action, float* env_action,
                    float* log_prob, float* value, const float* terminal_obs_soa, const float* reward,
                    const uint8_t* term, const uint8_t* trunc, float gamma, float* reward_out, float* done_out,
                    void* stream);

/* value [n] = critic(obs_soa) (SB3 policy.predict_values; last_values of a rollout). */
int ackppo_value(const float* params, const float* obs_soa, int n_env, float* value, void* stream);

/* After one ackphys_step with auto-reset (SB3 collect_rollouts truncation bootstrap):
 * reward_out[e] = reward[e] + gamma * V(terminal_obs[:, e]) if trunc[e] && !term[e], else reward[e];
 * done_out[e] = term[e] || trunc[e] (float 0/1: the next step's episode_start). */
int ackppo_bootstrap(const float* params, const float* terminal_obs_soa, const float* reward, const uint8_t* term,
                     const uint8_t* trunc, int n_env, float gamma, float* reward_out, float* done_out, void* stream);

/* RolloutBuffer.compute_returns_and_advantage: GAE over T steps, all [T][n].
 * episode_starts[t] = done flag of step t-1; last_values/last_dones are the state after step T-1. */
int ackppo_gae(const float* rewards, const float* values, const float* episode_starts, const float* last_values,
               const float* last_dones, int T, int n_env, float gamma, float gae_lambda, float* advantages,
               float* returns, void* stream);

/* Per-minibatch advantage statistics for one epoch: minibatch m covers idx[m*batch ..
 * min((m+1)*batch, n_idx)). stats[m] = (mean, 1/(std+1e-8)) with the unbiased std; (0, 1)
 * when normalize == 0 or the minibatch has one sample (SB3: len(advantages) > 1). */
int ackppo_adv_stats(const float* advantages, const int32_t* idx, int n_idx, int batch, int normalize,
                     float* stats, void* stream);

/* Data-parallel advantage statistics (a world minibatch m = the union of every rank's minibatch m,
 * so all ranks normalise with the statistics of the whole world minibatch, as one SB3 learner
 * with world x batch samples would). moments [3][nmb] float64, nmb = ceil(n_idx / batch):
 *   phase 0: moments[0][m] = count, moments[1][m] = sum of this rank's advantages, moments[2][m] = 0;
 *   (caller all-reduces rows 0..1 with SUM)
 *   phase 1: moments[2][m] = sum of (a - mean_m)^2 about the global mean moments[1][m] / moments[0][m];
 *   (caller all-reduces row 2 with SUM)
 * then ackppo_adv_finalize: stats[m] = (mean, 1/(std+1e-8)), unbiased std over the world
 * minibatch; (0, 1) when normalize == 0 or the world minibatch has one sample. At world 1 the
 * three calls give ackppo_adv_stats' stats bit for bit. */
int ackppo_adv_moments(const float* advantages, const int32_t* idx, int n_idx, int batch, int phase,
                       double* moments, void* stream);
int ackppo_adv_finalize(const double* moments, int nmb, int normalize, float* stats, void* stream);

/* out [n] = a keyed pseudo-random permutation of 0..n-1 (the minibatch shuffle of one epoch,
 * SB3 rollout_buffer.get: np.random.permutation(buffer_size * n_envs)): a 4-round Feistel
 * bijection with cycle walking, keyed by (seed, epoch); one launch, no sort. */
int ackppo_permutation(int n, uint64_t seed, uint32_t epoch, int32_t* out, void* stream);

/* Gradient of the PPO loss of one minibatch (samples idx[0..batch)), split over
 * nblk = ackppo_grad_blocks(batch) workgroups (one per CU at most), each writing its row of
 * grad_partial [nblk][NPARAM] (pad words are never written: zero them once) and of
 * loss_partial [nblk][8] = (sum pg_loss, sum (R-V)^2, n clipped, sum approx_kl, n samples, 0, 0, 0).
 * stats: (mean, inv_std) of this minibatch (ackppo_adv_stats). The entropy term is
 * sample-independent and is added by ackppo_reduce. */
int ackppo_grad(const float* params, const float* obs_rows, const float* actions, const float* old_log_prob,
                const float* advantages, const float* returns, const int32_t* idx, int batch, const float* stats,
                float clip_range, float ent_coef, float vf_coef, float* grad_partial, float* loss_partial,
                void* stream);

/* Number of partial rows ackppo_grad writes for a minibatch of `batch` samples. */
int ackppo_grad_blocks(int batch);

/* grad [NPARAM] = sum of nblk partial rows (grad is overwritten); d(-ent_coef * entropy)/d log_std = -ent_coef added;
 * loss [8] = column sums of loss_partial. grad_partial is CONSUMED: the library may overwrite its rows with
 * intermediate sums (no library-owned scratch; the next ackppo_grad rewrites every row). */
int ackppo_reduce(float* grad_partial, const float* loss_partial, int nblk, float ent_coef, float* grad,
                  float* loss, void* stream);

/* clip_grad_norm_(max_grad_norm) + torch.optim.Adam step on grad * grad_scale (grad_scale =
 * 1/world after an all-reduce SUM). step_size = lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t)
 * (host-computed in float64 as torch does). grad_norm_out [1] (nullable): pre-clip norm. */
int ackppo_adam(float* params, const float* grad, float* exp_avg, float* exp_avg_sq, float grad_scale,
                float max_grad_norm, float beta1, float beta2, float eps, float step_size, float bc2_sqrt,
                float* grad_norm_out, void* stream);

/* One epoch of minibatch updates on a single rank (world 1: no all-reduce between the gradient
 * and the Adam step). For m in [0, ceil(n_idx / batch)): ackppo_grad on idx[m * batch ...] with
 * stats[2m .. 2m+1], the reduction of the partial rows (the loss columns ADDED to loss_acc [8])
 * and the Adam step with grad_scale 1 and t = adam_step0 + m + 1 (step_size = learning_rate /
 * (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t), float64 as torch computes them): ackppo_reduce +
 * ackppo_adam's arithmetic, with the gradient sums over 8 row groups and the global norm in the
 * blocked order of 128-parameter blocks (the reduction hands each block's sum of squares to the
 * Adam launch; SB3 PPO.train, on_policy_algorithm / ppo.py:196-279 of SB3 2.7.0). The loop runs on
 * the host in C so the launches queue back to back. ackppo_train (below) runs whole training
 * phases, single-rank or data-parallel, with the same kernels. */
int ackppo_epoch(float* params, const float* obs_rows, const float* actions, const float* old_log_prob,
                 const float* advantages, const float* returns, const int32_t* idx, int n_idx, int batch,
                 const float* stats, float clip_range, float ent_coef, float vf_coef, float max_grad_norm,
                 double learning_rate, double beta1, double beta2, float eps, int64_t adam_step0,
                 float* grad_partial, float* loss_partial, float* grad, float* loss_acc, float* exp_avg,
                 float* exp_avg_sq, float* grad_norm_out, void* stream);

/* ---- the whole PPO.train() in one host call, single rank or data-parallel ----
 *
 * Collective hook: SUM all-reduce, in place, of `count` elements of `dtype` (ACKPPO_F32 / ACKPPO_F64)
 * at device pointer `buf`, ordered on `stream` after the work already enqueued there; 0 = success.
 * ackppo_rccl_allreduce (below) is one, over a native RCCL communicator; a caller may pass its own
 * (e.g. a host-staged gloo rehearsal). NULL with world == 1: no collective. */
#define ACKPPO_F32 0
#define ACKPPO_F64 1
typedef int (*ackppo_allreduce_fn)(void* buf, int64_t count, int dtype, void* user, void* stream);

typedef struct {
  /* rollout buffer (this rank's shard, [T*N] samples, include order as above) */
  const float* obs_rows;
  const float* actions;
  const float* old_log_prob;
  const float* advantages;
  const float* returns;
  int n_idx;                /* T * N */
  int batch;                /* per-rank minibatch (a world minibatch is world x batch samples) */
  int n_epochs;
  uint64_t perm_key;        /* ackppo_permutation key (seed, rank) */
  uint32_t perm_epoch0;     /* epoch counter of the first epoch (advanced by n_epochs) */
  int normalize_advantage;
  float clip_range, ent_coef, vf_coef, max_grad_norm;
  double learning_rate, beta1, beta2;
  float eps;
  int64_t adam_step0;       /* Adam steps taken before this call (advanced by n_epochs x nmb) */
  /* state and scratch (device) */
  float* params;
  float* exp_avg;
  float* exp_avg_sq;
  int32_t* perm;            /* [n_idx] */
  float* stats;             /* [nmb][2] */
  double* moments;          /* with a hook: [3][nmb] float64, or [3][n_epochs][nmb] with perm_epochs / stats_epochs
                             * (its size in moments_count, the last field) */
  float* grad_partial;      /* [ackppo_grad_blocks(batch)][NPARAM], pad words zero */
  float* loss_partial;      /* [ackppo_grad_blocks(batch)][8] */
  float* grad;              /* [NPARAM] */
  float* loss_acc;          /* [8]: zeroed, then the loss columns of every minibatch added */
  float* grad_norm_out;     /* [1] nullable: pre-clip norm of the last minibatch */
  /* data parallelism */
  int world;
  ackppo_allreduce_fn allreduce;
  void* allreduce_user;
  /* opt-in entropy floor (not an SB3 parameter; -INFINITY = SB3, bit for bit): log_std is held at or
   * above this value after every Adam step, so the DiagGaussian's spread cannot collapse below
   * exp(log_std_min) */
  float log_std_min;
  /* optional scratch, 2 * ACKPPO_WIMAGE floats (NULL: off): each net's gradient-kernel weight block
   * in the kernel's LDS layout, written by every Adam step beside the parameters (and built from
   * them when the call starts), so the gradient launches copy it into LDS with plain DMA instead of
   * transposing the parameters. Same results bit for bit */
  float* weight_image;
  /* optional scratch (NULL: one shuffle and one statistics launch per epoch into perm / stats):
   * [n_epochs][n_idx] int32 and [n_epochs][nmb][2] floats -- every epoch's shuffle and minibatch
   * advantage statistics formed at the start of the call, the same values as the per-epoch launches
   * (the advantages do not change during the call). Single rank: ONE launch. With a hook: one
   * launch of every epoch's shuffle and (count, sum) into moments [0..1][n_epochs][nmb], ONE
   * all-reduce of 2 x n_epochs x nmb f64, one launch of the squared deviations, ONE all-reduce of
   * n_epochs x nmb f64, one finalize launch -- 2 collectives per call instead of 2 per epoch */
  int32_t* perm_epochs;
  float* stats_epochs;
  /* float64 elements available at `moments` (required with a hook): at least 3 * nmb, or
   * 3 * n_epochs * nmb with perm_epochs / stats_epochs; a smaller buffer is refused (EINVAL) */
  int64_t moments_count;
} ackppo_train_desc;

/* SB3 PPO.train (ppo.py:196-279 of SB3 2.7.0) on the device: for each epoch, the minibatch
 * shuffle (ackppo_permutation), the advantage statistics of every minibatch (world 1:
 * ackppo_adv_stats; world > 1: ackppo_adv_moments phase 0 -> all-reduce of 2 x nmb f64 -> phase 1 ->
 * all-reduce of nmb f64 -> ackppo_adv_finalize; with perm_epochs / stats_epochs all of it for every
 * epoch at the start of the call), then per minibatch ackppo_grad -> the reduction ->
 * the Adam step (world 1 without a hook; ackppo_epoch's launches), or the reduction -> all-reduce of
 * NPARAM f32 -> the norm blocks' sums -> the Adam step (grad_scale 1/world; the same arithmetic).
 * Every launch and collective is
 * enqueued back to back from this one call: no per-minibatch host round trip (the host never waits
 * on the device, unless the hook itself does). World 1 without a hook: the same launches as
 * ackppo_epoch per epoch, bit for bit. A hook at world 1 runs the data-parallel sequence over one
 * rank (the same results: the moments give ackppo_adv_stats' statistics bit for bit). */
int ackppo_train(const ackppo_train_desc* d, void* stream);

/* RCCL for the trainer's collectives (one process per GPU). The library is the RCCL already loaded
 * in the process (torch's librccl.so.1; dlopen RTLD_NOLOAD -- never a second copy): these calls fail
 * if none is loaded. ackppo_rccl_allreduce takes any communicator of that library: the one torch's
 * ProcessGroupNCCL built (its _comm_ptr(); the default, shard.TrainerCollective kind "torch"), or one
 * of this library's own (ackppo_rccl_unique_id on rank 0, the id distributed by the caller, then
 * ackppo_rccl_init on every rank's current device; kind "rccl", opt-in).
 * ackppo_rccl_library writes the path of the RCCL these calls use into `path` (0 = found). */
int ackppo_rccl_unique_id(void* id128);
int ackppo_rccl_init(const void* id128, int nranks, int rank, void** comm);
int ackppo_rccl_allreduce(void* buf, int64_t count, int dtype, void* comm, void* stream); /* an ackppo_allreduce_fn */
int ackppo_rccl_destroy(void* comm);
int ackppo_rccl_library(char* path, int size);

const char* ackppo_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
