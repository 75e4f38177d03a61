/* ackphys_oracle.h -- host twin of include/ackphys.h's step/reset (SURVEY.md §8b "ackphys_step_cpu").
 *
 * TEST INFRASTRUCTURE ONLY. Exported by oracle/build/libackphys_oracle.so (the f64 CPU restatement
 * of mj_step + the env glue, oracle/ackphys_oracle.c), never by libackphys.so: the product path
 * has no CPU fallback. Same argument meaning and buffer layouts as ackphys_step/ackphys_reset
 * (SoA f32 [44][N] state, [79][N] obs, [4][N] info/episode) on HOST pointers, so a parity check
 * or a CPU baseline can drive both sides with identical buffers. Arithmetic is f64 internally;
 * the f32 state is widened on entry and rounded on exit (u32 step/episode words bit-cast).
 */
#ifndef ACKPHYS_ORACLE_H
#define ACKPHYS_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_ctx or_ctx;

int or_create(const void* model_blob, size_t nbytes, or_ctx** out);
void or_destroy(or_ctx* ctx);
void or_set_env_offset(or_ctx* ctx, int env_offset);
void or_set_env_params(or_ctx* ctx, int max_episode_steps, double goal_distance_threshold,
                      double collision_threshold, double max_linear_velocity, double max_angular_velocity);
/* opt-in task variant (not the reference): action_repeat mj_steps per env step; nohit_clear != 0
 * ignores -1 (no-hit) rangefinder readings in the collision test (include/ackphys.h) */
void or_set_env_variant(or_ctx* ctx, int action_repeat, int nohit_clear);
/* opt-in maze goals (not the reference): goal_cells > 0 draws reset goals at the centres of the free
 * box-lattice cells within goal_cells breadth-first cells of the spawn (include/ackphys.h);
 * -1 if the world has no such lattice */
int or_set_goal_cells(or_ctx* ctx, int goal_cells);
/* obstacle scene: the wheel-on-box-edge kink snap (on by default; off = the plain search) */
void or_set_kink_snap(int on);

/* ackphys_step on host buffers (flags: ACKPHYS_CONTACTS | ACKPHYS_AUTORESET | ACKPHYS_POSTSTEP_OBS).
 * terminal_obs, info, episode may be NULL. nthreads <= 0: OpenMP default. */
int ackphys_step_cpu(or_ctx* ctx, int n_env, const float* action, float* state, float* obs, float* reward,
                     uint8_t* terminated, uint8_t* truncated, float* terminal_obs, float* info, float* episode,
                     uint32_t flags, uint64_t seed, int nthreads);
/* ackphys_reset on host buffers (mask may be NULL = all envs). */
int ackphys_reset_cpu(or_ctx* ctx, int n_env, const uint8_t* mask, uint64_t seed, float* state, float* obs);

#ifdef __cplusplus
}
#endif
#endif
