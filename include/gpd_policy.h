/*
 * gpd_policy.h — C ABI of the fused rollout policy (libgpd_policy.so, csrc/gpd_policy.hip).
 *
 * The caller side of the hot path: the reference trains stable-baselines3 PPO
 * ('MlpPolicy', examples/learn.py:52-94), whose rollout (SB3 OnPolicyAlgorithm.collect_rollouts)
 * runs, per env.step:
 *     actions, values, log_probs = policy(obs)          # actor + critic 64-64 tanh MLPs,
 *                                                        # Normal(mu, exp(log_std)) sample
 *     clipped = clip(actions, low, high)                # the Box action space [-1, 1]
 *     new_obs, rewards, dones, infos = env.step(clipped)
 *     rewards[i] += gamma * V(infos[i]["terminal_observation"])   if TimeLimit.truncated
 *     rollout_buffer.add(obs, actions, rewards, episode_starts, values, log_probs)
 * gpd_policy_rollout_step fuses everything except env.step (gpd_step) into ONE kernel: the
 * bootstrap and buffer write of the PREVIOUS step's reward, then the actor + critic forward, the
 * Normal sample, the clip and the buffer writes of THIS step, with the weight slices in VGPRs.
 *
 * Conventions as in gpd.h: device pointers, caller-owned buffers, asynchronous on `stream`,
 * GPD_OK (0) or a negative GPD_E* code with gpd_policy_last_error().
 */
#ifndef GPD_POLICY_H_
#define GPD_POLICY_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPD_POLICY_ABI_VERSION 2
#define GPD_POLICY_HIDDEN 64      /* SB3 MlpPolicy net_arch [64, 64], tanh */
#define GPD_POLICY_MAX_OBS 192    /* obs row width: both networks' layers staged in 160 KB of LDS */
#define GPD_POLICY_MAX_ACT 8

/* The actor (pi) and critic (vf) networks, torch nn.Linear layout (weight [out][in] row-major,
 * bias [out]), float32 device memory: n_obs -> 64 -> tanh -> 64 -> tanh -> n_act (pi) / 1 (vf). */
typedef struct gpd_mlp_policy {
  int n_obs, n_act;
  const float *pi_w1, *pi_b1, *pi_w2, *pi_b2, *pi_w3, *pi_b3;
  const float *vf_w1, *vf_b1, *vf_w2, *vf_b2, *vf_w3, *vf_b3;
  const float* log_std;      /* [n_act]: scale = exp(log_std) */
} gpd_mlp_policy;

/* One rollout step for n_rows envs.
 *   obs       [n_rows][n_obs]  the observation the policy acts on (nullable: bootstrap only)
 *   act_env   [n_rows][n_act]  clip(action, -1, 1): what gpd_step reads (nullable)
 *   buf_obs / buf_act / buf_logp / buf_val: this step's rollout-buffer rows (each nullable);
 *             buf_val alone (act_env, buf_act, buf_logp NULL) = the critic only (last value)
 *   deterministic: 1 = action = mean (EvalCallback), no sample
 *   rng       device uint64[2 + rng_groups] = {seed, 0, counter of row group 0, of group 1, ...}: the
 *             Philox4x32-10 key and a call counter per group of 16 rows (rows 16 g .. 16 g + 15); every
 *             call that samples advances the counters of the groups it covers by one, each in the
 *             block that samples the group (no atomic: one reader-writer per counter and call).
 *             Calls over the same n_rows keep the counters equal: the call count of the whole batch
 *   rng_groups  counters in rng (>= ceil(n_rows / 16) when sampling)
 * Previous step (all nullable together; reward == NULL skips the part):
 *   reward [n_rows] f32, terminated / truncated [n_rows] u8 (gpd_step's outputs),
 *   terminal_obs [n_rows][n_obs] (the env's terminal rows), gamma:
 *   buf_rew[i]  = reward[i] + gamma * V(terminal_obs[i])  if truncated[i] && !terminated[i]
 *               = reward[i]                                 otherwise
 *   buf_done[i] = terminated[i] || truncated[i]  (1.0f / 0.0f) */
int gpd_policy_rollout_step(const gpd_mlp_policy* policy, int n_rows, const float* obs, float* act_env,
                            float* buf_obs, float* buf_act, float* buf_logp, float* buf_val, int deterministic,
                            uint64_t* rng, int rng_groups, const float* reward, const uint8_t* terminated,
                            const uint8_t* truncated, const float* terminal_obs, float gamma, float* buf_rew,
                            float* buf_done, void* stream);

/* GAE(gamma, lambda) over a finished rollout (SB3 RolloutBuffer.compute_returns_and_advantage):
 * rew / val / done [n_steps][n_rows] f32, last_val [n_rows] -> adv, ret [n_steps][n_rows];
 * done[t] = the env finished at step t (its next value is not bootstrapped). */
int gpd_policy_gae(int n_steps, int n_rows, const float* rew, const float* val, const float* done,
                   const float* last_val, double gamma, double lam, float* adv, float* ret, void* stream);

int gpd_policy_abi_version(void);
const char* gpd_policy_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* GPD_POLICY_H_ */
