"""On-device PPO for the batched Ackermann env (BASELINE configs[3]).

The reference trains with stable-baselines3 `PPO('MlpPolicy', DummyVecEnv([Monitor(env)]), ...)`
(src/rl/train.py:99-128, learn at :175-179). This class keeps that constructor / `learn` /
`predict` / `save` surface and its semantics, but every per-sample computation runs in
libackppo.so (include/ackppo.h) on the GPU, next to the env step:

  rollout      : one ackphys_ppo_rollout launch (policy + env steps + TimeLimit bootstrap fused), or
                 per step ackppo_act (policy -> action, log_prob, value, obs row) -> ackphys_step
                 (auto-reset) -> ackppo_bootstrap; then ackppo_value (last values) -> ackppo_gae
  train()      : ONE ackppo_train call (include/ackppo.h), which enqueues for each epoch the device
                 permutation (the SB3 minibatch shuffle) and the advantage statistics, then per
                 minibatch ackppo_grad -> ackppo_reduce -> [all-reduce of 75 KB] -> ackppo_adam

Nothing leaves the device inside `learn` except the logging scalars at the end of an update.
Torch tensors are the buffer container only.

Data-parallel (one process per GPU, torchrun): every rank steps its own env shard (env_offset
= rank * n_envs), parameters are broadcast from rank 0 once, and each minibatch gradient is
summed over ranks with one all-reduce; the Adam kernel scales by 1/world. A minibatch is then
world x batch_size samples, split evenly over ranks, and its advantages are normalised with the
statistics of all world x batch_size samples (ackppo_adv_moments: two small all-reduces of the
per-minibatch count / sum / squared deviations per epoch), as one SB3 learner would. The
collectives are enqueued from C by ackppo_train through a hook (shard.TrainerCollective): a native
RCCL communicator (ackppo_rccl_allreduce) on GPU nodes, a host-staged torch.distributed callback in
gloo rehearsals -- per iteration n_epochs x nmb + 2 all-reduces (the advantage moments of every
epoch formed at the start of train()), none of them a host round trip on the RCCL path.
"""
from __future__ import annotations

import collections
import ctypes as C
import math
import time

import torch

from .. import _lib, shard

NOBS, NACT, HID = 79, 2, 64
NPARAM, NLOSS = 18764, 8
# flat parameter layout = include/ackppo.h ACKPPO_OFF_* (policy.pth key names)
LAYOUT = collections.OrderedDict([
    ("log_std", (0, (2,))),
    ("mlp_extractor.policy_net.0.weight", (4, (HID, NOBS))),
    ("mlp_extractor.policy_net.0.bias", (5060, (HID,))),
    ("mlp_extractor.policy_net.2.weight", (5124, (HID, HID))),
    ("mlp_extractor.policy_net.2.bias", (9220, (HID,))),
    ("mlp_extractor.value_net.0.weight", (9284, (HID, NOBS))),
    ("mlp_extractor.value_net.0.bias", (14340, (HID,))),
    ("mlp_extractor.value_net.2.weight", (14404, (HID, HID))),
    ("mlp_extractor.value_net.2.bias", (18500, (HID,))),
    ("action_net.weight", (18564, (NACT, HID))),
    ("action_net.bias", (18692, (NACT,))),
    ("value_net.weight", (18696, (1, HID))),
    ("value_net.bias", (18760, (1,))),
])


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def state_dict_from_flat(flat: torch.Tensor) -> "collections.OrderedDict[str, torch.Tensor]":
    """SB3 ActorCriticPolicy state_dict (policy.pth key names) from the flat vector."""
    f = flat.detach().float().cpu()
    return collections.OrderedDict((k, f[o:o + math.prod(s)].reshape(s).clone()) for k, (o, s) in LAYOUT.items())


def flat_from_state_dict(sd) -> torch.Tensor:
    flat = torch.zeros(NPARAM, dtype=torch.float32)
    for k, (o, s) in LAYOUT.items():
        v = torch.as_tensor(sd[k], dtype=torch.float32).reshape(-1)
        if v.numel() != math.prod(s):
            raise ValueError(f"{k}: expected shape {s}, got {tuple(torch.as_tensor(sd[k]).shape)}")
        flat[o:o + v.numel()] = v
    return flat


def init_params(seed: int | None = None, ortho_init: bool = True, log_std_init: float = 0.0) -> torch.Tensor:
    """ActorCriticPolicy initialisation: orthogonal weights (gain sqrt(2) in the MLP extractor,
    0.01 for action_net, 1 for value_net), zero biases, log_std = log_std_init."""
    g = torch.Generator().manual_seed(0 if seed is None else int(seed))
    sd = {}
    for k, (_, s) in LAYOUT.items():
        if k.endswith("weight"):
            w = torch.empty(s)
            gain = 0.01 if k.startswith("action_net") else 1.0 if k.startswith("value_net") else math.sqrt(2)
            if ortho_init:
                torch.nn.init.orthogonal_(w, gain=gain, generator=g)
            else:
                bound = 1.0 / math.sqrt(s[1])
                w.uniform_(-bound, bound, generator=g)
            sd[k] = w
        elif k == "log_std":
            sd[k] = torch.full(s, float(log_std_init))
        else:
            sd[k] = torch.zeros(s)
    return flat_from_state_dict(sd)


class PPO:
    """stable-baselines3 PPO('MlpPolicy') semantics on libackppo.so (see module docstring).

    `env` is an AckermannVecEnv (rl/envs/vec_env.py); its sim is stepped directly."""

    def __init__(self, policy, env, learning_rate: float = 3e-4, n_steps: int = 2048, batch_size: int = 64,
                 n_epochs: int = 10, gamma: float = 0.99, gae_lambda: float = 0.95, clip_range: float = 0.2,
                 clip_range_vf=None, normalize_advantage: bool = True, ent_coef: float = 0.0, vf_coef: float = 0.5,
                 max_grad_norm: float = 0.5, target_kl=None, seed: int | None = None, verbose: int = 0,
                 policy_kwargs: dict | None = None, device=None, world: int | None = None, rank: int | None = None,
                 fused_rollout: bool | None = None, collective: str | None = None, log_std_min: float | None = None):
        if policy != "MlpPolicy":
            raise ValueError("only 'MlpPolicy' (the reference's policy, train.py:126) is provided")
        if clip_range_vf is not None or target_kl is not None:
            raise NotImplementedError("clip_range_vf / target_kl are not used by the reference (both None)")
        if policy_kwargs:
            raise NotImplementedError("policy_kwargs: the reference uses the default 64-64 tanh MlpPolicy")
        if callable(learning_rate) or callable(clip_range):
            raise NotImplementedError("schedules: the reference uses constant learning_rate / clip_range")
        self.env = env
        self.sim = env.sim
        # opt-in entropy floor (NOT an SB3 argument; None = SB3): log_std held >= log_std_min after every
        # Adam step, so the policy's spread cannot collapse (include/ackppo.h ackppo_train_desc)
        self.log_std_min = log_std_min
        # the policy-in-the-loop rollout in one launch (ackphys_ppo_rollout) where the kernels provide
        # it -- contacts on, the quad mapping, pre-integration observations -- else one act launch and
        # one step launch per step; both give the same rollout bit for bit
        can_fuse = self.sim.contacts and self.sim.variant in ("auto", "quad") and not self.sim.poststep_obs
        if fused_rollout and not can_fuse:
            raise ValueError("fused_rollout needs contacts, the quad mapping and pre-integration observations")
        self.fused_rollout = can_fuse if fused_rollout is None else bool(fused_rollout)
        self.device = self.sim.device
        self.n_envs = self.sim.n
        self.learning_rate, self.n_steps, self.batch_size, self.n_epochs = learning_rate, n_steps, batch_size, n_epochs
        self.gamma, self.gae_lambda, self.clip_range = gamma, gae_lambda, clip_range
        self.normalize_advantage, self.ent_coef, self.vf_coef = normalize_advantage, ent_coef, vf_coef
        self.max_grad_norm, self.verbose = max_grad_norm, verbose
        self.seed = 0 if seed is None else int(seed)
        r, w, _ = shard.dist_env()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.env_offset = self.sim.env_offset
        self.L = _lib.ppo_lib()
        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        self.params = init_params(self.seed).to(dev)
        shard.broadcast_(self.params, self.world)
        self.exp_avg = torch.zeros(NPARAM, **f32)
        self.exp_avg_sq = torch.zeros(NPARAM, **f32)
        self.adam_step = 0
        T, N = n_steps, self.n_envs
        self.buf_obs = torch.zeros(T * N, NOBS, **f32)
        self.buf_act = torch.zeros(T * N, NACT, **f32)
        self.buf_logp = torch.zeros(T, N, **f32)
        self.buf_val = torch.zeros(T, N, **f32)
        self.buf_rew = torch.zeros(T, N, **f32)
        self.buf_start = torch.zeros(T, N, **f32)
        self.buf_adv = torch.zeros(T, N, **f32)
        self.buf_ret = torch.zeros(T, N, **f32)
        self.env_action = torch.zeros(N, NACT, **f32)
        self.last_dones = torch.ones(N, **f32)  # SB3 _last_episode_starts = ones at the first rollout
        self.last_values = torch.zeros(N, **f32)
        nblk = self.L.ackppo_grad_blocks(batch_size)
        self.gpart = torch.zeros(nblk, NPARAM, **f32)  # pad words are never written: zero once
        self.lpart = torch.zeros(nblk, NLOSS, **f32)
        self.grad = torch.zeros(NPARAM, **f32)
        # both nets' gradient-kernel weight blocks in the kernel's LDS layout (ackppo_train_desc weight_image)
        self.weight_image = torch.zeros(2 * _lib.ACKPPO_WIMAGE, **f32)
        self.loss = torch.zeros(NLOSS, **f32)
        self.loss_acc = torch.zeros(NLOSS, **f32)
        self.gnorm = torch.zeros(1, **f32)
        nmb = (T * N + batch_size - 1) // batch_size
        self.mb_stats = torch.zeros(nmb, 2, **f32)
        # DP advantage statistics: [3][n_epochs][nmb] (all epochs at the start of train(); the per-epoch
        # path uses its first [3][nmb] words)
        self.mb_moments = torch.zeros(3, n_epochs * nmb, dtype=torch.float64, device=dev)
        # per-epoch minibatch shuffle: ackppo_permutation keyed by (seed, rank) and the epoch count
        self.perm_key = (self.seed * 7919 + self.rank) & 0xFFFFFFFFFFFFFFFF
        self.perm_epoch = 0
        self.perm = torch.empty(self.n_steps * self.n_envs, dtype=torch.int32, device=dev)
        # every epoch's shuffle and statistics of one train() call, formed at its start (ackppo_train_desc
        # perm_epochs / stats_epochs: one launch single-rank; 2 all-reduces per call data-parallel)
        self.perm_epochs = torch.empty(self.n_epochs, self.n_steps * self.n_envs, dtype=torch.int32, device=dev)
        self.stats_epochs = torch.zeros(self.n_epochs, nmb, 2, **f32)
        # the all-reduce hook of the data-parallel update (shard.TrainerCollective): on GPU nodes RCCL on
        # libackppo's own communicator ("rccl", the default) or on torch's ("torch", opt-in); host-staged in
        # gloo rehearsals; a kind at world 1 runs the data-parallel path over one rank (timing it on one GPU)
        self.collective = None
        self._desc = self._train_desc()
        if self.world > 1 or collective is not None:
            self.set_collective(collective)
        self.num_timesteps = 0
        self.episodes_total = 0
        self._rollout_step = 0
        self._last_obs_ready = False
        self.logger = {}
        self.ep_info_buffer = collections.deque(maxlen=100)

    # ------------------------------------------------------------------ policy API
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def predict(self, observation, state=None, episode_start=None, deterministic: bool = False):
        """BasePolicy.predict: observation [n, 79] (or [79]) -> (actions clipped to the Box, None)."""
        obs = torch.as_tensor(observation, dtype=torch.float32, device=self.device)
        single = obs.dim() == 1
        obs = obs.reshape(-1, NOBS)
        n = obs.shape[0]
        soa = obs.t().contiguous()
        out = torch.empty(n, NACT, dtype=torch.float32, device=self.device)
        _lib.ppo_check(self.L.ackppo_act(_ptr(self.params), _ptr(soa), n, 0, self.seed, self._rollout_step,
                                         1 if deterministic else 0, None, None, _ptr(out), None, None,
                                         self._stream()), "ackppo_act")
        self._rollout_step += 0 if deterministic else 1
        return (out[0] if single else out), None

    def policy_state_dict(self):
        return state_dict_from_flat(self.params)

    def load_policy_state_dict(self, sd):
        self.params.copy_(flat_from_state_dict(sd).to(self.device))

    def save(self, path: str):
        """policy.pth-style file (SB3 key names) + optimizer moments; loads with weights_only=True."""
        torch.save({"policy": self.policy_state_dict(), "exp_avg": self.exp_avg.cpu(),
                    "exp_avg_sq": self.exp_avg_sq.cpu(), "adam_step": self.adam_step,
                    "num_timesteps": self.num_timesteps}, path)

    def load(self, path: str):
        d = torch.load(path, weights_only=True, map_location="cpu")
        self.load_policy_state_dict(d["policy"])
        self.exp_avg.copy_(d["exp_avg"])
        self.exp_avg_sq.copy_(d["exp_avg_sq"])
        self.adam_step = int(d["adam_step"])
        self.num_timesteps = int(d["num_timesteps"])

    # ------------------------------------------------------------------ training
    def collect_rollouts(self):
        L, s, N, sim = self.L, self._stream(), self.n_envs, self.sim
        if not self._last_obs_ready:
            self.env.reset()
            self._last_obs_ready = True
        if self.fused_rollout:
            self._collect_fused()
        else:
            self._collect_per_step()
        _lib.ppo_check(L.ackppo_gae(_ptr(self.buf_rew), _ptr(self.buf_val), _ptr(self.buf_start),
                                    _ptr(self.last_values), _ptr(self.last_dones), self.n_steps, N, self.gamma,
                                    self.gae_lambda, _ptr(self.buf_adv), _ptr(self.buf_ret), s), "ackppo_gae")

    def _collect_fused(self):
        """The whole rollout as one ackphys_ppo_rollout launch (include/ackphys.h)."""
        sim, c = self.sim, self.sim._c
        self.buf_start[0].copy_(self.last_dones)
        rc = _lib.lib().ackphys_ppo_rollout(
            sim._ctx, _ptr(self.params), self.n_steps, self._rollout_step, self.seed, 0, self.gamma, c["state"],
            c["obs_soa"], c["reward"], c["term"], c["trunc"], c["terminal_obs_soa"], c["episode"], _ptr(self.buf_obs),
            _ptr(self.buf_act), _ptr(self.buf_logp), _ptr(self.buf_val), _ptr(self.buf_rew), _ptr(self.buf_start),
            _ptr(self.last_dones), _ptr(self.last_values), sim.flags | 2, sim.seed, self._stream())
        if rc:
            _lib.check(rc, "ackphys_ppo_rollout")
        self._rollout_step += self.n_steps
        self.num_timesteps += self.n_steps * self.n_envs * self.world

    def _collect_per_step(self):
        """One ackppo_act(_boot) launch and one ackphys_step launch per rollout step."""
        L, s, N, sim = self.L, self._stream(), self.n_envs, self.sim
        # episode starts: step t's done flags are step t + 1's starts, so the bootstrap writes them
        # straight into buf_start[t + 1] (the last step's into last_dones): one copy per rollout
        self.buf_start[0].copy_(self.last_dones)
        # The TimeLimit bootstrap of step t rides in step t + 1's act launch (ackppo_act_boot); the
        # last step's is its own launch.
        for t in range(self.n_steps):
            out = (_ptr(self.params), _ptr(sim.obs_soa), N, self.env_offset, self.seed, self._rollout_step, 0,
                   _ptr(self.buf_obs[t * N]), _ptr(self.buf_act[t * N]), _ptr(self.env_action),
                   _ptr(self.buf_logp[t]), _ptr(self.buf_val[t]))
            if t == 0:
                _lib.ppo_check(L.ackppo_act(*out, s), "ackppo_act")
            else:
                _lib.ppo_check(L.ackppo_act_boot(*out, _ptr(sim.terminal_obs_soa), _ptr(sim.reward), _ptr(sim.term),
                                                 _ptr(sim.trunc), self.gamma, _ptr(self.buf_rew[t - 1]),
                                                 _ptr(self.buf_start[t]), s), "ackppo_act_boot")
            sim.step(self.env_action, autoreset=True, want_info=False, want_terminal=True, track_episodes=True)
            self._rollout_step += 1
        _lib.ppo_check(L.ackppo_bootstrap(_ptr(self.params), _ptr(sim.terminal_obs_soa), _ptr(sim.reward),
                                          _ptr(sim.term), _ptr(sim.trunc), N, self.gamma,
                                          _ptr(self.buf_rew[self.n_steps - 1]), _ptr(self.last_dones), s),
                       "ackppo_bootstrap")
        self.num_timesteps += self.n_steps * N * self.world
        _lib.ppo_check(L.ackppo_value(_ptr(self.params), _ptr(sim.obs_soa), N, _ptr(self.last_values), s),
                       "ackppo_value")

    def _train_desc(self):
        """ackppo_train_desc with every pointer of this learner (the buffers are never reallocated)."""
        d = _lib.TrainDesc()
        d.obs_rows, d.actions, d.old_log_prob = (t.data_ptr() for t in (self.buf_obs, self.buf_act, self.buf_logp))
        d.advantages, d.returns = self.buf_adv.data_ptr(), self.buf_ret.data_ptr()
        d.n_idx, d.batch = self.n_steps * self.n_envs, self.batch_size
        d.params, d.exp_avg, d.exp_avg_sq = (t.data_ptr() for t in (self.params, self.exp_avg, self.exp_avg_sq))
        d.perm, d.stats, d.moments = self.perm.data_ptr(), self.mb_stats.data_ptr(), self.mb_moments.data_ptr()
        d.moments_count = self.mb_moments.numel()
        self.set_epoch_buffers(True, d)
        d.grad_partial, d.loss_partial = self.gpart.data_ptr(), self.lpart.data_ptr()
        d.grad, d.loss_acc, d.grad_norm_out = self.grad.data_ptr(), self.loss_acc.data_ptr(), self.gnorm.data_ptr()
        d.world = self.world
        d.log_std_min = float("-inf") if self.log_std_min is None else float(self.log_std_min)
        self.set_weight_image(True, d)
        return d

    def set_epoch_buffers(self, on: bool, d=None):
        """on (default): every epoch's shuffle and advantage statistics of a train() call come from
        one launch at its start (ackppo_train_desc perm_epochs / stats_epochs); off: one shuffle and
        one statistics launch per epoch. The same values either way."""
        d = self._desc if d is None else d
        d.perm_epochs, d.stats_epochs = ((self.perm_epochs.data_ptr(), self.stats_epochs.data_ptr()) if on
                                         else (None, None))

    def set_weight_image(self, on: bool, d=None):
        """on (default): the gradient launches copy each net's weights into LDS from a pre-laid-out
        image that every Adam step keeps current (ackppo_train_desc weight_image; the same bits), by
        LDS-DMA, with the first tile's index and observation-row gathers in flight under the copies;
        off: they load and transpose the parameter vector themselves, then gather. (Round 4, before the
        gathers overlapped the copies: 32.5 us per minibatch with the image against 32.1 without.)"""
        d = self._desc if d is None else d
        d.weight_image = self.weight_image.data_ptr() if on else None

    def set_collective(self, kind: str | None):
        """The update's all-reduce hook (shard.TrainerCollective): "torch", "rccl", "host", None = the
        backend's default at world > 1 ("rccl" on RCCL, "host" on gloo), or no hook at all at world 1."""
        if self.collective is not None:
            self.collective.close()
            self.collective = None
        d = self._desc
        d.allreduce, d.allreduce_user = None, None
        if self.world == 1 and kind is None:
            return
        c = shard.TrainerCollective(self.world, self.device, kind=kind)
        c.register(self.grad)
        flat = self.mb_moments.view(-1)
        nm, nmb = self.mb_moments.shape[1], self.mb_moments.shape[1] // self.n_epochs
        c.register(flat[0:2 * nm])              # all-epoch moments: (count, sum) rows, then deviations
        c.register(flat[2 * nm:3 * nm])
        c.register(flat[0:2 * nmb])             # per-epoch layout [3][nmb] (set_epoch_buffers(False))
        c.register(flat[2 * nmb:3 * nmb])
        self.collective = c
        d.allreduce, d.allreduce_user = c.fn.value, c.user

    def train(self):
        """SB3 PPO.train: n_epochs over shuffled minibatches -- ONE ackppo_train call (every launch
        and collective of the update enqueued from C), then the logging scalars."""
        d = self._desc
        S, B = self.n_steps * self.n_envs, self.batch_size
        nmb = (S + B - 1) // B
        d.n_epochs, d.perm_key, d.perm_epoch0 = self.n_epochs, self.perm_key, self.perm_epoch
        d.normalize_advantage = int(self.normalize_advantage)
        d.clip_range, d.ent_coef, d.vf_coef, d.max_grad_norm = (self.clip_range, self.ent_coef, self.vf_coef,
                                                                self.max_grad_norm)
        d.learning_rate, d.beta1, d.beta2, d.eps, d.adam_step0 = self.learning_rate, 0.9, 0.999, 1e-5, self.adam_step
        _lib.ppo_check(self.L.ackppo_train(C.byref(d), self._stream()), "ackppo_train")
        self.perm_epoch += self.n_epochs
        self.adam_step += self.n_epochs * nmb
        la = self.loss_acc.cpu().tolist()
        n = max(la[4], 1.0)
        log_std = self.params[:2].detach().cpu()
        self.logger = {"train/policy_gradient_loss": la[0] / n, "train/value_loss": la[1] / n,
                       "train/clip_fraction": la[2] / n, "train/approx_kl": la[3] / n,
                       "train/entropy_loss": -float((0.5 + 0.5 * math.log(2 * math.pi) + log_std).sum()),
                       "train/std": float(log_std.exp().mean()), "train/n_updates": self.adam_step,
                       "train/grad_norm": float(self.gnorm.item())}

    def learn(self, total_timesteps: int, callback=None, log_interval: int = 1, reset_num_timesteps: bool = True,
              progress_bar: bool = False):
        if reset_num_timesteps:
            self.num_timesteps = 0
        else:  # stable-baselines3 semantics: a continued run learns total_timesteps more
            total_timesteps += self.num_timesteps
        it = 0
        t0 = time.perf_counter()
        while self.num_timesteps < total_timesteps:
            self.collect_rollouts()
            self.train()
            it += 1
            ep = shard.summarize_returns(shard.gather_episode_stats(self.sim.episode, self.world))
            self.sim.episode[2:].zero_()  # per-rollout completed-episode statistics
            self.episodes_total += ep["episodes"]
            self.logger.update({"rollout/episodes": ep["episodes"], "rollout/ep_rew_mean": ep["mean_return"],
                                "rollout/episodes_total": self.episodes_total,
                                "time/iterations": it, "time/total_timesteps": self.num_timesteps,
                                "time/fps": self.num_timesteps / max(time.perf_counter() - t0, 1e-9)})
            if callback is not None and callback(self) is False:
                break
            if self.verbose and self.rank == 0 and it % log_interval == 0:
                print({k: (round(v, 6) if isinstance(v, float) else v) for k, v in self.logger.items()}, flush=True)
        return self
