"""BatchedAckermannSim: device-resident state for N Ackermann-robot envs + the HIP step.

Torch tensors are only the device array container; every byte of physics is computed by
libackphys.so (include/ackphys.h). This is the batched replacement for the reference's
`mujoco.MjData` + `mujoco.mj_step` pair (src/rl/envs/ackermann_env.py:150-153, :200).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

NSTATE, NOBS = 44, 79
CONTACTS, AUTORESET, POSTSTEP_OBS = 1, 2, 4

# state word offsets (include/ackphys.h)
ST_QPOS, ST_QVEL, ST_WARM, ST_GOAL, ST_REF, ST_STEP, ST_EPIS = 0, 13, 25, 37, 39, 42, 43


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _raw_stream(device_index: int) -> int:
    """hipStream_t of torch's current stream on the device (the stream every launch is enqueued on)."""
    return torch.cuda.current_stream(device_index).cuda_stream


if hasattr(torch._C, "_cuda_getCurrentRawStream"):  # same value, without building a Stream object
    def _raw_stream(device_index: int) -> int:  # noqa: F811
        return torch._C._cuda_getCurrentRawStream(device_index)


class BatchedAckermannSim:
    def __init__(self, num_envs: int, device="cuda:0", seed: int = 0, contacts: bool = True,
                 env_offset: int = 0, model_blob: bytes | None = None, max_episode_steps: int = 1000,
                 goal_distance_threshold: float = 0.5, collision_threshold: float = 0.15,
                 max_linear_velocity: float = 1.0, max_angular_velocity: float = 1.0, variant: str = "auto",
                 poststep_obs: bool = False, scene: str = "flat", action_repeat: int = 1, nohit_clear: bool = False,
                 goal_cells: int = 0):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("BatchedAckermannSim runs on the GPU only (no CPU fallback)")
        self.n = int(num_envs)
        self.seed = int(seed)
        self.contacts = bool(contacts)
        # render_mode="human" semantics: obs/reward from the post-step pose (ackermann_env.py:202-207)
        self.poststep_obs = bool(poststep_obs)
        L = _lib.lib()
        self.scene = scene
        blob = model_blob if model_blob is not None else _lib.load_blob(scene)
        ctx = C.c_void_p()
        _lib.check(L.ackphys_create(blob, len(blob), self.n, self.device.index or 0, C.byref(ctx)), "ackphys_create")
        self._ctx = ctx
        self.env_offset = int(env_offset)
        _lib.check(L.ackphys_set_env_offset(ctx, self.env_offset), "ackphys_set_env_offset")
        # action_repeat / nohit_clear / goal_cells: opt-in task variants, NOT the reference env
        # (include/ackphys.h; goal_cells: maze goals in free cells of the obstacle scene)
        self.params = _lib.EnvParams(int(max_episode_steps), float(goal_distance_threshold), float(collision_threshold),
                                     float(max_linear_velocity), float(max_angular_velocity), int(action_repeat),
                                     1 if nohit_clear else 0, int(goal_cells))
        _lib.check(L.ackphys_set_env_params(ctx, C.byref(self.params)), "ackphys_set_env_params")
        self.variant = variant
        _lib.check(L.ackphys_set_variant(ctx, {"lane": 0, "quad": 1, "auto": 2, "lane16": 3}[variant]), "ackphys_set_variant")
        f32, u8 = torch.float32, torch.uint8
        d = self.device
        self.state = torch.zeros(NSTATE, self.n, dtype=f32, device=d)
        self.obs_soa = torch.zeros(NOBS, self.n, dtype=f32, device=d)
        self.terminal_obs_soa = torch.zeros(NOBS, self.n, dtype=f32, device=d)
        self.reward = torch.zeros(self.n, dtype=f32, device=d)
        self.term = torch.zeros(self.n, dtype=u8, device=d)
        self.trunc = torch.zeros(self.n, dtype=u8, device=d)
        self.info = torch.zeros(4, self.n, dtype=f32, device=d)
        self.episode = torch.zeros(4, self.n, dtype=f32, device=d)
        # the buffers are never reallocated (set_state copies in place): their C pointers are built
        # once, so a step costs one ctypes call and a handful of attribute reads on the host
        self._c = {k: C.c_void_p(getattr(self, k).data_ptr()) for k in
                   ("state", "obs_soa", "terminal_obs_soa", "reward", "term", "trunc", "info", "episode")}
        self._dev_index = self.device.index or 0

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and _lib._lib is not None:
            _lib._lib.ackphys_destroy(ctx)
            self._ctx = None

    @property
    def flags(self) -> int:
        return (CONTACTS if self.contacts else 0) | (POSTSTEP_OBS if self.poststep_obs else 0)

    def _stream(self):
        return C.c_void_p(_raw_stream(self._dev_index))

    def set_goal_cells(self, goal_cells: int):
        """Opt-in maze goals (obstacle scene): change goal_cells between launches; it applies to the
        goals of later resets (e.g. a curriculum over the maze)."""
        self.params.goal_cells = int(goal_cells)
        _lib.check(_lib.lib().ackphys_set_env_params(self._ctx, C.byref(self.params)), "ackphys_set_env_params")

    def reset(self, mask: torch.Tensor | None = None, seed: int | None = None) -> torch.Tensor:
        if seed is not None:
            self.seed = int(seed)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        _lib.check(_lib.lib().ackphys_reset(self._ctx, _ptr(m), self.seed, _ptr(self.state), _ptr(self.obs_soa),
                                            self._stream()), "ackphys_reset")
        return self.obs_soa

    def step(self, actions: torch.Tensor, autoreset: bool = True, want_info: bool = True,
             want_terminal: bool = True, track_episodes: bool = True):
        """actions [N,2] float32 on device. Returns SoA obs [79,N], reward, term, trunc (views of
        the sim's buffers, overwritten by the next call)."""
        if actions.dtype != torch.float32 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.shape != (self.n, 2):
            raise ValueError(f"actions must be [{self.n}, 2], got {tuple(actions.shape)}")
        flags = self.flags | (AUTORESET if autoreset else 0)
        c = self._c
        rc = _lib.lib().ackphys_step(
            self._ctx, actions.data_ptr(), c["state"], c["obs_soa"], c["reward"], c["term"], c["trunc"],
            c["terminal_obs_soa"] if (autoreset and want_terminal) else None, c["info"] if want_info else None,
            c["episode"] if track_episodes else None, flags, self.seed, _raw_stream(self._dev_index))
        if rc:
            _lib.check(rc, "ackphys_step")
        return self.obs_soa, self.reward, self.term, self.trunc

    def rollout(self, actions: torch.Tensor, autoreset: bool = True, want_info: bool = True,
                want_terminal: bool = True, track_episodes: bool = True, per_step_outputs: bool = True):
        """K steps of an open-loop action sequence in one launch (ackphys_rollout): the same as
        K calls of `step(actions[k])`. actions [K,N,2] float32 on device. With per_step_outputs the
        result is freshly allocated [K,...] tensors (obs [K,79,N], reward [K,N], term, trunc; info
        [K,4,N] and terminal obs [K,79,N] when asked for); without, the sim's single-step buffers
        (holding step K-1's outputs) are returned, as after K `step` calls."""
        if actions.dtype != torch.float32 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.dim() != 3 or actions.shape[1:] != (self.n, 2) or actions.shape[0] < 1:
            raise ValueError(f"actions must be [K, {self.n}, 2], got {tuple(actions.shape)}")
        k = int(actions.shape[0])
        flags = self.flags | (AUTORESET if autoreset else 0)
        term_on = autoreset and want_terminal
        if per_step_outputs:
            f32, u8, d = torch.float32, torch.uint8, self.device
            obs = torch.empty(k, NOBS, self.n, dtype=f32, device=d)
            rew = torch.empty(k, self.n, dtype=f32, device=d)
            term = torch.empty(k, self.n, dtype=u8, device=d)
            trunc = torch.empty(k, self.n, dtype=u8, device=d)
            # terminal obs rows are written only for done envs: zero-filled like the sim's buffer
            tobs = torch.zeros(k, NOBS, self.n, dtype=f32, device=d) if term_on else None
            info = torch.empty(k, 4, self.n, dtype=f32, device=d) if want_info else None
            ptrs = (_ptr(obs), _ptr(rew), _ptr(term), _ptr(trunc), _ptr(tobs), _ptr(info))
        else:  # the sim's own buffers: their C pointers are prebuilt (one ctypes call, as in step)
            obs, rew, term, trunc = self.obs_soa, self.reward, self.term, self.trunc
            c = self._c
            ptrs = (c["obs_soa"], c["reward"], c["term"], c["trunc"], c["terminal_obs_soa"] if term_on else None,
                    c["info"] if want_info else None)
        rc = _lib.lib().ackphys_rollout(
            self._ctx, k, actions.data_ptr(), self._c["state"], *ptrs, self._c["episode"] if track_episodes else None,
            flags, self.seed, 1 if per_step_outputs else 0, _raw_stream(self._dev_index))
        if rc:
            _lib.check(rc, "ackphys_rollout")
        if per_step_outputs:
            self.last_rollout = {"terminal_obs": tobs, "info": info}
            # the single-step buffers hold step K-1's outputs afterwards, as after K `step` calls
            # (a policy or the VecEnv reading sim.obs_soa next must see the current observation)
            self.obs_soa.copy_(obs[-1])
            self.reward.copy_(rew[-1])
            self.term.copy_(term[-1])
            self.trunc.copy_(trunc[-1])
            if info is not None:
                self.info.copy_(info[-1])
            if tobs is not None:  # written only for envs done at step K-1 (earlier rows stay as step wrote them)
                done = (term[-1] | trunc[-1]).bool()
                if k > 1:  # an env done at an earlier step keeps that step's terminal row, as in K step calls
                    done_any = (term[:-1] | trunc[:-1]).bool()
                    last = torch.where(done_any, torch.arange(k - 1, device=self.device)[:, None], -1).amax(0)
                    earlier = (last >= 0) & ~done
                    rows = tobs.gather(0, last.clamp(min=0)[None, None, :].expand(1, NOBS, self.n))[0]
                    self.terminal_obs_soa.copy_(torch.where(earlier[None, :], rows, self.terminal_obs_soa))
                self.terminal_obs_soa.copy_(torch.where(done[None, :], tobs[-1], self.terminal_obs_soa))
        return obs, rew, term, trunc

    def rollout_buffers(self, k_steps: int, want_info: bool = False, want_terminal: bool = False) -> dict:
        """Preallocated per-step output slices for `rollout_launcher(..., outputs=...)`: obs
        [K,79,N], reward [K,N], term, trunc [K,N] (uint8), info [K,4,N] / terminal obs [K,79,N]
        when asked for (a rollout buffer a consumer of every step's observation reads)."""
        f32, u8, d, n, k = torch.float32, torch.uint8, self.device, self.n, int(k_steps)
        return {"obs": torch.empty(k, NOBS, n, dtype=f32, device=d), "reward": torch.empty(k, n, dtype=f32, device=d),
                "term": torch.empty(k, n, dtype=u8, device=d), "trunc": torch.empty(k, n, dtype=u8, device=d),
                "terminal_obs": torch.zeros(k, NOBS, n, dtype=f32, device=d) if want_terminal else None,
                "info": torch.empty(k, 4, n, dtype=f32, device=d) if want_info else None}

    def rollout_launcher(self, actions: torch.Tensor, autoreset: bool = True, want_info: bool = False,
                         want_terminal: bool = False, track_episodes: bool = True, outputs: dict | None = None):
        """A zero-argument callable that launches `rollout(actions, per_step_outputs=False)` on the
        stream current at launch time with the sim's seed at launch time (a later reset(seed=...)
        applies): every other C argument is converted once, here, so a launch costs one ctypes call
        and two conversions (for timed windows of a few tens of microseconds, where the Python
        checks and argument conversion of `rollout` are a visible share of the host clock)."""
        if actions.dtype != torch.float32 or actions.device != self.device or not actions.is_contiguous():
            raise ValueError("rollout_launcher: actions must be a contiguous float32 tensor on the sim's device")
        if actions.dim() != 3 or actions.shape[1:] != (self.n, 2) or actions.shape[0] < 1:
            raise ValueError(f"actions must be [K, {self.n}, 2], got {tuple(actions.shape)}")
        fn = _lib.lib().ackphys_rollout
        c = self._c
        flags = self.flags | (AUTORESET if autoreset else 0)
        k = int(actions.shape[0])
        term_on = autoreset and want_terminal
        if outputs is None:  # step K-1's outputs in the sim's own buffers (in place, as K step calls)
            outs = (c["obs_soa"], c["reward"], c["term"], c["trunc"], c["terminal_obs_soa"] if term_on else None,
                    c["info"] if want_info else None)
        else:  # every step's outputs in its own slice of the caller's [K, ...] buffers (rollout_buffers)
            shapes = {"obs": (k, NOBS, self.n), "reward": (k, self.n), "term": (k, self.n), "trunc": (k, self.n),
                      "terminal_obs": (k, NOBS, self.n), "info": (k, 4, self.n)}
            for name in ("obs", "reward", "term", "trunc") + (("terminal_obs",) if term_on else ()) + (
                    ("info",) if want_info else ()):
                t = outputs.get(name)
                if t is None or tuple(t.shape) != shapes[name] or not t.is_contiguous() or t.device != self.device:
                    raise ValueError(f"rollout_launcher: outputs[{name!r}] must be a contiguous {shapes[name]} tensor")
            outs = (_ptr(outputs["obs"]), _ptr(outputs["reward"]), _ptr(outputs["term"]), _ptr(outputs["trunc"]),
                    _ptr(outputs["terminal_obs"]) if term_on else None, _ptr(outputs["info"]) if want_info else None)
        args = (self._ctx, C.c_int(k), C.c_void_p(actions.data_ptr()), c["state"], *outs,
                c["episode"] if track_episodes else None, C.c_uint32(flags))
        per_step, dev = C.c_int(0 if outputs is None else 1), self._dev_index

        def launch():
            rc = fn(*args, self.seed, per_step, _raw_stream(dev))
            if rc:
                _lib.check(rc, "ackphys_rollout")
        launch.actions = actions  # keeps the action buffer (and the output slices) alive as long as the launcher
        launch.outputs = outputs
        return launch

    def random_actions(self, k_steps: int, seed: int = 0, step0: int = 0) -> torch.Tensor:
        """[K, N, 2] i.i.d. U[-1,1) actions from Philox(seed; env, step) on device."""
        out = torch.empty(k_steps, self.n, 2, dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().ackphys_random_actions(self._ctx, _ptr(out), int(k_steps), int(seed), int(step0),
                                                     self._stream()), "ackphys_random_actions")
        return out

    # state helpers (host-side views for tests / checkpoints)
    def get_state(self) -> torch.Tensor:
        return self.state.clone()

    def set_state(self, state: torch.Tensor):
        self.state.copy_(state.to(self.device, torch.float32))
