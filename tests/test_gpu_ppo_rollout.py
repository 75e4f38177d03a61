"""The fused policy-in-the-loop rollout (ackphys_ppo_rollout: policy + env step + bootstrap for all T
steps in one launch) against the per-step path it replaces (ackppo_act / ackppo_act_boot +
ackphys_step per step, ackppo_bootstrap and ackppo_value after the last), bit for bit.

The per-step path is the one tests/test_gpu_ppo.py holds to the PPO oracle (itself pinned to torch
autograd and the reference checkpoints' policy) and tests/test_gpu_parity.py holds to the physics
oracle; equality carries both over. Every rollout-buffer array (observations, actions, log-probs,
values, bootstrapped rewards, episode starts), last_values / last_dones, the GAE output and the sim's
own state, observation, episode statistics and last-step buffers are compared exactly, over two
consecutive rollouts (the second starts from the first's last_dones and step counter). Short
episodes (truncation -> TimeLimit bootstrap and auto-reset inside the launch), a goal threshold that
terminates some episodes at once (termination: no bootstrap), ragged N (not a multiple of the
16-env workgroup, including a last workgroup whose second observation wave and dynamics wave hold no
env), both scenes, and envs whose state trips mj_checkAcc (the redo barrier).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BUFFERS = ("buf_obs", "buf_act", "buf_logp", "buf_val", "buf_rew", "buf_start", "last_dones", "last_values",
           "buf_adv", "buf_ret")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _pair(n, scene, n_steps, eplen, thr):
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    out = []
    for fused in (True, False):
        venv = AckermannVecEnv(n, device=DEV, seed=5, contacts=True, scene=scene, max_episode_steps=eplen,
                               goal_distance_threshold=thr)
        out.append(PPO("MlpPolicy", venv, n_steps=n_steps, batch_size=64, n_epochs=1, seed=3, fused_rollout=fused))
    return out


def _compare(a, b, tag):
    for name in BUFFERS:
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x, y), f"{tag}: {name} differs (max |d| {float((x - y).abs().max()):.3g})"
    for name in ("state", "obs_soa", "episode", "reward", "term", "trunc"):
        assert torch.equal(getattr(a.sim, name), getattr(b.sim, name)), f"{tag}: sim.{name} differs"
    done = (a.sim.term | a.sim.trunc).bool()
    assert torch.equal(a.sim.terminal_obs_soa[:, done], b.sim.terminal_obs_soa[:, done]), f"{tag}: terminal obs"


@pytest.mark.parametrize("scene,n", [("flat", 301), ("obstacles", 301), ("flat", 35)])
def test_fused_rollout_equals_per_step(scene, n):
    T = 23
    a, b = _pair(n, scene, T, eplen=9, thr=2.4)
    assert a.fused_rollout and not b.fused_rollout
    for it in range(2):
        a.collect_rollouts()
        b.collect_rollouts()
        torch.cuda.synchronize()
        _compare(a, b, f"{scene} rollout {it}")
        assert a._rollout_step == b._rollout_step == T * (it + 1)
    starts = a.buf_start[1:]
    assert 0 < float(starts.sum()) < starts.numel()  # resets inside the launch
    assert float(a.last_dones.sum()) > 0 or float(starts.sum()) > n  # truncations every 9 steps


def test_fused_rollout_redo_path():
    """Envs whose hinge speeds trip mj_checkAcc are reset to qpos0 and their step redone: the
    observation wave observes again after barrier 2 and repeats the policy work."""
    n, T = 64, 5
    a, b = _pair(n, "flat", T, eplen=1000, thr=0.5)
    a.collect_rollouts()
    b.collect_rollouts()
    for p in (a, b):
        st = p.sim.state.clone()
        st[13 + 6:13 + 12, ::5] = 1e6
        p.sim.set_state(st)
    a.collect_rollouts()
    b.collect_rollouts()
    torch.cuda.synchronize()
    _compare(a, b, "redo")


def test_fused_rollout_bench_shape():
    """The bench's PPO leg shape: 4096 envs, n_steps 32 (configs[3] per GPU)."""
    a, b = _pair(4096, "flat", 32, eplen=1000, thr=0.5)
    a.collect_rollouts()
    b.collect_rollouts()
    torch.cuda.synchronize()
    _compare(a, b, "4096 x 32")


def test_fused_rollout_refuses_unsupported():
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    venv = AckermannVecEnv(64, device=DEV, contacts=False)
    assert not PPO("MlpPolicy", venv, n_steps=4, batch_size=64).fused_rollout  # contacts off: per-step path
    with pytest.raises(ValueError):
        PPO("MlpPolicy", venv, n_steps=4, batch_size=64, fused_rollout=True)
