"""ackphys_rollout (K steps per launch) against K ackphys_step calls, on the GPU.

The rollout kernels run the single-step kernels' code once per step inside one launch, so the
outputs must be bit-identical to K `step` calls on the same actions: every step's obs, reward,
terminated / truncated flags, info and terminal observations, and the final state and episode
statistics. The single-step kernels are the oracle-checked ones (test_gpu_parity.py,
test_gpu_obstacles.py); these tests carry that parity over to the rollout path. Sizes are ragged
(not a multiple of 64 or 16), episodes are short so auto-resets happen inside a launch, and a
few envs start from a non-finite state (mj_checkVel reset, the redo barrier inside the loop).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CASES = [  # (scene, contacts, variant, poststep)
    ("flat", False, "auto", False),    # BASELINE configs[1]: ackphys_rollout_nc_kernel
    ("flat", False, "lane16", False),  # 16 envs per wave
    ("flat", True, "auto", False),     # configs[2]: ackphys_rollout_quad_kernel (8 envs per wave)
    ("flat", True, "lane", False),     # ackphys_rollout_kernel (lane mapping with contacts)
    ("obstacles", True, "auto", False),  # configs[4]: ackphys_rollout_obst8_kernel (8 envs per wave)
    ("flat", True, "auto", True),      # post-step obs: K single-step launches
]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _pair(n, scene, contacts, variant, poststep, eplen):
    from mujoco_playground_amd.sim import BatchedAckermannSim
    kw = dict(seed=3, contacts=contacts, variant=variant, scene=scene, poststep_obs=poststep,
              max_episode_steps=eplen)
    a, b = BatchedAckermannSim(n, DEV, **kw), BatchedAckermannSim(n, DEV, **kw)
    a.reset()
    b.reset()
    return a, b


def _settle(a, b, k):
    acts = a.random_actions(k, seed=11)
    for i in range(k):
        a.step(acts[i])
        b.step(acts[i])


def _poison(a, b, envs):
    from mujoco_playground_amd.sim import ST_QVEL
    for s in (a, b):
        s.state[ST_QVEL + 2, envs] = float("nan")


@pytest.mark.parametrize("scene,contacts,variant,poststep", CASES)
def test_rollout_equals_steps(scene, contacts, variant, poststep):
    n, K = 301, 23
    a, b = _pair(n, scene, contacts, variant, poststep, eplen=9)
    _settle(a, b, 5)  # some envs mid-episode, some near truncation
    _poison(a, b, [7, 150])
    acts = a.random_actions(K, seed=21, step0=5)
    obs, rew, term, trunc = a.rollout(acts)
    tobs, info = a.last_rollout["terminal_obs"], a.last_rollout["info"]
    dones = 0
    for k in range(K):
        ob, rb, tb, trb = b.step(acts[k])
        assert torch.equal(obs[k], ob), f"obs differs at step {k}"
        assert torch.equal(rew[k], rb), f"reward differs at step {k}"
        assert torch.equal(term[k], tb) and torch.equal(trunc[k], trb), f"flags differ at step {k}"
        assert torch.equal(info[k], b.info), f"info differs at step {k}"
        done = (tb | trb).bool()
        dones += int(done.sum())
        assert torch.equal(tobs[k][:, done], b.terminal_obs_soa[:, done]), f"terminal obs differ at step {k}"
        assert not tobs[k][:, ~done].any(), "terminal obs written for an env that was not done"
    assert torch.equal(a.state, b.state)
    assert torch.equal(a.episode, b.episode)
    # the single-step buffers hold step K-1's outputs afterwards (a policy reads a.obs_soa next),
    # and every env's terminal-obs row is the one of its last done step, as after K step calls
    for name in ("obs_soa", "reward", "term", "trunc", "info", "terminal_obs_soa"):
        assert torch.equal(getattr(a, name), getattr(b, name)), f"single-step buffer {name} is stale"
    assert dones >= n  # every env truncated at least once inside the launch (eplen 9, 23 steps)
    assert bool(info[0][3, 7]) and bool(info[0][3, 150])  # the poisoned envs were reset (bad_state)


@pytest.mark.parametrize("contacts", [False, True])
def test_rollout_in_place_outputs(contacts):
    """per_step_outputs=False: the single-step buffers hold the last step's outputs, as after K
    step calls; the episode statistics and the state match too."""
    n, K = 4096, 40
    a, b = _pair(n, "flat", contacts, "auto", False, eplen=1000)
    acts = a.random_actions(K, seed=2)
    a.rollout(acts, want_info=False, per_step_outputs=False)
    for k in range(K):
        b.step(acts[k], want_info=False)
    for name in ("obs_soa", "reward", "term", "trunc", "state", "episode"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


def test_rollout_rejects_bad_shapes():
    from mujoco_playground_amd.sim import BatchedAckermannSim
    s = BatchedAckermannSim(64, DEV, contacts=False)
    s.reset()
    with pytest.raises(ValueError):
        s.rollout(torch.zeros(64, 2, device=DEV))
    with pytest.raises(ValueError):
        s.rollout(torch.zeros(0, 64, 2, device=DEV))


@pytest.mark.parametrize("scene,contacts", [("flat", False), ("flat", True), ("obstacles", True)])
def test_rollout_full_episode_4096(scene, contacts):
    """BASELINE sizes: 4096 envs through a whole episode (truncation at step 1000 inside the launch):
    the rollout's final state, episode statistics and every step's reward / flags are bit-identical
    to 1001 ackphys_step calls; the truncation step resets every env exactly once."""
    n, K = 4096, 1001
    a, b = _pair(n, scene, contacts, "auto", False, eplen=1000)
    acts = a.random_actions(K, seed=4)
    obs, rew, term, trunc = a.rollout(acts, want_info=False, want_terminal=False)
    rb = torch.empty(K, n, device=DEV)
    tb = torch.empty(K, n, dtype=torch.uint8, device=DEV)
    for k in range(K):
        _, r, t, tr = b.step(acts[k], want_info=False, want_terminal=False)
        rb[k] = r
        tb[k] = t | (tr << 1)
    assert torch.equal(rew, rb)
    assert torch.equal(term | (trunc << 1), tb)
    assert torch.equal(obs[-1], b.obs_soa)
    assert torch.equal(a.obs_soa, b.obs_soa)
    assert torch.equal(a.state, b.state)
    assert torch.equal(a.episode, b.episode)
    assert int(trunc[999].sum()) == n - int(term[:999].any(0).sum())  # envs not terminated earlier
