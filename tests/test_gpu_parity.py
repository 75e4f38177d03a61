"""GPU (MI355X) parity of libackphys.so against the f64 CPU oracle.

Tolerances (stated, f32 kernel vs f64 oracle, teacher-forced = both start every step from the
same GPU state): |dqpos| <= 1e-5, |dqvel| <= 1e-3, obs <= 1e-4 abs (+1e-5 rel), reward <= 1e-4.
Measured on MI355X: |dqpos| ~2e-7, |dqvel| ~3e-5. Discrete outputs
(terminated/truncated, reset goals' Philox draws, action streams) must match exactly.

Contact-activation boundary: a mesh vertex or wheel rim point lying within ~1e-7 m of the floor
can be in the f32 contact set and not in the f64 one (tests/golden/quad_miss_state.npz: a
second plate vertex at dist ~0). The contact force then legitimately differs. A step that misses
the tolerances is excused only if the oracle, with the body shifted along z by <= 1e-6 m,
reproduces the GPU step within the same tolerances; excused env-steps are counted and must stay
below 0.1 % of the env-steps checked.

Ray-horizon boundary: a rangefinder ray horizontal in the world to rounding reads the cutoff (a
floor hit far away, clamped) or -1 (no hit) depending on the last bit of the pose; such obs
entries (and that env's reward, whose collision term sees the same reading) are excused, counted
and capped the same way (`_horizon_rays_excused`).
"""
import numpy as np
import pytest
import torch

from conftest import f64_state

pytestmark = pytest.mark.gpu

TOL_QPOS, TOL_QVEL, TOL_OBS, TOL_REW = 1e-5, 1e-3, 1e-4, 1e-4
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def make_sim(n, **kw):
    from mujoco_playground_amd.sim import BatchedAckermannSim
    return BatchedAckermannSim(n, DEV, **kw)


def fresh_oracle(blob, **params):
    from oracle.oracle import Oracle
    o = Oracle(blob)
    if params:
        o.set_env_params(**params)
    return o


BOUNDARY_DZ = (1e-7, -1e-7, 1e-6, -1e-6)
LIDAR_CUTOFF, NRAYS = 12.0, 72  # rangefinder cutoff (ackermann_robot_v2.xml) and obs[0:72] = rays


def _horizon_rays_excused(g, o, d):
    """True if every obs entry over tolerance is a ray reading -1 (no hit) on one side and the
    cutoff on the other: a ray whose world direction is horizontal to rounding (z component ~1e-7)
    hits the floor arbitrarily far away (clamped to the cutoff) or never (-1), and which one is
    decided by the last bit of the pose. The reward's collision term sees the same flip, so the
    env's reward is not compared either; such env-steps are counted and capped like contact
    boundary cases."""
    bad = np.nonzero(d > TOL_OBS)[0]
    if bad.size == 0 or bad.max() >= NRAYS:
        return False
    pair = np.sort(np.stack([g[bad], o[bad]]), axis=0)
    return bool(np.all(np.abs(pair[0] + 1.0) <= 1e-6) and np.all(np.abs(pair[1] - LIDAR_CUTOFF) <= 1e-4))


def _boundary_excused(o, before_e, act_e, after_e, flags, seed):
    """True if the oracle reproduces the GPU step once the body is shifted by <= 1e-6 m in z."""
    for dz in BOUNDARY_DZ:
        s = before_e[None].copy()
        s[0, 2] += dz
        o.step(s, act_e[None], flags=flags, seed=seed)
        if (np.abs(after_e[:13] - s[0, :13]).max() <= TOL_QPOS and
                np.abs(after_e[13:25] - s[0, 13:25]).max() <= TOL_QVEL):
            return True
    return False


def teacher_forced(sim, o, acts, steps, flags, seed, check_obs=True, on_step=None):
    """Every step from the GPU's own state, against the oracle (tolerances above; boundary excuses
    counted and capped). on_step(k, ref, after, ok, oterm, otr, tobs): extra per-step checks."""
    worst = dict(qpos=0.0, qvel=0.0, obs=0.0, rew=0.0, excused=0, excused_rays=0)
    for k in range(steps):
        before = f64_state(sim.state)
        sim.step(acts[k], autoreset=bool(flags & 2))
        torch.cuda.synchronize()
        after = f64_state(sim.state)
        ref = before.copy()
        a_np = acts[k].cpu().numpy()
        oobs, orew, oterm, otr, tobs, _ = o.step(ref, a_np, flags=flags, seed=seed, terminal=True)
        dq = np.abs(after[:, :13] - ref[:, :13]).max(axis=1)
        dv = np.abs(after[:, 13:25] - ref[:, 13:25]).max(axis=1)
        ok = (dq <= TOL_QPOS) & (dv <= TOL_QVEL)
        for e in np.nonzero(~ok)[0]:
            assert _boundary_excused(o, before[e], a_np[e], after[e], flags, seed), (
                f"step {k} env {e}: |dqpos| {dq[e]:.3e} |dqvel| {dv[e]:.3e}")
            worst["excused"] += 1
        worst["qpos"] = max(worst["qpos"], dq[ok].max(initial=0.0))
        worst["qvel"] = max(worst["qvel"], dv[ok].max(initial=0.0))
        np.testing.assert_array_equal(sim.term.cpu().numpy().astype(bool)[ok], oterm[ok])
        np.testing.assert_array_equal(sim.trunc.cpu().numpy().astype(bool)[ok], otr[ok])
        np.testing.assert_array_equal(after[ok, 42:44], ref[ok, 42:44])
        if on_step is not None:
            on_step(k, ref, after, ok, oterm, otr, tobs)
        if check_obs:
            gobs = sim.obs_soa.cpu().numpy().T
            do = np.abs(gobs - oobs) / (1.0 + 0.1 * np.abs(oobs))
            horizon = np.zeros(sim.n, dtype=bool)
            for e in np.nonzero(do.max(axis=1) > TOL_OBS)[0]:  # only envs with an entry over tolerance
                horizon[e] = _horizon_rays_excused(gobs[e], oobs[e], do[e])
            worst["excused_rays"] += int((ok & horizon).sum())
            okr = ok & ~horizon
            worst["obs"] = max(worst["obs"], do[okr].max(initial=0.0))
            assert do[okr].max(initial=0.0) <= TOL_OBS, f"step {k}: obs {do[okr].max()}"
            dr = np.abs(sim.reward.cpu().numpy() - orew)[okr].max(initial=0.0)
            worst["rew"] = max(worst["rew"], dr)
            assert dr <= TOL_REW
    assert worst["excused"] <= 1e-3 * steps * sim.n, worst
    assert worst["excused_rays"] <= 1e-3 * steps * sim.n, worst
    return worst


def test_contact_boundary_state_is_excused(blob):
    """The recorded boundary case: a second plate vertex at dist ~0 whose contact activation depends
    on the last bits (the f32 kernels have put it in contact where the f64 oracle does not; which
    side a kernel lands on moves with its rounding). Each kernel's step must match the oracle or be
    excused; the excuse itself is checked independently of the kernels' rounding: the boundary is
    genuine (a 1e-7 m shift changes the oracle's step beyond the tolerances), the shifted step is
    excused, a wrong step is not."""
    d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                           "quad_miss_state.npz"))
    before, action = d["before"], d["action"].astype(np.float32)
    o = fresh_oracle(blob)
    ref = before[None].copy()
    o.step(ref, action[None], flags=3, seed=11)
    shifted = []
    for dz in BOUNDARY_DZ:
        s = before[None].copy()
        s[0, 2] += dz
        o.step(s, action[None], flags=3, seed=11)
        shifted.append(s[0])
    far = max(shifted, key=lambda s: np.abs(s[:13] - ref[0, :13]).max())
    assert np.abs(far[:13] - ref[0, :13]).max() > TOL_QPOS  # a 1e-7..1e-6 m shift flips the contact set
    assert _boundary_excused(o, before, action, far, 3, 11)
    wrong = ref[0].copy()
    wrong[13] += 0.1
    assert not _boundary_excused(o, before, action, wrong, 3, 11)
    for variant in ("lane", "quad"):
        sim = make_sim(1, seed=11, contacts=True, variant=variant)
        st = before[:, None].astype(np.float32)
        st[42:44] = before[42:44, None].astype(np.uint32).view(np.float32)
        sim.set_state(torch.tensor(st, device=DEV))
        sim.step(torch.tensor(action[None], device=DEV))
        torch.cuda.synchronize()
        after = f64_state(sim.state)[0]
        match = (np.abs(after[:13] - ref[0, :13]).max() <= TOL_QPOS and
                 np.abs(after[13:25] - ref[0, 13:25]).max() <= TOL_QVEL)
        assert match or _boundary_excused(o, before, action, after, 3, 11), variant


def test_reset_matches_oracle(blob):
    n = 300  # not a multiple of 64: partial last block
    sim = make_sim(n, seed=7)
    sim.reset()
    torch.cuda.synchronize()
    o = fresh_oracle(blob)
    st = np.zeros((n, 44))
    oobs = o.reset(st, seed=7)
    g = f64_state(sim.state)
    np.testing.assert_allclose(g[:, :37], st[:, :37], atol=1e-7)
    np.testing.assert_allclose(g[:, 37:39], st[:, 37:39], atol=1e-5)   # goals: f32 trig of the same Philox draws
    np.testing.assert_array_equal(g[:, 42:44], st[:, 42:44])
    np.testing.assert_allclose(sim.obs_soa.cpu().numpy().T, oobs, atol=1e-5)


@pytest.mark.parametrize("variant", ["quad", "lane"])
@pytest.mark.parametrize("contacts", [True, False])
def test_teacher_forced_step(blob, contacts, variant):
    n, steps, seed = 256, 150, 11
    sim = make_sim(n, seed=seed, contacts=contacts, variant=variant)
    sim.reset()
    acts = sim.random_actions(steps, seed=seed)
    o = fresh_oracle(blob)
    flags = (1 if contacts else 0) | 2
    w = teacher_forced(sim, o, acts, steps, flags, seed)
    print("worst", variant, contacts, w)


@pytest.mark.parametrize("variant", ["quad", "lane"])
def test_poststep_obs_mode(blob, variant):
    """render_mode="human" semantics (mj_forward after mj_step): obs/reward from the integrated pose."""
    n, steps, seed = 128, 40, 13
    sim = make_sim(n, seed=seed, contacts=True, variant=variant, poststep_obs=True, max_episode_steps=30)
    sim.reset()
    acts = sim.random_actions(steps, seed=seed)
    teacher_forced(sim, fresh_oracle(blob, max_episode_steps=30), acts, steps, 1 | 2 | 4, seed)


MAPPINGS = [("quad", True), ("lane", True), ("lane", False), ("lane16", False)]


@pytest.mark.parametrize("variant,contacts", MAPPINGS)
def test_autoreset_truncation_terminal_obs(blob, variant, contacts):
    n, seed = 64, 3
    sim = make_sim(n, seed=seed, max_episode_steps=25, variant=variant, contacts=contacts)
    sim.reset()
    acts = sim.random_actions(60, seed=seed)
    o = fresh_oracle(blob, max_episode_steps=25)
    st = f64_state(sim.state)
    flags = 2 | (1 if contacts else 0)
    for k in range(60):
        sim.step(acts[k])
        torch.cuda.synchronize()
        oobs, orew, oterm, otr, tobs, _ = o.step(st, acts[k].cpu().numpy(), flags=flags, seed=seed, terminal=True)
        g = f64_state(sim.state)
        done = oterm | otr
        assert np.array_equal(sim.trunc.cpu().numpy().astype(bool), otr)
        if k == 24:
            assert otr.all()
        if done.any():
            np.testing.assert_allclose(sim.terminal_obs_soa.cpu().numpy().T[done], tobs[done], atol=1e-4)
            np.testing.assert_allclose(sim.obs_soa.cpu().numpy().T[done], oobs[done], atol=1e-4)
            assert np.all(g[done, 42] == 0) and np.all(g[done, 43] == st[done, 43])
        np.testing.assert_allclose(g[:, :25], st[:, :25], atol=5e-4)
        st = g  # continue from the GPU state (teacher forcing)
    ep = sim.episode.cpu().numpy()
    assert np.all(ep[3] == 2)  # two completed episodes of 25 steps in 60


def test_termination_bonus(blob):
    n, seed = 64, 5
    sim = make_sim(n, seed=seed, goal_distance_threshold=100.0)
    sim.reset()
    acts = sim.random_actions(2, seed=seed)
    o = fresh_oracle(blob, goal_distance_threshold=100.0)
    teacher_forced(sim, o, acts, 2, 3, seed)
    assert sim.term.cpu().numpy().all()


def test_env_params_make_env_defaults(blob):
    """make_ackermann_env defaults (max_linear_velocity=0.5, goal threshold 0.3)."""
    n, seed = 128, 9
    kw = dict(max_linear_velocity=0.5, goal_distance_threshold=0.3)
    sim = make_sim(n, seed=seed, **kw)
    sim.reset()
    acts = sim.random_actions(40, seed=seed)
    teacher_forced(sim, o := fresh_oracle(blob, **kw), acts, 40, 3, seed)


def test_random_actions_are_philox_exact():
    from oracle.oracle import philox
    sim = make_sim(96, seed=0, env_offset=1000)
    a = sim.random_actions(3, seed=0x1234567890AB, step0=7).cpu().numpy()
    for k in range(3):
        for e in [0, 17, 95]:
            x = philox([1000 + e, 7 + k, 1, 0], [0x567890AB, 0x1234])
            u = ((x[:2] >> 8).astype(np.float64) / 16777216.0).astype(np.float32)
            np.testing.assert_array_equal(a[k, e], (2 * u - 1).astype(np.float32))


def test_bad_ctrl_nan_path(blob):
    """action -> R = inf -> 0*inf = NaN wheel speeds in the reference controller; ctrl zeroed."""
    n, seed = 64, 2
    sim = make_sim(n, seed=seed)
    sim.reset()
    a = torch.tensor([[0.5, 6e-6]] * n, device=DEV)
    acts = torch.stack([a] * 5)
    teacher_forced(sim, fresh_oracle(blob), acts, 5, 3, seed)


@pytest.mark.parametrize("variant,contacts", MAPPINGS)
def test_bad_state_resets(blob, variant, contacts):
    n, seed = 64, 4
    sim = make_sim(n, seed=seed, variant=variant, contacts=contacts)
    sim.reset()
    st = sim.state.clone()
    st[13, :8] = float("nan")          # bad qvel
    st[0, 8:16] = 3e10                  # bad qpos
    # steer angles away from qpos0 on the bad envs (and some good ones): a reset state is observed
    # and integrated from qpos0 whatever its loaded angles. (The contacts-off kernel's helper waves
    # also factor M / M + hB at qpos0 for it; from a resting qpos0 the steer-dependent entries --
    # wheel spin inertia times the spin axis -- move the result by less than the tolerances, as a
    # negative control with factors taken at the loaded angles showed, tools/negctl.sh)
    st[9, :24] = 0.4
    st[11, :24] = -0.3
    sim.set_state(st)
    acts = sim.random_actions(3, seed=seed)
    teacher_forced(sim, fresh_oracle(blob), acts, 3, 2 | (1 if contacts else 0), seed)
    assert torch.isfinite(sim.state).all()


@pytest.mark.parametrize("variant,contacts", MAPPINGS)
def test_bad_acceleration_redo(blob, variant, contacts):
    """mj_checkAcc: a finite state whose accelerations blow up (hinge speeds 1e6 rad/s) is reset to
    qpos0 and the step redone from there -- dynamics, observation (taken at qpos0), reward, info[3]."""
    n, seed = 64, 6
    sim = make_sim(n, seed=seed, variant=variant, contacts=contacts)
    sim.reset()
    acts = sim.random_actions(4, seed=seed)
    o = fresh_oracle(blob)
    flags = 2 | (1 if contacts else 0)
    teacher_forced(sim, o, acts[:1], 1, flags, seed)
    st = sim.state.clone()
    st[13 + 6:13 + 12, ::3] = 1e6      # every third env: hinge speeds that trip mj_checkAcc
    sim.set_state(st)
    before = f64_state(sim.state)
    sim.step(acts[1])
    torch.cuda.synchronize()
    ref = before.copy()
    oobs, orew, oterm, otr, _, oinfo = o.step(ref, acts[1].cpu().numpy(), flags=flags, seed=seed, terminal=True)
    after = f64_state(sim.state)
    assert np.abs(after[:, :25] - ref[:, :25]).max() <= TOL_QVEL
    np.testing.assert_allclose(sim.obs_soa.cpu().numpy().T, oobs, atol=TOL_OBS)
    np.testing.assert_allclose(sim.reward.cpu().numpy(), orew, atol=TOL_REW)
    np.testing.assert_array_equal(sim.info[3].cpu().numpy(), oinfo[:, 3])
    assert oinfo[::3, 3].all() and not oinfo[1::3, 3].any()
    teacher_forced(sim, o, acts[2:], 2, flags, seed)


@pytest.mark.parametrize("seed", [31, 32, 33])
def test_contacts_off_random_states(blob, seed):
    """The contacts-off kernel solves a predicted piece of the constraint problem first and falls
    back to Newton when the rows end elsewhere; on the benchmark workload every lane is exact at
    the prediction, so this test drives it from random states (tilted / airborne chassis, steers
    beyond their limits, large wheel and steer speeds, arbitrary warmstarts) where predictions
    miss, and holds every step to the oracle with the standard tolerances."""
    n = 512
    rng = np.random.default_rng(seed)
    sim = make_sim(n, seed=seed, contacts=False, variant="lane")
    sim.reset()
    st = f64_state(sim.state)
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    st[:, 0:3] = rng.uniform(-2, 2, (n, 3))
    st[:, 3:7] = q
    st[:, 7:13] = rng.uniform(-3, 3, (n, 6))
    st[:, [9, 11]] = rng.uniform(-0.8, 0.8, (n, 2))          # steers, limits at +-0.611
    st[:, 13:19] = rng.normal(0, 2, (n, 6))                   # chassis twist
    st[:, 19:25] = rng.normal(0, 20, (n, 6))                  # hinge speeds
    st[:, [21, 23]] = rng.normal(0, 3, (n, 2))                # steer speeds
    st[:, 25:37] = rng.normal(0, 50, (n, 12))                 # warmstarts
    g = st.T.astype(np.float32)
    g[42:44] = st[:, 42:44].T.astype(np.uint32).view(np.float32)
    sim.set_state(torch.tensor(g, device=DEV))
    acts = sim.random_actions(4, seed=seed)
    teacher_forced(sim, fresh_oracle(blob), acts, 4, 2, seed)


@pytest.mark.parametrize("variant", ["quad", "lane"])
def test_sharding_is_exact(variant):
    """Two half-size shards with env offsets reproduce the unsharded run bit for bit."""
    n, steps, seed = 128, 60, 21
    full = make_sim(n, seed=seed, max_episode_steps=20, variant=variant)
    a = make_sim(n // 2, seed=seed, env_offset=0, max_episode_steps=20, variant=variant)
    b = make_sim(n // 2, seed=seed, env_offset=n // 2, max_episode_steps=20, variant=variant)
    for s in (full, a, b):
        s.reset()
    acts_full = full.random_actions(steps, seed=seed)
    acts_a, acts_b = a.random_actions(steps, seed=seed), b.random_actions(steps, seed=seed)
    assert torch.equal(acts_full[:, : n // 2], acts_a) and torch.equal(acts_full[:, n // 2:], acts_b)
    for k in range(steps):
        full.step(acts_full[k])
        a.step(acts_a[k])
        b.step(acts_b[k])
    torch.cuda.synchronize()
    assert torch.equal(full.state, torch.cat([a.state, b.state], dim=1))
    assert torch.equal(full.obs_soa, torch.cat([a.obs_soa, b.obs_soa], dim=1))


def test_full_size_properties():
    """BASELINE size (4096 envs) through truncation: size-independent invariants."""
    n = 4096
    sim = make_sim(n, seed=1, contacts=True)
    sim.reset()
    acts = sim.random_actions(1010, seed=1)
    done_count = torch.zeros(n, device=DEV)
    for k in range(1010):
        _, rew, term, trunc = sim.step(acts[k], want_info=False)
        done_count += (term | trunc).float()
    torch.cuda.synchronize()
    st = sim.state
    assert torch.isfinite(st[:37]).all()
    qn = torch.linalg.norm(st[3:7], dim=0)
    assert (qn - 1).abs().max().item() < 1e-5
    steps = st[42].view(torch.int32)
    assert (steps >= 0).all() and (steps < 1000).all()
    assert torch.equal(sim.episode[3], done_count)
    assert (done_count >= 1).all()       # everybody truncated at least once
    assert torch.isfinite(sim.obs_soa).all()


def test_vec_env_and_gym_api():
    from mujoco_playground_amd.rl import AckermannRobotEnv, make_ackermann_env
    venv = make_ackermann_env(env_type="vec", num_envs=64, max_episode_steps=5, device=DEV)
    obs = venv.reset()
    assert obs.shape == (64, 79)
    for k in range(5):
        obs, rew, done, infos = venv.step(torch.zeros(64, 2, device=DEV))
    assert done.all() and len(infos) == 64
    assert infos[0]["terminal_observation"].shape == (79,) and infos[0]["TimeLimit.truncated"]
    assert infos[0]["episode"]["l"] == 5
    env = AckermannRobotEnv(device=DEV)
    o, info = env.reset(seed=0)
    assert o.shape == (79,) and o.dtype == np.float32 and set(info) == {"map_name", "goal_position",
                                                                         "start_position"}
    o2, r, te, tr, info = env.step(env.action_space.sample())
    assert np.array_equal(o2, o)  # obs lag: first step returns the reset pose's observation
    assert isinstance(r, float) and isinstance(te, bool) and isinstance(tr, bool)
    assert set(info) >= {"goal_distance", "collision", "min_lidar", "step", "linear_velocity", "angular_velocity"}


@pytest.mark.parametrize("variant", ["quad", "lane", "lane16"])
def test_ragged_env_count(blob, variant):
    """n = 301: a partial last wave (lane) / partial last quad group (quad) / partial 16-env wave."""
    n, steps, seed = 301, 30, 17
    sim = make_sim(n, seed=seed, contacts=True, variant=variant)
    sim.reset()
    acts = sim.random_actions(steps, seed=seed)
    teacher_forced(sim, fresh_oracle(blob), acts, steps, 3, seed)


def test_variants_agree_at_4096(blob):
    """All kernel mappings step the same 4096 envs to the same state within the stated f32
    tolerances (|dqpos| <= 1e-5, |dqvel| <= 1e-3; they differ in summation order only). An env-step
    where two mappings disagree beyond them is excused only if BOTH results are valid answers to the
    f64 oracle (within the tolerances, or reproduced by it from a state shifted <= 1e-6 m: a contact
    activation boundary, see the module docstring); excused env-steps are counted and capped at 0.1 %."""
    n, steps, seed = 4096, 50, 2
    sims = {v: make_sim(n, seed=seed, contacts=True, variant=v) for v in ("lane", "quad", "lane16")}
    acts = sims["lane"].random_actions(steps, seed=seed)
    for s in sims.values():
        s.reset()
    o = fresh_oracle(blob)
    excused, worst = 0, dict(qpos=0.0, qvel=0.0)
    for k in range(steps):
        start = sims["lane"].state.clone()
        for s in sims.values():
            s.state.copy_(start)
            s.step(acts[k])
        torch.cuda.synchronize()
        ref = f64_state(sims["lane"].state)
        before = None
        for v in ("quad", "lane16"):
            g = f64_state(sims[v].state)
            dq = np.abs(g[:, :13] - ref[:, :13]).max(axis=1)
            dv = np.abs(g[:, 13:25] - ref[:, 13:25]).max(axis=1)
            ok = (dq <= TOL_QPOS) & (dv <= TOL_QVEL)
            worst["qpos"] = max(worst["qpos"], dq[ok].max(initial=0.0))
            worst["qvel"] = max(worst["qvel"], dv[ok].max(initial=0.0))
            if ok.all():
                continue
            if before is None:
                before = f64_state(start)
            a_np = acts[k].cpu().numpy()
            for e in np.nonzero(~ok)[0]:
                for res in (g[e], ref[e]):
                    s1 = before[e][None].copy()
                    o.step(s1, a_np[e][None], flags=3, seed=seed)
                    good = (np.abs(res[:13] - s1[0, :13]).max() <= TOL_QPOS and
                            np.abs(res[13:25] - s1[0, 13:25]).max() <= TOL_QVEL)
                    assert good or _boundary_excused(o, before[e], a_np[e], res, 3, seed), (
                        f"step {k} env {e} {v}: |dqpos| {dq[e]:.3e} |dqvel| {dv[e]:.3e}, not an oracle answer")
                excused += 1
    print("variants_agree", worst, "excused", excused, "of", 2 * steps * n)
    assert excused <= 1e-3 * 2 * steps * n, excused
