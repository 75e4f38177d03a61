"""GPU parity at the BASELINE size: 4096 envs, the bench's own workload (bench.py run_gpu: seed 0,
env_offset 0, reset, Philox random actions keyed (seed 0; env, step)), every env-step teacher-forced
against the f64 CPU oracle (both sides start each step from the same GPU state).

  configs[1] (contacts off)   steps 0-50 from reset (the bench's headline workload);
  configs[2] (contacts on)    steps 200-300, after the bench's 200 settle steps (one rollout launch,
                              bit-identical to per-step launches: tests/test_gpu_rollout.py);
  obstacle scene (configs[4]'s world)  the same window;
  the episode boundary, both scenes   steps 990-1010 (ackermann_env.py:216-220 truncation at 1000,
                              then the auto-reset of :143-185): step counter, truncation, the
                              terminal observation, the reset state with its Philox goal redraw and
                              odometry reference, and the reset observation, all against the oracle.

Tolerances and boundary excuses are those of tests/test_gpu_parity.py (flat scene) and
tests/test_gpu_obstacles.py (obstacle scene); here every excused env-step is counted, reported and
capped at 0.1 % of the env-steps checked. The oracle runs ~1.4 M env-steps/s on the box's cores, so
each window costs seconds.
"""
import json

import numpy as np
import pytest
import torch

import test_gpu_obstacles as TO
import test_gpu_parity as TP

pytestmark = pytest.mark.gpu

N, SEED, SETTLE = 4096, 0, 200   # bench.py: 4096 envs/GPU, seed 0, SETTLE_STEPS


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bench_sim(contacts, scene="flat"):
    from mujoco_playground_amd.sim import BatchedAckermannSim
    sim = BatchedAckermannSim(N, TP.DEV, seed=SEED, contacts=contacts, env_offset=0, scene=scene)
    sim.reset()
    return sim


def _report(name, w, steps):
    checked = steps * N
    w = {k: (float(v) if isinstance(v, (float, np.floating)) else int(v)) for k, v in w.items()}
    print("full_size_parity", json.dumps({"window": name, "env_steps": checked, **w}))
    assert w["excused"] <= 1e-3 * checked, w


def test_configs1_contacts_off_steps_0_50(blob):
    sim = _bench_sim(False)
    acts = sim.random_actions(50, seed=SEED)
    w = TP.teacher_forced(sim, TP.fresh_oracle(blob), acts, 50, 2, SEED)
    _report("configs[1] contacts off, steps 0-50", w, 50)


def test_configs2_contacts_on_steps_200_300(blob):
    sim = _bench_sim(True)
    acts = sim.random_actions(SETTLE + 100, seed=SEED)
    sim.rollout(acts[:SETTLE], want_info=False, per_step_outputs=False)
    w = TP.teacher_forced(sim, TP.fresh_oracle(blob), acts[SETTLE:], 100, 3, SEED)
    _report("configs[2] contacts on, steps 200-300", w, 100)


def test_obstacle_scene_steps_200_300():
    from mujoco_playground_amd import _lib
    sblob = _lib.load_blob("obstacles")
    lo, hi = _boxes(sblob)
    sim = _bench_sim(True, scene="obstacles")
    acts = sim.random_actions(SETTLE + 100, seed=SEED)
    sim.rollout(acts[:SETTLE], want_info=False, per_step_outputs=False)
    w = TO.teacher_forced(sim, TO.oracle(sblob), acts[SETTLE:], 100, 3, SEED, lo, hi)
    _report("obstacle scene, steps 200-300", w, 100)
    assert w["grazing_rays"] <= 1e-3 * w["rays"], w


def _boxes(sblob):
    from mujoco_playground_amd.model import blob as B
    h = B.unpack_header(sblob)
    g = [i for i in range(h.ngeom) if h.geom_type[i] == 6]
    c = np.array([list(h.geom_pos[i]) for i in g])
    s = np.array([list(h.geom_size[i]) for i in g])
    return c - s, c + s


def _boundary_checks(sim, tol_obs):
    """on_step checks of the episode-boundary windows: the auto-reset state words the generic
    comparison does not cover (goal 37-38 drawn from Philox keyed (env, episode), odometry
    reference 39-41) and the terminal observation of every env that reset."""
    seen = {"resets": 0}

    def check(k, ref, after, ok, oterm, otr, tobs):
        done = ok & (oterm | otr)
        seen["resets"] += int(done.sum())
        np.testing.assert_allclose(after[ok, 37:42], ref[ok, 37:42], rtol=1e-6, atol=1e-5)  # f32 goals: ~6 ulp at 8 m
        if done.any():
            gt = sim.terminal_obs_soa.cpu().numpy().T
            d = np.abs(gt[done] - tobs[done]) / (1.0 + 0.1 * np.abs(tobs[done]))
            ray_pair = np.isin(gt[done], (-1.0, 12.0)) & np.isin(tobs[done], (-1.0, 12.0))  # ray-horizon pairs
            assert (d[~ray_pair] <= tol_obs).all(), f"step {k}: terminal obs {d[~ray_pair].max()}"
    return check, seen


@pytest.mark.parametrize("scene", ["flat", "obstacles"])
def test_episode_boundary_steps_990_1010(blob, scene):
    """The step-1000 truncation -> auto-reset -> terminal observation -> goal redraw boundary at the
    BASELINE size, teacher-forced against the oracle: every env truncates at
    step 1000 of its first episode unless it terminated earlier."""
    from mujoco_playground_amd import _lib
    K0, W = 990, 20
    sblob = blob if scene == "flat" else _lib.load_blob("obstacles")
    sim = _bench_sim(True, scene=scene)
    acts = sim.random_actions(K0 + W, seed=SEED)
    sim.rollout(acts[:K0], want_info=False, per_step_outputs=False)
    check, seen = _boundary_checks(sim, TP.TOL_OBS)
    if scene == "flat":
        w = TP.teacher_forced(sim, TP.fresh_oracle(sblob), acts[K0:], W, 3, SEED, on_step=check)
    else:
        lo, hi = _boxes(sblob)
        w = TO.teacher_forced(sim, TO.oracle(sblob), acts[K0:], W, 3, SEED, lo, hi, on_step=check)
    assert seen["resets"] >= N // 2, seen  # the boundary really was crossed inside the window
    _report(f"{scene} scene, episode boundary steps 990-1010", dict(w, resets=seen["resets"]), W)
