"""Closed-form physics pins on the HIP path (physics parity against real MuJoCo is unpinned, so the
analytic behaviour of this model is checked directly; the oracle passes the same pins,
tests/test_oracle_physics.py).

Contacts off (BASELINE configs[1]) the robot falls freely and its wheels spin free:
* each rear wheel settles where its velocity servo balances damping and friction loss,
  kv (c - w) = b w + floss sign(w) (ackermann_robot_v2.xml:44-51, :119-121);
* the steering servo (kp 40, kv 6, +-2 N m, :113-117) never settles (SURVEY finding 8): its force
  sits on the limit with alternating sign and the steer velocity alternates +-v with the same
  amplitude whatever the target -- a period-2 limit cycle, an attractor, so the free-running GPU
  trajectory reaches the oracle's amplitude although it does not follow the oracle step for step.
"""
import numpy as np
import pytest
import torch

from conftest import f64_state
from test_oracle_physics import (FMAX_STEER, QPOS_FL_STEER, QVEL_FL_STEER, QVEL_RL, QVEL_RR, steer_servo_force,
                                 wheel_steady_state)

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("variant", ["auto", "lane16", "quad"])
def test_free_wheel_steady_state(variant):
    from mujoco_playground_amd.sim import BatchedAckermannSim
    from oracle.oracle import controller
    n = 256
    v = np.linspace(-1.0, 1.0, n).astype(np.float32)
    v = v[np.abs(v) > 0.05][:n // 2]                   # wheel targets well outside the friction zone
    acts = np.stack([v, np.zeros_like(v)], 1).astype(np.float32)
    sim = BatchedAckermannSim(len(acts), DEV, seed=0, contacts=False, variant=variant)
    sim.reset()
    a = torch.tensor(acts, device=DEV)
    sim.rollout(a[None].expand(300, -1, -1).contiguous(), want_info=False, per_step_outputs=False)
    torch.cuda.synchronize()
    st = f64_state(sim.state)
    w = wheel_steady_state(np.array([controller(x) for x in acts])[:, 1:3])
    for j, dof in enumerate((QVEL_RL, QVEL_RR)):
        np.testing.assert_allclose(st[:, 13 + dof], w[:, j], rtol=1e-5)


@pytest.mark.parametrize("variant", ["auto", "quad"])
def test_steering_servo_limit_cycle(variant, oracle):
    """Targets 0.1-0.5 rad (away from the joint limits): from step 220 on the force is +-2 with the
    sign flipping every step, and each env's cycle amplitude equals the oracle's free-running one
    (the cycle is an attractor: perturbing the oracle's start by 1e-5 moves it by 2e-7)."""
    from mujoco_playground_amd.sim import BatchedAckermannSim
    from oracle.oracle import controller
    rng = np.random.default_rng(0)
    n, K, W = 128, 320, 220
    acts = np.stack([rng.uniform(0.2, 0.6, n), rng.choice([-1, 1], n) * rng.uniform(0.3, 0.6, n)], 1)
    acts = acts.astype(np.float32)
    ctrl = np.array([controller(x) for x in acts])[:, 0]
    sim = BatchedAckermannSim(n, DEV, seed=0, contacts=False, variant=variant)
    sim.reset()
    a = torch.tensor(acts, device=DEV)
    ost = np.zeros((n, 44))
    oracle.reset(ost, seed=0)
    F, V, OV = [], [], []
    for k in range(K):
        st = f64_state(sim.state)
        F.append(steer_servo_force(ctrl, st[:, QPOS_FL_STEER], st[:, 13 + QVEL_FL_STEER]))
        V.append(st[:, 13 + QVEL_FL_STEER])
        OV.append(ost[:, 13 + QVEL_FL_STEER].copy())
        sim.step(a, want_info=False)
        oracle.step(ost, acts, flags=0)
    F, V = np.array(F[W:]), np.array(V[W:])
    assert np.all(np.abs(F) == FMAX_STEER) and np.all(F[1:] * F[:-1] < 0)
    assert np.all(V[1:] * V[:-1] < 0)
    np.testing.assert_allclose(np.abs(V).mean(0), np.abs(np.array(OV[W:])).mean(0), rtol=1e-3)
