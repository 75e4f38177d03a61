"""Invariants that pin the oracle's mj_step restatement where no MuJoCo fixture exists
(physics parity vs real MuJoCo is unpinned)."""
import numpy as np
import pytest

from mujoco_playground_amd.model.compiler import mass_matrix
from mujoco_playground_amd.model.mathutil import quat_normalize, quat_to_mat


def rand_state(rng, z=0.3):
    st = np.zeros(44)
    st[0:3] = [rng.uniform(-1, 1), rng.uniform(-1, 1), z]
    st[3:7] = quat_normalize(rng.normal(size=4))
    st[7:13] = rng.uniform(-0.6, 0.6, 6)
    st[13:25] = rng.normal(size=12)
    return st


def test_mass_matrix_matches_independent_jacobian_form(oracle, cmodel):
    rng = np.random.default_rng(0)
    for _ in range(10):
        st = rand_state(rng)
        d = oracle.diag(st, [0, 0, 0], flags=0)
        M = mass_matrix(cmodel, st[:13])
        np.testing.assert_allclose(d["qM"], M, atol=1e-13)
        assert np.all(np.linalg.eigvalsh(d["qM"]) > 0)


def _bias_newton_euler(cmodel, st, eps=1e-6):
    """Independent bias: sum_b J_b^T (m (Jdot qd - g), I Jdot_w qd + w x I w), Jdot by central
    differences along the motion (quaternion integrated with the body-frame angular velocity)."""
    from mujoco_playground_amd.model.compiler import body_frames, point_jacobian

    def integ(q, qd, h):
        q = q.copy()
        q[0:3] += h * qd[0:3]
        w = qd[3:6]
        a = np.linalg.norm(w) * h
        ax = w / np.linalg.norm(w) if np.linalg.norm(w) > 0 else np.array([1.0, 0, 0])
        qr = np.array([np.cos(a / 2), *(np.sin(a / 2) * ax)])
        w1, x1, y1, z1 = q[3:7]
        w2, x2, y2, z2 = qr
        q[3:7] = [w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                  w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2]
        q[7:13] += h * qd[6:12]
        return q

    def jacs(q):
        xpos, xmat, _, xa, xx = body_frames(cmodel, q)
        out = []
        for b in range(1, cmodel.nbody):
            xi = xpos[b] + xmat[b] @ cmodel.body_ipos[b]
            out.append((point_jacobian(cmodel, xpos, xmat, xa, xx, b, xi), xmat[b]))
        return out

    q, qd = st[:13], st[13:25]
    J0, Jp, Jm = jacs(q), jacs(integ(q, qd, eps)), jacs(integ(q, qd, -eps))
    b = np.zeros(12)
    for k, bid in enumerate(range(1, cmodel.nbody)):
        m = cmodel.body_mass[bid]
        if m <= 0:
            continue
        J, R = J0[k]
        Jd = (Jp[k][0] - Jm[k][0]) / (2 * eps)
        Ri = R @ quat_to_mat(cmodel.body_iquat[bid])
        I = Ri @ np.diag(cmodel.body_inertia[bid]) @ Ri.T
        v_dot = Jd[:3] @ qd
        w = J[3:] @ qd
        w_dot = Jd[3:] @ qd
        f = m * (v_dot - cmodel.gravity)
        tau = I @ w_dot + np.cross(w, I @ w)
        b += J[:3].T @ f + J[3:].T @ tau
    return b


def test_bias_matches_finite_difference_newton_euler(oracle, cmodel):
    rng = np.random.default_rng(1)
    for _ in range(5):
        st = rand_state(rng)
        d = oracle.diag(st, [0, 0, 0], flags=0)
        np.testing.assert_allclose(d["qfrc_bias"], _bias_newton_euler(cmodel, st), rtol=1e-6, atol=1e-6)


def test_free_fall_closed_form(oracle):
    """contacts disabled: chassis z follows semi-implicit Euler exactly."""
    st = np.zeros((1, 44))
    oracle.reset(st, seed=0)
    h, g = 0.002, 9.81
    z0 = st[0, 2]
    for k in range(1, 51):
        oracle.step(st, np.zeros((1, 2), np.float32), flags=0)
        assert abs(st[0, 2] - (z0 - g * h * h * k * (k + 1) / 2)) < 1e-12
        assert abs(st[0, 15] + g * h * k) < 1e-12


# rear drive (ackermann_robot_v2.xml:119-121: velocity servo kv 1) on a rear wheel joint (:44-51:
# damping 0.15, frictionloss 0.02); steering servo (:113-117: kp 40, kv 6, forcerange +-2)
KV_REAR, B_REAR, FLOSS_REAR = 1.0, 0.15, 0.02
KP_STEER, KV_STEER, FMAX_STEER = 40.0, 6.0, 2.0
QVEL_RL, QVEL_RR, QVEL_FL_STEER, QPOS_FL_STEER = 6, 7, 8, 9


def wheel_steady_state(c):
    """With contacts off the wheels spin free. At a steady spin (qacc = 0) the rear wheel's
    generalised forces balance: kv (c - w) = b w + floss sign(w) (the friction-loss row saturates at
    +-floss once |w| is far above its Huber zone), so w* = (kv c - floss sign c) / (kv + b)."""
    c = np.asarray(c, dtype=np.float64)
    return (KV_REAR * c - FLOSS_REAR * np.sign(c)) / (KV_REAR + B_REAR)


def steer_servo_force(ctrl, q, qdot):
    return np.clip(KP_STEER * (ctrl - q) - KV_STEER * qdot, -FMAX_STEER, FMAX_STEER)


def test_free_wheel_steady_state_closed_form(oracle):
    from oracle.oracle import controller
    acts = np.array([[0.5, 0.0], [0.2, 0.0], [-0.7, 0.0], [1.0, 0.0], [0.5, 0.5], [-0.3, -0.8]], np.float32)
    st = np.zeros((len(acts), 44))
    oracle.reset(st, seed=0)
    for _ in range(300):
        oracle.step(st, acts, flags=0)
    ctrl = np.array([controller(a) for a in acts])
    w = wheel_steady_state(ctrl[:, 1:3])
    # straight: exact to rounding; turning: the steering servo's limit cycle (below) shakes the
    # chassis and couples into the wheel joints at the 1e-7 level
    rtol = np.where(acts[:, 1] == 0, 1e-9, 1e-6)
    for j, dof in enumerate((QVEL_RL, QVEL_RR)):
        assert np.all(np.abs(st[:, 13 + dof] - w[:, j]) <= rtol * np.abs(w[:, j])), (st[:, 13 + dof], w[:, j])


def test_steering_servo_period_two_limit_cycle(oracle):
    """SURVEY finding 8: the steer axis inertia is so small that kv dt / I >> 2, and MuJoCo does not
    integrate the actuator's kv term implicitly, so the servo never settles: once the transient is
    over its force sits on the force limit with the sign flipping every step and the steer
    velocity alternates +-v (a period-2 limit cycle) whose amplitude is the same whatever the
    target (targets away from the +-35 deg joint limits, whose rows would enter the cycle)."""
    from oracle.oracle import controller
    acts = np.array([[0.5, 0.5], [0.3, -0.4], [0.6, -0.2], [0.8, 0.1]], np.float32)
    ctrl = np.array([controller(a) for a in acts])
    st = np.zeros((len(acts), 44))
    oracle.reset(st, seed=0)
    F, v = [], []
    for k in range(300):
        F.append(steer_servo_force(ctrl[:, 0], st[:, QPOS_FL_STEER], st[:, 13 + QVEL_FL_STEER]))
        v.append(st[:, 13 + QVEL_FL_STEER].copy())
        oracle.step(st, acts, flags=0)
    F, v = np.array(F[100:]), np.array(v[100:])
    assert np.all(np.abs(F) == FMAX_STEER)                 # saturated every step
    assert np.all(F[1:] * F[:-1] < 0)                      # sign alternates every step
    assert np.all(v[1:] * v[:-1] < 0)
    amp = np.abs(v)
    assert np.all(np.abs(amp - amp.mean(0)) < 5e-3 * amp.mean(0))  # constant amplitude (period 2)
    m = amp.mean(0)
    assert np.all(np.abs(m - m.mean()) < 1e-4 * m.mean()) and 2.2 < m.mean() < 2.4  # target-independent


def test_static_rest_normal_force(oracle):
    st = np.zeros((1, 44))
    oracle.reset(st, seed=0)
    for _ in range(400):
        oracle.step(st, np.zeros((1, 2), np.float32))
    d = oracle.diag(st[0], [0, 0, 0])
    assert d["ncon"] == 8
    assert abs(d["qfrc_constraint"][2] - 10.3 * 9.81) < 1e-6
    assert np.abs(st[0, 13:25]).max() < 1e-6


def test_newton_solution_is_optimal(oracle):
    """KKT: the returned qacc minimises the primal cost (compare against perturbations)."""
    st = np.zeros((1, 44))
    oracle.reset(st, seed=0)
    rng = np.random.default_rng(2)
    for _ in range(120):
        oracle.step(st, rng.uniform(-1, 1, (1, 2)).astype(np.float32))
    d = oracle.diag(st[0], [0.3, 20.0, -15.0])
    assert d["nefc"] >= 11  # at least one contact (4 pyramid rows) besides eq + friction
    M, a0, a = d["qM"], d["qacc_smooth"], d["qacc"]
    J = d["efc_J"]
    typ, R, aref = d["efc"][:, 0], d["efc"][:, 2], d["efc"][:, 3]
    fl = np.where(typ == 1, np.array([0.0] * len(typ)), 0.0)
    # friction loss values by dof (rows of type 1 are dofs 6..11 in order)
    floss = np.array([0.02, 0.02, 0.005, 0.012, 0.005, 0.012])
    fl[typ == 1] = floss

    def cost(x):
        jar = J @ x - aref
        c = 0.5 * (x - a0) @ M @ (x - a0)
        for i, t in enumerate(typ):
            D = 1 / R[i]
            if t == 0:
                c += 0.5 * D * jar[i] ** 2
            elif t == 1:
                th = R[i] * fl[i]
                c += (-fl[i] * jar[i] - 0.5 * R[i] * fl[i] ** 2 if jar[i] <= -th else
                      fl[i] * jar[i] - 0.5 * R[i] * fl[i] ** 2 if jar[i] >= th else 0.5 * D * jar[i] ** 2)
            elif jar[i] < 0:
                c += 0.5 * D * jar[i] ** 2
        return c

    c0 = cost(a)
    for _ in range(200):
        dx = rng.normal(size=12) * 10 ** rng.uniform(-6, -2)
        assert cost(a + dx) >= c0 - 1e-9 * max(1, abs(c0))


def test_quaternion_stays_normalized(oracle):
    st = np.zeros((4, 44))
    oracle.reset(st, seed=3)
    rng = np.random.default_rng(3)
    for _ in range(300):
        oracle.step(st, rng.uniform(-1, 1, (4, 2)).astype(np.float32))
    assert np.abs(np.linalg.norm(st[:, 3:7], axis=1) - 1).max() < 1e-9


def test_poststep_obs_flag_uses_integrated_pose(oracle):
    """FLAG_POSTSTEP_OBS (render_mode="human"): obs[72:75] = odometry of the *new* qpos; default
    lags one step (obs of the pre-integration pose)."""
    from oracle.oracle import FLAG_AUTORESET, FLAG_CONTACTS, FLAG_POSTSTEP_OBS
    n = 4
    st = np.zeros((n, 44))
    oracle.reset(st, seed=3)
    acts = np.tile(np.array([[0.8, 0.3]], np.float32), (n, 1))
    for _ in range(200):   # get moving
        oracle.step(st, acts, flags=FLAG_CONTACTS | FLAG_AUTORESET, seed=3)
    lag, post = st.copy(), st.copy()
    obs_lag = oracle.step(lag, acts, flags=FLAG_CONTACTS | FLAG_AUTORESET, seed=3)[0]
    obs_post = oracle.step(post, acts, flags=FLAG_CONTACTS | FLAG_AUTORESET | FLAG_POSTSTEP_OBS, seed=3)[0]
    np.testing.assert_array_equal(lag[:, :37], post[:, :37])            # same dynamics
    np.testing.assert_allclose(obs_lag[:, 72:74], (st[:, 0:2] - st[:, 39:41]).astype(np.float32), atol=1e-6)
    np.testing.assert_allclose(obs_post[:, 72:74], (post[:, 0:2] - post[:, 39:41]).astype(np.float32), atol=1e-6)
    assert np.abs(obs_post[:, 72:74] - obs_lag[:, 72:74]).max() > 1e-5


def test_step_cpu_twin_matches_row_oracle(blob):
    """ackphys_step_cpu / ackphys_reset_cpu (oracle/ackphys_oracle.h): the SoA f32
    host twin of the C-ABI equals the f64 row oracle rounded to f32, including autoreset,
    terminal obs and the episode-stat words."""
    import ctypes as C
    from oracle.oracle import Oracle, lib
    L = lib()
    n, seed, flags = 32, 5, 1 | 2
    oracle = Oracle(blob)
    oracle.set_env_params(max_episode_steps=12)
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    state = np.zeros((44, n), np.float32)
    obs = np.zeros((79, n), np.float32)
    assert L.ackphys_reset_cpu(oracle._ctx, n, None, seed, p(state), p(obs)) == 0
    rows = np.zeros((n, 44))
    robs = oracle.reset(rows, seed=seed)
    np.testing.assert_array_equal(obs.T, robs.astype(np.float32))
    rng = np.random.default_rng(0)
    rew, term, trunc = np.zeros(n, np.float32), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    tobs, info, ep = np.zeros((79, n), np.float32), np.zeros((4, n), np.float32), np.zeros((4, n), np.float32)
    for k in range(20):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        rows = np.ascontiguousarray(state.T, dtype=np.float64)
        rows[:, 42] = state[42].view(np.uint32)
        rows[:, 43] = state[43].view(np.uint32)
        o, r, te, tr, to, inf = oracle.step(rows, act, flags=flags, seed=seed, terminal=True)
        assert L.ackphys_step_cpu(oracle._ctx, n, p(act), p(state), p(obs), p(rew), p(term), p(trunc), p(tobs),
                                  p(info), p(ep), flags, seed, 1) == 0
        np.testing.assert_array_equal(state[:42].T, rows[:, :42].astype(np.float32))
        np.testing.assert_array_equal(state[42:].view(np.uint32).T, rows[:, 42:].astype(np.uint32))
        np.testing.assert_array_equal(obs.T, o.astype(np.float32))
        np.testing.assert_array_equal(rew, r.astype(np.float32))
        np.testing.assert_array_equal(term.astype(bool), te)
        np.testing.assert_array_equal(trunc.astype(bool), tr)
        done = te | tr
        np.testing.assert_array_equal(tobs.T[done], to[done].astype(np.float32))
    assert np.all(ep[3] == 1)    # one truncated episode of 12 steps each in 20 steps
    np.testing.assert_array_equal(ep[1], np.full(n, 8, np.float32))


def test_flop_counting_build_matches_the_oracle(tmp_path):
    """The FLOP-counting oracle build (oracle/flops/fd.hpp, `make -C oracle flops`) computes the same
    states as the plain oracle (the counting double only observes) and attributes its operations to
    the stages the bench reports (tools/count_flops.py -> profiles/oracle_flops.json)."""
    import ctypes as C
    import os
    import subprocess

    import numpy as np

    from mujoco_playground_amd import _lib
    from oracle import oracle as orc

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-C", os.path.join(repo, "oracle"), "flops"], check=True, capture_output=True)
    F = C.CDLL(os.path.join(repo, "oracle", "build", "libackphys_oracle_flops.so"))
    R = orc.lib()
    P, i32, u32, u64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64
    ULL = C.c_ulonglong * 16
    for L in (F, R):
        L.or_create.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(P)]
        L.ackphys_reset_cpu.argtypes = [P, i32, P, u64, P, P]
        L.ackphys_step_cpu.argtypes = [P, i32] + [P] * 9 + [u32, u64, i32]
    F.or_flops_read.argtypes = [ULL, ULL, i32]
    blob = _lib.load_blob("flat")
    n, ptr = 16, (lambda x: x.ctypes.data_as(P))
    out = []
    for L in (F, R):
        ctx = P()
        assert L.or_create(blob, len(blob), C.byref(ctx)) == 0
        st, obs = np.zeros((44, n), np.float32), np.zeros((79, n), np.float32)
        rew, term, trunc = np.zeros(n, np.float32), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        assert L.ackphys_reset_cpu(ctx, n, None, 3, ptr(st), ptr(obs)) == 0
        if L is F:
            F.or_flops_reset()
        rng = np.random.default_rng(1)
        for _ in range(5):
            act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
            assert L.ackphys_step_cpu(ctx, n, ptr(act), ptr(st), ptr(obs), ptr(rew), ptr(term), ptr(trunc), None,
                                      None, None, 3, 3, 1) == 0
        out.append((st.copy(), obs.copy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    fl, tr = ULL(), ULL()
    F.or_flops_read(fl, tr, 16)
    per = np.array(fl[:13], dtype=float) / (n * 5)
    # controller, kinematics, mass matrix, collision, rays, bias, qacc_smooth, rows, Newton, Euler
    assert (per[[1, 2, 3, 4, 5, 6, 7, 8, 9, 10]] > 0).all()
    assert 2e4 < per.sum() < 2e5
