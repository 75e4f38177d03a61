"""Why the GPU parity tolerances are what they are ("stated and justified by an
oracle f32-vs-f64 self-comparison").

The GPU kernel computes in f32 and the oracle in f64. Two effects set the floor any correct f32
implementation must be allowed:
  1. representation: the GPU state lives in f32, so the oracle's own answer moves when its
     input is rounded to f32 (and by +-1 ulp more, the rounding of one previous step);
  2. the reference solver's own stopping rule: MuJoCo's Newton stops at tolerance 1e-8 on the
     scaled cost improvement, so "the" mj_step answer is only defined that well.
This test measures both with the oracle alone (contacts on, a trajectory with rolling/bouncing
contacts) and checks that the stated bounds (tests/test_gpu_parity.py: |dqpos| <= 1e-5,
|dqvel| <= 1e-3) sit above that floor by a margin but are not vacuous. The numbers are
printed (pytest -s) and recorded in DESIGN.md §Parity.
"""
import numpy as np

from oracle.oracle import FLAG_AUTORESET, FLAG_CONTACTS, Oracle

TOL_QPOS, TOL_QVEL = 1e-5, 1e-3


def _trajectory_states(o, n=64, steps=120, seed=4):
    st = np.zeros((n, 44))
    o.reset(st, seed=seed)
    rng = np.random.default_rng(seed)
    snaps, acts = [], []
    for k in range(steps):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        if k % 20 == 19:
            snaps.append(st.copy())
            acts.append(a)
        o.step(st, a, flags=FLAG_CONTACTS | FLAG_AUTORESET, seed=seed)
    return snaps, acts


def _one_step(o, st, a):
    s = st.copy()
    o.step(s, a, flags=FLAG_CONTACTS | FLAG_AUTORESET, seed=4)
    return s


def test_f32_floor_and_solver_tolerance_justify_bounds(blob):
    o = Oracle(blob)
    o.set_solver(1e-12, 100)
    snaps, acts = _trajectory_states(o)
    rng = np.random.default_rng(1)
    rep_q = rep_v = sol_q = sol_v = 0.0
    loose = Oracle(blob)
    loose.set_solver(1e-8, 100)  # MuJoCo defaults: tolerance 1e-8, 100 iterations
    for st, a in zip(snaps, acts):
        ref = _one_step(o, st, a)
        # 1. f32 representation of the input state (+ one ulp of jitter on every word)
        s32 = st.copy()
        w = s32[:, :37].astype(np.float32)
        w = np.nextafter(w, np.where(rng.random(w.shape) < 0.5, -np.inf, np.inf).astype(np.float32))
        s32[:, :37] = w
        r32 = _one_step(o, s32, a)
        live = (ref[:, 42] != 0)        # skip envs that auto-reset on this step
        rep_q = max(rep_q, np.abs(r32[live, :13] - ref[live, :13]).max())
        rep_v = max(rep_v, np.abs(r32[live, 13:25] - ref[live, 13:25]).max())
        # 2. reference solver tolerance
        rl = _one_step(loose, st, a)
        sol_q = max(sol_q, np.abs(rl[live, :13] - ref[live, :13]).max())
        sol_v = max(sol_v, np.abs(rl[live, 13:25] - ref[live, 13:25]).max())
    print(f"\nf32 input floor: |dqpos| {rep_q:.3e} |dqvel| {rep_v:.3e}; "
          f"solver tol 1e-8 vs 1e-12: |dqpos| {sol_q:.3e} |dqvel| {sol_v:.3e}")
    floor_q, floor_v = max(rep_q, sol_q), max(rep_v, sol_v)
    # bounds are above the unavoidable floor ...
    assert floor_q < TOL_QPOS / 5 and floor_v < TOL_QVEL / 5
    # ... and a real error would still trip them: a wrong solve (1 Newton iteration) exceeds them
    bad = Oracle(blob)
    bad.set_solver(1e-12, 1)
    worst_v = 0.0
    for st, a in zip(snaps, acts):
        ref = _one_step(o, st, a)
        rb = _one_step(bad, st, a)
        worst_v = max(worst_v, np.abs(rb[:, 13:25] - ref[:, 13:25]).max())
    print(f"1-iteration Newton: |dqvel| {worst_v:.3e}")
    assert worst_v > TOL_QVEL
