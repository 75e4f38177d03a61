"""Obstacle scene, CPU side: the scene merge, the compiled constants, and the
oracle's box narrowphase / ray casting against independent numpy restatements.

The reference has no loadable obstacle env (its MapSpawner is absent and the flat scene's mesh
paths dangle), so the scene semantics are ours (model/compiler.py merge_scene):
parity is oracle vs kernel; the narrowphase itself is checked here against brute-force
minimum-translation search with exact support functions (parity unpinned vs MuJoCo)."""
import os

import numpy as np
import pytest

from mujoco_playground_amd.model import blob as B
from mujoco_playground_amd.model.codegen import hull_features
from mujoco_playground_amd.model.compiler import (body_frames, compile_mjcf, compile_scene, default_model_path,
                                                  obstacle_scene_path)
from mujoco_playground_amd.model.mathutil import euler_to_quat, quat_to_mat

REF = "/root/reference"
ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mujoco_playground_amd", "model",
                      "assets")


def _scene_blob():
    return open(os.path.join(ASSETS, "ackermann_obstacles.apm"), "rb").read()


@pytest.fixture(scope="module")
def scene():
    from oracle.oracle import Oracle
    blob = _scene_blob()
    hdr = B.unpack_header(blob)
    return blob, hdr, Oracle(blob)


def test_scene_blob_facts(scene):
    blob, h, _ = scene
    types = list(h.geom_type[: h.ngeom])
    assert types.count(6) == 38 and types.count(0) == 1 and types.count(5) == 4 and types.count(7) == 2
    assert (h.nq, h.nv, h.nu, h.nsensor) == (13, 12, 3, 77)
    assert list(h.spawn) == pytest.approx([-2.9, -3.3, 0.1])
    # the flat scene's <default> reaches every geom: contacts use solref 0.01 1, solimp .95 .98 .002
    for g in range(h.ngeom):
        assert list(h.geom_solref[g]) == pytest.approx([0.01, 1.0])
        assert list(h.geom_solimp[g]) == pytest.approx([0.95, 0.98, 0.002, 0.5, 2.0])
    # joints keep MuJoCo's defaults
    assert list(h.dof_solref[0]) == pytest.approx([0.02, 1.0])


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent")
def test_scene_assets_up_to_date():
    from mujoco_playground_amd.model import build
    assert build.build(REF, check_only=True)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent")
def test_scene_robot_equals_robot_model():
    mr = compile_mjcf(default_model_path(REF))
    ms = compile_scene(obstacle_scene_path(REF), default_model_path(REF))
    k = len(ms.body_name) - len(mr.body_name) + 1   # robot bodies come after world + 38 obstacles
    np.testing.assert_allclose(ms.body_mass[k:], mr.body_mass[1:])
    np.testing.assert_allclose(ms.body_inertia[k:], mr.body_inertia[1:])
    np.testing.assert_allclose(ms.dof_invweight0, mr.dof_invweight0)
    assert ms.actuator_name == mr.actuator_name and ms.sensor_name == mr.sensor_name


def test_hull_features_match_oracle(scene):
    blob, h, o = scene
    tail = np.frombuffer(blob[h.hdr_bytes:], dtype=np.uint8)
    nv, nf = h.nmeshvert, h.nmeshface
    hv_all = np.frombuffer(tail[12 * nv + 12 * nf:].tobytes(), dtype="<f4").reshape(-1, 3)
    for k in range(h.nmesh):
        hv = hv_all[h.mesh_hulladr[k]: h.mesh_hulladr[k] + h.mesh_hullnum[k]]
        fn, ed = hull_features(hv)
        ofn, oed = o.hull_features(k)
        np.testing.assert_allclose(fn, ofn, atol=1e-12)
        np.testing.assert_allclose(ed, oed, atol=1e-12)
        # a thin plate: 2 caps + side faces; every face normal is a supporting direction
        proj = hv.astype(np.float64) @ fn.T
        assert np.all(proj <= proj.max(0) + 1e-9)


# ---------------------------------------------------------------- brute-force references
def _fib(n):
    i = np.arange(n) + 0.5
    phi, th = np.arccos(1 - 2 * i / n), np.pi * (1 + 5 ** 0.5) * i
    return np.stack([np.cos(th) * np.sin(phi), np.sin(th) * np.sin(phi), np.cos(phi)], 1)


class _Geo:
    def __init__(self):
        self.m = compile_scene(obstacle_scene_path(REF), default_model_path(REF))

    def pose(self, q, g):
        xp, xm, _, _, _ = body_frames(self.m, q)
        b = self.m.geom_bodyid[g]
        return xp[b] + xm[b] @ self.m.geom_pos[g], xm[b] @ quat_to_mat(self.m.geom_quat[g])

    def seps(self, q, g, gb, D):
        m = self.m
        c, R = self.pose(q, g)
        bc, bR = self.pose(q, gb)
        cb, rb = D @ bc, np.abs(D @ bR) @ m.geom_size[gb]
        if m.geom_type[g] == 5:
            an = D @ R[:, 2]
            r, hh = m.geom_size[g][:2]
            ext = hh * np.abs(an) + r * np.sqrt(np.maximum(0, 1 - an ** 2))
            lo, hi = D @ c - ext, D @ c + ext
        else:
            hv = m.meshes[m.geom_dataid[g]].hull_vert.astype(np.float64) @ R.T + c
            P = D @ hv.T
            lo, hi = P.min(1), P.max(1)
        return np.maximum((cb - rb) - hi, lo - (cb + rb))

    def true_sep(self, q, g, gb, rng, D):
        s = self.seps(q, g, gb, D)
        k = int(np.argmax(s))
        best, d = s[k], D[k]
        for scale in (0.02, 0.005, 0.001, 0.0002):
            C = d + scale * rng.normal(size=(3000, 3))
            C /= np.linalg.norm(C, axis=1, keepdims=True)
            s = self.seps(q, g, gb, C)
            k = int(np.argmax(s))
            if s[k] > best:
                best, d = s[k], C[k]
        return best


def _near_box_pose(m, rng, boxes):
    q = m.qpos0.copy()
    bc = m.geom_pos[rng.choice(boxes)]
    ang = rng.integers(4) * np.pi / 2
    dv = np.array([np.cos(ang), np.sin(ang)])
    q[:2] = bc[:2] + dv * (0.5 + rng.uniform(0.0, 0.2)) + rng.uniform(-0.5, 0.5) * np.array([-dv[1], dv[0]])
    q[2] = 0.065 + rng.uniform(-0.005, 0.01)
    q[3:7] = euler_to_quat(np.array([rng.normal(0, 0.05), rng.normal(0, 0.05), rng.uniform(0, 2 * np.pi)]))
    q[7:] = rng.normal(0, 0.3, 6)
    return q


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent")
def test_box_narrowphase_is_the_minimum_translation(scene):
    """Oracle box-cylinder / box-mesh contacts: same contact/no-contact decision as the exact
    separation, and (for penetrations up to 5 mm, the simulated regime) the same depth as a
    brute-force maximisation of the separation over all directions."""
    _, _, o = scene
    G = _Geo()
    m = G.m
    rng = np.random.default_rng(0)
    D = _fib(20000)
    boxes = [g for g in range(m.ngeom) if m.geom_type[g] == 6]
    robot = [g for g in range(m.ngeom) if m.geom_type[g] in (5, 7)]
    checked = {5: 0, 7: 0}
    for _ in range(120):
        q = _near_box_pose(m, rng, boxes)
        got = {(int(r[0]), int(r[1])): r for r in o.contacts(q)}
        for g in robot:
            c, _ = G.pose(q, g)
            for gb in boxes:
                if np.linalg.norm(c[:2] - m.geom_pos[gb][:2]) > 0.9:
                    continue
                key = (g, gb) if m.geom_type[g] == 5 else (gb, g)
                ts = G.true_sep(q, g, gb, rng, D)
                if abs(ts) < 1e-5:
                    continue   # grazing: either decision is within the search accuracy
                assert (key in got) == (ts < 0), (key, ts)
                if key in got and ts > -0.005:
                    r = got[key]
                    assert r[2] >= ts - 1e-5 and r[2] <= ts + 1e-4, (key, r[2], ts)
                    # the reported normal achieves the reported separation
                    assert abs(G.seps(q, g, gb, r[6:9][None])[0] - r[2]) < 1e-9
                    checked[m.geom_type[g]] += 1
    assert checked[5] >= 5 and checked[7] >= 5, checked


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent")
def test_ray_box_matches_slab_reference(scene):
    _, _, o = scene
    m = compile_scene(obstacle_scene_path(REF), default_model_path(REF))
    boxes = [g for g in range(m.ngeom) if m.geom_type[g] == 6]
    lo = np.array([m.geom_pos[g] - m.geom_size[g] for g in boxes])
    hi = np.array([m.geom_pos[g] + m.geom_size[g] for g in boxes])
    rng = np.random.default_rng(1)
    q = m.qpos0.copy()
    q[:3] = [30.0, 30.0, 5.0]   # robot far away: only floor and boxes can be hit
    hits = 0
    for _ in range(400):
        p = np.array([rng.uniform(-5, 4), rng.uniform(-5, 4), rng.uniform(0.02, 0.2)])
        v = rng.normal(size=3)
        v[2] *= 0.05
        v /= np.linalg.norm(v)
        with np.errstate(divide="ignore", invalid="ignore"):
            t1, t2 = (lo - p) / v, (hi - p) / v
        tn, tf = np.minimum(t1, t2).max(1), np.maximum(t1, t2).min(1)
        cand = np.where((tf >= tn) & (tf >= 0), np.where(tn >= 0, tn, tf), np.inf)
        tb = cand.min()
        tfl = -p[2] / v[2] if v[2] < 0 else np.inf
        if np.isfinite(tfl) and np.any(np.abs(p[:2] + tfl * v[:2]) > 40):
            tfl = np.inf   # the floor plane is a 40 x 40 rectangle
        ref = min(tb, tfl)
        got = o.ray(q, p, v)
        if np.isinf(ref):
            assert got == -1
        else:
            assert abs(got - ref) < 1e-9, (got, ref)
            hits += np.isfinite(tb) and tb < tfl
    assert hits > 100


def test_edge_family_kink_witness():
    """Oracle side of the edge-kink rule (tests/golden/edge_kink_state.npz): the wheel-box contact's
    normal is perpendicular to the wheel axis to rounding, so the witness is mid-rim (the cap-side
    tie), i.e. the contact point lies in the wheel's mid-plane."""
    import os
    from mujoco_playground_amd import _lib
    from mujoco_playground_amd.model import compiler as Cm
    from mujoco_playground_amd.model.mathutil import quat_to_mat
    from oracle.oracle import Oracle
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "edge_kink_state.npz"))
    c = Oracle(_lib.load_blob("obstacles")).contacts(d["before"][:13])
    box = c[(c[:, 0] >= 41) & (c[:, 1] < 41)]
    assert len(box) == 1
    n = box[0, 6:9]
    if not os.path.exists(Cm.obstacle_scene_path()):
        pytest.skip("reference MJCF not present")
    m = Cm.compile_scene(Cm.obstacle_scene_path(), Cm.default_model_path())
    xpos, xmat, _, _, _ = Cm.body_frames(m, d["before"][:13])
    g = int(box[0, 0])
    b = m.geom_bodyid[g]
    a = (xmat[b] @ quat_to_mat(m.geom_quat[g]))[:, 2]
    centre = xpos[b] + xmat[b] @ m.geom_pos[g]
    assert abs(a @ n) < 1e-9
    assert abs(a @ (box[0, 3:6] - centre)) < 1e-9   # mid-plane witness


def test_kink_snap_is_a_no_op_in_f64():
    """The kink snap (oracle edge_family / kernel cb_edge_family) is a deliberate departure from
    mj_collision: MuJoCo's general convex collider has no such rule; it exists because the kernel's
    f32 edge search is rounding-limited at the kink (|dqvel| 0.18 on the recorded state before it).
    It must not change the oracle's own f64 answer: with the snap off, the f64 search gives the same
    contacts (pairs, depth, normal, point) on the recorded state to 1e-9, so the rule cannot hide a
    discrepancy of the f64 restatement -- it only pulls the f32 kernel onto the answer the f64 search
    finds by itself."""
    import os
    from mujoco_playground_amd import _lib
    from oracle.oracle import Oracle, lib
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "edge_kink_state.npz"))
    o = Oracle(_lib.load_blob("obstacles"))
    on = o.contacts(d["before"][:13])
    lib().or_set_kink_snap(0)
    try:
        off = o.contacts(d["before"][:13])
    finally:
        lib().or_set_kink_snap(1)
    assert on.shape == off.shape and ((on[:, 0] >= 41) & (on[:, 1] < 41)).sum() == 1   # the wheel-box contact
    np.testing.assert_array_equal(on[:, :2], off[:, :2])
    np.testing.assert_allclose(on[:, 2:15], off[:, 2:15], rtol=0, atol=1e-9)
