"""GPU parity of the obstacle scene (the v2 robot in the flat obstacle world)
against the f64 CPU oracle: reset (spawn + goals), lidar against boxes at poses spread over the
maze, and teacher-forced steps of robots driven into box walls and corners.

Tolerances as tests/test_gpu_parity.py (|dqpos| <= 1e-5, |dqvel| <= 1e-3, obs <= 1e-4 abs +
1e-5 rel, reward <= 1e-4). Discontinuities the f32 kernel may legitimately resolve differently
from the f64 oracle, each excused only when the oracle itself reproduces the GPU step from a
state within 1e-6 of the same one (an axis shift of the body, or a seeded random perturbation of
qpos/qvel at 1e-7 / 1e-6; counted, capped at 0.5 % of env-steps):
  * contact activation (a vertex / rim point within ~1e-7 m of a floor or box face);
  * pyramid-edge activation in the contact solve (measured: the oracle's own qvel jumps by
    3.5e-2 under 1e-7 perturbations of such a state);
  * the separating axis of a box contact at a near-tie between two axes (box corners);
Lidar rays grazing a box edge (hit point within 1e-5 m of the edge) may hit in one precision and
miss in the other, and so may a ray descending at ~1e-3 whose floor hit ~50 m out lies on the
edge of the finite floor rectangle (cutoff vs -1); such rays are identified geometrically and
excluded from the obs comparison (counted, capped at 0.1 % of rays).
"""
import numpy as np
import pytest
import torch

from conftest import f64_state

pytestmark = pytest.mark.gpu

TOL_QPOS, TOL_QVEL, TOL_OBS, TOL_REW = 1e-5, 1e-3, 1e-4, 1e-4
DEV = "cuda:0"
SHIFTS = [(ax, d) for d in (1e-7, -1e-7, 1e-6, -1e-6) for ax in (2, 0, 1)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def sblob():
    from mujoco_playground_amd import _lib
    return _lib.load_blob("obstacles")


@pytest.fixture(scope="module")
def boxes(sblob):
    from mujoco_playground_amd.model import blob as B
    h = B.unpack_header(sblob)
    g = [i for i in range(h.ngeom) if h.geom_type[i] == 6]
    c = np.array([list(h.geom_pos[i]) for i in g])
    s = np.array([list(h.geom_size[i]) for i in g])
    return c - s, c + s


def make_sim(n, **kw):
    from mujoco_playground_amd.sim import BatchedAckermannSim
    return BatchedAckermannSim(n, DEV, scene="obstacles", **kw)


def oracle(blob, **params):
    from oracle.oracle import Oracle
    o = Oracle(blob)
    if params:
        o.set_env_params(**params)
    return o


def _yaw_quat(yaw, roll=0.0, pitch=0.0):
    from mujoco_playground_amd.model.mathutil import euler_to_quat
    return euler_to_quat(np.array([roll, pitch, yaw]))


def wall_states(n, lo, hi, rng, gap=(0.19, 0.26), speed=0.25, clearance=0.185):
    """Robots in front of exposed box faces, heading into them (+-60 deg), moving at `speed`;
    every box at least `clearance` (the robot's bounding radius) from the chassis centre."""
    occ = {(round(x), round(y)) for x, y in 0.5 * (lo[:, :2] + hi[:, :2])}
    faces = []
    for b in range(len(lo)):
        cx, cy = 0.5 * (lo[b, :2] + hi[b, :2])
        for nx, ny in ((1, 0), (-1, 0), (0, 1), (0, -1)):
            if (round(cx + nx), round(cy + ny)) not in occ:
                faces.append((cx, cy, nx, ny))
    st = np.zeros((n, 44))
    for e in range(n):
        while True:
            cx, cy, nx, ny = faces[rng.integers(len(faces))]
            t = rng.uniform(-0.55, 0.55)   # beyond +-0.5: the robot meets the box corner
            d = 0.5 + rng.uniform(*gap)
            x, y = cx + nx * d - ny * t, cy + ny * d + nx * t
            ex = np.maximum(np.maximum(lo[:, 0] - x, x - hi[:, 0]), 0.0)
            ey = np.maximum(np.maximum(lo[:, 1] - y, y - hi[:, 1]), 0.0)
            if np.sqrt(ex * ex + ey * ey).min() >= clearance:
                break
        yaw = np.arctan2(-ny, -nx) + rng.uniform(-1.0, 1.0)
        st[e, 0:3] = [x, y, 0.0649]
        st[e, 3:7] = _yaw_quat(yaw)
        st[e, 13:15] = -speed * np.array([nx, ny])
        st[e, 37:39] = [3.0, 1.0]   # odometry frame (relative to the episode start)
        st[e, 39:42] = [x, y, 0.0649]
        st[e, 43] = 1
    return st


def to_device(st):
    s = st.astype(np.float32)
    s[:, 42] = st[:, 42].astype(np.uint32).view(np.float32)
    s[:, 43] = st[:, 43].astype(np.uint32).view(np.float32)
    return torch.tensor(s.T.copy(), device=DEV)


def _excused(o, before_e, act_e, after_e, flags, seed):
    """The oracle reproduces the GPU step from a state within 1e-6 of `before_e`: axis shifts of
    the body, then seeded random perturbations of qpos/qvel at 1e-7 and 1e-6 (an activation
    boundary of a contact, pyramid edge or separating axis lies that close)."""
    def ok(s):
        o.step(s, act_e[None], flags=flags, seed=seed)
        return (np.abs(after_e[:13] - s[0, :13]).max() <= TOL_QPOS and
                np.abs(after_e[13:25] - s[0, 13:25]).max() <= TOL_QVEL)
    for ax, dz in SHIFTS:
        s = before_e[None].copy()
        s[0, ax] += dz
        if ok(s):
            return True
    rng = np.random.default_rng(1234)
    for scale in (1e-7, 1e-6):
        for _ in range(64):
            s = before_e[None].copy()
            s[0, :25] += rng.normal(0.0, scale, 25)
            if ok(s):
                return True
    return False


def _lidar_geometry():
    """RAY_ORG / RAY_DIR / RAY_Z (chassis frame) from the generated model header."""
    import os
    import re
    txt = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mujoco_playground_amd",
                            "csrc", "ackphys_model_gen.h")).read()

    def arr(name):
        body = re.search(name + r"\[72\]\[2\] = \{(.*?)\};", txt, re.S).group(1)
        return np.array([float(x.rstrip("f")) for x in re.findall(r"[-+0-9.e]+f", body)]).reshape(72, 2)
    z = float(re.search(r"RAY_Z = ([-+0-9.e]+)f", txt).group(1))
    return arr("RAY_ORG"), arr("RAY_DIR"), z


_LID = None


def _grazing(before_e, ray, lo, hi):
    """True if lidar ray `ray` of the pre-step pose passes within ~1e-4 m of a box edge
    (entry and exit of some box's slab intersection nearly coincide)."""
    global _LID
    from mujoco_playground_amd.model.mathutil import quat_to_mat
    if _LID is None:
        _LID = _lidar_geometry()
    org_c, dir_c, rz = _LID
    R = quat_to_mat(before_e[3:7] / np.linalg.norm(before_e[3:7]))
    org = before_e[:3] + R @ np.array([org_c[ray, 0], org_c[ray, 1], rz])
    d = R @ np.array([dir_c[ray, 0], dir_c[ray, 1], 0.0])
    for b in range(len(lo)):
        with np.errstate(divide="ignore", invalid="ignore"):
            t1, t2 = (lo[b] - org) / d, (hi[b] - org) / d
        tn, tf = np.nanmax(np.minimum(t1, t2)), np.nanmin(np.maximum(t1, t2))
        if tf >= 0 and abs(tn - tf) <= 1e-4:
            return True
    return False


def _floor_edge(state_e, ray, g, r):
    """True if the readings are the cutoff and -1 and ray `ray` meets the floor plane within 1e-3 of
    its length from the edge of the finite floor rectangle (mj_ray's plane test: inside -> a hit
    beyond the cutoff, clamped; outside -> no hit); the f32 hit point is that uncertain when the
    ray descends at ~1e-3 and meets the plane ~50 m out."""
    import os
    import re
    from mujoco_playground_amd.model.mathutil import quat_to_mat
    pair = sorted((float(g), float(r)))
    if not (abs(pair[0] + 1.0) <= 1e-6 and abs(pair[1] - 12.0) <= 1e-4):
        return False
    txt = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mujoco_playground_amd",
                            "csrc", "ackphys_model_gen.h")).read()
    half = [float(x.rstrip("f")) for x in
            re.findall(r"[-+0-9.e]+f", re.search(r"FLOOR_SIZE\[2\] = \{(.*?)\};", txt).group(1))]
    org_c, dir_c, rz = _lidar_geometry()
    R = quat_to_mat(state_e[3:7] / np.linalg.norm(state_e[3:7]))
    org = state_e[:3] + R @ np.array([org_c[ray, 0], org_c[ray, 1], rz])
    d = R @ np.array([dir_c[ray, 0], dir_c[ray, 1], 0.0])
    if d[2] >= 0:
        return False
    t = -org[2] / d[2]
    hit = org + t * d
    return min(abs(abs(hit[0]) - half[0]), abs(abs(hit[1]) - half[1])) <= 1e-3 * t and \
        abs(hit[0]) <= half[0] + 1e-3 * t and abs(hit[1]) <= half[1] + 1e-3 * t


def _ray_dir(state_e, ray, dir_c=None):
    from mujoco_playground_amd.model.mathutil import quat_to_mat
    if dir_c is None:
        dir_c = _lidar_geometry()[1]
    R = quat_to_mat(state_e[3:7] / np.linalg.norm(state_e[3:7]))
    return R @ np.array([dir_c[ray, 0], dir_c[ray, 1], 0.0])


HORIZ_TOL = 1e-6   # |dir_z| of a ray horizontal to rounding (the pose's f32 - f64 difference)


def _horizontal(before_e, ray, g, r):
    """True if ray `ray` is horizontal in the world to rounding (|dir_z| <= 1e-6) and the two
    readings are the rangefinder cutoff (a floor hit arbitrarily far away, clamped) and -1 (no
    hit): which one a ray gets is decided by the last bit of the pose (as in test_gpu_parity)."""
    global _LID
    from mujoco_playground_amd.model.mathutil import quat_to_mat
    if _LID is None:
        _LID = _lidar_geometry()
    _, dir_c, _ = _LID
    d = _ray_dir(before_e, ray, dir_c)
    pair = sorted((float(g), float(r)))
    return abs(d[2]) <= HORIZ_TOL * np.linalg.norm(d) and abs(pair[0] + 1.0) <= 1e-6 and abs(pair[1] - 12.0) <= 1e-4


def teacher_forced(sim, o, acts, steps, flags, seed, lo, hi, obs_pose=None, excuse=None, on_step=None):
    """obs_pose(before, actions) -> the states the observations are taken at (default: `before`, the
    pre-integration pose; with action_repeat R, the pose after R-1 mj_steps). excuse(k, e, before_e,
    act_e, after_e) replaces the boundary excuse (default: _excused with the oracle `o`).
    on_step(k, ref, after, ok, oterm, otr, tobs): extra per-step checks."""
    worst = dict(qpos=0.0, qvel=0.0, obs=0.0, rew=0.0, excused=0, grazing_rays=0, rays=0)
    for k in range(steps):
        before = f64_state(sim.state)
        seen = before if obs_pose is None else obs_pose(before, acts[k].cpu().numpy())
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
            ex = (excuse(k, e, before[e], a_np[e], after[e]) if excuse is not None
                  else _excused(o, before[e], a_np[e], after[e], flags, seed))
            assert ex, (
                f"step {k} env {e}: |dqpos| {dq[e]:.3e} |dqvel| {dv[e]:.3e}")
            worst["excused"] += 1
        worst["qpos"] = max(worst["qpos"], dq[ok].max(initial=0.0))
        worst["qvel"] = max(worst["qvel"], dv[ok].max(initial=0.0))
        # observations of the pre-step pose (rays 10..71 observed; 0..9 alias ray 71)
        gobs = sim.obs_soa.cpu().numpy().T
        do = np.abs(gobs - oobs) / (1.0 + 0.1 * np.abs(oobs))
        bad_ray = do[:, :72] > TOL_OBS
        if obs_pose is not None:  # the observed pose then depends on the step's own (excused) dynamics
            bad_ray &= ok[:, None]
        for e, i in zip(*np.nonzero(bad_ray)):
            ray = 71 if i < 10 else i
            assert (_grazing(seen[e], ray, lo, hi) or _horizontal(seen[e], ray, gobs[e, i], oobs[e, i]) or
                    _floor_edge(seen[e], ray, gobs[e, i], oobs[e, i])), (
                f"step {k} env {e} ray {i}: {gobs[e, i]} vs {oobs[e, i]} (dir {_ray_dir(seen[e], ray)})")
        graze_env = bad_ray.any(axis=1)
        worst["grazing_rays"] += int(bad_ray[:, 10:].sum())
        worst["rays"] += 62 * sim.n
        keep = ok & ~graze_env
        worst["obs"] = max(worst["obs"], do[keep].max(initial=0.0))
        assert do[keep].max(initial=0.0) <= TOL_OBS
        dr = np.abs(sim.reward.cpu().numpy() - orew)[keep].max(initial=0.0)
        worst["rew"] = max(worst["rew"], dr)
        assert dr <= TOL_REW
        np.testing.assert_array_equal(sim.term.cpu().numpy().astype(bool)[ok], oterm[ok])
        np.testing.assert_array_equal(sim.trunc.cpu().numpy().astype(bool)[ok], otr[ok])
        if on_step is not None:
            on_step(k, ref, after, ok, oterm, otr, tobs)
    assert worst["excused"] <= 5e-3 * steps * sim.n, worst
    assert worst["grazing_rays"] <= 1e-3 * worst["rays"], worst
    return worst


def test_obstacle_reset_matches_oracle(sblob):
    n = 300
    sim = make_sim(n, seed=7)
    sim.reset()
    torch.cuda.synchronize()
    o = oracle(sblob)
    st = np.zeros((n, 44))
    oobs = o.reset(st, seed=7)
    g = f64_state(sim.state)
    np.testing.assert_allclose(g[:, :37], st[:, :37], atol=1e-7)
    assert np.allclose(g[:, 0:3], [-2.9, -3.3, 0.1], atol=1e-6)
    np.testing.assert_allclose(g[:, 37:39], st[:, 37:39], atol=1e-5)
    np.testing.assert_array_equal(g[:, 42:44], st[:, 42:44])
    np.testing.assert_allclose(sim.obs_soa.cpu().numpy().T, oobs, atol=1e-5)
    # the spawn cell is walled: several rays hit boxes within 1.5 m
    assert (oobs[:, 10:72] > 0).all() and (oobs[0, 10:72] < 1.5).sum() >= 5


def test_obstacle_lidar_over_the_maze(sblob, boxes):
    """Rays at random poses all over the maze (mostly box hits; DDA vs brute force)."""
    lo, hi = boxes
    rng = np.random.default_rng(3)
    n = 1024
    st = np.zeros((n, 44))
    st[:, 0] = rng.uniform(-5.0, 4.0, n)
    st[:, 1] = rng.uniform(-5.0, 4.0, n)
    st[:, 2] = 0.0649 + rng.uniform(-0.003, 0.02, n)
    for e in range(n):
        st[e, 3:7] = _yaw_quat(rng.uniform(0, 2 * np.pi), rng.normal(0, 0.02), rng.normal(0, 0.02))
    st[:, 37:39] = rng.uniform(-6, 6, (n, 2))
    st[:, 43] = 1
    sim = make_sim(n, seed=1, contacts=False)   # some poses overlap boxes: rays only
    sim.set_state(to_device(st))
    acts = [torch.zeros(n, 2, device=DEV)]
    w = teacher_forced(sim, oracle(sblob), acts, 1, 0, 1, lo, hi)
    print("lidar", w)


def test_obstacle_wall_contacts(sblob, boxes):
    """Robots driven into exposed box faces and corners: box contacts on wheels and plates."""
    lo, hi = boxes
    rng = np.random.default_rng(5)
    n, steps = 512, 120
    st = wall_states(n, lo, hi, rng)
    sim = make_sim(n, seed=5)
    sim.set_state(to_device(st))
    gen = torch.Generator(device="cpu").manual_seed(5)
    acts = []
    for _ in range(steps):
        a = torch.rand(n, 2, generator=gen) * 2 - 1
        a[:, 0] = 0.4 + 0.6 * torch.rand(n, generator=gen)   # keep pushing forward
        acts.append(a.to(DEV))
    o = oracle(sblob)
    w = teacher_forced(sim, o, acts, steps, 1 | 2, 5, lo, hi)
    print("walls", w)
    # box contacts really happened: count them in the final oracle states
    fin = f64_state(sim.state)
    nbox = 0
    for e in range(0, n, 4):
        c = o.contacts(fin[e, :13])
        nbox += int(((c[:, 0] > 0) & (c[:, 2] < 0)).sum())
    assert nbox >= 20, nbox


def test_wheel_on_box_edge_kink(sblob):
    """A recorded state (tests/golden/edge_kink_state.npz, from the action-repeat parity run): a front
    wheel's rim pressed on a vertical box edge, wheels spinning. The best separating direction is the
    kink of the edge family (n = a x e_z, a.n = 0), where the witness sits mid-rim; the f32 search had
    landed ~5e-5 rad off it, flipped the cap-side tie and moved the contact point by the half-width
    (|dqvel| 0.18 against the oracle). Both sides now snap to the kink (cb_edge_family / edge_family)."""
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "edge_kink_state.npz"))
    before, action = d["before"], d["action"].reshape(1, 2)
    o = oracle(sblob)
    c = o.contacts(before[:13])
    box = c[(c[:, 0] >= 41) & (c[:, 1] < 41)]   # wheel (41-44) vs box
    assert len(box) == 1 and abs(box[0, 2]) > 1e-4   # one wheel-box contact, 0.45 mm deep
    ref = before[None].copy()
    o.step(ref, action, flags=1, seed=9)
    for variant_n in (1, 37):   # alone, and inside a wave of other envs
        sim = make_sim(variant_n, seed=9)
        st = np.repeat(before[None], variant_n, axis=0)
        sim.set_state(to_device(st))
        sim.step(torch.tensor(np.repeat(action, variant_n, axis=0), device=DEV), autoreset=False)
        torch.cuda.synchronize()
        after = f64_state(sim.state)
        assert np.abs(after[:, :13] - ref[0, :13]).max() <= TOL_QPOS
        assert np.abs(after[:, 13:25] - ref[0, 13:25]).max() <= TOL_QVEL
