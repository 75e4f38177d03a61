"""Emit `csrc/ackphys_model_gen.h`: the compiled Ackermann model as constexpr constants the
HIP kernels are specialised on.

The kernels work in CHASSIS-FRAME coordinates u = (v_b, w_b, qdot_hinges), v_b = R^T v_world.
In those coordinates every body's centre of mass is fixed (the wheel and steer bodies have
their CoM on their joint axes) and the wheel/steer inertias are isotropic, so the whole-robot
composite inertia about the chassis origin is CONSTANT; only the front spin axes depend on
the steer angles. This file checks every assumption that makes that true and refuses to
generate otherwise (so a different MJCF cannot silently run on kernels that do not fit it).

Model facts used (ackermann_robot_v2.xml): chassis free joint (:25-26); base/ceiling meshes
welded to the chassis (:28-36); rear wheels hinge-y (:39-52); front steer hinge-z + wheel
hinge-y (:55-80); lidar ring of 72 sites (:82-87); equality (:106-109); actuators (:111-123).
"""
from __future__ import annotations

import numpy as np

from .compiler import (ACT_POSITION, ACT_VELOCITY, GEOM_BOX, GEOM_CYLINDER, GEOM_MESH, GEOM_PLANE, JNT_FREE,
                       JNT_HINGE, CompiledModel)
from .mathutil import quat_to_mat


class ModelMismatch(ValueError):
    pass


def _req(cond, msg):
    if not cond:
        raise ModelMismatch(msg)


def _f(x) -> str:
    return f"{float(np.float32(x)):.9e}f"


def _d(x) -> str:
    return f"{float(x):.17e}"


def _arr(name, a, ty="float"):
    a = np.asarray(a, dtype=np.float64)
    fmt = _f if ty == "float" else _d
    if a.ndim == 1:
        body = ", ".join(fmt(v) for v in a)
        return f"constexpr {ty} {name}[{a.shape[0]}] = {{{body}}};"
    rows = ",\n    ".join("{" + ", ".join(fmt(v) for v in r) + "}" for r in a.reshape(a.shape[0], -1))
    dims = "".join(f"[{d}]" for d in a.shape)
    return f"constexpr {ty} {name}{dims} = {{\n    {rows}}};"


def analyse(m: CompiledModel) -> dict:
    """Derive the chassis-frame constants; raise ModelMismatch if the model does not fit."""
    _req(m.nq == 13 and m.nv == 12 and m.njnt == 7, "expected nq=13 nv=12 njnt=7")
    bid = {n: i for i, n in enumerate(m.body_name)}
    _req("chassis" in bid and m.jnt_type[0] == JNT_FREE and m.jnt_bodyid[0] == bid["chassis"],
         "joint 0 must be the chassis free joint")
    _req(all(t == JNT_HINGE for t in m.jnt_type[1:]), "joints 1..6 must be hinges")
    for n in ["chassis", "base", "ceiling", "rear_left", "rear_right", "front_left_steer", "front_left",
              "front_right_steer", "front_right", "lidar_360"]:
        _req(n in bid, f"body {n} missing")
    ch = bid["chassis"]
    # group G: every body welded to the chassis
    G = [b for b in range(1, m.nbody) if m.body_weldid[b] == ch]
    for b in G:
        _req(m.body_parentid[b] == ch or b == ch, "welded bodies must be direct chassis children")
    # chassis-frame poses of welded bodies (qpos0 config, which is also any config: rigid)
    def child_frame(b):
        if b == ch:
            return np.zeros(3), np.eye(3)
        return m.body_pos[b].copy(), quat_to_mat(m.body_quat[b])

    mG, sG = 0.0, np.zeros(3)
    for b in G:
        p, R = child_frame(b)
        ci = p + R @ m.body_ipos[b]
        mG += m.body_mass[b]
        sG += m.body_mass[b] * ci
    cG = sG / mG
    IG = np.zeros((3, 3))
    for b in G:
        p, R = child_frame(b)
        ci = p + R @ m.body_ipos[b]
        Ri = R @ quat_to_mat(m.body_iquat[b])
        Ic = Ri @ np.diag(m.body_inertia[b]) @ Ri.T
        r = ci - cG
        IG += Ic + m.body_mass[b] * (np.dot(r, r) * np.eye(3) - np.outer(r, r))
    # wheel chains
    wheels = [("rear_left", None), ("rear_right", None), ("front_left", "front_left_steer"),
              ("front_right", "front_right_steer")]
    W = []
    for wn, sn in wheels:
        wb = bid[wn]
        info = {}
        if sn is None:
            _req(m.body_parentid[wb] == ch, f"{wn} must hang from the chassis")
            anchor = m.body_pos[wb].copy()
            _req(np.allclose(m.body_quat[wb], [1, 0, 0, 0]), f"{wn}: identity body quat expected")
            info["steer_dof"] = -1
        else:
            sb = bid[sn]
            _req(m.body_parentid[sb] == ch and m.body_parentid[wb] == sb, f"{wn}/{sn} chain")
            _req(np.allclose(m.body_quat[sb], [1, 0, 0, 0]) and np.allclose(m.body_quat[wb], [1, 0, 0, 0]),
                 f"{sn}: identity quats expected")
            _req(np.allclose(m.body_pos[wb], 0), f"{wn} must sit at its steer body origin")
            anchor = m.body_pos[sb].copy()
            _req(m.body_jntnum[sb] == 1, f"{sn} has one hinge")
            sj = m.body_jntadr[sb]
            _req(np.allclose(m.jnt_pos[sj], 0), f"{sn}: hinge at the body origin")
            info["steer_dof"] = int(m.jnt_dofadr[sj])
            info["steer_qpos"] = int(m.jnt_qposadr[sj])
            info["steer_jnt"] = int(sj)
            info["steer_axis"] = m.jnt_axis[sj].copy()
            _req(np.allclose(m.body_ipos[sb], 0), f"{sn}: CoM on the joint axis")
            I = m.body_inertia[sb]
            _req(np.allclose(I, I[0]), f"{sn}: isotropic inertia required")
            info["steer_m"], info["steer_I"] = float(m.body_mass[sb]), float(I[0])
        _req(m.body_jntnum[wb] == 1, f"{wn} has one hinge")
        wj = m.body_jntadr[wb]
        _req(np.allclose(m.jnt_pos[wj], 0), f"{wn}: hinge at the body origin")
        _req(np.allclose(m.body_ipos[wb], 0), f"{wn}: CoM on the joint axis")
        I = m.body_inertia[wb]
        _req(np.allclose(I, I[0]), f"{wn}: isotropic inertia required")
        info.update(body=wb, anchor=anchor, m=float(m.body_mass[wb]), I=float(I[0]),
                    spin_dof=int(m.jnt_dofadr[wj]), spin_qpos=int(m.jnt_qposadr[wj]),
                    spin_axis=m.jnt_axis[wj].copy())
        # its cylinder geom
        gs = [g for g in range(m.ngeom) if m.geom_bodyid[g] == wb]
        _req(len(gs) == 1 and m.geom_type[gs[0]] == GEOM_CYLINDER, f"{wn}: one cylinder geom")
        g = gs[0]
        _req(np.allclose(m.geom_pos[g], 0), f"{wn}: cylinder centred on the hinge")
        gaxis = quat_to_mat(m.geom_quat[g])[:, 2]
        _req(abs(abs(np.dot(gaxis, info["spin_axis"])) - 1) < 1e-9, f"{wn}: cylinder axis = spin axis")
        info.update(geom=g, cyl_r=float(m.geom_size[g][0]), cyl_h=float(m.geom_size[g][1]),
                    cyl_axis=gaxis, friction=m.geom_friction[g].copy())
        W.append(info)
    # whole-robot composite about the chassis origin (chassis frame); constant, see module doc
    mt = mG
    st = mG * cG
    IO = IG + mG * (np.dot(cG, cG) * np.eye(3) - np.outer(cG, cG))
    for w in W:
        ms = w["m"] + w.get("steer_m", 0.0)
        Is = w["I"] + w.get("steer_I", 0.0)
        r = w["anchor"]
        mt += ms
        st += ms * r
        IO += Is * np.eye(3) + ms * (np.dot(r, r) * np.eye(3) - np.outer(r, r))
    ct = st / mt
    # floor
    fl = [g for g in range(m.ngeom) if m.geom_type[g] == GEOM_PLANE]
    _req(len(fl) == 1 and m.geom_bodyid[fl[0]] == 0, "one world floor plane")
    f = fl[0]
    _req(np.allclose(m.geom_pos[f], 0) and np.allclose(m.geom_quat[f], [1, 0, 0, 0]), "floor at the origin")
    # meshes (welded plates): hull vertices in the chassis frame
    meshes = []
    for g in range(m.ngeom):
        if m.geom_type[g] != GEOM_MESH:
            continue
        b = m.geom_bodyid[g]
        _req(b in G, "mesh geoms must be welded to the chassis")
        p, R = child_frame(b)
        gp = p + R @ m.geom_pos[g]
        gR = R @ quat_to_mat(m.geom_quat[g])
        mh = m.meshes[m.geom_dataid[g]]
        hv = (gR @ mh.hull_vert.astype(np.float64).T).T + gp
        vv = (gR @ mh.vert.astype(np.float64).T).T + gp
        meshes.append(dict(geom=g, body=int(b), hull=hv, lo=vv.min(0), hi=vv.max(0),
                           friction=np.maximum(m.geom_friction[g], m.geom_friction[f])))
    # static obstacle boxes (obstacle scene): world-welded, axis-aligned
    boxes = [g for g in range(m.ngeom) if m.geom_type[g] == GEOM_BOX]
    for g in boxes:
        _req(m.body_weldid[m.geom_bodyid[g]] == 0, "boxes must be static (welded to the world)")
        bq = quat_to_mat(m.geom_quat[g])
        b = m.geom_bodyid[g]
        _req(b == 0 or (np.allclose(m.body_quat[b], [1, 0, 0, 0]) and m.body_parentid[b] == 0),
             "static box bodies hang from the world unrotated")
        _req(np.allclose(bq, np.eye(3)), "boxes must be axis-aligned")
    _req(all(m.geom_type[g] in (GEOM_PLANE, GEOM_BOX, GEOM_CYLINDER, GEOM_MESH) for g in range(m.ngeom)),
         "geom types: plane, box, cylinder, mesh")
    # contact collision filter must give exactly the floor pairs (+ box pairs)
    for g1 in range(m.ngeom):
        for g2 in range(g1 + 1, m.ngeom):
            b1, b2 = m.geom_bodyid[g1], m.geom_bodyid[g2]
            w1, w2 = m.body_weldid[b1], m.body_weldid[b2]
            ok = (m.geom_contype[g1] & m.geom_conaffinity[g2]) or (m.geom_contype[g2] & m.geom_conaffinity[g1])
            pw1 = m.body_weldid[m.body_parentid[w1]]
            pw2 = m.body_weldid[m.body_parentid[w2]]
            filt = w1 == w2 or (w1 and w2 and (w1 == pw2 or w2 == pw1))
            active = ok and not filt
            wset = [f] + boxes
            world_pair = (g1 in wset) != (g2 in wset)   # world geom vs robot geom
            _req(active == world_pair, f"unexpected collision pair {g1},{g2}")
    # lidar: 72 rangefinders on sites welded to the chassis
    lid = [s for s in range(len(m.sensor_name)) if m.sensor_type[s] == 2]
    _req(len(lid) == 72, "72 rangefinders")
    org, dirs = [], []
    for s in lid:
        site = m.sensor_objid[s]
        b = m.site_bodyid[site]
        _req(b in G, "lidar sites welded to the chassis")
        p, R = child_frame(b)
        org.append(p + R @ m.site_pos[site])
        dirs.append((R @ quat_to_mat(m.site_quat[site]))[:, 2])
    org, dirs = np.array(org), np.array(dirs)
    # rays are horizontal in the chassis frame at height h; every robot geom lies strictly below
    # -> in ANY state the robot cannot occlude its own lidar; only the floor is tested on GPU.
    _req(np.allclose(dirs[:, 2], 0, atol=1e-12), "lidar rays must be horizontal in the chassis frame")
    hray = float(org[:, 2].min())
    _req(np.allclose(org[:, 2], hray), "lidar rays share one height")
    for w in W:
        top = w["anchor"][2] + np.hypot(w["cyl_r"], w["cyl_h"])
        _req(top < hray, "wheel could occlude lidar")
    for mh in meshes:
        _req(mh["hi"][2] < hray, "mesh could occlude lidar")
    # equality
    # robot collision geoms (wheels + meshes) share one contact solref/solimp with floor and boxes
    coll = [f] + boxes + [w["geom"] for w in W] + [mh["geom"] for mh in meshes]
    _req(np.allclose(m.geom_solref[coll], m.geom_solref[f]), "uniform contact solref")
    _req(np.allclose(m.geom_solimp[coll], m.geom_solimp[f]), "uniform contact solimp")
    _req(np.allclose(m.geom_solmix[coll], m.geom_solmix[f]), "uniform solmix")
    for g in boxes:   # wheel-box / mesh-box friction = wheel-floor / mesh-floor (max mix)
        for w in W:
            _req(np.allclose(np.maximum(w["friction"], m.geom_friction[g]),
                             np.maximum(w["friction"], m.geom_friction[f])), "box friction = floor friction")
        for mh in meshes:
            _req(np.allclose(np.maximum(m.geom_friction[mh["geom"]], m.geom_friction[g]), mh["friction"]),
                 "box friction = floor friction (meshes)")
    _req(m.neq == 1 and m.eq_obj2id[0] >= 0, "one joint-joint equality")
    # actuators
    _req(m.nu == 3, "three actuators")
    _req(m.actuator_type[0] == ACT_POSITION and m.actuator_type[1] == ACT_VELOCITY
         and m.actuator_type[2] == ACT_VELOCITY, "servo + two velocity drives")
    _req(np.allclose(m.actuator_gear, 1), "unit gears")
    chassis_R = {b: child_frame(b) for b in G}
    return dict(mG=mG, cG=cG, IG=IG, mt=mt, ct=ct, IO=IO, W=W, meshes=meshes, floor=f, lid=lid, org=org,
                dirs=dirs, hray=hray, boxes=boxes, child_frame=chassis_R)


def generate(m: CompiledModel, blob_fnv: int) -> str:
    A = analyse(m)
    L = []
    L.append("// GENERATED by mujoco_playground_amd/model/codegen.py -- do not edit.")
    L.append("// Compiled ackermann_robot_v2 model constants (chassis-frame specialisation).")
    L.append("#pragma once")
    L.append("#include <stdint.h>")
    L.append("namespace apg {")
    L.append(f"constexpr uint64_t MODEL_FNV = 0x{blob_fnv:016x}ull;")
    _req(np.allclose(m.geom_solref[A["floor"]], m.dof_solref[0])
         and np.allclose(m.geom_solimp[A["floor"]], m.dof_solimp[0]),
         "robot model: contact and joint solver parameters coincide (scene headers carry their own)")
    _req(not A["boxes"], "the robot header is generated from the obstacle-free model")
    L += _robot_lines(m, A)
    L.append("}  // namespace apg")
    return "\n".join(L) + "\n"


def _robot_lines(m: CompiledModel, A: dict) -> list:
    """Every robot constant the kernels use (identical for the robot alone and for the robot
    merged into a scene -- generate_scene() checks exactly that)."""
    W = A["W"]
    L = []
    L.append(f"constexpr float DT = {_f(m.timestep)};")
    L.append(_arr("GRAV", m.gravity))
    L.append(f"constexpr float MEANINERTIA = {_f(m.meaninertia)};")
    L.append(f"constexpr float IMPRATIO = {_f(m.impratio)};")
    L.append(f"constexpr float M_TOT = {_f(A['mt'])};")
    L.append(_arr("C_TOT", A["ct"]))
    L.append(_arr("I_O", A["IO"]))
    L.append(f"constexpr float M_G = {_f(A['mG'])};")
    L.append(_arr("C_G", A["cG"]))
    L.append(_arr("I_G", A["IG"]))
    # wheels
    L.append(_arr("W_ANCHOR", [w["anchor"] for w in W]))
    L.append(_arr("W_M", [w["m"] for w in W]))
    L.append(_arr("W_I", [w["I"] for w in W]))
    L.append(_arr("W_SPIN_AXIS", [w["spin_axis"] for w in W]))
    L.append(_arr("W_CYL_AXIS", [w["cyl_axis"] for w in W]))
    L.append(f"constexpr float CYL_R = {_f(W[0]['cyl_r'])};")
    L.append(f"constexpr float CYL_H = {_f(W[0]['cyl_h'])};")
    for w in W[1:]:
        _req(abs(w["cyl_r"] - W[0]["cyl_r"]) < 1e-12 and abs(w["cyl_h"] - W[0]["cyl_h"]) < 1e-12, "equal wheels")
    L.append("constexpr int W_SPIN_DOF[4] = {" + ", ".join(str(w["spin_dof"]) for w in W) + "};")
    L.append("constexpr int W_SPIN_QPOS[4] = {" + ", ".join(str(w["spin_qpos"]) for w in W) + "};")
    L.append("constexpr int W_STEER_DOF[4] = {" + ", ".join(str(w["steer_dof"]) for w in W) + "};")
    L.append("constexpr int W_STEER_QPOS[4] = {" + ", ".join(str(w.get("steer_qpos", -1)) for w in W) + "};")
    L.append(_arr("S_AXIS", [W[2]["steer_axis"], W[3]["steer_axis"]]))
    L.append(_arr("S_M", [W[2]["steer_m"], W[3]["steer_m"]]))
    L.append(_arr("S_I", [W[2]["steer_I"], W[3]["steer_I"]]))
    # friction of wheel-floor contacts (max mix) and body invweights (tran) of wheel bodies
    f = A["floor"]
    mu_w = np.maximum(W[0]["friction"], m.geom_friction[f])
    for w in W:
        _req(np.allclose(np.maximum(w["friction"], m.geom_friction[f]), mu_w), "equal wheel friction")
    L.append(f"constexpr float MU_WHEEL = {_f(mu_w[0])};")
    L.append(_arr("W_TRAN", [m.body_invweight0[w["body"]][0] for w in W]))
    # meshes
    Ms = A["meshes"]
    nh = max(len(mh["hull"]) for mh in Ms)
    L.append(f"constexpr int NMESH = {len(Ms)};")
    L.append(f"constexpr int NHULL = {nh};")
    hull = np.zeros((len(Ms), nh, 3))
    hvalid = []
    for k, mh in enumerate(Ms):
        hull[k, : len(mh["hull"])] = mh["hull"]
        hull[k, len(mh["hull"]):] = mh["hull"][0]   # pad by repeating a vertex (harmless duplicate)
        hvalid.append(len(mh["hull"]))
    L.append(_arr("HULL", hull))
    L.append("constexpr int HULL_N[" + str(len(Ms)) + "] = {" + ", ".join(map(str, hvalid)) + "};")
    L.append(_arr("HULL_LO", [mh["hull"].min(0) for mh in Ms]))
    L.append(_arr("HULL_HI", [mh["hull"].max(0) for mh in Ms]))
    L.append(_arr("MESH_MU", [mh["friction"][0] for mh in Ms]))
    L.append(_arr("MESH_TRAN", [m.body_invweight0[mh["body"]][0] for mh in Ms]))
    # dofs
    L.append(_arr("ARMATURE", m.dof_armature))
    L.append(_arr("DAMPING", m.dof_damping))
    L.append(_arr("FRICTIONLOSS", m.dof_frictionloss))
    L.append(_arr("DOF_INVW", m.dof_invweight0))
    # solver params: joint/dof/equality rows share one solref/solimp (asserted); contacts use the
    # collision geoms' (analyse() asserts those uniform). In ackermann_robot_v2 both are defaults.
    for arr in [m.dof_solref, m.jnt_solref, m.eq_solref]:
        _req(np.allclose(arr, m.dof_solref[0]), "uniform solref")
    for arr in [m.dof_solimp, m.jnt_solimp, m.eq_solimp]:
        _req(np.allclose(arr, m.dof_solimp[0]), "uniform solimp")
    _req(np.all(m.geom_margin == 0) and np.all(m.geom_gap == 0) and np.all(m.jnt_margin == 0), "zero margins")
    _req(np.all(m.geom_condim == 3), "condim 3")
    L.append(_arr("SOLREF", m.dof_solref[0]))
    L.append(_arr("SOLIMP", m.dof_solimp[0]))
    # equality
    e1, e2 = int(m.eq_obj1id[0]), int(m.eq_obj2id[0])
    L.append(f"constexpr int EQ_DOF1 = {int(m.jnt_dofadr[e1])}, EQ_DOF2 = {int(m.jnt_dofadr[e2])};")
    L.append(f"constexpr int EQ_QPOS1 = {int(m.jnt_qposadr[e1])}, EQ_QPOS2 = {int(m.jnt_qposadr[e2])};")
    L.append(_arr("EQ_POLY", m.eq_polycoef[0]))
    # limits: steer joints
    lims = [j for j in range(m.njnt) if m.jnt_limited[j]]
    _req(len(lims) == 2, "two limited joints (steer)")
    L.append("constexpr int LIM_DOF[2] = {" + ", ".join(str(int(m.jnt_dofadr[j])) for j in lims) + "};")
    L.append("constexpr int LIM_QPOS[2] = {" + ", ".join(str(int(m.jnt_qposadr[j])) for j in lims) + "};")
    L.append(_arr("LIM_RANGE", [m.jnt_range[j] for j in lims]))
    # actuators
    L.append(f"constexpr int ACT_STEER_DOF = {int(m.jnt_dofadr[m.actuator_trnid[0]])};")
    L.append(f"constexpr int ACT_STEER_QPOS = {int(m.jnt_qposadr[m.actuator_trnid[0]])};")
    L.append(f"constexpr int ACT_RL_DOF = {int(m.jnt_dofadr[m.actuator_trnid[1]])};")
    L.append(f"constexpr int ACT_RR_DOF = {int(m.jnt_dofadr[m.actuator_trnid[2]])};")
    L.append(_arr("ACT_GAIN", m.actuator_gainprm[:, 0]))
    L.append(_arr("ACT_BIAS1", m.actuator_biasprm[:, 1]))
    L.append(_arr("ACT_BIAS2", m.actuator_biasprm[:, 2]))
    L.append(_arr("ACT_CTRLRANGE", m.actuator_ctrlrange))
    L.append("constexpr int ACT_CTRLLIMITED[3] = {" + ", ".join(map(str, m.actuator_ctrllimited)) + "};")
    L.append(_arr("ACT_FORCERANGE", m.actuator_forcerange))
    L.append("constexpr int ACT_FORCELIMITED[3] = {" + ", ".join(map(str, m.actuator_forcelimited)) + "};")
    # lidar (chassis frame) and floor rectangle
    L.append(f"constexpr float RAY_Z = {_f(A['hray'])};")
    L.append(_arr("RAY_ORG", A["org"][:, :2]))
    L.append(_arr("RAY_DIR", A["dirs"][:, :2]))
    L.append(f"constexpr float RAY_CUTOFF = {_f(m.sensor_cutoff[A['lid'][0]])};")
    L.append(_arr("FLOOR_SIZE", m.geom_size[f][:2]))
    L.append(_arr("QPOS0", m.qpos0))
    return L


def hull_features(hv: np.ndarray):
    """Unique outward face normals and unique edge directions of a convex hull given by its
    vertices -- the same enumeration, tolerances and order as hull_features() in
    oracle/ackphys_oracle.c, so both sides test the same separating axes in the same order."""
    v = hv.astype(np.float32).astype(np.float64)
    n = len(v)
    scale = float(np.abs(v).max()) if n else 1.0
    tol = 1e-9 * (scale if scale > 0 else 1.0)
    fn = []

    def add(arr, x, sign_free):
        for y in arr:
            d = float(np.dot(y, x))
            if d > 1 - 1e-9 or (sign_free and d < -1 + 1e-9):
                return
        arr.append(x)

    for i in range(n):
        for j in range(i + 1, n):
            e1 = v[j] - v[i]
            for k in range(j + 1, n):
                nn = np.cross(e1, v[k] - v[i])
                ln = float(np.sqrt(np.dot(nn, nn)))
                if ln < 1e-12 * scale * scale:
                    continue
                nn = nn / ln
                sd = v @ nn - float(np.dot(nn, v[i]))
                above, below = int((sd > tol).sum()), int((sd < -tol).sum())
                if above and below:
                    continue
                if above:
                    nn = -nn
                add(fn, nn, False)
    off = [float((v @ f).max()) for f in fn]
    ed = []
    for i in range(n):
        for j in range(i + 1, n):
            e = v[j] - v[i]
            ln = float(np.sqrt(np.dot(e, e)))
            if ln < tol:
                continue
            on = sum(1 for f, o in zip(fn, off) if abs(np.dot(f, v[i]) - o) < tol and abs(np.dot(f, v[j]) - o) < tol)
            if on < 2:
                continue
            add(ed, e / ln, True)
    return np.array(fn), np.array(ed)


def maze_free_cells(cells, nx: int, ny: int, x0: float, y0: float, cell: float, spawn) -> list:
    """Free-cell goals of the opt-in maze task: (centre x, centre y, breadth-first distance in
    cells) of every box-free grid cell 4-connected to the spawn cell, the spawn cell excluded,
    sorted by distance, then row, then column."""
    sx, sy = int(np.floor((spawn[0] - x0) / cell)), int(np.floor((spawn[1] - y0) / cell))
    _req(0 <= sx < nx and 0 <= sy < ny and not cells[sy * nx + sx], "spawn in a free grid cell")
    dist = {(sx, sy): 0}
    todo = [(sx, sy)]
    for c in todo:  # breadth-first: `todo` grows while it is walked
        for dx, dy in ((1, 0), (-1, 0), (0, 1), (0, -1)):
            n = (c[0] + dx, c[1] + dy)
            if 0 <= n[0] < nx and 0 <= n[1] < ny and not cells[n[1] * nx + n[0]] and n not in dist:
                dist[n] = dist[c] + 1
                todo.append(n)
    out = [(x0 + (ix + 0.5) * cell, y0 + (iy + 0.5) * cell, d, iy, ix) for (ix, iy), d in dist.items() if d > 0]
    out.sort(key=lambda t: (t[2], t[3], t[4]))
    return [(x, y, d) for x, y, d, _, _ in out]


def generate_scene(ms: CompiledModel, blob_fnv: int, robot: CompiledModel, ns: str = "scene1") -> str:
    """Scene header: the static world the robot is merged into (obstacle scene). The robot part
    of `ms` must compile to exactly the robot header's constants."""
    A, Ar = analyse(ms), analyse(robot)
    _req(_robot_lines(ms, A) == _robot_lines(robot, Ar), "scene robot differs from the robot model")
    boxes = A["boxes"]
    _req(0 < len(boxes) <= 127, "1..127 boxes")
    lo = np.array([ms.geom_pos[g] - ms.geom_size[g] for g in boxes])
    hi = np.array([ms.geom_pos[g] + ms.geom_size[g] for g in boxes])
    for g in boxes:   # static bodies at the world origin frame: geom_pos is the world position
        _req(np.allclose(ms.body_pos[ms.geom_bodyid[g]], 0) or ms.geom_bodyid[g] == 0, "box body at origin")
    cell = float(min(min(2 * ms.geom_size[g][0], 2 * ms.geom_size[g][1]) for g in boxes))
    x0, y0 = float(lo[:, 0].min()), float(lo[:, 1].min())
    nx = int(np.ceil((hi[:, 0].max() - x0) / cell - 1e-9))
    ny = int(np.ceil((hi[:, 1].max() - y0) / cell - 1e-9))
    cells = [[] for _ in range(nx * ny)]
    eps = 1e-6
    for b in range(len(boxes)):
        for iy in range(ny):
            for ix in range(nx):
                cx0, cy0 = x0 + ix * cell, y0 + iy * cell
                if lo[b, 0] < cx0 + cell - eps and hi[b, 0] > cx0 + eps and lo[b, 1] < cy0 + cell - eps \
                        and hi[b, 1] > cy0 + eps:
                    cells[iy * nx + ix].append(b)
    ck = max(1, max(len(c) for c in cells))
    free = maze_free_cells(cells, nx, ny, x0, y0, cell, ms.spawn)
    table = np.full((nx * ny, ck), -1, np.int64)
    for i, c in enumerate(cells):
        table[i, : len(c)] = c
    L = []
    L.append("// GENERATED by mujoco_playground_amd/model/codegen.py -- do not edit.")
    L.append(f"// Obstacle scene: {ms.name} world + the ackermann_robot_v2 robot (model/compiler.py merge_scene).")
    L.append("#pragma once")
    L.append("#include <stdint.h>")
    L.append(f"namespace apg {{ namespace {ns} {{")
    L.append(f"constexpr uint64_t SCENE_FNV = 0x{blob_fnv:016x}ull;")
    f = A["floor"]
    L.append(_arr("SOLREF_C", ms.geom_solref[f]))
    L.append(_arr("SOLIMP_C", ms.geom_solimp[f]))
    L.append(_arr("SPAWN", ms.spawn))
    L.append(f"constexpr int NBOX = {len(boxes)};")
    L.append(_arr("BOX_LO", lo))
    L.append(_arr("BOX_HI", hi))
    L.append(f"constexpr float GRID_X0 = {_f(x0)}, GRID_Y0 = {_f(y0)}, GRID_CELL = {_f(cell)};")
    L.append(f"constexpr int GRID_NX = {nx}, GRID_NY = {ny}, CELL_K = {ck};")
    rows = ",\n    ".join("{" + ", ".join(str(int(x)) for x in r) + "}" for r in table)
    L.append(f"constexpr signed char CELL_BOX[{nx * ny}][{ck}] = {{\n    {rows}}};")
    # opt-in free-cell goals (ackphys_env_params.goal_cells): the box-free grid cells 4-connected to
    # the spawn cell, sorted by breadth-first distance; FREE_LE[d] = how many lie within d cells
    _req(len(free) > 0, "a free cell next to the spawn")
    maxd = max(d for _, _, d in free)
    L.append(f"constexpr int NFREE = {len(free)}, FREE_MAXD = {maxd};")
    L.append(_arr("FREE_XY", np.array([[x, y] for x, y, _ in free])))
    L.append("constexpr int FREE_LE[" + str(maxd + 1) + "] = {" +
             ", ".join(str(sum(1 for _, _, d in free if d <= k)) for k in range(maxd + 1)) + "};")
    # hull features of the welded meshes in the chassis frame (separating axes of box-mesh pairs)
    fns, eds = [], []
    for mh in A["meshes"]:
        g = mh["geom"]
        p, R = A["child_frame"][mh["body"]]
        gR = R @ quat_to_mat(ms.geom_quat[g])
        fnl, edl = hull_features(ms.meshes[ms.geom_dataid[g]].hull_vert)
        fns.append(fnl @ gR.T)
        eds.append(edl @ gR.T)
    nf, ne = max(len(x) for x in fns), max(len(x) for x in eds)
    FN = np.zeros((len(fns), nf, 3)); ED = np.zeros((len(eds), ne, 3))
    for k in range(len(fns)):
        FN[k, : len(fns[k])] = fns[k]
        ED[k, : len(eds[k])] = eds[k]
    L.append("constexpr int HULL_NF[" + str(len(fns)) + "] = {" + ", ".join(str(len(x)) for x in fns) + "};")
    L.append("constexpr int HULL_NE[" + str(len(eds)) + "] = {" + ", ".join(str(len(x)) for x in eds) + "};")
    L.append(_arr("HULL_FN", FN))
    L.append(_arr("HULL_ED", ED))
    L.append("} }  // namespace apg::" + ns)
    return "\n".join(L) + "\n"
