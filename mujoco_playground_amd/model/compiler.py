"""Offline MJCF-subset compiler: `models/ackermann_robot_v2.xml` -> compiled model.

This plays the role of `mujoco.MjModel.from_xml_path` (called at
`src/rl/envs/simple_map_spawner.py:37` of the reference) for the features the Ackermann
robot uses: a body tree with one free joint and hinge joints, explicit <inertial> and
mesh/cylinder/plane geoms (mass inferred from geoms), sites inside <replicate>,
jointpos/jointvel/rangefinder sensors, one joint equality, position/velocity actuators.

MuJoCo semantics restated here [ext, MuJoCo >= 3.1, not vendored in /root/reference]:
  * `euler` is intrinsic "xyz" (compiler default eulerseq), angles in degrees
    (`<compiler angle="degree"/>`, `ackermann_robot_v2.xml:3`);
  * mesh geoms are re-centred to the mesh CoM / principal axes and geom pos/quat absorb
    that offset; a body with no <inertial> takes mass/inertia from its geoms;
  * `<replicate count sep euler>` applies the frame offset k times to copy k and names it
    name + sep + zero-padded k; sensors referencing the replicated site are replicated too;
  * body_invweight0 / dof_invweight0 / stat.meaninertia are computed at qpos0 (mj_setConst).

Output: a `CompiledModel` of plain numpy arrays, serialised by `blob.py` for the C-ABI and
by `codegen.py` into the constexpr header the HIP kernels are specialised on.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from . import mesh as meshmod
from .mathutil import euler_to_quat, quat_mul, quat_normalize, quat_to_mat

# MuJoCo enums (mjtGeom / mjtJoint / mjtSensor subset)
GEOM_PLANE, GEOM_SPHERE, GEOM_CAPSULE, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = 0, 2, 3, 5, 6, 7
GEOM_TYPES = {"plane": GEOM_PLANE, "sphere": GEOM_SPHERE, "capsule": GEOM_CAPSULE,
              "cylinder": GEOM_CYLINDER, "box": GEOM_BOX, "mesh": GEOM_MESH}
JNT_FREE, JNT_HINGE = 0, 3
SENS_JOINTPOS, SENS_JOINTVEL, SENS_RANGEFINDER = 0, 1, 2
ACT_POSITION, ACT_VELOCITY = 0, 1

DEFAULT_FRICTION = (1.0, 0.005, 0.0001)
DEFAULT_SOLREF = (0.02, 1.0)
DEFAULT_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)


def _floats(s, n=None):
    v = [float(x) for x in s.split()]
    if n is not None and len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


@dataclass
class CompiledModel:
    name: str
    timestep: float
    gravity: np.ndarray
    # solver options (MuJoCo defaults; the reference sets only timestep/gravity)
    iterations: int = 100
    tolerance: float = 1e-8
    ls_iterations: int = 50
    impratio: float = 1.0
    meaninertia: float = 0.0
    # bodies
    body_name: list = field(default_factory=list)
    body_parentid: np.ndarray = None
    body_rootid: np.ndarray = None
    body_weldid: np.ndarray = None
    body_pos: np.ndarray = None
    body_quat: np.ndarray = None
    body_ipos: np.ndarray = None
    body_iquat: np.ndarray = None
    body_mass: np.ndarray = None
    body_inertia: np.ndarray = None
    body_jntadr: np.ndarray = None
    body_jntnum: np.ndarray = None
    body_dofadr: np.ndarray = None
    body_dofnum: np.ndarray = None
    body_invweight0: np.ndarray = None
    # joints / dofs
    jnt_name: list = field(default_factory=list)
    jnt_type: np.ndarray = None
    jnt_bodyid: np.ndarray = None
    jnt_qposadr: np.ndarray = None
    jnt_dofadr: np.ndarray = None
    jnt_pos: np.ndarray = None
    jnt_axis: np.ndarray = None
    jnt_limited: np.ndarray = None
    jnt_range: np.ndarray = None
    jnt_solref: np.ndarray = None
    jnt_solimp: np.ndarray = None
    jnt_margin: np.ndarray = None
    dof_bodyid: np.ndarray = None
    dof_jntid: np.ndarray = None
    dof_parentid: np.ndarray = None
    dof_armature: np.ndarray = None
    dof_damping: np.ndarray = None
    dof_frictionloss: np.ndarray = None
    dof_solref: np.ndarray = None
    dof_solimp: np.ndarray = None
    dof_invweight0: np.ndarray = None
    qpos0: np.ndarray = None
    # geoms
    geom_name: list = field(default_factory=list)
    geom_type: np.ndarray = None
    geom_bodyid: np.ndarray = None
    geom_pos: np.ndarray = None
    geom_quat: np.ndarray = None
    geom_size: np.ndarray = None
    geom_contype: np.ndarray = None
    geom_conaffinity: np.ndarray = None
    geom_condim: np.ndarray = None
    geom_friction: np.ndarray = None
    geom_solref: np.ndarray = None
    geom_solimp: np.ndarray = None
    geom_solmix: np.ndarray = None
    geom_margin: np.ndarray = None
    geom_gap: np.ndarray = None
    geom_rgba: np.ndarray = None
    geom_dataid: np.ndarray = None
    geom_rbound: np.ndarray = None
    # sites
    site_name: list = field(default_factory=list)
    site_bodyid: np.ndarray = None
    site_pos: np.ndarray = None
    site_quat: np.ndarray = None
    # sensors
    sensor_name: list = field(default_factory=list)
    sensor_type: np.ndarray = None
    sensor_objid: np.ndarray = None
    sensor_adr: np.ndarray = None
    sensor_cutoff: np.ndarray = None
    nsensordata: int = 0
    # actuators
    actuator_name: list = field(default_factory=list)
    actuator_type: np.ndarray = None
    actuator_trnid: np.ndarray = None     # joint id
    actuator_gear: np.ndarray = None
    actuator_gainprm: np.ndarray = None   # [nu,3]
    actuator_biasprm: np.ndarray = None   # [nu,3]
    actuator_ctrlrange: np.ndarray = None
    actuator_ctrllimited: np.ndarray = None
    actuator_forcerange: np.ndarray = None
    actuator_forcelimited: np.ndarray = None
    # equality (joint type only)
    eq_name: list = field(default_factory=list)
    eq_obj1id: np.ndarray = None
    eq_obj2id: np.ndarray = None
    eq_polycoef: np.ndarray = None
    eq_solref: np.ndarray = None
    eq_solimp: np.ndarray = None
    # meshes
    meshes: list = field(default_factory=list)
    mesh_inertia_mode: str = "legacy"
    # env spawn point (x, y, z) the reset writes into the free joint (scene property, see merge_scene)
    spawn: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, 0.1]))

    @property
    def nbody(self):
        return len(self.body_name)

    @property
    def njnt(self):
        return len(self.jnt_name)

    @property
    def nq(self):
        return len(self.qpos0)

    @property
    def nv(self):
        return len(self.dof_bodyid)

    @property
    def ngeom(self):
        return len(self.geom_name)

    @property
    def nsite(self):
        return len(self.site_name)

    @property
    def nu(self):
        return len(self.actuator_name)

    @property
    def neq(self):
        return len(self.eq_name)

    def name2id(self, kind: str, name: str) -> int:
        """MuJoCo `mj_name2id`: id, or -1 if absent (the Python bindings do not raise)."""
        lst = {"body": self.body_name, "joint": self.jnt_name, "geom": self.geom_name,
               "site": self.site_name, "sensor": self.sensor_name,
               "actuator": self.actuator_name}[kind]
        try:
            return lst.index(name)
        except ValueError:
            return -1


# ----------------------------------------------------------------------------- parsing

class _Body:
    def __init__(self, name, pos, quat, parent):
        self.name, self.pos, self.quat, self.parent = name, pos, quat, parent
        self.children, self.joints, self.geoms, self.sites = [], [], [], []
        self.inertial = None


def _frame(el, angle_scale):
    pos = np.array(_floats(el.get("pos", "0 0 0"), 3))
    if el.get("quat") is not None:
        quat = quat_normalize(_floats(el.get("quat"), 4))
    elif el.get("euler") is not None:
        quat = euler_to_quat(np.array(_floats(el.get("euler"), 3)) * angle_scale)
    elif el.get("axisangle") is not None:
        raise NotImplementedError("axisangle")
    else:
        quat = np.array([1.0, 0.0, 0.0, 0.0])
    return pos, quat


def _parse_body(el, parent, angle_scale, out_bodies):
    pos, quat = _frame(el, angle_scale)
    b = _Body(el.get("name", f"body{len(out_bodies)}"), pos, quat, parent)
    out_bodies.append(b)
    for ch in el:
        tag = ch.tag
        if tag in ("freejoint",):
            b.joints.append({"type": JNT_FREE, "name": ch.get("name", f"{b.name}_free")})
        elif tag == "joint":
            jt = ch.get("type", "hinge")
            if jt != "hinge":
                raise NotImplementedError(f"joint type {jt}")
            j = {"type": JNT_HINGE, "name": ch.get("name"),
                 "axis": np.array(_floats(ch.get("axis", "0 0 1"), 3)),
                 "pos": np.array(_floats(ch.get("pos", "0 0 0"), 3)),
                 "damping": float(ch.get("damping", 0)),
                 "frictionloss": float(ch.get("frictionloss", 0)),
                 "armature": float(ch.get("armature", 0)),
                 "range": None}
            if ch.get("range") is not None:
                j["range"] = np.array(_floats(ch.get("range"), 2)) * angle_scale
            j["axis"] = j["axis"] / np.linalg.norm(j["axis"])
            b.joints.append(j)
        elif tag == "inertial":
            ipos, iquat = _frame(ch, angle_scale)
            b.inertial = {"pos": ipos, "quat": iquat, "mass": float(ch.get("mass")),
                          "diaginertia": np.array(_floats(ch.get("diaginertia"), 3))}
        elif tag == "geom":
            b.geoms.append(_parse_geom(ch, angle_scale))
        elif tag == "site":
            spos, squat = _frame(ch, angle_scale)
            b.sites.append({"name": ch.get("name"), "pos": spos, "quat": squat})
        elif tag == "replicate":
            count = int(ch.get("count"))
            sep = ch.get("sep", "")
            rpos, rquat = _frame(ch, angle_scale)
            width = len(str(count))  # MuJoCo pads to the digit count of `count` (72 -> 2)
            for sub in ch:
                if sub.tag != "site":
                    raise NotImplementedError(f"replicate of <{sub.tag}>")
                spos, squat = _frame(sub, angle_scale)
                for k in range(count):
                    # offset frame applied k times: R_k = rquat^k, p_k = sum R_i rpos
                    qk = np.array([1.0, 0, 0, 0])
                    pk = np.zeros(3)
                    for _ in range(k):
                        pk = pk + quat_to_mat(qk) @ rpos
                        qk = quat_mul(qk, rquat)
                    b.sites.append({"name": f"{sub.get('name')}{sep}{k:0{width}d}",
                                    "pos": pk + quat_to_mat(qk) @ spos,
                                    "quat": quat_normalize(quat_mul(qk, squat)),
                                    "replicated_from": sub.get("name")})
        elif tag == "body":
            b.children.append(_parse_body(ch, b, angle_scale, out_bodies))
        elif tag in ("light", "camera"):
            pass
        else:
            raise NotImplementedError(f"<{tag}> in body")
    return b


def _parse_geom(ch, angle_scale):
    gpos, gquat = _frame(ch, angle_scale)
    gtype = ch.get("type", "sphere")
    g = {"name": ch.get("name"), "type": GEOM_TYPES[gtype], "pos": gpos, "quat": gquat,
         "size": np.array(_floats(ch.get("size", "0 0 0"))),
         "contype": int(ch.get("contype", 1)), "conaffinity": int(ch.get("conaffinity", 1)),
         "condim": int(ch.get("condim", 3)),
         "friction": np.array(_floats(ch.get("friction", " ".join(map(str, DEFAULT_FRICTION))))),
         "solref": np.array(_floats(ch.get("solref", " ".join(map(str, DEFAULT_SOLREF))))),
         "solimp": np.array(_floats(ch.get("solimp", " ".join(map(str, DEFAULT_SOLIMP))))),
         "solmix": float(ch.get("solmix", 1.0)), "margin": float(ch.get("margin", 0.0)),
         "gap": float(ch.get("gap", 0.0)), "mass": ch.get("mass"), "mesh": ch.get("mesh"),
         "rgba": np.array(_floats(ch.get("rgba", "0.5 0.5 0.5 1"), 4)),
         "group": int(ch.get("group", 0))}
    if g["mass"] is not None:
        g["mass"] = float(g["mass"])
    fr = list(g["friction"]) + list(DEFAULT_FRICTION[len(g["friction"]):])
    g["friction"] = np.array(fr[:3])
    # partially specified solref/solimp keep MuJoCo's defaults for the remaining entries
    g["solref"] = np.array((list(g["solref"]) + list(DEFAULT_SOLREF[len(g["solref"]):]))[:2])
    g["solimp"] = np.array((list(g["solimp"]) + list(DEFAULT_SOLIMP[len(g["solimp"]):]))[:5])
    sz = list(g["size"]) + [0.0] * (3 - len(g["size"]))
    g["size"] = np.array(sz[:3])
    return g


# ----------------------------------------------------------------------------- compile

def _apply_geom_defaults(root):
    """Top-level `<default><geom .../></default>`: attributes a geom does not set itself are
    taken from it (MJCF main default class; nested classes are not used by these models)."""
    dflt = root.find("default")
    if dflt is None:
        return
    for ch in dflt:
        if ch.tag == "default":
            raise NotImplementedError("nested default classes")
        if ch.tag != "geom":
            raise NotImplementedError(f"<default><{ch.tag}>")
        for g in root.iter("geom"):
            for k, v in ch.attrib.items():
                if k not in g.attrib:
                    g.set(k, v)


def compile_mjcf(xml_path: str, mesh_inertia: str = "legacy") -> CompiledModel:
    xml_path = os.path.abspath(xml_path)
    return compile_root(ET.parse(xml_path).getroot(), os.path.dirname(xml_path), mesh_inertia)


def compile_root(root, base: str, mesh_inertia: str = "legacy", spawn=(0.0, 0.0, 0.1)) -> CompiledModel:
    root = ET.fromstring(ET.tostring(root))   # private copy: defaults are applied in place
    _apply_geom_defaults(root)
    angle_scale = np.pi / 180.0
    comp = root.find("compiler")
    if comp is not None and comp.get("angle", "degree") == "radian":
        angle_scale = 1.0
    opt = root.find("option")
    timestep = float(opt.get("timestep", 0.002)) if opt is not None else 0.002
    gravity = np.array(_floats(opt.get("gravity", "0 0 -9.81"), 3)) if opt is not None else np.array([0, 0, -9.81])

    mesh_files = {}
    for asset in root.findall("asset"):
        for m in asset.findall("mesh"):
            mesh_files[m.get("name")] = os.path.join(base, m.get("file"))   # absolute paths pass through
    meshes, mesh_id = [], {}
    for name, path in mesh_files.items():
        mesh_id[name] = len(meshes)
        meshes.append(meshmod.compile_mesh(name, path, mesh_inertia))

    world = _Body("world", np.zeros(3), np.array([1.0, 0, 0, 0]), None)
    bodies = [world]
    wb = root.find("worldbody")
    for ch in wb:
        if ch.tag == "geom":
            world.geoms.append(_parse_geom(ch, angle_scale))
        elif ch.tag == "body":
            world.children.append(_parse_body(ch, world, angle_scale, bodies))
        elif ch.tag in ("light", "camera"):
            pass
        else:
            raise NotImplementedError(ch.tag)

    # MuJoCo body order is depth-first pre-order, which is the order _parse_body appends.
    m = CompiledModel(name=root.get("model", "model"), timestep=timestep, gravity=gravity)
    m.spawn = np.array(spawn, dtype=np.float64)
    m.meshes = meshes
    m.mesh_inertia_mode = mesh_inertia
    nb = len(bodies)
    idx = {id(b): i for i, b in enumerate(bodies)}
    m.body_name = [b.name for b in bodies]
    m.body_parentid = np.array([idx[id(b.parent)] if b.parent else 0 for b in bodies], np.int32)
    m.body_pos = np.array([b.pos for b in bodies])
    m.body_quat = np.array([b.quat for b in bodies])

    # joints / dofs / qpos0
    jn, jtype, jbody, jqadr, jdadr, jpos, jaxis, jlim, jrange = [], [], [], [], [], [], [], [], []
    dbody, djnt, dparent, darm, ddamp, dfloss = [], [], [], [], [], []
    qpos0 = []
    bjadr, bjnum, bdadr, bdnum = [], [], [], []
    last_dof_of_body = {0: -1}
    for bi, b in enumerate(bodies):
        bjadr.append(len(jn))
        bjnum.append(len(b.joints))
        bdadr.append(len(dbody))
        parent_last = last_dof_of_body.get(m.body_parentid[bi], -1) if bi > 0 else -1
        prev = parent_last
        for j in b.joints:
            jid = len(jn)
            jn.append(j["name"])
            jtype.append(j["type"])
            jbody.append(bi)
            jqadr.append(len(qpos0))
            jdadr.append(len(dbody))
            if j["type"] == JNT_FREE:
                qpos0.extend(list(b.pos) + list(b.quat))
                jpos.append(np.zeros(3))
                jaxis.append(np.array([0.0, 0.0, 1.0]))
                jlim.append(0)
                jrange.append(np.zeros(2))
                for k in range(6):
                    dbody.append(bi); djnt.append(jid); dparent.append(prev)
                    darm.append(0.0); ddamp.append(0.0); dfloss.append(0.0)
                    prev = len(dbody) - 1
            else:
                qpos0.append(0.0)
                jpos.append(j["pos"]); jaxis.append(j["axis"])
                lim = j["range"] is not None   # limited="auto" + range given -> limited
                jlim.append(1 if lim else 0)
                jrange.append(j["range"] if lim else np.zeros(2))
                dbody.append(bi); djnt.append(jid); dparent.append(prev)
                darm.append(j["armature"]); ddamp.append(j["damping"]); dfloss.append(j["frictionloss"])
                prev = len(dbody) - 1
        bdnum.append(len(dbody) - bdadr[-1])
        last_dof_of_body[bi] = prev
    m.jnt_name, m.jnt_type, m.jnt_bodyid = jn, np.array(jtype, np.int32), np.array(jbody, np.int32)
    m.jnt_qposadr, m.jnt_dofadr = np.array(jqadr, np.int32), np.array(jdadr, np.int32)
    m.jnt_pos, m.jnt_axis = np.array(jpos), np.array(jaxis)
    m.jnt_limited, m.jnt_range = np.array(jlim, np.int32), np.array(jrange)
    m.jnt_solref = np.tile(DEFAULT_SOLREF, (len(jn), 1))
    m.jnt_solimp = np.tile(DEFAULT_SOLIMP, (len(jn), 1))
    m.jnt_margin = np.zeros(len(jn))
    m.dof_bodyid, m.dof_jntid = np.array(dbody, np.int32), np.array(djnt, np.int32)
    m.dof_parentid = np.array(dparent, np.int32)
    m.dof_armature, m.dof_damping = np.array(darm), np.array(ddamp)
    m.dof_frictionloss = np.array(dfloss)
    m.dof_solref = np.tile(DEFAULT_SOLREF, (len(dbody), 1))
    m.dof_solimp = np.tile(DEFAULT_SOLIMP, (len(dbody), 1))
    m.qpos0 = np.array(qpos0)
    m.body_jntadr, m.body_jntnum = np.array(bjadr, np.int32), np.array(bjnum, np.int32)
    m.body_dofadr, m.body_dofnum = np.array(bdadr, np.int32), np.array(bdnum, np.int32)

    # root / weld ids
    rootid, weldid = np.zeros(nb, np.int32), np.zeros(nb, np.int32)
    for i in range(1, nb):
        p = m.body_parentid[i]
        rootid[i] = i if p == 0 else rootid[p]
        weldid[i] = i if bjnum[i] > 0 else weldid[p]
    m.body_rootid, m.body_weldid = rootid, weldid

    # geoms (MuJoCo order: by body, in XML order within a body)
    gl = []
    for bi, b in enumerate(bodies):
        for g in b.geoms:
            gl.append((bi, g))
    m.geom_name = [g["name"] if g["name"] else f"geom{i}" for i, (_, g) in enumerate(gl)]
    ng = len(gl)
    m.geom_type = np.array([g["type"] for _, g in gl], np.int32)
    m.geom_bodyid = np.array([bi for bi, _ in gl], np.int32)
    gpos, gquat, gsize, gdata, grb = [], [], [], [], []
    for bi, g in gl:
        pos, quat = g["pos"].copy(), g["quat"].copy()
        if g["type"] == GEOM_MESH:
            mh = meshes[mesh_id[g["mesh"]]]
            pos = pos + quat_to_mat(quat) @ mh.pos
            quat = quat_normalize(quat_mul(quat, mh.quat))
            gdata.append(mesh_id[g["mesh"]])
            grb.append(mh.rbound)
        else:
            gdata.append(-1)
            s = g["size"]
            grb.append({GEOM_PLANE: 0.0, GEOM_SPHERE: s[0], GEOM_CAPSULE: s[0] + s[1],
                        GEOM_CYLINDER: float(np.hypot(s[0], s[1])),
                        GEOM_BOX: float(np.linalg.norm(s))}[g["type"]])
        gpos.append(pos); gquat.append(quat); gsize.append(g["size"])
    m.geom_pos, m.geom_quat, m.geom_size = np.array(gpos), np.array(gquat), np.array(gsize)
    m.geom_dataid, m.geom_rbound = np.array(gdata, np.int32), np.array(grb)
    m.geom_contype = np.array([g["contype"] for _, g in gl], np.int32)
    m.geom_conaffinity = np.array([g["conaffinity"] for _, g in gl], np.int32)
    m.geom_condim = np.array([g["condim"] for _, g in gl], np.int32)
    m.geom_friction = np.array([g["friction"] for _, g in gl])
    m.geom_solref = np.array([g["solref"] for _, g in gl])
    m.geom_solimp = np.array([g["solimp"] for _, g in gl])
    m.geom_solmix = np.array([g["solmix"] for _, g in gl])
    m.geom_margin = np.array([g["margin"] for _, g in gl])
    m.geom_gap = np.array([g["gap"] for _, g in gl])
    m.geom_rgba = np.array([g["rgba"] for _, g in gl])

    # body inertials (explicit <inertial>, else inferred from geoms)
    bm, bi_pos, bi_quat, bi_in = np.zeros(nb), np.zeros((nb, 3)), np.tile([1.0, 0, 0, 0], (nb, 1)), np.zeros((nb, 3))
    for i, b in enumerate(bodies):
        if i == 0:
            continue
        if b.inertial is not None:
            bm[i] = b.inertial["mass"]
            bi_pos[i], bi_quat[i] = b.inertial["pos"], b.inertial["quat"]
            bi_in[i] = b.inertial["diaginertia"]
            continue
        gs = [(k, g) for k, (bb, g) in enumerate(gl) if bb == i]
        if not gs:
            continue
        if weldid[i] == 0:
            continue   # static body (welded to the world): its inertia never enters the dynamics
        if len(gs) != 1:
            raise NotImplementedError("multi-geom inertia inference")
        k, g = gs[0]
        if g["type"] != GEOM_MESH or g["mass"] is None:
            raise NotImplementedError("inertia inference only for mass-specified meshes")
        mh = meshes[mesh_id[g["mesh"]]]
        bm[i] = g["mass"]
        bi_pos[i], bi_quat[i] = m.geom_pos[k], m.geom_quat[k]
        bi_in[i] = mh.inertia * (g["mass"] / mh.volume)
    m.body_mass, m.body_ipos, m.body_iquat, m.body_inertia = bm, bi_pos, bi_quat, bi_in

    # sites
    sl = []
    for bi, b in enumerate(bodies):
        for s in b.sites:
            sl.append((bi, s))
    m.site_name = [s["name"] for _, s in sl]
    m.site_bodyid = np.array([bi for bi, _ in sl], np.int32)
    m.site_pos = np.array([s["pos"] for _, s in sl])
    m.site_quat = np.array([s["quat"] for _, s in sl])
    replicated = {}
    for k, (_, s) in enumerate(sl):
        if "replicated_from" in s:
            replicated.setdefault(s["replicated_from"], []).append(k)

    # sensors (XML order; a sensor on a replicated site expands in place)
    sn, st, so, sa, sc = [], [], [], [], []
    adr = 0
    sens = root.find("sensor")
    for ch in (sens if sens is not None else []):
        if ch.tag in ("jointpos", "jointvel"):
            sn.append(ch.get("name")); st.append(SENS_JOINTPOS if ch.tag == "jointpos" else SENS_JOINTVEL)
            so.append(m.name2id("joint", ch.get("joint"))); sa.append(adr); sc.append(float(ch.get("cutoff", 0)))
            adr += 1
        elif ch.tag == "rangefinder":
            site = ch.get("site")
            if site in replicated:
                ks = replicated[site]
                width = len(str(len(ks)))
                for r, k in enumerate(ks):
                    sn.append(f"{ch.get('name')}{m.site_name[k][len(site)]}{r:0{width}d}")
                    st.append(SENS_RANGEFINDER); so.append(k); sa.append(adr)
                    sc.append(float(ch.get("cutoff", 0))); adr += 1
            else:
                sn.append(ch.get("name")); st.append(SENS_RANGEFINDER); so.append(m.name2id("site", site))
                sa.append(adr); sc.append(float(ch.get("cutoff", 0))); adr += 1
        else:
            raise NotImplementedError(ch.tag)
    m.sensor_name, m.sensor_type = sn, np.array(st, np.int32)
    m.sensor_objid, m.sensor_adr = np.array(so, np.int32), np.array(sa, np.int32)
    m.sensor_cutoff, m.nsensordata = np.array(sc), adr

    # equality
    en, e1, e2, ep = [], [], [], []
    eqs = root.find("equality")
    for ch in (eqs if eqs is not None else []):
        if ch.tag != "joint":
            raise NotImplementedError(ch.tag)
        en.append(ch.get("name"))
        e1.append(m.name2id("joint", ch.get("joint1")))
        e2.append(m.name2id("joint", ch.get("joint2")) if ch.get("joint2") else -1)
        pc = _floats(ch.get("polycoef", "0 1 0 0 0"))
        ep.append((pc + [0.0] * 5)[:5])
    m.eq_name, m.eq_obj1id, m.eq_obj2id = en, np.array(e1, np.int32), np.array(e2, np.int32)
    m.eq_polycoef = np.array(ep).reshape(-1, 5)
    m.eq_solref = np.tile(DEFAULT_SOLREF, (len(en), 1))
    m.eq_solimp = np.tile(DEFAULT_SOLIMP, (len(en), 1))

    # actuators (gear 1; MuJoCo position: gain kp, bias (0,-kp,-kv); velocity: gain kv, bias (0,0,-kv))
    an, at, aj, gp, bp, cr, cl, fr, fl = [], [], [], [], [], [], [], [], []
    acts = root.find("actuator")
    for ch in (acts if acts is not None else []):
        an.append(ch.get("name")); aj.append(m.name2id("joint", ch.get("joint")))
        if ch.tag == "position":
            kp, kv = float(ch.get("kp", 1)), float(ch.get("kv", 0))
            at.append(ACT_POSITION); gp.append([kp, 0, 0]); bp.append([0, -kp, -kv])
        elif ch.tag == "velocity":
            kv = float(ch.get("kv", 1))
            at.append(ACT_VELOCITY); gp.append([kv, 0, 0]); bp.append([0, 0, -kv])
        else:
            raise NotImplementedError(ch.tag)
        c = ch.get("ctrlrange"); f = ch.get("forcerange")
        cr.append(_floats(c, 2) if c else [0, 0]); cl.append(1 if c else 0)
        fr.append(_floats(f, 2) if f else [0, 0]); fl.append(1 if f else 0)
    m.actuator_name, m.actuator_type = an, np.array(at, np.int32)
    m.actuator_trnid, m.actuator_gear = np.array(aj, np.int32), np.ones(len(an))
    m.actuator_gainprm, m.actuator_biasprm = np.array(gp), np.array(bp)
    m.actuator_ctrlrange, m.actuator_ctrllimited = np.array(cr), np.array(cl, np.int32)
    m.actuator_forcerange, m.actuator_forcelimited = np.array(fr), np.array(fl, np.int32)

    _set_const(m)
    return m


# ----------------------------------------------------------------------------- mj_setConst

def body_frames(m: CompiledModel, qpos: np.ndarray):
    """World poses (xpos, xmat) of all bodies, and hinge anchors/axes. float64 numpy."""
    nb = m.nbody
    xpos, xmat = np.zeros((nb, 3)), np.zeros((nb, 3, 3))
    xmat[0] = np.eye(3)
    xanchor, xaxis = np.zeros((m.njnt, 3)), np.zeros((m.njnt, 3))
    xquat = np.zeros((nb, 4)); xquat[0] = [1, 0, 0, 0]
    for i in range(1, nb):
        p = m.body_parentid[i]
        jadr, jnum = m.body_jntadr[i], m.body_jntnum[i]
        if jnum == 1 and m.jnt_type[jadr] == JNT_FREE:
            a = m.jnt_qposadr[jadr]
            xpos[i] = qpos[a:a + 3]
            xquat[i] = quat_normalize(qpos[a + 3:a + 7])
            xanchor[jadr] = xpos[i]; xaxis[jadr] = [0, 0, 1]
        else:
            xpos[i] = xpos[p] + xmat[p] @ m.body_pos[i]
            xquat[i] = quat_normalize(quat_mul(xquat[p], m.body_quat[i]))
            for j in range(jadr, jadr + jnum):
                R = quat_to_mat(xquat[i])
                xaxis[j] = R @ m.jnt_axis[j]
                xanchor[j] = R @ m.jnt_pos[j] + xpos[i]
                qa = m.jnt_qposadr[j]
                ang = qpos[qa] - m.qpos0[qa]
                s = np.sin(ang / 2)
                ql = np.array([np.cos(ang / 2), *(m.jnt_axis[j] * s)])
                xquat[i] = quat_normalize(quat_mul(xquat[i], ql))
                xpos[i] = xanchor[j] - quat_to_mat(xquat[i]) @ m.jnt_pos[j]
        xmat[i] = quat_to_mat(xquat[i])
    return xpos, xmat, xquat, xanchor, xaxis


def point_jacobian(m: CompiledModel, xpos, xmat, xanchor, xaxis, body: int, point):
    """6 x nv world-frame jacobian [lin; ang] of a point rigidly attached to `body`."""
    J = np.zeros((6, m.nv))
    d = m.body_dofadr[body] + m.body_dofnum[body] - 1
    b = body
    while b > 0 and m.body_dofnum[b] == 0:
        b = m.body_parentid[b]
    d = m.body_dofadr[b] + m.body_dofnum[b] - 1 if b > 0 else -1
    while d >= 0:
        j = m.dof_jntid[d]
        if m.jnt_type[j] == JNT_FREE:
            k = d - m.jnt_dofadr[j]
            jb = m.jnt_bodyid[j]
            if k < 3:
                J[k, d] = 1.0
            else:
                ax = xmat[jb][:, k - 3]
                J[3:, d] = ax
                J[:3, d] = np.cross(ax, point - xpos[jb])
        else:
            J[3:, d] = xaxis[j]
            J[:3, d] = np.cross(xaxis[j], point - xanchor[j])
        d = m.dof_parentid[d]
    return J


def mass_matrix(m: CompiledModel, qpos) -> np.ndarray:
    """Joint-space inertia (incl. armature) as Σ_b Jᵀ diag(m, I_world) J. Slow, exact."""
    xpos, xmat, _, xanchor, xaxis = body_frames(m, qpos)
    M = np.zeros((m.nv, m.nv))
    for b in range(1, m.nbody):
        if m.body_mass[b] <= 0:
            continue
        xipos = xpos[b] + xmat[b] @ m.body_ipos[b]
        ximat = xmat[b] @ quat_to_mat(m.body_iquat[b])
        Iw = ximat @ np.diag(m.body_inertia[b]) @ ximat.T
        J = point_jacobian(m, xpos, xmat, xanchor, xaxis, b, xipos)
        M += m.body_mass[b] * J[:3].T @ J[:3] + J[3:].T @ Iw @ J[3:]
    M += np.diag(m.dof_armature)
    return M


def _set_const(m: CompiledModel):
    q0 = m.qpos0
    M = mass_matrix(m, q0)
    Minv = np.linalg.inv(M)
    m.meaninertia = float(np.trace(M) / m.nv)
    xpos, xmat, _, xanchor, xaxis = body_frames(m, q0)
    iw = np.zeros((m.nbody, 2))
    for b in range(1, m.nbody):
        if m.body_weldid[b] == 0:
            continue
        xipos = xpos[b] + xmat[b] @ m.body_ipos[b]
        J = point_jacobian(m, xpos, xmat, xanchor, xaxis, b, xipos)
        A = J @ Minv @ J.T
        iw[b] = [np.trace(A[:3, :3]) / 3.0, np.trace(A[3:, 3:]) / 3.0]
    m.body_invweight0 = iw
    dw = np.zeros(m.nv)
    for j in range(m.njnt):
        d = m.jnt_dofadr[j]
        if m.jnt_type[j] == JNT_FREE:
            dw[d:d + 3] = np.trace(Minv[d:d + 3, d:d + 3]) / 3.0
            dw[d + 3:d + 6] = np.trace(Minv[d + 3:d + 6, d + 3:d + 6]) / 3.0
        else:
            dw[d] = Minv[d, d]
    m.dof_invweight0 = dw


def default_model_path(reference_root: str = "/root/reference") -> str:
    return os.path.join(reference_root, "models", "ackermann_robot_v2.xml")


def obstacle_scene_path(reference_root: str = "/root/reference") -> str:
    return os.path.join(reference_root, "models", "environments", "ackermann_maze_flat.xml")


# ----------------------------------------------------------------------------- scene merge

def merge_scene(scene_xml: str, robot_xml: str):
    """The obstacle scene: the v2 robot merged into a static world.

    The merge follows the reference's robot-into-maze rules
    (src/rl/envs/ackermann_gymnasium_maze_env.py:237-398):
      * the robot's <compiler> attributes override the scene's (:249-258), the robot's
        option gravity/timestep override the scene's (:262-271);
      * robot assets are added (:298-311) -- the robot's mesh files are used for the shared
        mesh names, because the scene file's own paths (`../CAD Models/` relative to
        models/environments/) point at a directory the reference does not have;
      * the robot's chassis subtree, sensors, actuators and equality constraints are appended
        (:354-398).
    Scene-specific choices (documented in DESIGN.md §11):
      * the scene file's OWN robot (its free-joint `chassis` body and the sensors/actuators that
        reference it; it has torque drives and 36 lidar sites, which the v2 controller and
        observation code cannot drive) is removed, and its chassis position becomes the env
        spawn point (x, y) -- the reference's spawn (0, 0) lies inside obstacle_22 here;
      * the maze rule that lowers geoms named *floor* to z = -0.5 and lifts *block* geoms
        (:322-352) is for gymnasium-robotics mazes; the flat scene's obstacles are named
        obstacle_*, so applying it would leave them hovering -- the scene geometry is kept;
      * the scene's top-level <default> applies to every geom of the merged file (MJCF
        semantics), so robot, floor and obstacle contacts all use its solref/solimp.
    Returns (root Element, base directory, spawn xyz).
    """
    scene = ET.parse(scene_xml).getroot()
    robot = ET.parse(robot_xml).getroot()
    rc, sc = robot.find("compiler"), scene.find("compiler")
    if rc is not None:
        if sc is None:
            sc = ET.SubElement(scene, "compiler")
        for k, v in rc.attrib.items():
            sc.set(k, v)
    ro, so = robot.find("option"), scene.find("option")
    if ro is not None:
        if so is None:
            so = ET.SubElement(scene, "option")
        for k in ("gravity", "timestep"):
            if k in ro.attrib:
                so.set(k, ro.get(k))
    rbase = os.path.dirname(os.path.abspath(robot_xml))
    sassets = scene.findall("asset")
    if not sassets:
        sassets = [ET.SubElement(scene, "asset")]
    for ra in robot.findall("asset"):
        for item in ra:
            item = ET.fromstring(ET.tostring(item))
            if "file" in item.attrib and not os.path.isabs(item.get("file")):
                item.set("file", os.path.normpath(os.path.join(rbase, item.get("file"))))
            for a in sassets:
                for old in list(a):
                    if old.tag == item.tag and old.get("name") == item.get("name"):
                        a.remove(old)
            sassets[0].append(item)
    swb, rwb = scene.find("worldbody"), robot.find("worldbody")
    spawn = None
    for b in list(swb):
        if b.tag == "body" and (b.find("freejoint") is not None or b.find("joint") is not None):
            if spawn is not None:
                raise NotImplementedError("more than one free body in the scene")
            p = _floats(b.get("pos", "0 0 0"), 3)
            spawn = (p[0], p[1], 0.1)   # reset height of AckermannRobotEnv.reset (robot_pos z = 0.1)
            swb.remove(b)
    if spawn is None:
        spawn = (0.0, 0.0, 0.1)
    for tag in ("sensor", "actuator", "equality"):
        for el in scene.findall(tag):
            scene.remove(el)
    chassis = rwb.find("body[@name='chassis']")
    swb.append(ET.fromstring(ET.tostring(chassis)))
    for tag in ("sensor", "actuator", "equality"):
        el = robot.find(tag)
        if el is not None:
            scene.append(ET.fromstring(ET.tostring(el)))
    return scene, os.path.dirname(os.path.abspath(scene_xml)), spawn


def compile_scene(scene_xml: str, robot_xml: str, mesh_inertia: str = "legacy") -> CompiledModel:
    root, base, spawn = merge_scene(scene_xml, robot_xml)
    m = compile_root(root, base, mesh_inertia, spawn)
    m.name = root.get("model", "scene")
    return m
