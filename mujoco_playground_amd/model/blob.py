"""Serialise a CompiledModel into the `apm_model_t` blob of include/ackphys_model.h.

The ctypes Structure below mirrors the C struct field for field (tests/test_model.py checks
sizeof against both compiled libraries). The blob is what `ackphys_create()` receives, the
counterpart of handing `mjModel*` to `mj_step` (reference call site
src/rl/envs/ackermann_env.py:200).
"""
from __future__ import annotations

import ctypes as C
import hashlib

import numpy as np

from .compiler import CompiledModel

APM_MAGIC = 0x4D504841
APM_VERSION = 2
MAXBODY, MAXJNT, MAXQ, MAXDOF, MAXGEOM, MAXSITE, MAXSENSOR, MAXU, MAXEQ, MAXMESH = (
    64, 8, 16, 16, 64, 80, 96, 4, 2, 4)

i32, f64, u32 = C.c_int32, C.c_double, C.c_uint32


def _a(t, *dims):
    for d in reversed(dims):
        t = t * d
    return t


class APMModel(C.Structure):
    _fields_ = [
        ("magic", u32), ("version", u32), ("nbytes", u32), ("hdr_bytes", u32),
        ("nbody", i32), ("njnt", i32), ("nq", i32), ("nv", i32), ("ngeom", i32), ("nsite", i32),
        ("nsensor", i32), ("nsensordata", i32), ("nu", i32), ("neq", i32), ("nmesh", i32),
        ("iterations", i32), ("ls_iterations", i32), ("pad0", i32),
        ("nmeshvert", i32), ("nmeshface", i32), ("nhullvert", i32), ("pad1", i32),
        ("timestep", f64), ("gravity", _a(f64, 3)), ("tolerance", f64), ("impratio", f64),
        ("meaninertia", f64),
        ("body_parentid", _a(i32, MAXBODY)), ("body_rootid", _a(i32, MAXBODY)),
        ("body_weldid", _a(i32, MAXBODY)), ("body_jntadr", _a(i32, MAXBODY)),
        ("body_jntnum", _a(i32, MAXBODY)), ("body_dofadr", _a(i32, MAXBODY)),
        ("body_dofnum", _a(i32, MAXBODY)),
        ("body_pos", _a(f64, MAXBODY, 3)), ("body_quat", _a(f64, MAXBODY, 4)),
        ("body_ipos", _a(f64, MAXBODY, 3)), ("body_iquat", _a(f64, MAXBODY, 4)),
        ("body_mass", _a(f64, MAXBODY)), ("body_inertia", _a(f64, MAXBODY, 3)),
        ("body_invweight0", _a(f64, MAXBODY, 2)),
        ("jnt_type", _a(i32, MAXJNT)), ("jnt_bodyid", _a(i32, MAXJNT)),
        ("jnt_qposadr", _a(i32, MAXJNT)), ("jnt_dofadr", _a(i32, MAXJNT)),
        ("jnt_limited", _a(i32, MAXJNT)), ("pad2", _a(i32, MAXJNT)),
        ("jnt_pos", _a(f64, MAXJNT, 3)), ("jnt_axis", _a(f64, MAXJNT, 3)),
        ("jnt_range", _a(f64, MAXJNT, 2)), ("jnt_solref", _a(f64, MAXJNT, 2)),
        ("jnt_solimp", _a(f64, MAXJNT, 5)), ("jnt_margin", _a(f64, MAXJNT)),
        ("dof_bodyid", _a(i32, MAXDOF)), ("dof_jntid", _a(i32, MAXDOF)),
        ("dof_parentid", _a(i32, MAXDOF)), ("pad3", _a(i32, MAXDOF)),
        ("dof_armature", _a(f64, MAXDOF)), ("dof_damping", _a(f64, MAXDOF)),
        ("dof_frictionloss", _a(f64, MAXDOF)), ("dof_solref", _a(f64, MAXDOF, 2)),
        ("dof_solimp", _a(f64, MAXDOF, 5)), ("dof_invweight0", _a(f64, MAXDOF)),
        ("qpos0", _a(f64, MAXQ)),
        ("geom_type", _a(i32, MAXGEOM)), ("geom_bodyid", _a(i32, MAXGEOM)),
        ("geom_contype", _a(i32, MAXGEOM)), ("geom_conaffinity", _a(i32, MAXGEOM)),
        ("geom_condim", _a(i32, MAXGEOM)), ("geom_dataid", _a(i32, MAXGEOM)),
        ("geom_pos", _a(f64, MAXGEOM, 3)), ("geom_quat", _a(f64, MAXGEOM, 4)),
        ("geom_size", _a(f64, MAXGEOM, 3)), ("geom_friction", _a(f64, MAXGEOM, 3)),
        ("geom_solref", _a(f64, MAXGEOM, 2)), ("geom_solimp", _a(f64, MAXGEOM, 5)),
        ("geom_solmix", _a(f64, MAXGEOM)), ("geom_margin", _a(f64, MAXGEOM)),
        ("geom_gap", _a(f64, MAXGEOM)), ("geom_rgba", _a(f64, MAXGEOM, 4)),
        ("geom_rbound", _a(f64, MAXGEOM)),
        ("site_bodyid", _a(i32, MAXSITE)), ("pad4", _a(i32, 2)),
        ("site_pos", _a(f64, MAXSITE, 3)), ("site_quat", _a(f64, MAXSITE, 4)),
        ("sensor_type", _a(i32, MAXSENSOR)), ("sensor_objid", _a(i32, MAXSENSOR)),
        ("sensor_adr", _a(i32, MAXSENSOR)), ("pad5", _a(i32, 2)),
        ("sensor_cutoff", _a(f64, MAXSENSOR)),
        ("actuator_type", _a(i32, MAXU)), ("actuator_trnid", _a(i32, MAXU)),
        ("actuator_ctrllimited", _a(i32, MAXU)), ("actuator_forcelimited", _a(i32, MAXU)),
        ("actuator_gear", _a(f64, MAXU)), ("actuator_gainprm", _a(f64, MAXU, 3)),
        ("actuator_biasprm", _a(f64, MAXU, 3)), ("actuator_ctrlrange", _a(f64, MAXU, 2)),
        ("actuator_forcerange", _a(f64, MAXU, 2)),
        ("eq_obj1id", _a(i32, MAXEQ)), ("eq_obj2id", _a(i32, MAXEQ)),
        ("eq_polycoef", _a(f64, MAXEQ, 5)), ("eq_solref", _a(f64, MAXEQ, 2)),
        ("eq_solimp", _a(f64, MAXEQ, 5)),
        ("mesh_vertadr", _a(i32, MAXMESH)), ("mesh_vertnum", _a(i32, MAXMESH)),
        ("mesh_faceadr", _a(i32, MAXMESH)), ("mesh_facenum", _a(i32, MAXMESH)),
        ("mesh_hulladr", _a(i32, MAXMESH)), ("mesh_hullnum", _a(i32, MAXMESH)),
        ("mesh_aabb", _a(f64, MAXMESH, 6)),
        ("spawn", _a(f64, 3)),
    ]


def _put(dst, src):
    src = np.asarray(src)
    arr = np.ctypeslib.as_array(dst)
    if src.size == 0:
        return
    arr.reshape(-1)[: src.size] = src.reshape(-1)


def pack(m: CompiledModel) -> bytes:
    for n, cap in [(m.nbody, MAXBODY), (m.njnt, MAXJNT), (m.nq, MAXQ), (m.nv, MAXDOF),
                   (m.ngeom, MAXGEOM), (m.nsite, MAXSITE), (len(m.sensor_name), MAXSENSOR),
                   (m.nu, MAXU), (m.neq, MAXEQ), (len(m.meshes), MAXMESH)]:
        if n > cap:
            raise ValueError(f"model exceeds blob capacity ({n} > {cap})")
    s = APMModel()
    s.magic, s.version = APM_MAGIC, APM_VERSION
    s.nbody, s.njnt, s.nq, s.nv = m.nbody, m.njnt, m.nq, m.nv
    s.ngeom, s.nsite, s.nsensor, s.nsensordata = m.ngeom, m.nsite, len(m.sensor_name), m.nsensordata
    s.nu, s.neq, s.nmesh = m.nu, m.neq, len(m.meshes)
    s.iterations, s.ls_iterations = m.iterations, m.ls_iterations
    s.timestep, s.tolerance, s.impratio, s.meaninertia = m.timestep, m.tolerance, m.impratio, m.meaninertia
    _put(s.gravity, m.gravity)
    _put(s.spawn, m.spawn)
    for f in ["body_parentid", "body_rootid", "body_weldid", "body_jntadr", "body_jntnum",
              "body_dofadr", "body_dofnum", "body_pos", "body_quat", "body_ipos", "body_iquat",
              "body_mass", "body_inertia", "body_invweight0",
              "jnt_type", "jnt_bodyid", "jnt_qposadr", "jnt_dofadr", "jnt_limited", "jnt_pos",
              "jnt_axis", "jnt_range", "jnt_solref", "jnt_solimp", "jnt_margin",
              "dof_bodyid", "dof_jntid", "dof_parentid", "dof_armature", "dof_damping",
              "dof_frictionloss", "dof_solref", "dof_solimp", "dof_invweight0", "qpos0",
              "geom_type", "geom_bodyid", "geom_contype", "geom_conaffinity", "geom_condim",
              "geom_dataid", "geom_pos", "geom_quat", "geom_size", "geom_friction", "geom_solref",
              "geom_solimp", "geom_solmix", "geom_margin", "geom_gap", "geom_rgba", "geom_rbound",
              "site_bodyid", "site_pos", "site_quat", "sensor_type", "sensor_objid", "sensor_adr",
              "sensor_cutoff", "actuator_type", "actuator_trnid", "actuator_ctrllimited",
              "actuator_forcelimited", "actuator_gear", "actuator_gainprm", "actuator_biasprm",
              "actuator_ctrlrange", "actuator_forcerange", "eq_obj1id", "eq_obj2id",
              "eq_polycoef", "eq_solref", "eq_solimp"]:
        _put(getattr(s, f), getattr(m, f))
    verts, faces, hulls = [], [], []
    nv = nf = nh = 0
    for k, mh in enumerate(m.meshes):
        s.mesh_vertadr[k], s.mesh_vertnum[k] = nv, len(mh.vert)
        s.mesh_faceadr[k], s.mesh_facenum[k] = nf, len(mh.face)
        s.mesh_hulladr[k], s.mesh_hullnum[k] = nh, len(mh.hull_vert)
        lo, hi = mh.vert.min(axis=0).astype(np.float64), mh.vert.max(axis=0).astype(np.float64)
        _put(s.mesh_aabb[k], np.concatenate([(lo + hi) / 2, (hi - lo) / 2]))
        verts.append(mh.vert); faces.append(mh.face); hulls.append(mh.hull_vert)
        nv += len(mh.vert); nf += len(mh.face); nh += len(mh.hull_vert)
    s.nmeshvert, s.nmeshface, s.nhullvert = nv, nf, nh
    tail = b""
    if m.meshes:
        tail = (np.concatenate(verts).astype("<f4").tobytes() + np.concatenate(faces).astype("<i4").tobytes()
                + np.concatenate(hulls).astype("<f4").tobytes())
    s.hdr_bytes = C.sizeof(APMModel)
    s.nbytes = C.sizeof(APMModel) + len(tail)
    return bytes(s) + tail


def unpack_header(blob: bytes) -> APMModel:
    return APMModel.from_buffer_copy(blob[: C.sizeof(APMModel)])


def blob_hash(blob: bytes) -> str:
    return hashlib.sha256(blob).hexdigest()


def fnv1a64(blob: bytes) -> int:
    """64-bit FNV-1a; the HIP library embeds this of the blob it was specialised on."""
    h = 0xCBF29CE484222325
    a = np.frombuffer(blob, dtype=np.uint8)
    for b in a.tobytes():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h
