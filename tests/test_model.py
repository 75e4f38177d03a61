"""Compiler known-answer tests and the C-ABI boundary (CPU only, no compute calls)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from mujoco_playground_amd import _lib
from mujoco_playground_amd.model import blob as blobmod


def test_counts_and_tree(cmodel):
    m = cmodel
    assert (m.nbody, m.njnt, m.nq, m.nv, m.ngeom, m.nsite, m.nu, m.neq) == (11, 7, 13, 12, 7, 72, 3, 1)
    assert list(m.dof_parentid) == [-1, 0, 1, 2, 3, 4, 5, 5, 5, 8, 5, 10]
    # sparse nM along the dof tree: sum of ancestor chain lengths
    depth = [0] * m.nv
    for i in range(m.nv):
        j, d = i, 0
        while j >= 0:
            d += 1
            j = m.dof_parentid[j]
        depth[i] = d
    assert sum(depth) == 65
    assert abs(m.body_mass.sum() - 10.3) < 1e-12
    assert m.nsensordata == 77 and len(m.sensor_name) == 77


def test_lidar_names_and_alias(cmodel):
    m = cmodel
    assert m.sensor_name[5] == "lidar-00" and m.sensor_name[76] == "lidar-71"
    assert m.name2id("sensor", "lidar-5") == -1 and m.name2id("sensor", "lidar-15") == 20
    # ray 0 along +x, ray 18 along +y, origin 0.035 from the lidar centre at chassis z +0.03
    dirs = [np.array([0, 0, 1.0]) @ np.array(__import__("mujoco_playground_amd.model.mathutil",
            fromlist=["quat_to_mat"]).quat_to_mat(q)).T for q in m.site_quat]
    assert np.allclose(dirs[0], [1, 0, 0], atol=1e-12) and np.allclose(dirs[18], [0, 1, 0], atol=1e-12)
    assert np.allclose(np.linalg.norm(m.site_pos[:, :2], axis=1), 0.035)


def test_mesh_geometry(cmodel):
    for mh in cmodel.meshes:
        ext = mh.vert.max(0) - mh.vert.min(0)
        assert np.allclose(sorted(ext), [0.004, 0.15, 0.275], atol=2e-3)  # principal axes ~ plate axes
        assert len(mh.hull_vert) >= 8
        assert np.all(mh.inertia > 0)


def test_codegen_assumptions_and_assets_current(cmodel):
    from mujoco_playground_amd.model import codegen
    A = codegen.analyse(cmodel)
    assert abs(A["mt"] - 10.3) < 1e-12
    from mujoco_playground_amd.model import build as mbuild
    assert mbuild.build(check_only=True), "committed model assets are stale: run python -m mujoco_playground_amd.model.build"


def test_blob_layout_matches_c(oracle, blob):
    from oracle.oracle import lib as olib
    assert olib().or_model_struct_size() == C.sizeof(blobmod.APMModel)
    h = blobmod.unpack_header(blob)
    assert h.magic == blobmod.APM_MAGIC and h.nbytes == len(blob) and h.nv == 12


def test_header_fnv_matches_blob(blob):
    hdr = open(os.path.join(_lib.CSRC, "ackphys_model_gen.h")).read()
    fnv = int(re.search(r"MODEL_FNV = 0x([0-9a-f]+)ull", hdr).group(1), 16)
    assert fnv == blobmod.fnv1a64(blob)


def test_capi_exports_every_declared_symbol():
    """libackphys.so loads (no GPU calls) and exports exactly what include/ackphys.h declares."""
    path = _lib.build()
    hdr = open(os.path.join(_lib.REPO, "include", "ackphys.h")).read()
    declared = set(re.findall(r"^\w[\w\s\*]*?\b(ackphys_\w+)\s*\(", hdr, re.M))
    assert declared == set(_lib.EXPORTS)
    L = C.CDLL(path)
    for name in declared:
        assert hasattr(L, name), name
    L.ackphys_model_fnv.restype = C.c_uint64
    assert L.ackphys_model_fnv() == blobmod.fnv1a64(_lib.load_blob())


def test_rebuild_check_covers_every_included_source():
    """The staleness check of _lib.build() sees every file the kernels #include (the obstacle-scene
    .inc and generated headers included), so an edit to any of them triggers a rebuild."""
    names = {os.path.basename(s) for s in _lib.SOURCES}
    assert {"ackphys_step.hip", "ackphys_quad.inc", "ackphys_scene.inc", "ackphys_ppo.inc", "ackppo_math.inc",
            "ackphys_model_gen.h", "ackphys_scene_gen.h", "ackphys.h", "ackphys_model.h", "ackppo.h"} <= names
    assert os.path.basename(_lib.SOURCES[0]) == "ackphys_step.hip"
    assert {os.path.basename(s) for s in _lib.PPO_SOURCES} == {"ackppo.hip", "ackppo.h", "ackppo_math.inc"}


def test_create_rejects_wrong_blob():
    L = _lib.lib()
    ctx = C.c_void_p()
    bad = bytearray(_lib.load_blob())
    bad[-1] ^= 0xFF
    rc = L.ackphys_create(bytes(bad), len(bad), 16, 0, C.byref(ctx))
    assert rc == -2 and b"specialised" in L.ackphys_last_error()
    rc = L.ackphys_create(b"\0" * 8, 8, 16, 0, C.byref(ctx))
    assert rc == -2


def test_rollout_rejects_bad_arguments_without_touching_the_gpu():
    """ackphys_rollout validates its arguments before any HIP call (EINVAL + message)."""
    L = _lib.lib()
    P = C.c_void_p
    dummy = P(16)  # never dereferenced: every call below fails validation first
    rc = L.ackphys_rollout(None, 4, dummy, dummy, dummy, dummy, dummy, dummy, None, None, None, 0, 0, 0, None)
    assert rc == -1 and b"NULL" in L.ackphys_last_error()
    # a fake (non-NULL) context is only ever compared, never followed, before k_steps is checked
    rc = L.ackphys_rollout(dummy, 0, dummy, dummy, dummy, dummy, dummy, dummy, None, None, None, 0, 0, 0, None)
    assert rc == -1 and b"k_steps" in L.ackphys_last_error()
    rc = L.ackphys_rollout(dummy, 3, None, dummy, dummy, dummy, dummy, dummy, None, None, None, 0, 0, 0, None)
    assert rc == -1 and b"NULL" in L.ackphys_last_error()


def test_ctypes_structs_match_the_c_layouts(tmp_path):
    """The ctypes mirrors of the C-ABI structs (_lib.TrainDesc = ackppo_train_desc, _lib.EnvParams =
    ackphys_env_params) have the C compiler's size and field offsets: a mismatch hands the library
    garbage (a misplaced field once read a scratch pointer as the all-reduce hook)."""
    import subprocess
    checks = {"ackppo_train_desc": ("ackppo.h", _lib.TrainDesc), "ackphys_env_params": ("ackphys.h", _lib.EnvParams)}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "include/ackppo.h"', '#include "include/ackphys.h"',
           "int main(void) {"]
    for cname, (_, py) in checks.items():
        src.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _t in py._fields_:
            src.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    src.append("  return 0;\n}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", _lib.REPO, str(c), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.splitlines())
    for cname, (_, py) in checks.items():
        assert int(got[f"{cname} size"]) == C.sizeof(py), cname
        for f, _t in py._fields_:
            assert int(got[f"{cname} {f}"]) == getattr(py, f).offset, (cname, f)


def test_weight_image_size_matches_the_header():
    """_lib.ACKPPO_WIMAGE (the PPO learner's weight-image buffer, floats per net) = include/ackppo.h."""
    import re
    with open(os.path.join(_lib.REPO, "include", "ackppo.h")) as f:
        m = re.search(r"#define ACKPPO_WIMAGE (\d+)", f.read())
    assert m and int(m.group(1)) == _lib.ACKPPO_WIMAGE
