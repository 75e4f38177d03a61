"""ctypes front-end of the CPU oracle (oracle/ackphys_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package (mujoco_playground_amd).

Every function mirrors a reference call path (file:line in ackphys_oracle.c's header):
  step()        AckermannRobotEnv.step      src/rl/envs/ackermann_env.py:187-229
  reset()       AckermannRobotEnv.reset     src/rl/envs/ackermann_env.py:143-185
  controller()  BicycleController           src/core/controller.py:98-140
Physics parity is UNPINNED (no MuJoCo in this image); see DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libackphys_oracle.so")

NSTATE, NOBS = 44, 79
FLAG_CONTACTS, FLAG_AUTORESET, FLAG_POSTSTEP_OBS = 1, 2, 4
DIAG_LEN = 8192


def build(force: bool = False) -> str:
    """make (incremental: rebuilds when ackphys_oracle.c or a header it includes changed)."""
    subprocess.run(["make", "-C", HERE] + (["-B"] if force else []), check=True, capture_output=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P, i32, u32, u64, f64p = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.POINTER(C.c_double)
        L.or_create.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(P)]
        L.or_destroy.argtypes = [P]
        L.or_last_error.restype = C.c_char_p
        L.or_set_solver.argtypes = [P, C.c_double, i32]
        L.or_set_env_offset.argtypes = [P, i32]
        L.or_step_batch.argtypes = [P, i32, P, P, u32, u64, P, P, P, P, P, P, i32]
        L.or_reset_batch.argtypes = [P, i32, P, u64, P, P]
        L.or_step_diag.argtypes = [P, P, P, u32, P]
        L.or_step_diag.restype = i32
        L.or_controller.argtypes = [P, P]
        L.or_controller2.argtypes = [P, C.c_double, C.c_double, P]
        L.or_set_env_params.argtypes = [P, i32, C.c_double, C.c_double, C.c_double, C.c_double]
        L.or_set_env_variant.argtypes = [P, i32, i32]
        L.or_set_goal_cells.argtypes = [P, i32]
        L.or_set_kink_snap.argtypes = [i32]
        L.or_philox.argtypes = [P, P, P]
        L.or_model_struct_size.restype = i32
        L.or_observe_raw.argtypes = [P, P, P, P, P, P, P, P, P, P]
        L.ackphys_step_cpu.argtypes = [P, i32] + [P] * 9 + [u32, u64, i32]
        L.ackphys_reset_cpu.argtypes = [P, i32, P, u64, P, P]
        L.or_contacts.argtypes = [P, P, P, i32]
        L.or_contacts.restype = i32
        L.or_ray.argtypes = [P, P, P, P]
        L.or_ray.restype = C.c_double
        L.or_hull_features.argtypes = [P, i32, P, P, P, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
    def __init__(self, blob: bytes):
        L = lib()
        self._ctx = C.c_void_p()
        rc = L.or_create(blob, len(blob), C.byref(self._ctx))
        if rc:
            raise RuntimeError(f"or_create failed ({rc}): {L.or_last_error().decode()}")

    def __del__(self):
        if getattr(self, "_ctx", None) and _lib is not None:
            _lib.or_destroy(self._ctx)
            self._ctx = None

    def set_solver(self, tolerance: float = 1e-12, maxiter: int = 100):
        lib().or_set_solver(self._ctx, tolerance, maxiter)

    def set_env_params(self, max_episode_steps=1000, goal_distance_threshold=0.5, collision_threshold=0.15,
                       max_linear_velocity=1.0, max_angular_velocity=1.0, action_repeat=1, nohit_clear=False,
                       goal_cells=0):
        lib().or_set_env_params(self._ctx, max_episode_steps, goal_distance_threshold, collision_threshold,
                                max_linear_velocity, max_angular_velocity)
        lib().or_set_env_variant(self._ctx, int(action_repeat), int(bool(nohit_clear)))
        if lib().or_set_goal_cells(self._ctx, int(goal_cells)) != 0:
            raise ValueError("goal_cells needs the obstacle scene (a world of static boxes)")

    def set_env_offset(self, off: int):
        lib().or_set_env_offset(self._ctx, off)

    def step(self, states: np.ndarray, actions: np.ndarray, flags: int = FLAG_CONTACTS, seed: int = 0,
             nthreads: int = 0, terminal: bool = False):
        """states float64 [n,44] updated in place; actions float32 [n,2]."""
        assert states.dtype == np.float64 and states.flags.c_contiguous and states.shape[1] == NSTATE
        n = states.shape[0]
        actions = np.ascontiguousarray(actions, dtype=np.float32).reshape(n, 2)
        obs = np.zeros((n, NOBS))
        rew = np.zeros(n)
        term = np.zeros(n, np.uint8)
        trunc = np.zeros(n, np.uint8)
        tobs = np.zeros((n, NOBS)) if terminal else None
        info = np.zeros((n, 4))
        lib().or_step_batch(self._ctx, n, _p(states), _p(actions), flags, seed, _p(obs), _p(rew), _p(term),
                            _p(trunc), _p(tobs), _p(info), nthreads)
        return obs, rew, term.astype(bool), trunc.astype(bool), tobs, info

    def reset(self, states: np.ndarray, mask=None, seed: int = 0):
        n = states.shape[0]
        obs = np.zeros((n, NOBS))
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        lib().or_reset_batch(self._ctx, n, _p(m), seed, _p(states), _p(obs))
        return obs

    def observe_raw(self, xpos, xquat, sensordata, goal, ref):
        """(obs[79], reward, terminated, (min_lidar, collision, goal_distance)) from raw mjData."""
        f = lambda x: np.ascontiguousarray(x, dtype=np.float64)
        obs, rew, term, info = np.zeros(NOBS), np.zeros(1), C.c_int(0), np.zeros(3)
        lib().or_observe_raw(self._ctx, _p(f(xpos)), _p(f(xquat)), _p(f(sensordata)), _p(f(goal)), _p(f(ref)),
                             _p(obs), _p(rew), C.byref(term), _p(info))
        return obs, float(rew[0]), bool(term.value), info

    def contacts(self, qpos) -> np.ndarray:
        """mj_collision at qpos: [ncon, 16] = geom1, geom2, dist, pos[3], frame[9], dim."""
        q = np.ascontiguousarray(qpos, dtype=np.float64)
        out = np.zeros((64, 16))
        n = lib().or_contacts(self._ctx, _p(q), _p(out), 64)
        return out[:n].copy()

    def ray(self, qpos, pnt, vec) -> float:
        f = lambda x: np.ascontiguousarray(x, dtype=np.float64)
        return float(lib().or_ray(self._ctx, _p(f(qpos)), _p(f(pnt)), _p(f(vec))))

    def hull_features(self, mesh: int):
        fn, ed = np.zeros((96, 3)), np.zeros((96, 3))
        nf, ne = C.c_int(0), C.c_int(0)
        lib().or_hull_features(self._ctx, mesh, _p(fn), _p(ed), C.byref(nf), C.byref(ne))
        return fn[: nf.value].copy(), ed[: ne.value].copy()

    def diag(self, state: np.ndarray, ctrl, flags: int = FLAG_CONTACTS, nv: int = 12, nq: int = 13,
             nsensordata: int = 77) -> dict:
        st = np.ascontiguousarray(state, dtype=np.float64)
        ct = np.zeros(4)
        ct[: len(ctrl)] = ctrl
        out = np.zeros(DIAG_LEN)
        n = lib().or_step_diag(self._ctx, _p(st), _p(ct), flags, _p(out))
        o = 0
        r = {}

        def take(name, k, shape=None):
            nonlocal o
            v = out[o:o + k].copy()
            o += k
            r[name] = v.reshape(shape) if shape else v

        take("qM", nv * nv, (nv, nv))
        for f in ["qfrc_bias", "qfrc_passive", "qfrc_actuator", "qacc_smooth", "qacc", "qfrc_constraint"]:
            take(f, nv)
        take("counts", 3)
        r["ncon"], r["nefc"], r["niter"] = (int(x) for x in r.pop("counts"))
        take("contacts", 32 * 5, (32, 5))
        r["contacts"] = r["contacts"][: r["ncon"]]
        take("sensordata", nsensordata)
        take("xpos_chassis", 3)
        take("xquat_chassis", 4)
        take("subtree_com", 3)
        take("efc", 96 * 6, (96, 6))
        r["efc"] = r["efc"][: r["nefc"]]
        take("efc_J", 96 * nv, (96, nv))
        r["efc_J"] = r["efc_J"][: r["nefc"]]
        take("qpos_next", nq)
        take("qvel_next", nv)
        assert o == n, (o, n)
        return r


def controller(action, max_linear_velocity: float = 1.0, max_angular_velocity: float = 1.0) -> np.ndarray:
    a = np.ascontiguousarray(action, dtype=np.float32).reshape(2)
    out = np.zeros(3)
    lib().or_controller2(_p(a), max_linear_velocity, max_angular_velocity, _p(out))
    return out


def philox(counter, key) -> np.ndarray:
    c = np.ascontiguousarray(counter, dtype=np.uint32).reshape(4)
    k = np.ascontiguousarray(key, dtype=np.uint32).reshape(2)
    out = np.zeros(4, np.uint32)
    lib().or_philox(_p(c), _p(k), _p(out))
    return out
