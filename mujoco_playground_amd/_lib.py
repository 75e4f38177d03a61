"""Loader for libackphys.so (the HIP C-ABI, include/ackphys.h) and its in-tree build.

There is no CPU fallback: if the library is missing or cannot be loaded the product raises.
(The CPU oracle under oracle/ is test infrastructure and is never imported here.)
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB_PATH = os.path.join(CSRC, "build", "libackphys.so")
REPO = os.path.dirname(PKG)
_INCLUDE_RE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def source_closure(main: str) -> list:
    """`main` plus every file it reaches through quoted #include lines (resolved relative to the
    including file), so the rebuild check sees edits to any .inc / generated header."""
    seen, todo = [], [os.path.abspath(main)]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.append(f)
        with open(f, encoding="utf-8", errors="replace") as fh:
            for inc in _INCLUDE_RE.findall(fh.read()):
                todo.append(os.path.normpath(os.path.join(os.path.dirname(f), inc)))
    return seen


SOURCES = source_closure(os.path.join(CSRC, "ackphys_step.hip"))
BLOB_PATH = os.path.join(PKG, "model", "assets", "ackermann_robot_v2.apm")
# static-world scenes the kernels are specialised on: "flat" = ackermann_robot_v2.xml alone,
# "obstacles" = the v2 robot in models/environments/ackermann_maze_flat.xml
SCENES = {"flat": BLOB_PATH, "obstacles": os.path.join(PKG, "model", "assets", "ackermann_obstacles.apm")}
PPO_LIB_PATH = os.path.join(CSRC, "build", "libackppo.so")
PPO_SOURCES = source_closure(os.path.join(CSRC, "ackppo.hip"))

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-fast-math",
               "-Wno-unused-result"]
# Step kernels: no SLP vectorisation. At -O3 the compiler packs adjacent scalar f32 ops into
# v_pk_*_f32, which needs operand pairs in consecutive registers: in these register-bound,
# one-wave-per-SIMD kernels that cost more in moves and AGPR spills than it saved (nc kernel:
# 10.9k -> 9.4k static instructions, 1109 -> 357 v_mov; measured 14.78 -> 13.67 us per step,
# contacts-on quad 75.4 -> 70.1 us, obstacles 82.3 -> 76.6 us). The PPO kernels measured even, and
# share it so the policy code common to both libraries compiles alike.
PHYS_FLAGS = ["-fno-slp-vectorize"]


class ExtensionMissing(RuntimeError):
    pass


class EnvParams(C.Structure):
    """ackphys_env_params (include/ackphys.h) = AckermannRobotEnv.__init__ kwargs."""
    _fields_ = [("max_episode_steps", C.c_int32), ("goal_distance_threshold", C.c_double),
                ("collision_threshold", C.c_double), ("max_linear_velocity", C.c_double),
                ("max_angular_velocity", C.c_double),
                # opt-in task variants (NOT the reference; 1 / 0 = ackermann_env.py exactly)
                ("action_repeat", C.c_int32), ("nohit_clear", C.c_int32), ("goal_cells", C.c_int32)]


ACKPPO_WIMAGE = 9728  # floats per net of ackppo_train_desc::weight_image (include/ackppo.h)

# ackppo_allreduce_fn (include/ackppo.h): SUM all-reduce in place of (buf, count, dtype, user, stream)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p)


class TrainDesc(C.Structure):
    """ackppo_train_desc (include/ackppo.h): one PPO.train() call."""
    _fields_ = [("obs_rows", C.c_void_p), ("actions", C.c_void_p), ("old_log_prob", C.c_void_p),
                ("advantages", C.c_void_p), ("returns", C.c_void_p), ("n_idx", C.c_int), ("batch", C.c_int),
                ("n_epochs", C.c_int), ("perm_key", C.c_uint64), ("perm_epoch0", C.c_uint32),
                ("normalize_advantage", C.c_int), ("clip_range", C.c_float), ("ent_coef", C.c_float),
                ("vf_coef", C.c_float), ("max_grad_norm", C.c_float), ("learning_rate", C.c_double),
                ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_float), ("adam_step0", C.c_int64),
                ("params", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p), ("perm", C.c_void_p),
                ("stats", C.c_void_p), ("moments", C.c_void_p), ("grad_partial", C.c_void_p),
                ("loss_partial", C.c_void_p), ("grad", C.c_void_p), ("loss_acc", C.c_void_p),
                ("grad_norm_out", C.c_void_p), ("world", C.c_int), ("allreduce", C.c_void_p),
                ("allreduce_user", C.c_void_p), ("log_std_min", C.c_float),
                ("weight_image", C.c_void_p), ("perm_epochs", C.c_void_p), ("stats_epochs", C.c_void_p),
                ("moments_count", C.c_int64)]


def _hipcc(out: str, sources: list, verbose: bool, force: bool, extra: tuple = ()) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *HIPCC_FLAGS, *extra, "-o", out + ".tmp", sources[0]]
    # the compile command is part of the up-to-date check: a flag-only change rebuilds (a stale
    # library would silently skew kernel timings and register counts)
    stamp = out + ".cmd"
    cmd_text = " ".join(cmd) + "\n"
    if not force and os.path.exists(out) and os.path.exists(stamp):
        t = os.path.getmtime(out)
        with open(stamp) as f:
            same_cmd = f.read() == cmd_text
        if same_cmd and all(os.path.getmtime(s) <= t for s in sources):
            return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(cmd_text)
    if verbose:
        print(f"built {out}")
    return out


def build(verbose: bool = False, force: bool = False) -> str:
    """Compile the HIP sources for gfx950 into csrc/build/ (in-tree): libackphys.so (physics
    step, include/ackphys.h) and libackppo.so (PPO learner, include/ackppo.h)."""
    # both libraries with the same flags: the policy arithmetic they share (csrc/ackppo_math.inc)
    # then compiles alike, and the fused rollout's actions equal ackppo_act's bit for bit
    # libackppo opens the process's librccl.so.1 at run time (dlopen) for the trainer's collectives
    _hipcc(PPO_LIB_PATH, PPO_SOURCES, verbose, force, tuple(PHYS_FLAGS) + ("-ldl",))
    return _hipcc(LIB_PATH, SOURCES, verbose, force, tuple(PHYS_FLAGS))


EXPORTS = ["ackphys_create", "ackphys_destroy", "ackphys_set_env_params", "ackphys_set_variant", "ackphys_set_env_offset", "ackphys_step", "ackphys_rollout",
           "ackphys_ppo_rollout", "ackphys_reset",
           "ackphys_random_actions", "ackphys_model_fnv", "ackphys_last_error", "ackphys_version"]

PPO_EXPORTS = ["ackppo_act", "ackppo_act_boot", "ackppo_value", "ackppo_bootstrap", "ackppo_gae", "ackppo_adv_stats",
               "ackppo_adv_moments", "ackppo_adv_finalize", "ackppo_grad",
               "ackppo_grad_blocks", "ackppo_reduce", "ackppo_adam", "ackppo_epoch", "ackppo_permutation",
               "ackppo_train", "ackppo_rccl_unique_id", "ackppo_rccl_init", "ackppo_rccl_allreduce",
               "ackppo_rccl_destroy", "ackppo_rccl_library", "ackppo_last_error"]

_lib = None
_ppo = None


def lib():
    """The loaded C-ABI; raises ExtensionMissing if the HIP build is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ExtensionMissing(f"{LIB_PATH} not found: build it with `python -c \"import __graft_entry__ as g; "
                               f"g.build()\"` (hipcc --offload-arch=gfx950)")
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:
        raise ExtensionMissing(f"cannot load {LIB_PATH}: {e}") from e
    P, i32, i64, u32, u64, sz = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_size_t
    L.ackphys_create.argtypes = [C.c_char_p, sz, i32, i32, C.POINTER(P)]
    L.ackphys_destroy.argtypes = [P]
    L.ackphys_set_env_offset.argtypes = [P, i64]
    L.ackphys_set_variant.argtypes = [P, i32]
    L.ackphys_set_env_params.argtypes = [P, C.POINTER(EnvParams)]
    L.ackphys_step.argtypes = [P, P, P, P, P, P, P, P, P, P, u32, u64, P]
    L.ackphys_rollout.argtypes = [P, i32, P, P, P, P, P, P, P, P, P, u32, u64, i32, P]
    L.ackphys_ppo_rollout.argtypes = [P, P, i32, u32, u64, i32, C.c_float] + [P] * 15 + [u32, u64, P]
    L.ackphys_reset.argtypes = [P, P, u64, P, P, P]
    L.ackphys_random_actions.argtypes = [P, P, i32, u64, u32, P]
    L.ackphys_model_fnv.restype = u64
    L.ackphys_last_error.restype = C.c_char_p
    L.ackphys_version.restype = C.c_char_p
    _lib = L
    return L


def ppo_lib():
    """The PPO learner C-ABI (libackppo.so); raises ExtensionMissing if the HIP build is absent."""
    global _ppo
    if _ppo is not None:
        return _ppo
    if not os.path.exists(PPO_LIB_PATH):
        raise ExtensionMissing(f"{PPO_LIB_PATH} not found: build it with `python -c \"import __graft_entry__ as g; "
                               f"g.build()\"` (hipcc --offload-arch=gfx950)")
    try:
        L = C.CDLL(PPO_LIB_PATH)
    except OSError as e:
        raise ExtensionMissing(f"cannot load {PPO_LIB_PATH}: {e}") from e
    P, i32, i64, u32, u64, f32 = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_float
    L.ackppo_act.argtypes = [P, P, i32, i64, u64, u32, i32, P, P, P, P, P, P]
    L.ackppo_act_boot.argtypes = [P, P, i32, i64, u64, u32, i32, P, P, P, P, P, P, P, P, P, f32, P, P, P]
    L.ackppo_value.argtypes = [P, P, i32, P, P]
    L.ackppo_bootstrap.argtypes = [P, P, P, P, P, i32, f32, P, P, P]
    L.ackppo_gae.argtypes = [P, P, P, P, P, i32, i32, f32, f32, P, P, P]
    L.ackppo_adv_stats.argtypes = [P, P, i32, i32, i32, P, P]
    L.ackppo_adv_moments.argtypes = [P, P, i32, i32, i32, P, P]
    L.ackppo_adv_finalize.argtypes = [P, i32, i32, P, P]
    L.ackppo_grad.argtypes = [P, P, P, P, P, P, P, i32, P, f32, f32, f32, P, P, P]
    L.ackppo_grad_blocks.argtypes = [i32]
    L.ackppo_reduce.argtypes = [P, P, i32, f32, P, P, P]
    L.ackppo_adam.argtypes = [P, P, P, P, f32, f32, f32, f32, f32, f32, f32, P, P]
    L.ackppo_permutation.argtypes = [i32, u64, u32, P, P]
    L.ackppo_epoch.argtypes = ([P] * 7 + [i32, i32, P, f32, f32, f32, f32, C.c_double, C.c_double, C.c_double, f32,
                                          i64] + [P] * 8)
    L.ackppo_train.argtypes = [C.POINTER(TrainDesc), P]
    L.ackppo_rccl_unique_id.argtypes = [P]
    L.ackppo_rccl_init.argtypes = [P, i32, i32, C.POINTER(P)]
    L.ackppo_rccl_allreduce.argtypes = [P, i64, i32, P, P]
    L.ackppo_rccl_destroy.argtypes = [P]
    L.ackppo_rccl_library.argtypes = [C.c_char_p, i32]
    L.ackppo_last_error.restype = C.c_char_p
    _ppo = L
    return L


def ppo_check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {ppo_lib().ackppo_last_error().decode()}")


def load_blob(scene: str = "flat") -> bytes:
    if scene not in SCENES:
        raise ValueError(f"unknown scene {scene!r} (one of {sorted(SCENES)})")
    with open(SCENES[scene], "rb") as f:
        return f.read()


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {lib().ackphys_last_error().decode()}")
