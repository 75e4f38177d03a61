"""Generate golden vectors from the REFERENCE's own Python (run in the build container only).

    python tests/golden/make_golden.py [--reference /root/reference]

mujoco / gymnasium are not installable here (ModuleNotFoundError, not a
permission denial), so throwaway stand-in modules are placed on sys.path that provide only the
names the reference glue touches (mj_name2id, mjtObj, a no-op mj_step that swaps in the next
pre-generated forward data, gymnasium.Env/spaces.Box). The reference's OWN code then runs
unmodified:
  src/core/controller.py   BicycleController.cmd_vel_to_controls / apply_cmd_vel (:98-140)
  src/core/odometry.py     Odometry.calculate_odom / _quat_to_yaw (:62-103, :154-170)
  src/rl/envs/ackermann_env.py  AckermannRobotEnv.reset / step / _setup_lidar /
                                _get_observation / _calculate_reward (:126-312)
and its inputs/outputs are saved as tests/golden/reference_glue.npz. Physics (mj_step) is NOT
covered by these vectors (parity unpinned). Name lookups use the compiled
model's names (lidar-00..lidar-71): the stub mj_name2id returns -1 for unknown names, as the
real bindings do, so the reference's own aliasing (sensor_adr[-1]) is reproduced.
Also decodes the checkpoint pins (rl_logs/ppo/*.zip:data, JSON + pickletools opcode walk;
nothing is unpickled) into tests/golden/checkpoint_obs.npz.
"""
from __future__ import annotations

import argparse
import base64
import importlib.util
import io
import json
import os
import pickletools
import random
import sys
import types
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def install_stubs(model_names):
    mj = types.ModuleType("mujoco")

    class mjtObj:
        mjOBJ_BODY, mjOBJ_SITE, mjOBJ_SENSOR, mjOBJ_ACTUATOR = "body", "site", "sensor", "actuator"

    def mj_name2id(model, objtype, name):
        try:
            return model.names[objtype].index(name)
        except ValueError:
            return -1

    mj.mjtObj = mjtObj
    mj.mj_name2id = mj_name2id
    mj.mj_step = lambda model, data: data.advance()
    mj.mj_forward = lambda model, data: None
    viewer = types.ModuleType("mujoco.viewer")
    viewer.launch_passive = lambda *a, **k: None
    mj.viewer = viewer
    sys.modules["mujoco"] = mj
    sys.modules["mujoco.viewer"] = viewer

    gym = types.ModuleType("gymnasium")

    class Env:
        def reset(self, seed=None, options=None):
            return None

    class Box:
        def __init__(self, low, high, shape, dtype):
            self.low = np.full(shape, low, dtype=dtype)
            self.high = np.full(shape, high, dtype=dtype)
            self.shape = shape
            self.dtype = dtype

    sp = types.ModuleType("gymnasium.spaces")
    sp.Box = Box
    gym.Env = Env
    gym.spaces = sp
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = sp


class StubModel:
    def __init__(self, cm):
        self.names = {"body": list(cm.body_name), "site": list(cm.site_name), "sensor": list(cm.sensor_name),
                      "actuator": list(cm.actuator_name)}
        self.sensor_adr = np.array(cm.sensor_adr, dtype=np.int32)


class StubData:
    """Holds what mj_forward would leave in mjData; mj_step swaps in the next frame."""

    def __init__(self, frames):
        self.frames = frames
        self.k = 0
        self.ctrl = np.zeros(3)
        self.ctrl_log = []
        self._load(0)

    def _load(self, k):
        f = self.frames[k]
        self.xpos = np.zeros((11, 3))
        self.xquat = np.zeros((11, 4))
        self.xquat[:, 0] = 1
        self.xpos[1] = f["xpos"]
        self.xquat[1] = f["xquat"]
        self.sensordata = f["sensordata"].copy()

    def advance(self):
        self.ctrl_log.append(self.ctrl.copy())
        self.k += 1
        self._load(self.k)


class StubSpawner:
    def __init__(self, model, data):
        self.model, self.data = model, data

    def load_random_environment(self, robot_pos=None, robot_quat=None):
        return self.model, self.data, "simple_floor"


def make_frames(rng, n):
    frames = [{"xpos": np.array([0.0, 0.0, 0.1]), "xquat": np.array([1.0, 0, 0, 0]),
               "sensordata": np.concatenate([np.zeros(5), -np.ones(72)])}]
    for k in range(n):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = rng.uniform(-0.3, 0.3) if k % 3 else rng.uniform(-np.pi, np.pi)
        yaw = rng.uniform(-np.pi, np.pi)
        qz = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
        qt = np.array([np.cos(ang / 2), *(np.sin(ang / 2) * ax)])
        w1, x1, y1, z1 = qz
        w2, x2, y2, z2 = qt
        q = np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                      w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])
        sd = rng.uniform(0.05, 12.0, 77)
        mode = k % 4
        if mode == 0:
            sd[5:] = -1.0
        elif mode == 1:
            sd[5 + rng.integers(0, 72, 20)] = -1.0
        elif mode == 2:
            sd[5:] = rng.uniform(0.2, 12.0, 72)
        sd[:5] = rng.normal(size=5)
        pos = np.array([rng.uniform(-8, 8), rng.uniform(-8, 8), 0.065 + rng.normal() * 0.01])
        frames.append({"xpos": pos, "xquat": q, "sensordata": sd})
    return frames


def make_actions(rng, n):
    a = rng.uniform(-1.3, 1.3, (n, 2)).astype(np.float32)
    special = np.array([[0, 0], [1, 0], [0, 1], [0, -1], [1e-6, 0.5], [-1e-6, -0.5], [0.5, 3e-6], [0.5, 6e-6],
                        [1.0, 2e-5], [-1.0, 2e-5], [0.3, -1e-5], [1, 1], [-1, -1], [2, -2], [1e-7, 1e-7],
                        [0.9, 0.0000009], [0.0, 0.7], [-0.2, 0.2]], dtype=np.float32)
    a[: len(special)] = special
    return a


def gen_glue(reference, n=240, seed=1234):
    from mujoco_playground_amd.model.compiler import compile_mjcf, default_model_path
    cm = compile_mjcf(default_model_path(reference))
    install_stubs(None)
    sys.path.insert(0, os.path.join(reference, "src"))
    spec = importlib.util.spec_from_file_location("ref_ackermann_env",
                                                  os.path.join(reference, "src", "rl", "envs", "ackermann_env.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(seed)
    frames = make_frames(rng, n)
    actions = make_actions(rng, n)
    model = StubModel(cm)
    data = StubData(frames)
    env = mod.AckermannRobotEnv(map_spawner=StubSpawner(model, data))
    random.seed(seed)
    obs0, info0 = env.reset()
    out = {k: [] for k in ["obs", "reward", "terminated", "truncated", "goal_distance", "collision", "min_lidar"]}
    env.max_episode_steps = n - 40  # exercise truncation inside the vector set
    for k in range(n):
        obs, r, te, tr, info = env.step(actions[k])
        out["obs"].append(obs)
        out["reward"].append(r)
        out["terminated"].append(te)
        out["truncated"].append(tr)
        out["goal_distance"].append(info["goal_distance"])
        out["collision"].append(info["collision"])
        out["min_lidar"].append(info["min_lidar"])
    res = {
        "actions": actions, "ctrl": np.array(data.ctrl_log), "reset_obs": obs0,
        "goal": np.array(info0["goal_position"]), "ref": np.array([0.0, 0.0, 0.1]),
        "xpos": np.array([f["xpos"] for f in frames[1:]]), "xquat": np.array([f["xquat"] for f in frames[1:]]),
        "sensordata": np.array([f["sensordata"] for f in frames[1:]]), "lidar_addrs": np.array(env.lidar_addrs),
        "max_episode_steps": np.array(env.max_episode_steps),
        **{k: np.array(v) for k, v in out.items()},
    }
    return res


def decode_checkpoint_obs(reference):
    """_last_obs of each SB3 checkpoint: JSON member 'data' -> base64 cloudpickle bytes ->
    pickletools.genops (opcode walk, nothing executed) -> largest bytes operand as <f4[79]."""
    out = {}
    for steps in (10000, 20000, 30000):
        p = os.path.join(reference, "rl_logs", "ppo", f"ppo_model_{steps}_steps.zip")
        d = json.loads(zipfile.ZipFile(p).read("data"))
        raw = base64.b64decode(d["_last_obs"][":serialized:"])
        best = b""
        for op, arg, _ in pickletools.genops(io.BytesIO(raw)):
            if isinstance(arg, (bytes, bytearray)) and len(arg) > len(best):
                best = bytes(arg)
        obs = np.frombuffer(best[-79 * 4:], dtype="<f4").copy()
        out[f"obs_{steps}"] = obs
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    res = gen_glue(a.reference)
    np.savez_compressed(os.path.join(HERE, "reference_glue.npz"), **res)
    ck = decode_checkpoint_obs(a.reference)
    np.savez_compressed(os.path.join(HERE, "checkpoint_obs.npz"), **ck)
    print("wrote reference_glue.npz", {k: v.shape for k, v in res.items()})
    print("wrote checkpoint_obs.npz", {k: v[:3] for k, v in ck.items()})
