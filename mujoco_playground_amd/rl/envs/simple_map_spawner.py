"""SimpleMapSpawner: the reference's per-reset scene loader (src/rl/envs/simple_map_spawner.py:22-54)
for the batched simulator.

The reference recompiles `models/ackermann_robot_v2.xml` on every reset (`MjModel.from_xml_path`,
:37), sets the free joint to robot_pos / identity quaternion (:43-50) and runs `mj_forward` (:52).
Here the scene is compiled once, offline (`model/compiler.py` -> the committed `.apm` blob the
kernels are specialised on), and the spawn pose is the reset kernel's (`ackphys_reset`: the
same (0, 0, 0.1) / identity pose, zero velocities, observation at the reset state). The spawner
therefore only names the scene; `load_random_environment` returns the compiled blob in the
reference's (model, data, map_name) shape, with data None (the per-env state lives on the GPU).
"""
from __future__ import annotations

from ... import _lib

_MAP_NAMES = {"flat": "simple_floor", "obstacles": "ackermann_maze_flat"}
SPAWN_POS = (0.0, 0.0, 0.1)  # simple_map_spawner.py:43 / ackermann_env.py:151


class SimpleMapSpawner:
    def __init__(self, scene: str = "flat"):
        if scene not in _MAP_NAMES:
            raise ValueError(f"unknown scene {scene!r} (one of {sorted(_MAP_NAMES)})")
        self.scene = scene

    @property
    def map_name(self) -> str:
        return _MAP_NAMES[self.scene]

    def load_random_environment(self, robot_pos=None, robot_quat=None):
        """(model blob, None, map_name). robot_pos / robot_quat are accepted for the reference's call
        shape (:22); the reset kernel's spawn pose is compiled in (flat scene: SPAWN_POS, the
        reference's; obstacle scene: the flat file's free cell) and the reference
        ignores robot_quat too ("random orientation" is not implemented, :44-50)."""
        return _lib.load_blob(self.scene), None, self.map_name
