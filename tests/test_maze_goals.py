"""The opt-in maze goals (NOT the reference env; ackphys_env_params.goal_cells, obstacle scene):
each reset draws the goal at the centre of a box-free grid cell 4-connected to the spawn cell and
within goal_cells breadth-first cells of it (include/ackphys.h).

CPU side, two independent restatements pinned to each other: the scene codegen's Python
breadth-first search (model/codegen.py maze_free_cells -> csrc/ackphys_scene_gen.h FREE_XY /
FREE_LE, the table the kernels read) and the oracle's C one (oracle/ackphys_oracle.c free_cells,
computed from the blob's box geoms); the oracle's goals are the header's cells picked by the
integer draw floor((philox word >> 8) * FREE_LE[d] / 2^24). The GPU tests hold the kernels'
reset and auto-reset goals to the oracle (tests/test_gpu_variant.py).
"""
import os
import re

import numpy as np
import pytest

from mujoco_playground_amd import _lib
from mujoco_playground_amd.sim import ST_GOAL

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mujoco_playground_amd", "csrc",
                   "ackphys_scene_gen.h")


def header_table():
    s = open(HDR).read()
    n = int(re.search(r"constexpr int NFREE = (\d+), FREE_MAXD = (\d+);", s).group(1))
    maxd = int(re.search(r"FREE_MAXD = (\d+);", s).group(1))
    xy = re.search(r"FREE_XY\[\d+\]\[2\] = \{(.*?)\};", s, re.S).group(1)
    xy = np.array([float(v.rstrip("f")) for v in re.findall(r"[-0-9.e+]+f", xy)]).reshape(-1, 2)
    le = [int(v) for v in re.search(r"FREE_LE\[\d+\] = \{(.*?)\}", s).group(1).split(",")]
    sp = re.search(r"SPAWN\[3\] = \{(.*?)\};", s).group(1)
    spawn = np.array([float(v.rstrip("f")) for v in re.findall(r"[-0-9.e+]+f", sp)])
    assert xy.shape == (n, 2) and len(le) == maxd + 1 and le[-1] == n
    return xy, le, spawn


def _oracle(scene, **params):
    from oracle.oracle import Oracle
    o = Oracle(_lib.load_blob(scene))
    o.set_env_params(**params)
    return o


def test_header_table_is_a_breadth_first_maze():
    """Every listed cell is box-free, not the spawn cell, one step from a cell one step nearer
    (or from the spawn cell), and the list is sorted by distance."""
    xy, le, spawn = header_table()
    s = open(HDR).read()
    lo = np.array([float(v.rstrip("f")) for v in re.findall(r"[-0-9.e+]+f",
                   re.search(r"BOX_LO\[\d+\]\[3\] = \{(.*?)\};", s, re.S).group(1))]).reshape(-1, 3)
    hi = np.array([float(v.rstrip("f")) for v in re.findall(r"[-0-9.e+]+f",
                   re.search(r"BOX_HI\[\d+\]\[3\] = \{(.*?)\};", s, re.S).group(1))]).reshape(-1, 3)
    for c in xy:
        inside = (lo[:, 0] < c[0]) & (c[0] < hi[:, 0]) & (lo[:, 1] < c[1]) & (c[1] < hi[:, 1])
        assert not inside.any(), f"cell {c} lies in a box"
    d = np.concatenate([np.full(le[k] - (le[k - 1] if k else 0), k) for k in range(len(le))])
    assert d[0] == 1 and np.all(np.diff(d) >= 0)
    cell = float(np.min(hi[:, :2] - lo[:, :2]))
    centre0 = lo[:, :2].min(axis=0) + cell * (np.floor((spawn[:2] - lo[:, :2].min(axis=0)) / cell) + 0.5)
    assert not np.any(np.all(np.isclose(xy, centre0), axis=1)), "the spawn cell is not a goal"
    for i in range(len(xy)):
        prev = np.vstack([centre0[None], xy[d == d[i] - 1]]) if d[i] == 1 else xy[d == d[i] - 1]
        steps = np.abs(prev - xy[i]).sum(axis=1) / cell
        assert np.any(np.isclose(steps, 1.0)), f"cell {i} (distance {d[i]}) has no neighbour one step nearer"


@pytest.mark.parametrize("goal_cells", [1, 2, 3, 6, 10, 50])
def test_oracle_goals_are_the_header_cells(goal_cells):
    """The oracle's free-cell goals equal the kernels' table entry the integer draw selects, for
    every env and episode (independent BFS restatements agree cell for cell, in the same order)."""
    from oracle.oracle import philox
    xy, le, spawn = header_table()
    n, seed = 512, 77
    o = _oracle("obstacles", goal_cells=goal_cells)
    st = np.zeros((n, 44))
    for ep in range(3):
        o.reset(st, seed=seed)  # each reset bumps the episode counter
        nle = le[min(goal_cells, len(le) - 1)]
        for e in range(0, n, 37):
            c = philox(np.array([e, ep + 1, 0, 0], np.uint32), np.array([seed & 0xFFFFFFFF, seed >> 32], np.uint32))
            i = (int(c[0]) >> 8) * nle >> 24
            np.testing.assert_allclose(st[e, ST_GOAL:ST_GOAL + 2], xy[i] - spawn[:2], atol=1e-6)


def test_goal_cells_default_is_the_reference():
    o_ref, o_var = _oracle("obstacles"), _oracle("obstacles", goal_cells=0)
    a, b = np.zeros((64, 44)), np.zeros((64, 44))
    o_ref.reset(a, seed=3)
    o_var.reset(b, seed=3)
    assert np.array_equal(a, b)
    r = np.hypot(a[:, ST_GOAL], a[:, ST_GOAL + 1])
    assert r.min() >= 2.0 and r.max() <= 8.0  # ackermann_env.py:167


def test_goal_cells_refused_without_boxes():
    with pytest.raises(ValueError):
        _oracle("flat", goal_cells=3)
