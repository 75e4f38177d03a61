"""Host probe: how often MuJoCo's Newton-start rule picks qacc_smooth over qacc_warmstart in the
f64 oracle on the bench workload (random actions, contacts off / on). Needs an instrumented oracle
build exporting or_pick_w / or_pick_s:  python tools/probes/warm_choice_probe.py /path/lib.so"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle.oracle as om  # noqa: E402
from mujoco_playground_amd import _lib  # noqa: E402

om.LIB_PATH = sys.argv[1]
om.build = lambda force=False: om.LIB_PATH
L = om.lib()
L.or_pick_w.restype = C.c_long
L.or_pick_s.restype = C.c_long
n = 512
for contacts in (0, 1):
    o = om.Oracle(_lib.load_blob())
    st = np.zeros((n, 44))
    o.reset(st, seed=0)
    rng = np.random.default_rng(0)
    w0, s0 = L.or_pick_w(), L.or_pick_s()
    for k in range(80):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        o.step(st, a, flags=2 | contacts, seed=0)
        if k in (9, 39, 79):
            w, s = L.or_pick_w() - w0, L.or_pick_s() - s0
            print(f"contacts={contacts} steps<={k + 1}: warm {w} smooth {s} ({100 * s / (w + s):.1f}% smooth)")
