"""Find a finite state whose step trips mj_checkAcc in the oracle (host-only probe)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd import _lib  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

o = Oracle(_lib.load_blob())
st = np.zeros((4, 44))
o.reset(st, seed=4)
for v in [1e6, 1e8, 1e9, 5e9]:
    s = st.copy()
    s[:, 13 + 6:13 + 12] = v
    s[:, 13 + 3] = v / 10
    r = o.step(s, np.full((4, 2), 0.3, np.float32), flags=3, seed=4, terminal=True)
    print(v, "qpos", s[0, :7], "max|qvel|", np.abs(s[0, 13:25]).max(), "extra", r[5])
