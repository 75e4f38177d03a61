"""CPU probe: how often can the final constraint active set of a step be predicted before the solve?

Runs the f64 oracle on the benchmark workload (uniform random actions from reset) and, for every
env-step after a warm-up, compares the row states at the oracle's optimum (equality: always
quadratic; friction loss: lower-linear / quadratic / upper-linear; limits and contacts: active or
not) with the states predicted by
  warm   : the rows at qacc_warmstart with this step's aref (= the Newton's first iteration from it)
  smooth : the rows at qacc_smooth
  oned   : each friction-loss row as a one-dof problem at qacc_smooth moved onto the steering
           equality: quadratic zone iff |x| <= R floss + floss invweight
  kernel : oned, with the two steer rows from the exact two-dof sub-problem (diagonal masses,
           equality row, both Huber rows) -- the contacts-off kernel's rule
and, with --contacts 1, "kernel+contacts": the kernel rule for the scalar rows plus pyramid-edge
states from the steer-projected qacc_smooth ("kernel" then scores the scalar rows alone). The
contact kernels do not use a prediction: too few hits.
If a prediction is right, one solve of that piece's quadratic is the exact optimum (convexity).

    python tools/probes/active_set_probe.py [--envs 256] [--steps 200] [--warm 60] [--contacts 0]
"""
import argparse
import itertools
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402
from oracle.oracle import FLAG_AUTORESET, FLAG_CONTACTS, Oracle, controller  # noqa: E402

FRICTIONLOSS = np.array([0, 0, 0, 0, 0, 0, 0.02, 0.02, 0.005, 0.012, 0.005, 0.012])
STEER = (8, 10)  # the equality's dofs (fl_steer = fr_steer)


def states(typ, R, fl, x):
    s = np.zeros(len(typ), int)
    f1 = typ == 1
    s[f1 & (x <= -R * fl)] = -1
    s[f1 & (x >= R * fl)] = 1
    s[(typ >= 2) & (x < 0)] = 1
    return s


def pair_states(M, a0, D, R, fl, aref, J, typ, i1, i2, ie, guess):
    """exact states of the steer pair's two-dof sub-problem; the one-dof guess first"""
    c = J[ie, STEER[1]] / J[ie, STEER[0]]
    m1, m2 = M[STEER[0], STEER[0]], M[STEER[1], STEER[1]]
    ae = aref[ie] / J[ie, STEER[0]]
    for s1, s2 in [guess] + list(itertools.product((-1, 0, 1), repeat=2)):
        H = np.diag([m1, m2]) + D[ie] * np.outer([1, c], [1, c])
        b = np.array([m1 * a0[STEER[0]], m2 * a0[STEER[1]]]) + D[ie] * ae * np.array([1, c])
        for k, (s, i) in enumerate(((s1, i1), (s2, i2))):
            if s == 0:
                H[k, k] += D[i]
                b[k] += D[i] * aref[i]
            else:
                b[k] -= s * fl[i]
        a = np.linalg.solve(H, b)
        t = states(typ[[i1, i2]], R[[i1, i2]], fl[[i1, i2]], a - aref[[i1, i2]])
        if (t[0], t[1]) == (s1, s2):
            return s1, s2
    return guess


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warm", type=int, default=60)
    ap.add_argument("--contacts", type=int, default=0)
    a = ap.parse_args()
    o = Oracle(_lib.load_blob())
    n = a.envs
    st = np.zeros((n, 44))
    o.reset(st, seed=3)
    rng = np.random.default_rng(0)
    fl_c = FLAG_CONTACTS if a.contacts else 0
    names = ("warm", "smooth", "oned", "kernel") + (("kernel+contacts",) if a.contacts else ())
    hits = {k: 0 for k in names}
    total = 0
    for k in range(a.steps):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        for e in range(n):
            if k < a.warm:
                continue
            d = o.diag(st[e], controller(act[e]), flags=fl_c)
            total += 1
            if d["nefc"] == 0:
                for kk in names:
                    hits[kk] += 1
                continue
            efc, J = d["efc"], d["efc_J"]
            typ = efc[:, 0].astype(int)
            R, aref, invw = efc[:, 2], efc[:, 3], efc[:, 5]
            D = 1.0 / R
            dofs = np.array([int(np.argmax(np.abs(j))) for j in J])
            fl = np.where(typ == 1, FRICTIONLOSS[dofs], 0.0)
            M, a0 = d["qM"], d["qacc_smooth"]
            fin = states(typ, R, fl, J @ d["qacc"] - aref)
            pred = {"warm": states(typ, R, fl, J @ st[e, 25:37] - aref), "smooth": states(typ, R, fl, J @ a0 - aref)}
            ap_ = a0.copy()
            w1, w2 = M[STEER[0], STEER[0]], M[STEER[1], STEER[1]]
            ap_[STEER[0]] = ap_[STEER[1]] = (w1 * a0[STEER[0]] + w2 * a0[STEER[1]]) / (w1 + w2)
            xp = J @ ap_ - aref
            thr = R * fl + fl * invw
            oned = np.where(typ == 1, np.where(xp < -thr, -1, np.where(xp > thr, 1, 0)), states(typ, R, fl, xp))
            pred["oned"] = oned
            kern = oned.copy()
            i1 = np.nonzero((typ == 1) & (dofs == STEER[0]))[0][0]
            i2 = np.nonzero((typ == 1) & (dofs == STEER[1]))[0][0]
            ie = np.nonzero(typ == 0)[0][0]
            kern[i1], kern[i2] = pair_states(M, a0, D, R, fl, aref, J, typ, i1, i2, ie, (oned[i1], oned[i2]))
            pred["kernel"] = kern
            if a.contacts:
                pred["kernel+contacts"] = np.where(typ >= 3, states(typ, R, fl, xp), kern)
                pred["kernel"] = np.where(typ >= 3, fin, kern)  # scalar rows only
            for kk in names:
                hits[kk] += int(np.array_equal(pred[kk], fin))
        o.step(st, act, flags=fl_c | FLAG_AUTORESET, seed=3)
    for kk in names:
        print(f"{kk:16s} env-step hit rate {hits[kk] / max(total, 1):.5f}  ({total} env-steps)")


if __name__ == "__main__":
    main()
