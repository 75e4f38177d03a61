"""CPU probe: how often can the final constraint active set of a step be predicted before the solve?

Runs the f64 oracle on the benchmark workload (uniform random actions from reset) and, for every
env-step after a warm-up, compares the row states at the oracle's optimum (equality: always
quadratic; friction loss: lower-linear / quadratic / upper-linear; limits and contacts: active or
not) with the states predicted by
  warm   : the rows at qacc_warmstart with this step's aref (= the current Newton's first iteration)
  prev   : the previous step's final states (rows matched by type and dof)
  prev2  : the final states two steps back (period-2 chatter of the steering servo)
  smooth : the rows at qacc_smooth
  oned   : (the kernel's rule) each friction-loss row as a one-dof problem at qacc_smooth moved
           onto the steering equality: quadratic zone iff |x| <= R floss + floss invweight
If a prediction is right, one solve of that piece's quadratic is the exact optimum (convexity), so
the hit rate bounds what a predicted-active-set start can save over Newton from a start point.

    python tools/probes/active_set_probe.py [--envs 256] [--steps 300] [--contacts 0]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402
from oracle.oracle import FLAG_AUTORESET, FLAG_CONTACTS, Oracle, controller  # noqa: E402

FRICTIONLOSS = np.array([0, 0, 0, 0, 0, 0, 0.02, 0.02, 0.005, 0.012, 0.005, 0.012])


def row_keys(typ, J):
    keys = []
    for t, j in zip(typ, J):
        d = int(np.argmax(np.abs(j)))
        keys.append((int(t), d if t in (1, 2) else -1, int(np.sign(j[d])) if t == 2 else 0))
    return keys


def states(typ, R, fl, x):
    s = np.zeros(len(typ), int)
    f1 = typ == 1
    s[f1 & (x <= -R * fl)] = -1
    s[f1 & (x >= R * fl)] = 1
    s[(typ >= 2) & (x < 0)] = 1
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warm", type=int, default=50)
    ap.add_argument("--contacts", type=int, default=0)
    a = ap.parse_args()
    o = Oracle(_lib.load_blob())
    n = a.envs
    st = np.zeros((n, 44))
    o.reset(st, seed=3)
    rng = np.random.default_rng(0)
    fl_c = FLAG_CONTACTS if a.contacts else 0
    prevs = [[None, None] for _ in range(n)]
    hits = {k: 0 for k in ("warm", "prev", "prev2", "smooth", "prev|prev2", "warm|prev2", "oned")}
    total = 0
    wave = {k: [] for k in hits}
    for k in range(a.steps):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        if k >= a.warm:
            ok = {kk: np.zeros(n, bool) for kk in hits}
        for e in range(n):
            d = o.diag(st[e], controller(act[e]), flags=fl_c)
            if d["nefc"] == 0:
                prevs[e] = [{}, prevs[e][0]]
                if k >= a.warm:
                    for kk in hits:
                        ok[kk][e] = True
                continue
            efc, J = d["efc"], d["efc_J"]
            typ = efc[:, 0].astype(int)
            R, aref = efc[:, 2], efc[:, 3]
            fl = np.array([FRICTIONLOSS[np.argmax(np.abs(j))] if t == 1 else 0.0 for t, j in zip(typ, J)])
            keys = row_keys(typ, J)
            fin = states(typ, R, fl, J @ d["qacc"] - aref)
            if k >= a.warm and a.contacts == 0:
                pw = states(typ, R, fl, J @ st[e, 25:37] - aref)
                ps = states(typ, R, fl, J @ d["qacc_smooth"] - aref)
                p1 = np.array([prevs[e][0].get(kk, -9) if prevs[e][0] is not None else -9 for kk in keys])
                p2 = np.array([prevs[e][1].get(kk, -9) if prevs[e][1] is not None else -9 for kk in keys])
                ok["warm"][e] = np.array_equal(pw, fin)
                ok["smooth"][e] = np.array_equal(ps, fin)
                ok["prev"][e] = np.array_equal(p1, fin)
                ok["prev2"][e] = np.array_equal(p2, fin)
                ok["prev|prev2"][e] = ok["prev"][e] or ok["prev2"][e]
                ok["warm|prev2"][e] = ok["warm"][e] or ok["prev2"][e]
                M = d["qM"]
                ap = d["qacc_smooth"].copy()
                ap[8] = ap[10] = (M[8, 8] * ap[8] + M[10, 10] * ap[10]) / (M[8, 8] + M[10, 10])
                xp = J @ ap - aref
                thr = R * fl + fl * efc[:, 5]
                po = states(typ, R, fl, xp)
                po = np.where(typ == 1, np.where(xp < -thr, -1, np.where(xp > thr, 1, 0)), po)
                ok["oned"][e] = np.array_equal(po, fin)
            prevs[e] = [dict(zip(keys, fin.tolist())), prevs[e][0]]
        if k >= a.warm:
            total += n
            for kk in hits:
                hits[kk] += int(ok[kk].sum())
                wave[kk].append(ok[kk].reshape(-1, 64).all(1).mean())
        o.step(st, act, flags=fl_c | FLAG_AUTORESET, seed=3)
    for kk in hits:
        print(f"{kk:11s} env-step hit rate {hits[kk] / max(total, 1):.4f}   all-64-lanes-hit rate "
              f"{np.mean(wave[kk]) if wave[kk] else 0:.4f}")


if __name__ == "__main__":
    main()
