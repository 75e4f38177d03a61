"""CPU probe: Newton stopping rules on the contacts-on constraint problems of the f64 oracle.

Runs the oracle (contacts on, uniform random actions) and, for a sample of env-steps, re-solves
the step's primal problem in numpy (from MuJoCo's start: the cheaper of qacc_warmstart and
qacc_smooth) with the GPU kernel's exact-termination rule and with a Newton-decrement stop
(scale * (-g.p) < dtol, scale = 1 / (meaninertia * nv)). Prints the iteration histograms,
the wave max over groups of 16 envs (the quad mapping's wave) and max |dqacc| * dt against
the oracle's converged qacc.

    python tools/probes/newton_stop_probe.py [--envs 256] [--steps 200]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from mujoco_playground_amd import _lib  # noqa: E402
from oracle.oracle import Oracle, FLAG_CONTACTS, FLAG_AUTORESET  # noqa: E402

FRICTIONLOSS = np.array([0, 0, 0, 0, 0, 0, 0.02, 0.02, 0.005, 0.012, 0.005, 0.012])
MEANINERTIA, NV, DT = 2.589511871, 12, 0.002


def row_terms(typ, D, R, fl, x, jp):
    """per-row phi' contribution (g) and curvature (h) at x along jp; quad flag."""
    g = np.zeros_like(x); h = np.zeros_like(x); q = np.zeros(x.shape, bool)
    eq = typ == 0
    q |= eq
    f1 = typ == 1
    lo, hi = f1 & (x <= -R * fl), f1 & (x >= R * fl)
    mid = f1 & ~lo & ~hi
    q |= mid
    cl = (typ >= 2) & (x < 0)
    q |= cl
    g[q] = D[q] * x[q] * jp[q]
    h[q] = D[q] * jp[q] ** 2
    g[lo] = -fl[lo] * jp[lo]
    g[hi] = fl[hi] * jp[hi]
    return g, h, q


def solve(M, a0, J, aref, typ, D, R, fl, start, rule, dtol, maxit=30):
    a = start.copy()
    for it in range(maxit):
        jar = J @ a - aref
        _, _, q = row_terms(typ, D, R, fl, jar, np.zeros_like(jar))
        f = np.where(q, -D * jar, 0.0)
        f1 = typ == 1
        f = np.where(f1 & (jar <= -R * fl), fl, f)
        f = np.where(f1 & (jar >= R * fl), -fl, f)
        grad = M @ (a - a0) - J.T @ f
        H = M + (J[q].T * D[q]) @ J[q]
        p = -np.linalg.solve(H, grad)
        dec = -(grad @ p)
        if rule == "dec" and dec / (MEANINERTIA * NV) < dtol:
            return a + p, it + 1
        if dec <= 0:
            return a, it + 1
        Jp = J @ p
        Mp = M @ p
        pMp, pg0 = p @ Mp, Mp @ (a - a0)
        # exact line search by bisection on the piecewise-linear phi'
        def dphi(al):
            g, h, _ = row_terms(typ, D, R, fl, jar + al * Jp, Jp)
            return g.sum() + pg0 + al * pMp
        lo, hi = 0.0, 1.0
        while dphi(hi) < 0 and hi < 1e6:
            lo, hi = hi, 2 * hi
        full = abs(dphi(1.0)) <= 1e-9 * max(1.0, abs(dec))
        if full:
            al = 1.0
        else:
            for _ in range(80):
                mdl = 0.5 * (lo + hi)
                if dphi(mdl) < 0: lo = mdl
                else: hi = mdl
            al = 0.5 * (lo + hi)
        x0, x1 = jar, jar + al * Jp
        _, _, q0 = row_terms(typ, D, R, fl, x0, Jp)
        _, _, q1 = row_terms(typ, D, R, fl, x1, Jp)
        s0 = np.sign(np.where(f1, np.where(x0 <= -R * fl, -1, np.where(x0 >= R * fl, 1, 0)), 0))
        s1 = np.sign(np.where(f1, np.where(x1 <= -R * fl, -1, np.where(x1 >= R * fl, 1, 0)), 0))
        changed = np.any(q0 != q1) or np.any(s0 != s1)
        a = a + al * p
        if full and not changed:
            return a, it + 1
    return a, maxit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--every", type=int, default=10)
    a = ap.parse_args()
    o = Oracle(_lib.load_blob())
    n = a.envs
    st = np.zeros((n, 44))
    o.reset(st, seed=3)
    rng = np.random.default_rng(0)
    rules = [("exact", 0.0), ("warm", 0.0), ("smooth", 0.0), ("warm2", 0.0), ("best3", 0.0)]
    warm_prev = np.zeros((n, 12))  # qacc of step k - 2 (the steering servo's limit cycle has period 2)
    its = {r: [] for r in rules}
    errs = {r: [] for r in rules}
    for k in range(a.steps):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        if k >= 20 and k % a.every == 0:
            row_its = {r: np.zeros(n, int) for r in rules}
            for e in range(n):
                ctrl = _ctrl_of(o, act[e])
                d = o.diag(st[e], ctrl, flags=FLAG_CONTACTS)
                if d["nefc"] == 0:
                    continue
                efc, J = d["efc"], d["efc_J"]
                typ = efc[:, 0].astype(int)
                R = efc[:, 2]
                D = 1.0 / R
                aref = efc[:, 3]
                fl = np.array([FRICTIONLOSS[np.argmax(np.abs(j))] if t == 1 else 0.0 for t, j in zip(typ, J)])
                M, a0 = d["qM"], d["qacc_smooth"]
                warm = st[e, 25:37]

                def cost(x):
                    jar = J @ x - aref
                    c = 0.5 * (x - a0) @ M @ (x - a0)
                    for t, xx, DD, RR, ff in zip(typ, jar, D, R, fl):
                        if t == 0: c += 0.5 * DD * xx * xx
                        elif t == 1:
                            c += (-ff * xx - 0.5 * RR * ff * ff) if xx <= -RR * ff else (
                                (ff * xx - 0.5 * RR * ff * ff) if xx >= RR * ff else 0.5 * DD * xx * xx)
                        elif xx < 0: c += 0.5 * DD * xx * xx
                    return c
                start = warm if cost(warm) < cost(a0) else a0
                w2 = warm_prev[e]
                best3 = min((warm, w2, a0), key=cost)
                for r in rules:
                    s0 = {"warm": warm, "smooth": a0, "warm2": w2, "best3": best3}.get(r[0], start)
                    x, itn = solve(M, a0, J, aref, typ, D, R, fl, s0, r[0], r[1],
                                   maxit=int(r[1]) if r[0] == "cap" else 30)
                    row_its[r][e] = itn
                    errs[r].append(np.abs(x - d["qacc"]).max() * DT)
            for r in rules:
                its[r].append(row_its[r])
        warm_prev = st[:, 25:37].copy()
        o.step(st, act, flags=FLAG_CONTACTS | FLAG_AUTORESET, seed=3)
    # dual start: the iterations a solver racing both starts would need (the first to converge)
    mn = np.concatenate([np.minimum(a, b) for a, b in zip(its[("warm", 0.0)], its[("smooth", 0.0)])])
    for g in (16, 8):
        W = mn.reshape(-1, g).max(1)
        print(f"race min(warm, smooth): mean it {mn.mean():.2f}  hist {np.bincount(mn, minlength=10)[:12]}  "
              f"wave-max hist ({g} envs/wave) {np.bincount(W, minlength=10)[:12]}", flush=True)
    for r in rules:
        I = np.concatenate(its[r])
        W = np.concatenate([x.reshape(-1, 16).max(1) for x in its[r]])
        E = np.array(errs[r])
        print(f"{r[0]:5s} {r[1]:7.0e}: mean it {I.mean():.2f}  hist {np.bincount(I, minlength=10)[:12]}  "
              f"wave-max hist {np.bincount(W, minlength=10)[:12]}  max|dqvel| {E.max():.2e}  p99.9 "
              f"{np.quantile(E, 0.999):.2e}", flush=True)


def _ctrl_of(o, act):
    from oracle.oracle import controller
    return controller(act)


if __name__ == "__main__":
    main()
