"""GPU probe: why the first tens of contacts-off steps after reset cost more than steady state.

(1) product library: event-timed ackphys_rollout windows of K = 20 steps starting at several
    steps after reset (best of 3; the state is restored before each try);
(2) diagnostic build (tools/build_diag.sh -> libackphys_stamps.so): single-step launches of the
    nc kernel from reset (steps 0..STEPS) and from step 540, recording per step the dynamics
    wave's cycles (median / max over the 64 waves), the lanes that missed the predicted active set
    (Newton fallback), the wave-max Newton iterations, and the lanes whose one-dof steer guess was
    inconsistent (the 9-pair search; the wave runs it when any lane needs it).

    python tools/probes/post_reset_probe.py > gpurun_out/post_reset.jsonl
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
NSTAMP = 24
STEPS = int(os.environ.get("PROBE_STEPS", "120"))


def windows():
    from mujoco_playground_amd.sim import BatchedAckermannSim
    sim = BatchedAckermannSim(4096, "cuda:0", seed=0, contacts=False)
    acts = sim.random_actions(1000, seed=0)
    for start in (0, 5, 25, 45, 65, 85, 105, 150, 200, 300, 400, 550, 800):
        sim.reset()
        if start:
            sim.rollout(acts[:start], want_info=False, per_step_outputs=False)
        snap = sim.state.clone(), sim.episode.clone()
        best = None
        for _ in range(3):
            sim.state.copy_(snap[0])
            sim.episode.copy_(snap[1])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            sim.rollout(acts[start:start + 20], want_info=False, per_step_outputs=False)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) * 1e3 / 20
            best = t if best is None or t < best else best
        print(json.dumps({"probe": "window", "start_step": start, "K": 20, "gpu_us_per_step": round(best, 3)}),
              flush=True)


def diag_steps():
    L = C.CDLL(os.path.join(REPO, "mujoco_playground_amd", "csrc", "build", "libackphys_stamps.so"))
    P = C.c_void_p
    L.ackphys_create.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(P)]
    L.ackphys_step.argtypes = [P] * 10 + [C.c_uint32, C.c_uint64, P]
    L.ackphys_reset.argtypes = [P, P, C.c_uint64, P, P, P]
    L.ackphys_random_actions.argtypes = [P, P, C.c_int, C.c_uint64, C.c_uint32, P]
    L.ackphys_diag_set_stamps.argtypes = [P]
    L.ackphys_set_variant.argtypes = [P, C.c_int]
    from mujoco_playground_amd import _lib
    blob = _lib.load_blob()
    n = 4096
    dev = torch.device("cuda:0")
    ctx = P()
    assert L.ackphys_create(blob, len(blob), n, 0, C.byref(ctx)) == 0
    assert L.ackphys_set_variant(ctx, 0) == 0
    p = lambda t: P(t.data_ptr())
    stream = P(torch.cuda.current_stream().cuda_stream)
    nb = (n + 63) // 64
    st = torch.zeros(NSTAMP * nb + nb * 64 + 5 * nb, dtype=torch.int64, device=dev)
    assert L.ackphys_diag_set_stamps(p(st)) == 0
    state, obs = torch.zeros(44, n, device=dev), torch.zeros(79, n, device=dev)
    rew = torch.zeros(n, device=dev)
    term, trunc = torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev)
    acts = torch.zeros(600, n, 2, device=dev)
    L.ackphys_random_actions(ctx, p(acts), 600, 0, 0, stream)
    L.ackphys_reset(ctx, None, 0, p(state), p(obs), stream)
    record = set(range(STEPS)) | set(range(540, 560))
    for k in range(560):
        st.zero_()
        L.ackphys_step(ctx, p(acts[k]), p(state), p(obs), p(rew), p(term), p(trunc), None, None, None, 2, 0, stream)
        if k not in record:
            continue
        torch.cuda.synchronize()
        a = st.cpu().numpy()
        s = a[:NSTAMP * nb].reshape(NSTAMP, nb)
        dyn = (s[10] - s[0]).astype(np.int64)
        rec = a[NSTAMP * nb: NSTAMP * nb + 64 * nb]
        it = (rec & 0xFF) // 8
        pair = (rec >> 16) & 1
        miss = (rec >> 17) & 1
        sv = state.cpu().numpy()
        print(json.dumps({
            "probe": "diag", "step": k, "dyn_cycles_median": int(np.median(dyn)), "dyn_cycles_max": int(dyn.max()),
            "newton_wave_max": int(it.reshape(nb, 64).max(1).max()),
            "waves_with_newton": int((it.reshape(nb, 64).max(1) > 0).sum()),
            "lanes_missed_prediction": int(miss.sum()), "lanes_pair_search": int(pair.sum()),
            "waves_pair_search": int((pair.reshape(nb, 64).max(1) > 0).sum()),
            "mean_abs_steer_qvel": float(np.abs(sv[13 + 8]).mean()),
            "chassis_z": float(np.median(sv[2])),
            "stamps_median": {i: int(np.median(s[i] - s[0])) for i in range(NSTAMP) if s[i].any()},
            "mean_abs_rear_qvel": float(np.abs(sv[13 + 6]).mean())}), flush=True)


if __name__ == "__main__":
    windows()
    diag_steps()
