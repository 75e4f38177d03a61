"""Benchmark: batched Ackermann-robot env step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

A "step" is one AckermannRobotEnv.step for every env of the shard (4096 per GPU): one launch
of ackphys_step_kernel (controller, kinematics, dynamics, contacts, Newton solve, Euler,
lidar, obs, reward, done, auto-reset). Inputs are resident in HBM before timing: the K+W
action batches are drawn on device from Philox (seed 0; counter = (env, step)).
Prints ONE JSON line (rank 0).

Workload (value): BASELINE.json configs[1] -- 4096 envs/GPU, random ctrl, contacts disabled.
The contacts-enabled variant (configs[2]) is reported under "secondary"; the obstacle scene
(configs[4]'s world: the v2 robot in models/environments/ackermann_maze_flat.xml, 38 boxes)
under "obstacles" (env steps, contacts on) and its PPO rollout under "obstacles.ppo".
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from mujoco_playground_amd import shard  # noqa: E402
from mujoco_playground_amd.sim import NOBS, NSTATE, BatchedAckermannSim  # noqa: E402

METRIC = "env-steps/sec at 4096 envs/GPU, 1/2/4/8 MI355X; max |qpos| err vs CPU mj_step"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def algorithmic_bytes_per_env_step() -> int:
    """Minimal HBM I/O of one env step:
    in : state 44 words (176 B) + action 2 floats (8 B) + episode stats 4 words (16 B)
    out: modified state words 38 (qpos 13, qvel 12, warmstart 12, step 1) = 152 B,
         obs 79 floats (316 B), reward (4 B), term + trunc (2 B), episode stats (16 B)."""
    return 176 + 8 + 16 + 152 + 316 + 4 + 2 + 16


# With contacts the robot spawns 0.1 m above the floor (simple_map_spawner.py:43) and lands after
# ~70 steps; until then a contacts-on step is a free-fall step. The contacts legs therefore run at
# least SETTLE_STEPS untimed steps (the driver's short --warmup included) so the timed steps are
# ground-contact steps whatever --warmup is.
SETTLE_STEPS = 200


def run_gpu(n_env, steps, warmup, contacts, rank, world, device, seed=0, variant="auto", scene="flat", graph=False,
            per_step=False, buffers=False):
    """Times `steps` random-ctrl steps of the env shard. Default: ONE ackphys_rollout launch runs the
    K pre-drawn action rows (every step computed and its outputs written, exactly K ackphys_step
    calls' results -- tests/test_gpu_rollout.py), each step's outputs overwriting the last in place;
    buffers=True: the same launch writing every step's obs / reward / flags into its own slice of a
    [K, ...] rollout buffer (per_step_outputs=1: the bytes a consumer of every step's observation
    needs leave the chip); per_step=True: K ackphys_step launches (the call pattern of a
    policy-in-the-loop RL step), graph=True: those K launches replayed from a hipGraph."""
    sim = BatchedAckermannSim(n_env, device, seed=seed, contacts=contacts,
                              env_offset=shard.env_offset(rank, n_env), variant=variant, scene=scene)
    sim.reset()
    pre = max(warmup, SETTLE_STEPS) if contacts else warmup
    actions = sim.random_actions(pre + steps, seed=seed)
    warmup = pre
    if per_step or graph:
        for k in range(warmup):
            sim.step(actions[k], want_info=False)
    elif warmup:  # through a launcher like the timed one (the same C call, warmed before the window)
        sim.rollout_launcher(actions[:warmup].contiguous(), want_terminal=True)()
    timed_actions = actions[warmup:]  # [K, N, 2], contiguous, resident before the timed region
    step_actions = timed_actions.unbind(0)  # per-step views, made before the timed region
    g = None
    if graph:  # the K timed steps as one captured hipGraph (same launches, same buffers)
        snap = sim.state.clone(), sim.episode.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(steps):
                sim.step(step_actions[k], want_info=False)
        sim.state.copy_(snap[0])  # capture launches nothing, but restore anyway
        sim.episode.copy_(snap[1])
    stream = torch.cuda.current_stream(device)
    launch = None if (per_step or g is not None) else sim.rollout_launcher(
        timed_actions, outputs=sim.rollout_buffers(steps) if buffers else None)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev1.record(stream)  # the end event's HIP event is created here, not by its record inside the window
    torch.cuda.synchronize(device)
    shard.barrier(world, device)
    torch.cuda.synchronize(device)
    gc.disable()  # no collector pass inside the host-clocked window
    ev0.record(stream)  # enqueued before the clock starts: the window holds the launch(es) and the drain
    t0 = time.perf_counter()
    if g is not None:
        g.replay()
    elif per_step:
        for k in range(steps):
            sim.step(step_actions[k], want_info=False)
    else:
        launch()
    ev1.record(stream)
    gathered = shard.gather_episode_stats(sim.episode, world)  # the per-rollout RCCL exchange
    torch.cuda.synchronize(device)
    shard.barrier(world, device)
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    gc.enable()
    elapsed = shard.max_over_ranks(t1 - t0, world, device)
    kern_ms = ev0.elapsed_time(ev1) / steps
    return sim, elapsed, kern_ms, shard.summarize_returns(gathered), actions


def clock_warm(device, n_env: int, seconds: float = 0.2):
    """Untimed GPU work on a throwaway sim until ~`seconds` have passed (clock ramp-up)."""
    sim = BatchedAckermannSim(n_env, device, seed=1, contacts=False)
    sim.reset()
    acts = sim.random_actions(200, seed=1)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        sim.rollout(acts, want_info=False, per_step_outputs=False)
        torch.cuda.synchronize(device)


def run_ppo(n_env, rank, world, device, iters=3, n_steps=32, batch_size=8192, n_epochs=10, seed=0, scene="flat"):
    """BASELINE configs[3]: PPO rollout on the env shard (contacts enabled, SB3 PPO('MlpPolicy')
    semantics on libackppo.so). One warm-up iteration, then `iters` timed iterations of
    collect_rollouts (n_steps policy+env steps) + train (n_epochs over minibatches)."""
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    venv = AckermannVecEnv(n_env, device=device, seed=seed, contacts=True, env_offset=shard.env_offset(rank, n_env),
                           scene=scene)
    model = PPO("MlpPolicy", venv, n_steps=n_steps, batch_size=batch_size, n_epochs=n_epochs, seed=seed,
                ent_coef=0.0, world=world, rank=rank)
    model.collect_rollouts()
    model.train()
    stream = torch.cuda.current_stream(device)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters + 1)]
    torch.cuda.synchronize(device)
    shard.barrier(world, device)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    e[0].record(stream)
    for i in range(iters):
        model.collect_rollouts()
        e[2 * i + 1].record(stream)
        model.train()
        e[2 * i + 2].record(stream)
    torch.cuda.synchronize(device)
    shard.barrier(world, device)
    el = shard.max_over_ranks(time.perf_counter() - t0, world, device)
    roll_ms = sum(e[2 * i].elapsed_time(e[2 * i + 1]) for i in range(iters)) / iters
    train_ms = sum(e[2 * i + 1].elapsed_time(e[2 * i + 2]) for i in range(iters)) / iters
    steps = iters * n_steps * n_env * world
    nmb = (n_steps * n_env + batch_size - 1) // batch_size
    dp_path = None
    if world == 1:
        dp_path = time_dp_update(model, device, stream, iters, train_ms, n_epochs, nmb)
    return {"value": steps / el, "unit": "env-steps/s (rollout + update, all ranks)",
            "rollout_env_steps_per_s": n_steps * n_env * world / (roll_ms * 1e-3),
            "rollout_ms": roll_ms, "update_ms": train_ms, "minibatch_updates_per_iter": nmb * n_epochs,
            "update_us_per_minibatch": train_ms * 1e3 / (nmb * n_epochs), "dp_update_path": dp_path,
            "rollout_path": ("one ackphys_ppo_rollout launch per rollout (policy + env steps + bootstrap fused)"
                             if model.fused_rollout else "ackppo_act + ackphys_step launches per step"),
            "config": f"{scene} scene, {n_env} envs/GPU x {world}, n_steps {n_steps}, batch {batch_size} x {world} "
                      f"ranks, {n_epochs} epochs, contacts on, {iters} timed iterations after 1 warm-up",
            "last_logger": {k: v for k, v in model.logger.items() if isinstance(v, (int, float)) or v is None}}


def time_dp_update(model, device, stream, iters, train_ms, n_epochs, nmb):
    """The world > 1 update path timed on one GPU: ackppo_train's data-parallel sequence (every epoch's
    shuffle and advantage moments at the start of the call with 2 f64 all-reduces, then per minibatch
    the reduction, one 75 KB f32 all-reduce, the norm blocks and Adam) over a one-rank communicator,
    on the same rollout buffer (untimed first call). "rccl" = the default at world > 1: libackppo's own
    communicator; "torch" = RCCL calls on the communicator of torch's own ProcessGroupNCCL (a one-rank
    nccl process group here; opt-in until it has run on a multi-GPU node)."""
    import torch.distributed as dist
    out = {}
    made_pg = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)  # as shard.init: lazy comm
        made_pg = True
    try:
        for kind in ("rccl", "torch"):
            model.set_collective(kind)
            model.train()
            ed = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize(device)
            ed[0].record(stream)
            for _ in range(iters):
                model.train()
            ed[1].record(stream)
            torch.cuda.synchronize(device)
            dp_ms = ed[0].elapsed_time(ed[1]) / iters
            model.set_collective(None)
            out[kind] = {"update_ms": dp_ms, "update_us_per_minibatch": dp_ms * 1e3 / (nmb * n_epochs),
                         "ratio_to_single_rank_update": dp_ms / train_ms}
    finally:
        if made_pg:
            dist.destroy_process_group()
    d = dict(out["rccl"])
    d.update({"collective": "rccl (libackppo's own communicator, the default at world > 1)",
              "torch_communicator": out["torch"],
              "collectives_per_iteration": n_epochs * nmb + 2, "bytes_per_minibatch_allreduce": 4 * 18764,
              "note": "ackppo_train with the RCCL hook on a one-rank communicator: the data-parallel sequence "
                      "every rank of configs[3] runs, each collective enqueued from C (no per-minibatch host "
                      "round trip); the advantage moments of all epochs in 2 collectives per train() call"})
    return d


def to_f64_state(st: torch.Tensor) -> np.ndarray:
    s = st.detach().cpu().numpy().T.copy()
    out = s.astype(np.float64)
    out[:, 42] = s[:, 42].view(np.uint32)
    out[:, 43] = s[:, 43].view(np.uint32)
    return out


TOL_QPOS, TOL_QVEL = 1e-5, 1e-3  # tests/test_gpu_parity.py's stated f32 tolerances
BOUNDARY_DZ = (1e-7, -1e-7, 1e-6, -1e-6)  # tests/test_gpu_parity.py's contact-activation boundary rule


def boundary_excused(o, before_e, act_e, after_e, flags, seed) -> bool:
    """The parity tests' excuse (tests/test_gpu_parity.py _boundary_excused): an env-step
    over the tolerances counts as a contact-activation boundary case only if the oracle, with the body
    shifted <= 1e-6 m in z, reproduces the GPU step within the same tolerances."""
    for dz in BOUNDARY_DZ:
        s = before_e[None].copy()
        s[0, 2] += dz
        o.step(s, act_e[None], flags=flags, seed=seed)
        if (np.abs(after_e[:13] - s[0, :13]).max() <= TOL_QPOS and
                np.abs(after_e[13:25] - s[0, 13:25]).max() <= TOL_QVEL):
            return True
    return False


def parity_sample(o, device, contacts, flags, seed, n, steps, settle=0, drift=True):
    """Teacher-forced parity on a sample (same flags / seed as the timed run): every step starts the
    oracle from the GPU's state. An env-step over the stated tolerances is classified with the parity
    tests' rule: excused (a contact-activation boundary, DESIGN.md §5: the oracle reproduces the GPU
    step from the state shifted <= 1e-6 m in z) or unexcused; the max errors are over the env-steps
    within tolerance and, separately, over all of them (raw)."""
    sim = BatchedAckermannSim(n, device, seed=seed, contacts=contacts)
    sim.reset()
    acts = sim.random_actions(settle + steps, seed=seed)
    if settle:
        sim.rollout(acts[:settle], want_info=False, per_step_outputs=False)
    eq = ev = eo = rq = rv = 0.0
    excused = unexcused = 0
    for k in range(settle, settle + steps):
        s_before = to_f64_state(sim.state)
        sim.step(acts[k], want_info=False)
        torch.cuda.synchronize(device)
        s_after = to_f64_state(sim.state)
        ref = s_before.copy()
        a_np = acts[k].cpu().numpy()
        oobs, orew, _, _, _, _ = o.step(ref, a_np, flags=flags, seed=seed)
        dq = np.abs(s_after[:, 0:13] - ref[:, 0:13]).max(1)
        dv = np.abs(s_after[:, 13:25] - ref[:, 13:25]).max(1)
        ok = (dq <= TOL_QPOS) & (dv <= TOL_QVEL)
        for e in np.nonzero(~ok)[0]:
            if boundary_excused(o, s_before[e], a_np[e], s_after[e], flags, seed):
                excused += 1
            else:
                unexcused += 1
        rq, rv = max(rq, float(dq.max())), max(rv, float(dv.max()))
        eq, ev = max(eq, float(dq[ok].max(initial=0.0))), max(ev, float(dv[ok].max(initial=0.0)))
        eo = max(eo, float(np.abs(sim.obs_soa.cpu().numpy().T - oobs)[ok].max(initial=0.0)))
    out = {"max_abs_qpos_err": eq, "max_abs_qvel_err": ev, "max_abs_obs_err": eo,
           "env_steps_over_tolerance": excused + unexcused, "excused_boundary_env_steps": excused,
           "unexcused_env_steps": unexcused, "raw_max_abs_qpos_err": rq, "raw_max_abs_qvel_err": rv,
           "tolerance": {"qpos": TOL_QPOS, "qvel": TOL_QVEL},
           "classification": "tests/test_gpu_parity.py rule: an over-tolerance env-step is excused only if the "
                             "oracle reproduces the GPU step from the state shifted <= 1e-6 m in z (contact "
                             "activation boundary); max_abs_* are over the env-steps within tolerance, raw_* over all",
           "sample": f"{n} envs x {steps} teacher-forced steps, contacts {'on' if contacts else 'off'}, "
                     + (f"after {settle} settle steps" if settle else "from reset") + " (f32 GPU vs f64 oracle)"}
    if drift:
        # free-running drift (not gated): GPU and oracle both run their own state from the
        # same reset under the same actions; max |dqpos| after 1/10/100 steps
        fsim = BatchedAckermannSim(n, device, seed=seed, contacts=contacts)
        fsim.reset()
        facts = fsim.random_actions(100, seed=seed)
        fst = to_f64_state(fsim.state)
        d = {}
        for k in range(100):
            fsim.step(facts[k], want_info=False)
            o.step(fst, facts[k].cpu().numpy(), flags=flags, seed=seed)
            if k + 1 in (1, 10, 100):
                torch.cuda.synchronize(device)
                d[str(k + 1)] = float(np.abs(to_f64_state(fsim.state)[:, 0:13] - fst[:, 0:13]).max())
        out["free_running_qpos_drift"] = d
    return out


def cpu_leg(device, contacts, seed=0, parity_envs=256, parity_steps=20, budget_s=12.0, do_timing=True):
    """Oracle as the checker: teacher-forced max|qpos| error on a sample, and the CPU baseline
    (oracle on the host cores, bounded sample of the same workload)."""
    from mujoco_playground_amd import _lib
    from oracle.oracle import FLAG_AUTORESET, FLAG_CONTACTS, Oracle
    o = Oracle(_lib.load_blob())
    flags = (FLAG_CONTACTS if contacts else 0) | FLAG_AUTORESET
    parity = parity_sample(o, device, contacts, flags, seed, parity_envs, parity_steps, settle=0)
    if contacts is False:  # the contacts-on sample too, on ground-contact steps (after the settle steps)
        parity["contacts_on"] = parity_sample(o, device, True, FLAG_CONTACTS | FLAG_AUTORESET, seed, parity_envs,
                                              parity_steps, settle=SETTLE_STEPS, drift=False)
    if not do_timing:
        return parity, None
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    n = 4096
    st = np.zeros((n, NSTATE))
    o.reset(st, seed=seed)
    asim = BatchedAckermannSim(n, device, seed=seed, contacts=contacts)
    # probe a few steps, then size the sample to ~budget_s of CPU work (same Philox action stream)
    acts = asim.random_actions(8, seed=seed, step0=0).cpu().numpy()
    t0 = time.perf_counter()
    for i in range(8):
        o.step(st, acts[i], flags=flags, seed=seed, nthreads=threads)
    probe = (time.perf_counter() - t0) / 8
    k = int(max(8, min(4000, budget_s / max(probe, 1e-6))))
    acts = asim.random_actions(k, seed=seed, step0=8).cpu().numpy()
    t0 = time.perf_counter()
    for i in range(k):
        o.step(st, acts[i], flags=flags, seed=seed, nthreads=threads)
    dt = time.perf_counter() - t0
    # 1 core, same per-env work on a smaller batch (~3 s)
    n1 = 256
    st1 = np.zeros((n1, NSTATE))
    o.reset(st1, seed=seed)
    k1 = int(max(4, min(2000, 3.0 / max(probe * n1 / n * threads, 1e-6))))
    t1 = time.perf_counter()
    for i in range(k1):
        o.step(st1, acts[i % k, :n1], flags=flags, seed=seed, nthreads=1)
    one_core = n1 * k1 / (time.perf_counter() - t1)
    # BASELINE configs[0]: one env driven step by step from Python, the oracle standing in for
    # mj_step (the reference's per-env call pattern: one step call per env per step)
    st0 = np.zeros((1, NSTATE))
    o.reset(st0, seed=seed)
    k0, t2 = 2000, time.perf_counter()
    for i in range(k0):
        o.step(st0, acts[i % k, :1], flags=flags, seed=seed, nthreads=1)
    one_env = k0 / (time.perf_counter() - t2)
    base = {"value": n * k / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ackphys_oracle.c (f64 restatement of mj_step + env glue), {n} envs x {k} steps "
                      f"after 8 probe steps from reset, same Philox actions/flags, OpenMP {threads} threads, {dt:.1f} s",
            "one_core": {"value": one_core, "sample": f"{n1} envs x {k1} steps, 1 thread"},
            "config0_python_1env": {"value": one_env, "sample": f"1 env x {k0} steps, one Python call per step "
                                                                "(BASELINE configs[0] call pattern)"}}
    return parity, base


def _profile(name: str):
    """A committed measurement summary under profiles/ (None if absent)."""
    try:
        with open(os.path.join(HERE, "profiles", name)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def load_pmc(kern_name: str, contacts: bool, steps: int, buffers: bool = False):
    """PMC summary of the kernel from the committed rocprofv3 passes (tools/profile_pmc.py ->
    profiles/pmc_latest.json), for the launch length K nearest to `steps` (a launch's first-step
    loads and last-step stores are spread over its K steps); None if absent. The counters are NOT
    measured in this run: the returned entry names its source."""
    d = _profile("pmc_latest.json") or {}
    cands = [v for v in d.values() if isinstance(v, dict) and v.get("kernel") == kern_name
             and bool(v.get("contacts")) == contacts and bool(v.get("per_step_outputs")) == buffers]
    if not cands:
        return None
    best = min(cands, key=lambda v: abs(v["launch_steps"] - steps))
    return dict(best, source=f"profiles/pmc_latest.json ({d.get('_round', '?')}; rocprofv3 --pmc, separate passes, "
                            f"launch of K={best['launch_steps']} steps{'' if best['launch_steps'] == steps else ', nearest to --steps'})")


CLOCK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md constants table)
STAMP_OVERHEAD = 0.11  # cycles the diagnostic build's LDS stamps add to the dynamics wave


def valu_block(pmc, kern_ms: float):
    """VALU issue share of a kernel from its committed PMC entry (None without one)."""
    if not (pmc and pmc.get("valu_insts_per_wave_step")):
        return None
    # one wave alone issues a dependent VALU op every ~4 cycles (MI355X_MICROARCH.md constants
    # table; tools/probes/launch_floor.py measures 4.1 cycles per op of a dependent FMA chain)
    return {"insts_per_wave_step": pmc["valu_insts_per_wave_step"], "waves": pmc["SQ_WAVES"],
            "issue_frac_of_kernel_time": pmc["valu_insts_per_wave_step"] * 4 / (kern_ms * 1e-3 * CLOCK_GHZ * 1e9),
            "source": pmc["source"],
            "note": "fraction of the kernel's duration one wave spends issuing VALU at the lone-wave "
                    "dependent-op rate (4 cyc/op), per-wave average over the kernel's waves (contacts off: "
                    "dynamics, observation and prep waves); the rest is dependency/memory latency"}


def critical_path(kern_name: str, kern_ms: float):
    """The dynamics wave's dependent chain against the kernel time: cycles per step from the
    stamped diagnostic build (tools/stamps.py -> profiles/critical_path_latest.json), not this run."""
    d = _profile("critical_path_latest.json") or {}
    e = next((v for v in d.values() if isinstance(v, dict) and v.get("kernel") == kern_name), None)
    if e is None:
        return None
    kc = kern_ms * 1e-3 * CLOCK_GHZ * 1e9
    ratio = e["dyn_wave_cycles_per_step_median"] / kc
    frac = ratio / (1.0 + STAMP_OVERHEAD)
    return {"dyn_wave_cycles_per_step": e["dyn_wave_cycles_per_step_median"], "kernel_cycles_per_step": kc,
            "diag_over_kernel_cycles": ratio, "stamp_overhead": STAMP_OVERHEAD,
            "frac_of_kernel_time": frac, "consistent": frac <= 1.0, "clock_ghz_assumed": CLOCK_GHZ,
            "note": "stamped diagnostic build (its stamps add ~11 %, removed in frac_of_kernel_time; not clamped: "
                    "consistent = false when the stamped chain exceeds this run's kernel time, e.g. when the "
                    "profile predates a kernel change) against this run's kernel time at the assumed peak clock",
            "phases_median": e.get("phases_median"),
            "source": f"profiles/critical_path_latest.json ({d.get('_round', '?')}): {e.get('measured', '')}"}


def mfma_summary():
    """MFMA utilisation of the PPO kernels (tools/profile_mfma.py -> profiles/mfma_latest.json)."""
    d = _profile("mfma_latest.json")
    if not d:
        return None
    out = {k: {"mfma_util": v.get("mfma_util"), "mfma_tflops": v.get("mfma_tflops"),
               "peak_tflops": v.get("f32_mfma_peak_tflops"), "duration_us": v.get("median_duration_ns", 0) / 1e3}
           for k, v in d.items() if isinstance(v, dict) and k.startswith("ackppo")}
    out["source"] = f"profiles/mfma_latest.json ({d.get('_round', '?')}; rocprofv3 --pmc on tools/ppo_train_workload.py: PPO.train() as the product runs it)"
    out["note"] = ("the physics step kernels use no MFMA (per-lane scalar f32 work); the PPO learner's GEMM-shaped "
                   "layers run v_mfma_f32_16x16x4_f32")
    return out


FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md constants table (spec)


def oracle_flops(config_key: str, rate: float):
    """The reference algorithm's FLOPs per env-step for this workload, counted in the CPU oracle
    (tools/count_flops.py -> profiles/oracle_flops.json), and the effective FP32 rate
    they imply at `rate` env-steps/s; None if that profile is absent."""
    try:
        with open(os.path.join(HERE, "profiles", "oracle_flops.json")) as f:
            c = json.load(f)["configs"][config_key]
    except (OSError, ValueError, KeyError):
        return None
    eff = c["flops_per_env_step"] * rate / 1e12
    return {"oracle_flops_per_env_step": c["flops_per_env_step"], "effective_tflops": eff,
            "fp32_vector_peak_tflops": FP32_VECTOR_PEAK_TFLOPS, "frac": eff / FP32_VECTOR_PEAK_TFLOPS,
            "note": "FLOPs of the reference's algorithm (f64 oracle, + - * / sqrt) per env-step x env-steps/s; "
                    "the kernels execute fewer (structured factorisations, floor-only rays, predicted pieces)"}


def launch_command(argv: list, gpus: int, port: int) -> list:
    """The torchrun command that runs this bench with one rank per GPU (the driver's own N>1 verb:
    torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py ...)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def spawn_ranks(argv: list, gpus: int) -> int:
    """`bench.py --gpus N` (N > 1) started without a torchrun environment: start the N rank
    processes as children and return their exit status. This process never touches the GPU (no
    HIP call before the children exist; nothing is exec'ed from a GPU-initialised process); rank 0
    prints the JSON line on the inherited stdout."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between the rank processes)
    env["ACKPHYS_SPAWNED"] = "1"
    return subprocess.run(launch_command(argv, gpus, port), env=env).returncode


def check_world(gpus: int, world: int, rank: int) -> str:
    """Each rank refuses a run whose world is not the --gpus it was asked for, or (on a GPU node)
    a multi-GPU world whose backend is not RCCL ("nccl" on ROCm). The only exception is a
    rehearsal of N ranks on one device (ACKPHYS_DEVICE_OVERRIDE, tools/rehearse_dist.sh), where
    RCCL cannot run and gloo stands in. Returns the backend name ("none" at world 1)."""
    import torch.distributed as dist
    if world != gpus:
        raise SystemExit(f"bench.py rank {rank}: world size {world} != --gpus {gpus}")
    if world == 1:
        return "none"
    backend = dist.get_backend()
    if (torch.cuda.is_available() and backend != "nccl" and os.environ.get("ACKPHYS_DEVICE_OVERRIDE") is None):
        raise SystemExit(f"bench.py rank {rank}: backend {backend!r} on a GPU node (RCCL 'nccl' required)")
    return backend


_JSON_OUT = None


def quiet_stdout():
    """Everything but the result line goes to stderr: libraries print to fd 1 on their own (RCCL's
    version banner when a communicator is created, for one), and the driver parses this process's
    stdout as ONE JSON line. fd 1 is pointed at stderr; the line is written to a dup of the original."""
    global _JSON_OUT
    if _JSON_OUT is None:
        sys.stdout.flush()
        _JSON_OUT = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)


def emit(line: dict):
    out = _JSON_OUT or sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


def main():
    argv = sys.argv[1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--contacts", type=int, default=0, help="0 = configs[1] (default), 1 = configs[2]")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--variant", default="auto", choices=["auto", "quad", "lane", "lane16"], help="step-kernel lane mapping")
    ap.add_argument("--no-ppo", action="store_true", help="skip the PPO-rollout leg (BASELINE configs[3])")
    ap.add_argument("--no-obstacles", action="store_true", help="skip the obstacle-scene leg (configs[4] world)")
    ap.add_argument("--graph", action="store_true", help="replay the timed steps' launches as one captured hipGraph")
    ap.add_argument("--per-step", action="store_true",
                    help="time K ackphys_step launches instead of one ackphys_rollout launch of K steps")
    ap.add_argument("--no-per-step", action="store_true",
                    help="skip the per-step-launch legs (K ackphys_step launches of the same workloads)")
    ap.add_argument("--no-buffer-leg", action="store_true",
                    help="skip the rollout-buffer leg (the headline launch with per-step output slices)")
    ap.add_argument("--buffers", action="store_true",
                    help="time the headline launch with per-step output slices (tools/profile_pmc.py --buffers)")
    ap.add_argument("--scene", default="flat", choices=["flat", "obstacles"],
                    help="scene of the headline launch (profiling: tools/profile_pmc.py --obstacles); the "
                         "driver's bench line is the flat scene")
    ap.add_argument("--check-launch", action="store_true",
                    help="ranks check the world and backend, print one JSON line and exit (no GPU work)")
    a = ap.parse_args()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(argv, a.gpus))  # before any GPU call in this process
    quiet_stdout()
    rank, world, local = shard.init()
    backend = check_world(a.gpus, world, rank)
    if a.check_launch:
        ranks = [rank]
        if world > 1:
            import torch.distributed as dist
            got = [None] * world
            dist.all_gather_object(got, rank)
            ranks = got
        if rank == 0:
            emit({"check_launch": True, "n_gpus": world, "ranks": ranks, "backend": backend})
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    device = shard.device_for(local)
    torch.cuda.set_device(device)
    contacts = bool(a.contacts)
    fused = not (a.per_step or a.graph)
    total_envs = a.envs * world
    sec_run = None
    if not a.no_secondary:
        sec_run = run_gpu(a.envs, a.steps, a.warmup, not contacts, rank, world, device, variant=a.variant,
                          graph=a.graph, per_step=a.per_step)
    # the headline window must not start on a GPU whose clocks are still low after an idle spell (a
    # 20-step window right after start-up measured ~15 % slower per step): ~0.2 s of untimed work on
    # a throwaway sim first, whatever ran before (so the value does not depend on --no-secondary)
    clock_warm(device, a.envs)
    sim, elapsed, kern_ms, rets, _ = run_gpu(a.envs, a.steps, a.warmup, contacts, rank, world, device,
                                             variant=a.variant, graph=a.graph, per_step=a.per_step,
                                             buffers=a.buffers, scene=a.scene)
    value = total_envs * a.steps / elapsed

    def per_step_leg(c, scene="flat"):
        """the same workload as K ackphys_step launches (policy-in-the-loop call pattern)"""
        _, el, km, _, _ = run_gpu(a.envs, a.steps, a.warmup, c, rank, world, device, variant=a.variant, scene=scene,
                                  per_step=True)
        return {"value": total_envs * a.steps / el, "ms_per_step": el * 1e3 / a.steps, "kernel_ms": km,
                "note": "K ackphys_step launches (one per step) instead of one ackphys_rollout launch"}
    do_per_step = fused and not a.no_per_step
    per_step_launch = per_step_leg(contacts) if do_per_step else None

    def buffer_leg(c):
        """the headline launch with per-step output slices (a [K][79][N] obs + reward / flag rollout
        buffer): every step's 690 algorithmic bytes per env really leave the chip"""
        _, el, km, _, _ = run_gpu(a.envs, a.steps, a.warmup, c, rank, world, device, variant=a.variant, buffers=True)
        ach = bpe * a.envs / (km * 1e-3) / 1e9
        pm = load_pmc(kern, c, a.steps, buffers=True)
        return {"value": total_envs * a.steps / el, "ms_per_step": el * 1e3 / a.steps, "kernel_ms": km,
                "achieved_GBps": ach, "peak_GBps": HBM_PEAK_GBS, "frac": ach / HBM_PEAK_GBS,
                "counter_bytes_per_step": pm.get("hbm_bytes_per_step") if pm else None,
                "counter_source": pm["source"] if pm else None,
                "note": "same kernel and workload as the headline with per_step_outputs=1: obs [K][79][N], reward "
                        "and term/trunc [K][N] each step into its own slice (ackermann_env.py:210-229 returns the "
                        "obs every step); achieved = the algorithmic 690 B per env-step / event-timed kernel time"}
    bpe = algorithmic_bytes_per_env_step()
    kern = "quad" if (a.variant == "quad" or (a.variant == "auto" and contacts)) else ("" if contacts else "nc")
    kern = ("ackphys_rollout" if fused else "ackphys_step") + (f"_{kern}" if kern else "") + "_kernel"
    if a.scene == "obstacles":
        kern = "ackphys_rollout_obst8_kernel" if fused else "ackphys_step_obst_kernel"
    rollout_buffer = buffer_leg(contacts) if (fused and not a.no_buffer_leg) else None

    def leg_roofline(kname, c, km):
        """the roofline block of a non-headline leg: the same algorithmic-bytes HBM figure, the
        counter bytes, VALU issue share and the dynamics wave's critical path where profiled"""
        ach = bpe * a.envs / (km * 1e-3) / 1e9
        pm = load_pmc(kname, c, a.steps)
        return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "limiter": "valu-latency", "kernel": kname, "kernel_ms": km,
                "traffic": (pm["hbm_bytes_per_step"] * a.steps if (pm and fused) else None),
                "traffic_unit": "HBM bytes per launch (PMC, profiled separately)",
                "counter_source": pm["source"] if pm else None,
                "critical_path": critical_path(kname, km), "valu": valu_block(pm, km)}
    secondary = None
    if sec_run is not None:
        _, el2, km2, _, _ = sec_run
        k2 = "quad" if (a.variant == "quad" or (a.variant == "auto" and not contacts)) else ("" if not contacts else "nc")
        kern2 = "ackphys_rollout" + (f"_{k2}" if k2 else "") + "_kernel"
        secondary = {"contacts": not contacts, "value": total_envs * a.steps / el2, "ms_per_step": el2 * 1e3 / a.steps,
                     "kernel_ms": km2, "per_step_launch": per_step_leg(not contacts) if do_per_step else None,
                     "roofline": leg_roofline(kern2, not contacts, km2) if fused else None,
                     "untimed_steps": max(a.warmup, SETTLE_STEPS) if not contacts else a.warmup,
                     "flops": oracle_flops("configs[1] contacts off" if contacts else "configs[2] contacts on",
                                           total_envs * a.steps / el2)}
    ppo = None if a.no_ppo else run_ppo(a.envs, rank, world, device)
    obstacles = None
    if not a.no_obstacles:
        _, el3, km3, rets3, _ = run_gpu(a.envs, a.steps, a.warmup, True, rank, world, device, scene="obstacles",
                                        graph=a.graph, per_step=a.per_step)
        obstacles = {"workload": f"v2 robot in ackermann_maze_flat.xml (38 static boxes), {a.envs} envs/GPU, "
                                 "random ctrl, contacts enabled, spawn at the scene's free cell",
                     "value": total_envs * a.steps / el3, "unit": "env-steps/s", "ms_per_step": el3 * 1e3 / a.steps,
                     "kernel": "ackphys_rollout_obst8_kernel" if fused else "ackphys_step_obst_kernel", "kernel_ms": km3,
                     "per_step_launch": per_step_leg(True, "obstacles") if do_per_step else None, "episodes": rets3,
                     "untimed_steps": max(a.warmup, SETTLE_STEPS),
                     "flops": oracle_flops("configs[4] obstacle scene, contacts on", total_envs * a.steps / el3),
                     "roofline": leg_roofline("ackphys_rollout_obst8_kernel", True, km3) if fused else None,
                     "ppo": None if a.no_ppo else run_ppo(a.envs, rank, world, device, scene="obstacles")}
    parity = base = None
    if rank == 0 and not a.no_cpu:
        parity, base = cpu_leg(device, contacts, do_timing=(world == 1))
    achieved = bpe * a.envs / (kern_ms * 1e-3) / 1e9
    pmc = load_pmc(kern, contacts, a.steps)
    valu = valu_block(pmc, kern_ms)
    hbm = {"nominal_bytes_per_step": bpe * a.envs,
           "counter_bytes_per_step": pmc.get("hbm_bytes_per_step") if pmc else None,
           "counter_source": pmc["source"] if pmc else None,
           "note": ("nominal = the algorithmic 690 B per env-step (state in/out, action, obs, reward, flags, "
                    "episode stats); counter = FETCH_SIZE x2 + WRITE_SIZE per step of the profiled launch: "
                    "between steps the state lives in an LDS mirror and in-place outputs stay in L2, so real "
                    "HBM traffic is far below the nominal figure")}
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (Philox random actions from "
            "the reference reset state; random goals)",
            "config": {"workload": f"ackermann_robot_v2.xml, {a.envs} envs/GPU, random ctrl, contacts "
                                   f"{'enabled' if contacts else 'disabled'} (BASELINE configs[{2 if contacts else 1}])",
                       "envs_per_gpu": a.envs, "total_envs": total_envs, "episode_len": 1000,
                       "parallelism": f"dp{world} (independent env shards, 1 all_gather of episode stats)",
                       "backend": backend,
                       "launcher": ("bench.py --gpus N (torch.distributed.run children)" if os.environ.get(
                           "ACKPHYS_SPAWNED") else ("torchrun" if world > 1 else "single process"))},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "limiter": "valu-latency",
                         "frac_basis": ("the headline launch (per-step outputs overwritten in place); the rollout_buffer "
                                        "leg gives the same figure with every step's outputs written to its own slice"),
                         "traffic": (pmc["hbm_bytes_per_step"] * a.steps if (pmc and fused) else
                                     (pmc["hbm_bytes_per_step"] if pmc else None)),
                         "traffic_unit": "HBM bytes per launch (PMC, profiled separately: see hbm.counter_source)",
                         "kernel": kern, "kernel_ms": kern_ms,
                         "critical_path": critical_path(kern, kern_ms), "valu": valu, "hbm": hbm,
                         "mfma": mfma_summary(),
                         "flops": oracle_flops("configs[2] contacts on" if contacts else "configs[1] contacts off",
                                               value),
                         "algorithmic_bytes_per_env_step": bpe,
                         "unit_of_work": (f"one step of {a.envs} envs: achieved = {bpe} B x envs / kernel_ms (HBM, "
                                          "nominal bytes); " + (f"one launch runs all {a.steps} timed steps, so per "
                                                                "launch bytes and time both scale by the step count"
                                                                if fused else "one launch per step")),
                         "note": ("bound/achieved/peak/frac: the HBM roofline the contract asks for, algorithmic "
                                  "bytes over kernel time. HBM is not what limits this kernel: limiter = the "
                                  "dynamics wave's dependent f32 VALU chain (critical_path: its cycles per step "
                                  "are the kernel's); 4096 envs = 64 dynamics + 64 observation + 64 prep waves "
                                  "(lane mapping, contacts off), 192 of 1024 SIMDs")},
            "timing": ("one ackphys_rollout launch of the K timed steps (pre-drawn actions resident in HBM; every "
                       "step computed and its outputs written)" if fused else
                       ("K ackphys_step launches replayed from a hipGraph" if a.graph else
                        "K ackphys_step launches")),
            "per_step_launch": per_step_launch, "rollout_buffer": rollout_buffer,
            "cpu_baseline": base, "parity": parity, "episodes": rets, "secondary": secondary, "ppo": ppo,
            "obstacles": obstacles,
        }
        emit(line)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
