"""GPU parity of libackppo.so (include/ackppo.h) against oracle/ppo_oracle.py (numpy f64).

Tolerances (f32 kernels vs f64 oracle): forward/log_prob/value rel 1e-5 (abs 1e-5), gradient
rel 2e-4 of the gradient's max magnitude per tensor, Adam-updated parameters abs 1e-7 (the step
is lr-scaled), GAE rel 1e-5. Discrete outputs (done flags, minibatch counts) exact.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import ppo_oracle as po

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def P(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def L():
    from mujoco_playground_amd import _lib
    return _lib.ppo_lib()


def S():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def params_dev(seed=1):
    from test_ppo_oracle import _random_params
    flat = _random_params(seed)
    return flat, torch.tensor(flat, dtype=torch.float32, device=DEV)


def test_act_matches_oracle():
    flat, p = params_dev()
    n = 300
    rng = np.random.default_rng(0)
    obs = rng.normal(0, 2, (n, 79)).astype(np.float32)
    soa = torch.tensor(obs.T.copy(), device=DEV)
    rows = torch.zeros(n, 79, device=DEV)
    act, eact, lp, val = (torch.zeros(n, 2, device=DEV), torch.zeros(n, 2, device=DEV), torch.zeros(n, device=DEV),
                          torch.zeros(n, device=DEV))
    f32 = flat.astype(np.float32).astype(np.float64)
    for det in (0, 1):
        assert L().ackppo_act(P(p), P(soa), n, 1000, 0xABCDEF12345, 17, det, P(rows), P(act), P(eact), P(lp), P(val),
                              S()) == 0
        torch.cuda.synchronize()
        a, ea, olp, ov = po.act(f32, obs.astype(np.float64), 0xABCDEF12345, 17, 1000, deterministic=bool(det))
        np.testing.assert_allclose(act.cpu().numpy(), a, rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(eact.cpu().numpy(), ea, rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(lp.cpu().numpy(), olp, rtol=1e-5, atol=2e-5)
        np.testing.assert_allclose(val.cpu().numpy(), ov, rtol=1e-5, atol=2e-5)
        np.testing.assert_array_equal(rows.cpu().numpy(), obs)
    vv = torch.zeros(n, device=DEV)
    assert L().ackppo_value(P(p), P(soa), n, P(vv), S()) == 0
    torch.cuda.synchronize()
    np.testing.assert_allclose(vv.cpu().numpy(), ov, rtol=1e-5, atol=2e-5)


def test_act_boot_equals_act_plus_bootstrap():
    """ackppo_act_boot = ackppo_act (bit-identical: the same kernel path for the policy outputs) and
    ackppo_bootstrap's rewards / done flags for the previous step (the oracle's bootstrap); the
    truncations sit in a few 16-env workgroups only, so both the critic branch and its skip run."""
    flat, p = params_dev(3)
    n = 301
    rng = np.random.default_rng(5)
    obs = rng.normal(0, 2, (n, 79)).astype(np.float32)
    tobs = rng.normal(0, 1, (n, 79)).astype(np.float32)
    rew = rng.normal(0, 1, n).astype(np.float32)
    term = np.zeros(n, np.uint8)
    trunc = np.zeros(n, np.uint8)
    trunc[[3, 17, 18, 200, 300]] = 1
    term[[17, 40]] = 1                     # env 17: terminated and truncated -> no bootstrap
    t = lambda a: torch.tensor(a, device=DEV)
    soa, tsoa = t(obs.T.copy()), t(tobs.T.copy())

    def outs():
        return [torch.zeros(n, 79, device=DEV), torch.zeros(n, 2, device=DEV), torch.zeros(n, 2, device=DEV),
                torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)]
    a1, a2 = outs(), outs()
    assert L().ackppo_act(P(p), P(soa), n, 7, 99, 3, 0, *[P(x) for x in a1], S()) == 0
    ro, do = torch.full((n,), -7.0, device=DEV), torch.full((n,), -7.0, device=DEV)
    assert L().ackppo_act_boot(P(p), P(soa), n, 7, 99, 3, 0, *[P(x) for x in a2], P(tsoa), P(t(rew)), P(t(term)),
                               P(t(trunc)), 0.99, P(ro), P(do), S()) == 0
    torch.cuda.synchronize()
    for x, y in zip(a1, a2):
        assert torch.equal(x, y)
    r_ref, d_ref = po.bootstrap(flat.astype(np.float32).astype(np.float64), tobs, rew, term, trunc, 0.99)
    np.testing.assert_allclose(ro.cpu().numpy(), r_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(do.cpu().numpy(), d_ref)
    boot = (trunc == 1) & (term == 0)
    assert np.array_equal(ro.cpu().numpy()[~boot], rew[~boot]) and not np.allclose(r_ref[boot], rew[boot])
    # the rollout's last step bootstraps through ackppo_bootstrap: bit for bit the same rewards and
    # flags as act_boot gives every other step (one critic path for the whole rollout)
    rb, db = torch.full((n,), -7.0, device=DEV), torch.full((n,), -7.0, device=DEV)
    assert L().ackppo_bootstrap(P(p), P(tsoa), P(t(rew)), P(t(term)), P(t(trunc)), n, 0.99, P(rb), P(db), S()) == 0
    vv = torch.zeros(n, device=DEV)
    assert L().ackppo_value(P(p), P(soa), n, P(vv), S()) == 0
    torch.cuda.synchronize()
    assert torch.equal(rb, ro) and torch.equal(db, do)
    assert torch.equal(vv, a1[4])  # ackppo_value = the act kernel's values bit for bit


def test_checkpoint_policy_on_gpu():
    d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "ppo_policy.npz"))
    for k in (10000, 20000, 30000):
        p = torch.tensor(d[f"params_{k}"], device=DEV)
        soa = torch.tensor(d[f"obs_{k}"].reshape(79, 1).astype(np.float32), device=DEV)
        ea, a, v = torch.zeros(1, 2, device=DEV), torch.zeros(1, 2, device=DEV), torch.zeros(1, device=DEV)
        assert L().ackppo_act(P(p), P(soa), 1, 0, 0, 0, 1, None, P(a), P(ea), None, P(v), S()) == 0
        torch.cuda.synchronize()
        np.testing.assert_allclose(a.cpu().numpy()[0], d[f"mu_{k}"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(v.item(), d[f"value_{k}"][0], rtol=1e-5)


def test_bootstrap_and_gae_match_oracle():
    flat, p = params_dev(2)
    n, T = 257, 9
    rng = np.random.default_rng(1)
    tobs = rng.normal(0, 1, (n, 79)).astype(np.float32)
    rew = rng.normal(0, 1, n).astype(np.float32)
    term = (rng.random(n) < 0.2).astype(np.uint8)
    trunc = (rng.random(n) < 0.3).astype(np.uint8)
    ro, do = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    assert L().ackppo_bootstrap(P(p), P(torch.tensor(tobs.T.copy(), device=DEV)), P(torch.tensor(rew, device=DEV)),
                                P(torch.tensor(term, device=DEV)), P(torch.tensor(trunc, device=DEV)), n, 0.99, P(ro),
                                P(do), S()) == 0
    torch.cuda.synchronize()
    r_ref, d_ref = po.bootstrap(flat.astype(np.float32).astype(np.float64), tobs, rew, term, trunc, 0.99)
    np.testing.assert_allclose(ro.cpu().numpy(), r_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(do.cpu().numpy(), d_ref)
    R, V = rng.normal(size=(T, n)).astype(np.float32), rng.normal(size=(T, n)).astype(np.float32)
    ST = (rng.random((T, n)) < 0.1).astype(np.float32)
    lv, ld = rng.normal(size=n).astype(np.float32), (rng.random(n) < 0.2).astype(np.float32)
    adv, ret = torch.zeros(T, n, device=DEV), torch.zeros(T, n, device=DEV)
    t = lambda a: torch.tensor(a, device=DEV)
    assert L().ackppo_gae(P(t(R)), P(t(V)), P(t(ST)), P(t(lv)), P(t(ld)), T, n, 0.99, 0.95, P(adv), P(ret), S()) == 0
    torch.cuda.synchronize()
    a_ref, r_ref = po.gae(R.astype(np.float64), V.astype(np.float64), ST, lv, ld, 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), a_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.cpu().numpy(), r_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("batch,ent_coef", [(64, 0.0), (200, 0.01), (1, 0.0), (4096, 0.0)])
def test_minibatch_gradient_and_adam_match_oracle(batch, ent_coef):
    flat, p = params_dev(3)
    f32 = flat.astype(np.float32).astype(np.float64)
    rng = np.random.default_rng(batch)
    S_ = 5000
    obs = rng.normal(0, 1.5, (S_, 79)).astype(np.float32)
    f = po.forward(f32, obs)
    acts = (f["mu"] + np.exp(f["log_std"]) * rng.normal(0, 1, (S_, 2))).astype(np.float32)
    old = (po.log_prob(f["mu"], f["log_std"], acts.astype(np.float64)) + rng.normal(0, 0.3, S_)).astype(np.float32)
    adv = rng.normal(0.3, 2.0, S_).astype(np.float32)
    ret = (f["value"] + rng.normal(0, 1, S_)).astype(np.float32)
    idx = rng.permutation(S_)[:batch].astype(np.int32)
    t = lambda a: torch.tensor(a, device=DEV)
    stats = torch.zeros(1, 2, device=DEV)
    assert L().ackppo_adv_stats(P(t(adv)), P(t(idx)), batch, batch, 1, P(stats), S()) == 0
    nblk = L().ackppo_grad_blocks(batch)
    gpart, lpart = torch.zeros(nblk, po.NPARAM, device=DEV), torch.zeros(nblk, 8, device=DEV)
    grad, loss = torch.zeros(po.NPARAM, device=DEV), torch.zeros(8, device=DEV)
    assert L().ackppo_grad(P(p), P(t(obs)), P(t(acts)), P(t(old)), P(t(adv)), P(t(ret)), P(t(idx)), batch, P(stats),
                           0.2, ent_coef, 0.5, P(gpart), P(lpart), S()) == 0
    assert L().ackppo_reduce(P(gpart), P(lpart), nblk, ent_coef, P(grad), P(loss), S()) == 0
    torch.cuda.synchronize()
    st, g_ref = po.loss_and_grad(f32, obs[idx].astype(np.float64), acts[idx].astype(np.float64),
                                 old[idx].astype(np.float64), adv[idx].astype(np.float64), ret[idx].astype(np.float64),
                                 0.2, ent_coef, 0.5)
    g = grad.cpu().numpy().astype(np.float64)
    for k, (o, s) in po.LAYOUT.items():
        n_ = int(np.prod(s))
        scale = max(np.abs(g_ref[o:o + n_]).max(), 1e-6)
        err = np.abs(g[o:o + n_] - g_ref[o:o + n_]).max() / scale
        assert err < 2e-4, f"{k}: rel err {err:.2e}"
    lo = loss.cpu().numpy()
    assert lo[4] == batch
    np.testing.assert_allclose(lo[0] / batch, st["policy_gradient_loss"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(lo[1] / batch, st["value_loss"], rtol=1e-4)
    # Adam + clip on the same gradient
    m, v, norm_out = torch.zeros(po.NPARAM, device=DEV), torch.zeros(po.NPARAM, device=DEV), torch.zeros(1, device=DEV)
    p2 = p.clone()
    assert L().ackppo_adam(P(p2), P(grad), P(m), P(v), 1.0, 0.5, 0.9, 0.999, 1e-5, 3e-4 / 0.1, (1 - 0.999) ** 0.5,
                           P(norm_out), S()) == 0
    torch.cuda.synchronize()
    new_ref, _, _, norm_ref = po.clip_and_adam(f32, g, np.zeros(po.NPARAM), np.zeros(po.NPARAM), 1)
    np.testing.assert_allclose(norm_out.item(), norm_ref, rtol=1e-5)
    np.testing.assert_allclose(p2.cpu().numpy(), new_ref, atol=1e-7)


def test_ppo_learn_end_to_end():
    """PPO.learn on the batched env: Adam step structure, finite state, surrogate improves."""
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    venv = make_ackermann_env(env_type="vec", num_envs=256, max_episode_steps=64, device=DEV)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=1024, n_epochs=4, seed=3, ent_coef=0.01)
    model.learn(total_timesteps=3 * 32 * 256)
    assert model.adam_step == 3 * 4 * (32 * 256 // 1024)
    assert model.num_timesteps == 3 * 32 * 256
    assert torch.isfinite(model.params).all()
    lg = model.logger
    assert np.isfinite(lg["train/value_loss"]) and 0.0 <= lg["train/clip_fraction"] <= 1.0
    assert lg["rollout/episodes_total"] >= 256  # every env truncated at 64 steps at least once in 96
    a, _ = model.predict(venv.sim.obs_soa.t(), deterministic=True)
    assert a.shape == (256, 2) and float(a.abs().max()) <= 1.0


def _perm_ref(n, seed, epoch):
    """Python restatement of ackppo_permutation (4-round Feistel + cycle walking)."""
    M64, M32 = (1 << 64) - 1, (1 << 32) - 1
    bits = 1
    while (1 << bits) < n:
        bits += 1
    half = (bits + 1) // 2
    z = (seed ^ (0x9E3779B97F4A7C15 * (epoch + 1))) & M64
    keys = []
    for _ in range(4):
        z = (z + 0x9E3779B97F4A7C15) & M64
        y = z
        y = ((y ^ (y >> 30)) * 0xBF58476D1CE4E5B9) & M64
        y = ((y ^ (y >> 27)) * 0x94D049BB133111EB) & M64
        keys.append((y ^ (y >> 31)) & M32)

    def h(x, k):
        x = ((x ^ k) * 0x9E3779B1) & M32
        x ^= x >> 16
        x = (x * 0x85EBCA6B) & M32
        x ^= x >> 13
        x = (x * 0xC2B2AE35) & M32
        return x ^ (x >> 16)
    mask = (1 << half) - 1
    out = []
    for i in range(n):
        x = i
        while True:
            L, R = x >> half, x & mask
            for k in keys:
                L, R = R, L ^ (h(R, k) & mask)
            x = (L << half) | R
            if x < n:
                break
        out.append(x)
    return np.array(out, np.int32)


def test_permutation_kernel():
    """ackppo_permutation: a bijection of 0..n-1, bit-exact with the Python restatement, keyed by
    (seed, epoch)."""
    for n in (1, 2, 3, 7, 1000, 4096, 100003, 131072):
        out = torch.empty(n, dtype=torch.int32, device=DEV)
        assert L().ackppo_permutation(n, 12345, 3, P(out), S()) == 0
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        np.testing.assert_array_equal(np.sort(o), np.arange(n))
        if n <= 4096:
            np.testing.assert_array_equal(o, _perm_ref(n, 12345, 3))
    n = 131072
    a, b, c = (torch.empty(n, dtype=torch.int32, device=DEV) for _ in range(3))
    L().ackppo_permutation(n, 12345, 3, P(a), S())
    L().ackppo_permutation(n, 12345, 4, P(b), S())
    L().ackppo_permutation(n, 12346, 3, P(c), S())
    torch.cuda.synchronize()
    assert (a != b).float().mean().item() > 0.99 and (a != c).float().mean().item() > 0.99


def _moments_stats(adv_list, idx_list, n_idx, batch, normalize=1):
    """The data-parallel statistics path with the all-reduces done on the host: one moments
    buffer per 'rank', rows 0..1 summed after phase 0 and row 2 after phase 1."""
    nmb = (n_idx + batch - 1) // batch
    moms = [torch.zeros(3, nmb, dtype=torch.float64, device=DEV) for _ in adv_list]
    for a, i, m in zip(adv_list, idx_list, moms):
        assert L().ackppo_adv_moments(P(a), P(i), n_idx, batch, 0, P(m), S()) == 0
    tot = sum(m[0:2] for m in moms)
    for m in moms:
        m[0:2].copy_(tot)
    for a, i, m in zip(adv_list, idx_list, moms):
        assert L().ackppo_adv_moments(P(a), P(i), n_idx, batch, 1, P(m), S()) == 0
    tot2 = sum(m[2] for m in moms)
    stats = torch.zeros(nmb, 2, device=DEV)
    moms[0][2].copy_(tot2)
    assert L().ackppo_adv_finalize(P(moms[0]), nmb, normalize, P(stats), S()) == 0
    torch.cuda.synchronize()
    return stats.cpu().numpy()


@pytest.mark.parametrize("n_idx,batch", [(5000, 1000), (20000, 8192), (9, 1), (70000, 65536)])
def test_adv_moments_world1_equals_adv_stats(n_idx, batch):
    """At world 1 the data-parallel statistics path reproduces ackppo_adv_stats bit for bit."""
    rng = np.random.default_rng(n_idx)
    adv = torch.tensor(rng.normal(0.4, 3.0, n_idx).astype(np.float32), device=DEV)
    idx = torch.tensor(rng.permutation(n_idx).astype(np.int32), device=DEV)
    nmb = (n_idx + batch - 1) // batch
    ref = torch.zeros(nmb, 2, device=DEV)
    assert L().ackppo_adv_stats(P(adv), P(idx), n_idx, batch, 1, P(ref), S()) == 0
    np.testing.assert_array_equal(_moments_stats([adv], [idx], n_idx, batch), ref.cpu().numpy())


def test_adv_moments_two_ranks_normalise_the_world_minibatch():
    """Two ranks' minibatch m together form the world minibatch; the statistics are those of the
    union (mean and unbiased std in float64), as one SB3 learner with 2 x batch samples."""
    rng = np.random.default_rng(5)
    n_idx, batch = 6000, 1500
    advs = [rng.normal(mu, sd, n_idx).astype(np.float32) for mu, sd in ((0.0, 1.0), (2.0, 4.0))]
    idxs = [rng.permutation(n_idx).astype(np.int32) for _ in advs]
    got = _moments_stats([torch.tensor(a, device=DEV) for a in advs], [torch.tensor(i, device=DEV) for i in idxs],
                         n_idx, batch)
    for m in range(n_idx // batch):
        u = np.concatenate([a[i[m * batch:(m + 1) * batch]].astype(np.float64) for a, i in zip(advs, idxs)])
        np.testing.assert_allclose(got[m, 0], u.mean(), rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(got[m, 1], 1.0 / (u.std(ddof=1) + 1e-8), rtol=1e-6)


def test_train_paths_bit_identical():
    """PPO.train is one ackppo_train call. Its single-rank sequence (no hook) and the data-parallel
    sequence over one rank -- RCCL on libackppo's own communicator (kind "rccl", the default at world > 1),
    on torch's own communicator ("torch"; a one-rank nccl process group here) and the host-staged
    hook (the gloo rehearsals' path, a no-op at world 1), each with every epoch's advantage moments
    formed at the start of the call (2 collectives per call) and with per-epoch moments -- give
    bit-identical parameters, Adam moments and loss statistics."""
    import torch.distributed as dist
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    made = False
    if not dist.is_initialized():
        # the way shard.init builds it (no device_id: torch creates the communicator lazily, at the first
        # collective on the rank's current device), so the communicator under test is the production one
        torch.cuda.set_device(torch.device(DEV))
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
        made = True
    out = []
    try:
        for coll, epochs_buf in ((None, True), ("torch", True), ("torch", False), ("rccl", True), ("rccl", False),
                                 ("host", True), ("host", False)):
            venv = make_ackermann_env(env_type="vec", num_envs=256, max_episode_steps=64, device=DEV)
            model = PPO("MlpPolicy", venv, n_steps=16, batch_size=1000, n_epochs=3, seed=7, ent_coef=0.01,
                        collective=coll)
            model.set_epoch_buffers(epochs_buf)
            assert (model.collective is None) == (coll is None)
            model.learn(total_timesteps=2 * 16 * 256)
            out.append((model.params.cpu().numpy(), model.exp_avg_sq.cpu().numpy(), model.adam_step,
                        model.logger["train/value_loss"], model.logger["train/approx_kl"]))
            if coll is not None:
                model.set_collective(None)
    finally:
        if made:
            dist.destroy_process_group()
    for o in out[1:]:
        np.testing.assert_array_equal(out[0][0], o[0])
        np.testing.assert_array_equal(out[0][1], o[1])
        assert out[0][2:] == o[2:]


def _ppo_rank_rccl(rank, world, port, kind, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from mujoco_playground_amd import shard
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    if kind == "host":
        shard.init(backend="gloo")
    else:
        shard.init(backend="nccl")
    dev = shard.device_for(rank) if kind != "host" else torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    venv = AckermannVecEnv(128, device=dev, seed=0, contacts=True, env_offset=shard.env_offset(rank, 128))
    model = PPO("MlpPolicy", venv, n_steps=8, batch_size=256, n_epochs=2, seed=rank + 1,
                collective=None if kind == "host" else kind)
    model.learn(total_timesteps=2 * 8 * 128 * world)
    q.put((rank, model.params.cpu().numpy(), model.adam_step))
    dist.destroy_process_group()


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs 2 GPUs")
def test_ppo_data_parallel_rccl_two_gpus():
    """Two ranks on two GPUs over RCCL (libackppo's own communicator, the default; and torch's): both
    ranks end with bit-identical parameters, equal to the host-hook (gloo) result of the same run."""
    import socket
    import torch.multiprocessing as mp
    res = {}
    for kind in ("host", "torch", "rccl"):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_ppo_rank_rccl, args=(r, 2, port, kind, q)) for r in range(2)]
        for p in ps:
            p.start()
        got = sorted((q.get(timeout=300) for _ in ps), key=lambda t: t[0])
        for p in ps:
            p.join(timeout=60)
        assert np.array_equal(got[0][1], got[1][1]), kind
        res[kind] = got[0][1]
    np.testing.assert_array_equal(res["host"], res["torch"])
    np.testing.assert_array_equal(res["host"], res["rccl"])


def test_train_matches_epoch_calls():
    """ackppo_train (world 1, no hook: every epoch's shuffle and statistics from one launch) = per epoch
    ackppo_permutation + ackppo_adv_stats + ackppo_epoch (grad -> reduce + Adam launches), bit for bit."""
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    venv = make_ackermann_env(env_type="vec", num_envs=256, max_episode_steps=64, device=DEV)
    model = PPO("MlpPolicy", venv, n_steps=16, batch_size=1000, n_epochs=3, seed=7, ent_coef=0.01)
    model.collect_rollouts()
    snap = [t.clone() for t in (model.params, model.exp_avg, model.exp_avg_sq)]
    model.train()
    got = [t.clone() for t in (model.params, model.exp_avg, model.exp_avg_sq, model.loss_acc)]
    for t, v in zip((model.params, model.exp_avg, model.exp_avg_sq), snap):
        t.copy_(v)
    model.loss_acc.zero_()
    n_idx, B = 16 * 256, 1000
    nmb = (n_idx + B - 1) // B
    step0 = model.adam_step - 3 * nmb
    for ep in range(3):
        assert L().ackppo_permutation(n_idx, model.perm_key, ep, P(model.perm), S()) == 0
        assert L().ackppo_adv_stats(P(model.buf_adv), P(model.perm), n_idx, B, 1, P(model.mb_stats), S()) == 0
        assert L().ackppo_epoch(P(model.params), P(model.buf_obs), P(model.buf_act), P(model.buf_logp),
                                P(model.buf_adv), P(model.buf_ret), P(model.perm), n_idx, B, P(model.mb_stats), 0.2, 0.01,
                                0.5, 0.5, 3e-4, 0.9, 0.999, 1e-5, step0 + ep * nmb, P(model.gpart), P(model.lpart),
                                P(model.grad), P(model.loss_acc), P(model.exp_avg), P(model.exp_avg_sq),
                                P(model.gnorm), S()) == 0
    for a, b in zip(got, (model.params, model.exp_avg, model.exp_avg_sq, model.loss_acc)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("normalize", [True, False])
def test_train_options_bit_identical(normalize):
    """ackppo_train's optional buffers change where work happens, not the result: every epoch's
    shuffle and statistics from one launch (perm_epochs / stats_epochs; here with a 10 000-sample
    minibatch, past the statistics kernel's 8 192 register-cached samples, and a ragged last one) or
    per-epoch launches, and the gradient kernel staging from the weight image or from the
    parameters -- the same parameters, Adam moments and losses, bit for bit."""
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    out = []
    for epochs_buf, image in ((True, False), (False, False), (True, True), (False, True)):
        venv = make_ackermann_env(env_type="vec", num_envs=1024, max_episode_steps=64, device=DEV)
        model = PPO("MlpPolicy", venv, n_steps=16, batch_size=10000, n_epochs=2, seed=11, ent_coef=0.01,
                    normalize_advantage=normalize)
        model.set_epoch_buffers(epochs_buf)
        model.set_weight_image(image)
        model.learn(total_timesteps=2 * 16 * 1024)
        out.append((model.params.cpu().numpy(), model.exp_avg_sq.cpu().numpy(), model.logger["train/value_loss"],
                    model.logger["train/approx_kl"]))
    for o in out[1:]:
        np.testing.assert_array_equal(out[0][0], o[0])
        np.testing.assert_array_equal(out[0][1], o[1])
        assert out[0][2:] == o[2:]


@pytest.mark.parametrize("variant", [{}, {"action_repeat": 5, "nohit_clear": True}])
def test_obstacle_scene_ppo_4096(variant):
    """PPO on the obstacle scene at the bench's per-GPU shape (4096 envs; the fused rollout in the obst8
    kernel), the single-rank update and the data-parallel one over a one-rank RCCL communicator
    bit-equal, with the reference task and with the opt-in learnable variant."""
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    out = []
    for coll in (None, "rccl"):
        venv = AckermannVecEnv(4096, device=DEV, seed=4, contacts=True, scene="obstacles", max_episode_steps=24,
                               **variant)
        model = PPO("MlpPolicy", venv, n_steps=16, batch_size=8192, n_epochs=2, seed=5, ent_coef=0.01,
                    collective=coll)
        assert model.fused_rollout
        model.learn(total_timesteps=3 * 16 * 4096)
        assert torch.isfinite(model.params).all()
        lg = model.logger
        assert np.isfinite(lg["train/value_loss"]) and np.isfinite(lg["train/policy_gradient_loss"])
        assert lg["rollout/episodes_total"] >= 4096   # truncation at 24 steps within 48
        out.append((model.params.cpu().numpy(), model.exp_avg_sq.cpu().numpy(), model.adam_step,
                    lg["train/value_loss"], lg["train/approx_kl"], lg["rollout/ep_rew_mean"]))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert out[0][2:] == out[1][2:]


def _ppo_rank(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from mujoco_playground_amd import shard
    from mujoco_playground_amd.rl import AckermannVecEnv
    from mujoco_playground_amd.rl.ppo import PPO
    shard.init(backend="gloo")  # both ranks share cuda:0 here; on a node each rank owns a GPU (RCCL)
    venv = AckermannVecEnv(128, device="cuda:0", seed=0, contacts=True, env_offset=shard.env_offset(rank, 128))
    model = PPO("MlpPolicy", venv, n_steps=8, batch_size=256, n_epochs=2, seed=rank + 1)  # rank-dependent init ...
    model.learn(total_timesteps=2 * 8 * 128 * world)
    q.put((rank, model.params.cpu().numpy(), model.adam_step, model.num_timesteps))
    dist.destroy_process_group()


def test_ppo_data_parallel_two_ranks():
    """DP PPO: rank 0's parameters are broadcast once and every minibatch gradient is summed over
    ranks, so both ranks hold bit-identical parameters after learning."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ppo_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    (_, p0, s0, n0), (_, p1, s1, n1) = res
    assert np.isfinite(p0).all() and np.array_equal(p0, p1)  # ... yet identical after the broadcast + all-reduce
    assert s0 == s1 == 2 * 2 * (8 * 128 // 256) and n0 == n1 == 2 * 8 * 128 * 2


def test_ppo_learns_the_variant_task():
    """The learner learns goal reaching on the opt-in learnable variant (action_repeat 10, nohit_clear;
    include/ackphys.h): deterministic-policy success from fresh resets rises from 0 to >= 5 % within 200
    PPO iterations (52 M env-steps; profiles/train/r03_variant_r10*.jsonl: 11 % at 100, 69 % at 1500).
    At 100 iterations the number is seed noise (1-24 % over seeds 0-3 and 1-ulp solver changes,
    tools/probes/variant_learn.py); at 200 every measured seed and build is >= 10 %.
    The reference task itself cannot be learned."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from train_ppo import evaluate
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    kw = dict(action_repeat=10, nohit_clear=True)
    venv = make_ackermann_env(env_type="vec", num_envs=4096, device=DEV, seed=0, max_episode_steps=1000, **kw)
    model = PPO("MlpPolicy", venv, n_steps=64, batch_size=8192, n_epochs=10, seed=0)
    assert model.fused_rollout
    s0, _, _ = evaluate(model, horizon=1000, **kw)
    model.learn(total_timesteps=200 * 64 * 4096)
    s1, steps, _ = evaluate(model, horizon=1000, **kw)
    print("success", s0, "->", s1, "steps to goal", steps)
    assert s0 == 0.0 and s1 >= 0.05


def test_log_std_floor():
    """The opt-in entropy floor (log_std_min; include/ackppo.h): after every Adam step log_std >= the
    floor -- a policy started below it is lifted to it at the first update -- the same bits on the
    single-rank launch and on the data-parallel sequence (one-rank RCCL hook: separate Adam launch);
    None leaves the SB3 update untouched."""
    from mujoco_playground_amd.rl import make_ackermann_env
    from mujoco_playground_amd.rl.ppo import PPO
    out = []
    for coll in (None, "rccl"):
        venv = make_ackermann_env(env_type="vec", num_envs=256, max_episode_steps=64, device=DEV)
        model = PPO("MlpPolicy", venv, n_steps=16, batch_size=1000, n_epochs=2, seed=3, log_std_min=-0.5,
                    collective=coll)
        model.params[:2] = -2.0
        model.learn(total_timesteps=2 * 16 * 256)
        ls = model.params[:2].cpu().numpy()
        assert (ls >= -0.5).all(), ls
        out.append(model.params.cpu().numpy())
    np.testing.assert_array_equal(out[0], out[1])
