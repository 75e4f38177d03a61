"""Philox4x32-10 known-answer tests (Random123 kat_vectors) and the sharded (gloo) data path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.oracle import philox


@pytest.mark.parametrize("ctr,key,expect", [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
])
def test_philox_kat(ctr, key, expect):
    assert list(philox(ctr, key)) == expect


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from mujoco_playground_amd import shard
    r, w, _ = shard.init(backend="gloo")
    n = 8
    ep = torch.zeros(4, n)
    ep[2] = torch.arange(n, dtype=torch.float32) + 100 * r   # completed-return sums
    ep[3] = 1.0 + r                                           # completed counts
    g = shard.gather_episode_stats(ep, w)
    s = shard.summarize_returns(g)
    m = shard.max_over_ranks(float(r + 1) * 0.5, w, torch.device("cpu"))
    # the PPO learner's collectives: gradient all-reduce (SUM) and the initial parameter broadcast
    grad = torch.full((5,), float(r + 1))
    shard.all_reduce_sum_(grad, w)
    params = torch.full((3,), float(10 * r + 7))
    shard.broadcast_(params, w)
    # the trainer's host-staged all-reduce hook (gloo rehearsals), called through its C function
    # pointer as ackppo_train calls it: f32 gradient and f64 moments buffers, SUM in place
    import ctypes as C
    from mujoco_playground_amd import _lib
    coll = shard.TrainerCollective(w, torch.device("cpu"))
    assert coll.kind == "host"
    g32 = torch.full((6,), float(r + 1))
    m64 = torch.full((4,), 0.5 * (r + 1), dtype=torch.float64)
    coll.register(g32)
    coll.register(m64)
    fn = _lib.ALLREDUCE_FN(coll.fn.value)
    rc = (fn(g32.data_ptr(), 6, 0, None, None), fn(m64.data_ptr(), 4, 1, None, None),
          fn(g32.data_ptr(), 5, 0, None, None))   # an unregistered (ptr, count): reported, not a crash
    q.put((r, shard.env_offset(r, n), tuple(g.shape), s, m, grad.tolist(), params.tolist(),
           (rc, g32.tolist(), m64.tolist())))
    dist.destroy_process_group()


def test_sharded_gather_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    (r0, off0, sh0, s0, m0, g0, p0, h0), (r1, off1, sh1, s1, m1, g1, p1, h1) = res
    assert h0 == h1 == ((0, 0, -1), [3.0] * 6, [1.5] * 4)   # the hook's SUMs; -1 for the unknown buffer
    assert g0 == g1 == [3.0] * 5          # 1 + 2 summed over ranks
    assert p0 == p1 == [7.0] * 3          # rank 0's parameters everywhere
    assert (off0, off1) == (0, 8)
    assert sh0 == sh1 == (2, 4, 8)
    total = sum(range(8)) + sum(100 + i for i in range(8))
    assert s0 == s1 and s0["episodes"] == 8 * 1 + 8 * 2
    assert abs(s0["mean_return"] - total / 24) < 1e-6
    assert m0 == m1 == 1.0
