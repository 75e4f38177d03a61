"""Env sharding across ranks (one process per GPU, torch.distributed over RCCL/xGMI).

Envs are independent (no coupling anywhere in the step), so rank r simply owns global envs
[r*n, (r+1)*n) and keys its Philox streams with that offset: an 8-GPU run steps exactly the
envs an unsharded run would. The only collective on the data path is one all-gather of the
per-env episode statistics per rollout (16 B/env, latency-bound over xGMI).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def dist_env():
    """(rank, world, local_rank) from torchrun's environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env. Backend: "nccl" (= RCCL on ROCm) when a
    GPU is present; ACKPHYS_DIST_BACKEND overrides it (rehearsals of N ranks on one GPU use gloo)."""
    rank, world, local = dist_env()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or os.environ.get("ACKPHYS_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":  # RCCL binds the rank's communicator to its current device
            torch.cuda.set_device(device_for(local))
        dist.init_process_group(backend=backend)
    return rank, world, local


def device_for(local_rank: int) -> torch.device:
    """cuda:<local_rank>; ACKPHYS_DEVICE_OVERRIDE pins every rank to one device (rehearsal only)."""
    ov = os.environ.get("ACKPHYS_DEVICE_OVERRIDE")
    return torch.device("cuda", int(ov) if ov is not None else local_rank)


def _backend_is_gloo() -> bool:
    return dist.is_initialized() and dist.get_backend() == "gloo"


def env_offset(rank: int, envs_per_rank: int) -> int:
    return rank * envs_per_rank


def gather_episode_stats(episode: torch.Tensor, world: int) -> torch.Tensor:
    """episode [4, n] (running return, running length, completed-return sum, completed count)
    -> [world, 4, n] on every rank (one all_gather_into_tensor)."""
    if world == 1:  # nothing to exchange: a view, no copy launch inside a timed region
        return episode.unsqueeze(0)
    src = episode.contiguous()
    if _backend_is_gloo() and src.is_cuda:
        src = src.cpu()
    out = torch.empty((world * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src)
    return out.view((world,) + tuple(episode.shape)).to(episode.device)


def summarize_returns(gathered: torch.Tensor) -> dict:
    """Mean completed-episode return / count over all ranks and envs."""
    s = gathered[:, 2].sum().item()
    c = gathered[:, 3].sum().item()
    return {"episodes": int(c), "mean_return": (s / c) if c > 0 else None}


def max_over_ranks(x: float, world: int, device) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if _backend_is_gloo() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(world: int, device=None):
    if world > 1:
        if device is not None and device.type == "cuda" and not _backend_is_gloo():
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def all_reduce_sum_(t: torch.Tensor, world: int) -> torch.Tensor:
    """In-place SUM over ranks (RCCL on device; gloo rehearsals go through host memory)."""
    if world == 1:
        return t
    if _backend_is_gloo() and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)
    return t


def broadcast_(t: torch.Tensor, world: int, src: int = 0) -> torch.Tensor:
    if world == 1:
        return t
    if _backend_is_gloo() and t.is_cuda:
        h = t.cpu()
        dist.broadcast(h, src)
        t.copy_(h)
    else:
        dist.broadcast(t, src)
    return t
