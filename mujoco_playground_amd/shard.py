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


def _abort_group():
    """Tear the default process group down after a local collective error, so the other ranks'
    pending collectives fail (connection closed / communicator aborted) instead of waiting forever
    for this rank -- a local error must not become a distributed hang."""
    try:
        from torch.distributed import distributed_c10d as c10d
        if hasattr(c10d, "_abort_process_group"):
            c10d._abort_process_group()
        else:
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001 -- best effort on an already failing path
        pass


def torch_rccl_comm(device) -> int:
    """The ncclComm_t of torch's ProcessGroupNCCL for `device` (the communicator the default process
    group built and already uses for every other collective of the run). One all-reduce first, so
    the communicator exists (torch creates it lazily on the first collective of the device)."""
    with torch.cuda.device(device):
        t = torch.zeros(1, device=device)
        dist.all_reduce(t)
        torch.cuda.synchronize(device)
        backend = dist.distributed_c10d._get_default_group()._get_backend(torch.device("cuda", device.index))
        ptr = int(backend._comm_ptr())
    if not ptr:
        raise RuntimeError("torch's ProcessGroupNCCL has no communicator for this device")
    return ptr


class TrainerCollective:
    """The all-reduce hook libackppo's ackppo_train calls between a minibatch's gradient and its Adam
    step (include/ackppo.h ackppo_allreduce_fn), so a data-parallel PPO update is one C call per
    train() with no per-minibatch host round trip.

    kind "rccl" (default on the nccl = RCCL backend): a communicator of libackppo's own (ackppo_rccl_*)
      over the ranks of the default process group (its unique id broadcast once over that group), or
      over this process alone at world 1 (a one-rank communicator: the data-parallel path with real
      RCCL calls, for timing it on one GPU). The standard RCCL pattern: ncclCommInitRank from a
      unique id, every collective enqueued from C on the trainer's stream.
    kind "torch" (opt-in until it has run on a multi-GPU node): ackppo_rccl_allreduce on the communicator of
      torch's own ProcessGroupNCCL (torch_rccl_comm): no second communicator, no unique-id exchange,
      and the RCCL library is checked to be the one torch loaded; each collective is enqueued from C
      on the trainer's stream (torch's current stream, so torch's later collectives on the same
      communicator are ordered after them on the device).
    kind "host": a Python callback that all-reduces through torch.distributed on host copies --
      the gloo rehearsals (several ranks on one device, where RCCL cannot run); the callback
      synchronises the stream, so it is the slow path, for tests only. On an error it aborts the
      process group, so the other ranks fail too rather than wait.
    Buffers handed to the "host" hook must be registered (`register`)."""

    def __init__(self, world: int, device, kind: str | None = None):
        import ctypes as C

        from . import _lib
        self.world, self.device = world, device
        self.kind = kind or ("host" if _backend_is_gloo() else "rccl")
        self.L = _lib.ppo_lib()
        self._bufs = {}
        self.comm = C.c_void_p()
        if self.kind in ("torch", "rccl"):
            path = C.create_string_buffer(4096)
            _lib.ppo_check(self.L.ackppo_rccl_library(path, 4096), "ackppo_rccl_library")
            self.library = path.value.decode()
        if self.kind == "torch":
            if not (dist.is_initialized() and dist.get_backend() == "nccl"):
                raise RuntimeError('collective "torch" needs the default process group on the nccl (RCCL) backend')
            torch_lib = _torch_rccl_path()
            if torch_lib is not None and os.path.realpath(torch_lib) != os.path.realpath(self.library):
                raise RuntimeError(f"libackppo resolved RCCL at {self.library}, torch's is {torch_lib}")
            self.user = C.c_void_p(torch_rccl_comm(device))
            self.fn = C.cast(self.L.ackppo_rccl_allreduce, C.c_void_p)
        elif self.kind == "rccl":
            idb = (C.c_char * 128)()
            rank = dist.get_rank() if world > 1 else 0
            if rank == 0:
                _lib.ppo_check(self.L.ackppo_rccl_unique_id(idb), "ackppo_rccl_unique_id")
            if world > 1:
                t = torch.frombuffer(bytearray(bytes(idb)), dtype=torch.uint8).to(device)
                dist.broadcast(t, 0)
                idb = (C.c_char * 128).from_buffer_copy(bytes(t.cpu().numpy()))
            _lib.ppo_check(self.L.ackppo_rccl_init(idb, world, rank, C.byref(self.comm)), "ackppo_rccl_init")
            self.fn = C.cast(self.L.ackppo_rccl_allreduce, C.c_void_p)
            self.user = self.comm
        elif self.kind == "host":
            def hook(buf, count, dtype, user, stream):
                try:
                    t = self._bufs[(buf, count, dtype)]
                    all_reduce_sum_(t, self.world)
                    return 0
                except Exception as e:  # noqa: BLE001 -- reported through the C return code
                    print(f"TrainerCollective host hook: {e!r}; aborting the process group", flush=True)
                    if self.world > 1:
                        _abort_group()
                    return -1
            self._cb = _lib.ALLREDUCE_FN(hook)  # kept alive with the collective
            self.fn = C.cast(self._cb, C.c_void_p)
            self.user = None
        else:
            raise ValueError(f"unknown collective kind {kind!r}")

    def register(self, t: torch.Tensor):
        """A contiguous buffer the trainer all-reduces (host hook lookup by pointer, count, dtype)."""
        dtype = {torch.float32: 0, torch.float64: 1}[t.dtype]
        self._bufs[(t.data_ptr(), t.numel(), dtype)] = t

    def close(self):
        if self.kind == "rccl" and self.comm:
            self.L.ackppo_rccl_destroy(self.comm)
            self.comm = type(self.comm)()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


def _torch_rccl_path():
    """Path of the librccl mapped into this process by torch (None if it cannot be told)."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "librccl" in line:
                    return line.split()[-1]
    except OSError:
        pass
    return None


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
