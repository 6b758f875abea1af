"""One process per GPU: frame sharding and the error-counter all-reduce.

The Monte-Carlo frame loop (run_fer_sweep.py:79-121) has no cross-frame state except the
RNG stream and the counters, so frames are split into contiguous global index ranges per
rank and decoded independently; the only collective is one SUM all-reduce of an int64
counter vector per SNR point (RCCL over xGMI under backend "nccl", gloo on CPU).
The reference is single-process; this module has no reference counterpart.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


@dataclass
class Context:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = ""
    group: bool = False  # a torch.distributed process group is initialised (any world size)

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    @property
    def device(self) -> int:
        """GPU of this rank: its local rank (one process per GPU).  PSCL_SHARE_GPU=1 (one-GPU
        rehearsals of the multi-rank path, gloo backend) folds the ranks onto the visible GPUs."""
        if os.environ.get("PSCL_SHARE_GPU") == "1":
            from . import _native

            return self.local_rank % max(_native.device_count(), 1)
        return self.local_rank


_CTX: Context | None = None


def launcher_env() -> bool:
    """True under a rank launcher (torchrun / bench.py --gpus N): WORLD_SIZE and MASTER_ADDR set."""
    return "WORLD_SIZE" in os.environ and "MASTER_ADDR" in os.environ


def init(backend: str | None = None) -> Context:
    """Initialise torch.distributed from a launcher's environment -- at any world size, so a
    world-1 torchrun job runs the same RCCL collectives as an 8-GPU one -- else a single-process
    context with no group.  backend: "nccl" (RCCL) when the ranks own GPUs, else "gloo"."""
    global _CTX
    if _CTX is not None:
        return _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    group = False
    if world > 1 or launcher_env():
        import torch
        import torch.distributed as dist

        if backend is None:  # PSCL_DIST_BACKEND overrides (gloo rehearsals on a shared GPU)
            backend = os.environ.get("PSCL_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if not dist.is_initialized():
            # an explicit bound: a rank that never joins fails the others' init and collectives
            # instead of holding them to the library default (PSCL_PG_TIMEOUT_S, default 600 s)
            import datetime

            timeout = datetime.timedelta(seconds=float(os.environ.get("PSCL_PG_TIMEOUT_S", "600")))
            if backend == "nccl":
                torch.cuda.set_device(local)
                dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local), timeout=timeout)
            else:
                dist.init_process_group(backend=backend, timeout=timeout)
        group = True
        import sys

        print(f"[dist] process group: backend={dist.get_backend()} world={world} rank={rank}", file=sys.stderr,
              flush=True)
    _CTX = Context(rank=rank, world=world, local_rank=local, backend=backend or "", group=group)
    return _CTX


def _collective(ctx: Context) -> bool:
    """Whether the helpers below run a collective: whenever a process group exists (world 1
    included: the RCCL path then runs on one GPU), never without one."""
    return ctx.group or ctx.world > 1


def shard(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous global frame range [start, stop) of `rank`; ranks differ by at most one frame."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def allreduce_sum(vec: np.ndarray, ctx: Context | None = None) -> np.ndarray:
    """SUM of an int64/float64 vector over all ranks (identity when world == 1)."""
    ctx = ctx or _CTX or Context()
    if not _collective(ctx):
        return np.asarray(vec)
    import torch
    import torch.distributed as dist

    t = torch.as_tensor(np.ascontiguousarray(vec))
    if ctx.backend == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def allgather(vec: np.ndarray, ctx: Context | None = None) -> np.ndarray:
    """[world, len(vec)]: every rank's vector, in rank order (vec[None] when world == 1)."""
    ctx = ctx or _CTX or Context()
    v = np.ascontiguousarray(vec)
    if not _collective(ctx):
        return v[None, :].copy()
    import torch
    import torch.distributed as dist

    t = torch.as_tensor(v)
    if ctx.backend == "nccl":
        t = t.cuda()
    out = [torch.empty_like(t) for _ in range(ctx.world)]
    dist.all_gather(out, t)
    return torch.stack(out).cpu().numpy()


def allreduce_min(x: float, ctx: Context | None = None) -> float:
    ctx = ctx or _CTX or Context()
    if not _collective(ctx):
        return float(x)
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64)
    if ctx.backend == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def allreduce_max(x: float, ctx: Context | None = None) -> float:
    ctx = ctx or _CTX or Context()
    if not _collective(ctx):
        return float(x)
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(x)], dtype=torch.float64)
    if ctx.backend == "nccl":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(ctx: Context | None = None) -> None:
    ctx = ctx or _CTX or Context()
    if _collective(ctx):
        import torch.distributed as dist

        dist.barrier()


def finalize() -> None:
    global _CTX
    if _CTX is not None and _collective(_CTX):
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()
    _CTX = None
