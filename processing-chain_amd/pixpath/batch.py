"""PVS batches over the GPUs of one node (BASELINE config 5).

The reference's unit of parallel work is one PVS command run by a
``ParallelRunner`` pool of OS processes (lib/cmd_utils.py:93-101).  Here the
unit stays the PVS and the pool becomes one process per GPU:

* ``spawn_local(n, argv)`` -- the parent starts ``n`` copies of ``argv`` with
  RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (the same
  variables ``torch.distributed.run`` sets) and waits for them.  The parent
  never initialises HIP: it imports neither torch nor the native library.
* ``rank_env()`` -- (rank, world, local_rank) of this process; GPU = local_rank
  (a deterministic slot, not a function of the process id).
* ``init_group(world)`` -- a gloo process group for the host-side exchange
  (timing barrier, max-reduce, SI/TI gather).  No RCCL: the path has no
  device-side exchange.
* ``my_pvs(ids, rank, world)`` -- this rank's share (pixpath.shard.assign_pvs,
  longest-first balancing).
* ``gather_results(local, rank, world)`` -- per-PVS per-frame SI/TI of every
  rank to rank 0, which derives SI = max_n SI_n and TI = max_n TI_n per PVS.
"""
import os
import socket
import subprocess

import numpy as np

from . import shard


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_local(nprocs, argv, port=None, env=None):
    """Run ``argv`` as ``nprocs`` ranks on this node; return the worst exit code.

    Children inherit stdout/stderr (rank 0 prints the result)."""
    port = port or free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(argv, env=e))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def rank_env():
    """(rank, world, local_rank) from the launcher's environment (1 process: 0, 1, 0)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_group(world):
    """gloo group over MASTER_ADDR/MASTER_PORT (env://); None for one process."""
    if world <= 1:
        return None
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    return dist.group.WORLD


def my_pvs(ids, rank, world, cost=None):
    return shard.assign_pvs(list(ids), world, cost=cost)[rank]


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(value, world):
    if world <= 1:
        return float(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_values(value, rank, world):
    """[value of rank 0, value of rank 1, ...] on rank 0 (None elsewhere)."""
    if world == 1:
        return [value]
    import torch.distributed as dist
    parts = [None] * world if rank == 0 else None
    dist.gather_object(value, parts, dst=0)
    return parts if rank == 0 else None


def gather_results(local, rank, world):
    """``local``: {pvs_id: (si_frames, ti_frames)} of this rank.  Returns, on
    rank 0, {pvs_id: {"si", "ti", "SI", "TI", "rank"}} over all ranks (None on
    the others).  TI ignores its undefined first frame (NaN)."""
    payload = {k: (np.asarray(v[0], np.float64), np.asarray(v[1], np.float64)) for k, v in local.items()}
    parts = gather_values(payload, rank, world)
    if rank != 0:
        return None
    out = {}
    for r, part in enumerate(parts):
        for k, (si, ti) in part.items():
            valid = ti[~np.isnan(ti)]
            out[k] = {"si": si, "ti": ti, "SI": float(si.max()) if si.size else float("nan"),
                      "TI": float(valid.max()) if valid.size else float("nan"), "rank": r}
    return out
