"""Multi-GPU work split: one process per GPU, no device collective.

* PVS sharding: whole PVSes per rank, longest-first greedy balancing (the
  reference's unit of parallel work, lib/cmd_utils.py ParallelRunner);
* SRC frame-range sharding for SI/TI: contiguous ranges, each rank also reads
  the frame before its range (1-frame halo) so TI is exact at the seams;
* host-side gather of per-frame SI/TI to rank 0 (torch.distributed object
  gather over whatever process group is up -- gloo on CPU, or none at all when
  ranks write files), final SI/TI = max over frames.
"""
import numpy as np


def assign_pvs(items, world, cost=None):
    """Longest-first greedy: list of per-rank item lists.  `cost(item)` defaults to 1."""
    cost = cost or (lambda _: 1)
    order = sorted(items, key=lambda it: (-cost(it), str(it)))
    loads = [0.0] * world
    out = [[] for _ in range(world)]
    for it in order:
        r = min(range(world), key=lambda k: (loads[k], k))
        out[r].append(it)
        loads[r] += cost(it)
    return out


def frame_ranges(n_frames, world):
    """[(start, end)] contiguous split of n_frames over world ranks (sizes differ by <= 1)."""
    base, rem = divmod(n_frames, world)
    out, s = [], 0
    for r in range(world):
        e = s + base + (1 if r < rem else 0)
        out.append((s, e))
        s = e
    return out


def siti_shard(frames, start, end, siti_fn):
    """Run ``siti_fn(frames[start:end], prev)`` with the 1-frame halo."""
    prev = frames[start - 1] if start > 0 else None
    return siti_fn(frames[start:end], prev)


def gather_siti(si, ti, rank, world, group=None):
    """Gather per-frame arrays of every rank to rank 0 (in rank order).  Returns
    (si_all, ti_all, SI, TI) on rank 0 and None elsewhere."""
    import torch.distributed as dist
    obj = (np.asarray(si, np.float64).tolist(), np.asarray(ti, np.float64).tolist())
    if world == 1:
        parts = [obj]
    else:
        parts = [None] * world if rank == 0 else None
        dist.gather_object(obj, parts, dst=0, group=group)
    if rank != 0:
        return None
    si_all = np.concatenate([np.asarray(p[0]) for p in parts])
    ti_all = np.concatenate([np.asarray(p[1]) for p in parts])
    valid = ti_all[~np.isnan(ti_all)]
    return si_all, ti_all, float(si_all.max()), float(valid.max()) if valid.size else float("nan")
