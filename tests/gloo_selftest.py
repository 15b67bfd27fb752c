"""Rank program of tests/test_distributed_gloo.py's launcher test (test code,
not product): run as N ranks by pixpath.batch.spawn_local, each rank takes
its PVS share (pixpath.batch.my_pvs), computes SI/TI with the numpy oracle
(no GPU on CPU runs) and rank 0 saves the gloo-gathered result.

usage: python tests/gloo_selftest.py OUT.npz [N_PVS]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "processing-chain_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def frames(pvs_index):
    rng = np.random.default_rng(1000 + pvs_index)
    return rng.integers(0, 1024, (5, 24, 40)).astype(np.uint16)


def main(out_path, n_pvs):
    import siti_ref
    from pixpath import batch
    rank, world, _ = batch.rank_env()
    batch.init_group(world)
    ids = ["PVS%03d" % i for i in range(n_pvs)]
    local = {pid: siti_ref.siti(frames(int(pid[3:]))) for pid in batch.my_pvs(ids, rank, world)}
    res = batch.gather_results(local, rank, world)
    if rank == 0:
        keys = sorted(res)
        np.savez(out_path, ids=np.array(keys), world=world, ranks=np.array([res[k]["rank"] for k in keys]),
                 SI=np.array([res[k]["SI"] for k in keys]), TI=np.array([res[k]["TI"] for k in keys]),
                 si=np.stack([res[k]["si"] for k in keys]), ti=np.stack([res[k]["ti"] for k in keys]))
    batch.barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6)
