"""N>1 path on CPU: world_size-2 gloo process group.

Frame-range sharding of one SRC with a 1-frame TI halo, per-rank SI/TI, host
gather to rank 0 == the single-process result; PVS assignment is balanced and
complete.  The per-rank compute is the numpy reference here (no GPU); the GPU
tests check the HIP kernel gives the same numbers with the halo."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import siti_ref
from pixpath import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frames():
    rng = np.random.default_rng(2024)
    base = rng.integers(64, 941, (48, 64)).astype(np.int64)
    return np.stack([(np.roll(base, t, axis=1) + 3 * t) % 1024 for t in range(11)]).astype(np.uint16)


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = _frames()
    s, e = shard.frame_ranges(len(frames), world)[rank]
    si, ti = shard.siti_shard(frames, s, e, lambda f, p: siti_ref.siti(f, prev=p))
    res = shard.gather_siti(si, ti, rank, world)
    if rank == 0:
        np.savez(os.path.join(out_dir, "res.npz"), si=res[0], ti=res[1], SI=res[2], TI=res[3])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_siti_gather_equals_single_pass():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r = np.load(os.path.join(d, "res.npz"))
        si, ti = siti_ref.siti(_frames())
        np.testing.assert_array_equal(r["si"], si)
        np.testing.assert_array_equal(np.isnan(r["ti"]), np.isnan(ti))
        np.testing.assert_array_equal(r["ti"][1:], ti[1:])
        assert float(r["SI"]) == si.max() and float(r["TI"]) == np.nanmax(ti)


@pytest.mark.parametrize("n,world", [(10, 2), (11, 2), (1, 2), (600, 8), (7, 8)])
def test_frame_ranges_cover(n, world):
    rs = shard.frame_ranges(n, world)
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    sizes = [e - s for s, e in rs]
    assert max(sizes) - min(sizes) <= 1


def test_assign_pvs_balanced_and_complete():
    items = ["PVS%03d" % i for i in range(256)]
    parts = shard.assign_pvs(items, 8)
    assert sorted(sum(parts, [])) == items and all(len(p) == 32 for p in parts)
    cost = {it: (i % 5) + 1 for i, it in enumerate(items)}
    parts = shard.assign_pvs(items, 8, cost=cost.get)
    loads = [sum(cost[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= 5


# ---- the launcher bench.py uses (pixpath.batch), driven for real on CPU -----
def test_spawn_local_two_ranks_gather_equals_single_pass(tmp_path):
    """`bench.py --gpus 2` path: the parent spawns 2 ranks (RANK/LOCAL_RANK/
    WORLD_SIZE/MASTER_*), each takes its PVS share, SI/TI is gathered over gloo
    to rank 0 and equals the single-process result for every PVS."""
    import sys

    import gloo_selftest
    from pixpath import batch
    out = tmp_path / "res.npz"
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(sys.path))
    prog = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gloo_selftest.py")
    rc = batch.spawn_local(2, [sys.executable, prog, str(out), "6"], env=env)
    assert rc == 0
    r = np.load(out)
    assert int(r["world"]) == 2
    assert list(r["ids"]) == ["PVS%03d" % i for i in range(6)]
    assert sorted(set(r["ranks"].tolist())) == [0, 1]
    assert np.bincount(r["ranks"]).tolist() == [3, 3]
    for i in range(6):
        si, ti = siti_ref.siti(gloo_selftest.frames(i))
        np.testing.assert_array_equal(r["si"][i], si)
        np.testing.assert_array_equal(r["ti"][i][1:], ti[1:])
        assert r["SI"][i] == si.max() and r["TI"][i] == np.nanmax(ti)


def test_spawn_local_reports_failure(tmp_path):
    import sys
    from pixpath import batch
    rc = batch.spawn_local(2, [sys.executable, "-c", "import os,sys; sys.exit(3 if os.environ['RANK']=='1' else 0)"])
    assert rc == 3


def test_my_pvs_config5_split():
    from pixpath import batch
    ids = ["PVS%03d" % i for i in range(256)]
    parts = [batch.my_pvs(ids, r, 8) for r in range(8)]
    assert sorted(sum(parts, [])) == ids and {len(p) for p in parts} == {32}


def test_device_slots_spread_over_gpus(tmp_path):
    """pixpath.cli processes under a Pool(-p 4) on 2 GPUs: devices 0,1,0,1 (not pid % n)."""
    import subprocess
    import sys
    env = dict(os.environ, PIXPATH_SLOT_DIR=str(tmp_path), PYTHONPATH=os.pathsep.join(sys.path))
    procs = []
    for _ in range(4):
        procs.append(subprocess.Popen([sys.executable, "-m", "pixpath.devslot", "2", "3"], env=env,
                                      stdout=subprocess.PIPE, text=True))
        # wait until this process holds its slot before starting the next
        procs[-1].stdout_line = procs[-1].stdout.readline().strip()
    devs = sorted(int(p.stdout_line) for p in procs)
    for p in procs:
        p.wait()
    assert devs == [0, 0, 1, 1]
