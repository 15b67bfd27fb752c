"""BASELINE config 5 on the GPU (test code, not product): a batch of PVS
sharded over ranks exactly as bench.py runs it -- pixpath.batch.my_pvs for the
rank's share, the HIP scaler (720p -> 1080p yuv422p10le lanczos) and pp_siti
per PVS, pixpath.batch.gather_results to rank 0 over gloo -- at a reduced
number of frames per PVS.  Each rank checks the scaled frames of the sampled
PVSes it owns against the oracle; rank 0 checks the gathered SI/TI of
sampled PVSes (regenerated from their seeds) against the numpy / C oracle.

Run in-process (run(...)) or as N ranks: python tests/config5_worker.py OUT.npz
N_PVS FRAMES (under pixpath.batch.spawn_local; every rank uses GPU
LOCAL_RANK % device_count, so 2 ranks share a 1-GPU box).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "processing-chain_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

SCALE_SAMPLE = ("PVS000", "PVS085", "PVS170", "PVS255")
SITI_SAMPLE = tuple("PVS%03d" % i for i in range(0, 256, 16))  # 16 PVSes, both halves of the split


def pvs_inputs(index, frames, dev):
    """Seeded legal-range inputs of one PVS, generated on the device (same
    generator as bench.make_inputs): 1280x720 yuv422p10le frames + 1080p luma."""
    import torch
    from pixpath.frames import FrameBatch
    g = torch.Generator(device=dev)
    g.manual_seed(910 + index)
    src = FrameBatch("yuv422p10le", 1280, 720, frames, device=dev)
    for p, (lo, hi) in enumerate([(64, 941), (64, 961), (64, 961)]):
        v = src.view(p)
        v.copy_(torch.randint(lo, hi, v.shape, generator=g, device=dev, dtype=torch.int32).to(v.dtype))
    luma = torch.randint(64, 941, (frames, 1080, 1920), generator=g, device=dev, dtype=torch.int32).to(torch.uint16)
    return src, luma


def run(out_path, n_pvs=256, frames=8):
    import torch
    import pyoracle as po
    from pixpath import batch, ops
    rank, world, local = batch.rank_env()
    batch.init_group(world)
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    ids = ["PVS%03d" % i for i in range(n_pvs)]
    mine = batch.my_pvs(ids, rank, world)
    scaler = ops.Scaler("yuv422p10le", 1280, 720, "yuv422p10le", 1920, 1080, flags="lanczos")
    res, scale_ok = {}, {}
    for pid in mine:
        src, luma = pvs_inputs(int(pid[3:]), frames, dev)
        out = scaler(src)
        si, ti = ops.siti(luma, 10)
        res[pid] = (si.cpu().numpy(), ti.cpu().numpy())
        if pid in SCALE_SAMPLE:
            got = out.to_numpy()
            sp = src.to_numpy()
            ok = True
            for f in range(frames):
                ref = po.scale(po.YUV422P10LE, [p[f] for p in sp], po.YUV422P10LE, 1920, 1080, po.SWS_LANCZOS)
                ok = ok and all(np.array_equal(got[p][f], ref[p]) for p in range(3))
            scale_ok[pid] = ok
    gathered = batch.gather_results(res, rank, world)
    checks = batch.gather_values(scale_ok, rank, world)
    if rank == 0:
        import siti_ref
        siti_err = {}
        for k, pid in enumerate(SITI_SAMPLE):
            if pid not in gathered:
                continue
            _, luma = pvs_inputs(int(pid[3:]), frames, dev)
            host = luma.cpu().numpy()
            rsi, rti = siti_ref.siti(host) if k < 2 else po.siti_c(host, 10)
            g = gathered[pid]
            e_si = float(np.max(np.abs(g["si"] - rsi) / np.abs(rsi)))
            e_ti = float(np.max(np.abs(g["ti"][1:] - rti[1:]) / np.abs(rti[1:])))
            siti_err[pid] = (e_si, e_ti, bool(np.isnan(g["ti"][0])), g["SI"] == float(np.max(rsi)) or
                             abs(g["SI"] - float(np.max(rsi))) <= 1e-4 * abs(float(np.max(rsi))))
        keys = sorted(gathered)
        merged = {}
        for part in checks:
            merged.update(part)
        np.savez(out_path, ids=np.array(keys), world=world, ranks=np.array([gathered[k]["rank"] for k in keys]),
                 SI=np.array([gathered[k]["SI"] for k in keys]), TI=np.array([gathered[k]["TI"] for k in keys]),
                 scale_ids=np.array(sorted(merged)), scale_ok=np.array([merged[k] for k in sorted(merged)]),
                 siti_ids=np.array(sorted(siti_err)),
                 siti_err=np.array([siti_err[k][:2] for k in sorted(siti_err)]),
                 siti_flags=np.array([siti_err[k][2:] for k in sorted(siti_err)]))
    batch.barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 256, int(sys.argv[3]) if len(sys.argv) > 3 else 8)
