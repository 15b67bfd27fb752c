"""BASELINE config 5 (256 synthetic PVS, per-GPU process, host gather of SI/TI)
through the HIP kernels, as bench.py runs it (tests/config5_worker.py): the
whole batch on one rank in this process, and split over 2 gloo ranks that
share the box's GPU.  Checked: every PVS id gathered exactly once, the rank
split, scaled frames of 4 sampled PVSes bit-exact vs the oracle, per-frame
SI/TI of 16 sampled PVSes within 1e-4 (SI) / 1e-12 (TI) of the numpy / C
oracle, TI_0 undefined, SI = max_n SI_n."""
import os
import sys

import numpy as np
import pytest

import config5_worker

pytestmark = pytest.mark.gpu
FRAMES = 8


def _check(r, world):
    ids = ["PVS%03d" % i for i in range(256)]
    assert list(r["ids"]) == ids and int(r["world"]) == world
    assert np.bincount(r["ranks"], minlength=world).tolist() == [256 // world] * world
    assert sorted(r["scale_ids"].tolist()) == sorted(config5_worker.SCALE_SAMPLE) and r["scale_ok"].all()
    assert sorted(r["siti_ids"].tolist()) == sorted(config5_worker.SITI_SAMPLE)
    assert (r["siti_err"][:, 0] <= 1e-4).all(), r["siti_err"]
    assert (r["siti_err"][:, 1] <= 1e-12).all(), r["siti_err"]
    assert r["siti_flags"].all()
    assert np.isfinite(r["SI"]).all() and np.isfinite(r["TI"]).all()


def test_config5_one_rank(gpu, tmp_path):
    out = str(tmp_path / "c5.npz")
    config5_worker.run(out, 256, FRAMES)
    _check(np.load(out), 1)


def test_config5_two_ranks_gloo_gather(gpu, tmp_path):
    from pixpath import batch
    out = str(tmp_path / "c5w2.npz")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(sys.path))
    rc = batch.spawn_local(2, [sys.executable, "-u", config5_worker.__file__, out, "256", str(FRAMES)], env=env)
    assert rc == 0
    _check(np.load(out), 2)
