"""pixpath.spinner.load_apng (the APNG compose/dispose logic feeding the stall
kernel) checked independently against PIL's APNG reader, on both spinner
assets the reference ships (util/spinner-128-white.png, the default of
lib/parse_args.py:99, and util/5.png): every composed RGBA frame and every
frame delay."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
PIL = pytest.importorskip("PIL.Image")


@pytest.mark.parametrize("name", ["spinner-128-white.png", "spinner-5.png"])
def test_apng_frames_and_delays_match_pil(name):
    from pixpath import spinner
    path = os.path.join(GOLDEN, name)
    anim, delays = spinner.load_apng(path)
    im = PIL.open(path)
    assert im.n_frames == anim.shape[0]
    for i in range(im.n_frames):
        im.seek(i)
        ref = np.array(im.convert("RGBA"))
        assert ref.shape == anim[i].shape
        np.testing.assert_array_equal(anim[i], ref, err_msg="frame %d" % i)
        assert abs(delays[i] * 1000.0 - im.info["duration"]) < 1e-6
