"""libpixpath.so C ABI on the CPU (no kernels launched).

* the library loads and exports every function include/pixpath.h declares;
* without a GPU the product fails loudly (no CPU fallback);
* host-only scaler plans (ctx = NULL) build FFmpeg's exact filter tables --
  compared with the oracle's independent restatement over the reference's
  scale call sites and ragged sizes;
* pp_fps_map / pp_v210_linesize agree with the oracle and pixpath.chain."""
import ctypes
import os
import re

import numpy as np
import pytest

import pyoracle as po
from pixpath import _native, chain, ops

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "pixpath.h")


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    declared = set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(pp_\w+)\s*\(", open(HEADER).read(), re.M))
    assert declared == set(_native.EXPORTS)
    for name in declared:
        assert hasattr(L, name)
    assert L.pp_abi_version() == 7


def test_host_transfer_argument_checks():
    """The host-transfer entry points validate before touching HIP: bad sizes,
    kinds and pitches are PP_ERR_INVALID with a message (no GPU needed)."""
    L = _native.lib()
    buf = (ctypes.c_uint8 * 64)()
    assert L.pp_copy_async(buf, buf, -1, _native.PP_COPY_H2D, None) == -1
    assert L.pp_copy_async(buf, buf, 8, 7, None) == -1
    assert b"kind" in L.pp_last_error()
    assert L.pp_copy2d_async(buf, 4, buf, 8, 8, 2, _native.PP_COPY_D2D, None) == -1
    assert b"pitch" in L.pp_last_error()
    assert L.pp_copy_async(None, None, 0, _native.PP_COPY_D2H, None) == 0
    out = ctypes.c_void_p()
    assert L.pp_device_alloc(None, 16, ctypes.byref(out)) == -1
    assert L.pp_host_alloc(-5, ctypes.byref(out)) == -1
    assert L.pp_frames_copy_async(99, 8, 8, ctypes.byref(_native.pp_frames()), ctypes.byref(_native.pp_frames()),
                                  1, 1, None) == -1


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    rc = _native.lib().pp_ctx_create(0, ctypes.byref(h))
    assert rc < 0 and _native.lib().pp_last_error()
    with pytest.raises(Exception):
        ops.Scaler("yuv422p10le", 1280, 720, "yuv422p10le", 1920, 1080, flags="lanczos")


def test_errors_carry_messages():
    h = ctypes.c_void_p()
    rc = _native.lib().pp_scale_plan_create(None, 99, 10, 10, 0, 10, 10, 4, 123456.0, 123456.0, ctypes.byref(h))
    assert rc == -1 and b"format" in _native.lib().pp_last_error()
    with pytest.raises(_native.PixpathError):
        _native.check(rc)


CONFIGS = [
    # reference scale call sites: lib/ffmpeg.py:992 (short AVPVS), :1038 (segment), :1213 (mobile), :800 (p01)
    ("yuv420p", 1280, 720, "yuv420p", 1920, 1080, 4),
    ("yuv422p10le", 1280, 720, "yuv422p10le", 1920, 1080, 4),
    ("yuv422p10le", 1280, 720, "yuv422p10le", 1920, 1080, 0x200),
    ("yuv420p10le", 960, 540, "yuv420p", 1920, 1080, 4),
    ("yuv420p", 1920, 1080, "yuv422p10le", 1920, 1080, 4),
    ("yuv420p", 1920, 1080, "yuv420p", 1280, 720, 4),
    ("yuv422p10le", 3840, 2160, "yuv422p10le", 1920, 1080, 4),
    ("yuv420p", 3840, 2160, "yuv420p", 640, 360, 4),
    ("yuv420p", 3840, 1600, "yuv420p", 1920, 800, 4),
    ("yuv420p", 4096, 2160, "yuv420p", 1920, 1012, 0x200),
    ("yuv420p", 640, 360, "yuv420p", 3840, 2160, 4),
    ("yuv422p", 250, 99, "yuv420p10le", 77, 61, 0x200),
    ("yuv444p10le", 64, 48, "yuv422p", 130, 90, 4),
    ("yuv420p", 333, 197, "yuv420p", 500, 301, 2),
    ("yuv420p", 1920, 1080, "uyvy422", 1920, 1080, 4),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "%s%dx%d-%s%dx%d-%x" % c)
def test_host_plan_filters_equal_oracle(cfg):
    sf, sw, sh, df, dw, dh, fl = cfg
    h = ctypes.c_void_p()
    L = _native.lib()
    _native.check(L.pp_scale_plan_create(None, po.FMT_BY_NAME[sf], sw, sh, po.FMT_BY_NAME[df], dw, dh, fl,
                                         123456.0, 123456.0, ctypes.byref(h)))
    try:
        s = po.Sws(po.FMT_BY_NAME[sf], sw, sh, po.FMT_BY_NAME[df], dw, dh, fl)
        for which in range(4):
            ref = s.filter(which)
            n = len(ref[1])
            coef = np.zeros(n * 64, np.int16)
            pos = np.zeros(n, np.int32)
            size = _native.check(L.pp_scale_plan_filter(h, which, coef.ctypes.data, pos.ctypes.data, n * 64))
            assert size == ref[0].shape[1]
            assert np.array_equal(coef[:n * size].reshape(n, size), ref[0])
            assert np.array_equal(pos, ref[1])
    finally:
        L.pp_scale_plan_destroy(h)


@pytest.mark.parametrize("n,a,b", [(600, 60, 60), (10, 24, 60), (301, 30, 60), (250, 25, 60), (123, 60, 30),
                                   (77, "30000/1001", 60), (600, 60, 24), (5, 50, 60), (1, 60, 60), (0, 30, 60)])
def test_fps_map_three_way(n, a, b):
    m = ops.fps_map(n, a, b)
    assert m.tolist() == po.fps_map(n, a, b).tolist() == chain.fps_index_map(n, a, b)


@pytest.mark.parametrize("w", [1, 6, 47, 48, 49, 1280, 1920, 3840, 4096])
def test_v210_linesize(w):
    assert _native.lib().pp_v210_linesize(w) == po.v210_linesize(w)


@pytest.mark.parametrize("sf,sw,sh,df,dw,dh,fused", [
    ("yuv420p10le", 1280, 720, "yuv422p10le", 1920, 1080, True),   # config 4 canvas: one launch
    ("yuv422p10le", 1280, 720, "yuv422p10le", 1920, 1080, True),
    ("yuv420p", 1280, 720, "yuv422p", 1920, 1080, True),
    ("yuv420p", 1280, 720, "yuv420p10le", 1920, 1080, True),
    ("yuv420p", 1920, 1080, "yuv422p10le", 1920, 1080, False),     # unscaled first stage: two launches
])
def test_chain_plan_host_only(sf, sw, sh, df, dw, dh, fused):
    """pp_scale_chain_plan_create (create_avpvs_segment's two stages) decides
    its launch shape on the host: fused into one strip_kernel launch or two."""
    L = _native.lib()
    h = ctypes.c_void_p()
    _native.check(L.pp_scale_chain_plan_create(None, po.FMT_BY_NAME[sf], sw, sh, po.FMT_BY_NAME[df], dw, dh,
                                               ops.FLAGS["bicubic"], ops.PARAM_DEFAULT, ops.PARAM_DEFAULT,
                                               ctypes.byref(h)))
    try:
        assert (L.pp_scale_plan_path(h) > 0) == fused
    finally:
        L.pp_scale_plan_destroy(h)
    assert L.pp_scale_chain_plan_create(None, 0, 64, 64, po.FMT_BY_NAME["uyvy422"], 64, 64, 4, 1.0, 1.0,
                                        ctypes.byref(h)) == -1
