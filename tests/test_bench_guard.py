"""bench.py refuses measurement overrides: a PIXPATH_*
tuning variable, or a library other than the in-tree libpixpath.so, voids a
bench line, so the bench exits non-zero before touching a GPU unless
--allow-tuning is given (then the overrides are recorded in the line).  The
product library itself reads no environment: its knob names are not even in
the binary."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "processing-chain_amd", "pixpath", "libpixpath.so")


def _bench(env_extra, *args):
    env = {k: v for k, v in os.environ.items() if not k.startswith("PIXPATH_")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), env=env,
                          capture_output=True, text=True, timeout=120)


def test_bench_refuses_tuning_overrides():
    for var, val in (("PIXPATH_SCALE_DEBUG", "1"), ("PIXPATH_STRIP_TW", "512"), ("PIXPATH_PITCH_PAD", "256"),
                     ("PIXPATH_LIB", "/tmp/other/libpixpath.so")):
        p = _bench({var: val})
        assert p.returncode == 2, (var, p.stdout, p.stderr)
        assert "refusing" in p.stderr and var in p.stderr


def test_product_settings_and_default_lib_are_allowed():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    old = dict(os.environ)
    try:
        for k in [k for k in os.environ if k.startswith("PIXPATH_")]:
            del os.environ[k]
        os.environ.update(PIXPATH_FFV1="gpu", PIXPATH_FFV1_SLICES="8x8", PIXPATH_DEVICE="0", PIXPATH_LIB=LIB)
        assert bench.tuning_overrides() == {}
        os.environ["PIXPATH_CHAIN_LUMA_CHO"] = "24"
        assert bench.tuning_overrides() == {"PIXPATH_CHAIN_LUMA_CHO": "24"}
    finally:
        os.environ.clear()
        os.environ.update(old)


def test_product_library_reads_no_knobs():
    data = open(LIB, "rb").read()
    for knob in (b"PIXPATH_SCALE_DEBUG", b"PIXPATH_FFV1_DEBUG", b"PIXPATH_STRIP_TW", b"PIXPATH_SCALE_LDS_KB",
                 b"PIXPATH_FFV1_LPW", b"PIXPATH_CHAIN_LUMA_CHO", b"PIXPATH_SCALE_KERNEL", b"getenv"):
        assert knob not in data, knob


def test_layout_padding_ignored_by_the_product_library():
    """The frame-layout padding knobs (tools/gpu_pad_sweep.sh) take effect only
    with the measurement build loaded; with the product library the layout is
    the unpadded one whatever the environment says."""
    code = ("import sys; sys.path.insert(0, %r); from pixpath import frames; "
            "print(frames._PITCH_PAD, frames._ROWS_PAD, frames._pitch(1920, 2))"
            % os.path.join(ROOT, "processing-chain_amd"))
    env = {k: v for k, v in os.environ.items() if not k.startswith("PIXPATH_")}
    env.update({"PIXPATH_PITCH_PAD": "256", "PIXPATH_ROWS_PAD": "3"})
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["0", "0", "1920"]
