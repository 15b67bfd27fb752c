"""The documented reference-side binding (INTEGRATION.md sections 2 and 3)
routes every pixel-path command of p03 / p04 to the MI355X.

tests/golden/pipeline_fixtures.json holds what the reference's own p03 and
p04 (`--dry-run`, p03_generateAvPvs.py:62, p04_generateCpvs.py:31) returned
from each builder call on a synthetic short database (stall and freeze
PVSes) and a config-4-shaped long database (2-s segments, stalls [[2,1.5],
[4,1.0]]), once unchanged and once with the binding applied
(tests/golden/gen_pipeline_fixtures.py).  Here: the binding recorded there is
the one INTEGRATION.md documents today; with it, segment, concat, short
AVPVS, bufferer, CPVS and preview are all `pixpath.cli` commands under the
GPU-FFV1 default; what stays ffmpeg is the audio mux's stream copy; and
without it the reference's strings are untouched -- equal to what
pixpath.ffmpeg's ffmpeg backend reproduces."""
import json
import os
import shlex

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "pipeline_fixtures.json")))

PIXEL_BUILDERS = {"create_avpvs_short": "avpvs", "create_avpvs_segment": "avpvs", "create_avpvs_long_concat": "concat",
                  "bufferer_command": "stall", "create_cpvs": "cpvs", "create_preview": "preview"}


def _gen():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_pipeline_fixtures",
                                                  os.path.join(HERE, "golden", "gen_pipeline_fixtures.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_fixture_binding_is_the_documented_one():
    sec2, sec3 = _gen().integration_blocks()
    assert FIX["integration_section2"] == sec2
    assert FIX["integration_section3"] == sec3


@pytest.mark.parametrize("db", ["P2SXM00", "P2LXM00"])
def test_gpu_binding_routes_every_pixel_command(db):
    run = FIX["runs"][db + "/gpu"]
    seen = set()
    for script in ("p03", "p04"):
        for name, cmd in run[script]:
            assert cmd, (name, cmd)
            if name == "audio_mux":  # a stream copy: ffmpeg demuxes, never decodes the FFV1
                assert cmd.startswith("ffmpeg -nostdin") and "-c:v copy" in cmd
                continue
            a = shlex.split(cmd.split(" && ")[0])
            assert a[1:4] == ["python3", "-m", "pixpath.cli"] and a[4] == PIXEL_BUILDERS[name], cmd
            seen.add(name)
            if a[4] == "avpvs":  # AVPVS writers: GPU FFV1, codec and grid in the logged command
                assert a[-4:-1] == ["--gpu-ffv1", "--ffv1-slices", "8x8"], cmd
            elif a[4] in ("cpvs", "stall"):
                assert "--gpu-ffv1" in a
    if db == "P2LXM00":
        assert seen == set(PIXEL_BUILDERS) - {"create_avpvs_short"}
        # the bufferer step came through the section-3 change of p03
        sched = dict(run["p03_scheduled"])
        buf = [c for n, c in sched.items() if n.endswith("buffering")]
        assert len(buf) == 1 and " -m pixpath.cli stall " in buf[0]
    else:
        assert seen == {"create_avpvs_short", "create_cpvs", "create_preview"}
        stalls = [c for n, c in run["p03"] if "--stall-output" in c]
        assert len(stalls) == 2 and any("--skipping" in c for c in stalls)


@pytest.mark.parametrize("db", ["P2SXM00", "P2LXM00"])
def test_reference_unchanged_without_the_backend(db):
    """ffmpeg backend: the binding block is inert; every command is the
    reference's own ffmpeg / bufferer string."""
    run = FIX["runs"][db + "/ffmpeg"]
    for script in ("p03", "p04"):
        for name, cmd in run[script]:
            assert name != "bufferer_command"
            assert cmd.startswith("ffmpeg -nostdin"), cmd
    if db == "P2LXM00":
        buf = [c for n, c in run["p03_scheduled"] if n.endswith("buffering")]
        assert len(buf) == 1 and buf[0].startswith("bufferer -i ")


@pytest.mark.parametrize("db", ["P2SXM00", "P2LXM00"])
def test_same_builder_calls_in_both_backends(db):
    """The binding changes the commands, never which builders p03/p04 call
    (the bufferer aside: inline in the reference, a builder with the binding)."""
    for script in ("p03", "p04"):
        ref = [n for n, _ in FIX["runs"][db + "/ffmpeg"][script]]
        gpu = [n for n, _ in FIX["runs"][db + "/gpu"][script] if n != "bufferer_command"]
        assert ref == gpu
