"""PP-STALL-1 streaming (pixpath.stall.StallStream, what `pixpath.cli stall`
runs) == the whole-sequence definition (stall_schedule) on many event lists,
including stalls at t=0, at/after the end, back-to-back and overlapping
freezes; and the audio graph that inserts the stalls' silence."""
import itertools

import numpy as np
import pytest

from pixpath.stall import StallStream, stall_audio_graph, stall_schedule, stall_times

DELAYS = [0.0898876404494382] * 8  # spinner-128-white.png


def _stream(events, rate, n_in, skipping, black):
    out = []
    st = StallStream(events, rate, skipping, DELAYS, black_frame=black)
    st.run(iter(range(n_in)), lambda f: out.append((f, -1)),
           lambda f, spin: out.extend(((-1 if f is None else f), s) for s in spin))
    return out


CASES = [
    [[2, 1.5], [4, 1.0]],            # config 4's events
    [[0, 0.5]], [[0, 0.5], [1, 0.2]], [[8, 1.0]], [[10, 1.0]], [[12, 2.0]],
    [[1, 0.0]], [[0.05, 0.3], [0.05, 0.3]], [[3.3333, 0.7], [1.1, 0.25]], [],
]


@pytest.mark.parametrize("black", [True, False])
@pytest.mark.parametrize("events", CASES, ids=lambda e: str(e).replace(" ", ""))
def test_stream_equals_schedule_stalls(events, black):
    for rate, n_in in ((60, 600), (24, 241), (30, 1)):
        assert _stream(events, rate, n_in, False, black) == stall_schedule(events, rate, n_in, False, DELAYS, black)


@pytest.mark.parametrize("events", CASES + [[[1, 2], [2, 0.5]], [[0, 1], [0.5, 1]], [[3, 5]]],
                         ids=lambda e: str(e).replace(" ", ""))
def test_stream_equals_schedule_freezes(events):
    for rate, n_in in ((60, 600), (25, 101)):
        assert _stream(events, rate, n_in, True, True) == stall_schedule(events, rate, n_in, True, DELAYS, True)


def test_stream_random_events():
    rng = np.random.default_rng(5)
    for _ in range(200):
        ev = [[round(float(rng.uniform(0, 12)), 3), round(float(rng.uniform(0, 2)), 3)] for _ in range(rng.integers(0, 4))]
        for skipping, black in itertools.product((False, True), (False, True)):
            n_in = int(rng.integers(0, 700))
            assert _stream(ev, 60, n_in, skipping, black) == stall_schedule(ev, 60, n_in, skipping, DELAYS, black)


def test_audio_graph_inserts_silence_on_the_video_grid():
    g = stall_audio_graph(stall_times([[4, 1.0], [2, 1.5]], 60), 48000, "stereo")
    assert g == ("[1:a]asplit=3[s0][s1][s2];"
                 "[s0]atrim=start=0:end=2,asetpts=PTS-STARTPTS[p0];anullsrc=r=48000:cl=stereo,atrim=end=1.5[z0];"
                 "[s1]atrim=start=2:end=4,asetpts=PTS-STARTPTS[p1];anullsrc=r=48000:cl=stereo,atrim=end=1[z1];"
                 "[s2]atrim=start=4,asetpts=PTS-STARTPTS[p2];[p0][z0][p1][z1][p2]concat=n=5:v=0:a=1[aout]")
    # stall times snap to the frame grid the video uses
    from fractions import Fraction
    assert stall_times([[1.01, 0.5]], 60) == [(Fraction(61, 60), Fraction(1, 2))]
    assert stall_audio_graph([], 48000, "stereo") is None
    assert stall_audio_graph(stall_times([[1, 0.0]], 60), 48000, "stereo") is None
