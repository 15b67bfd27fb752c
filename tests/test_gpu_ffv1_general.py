"""The GPU decoder on general FFV1 version 3 streams -- the reference's own
AVPVS codec settings `-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1
-slicecrc 1` (/root/reference/lib/ffmpeg.py:993, :1047): a transmitted state
table, -context 1's 5-input set (two sets in the record), 2x2 slices, GOPs of
12 with the context states carried from frame to frame; plus initial context
states and per-plane table sets.  Streams come from the oracle's general
restatement (oracle/ffv1_oracle.c); every decoded frame must equal the input
exactly (FFV1 is lossless).  FFmpeg's own files stay parity unpinned."""
import numpy as np
import pytest

import ffv1_ref as ref
import pyoracle as po
import synth
from test_ffv1_general import FMTS, ffmpeg_like

pytestmark = pytest.mark.gpu


def _sequence(pf, fid, w, h, n, seed):
    rng = np.random.default_rng(seed)
    frames = [synth.noise_frame(rng, fid, w, h) if i % 5 == 2 else synth.smooth_frame(i, fid, w, h) for i in range(n)]
    enc = ref.GenEncoder(pf, w, h)
    return frames, [enc.encode(f) for f in frames]


def _check(out, frames, first=0):
    for i, f in enumerate(frames):
        for p in range(3):
            np.testing.assert_array_equal(out[p][first + i], f[p], err_msg="frame %d plane %d" % (i, p))


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
def test_ffmpeg_like_gops_in_one_decode(gpu, name, fid, bits, hs, vs):
    """26 frames = two GOPs of 12 and two frames of a third, one decode call:
    per slice, one lane walks each GOP with its states carried."""
    from pixpath import ffv1
    w, h = 640, 360
    pf = ffmpeg_like(bits, hs, vs)
    frames, pkts = _sequence(pf, fid, w, h, 26, bits + hs + vs)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=26, device=gpu)
    assert dec.info["pixpath_tables"] == 0 and dec.info["coder_type"] == 2
    _check(dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy(), frames)


@pytest.mark.parametrize("split", [1, 7, 12, 17])
def test_gop_continues_across_decode_calls(gpu, split):
    """A batch that starts inside a GOP continues the states the previous
    call left (a 600-frame reader batch need not align with the GOPs); after
    reset() such a batch is refused instead of decoded from wrong states."""
    from pixpath import ffv1
    w, h, fid = 320, 180, po.YUV422P10LE
    pf = ffmpeg_like(10, 1, 0, gop=12)
    frames, pkts = _sequence(pf, fid, w, h, 30, split)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=30, device=gpu)
    a = dec.decode(b"".join(pkts[:split]), [len(p) for p in pkts[:split]]).to_numpy()
    b = dec.decode(b"".join(pkts[split:]), [len(p) for p in pkts[split:]]).to_numpy()
    _check(a, frames[:split])
    _check(b, frames[split:])
    if split % 12:
        dec.reset()
        with pytest.raises(Exception, match="keyframe"):
            dec.decode(b"".join(pkts[split:]), [len(p) for p in pkts[split:]])


def test_initial_states_and_table_sets_per_plane(gpu):
    """Three table sets, luma on a 5-input set and chroma on a 3-input one,
    both with transmitted initial states (a 2-pass encode's record), GOP 4."""
    from pixpath import ffv1
    w, h, bits = 480, 270, 10
    a, b = ref.QUANT9_10, ref.QUANT5_10
    sets = [[a, a, a, ref.ZERO, ref.ZERO], [a, a, b, b, b], [b, a, b, ref.QUANT5, b]]
    pf = ffmpeg_like(bits, 1, 0, 3, 2, gop=4, init=True, tidx=(2, 0), sets=sets)
    frames, pkts = _sequence(pf, po.YUV422P10LE, w, h, 9, 44)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=9, device=gpu)
    assert dec.info["initial_states_mask"] == 0b101
    _check(dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy(), frames)


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS[:2], ids=[f[0] for f in FMTS[:2]])
def test_1080p_reference_avpvs_shape(gpu, name, fid, bits, hs, vs):
    """The reference's AVPVS shape: 1920x1080, 2x2 slices (FFmpeg's choice
    for -threads 4), GOP 12: a GOP and one more keyframe."""
    from pixpath import ffv1
    w, h = 1920, 1080
    pf = ffmpeg_like(bits, hs, vs)
    frames, pkts = _sequence(pf, fid, w, h, 13, 1080 + bits)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=13, device=gpu)
    _check(dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy(), frames)


def test_inter_frame_corruption_is_reported(gpu):
    from pixpath import ffv1
    w, h = 320, 180
    pf = ffmpeg_like(8, 1, 1, gop=6)
    frames, pkts = _sequence(pf, po.YUV420P, w, h, 6, 9)
    bad = bytearray(pkts[3])
    bad[len(bad) // 3] ^= 0x08
    pkts[3] = bytes(bad)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=6, device=gpu)
    with pytest.raises(Exception, match="frame 3 .*CRC"):
        dec.decode(b"".join(pkts), [len(p) for p in pkts])


def test_reference_made_avpvs_routes_to_the_gpu_decoder(gpu, tmp_path):
    """An AVI holding an FFmpeg-like FFV1 stream (what the reference's p03
    writes) opens with the GPU decoder (open_avpvs_reader -> Ffv1AviReader,
    no ffmpeg), reads back every frame across reader batches that cut its
    GOPs, and `cli cpvs` turns it into the oracle's v210 frames."""
    from pixpath import avi, cli, ffv1
    w, h, n = 640, 360, 30
    pf = ffmpeg_like(10, 1, 0, gop=12)
    frames, pkts = _sequence(pf, po.YUV422P10LE, w, h, n, 77)
    path = str(tmp_path / "P2SXM00_SRC000_HRC000.avi")
    wr = avi.AviWriter(path, w, h, 60, extradata=ref.gen_extradata(pf))
    for i, p in enumerate(pkts):
        wr.write_packet(p, key=i % 12 == 0)
    wr.close()
    rd = ffv1.open_avpvs_reader(path, device=gpu.index, batch=8)
    assert isinstance(rd, ffv1.Ffv1AviReader)
    got = []
    while True:
        b = rd.read_device(5)
        if b is None:
            break
        planes = b.to_numpy()
        got.extend([[planes[p][i] for p in range(3)] for i in range(b.n)])
    rd.close()
    assert len(got) == n
    for i in range(n):
        for p in range(3):
            np.testing.assert_array_equal(got[i][p], frames[i][p], err_msg="frame %d plane %d" % (i, p))
    out = str(tmp_path / "cpvs.raw")
    assert cli.main(["cpvs", "-y", "--input", path, "--fps", "60", "--vcodec", "v210", "--pix-fmt", "yuv422p10le",
                     "--pad", "640x400", "--gpu-ffv1", out]) == 0
    raw = np.fromfile(out, np.uint8)
    fb = po.v210_linesize(640) * 400
    assert raw.size == n * fb
    for j in (0, 13, n - 1):
        want = po.v210_pack(po.pad(po.YUV422P10LE, frames[j], 640, 400, 0, 20))
        np.testing.assert_array_equal(raw[j * fb:(j + 1) * fb], want.reshape(-1))


@pytest.mark.parametrize("fmt,fid,bits,hs,vs,w,h,grid", [
    ("yuv420p", po.YUV420P, 8, 1, 1, 333, 190, (3, 2)),        # ragged: odd width, unequal slices
    ("yuv422p10le", po.YUV422P10LE, 10, 1, 0, 250, 66, (4, 1)),
    ("yuv444p10le", po.YUV444P10LE, 10, 0, 0, 320, 176, (2, 2)),  # 4:4:4 (FFmpeg's ffv1 writes it too)
    ("yuv444p", po.YUV444P, 8, 0, 0, 96, 40, (1, 1))])
def test_ragged_and_444_streams(gpu, fmt, fid, bits, hs, vs, w, h, grid):
    """Odd frame sizes (chroma planes rounded up, slices of unequal width, a
    chroma column two slices share) and 4:4:4 chroma, GOP 5 with states
    carried: every frame exact."""
    from pixpath import ffv1
    pf = ffmpeg_like(bits, hs, vs, *grid, gop=5)
    frames, pkts = _sequence(pf, fid, w, h, 11, w + h)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=11, device=gpu)
    assert dec.fmt.name == fmt
    _check(dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy(), frames)


@pytest.mark.parametrize("bounds", [[1, 2, 4, 8, 16], [3, 8, 32], [2, 6, 16, 48], [1], [1, 3, 8, 24, 64]],
                         ids=["round4_666", "t3_8_32", "t2_6_16_48", "t1", "t1_3_8_24_64"])
@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS[:2], ids=[f[0] for f in FMTS[:2]])
def test_threshold_quantiser_streams_take_the_pixpath_path(gpu, bounds, name, fid, bits, hs, vs):
    """pixpath-form records with any threshold quantiser -- round 4's files
    (min(5, bit length), 666 contexts) and other sets -- decode through the
    one-line-row path with the thresholds read back from the record (the
    first quantiser as ALU compares): every frame exact."""
    from pixpath import ffv1
    w, h = 480, 270
    t = ref._runs(bounds)
    pf = ref.make_prof(bits, hs, vs, 8, 4, [[t, t, t, ref.ZERO, ref.ZERO]], tidx=(0, 0), coder=1, gop=1)
    frames, pkts = _sequence(pf, fid, w, h, 6, len(bounds) + bits)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), w, h, max_frames=6, device=gpu)
    assert dec.info["pixpath_tables"] == 1
    _check(dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy(), frames)


def test_group_decode_of_several_streams(gpu):
    """pp_ffv1_decode_group: four streams of one record (FFmpeg's GOP shape,
    each its own content and GOP phase) decoded in ONE launch, then each
    continued by a second group call that starts inside a GOP (every stream
    carries its own states); every frame equals the one-stream decode's
    input.  A stream whose frame 0 is not a keyframe after reset() fails the
    group with a message naming it; a record mismatch is refused."""
    from pixpath import ffv1
    w, h, fid = 320, 180, po.YUV422P10LE
    pf = ffmpeg_like(10, 1, 0, gop=12)
    extra = ref.gen_extradata(pf)
    seqs = [_sequence(pf, fid, w, h, n, 500 + k) for k, n in enumerate((30, 17, 24, 5))]
    decs = [ffv1.Ffv1Decoder(extra, w, h, max_frames=30, device=gpu) for _ in seqs]
    cut = (7, 12, 13, 5)  # first call: frames [0, cut), second: the rest
    first = ffv1.decode_group(decs, [b"".join(p[:c]) for (_, p), c in zip(seqs, cut)],
                              [[len(x) for x in p[:c]] for (_, p), c in zip(seqs, cut)]).to_numpy()
    o = 0
    for (frames, _), c in zip(seqs, cut):
        _check(first, frames[:c], first=o)
        o += c
    rest = [(f[c:], p[c:]) for (f, p), c in zip(seqs, cut)]
    second = ffv1.decode_group(decs, [b"".join(p) for _, p in rest], [[len(x) for x in p] for _, p in rest]).to_numpy()
    o = 0
    for frames, _ in rest:
        _check(second, frames, first=o)
        o += len(frames)
    decs[2].reset()
    with pytest.raises(Exception, match="stream 2.*keyframe"):
        ffv1.decode_group(decs[:3], [b"".join(p[c:]) for (_, p), c in zip(seqs[:3], cut)],
                          [[len(x) for x in p[c:]] for (_, p), c in zip(seqs[:3], cut)])
    other = ffv1.Ffv1Decoder(ref.gen_extradata(ffmpeg_like(10, 1, 0, nh=1, nv=1)), w, h, max_frames=30, device=gpu)
    with pytest.raises(Exception, match="one configuration record"):
        ffv1.decode_group([decs[0], other], [b"".join(seqs[0][1][:12])] * 2, [[len(x) for x in seqs[0][1][:12]]] * 2)
