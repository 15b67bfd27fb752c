"""General FFV1 version 3 streams -- what the reference's AVPVS encode
`ffmpeg -c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1`
(/root/reference/lib/ffmpeg.py:993, :1047) writes and pixpath's own encoder
does not: a transmitted state table, 5-input context sets (several of them,
chosen per slice), initial context states, and GOPs whose context states carry
from frame to frame.

CPU side (this file): the oracle's general restatement (oracle/ffv1_oracle.c,
"General FFV1 version 3") round-trips every feature, reproduces pixpath's
intra packets byte for byte when given pixpath's profile, and the product's
record parser (pp_ffv1_decoder_create, host only) reads what it writes.  The
GPU decode of these streams is tests/test_gpu_ffv1_general.py.  FFmpeg itself
is absent, so parity against FFmpeg's own files stays unpinned."""
import numpy as np
import pytest

import ffv1_ref as ref
import pyoracle as po
import synth

FMTS = [("yuv422p10le", po.YUV422P10LE, 10, 1, 0), ("yuv420p", po.YUV420P, 8, 1, 1),
        ("yuv420p10le", po.YUV420P10LE, 10, 1, 1), ("yuv422p", po.YUV422P, 8, 1, 0)]


def _frames(rng, fid, w, h, n):
    return [synth.noise_frame(rng, fid, w, h) if i % 3 == 1 else synth.smooth_frame(i, fid, w, h) for i in range(n)]


def _init_states(sets, k, seed):
    """Transmitted initial states for set k: what a 2-pass FFmpeg encode
    stores (trained probabilities), here seeded values in 1..255."""
    rng = np.random.default_rng(seed)
    return rng.integers(1, 256, (ref.context_count(sets[k]), 32), dtype=np.uint8)


def ffmpeg_like(bits, hs, vs, nh=2, nv=2, gop=12, init=False, tidx=(1, 1), sets=None):
    sets = sets or ref.ffmpeg_context1_sets(bits)
    ini = {i: _init_states(sets, i, 7 + i) for i in set(tidx)} if init else None
    return ref.make_prof(bits, hs, vs, nh, nv, sets, tidx=tidx, coder=2, init=ini, gop=gop)


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
@pytest.mark.parametrize("grid", [(3, 2), (1, 1), (4, 4)])
def test_pixpath_profile_equals_the_intra_restatement(name, fid, bits, hs, vs, grid):
    """The general encoder given pixpath's profile (default table, one 3-input
    set, intra) writes the packets of the intra restatement the GPU encoder is
    tested against: the sample-buffer border rules of the general path agree
    with the intra path's neighbour rules."""
    rng = np.random.default_rng(bits * 7 + grid[0])
    w, h = 330, 190
    q = ref.pixpath_quant(bits)
    pf = ref.make_prof(bits, hs, vs, *grid, [[q] * 3 + [ref.ZERO] * 2], tidx=(0, 0), coder=1, gop=1)
    enc = ref.GenEncoder(pf, w, h)
    for f in (synth.noise_frame(rng, fid, w, h), synth.smooth_frame(2, fid, w, h)):
        assert enc.encode(f) == ref.encode_frame(f, bits, hs, vs, *grid)


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
@pytest.mark.parametrize("init", [False, True], ids=["states128", "initial_states"])
def test_ffmpeg_like_sequence_round_trips(name, fid, bits, hs, vs, init):
    """Custom state table, -context 1's two sets (5-input slices), GOP 3 with
    states carried: every frame decodes back; keyframes where the GOP says."""
    rng = np.random.default_rng(bits + 3 * hs + vs + init)
    w, h = 200, 120
    pf = ffmpeg_like(bits, hs, vs, gop=3, init=init)
    x = ref.gen_extradata(pf)
    dec = ref.GenDecoder(x, w, h)
    assert dec.info["coder_type"] == 2 and dec.info["quant_table_sets"] == 2 and dec.info["intra"] == 0
    assert dec.info["context_count1"] == (7563 if bits == 8 else 5063)
    assert dec.info["initial_states1"] == int(init)
    enc = ref.GenEncoder(pf, w, h)
    for i, f in enumerate(_frames(rng, fid, w, h, 7)):
        rc, out, key = dec.decode(enc.encode(f))
        assert rc == 0 and key == (i % 3 == 0)
        for p in range(3):
            np.testing.assert_array_equal(out[p], f[p], err_msg="frame %d plane %d" % (i, p))


def test_table_sets_per_plane_and_three_sets():
    """Three sets, luma on set 2 (5-input), chroma on set 0 (3-input), with
    initial states on both: the slice header's per-plane set index."""
    rng = np.random.default_rng(5)
    w, h, bits = 160, 96, 10
    a, b = ref.QUANT9_10, ref.QUANT5_10
    sets = [[a, a, a, ref.ZERO, ref.ZERO], [a, a, b, b, b], [b, a, b, ref.QUANT5, b]]
    pf = ffmpeg_like(bits, 1, 0, 3, 1, gop=4, init=True, tidx=(2, 0), sets=sets)
    x = ref.gen_extradata(pf)
    dec = ref.GenDecoder(x, w, h)
    enc = ref.GenEncoder(pf, w, h)
    for i, f in enumerate(_frames(rng, po.YUV422P10LE, w, h, 6)):
        rc, out, key = dec.decode(enc.encode(f))
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(out[p], f[p])


def test_states_carry_across_frames():
    """An inter frame's packet depends on the frames before it in its GOP:
    the same picture coded as the second frame of a GOP differs from its
    keyframe coding, and decoding it without its GOP's first frame fails."""
    rng = np.random.default_rng(8)
    w, h = 128, 64
    f0, f1 = synth.noise_frame(rng, po.YUV420P, w, h), synth.noise_frame(rng, po.YUV420P, w, h)
    pf = ffmpeg_like(8, 1, 1, gop=2)
    enc = ref.GenEncoder(pf, w, h)
    p0, p1 = enc.encode(f0), enc.encode(f1)
    assert p1 != ref.GenEncoder(pf, w, h).encode(f1)
    dec = ref.GenDecoder(ref.gen_extradata(pf), w, h)
    assert dec.decode(p1)[0] == -6  # non-keyframe first
    assert dec.decode(p0)[0] == 0
    rc, out, key = dec.decode(p1)
    assert rc == 0 and key == 0 and all(np.array_equal(out[p], f1[p]) for p in range(3))


def test_record_crc_and_state_table_checks():
    pf = ffmpeg_like(10, 1, 0)
    x = bytearray(ref.gen_extradata(pf))
    x[5] ^= 1
    with pytest.raises(ValueError):
        ref.GenDecoder(bytes(x), 64, 64)


# ---- the product's record parser (host only) ---------------------------------

def _native_info(dec):
    import ctypes
    from pixpath._native import check, lib
    info = (ctypes.c_int * 8)()
    n = check(lib().pp_ffv1_decoder_info(dec.handle, info, 8))
    return dict(zip(("micro", "coder", "tables", "max_ctx", "intra", "ec", "init_mask", "pix"), list(info)[:n]))


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
@pytest.mark.parametrize("init", [False, True], ids=["states128", "initial_states"])
def test_product_parser_reads_ffmpeg_like_records(name, fid, bits, hs, vs, init):
    """pp_ffv1_decoder_create accepts the general records (the round-4
    parser refused coder 2, two sets, 5-input tables and inter frames) and
    reads the same fields the restatement's decoder reads."""
    from pixpath import ffv1
    pf = ffmpeg_like(bits, hs, vs, init=init)
    x = ref.gen_extradata(pf)
    dec = ffv1.Ffv1Decoder(x, 1920, 1080, host_only=True)
    assert dec.fmt.name == name and dec.slices == (2, 2)
    info = _native_info(dec)
    assert info == {"micro": 4, "coder": 2, "tables": 2, "max_ctx": 7563 if bits == 8 else 5063, "intra": 0,
                    "ec": 1, "init_mask": 2 if init else 0, "pix": 0}
    # 2 line rows per slice for the 5-input context: 960-sample rows, 16 per workgroup
    assert (dec.slices_per_workgroup, dec.row_cap) == (16, 960)


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
def test_product_parser_marks_pixpath_records(name, fid, bits, hs, vs):
    from pixpath import ffv1
    dec = ffv1.Ffv1Decoder(ref.extradata(bits, hs, vs, 8, 8), 1920, 1080, host_only=True)
    assert _native_info(dec) == {"micro": 4, "coder": 1, "tables": 1, "max_ctx": ref.pixpath_contexts(bits),
                                 "intra": 1, "ec": 1,
                                 "init_mask": 0, "pix": 1}


@pytest.mark.parametrize("bounds", [[1, 2, 4, 8, 16], [3, 8, 32], [2, 6, 16, 48], [4, 32], [1, 3, 8]])
def test_product_parser_marks_threshold_quantisers(bounds):
    """Any one-set, 3-input record whose quantisers are one threshold
    quantiser at scales 1, L, L^2 takes the decoder's pixpath path (ALU first
    quantiser, one line row): the thresholds are read back from the record."""
    from pixpath import ffv1
    t = ref._runs(bounds)
    pf = ref.make_prof(10, 1, 0, 8, 8, [[t, t, t, ref.ZERO, ref.ZERO]], tidx=(0, 0), coder=1, gop=1)
    dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), 1920, 1080, host_only=True)
    L = 2 * len(bounds) + 1
    info = _native_info(dec)
    assert info["pix"] == 1 and info["max_ctx"] == (L ** 3 + 1) // 2 and info["tables"] == 1


def test_product_parser_leaves_other_quantisers_general():
    """A set whose three inputs use different quantisers (every FFV1 input
    quantiser is threshold-shaped: read_quant_table's runs step by one), or
    whose inputs 4 and 5 are used, decodes through the general path."""
    from pixpath import ffv1
    for sets in ([[ref.QUANT11, ref.PIXPATH3, ref.PIXPATH3, ref.ZERO, ref.ZERO]],
                 [[ref.PIXPATH3, ref.PIXPATH3, ref.QUANT5, ref.ZERO, ref.ZERO]],
                 [[ref.PIXPATH3, ref.PIXPATH3, ref.PIXPATH3, ref.QUANT5, ref.ZERO]]):
        pf = ref.make_prof(10, 1, 0, 8, 8, sets, tidx=(0, 0), coder=1, gop=1)
        dec = ffv1.Ffv1Decoder(ref.gen_extradata(pf), 1920, 1080, host_only=True)
        assert _native_info(dec)["pix"] == 0


def test_product_parser_refuses_corrupt_records():
    from pixpath import ffv1
    x = ref.gen_extradata(ffmpeg_like(8, 1, 1, init=True))
    for k in (3, len(x) // 2, len(x) - 6):
        bad = bytearray(x)
        bad[k] ^= 0x10
        with pytest.raises(Exception, match="CRC"):
            ffv1.Ffv1Decoder(bytes(bad), 640, 360, host_only=True)
    with pytest.raises(Exception):
        ffv1.Ffv1Decoder(x[:12], 640, 360, host_only=True)


def test_keyframe_flag_from_the_packet():
    """packet_is_keyframe reads the frame coder's first decision (what the
    decoder's host side uses to cut GOPs, ffv1host.cpp ffv1_keyframe_bit):
    true exactly on the GOP's first frames of an FFmpeg-like stream and on
    every frame of pixpath's intra stream."""
    from pixpath.ffv1 import packet_is_keyframe
    rng = np.random.default_rng(4)
    w, h = 96, 64
    pf = ffmpeg_like(8, 1, 1, gop=4)
    enc = ref.GenEncoder(pf, w, h)
    keys = [packet_is_keyframe(enc.encode(f)) for f in _frames(rng, po.YUV420P, w, h, 9)]
    assert keys == [i % 4 == 0 for i in range(9)]
    f = synth.noise_frame(rng, po.YUV420P, w, h)
    assert packet_is_keyframe(ref.encode_frame(f, 8, 1, 1, 2, 2))


def test_concat_keeps_gop_keyframe_flags(tmp_path):
    """`cli concat` of FFmpeg-like GOP segment AVIs (create_avpvs_long_concat's
    packet copy): packets byte for byte, the index's keyframe flags from the
    packets."""
    import struct
    from pixpath import avi, cli
    rng = np.random.default_rng(6)
    w, h = 96, 64
    pf = ffmpeg_like(10, 1, 0, gop=3)
    x = ref.gen_extradata(pf)
    segs, allp = [], []
    for k in range(2):
        enc = ref.GenEncoder(pf, w, h)
        pk = [enc.encode(f) for f in _frames(rng, po.YUV422P10LE, w, h, 5)]
        path = str(tmp_path / ("seg%d.avi" % k))
        wr = avi.AviWriter(path, w, h, 60, extradata=x)
        for i, p in enumerate(pk):
            wr.write_packet(p, key=i % 3 == 0)
        wr.close()
        segs.append(path)
        allp += pk
    fl = tmp_path / "list.txt"
    fl.write_text("".join("file '%s'\n" % s for s in segs))
    out = str(tmp_path / "long.avi")
    assert cli.main(["concat", "-y", "--filelist", str(fl), out]) == 0
    info, pk = avi.read_packets(out)
    assert pk == allp and info["extradata"] == x
    data = open(out, "rb").read()
    i = data.index(b"idx1")
    n = struct.unpack_from("<I", data, i + 4)[0] // 16
    flags = [struct.unpack_from("<4sIII", data, i + 8 + 16 * j)[1] for j in range(n)]
    assert [bool(f & 0x10) for f in flags] == [j % 5 % 3 == 0 for j in range(10)]
