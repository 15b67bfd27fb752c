"""FFV1 encoder on the GPU against the CPU
restatement: every frame packet byte-identical to oracle/ffv1_oracle.c's,
and decoded back to the input by the oracle's decoder (lossless; the slice
CRCs and FFmpeg's end-of-slice position check pass).  Parity against FFmpeg
itself is unpinned (no FFV1 implementation exists in this container or on
the box)."""
import os

import numpy as np
import pytest

import ffv1_ref as ref
import pyoracle as po
import synth

pytestmark = pytest.mark.gpu

CASES = [("yuv422p10le", po.YUV422P10LE, 10, 1, 0), ("yuv420p", po.YUV420P, 8, 1, 1),
         ("yuv420p10le", po.YUV420P10LE, 10, 1, 1), ("yuv422p", po.YUV422P, 8, 1, 0)]


def _const_frame(fid, w, h, v):
    depth, hs, vs = po.fmt_info(fid)
    dt = np.uint16 if depth > 8 else np.uint8
    return [np.full(sh, v << (depth - 8), dt) for sh in po.plane_shapes(fid, w, h)]


def _gradient_frame(fid, w, h, t, rng):
    """bench.py --workload ffv1 content: moving gradients + noise in [-4, 4]."""
    depth, hs, vs = po.fmt_info(fid)
    dt = np.uint16 if depth > 8 else np.uint8
    hi = (1 << depth) - 1
    out = []
    for p, (r, c) in enumerate(po.plane_shapes(fid, w, h)):
        yy, xx = np.mgrid[0:r, 0:c]
        v = (xx * (p + 1) + yy * 2 + 3 * t) % (hi * 4 // 5) + hi // 10 + rng.integers(-4, 5, (r, c))
        out.append(np.clip(v, 0, hi).astype(dt))
    return out


@pytest.mark.parametrize("name,fid,bits,hs,vs", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("grid", [(8, 8), (16, 16)])
def test_gpu_constant_and_gradient_content(gpu, name, fid, bits, hs, vs, grid):
    """Content with very few contexts (a constant frame: tiny slices, the
    |residual| = 2^(bits-1) border samples) and the bench's moving gradients:
    GPU packets byte-identical to the C restatement, and the GPU decoder
    returns the input from both its own and the restatement's packets."""
    from pixpath import ffv1
    w, h = 1920, 1080
    rng = np.random.default_rng(bits + grid[0])
    frames = [_const_frame(fid, w, h, 128), _gradient_frame(fid, w, h, 3, rng)]
    enc = ffv1.Ffv1Encoder(name, w, h, slices=grid, max_frames=len(frames), device=gpu)
    pkts = enc.encode_to_host(_batch(gpu, name, frames))
    dec = ffv1.Ffv1Decoder(enc.extradata, w, h, max_frames=len(frames), device=gpu)
    for f, planes in enumerate(frames):
        want = ref.encode_frame(planes, bits, hs, vs, *grid)
        if pkts[f] != want:
            n = min(len(pkts[f]), len(want))
            first = next((i for i in range(n) if pkts[f][i] != want[i]), n)
            pytest.fail("frame %d: %d vs %d bytes, first difference at %d" % (f, len(pkts[f]), len(want), first))
        for pk in (pkts[f], want):
            out = dec.decode(pk, [len(pk)]).to_numpy()
            for p in range(3):
                np.testing.assert_array_equal(out[p][0], planes[p])


def _batch(gpu, name, frames):
    from pixpath.frames import FrameBatch
    return FrameBatch.from_numpy(name, [np.stack([f[p] for f in frames]) for p in range(3)], device=gpu)


@pytest.mark.parametrize("name,fid,bits,hs,vs", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("w,h,grid", [(640, 360, (4, 4)), (330, 190, (3, 2)), (1920, 1080, (4, 4)),
                                      (640, 360, (8, 8)), (1280, 720, (16, 16)), (200, 90, (7, 5))])
def test_gpu_packets_match_oracle(gpu, name, fid, bits, hs, vs, w, h, grid):
    from pixpath import ffv1
    rng = np.random.default_rng(w + h)
    frames = [synth.noise_frame(rng, fid, w, h), synth.smooth_frame(3, fid, w, h),
              synth.extreme_frame("steps", fid, w, h, seams_x=(w // 3,), seams_y=(h // 2,))]
    if w * h > 1_000_000:
        frames = frames[1:2]  # the C oracle takes ~1 s per 1080p frame
    enc = ffv1.Ffv1Encoder(name, w, h, slices=grid, max_frames=len(frames), device=gpu)
    pkts = enc.encode_to_host(_batch(gpu, name, frames))
    extra = enc.extradata
    assert extra == ref.extradata(bits, hs, vs, *grid)
    for f, planes in enumerate(frames):
        want = ref.encode_frame(planes, bits, hs, vs, *grid)
        if pkts[f] != want:
            n = min(len(pkts[f]), len(want))
            first = next((i for i in range(n) if pkts[f][i] != want[i]), n)
            pytest.fail("frame %d: %d vs %d bytes, first difference at %d" % (f, len(pkts[f]), len(want), first))
        rc, dec = ref.decode_frame(extra, pkts[f], w, h, bits, hs, vs)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], planes[p])


def test_gpu_600_frames_lossless(gpu):
    """A config-2-sized AVPVS batch (600 distinct 1080p yuv422p10le frames) in
    one encode: packet sizes add up, and the first, a middle and the last
    frame decode back to their inputs."""
    import torch
    from pixpath import ffv1
    from pixpath.frames import FrameBatch
    n = 600
    src = FrameBatch("yuv422p10le", 1920, 1080, n, device=gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(600)
    base = torch.arange(1920, device=gpu, dtype=torch.int32)
    for p in range(3):
        v = src.view(p)
        ramp = (base[: v.shape[2]] * (p + 1)) % 880 + 64
        noise = torch.randint(0, 8, v.shape, generator=g, device=gpu, dtype=torch.int32)
        fr = torch.arange(n, device=gpu, dtype=torch.int32).view(n, 1, 1)
        v.copy_(((ramp.view(1, 1, -1) + noise + fr) % 1024).to(v.dtype))
    enc = ffv1.Ffv1Encoder("yuv422p10le", 1920, 1080, slices=(4, 4), max_frames=n, device=gpu)
    buf, sizes = enc.encode(src)
    assert buf.numel() == int(sizes.sum()) and (sizes > 0).all()
    data = buf.cpu().numpy().tobytes()
    offs = np.concatenate([[0], np.cumsum(sizes)])
    extra = enc.extradata
    for f in (0, 299, n - 1):
        rc, dec = ref.decode_frame(extra, data[offs[f]:offs[f + 1]], 1920, 1080, 10, 1, 0)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], src.view(p)[f].cpu().numpy())


@pytest.mark.parametrize("name,fid,bits,hs,vs", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("w,h,grid", [(640, 360, (4, 4)), (330, 190, (3, 2)), (1920, 1080, (8, 8))])
def test_gpu_decoder_round_trip(gpu, name, fid, bits, hs, vs, w, h, grid):
    """GPU encode -> GPU decode returns the input frames; the GPU decoder
    also reads the C restatement's packets (the same bytes)."""
    from pixpath import ffv1
    rng = np.random.default_rng(w * 7 + h)
    frames = [synth.noise_frame(rng, fid, w, h), synth.smooth_frame(5, fid, w, h),
              synth.extreme_frame("checker", fid, w, h)]
    enc = ffv1.Ffv1Encoder(name, w, h, slices=grid, max_frames=len(frames), device=gpu)
    pkts = enc.encode_to_host(_batch(gpu, name, frames))
    dec = ffv1.Ffv1Decoder(enc.extradata, w, h, max_frames=len(frames), device=gpu)
    out = dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy()
    for f, planes in enumerate(frames):
        for p in range(3):
            np.testing.assert_array_equal(out[p][f], planes[p])
    if w * h < 1_000_000:
        ref_pkt = ref.encode_frame(frames[0], bits, hs, vs, *grid)
        out0 = dec.decode(ref_pkt, [len(ref_pkt)]).to_numpy()
        for p in range(3):
            np.testing.assert_array_equal(out0[p][0], frames[0][p])


def test_gpu_decoder_rejects_corruption(gpu):
    from pixpath import ffv1
    rng = np.random.default_rng(3)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 320, 180)]
    enc = ffv1.Ffv1Encoder("yuv422p10le", 320, 180, slices=(2, 2), max_frames=1, device=gpu)
    pkt = bytearray(enc.encode_to_host(_batch(gpu, "yuv422p10le", frames))[0])
    dec = ffv1.Ffv1Decoder(enc.extradata, 320, 180, max_frames=1, device=gpu)
    pkt[len(pkt) // 2] ^= 0x20
    with pytest.raises(Exception, match="CRC|chain"):
        dec.decode(bytes(pkt), [len(pkt)])


def test_gpu_decode_600_frames(gpu):
    """A whole 600-frame 1080p yuv422p10le AVPVS: GPU encode -> GPU decode, every frame equal."""
    import torch
    from pixpath import ffv1
    from pixpath.frames import FrameBatch
    n = 600
    src = FrameBatch("yuv422p10le", 1920, 1080, n, device=gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(60)
    for p in range(3):
        v = src.view(p)
        v.copy_((torch.randint(0, 1024, v.shape, generator=g, device=gpu, dtype=torch.int32) // 16 * 16).to(v.dtype))
    enc = ffv1.Ffv1Encoder("yuv422p10le", 1920, 1080, slices=(8, 8), max_frames=n, device=gpu)
    buf, sizes = enc.encode(src)
    dec = ffv1.Ffv1Decoder(enc.extradata, 1920, 1080, max_frames=n, device=gpu)
    out = dec.decode(buf.cpu().numpy().tobytes(), sizes)
    for p in range(3):
        assert torch.equal(out.view(p)[:n], src.view(p)[:n])


def test_cli_avpvs_cpvs_through_gpu_ffv1(gpu, tmp_path):
    """create_avpvs_short -> create_cpvs with the FFV1 AVPVS encoded and decoded
    on the GPU (`--gpu-ffv1`): the AVI holds FFV1 packets the C restatement
    decodes to the oracle's scaled frames, and the CPVS read back from it
    equals the oracle's pad + v210 of those frames."""
    from fractions import Fraction
    from pixpath import avi, cli, io as pio
    rng = np.random.default_rng(12)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 640, 360) for _ in range(70)]
    seg, avpvs, cpvs = (str(tmp_path / n) for n in ("seg.y4m", "avpvs.avi", "cpvs.raw"))
    wr = pio.Y4MWriter(seg, "yuv422p10le", 640, 360, 60)
    wr.write(pio.join_planes(synth.batch(frames)))
    wr.close()
    assert cli.main(["avpvs", "-y", "--input", seg, "--size", "1280x720", "--pix-fmt", "yuv422p10le",
                     "--aopts=-an", "--gpu-ffv1", "--batch", "32", avpvs]) == 0
    info, pk = avi.read_packets(avpvs)
    assert (info["w"], info["h"], info["rate"], len(pk)) == (1280, 720, Fraction(60), 70)
    want = [po.scale(po.YUV422P10LE, f, po.YUV422P10LE, 1280, 720, po.SWS_BICUBIC) for f in frames]
    for j in (0, 33, 69):
        rc, dec = ref.decode_frame(info["extradata"], pk[j], 1280, 720, 10, 1, 0)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], want[j][p])
    assert cli.main(["cpvs", "-y", "--input", avpvs, "--fps", "60", "--vcodec", "v210", "--pix-fmt", "yuv422p10le",
                     "--pad", "1280x800", "--gpu-ffv1", cpvs]) == 0
    raw = np.fromfile(cpvs, np.uint8)
    fb = po.v210_linesize(1280) * 800
    assert raw.size == 70 * fb
    for j in (0, 69):
        ref_v210 = po.v210_pack(po.pad(po.YUV422P10LE, want[j], 1280, 800, 0, 40))
        np.testing.assert_array_equal(raw[j * fb:(j + 1) * fb], ref_v210.reshape(-1))


def test_cli_stall_through_gpu_ffv1(gpu, tmp_path):
    """The stall path with FFV1 AVIs coded on the GPU: the fused pass
    (`avpvs --stall-output --gpu-ffv1`) and the bufferer step on the AVPVS AVI
    (`stall --gpu-ffv1`) give the same frames."""
    from pixpath import avi, cli, io as pio
    rng = np.random.default_rng(13)
    frames = [synth.noise_frame(rng, po.YUV420P, 320, 180) for _ in range(30)]
    seg, wo, fused, plain = (str(tmp_path / n) for n in ("seg.y4m", "wo.avi", "pvs.avi", "plain.avi"))
    wr = pio.Y4MWriter(seg, "yuv420p", 320, 180, 60)
    wr.write(pio.join_planes(synth.batch(frames)))
    wr.close()
    spinner = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spinner-128-white.png")
    buf = "[[0.1,0.1],[0.4,0.05]]"
    assert cli.main(["avpvs", "-y", "--input", seg, "--size", "640x360", "--pix-fmt", "yuv420p", "--aopts=-an",
                     "--gpu-ffv1", "--stall-output", fused, "--buffer", buf, "--black-frame", "--spinner", spinner,
                     wo]) == 0
    assert cli.main(["stall", "-y", "--input", wo, "--buffer", buf, "--pix-fmt", "yuv420p", "--black-frame",
                     "--spinner", spinner, "--vopts", "-c:v ffv1", "--aopts=-an", "--gpu-ffv1", plain]) == 0
    (i1, p1), (i2, p2) = avi.read_packets(fused), avi.read_packets(plain)
    assert len(p1) == len(p2) == 30 + 6 + 3
    for a_, b_ in zip(p1, p2):
        r1, d1 = ref.decode_frame(i1["extradata"], a_, 640, 360, 8, 1, 1)
        r2, d2 = ref.decode_frame(i2["extradata"], b_, 640, 360, 8, 1, 1)
        assert r1 == r2 == 0
        for p in range(3):
            np.testing.assert_array_equal(d1[p], d2[p])


def _black(fid, w, h):
    depth, hs, vs = po.fmt_info(fid)
    dt = np.uint16 if depth > 8 else np.uint8
    return [np.full(s, (16 if p == 0 else 128) << (depth - 8), dt) for p, s in enumerate(po.plane_shapes(fid, w, h))]


@pytest.mark.parametrize("skipping,buf", [(False, "[[0,0.1],[0.3,0.05],[9,0.05]]"), (True, "[[0.1,0.1],[0.25,0.2]]")])
def test_packet_level_stall_matches_oracle(gpu, tmp_path, skipping, buf):
    """PP-STALL-1 on a GPU-FFV1 AVPVS at the packet level (ffv1.stall_avi,
    what `cli stall --gpu-ffv1` and the fused `avpvs --stall-output --gpu-ffv1`
    run): every output packet decodes (C restatement) to the oracle's frame --
    the scaled input, the frozen / black frame with the spinner -- and every
    pass-through frame is the input packet byte for byte."""
    import ast
    from pixpath import avi, cli, io as pio, spinner, stall
    rng = np.random.default_rng(21)
    n, fid = 30, po.YUV420P
    frames = [synth.noise_frame(rng, fid, 320, 180) for _ in range(n)]
    seg, wo, out = (str(tmp_path / x) for x in ("seg.y4m", "wo.avi", "pvs.avi"))
    wr = pio.Y4MWriter(seg, "yuv420p", 320, 180, 60)
    wr.write(pio.join_planes(synth.batch(frames)))
    wr.close()
    sp_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spinner-128-white.png")
    assert cli.main(["avpvs", "-y", "--input", seg, "--size", "640x360", "--pix-fmt", "yuv420p", "--aopts=-an",
                     "--gpu-ffv1", wo]) == 0
    args = ["stall", "-y", "--input", wo, "--buffer", buf, "--pix-fmt", "yuv420p", "--spinner", sp_path,
            "--black-frame", "--aopts=-an", "--gpu-ffv1", out]
    if skipping:
        args.insert(-1, "--skipping")
    assert cli.main(args) == 0
    iw, pin = avi.read_packets(wo)
    io_, pout = avi.read_packets(out)
    assert io_["extradata"] == iw["extradata"]
    anim, delays = spinner.load_apng(sp_path)
    seq = stall.stall_schedule(ast.literal_eval(buf), 60, n, skipping, delays, True)
    assert len(pout) == len(seq)
    scaled = [po.scale(fid, f, fid, 640, 360, po.SWS_BICUBIC) for f in frames]
    for k in range(n):  # the AVPVS itself: every packet decodes to the scaled frame
        rc, dec = ref.decode_frame(iw["extradata"], pin[k], 640, 360, 8, 1, 1)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], scaled[k][p], err_msg="AVPVS frame %d plane %d" % (k, p))
    yuva = {}
    for k, (s, sp) in enumerate(seq):
        if sp < 0 and s >= 0:
            assert pout[k] == pin[s], "pass-through frame %d is not the input packet" % k
            continue
        base = scaled[s] if s >= 0 else _black(fid, 640, 360)
        if sp >= 0:
            if sp not in yuva:
                yuva[sp] = po.spinner_to_yuva(anim[sp], fid)
            base = po.overlay_spinner(fid, base, yuva[sp])
        rc, dec = ref.decode_frame(io_["extradata"], pout[k], 640, 360, 8, 1, 1)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], base[p], err_msg="output frame %d plane %d" % (k, p))


def test_writer_device_batches_and_canvas_repeat(gpu, tmp_path):
    """create_avpvs_segment through the GPU FFV1 writer fed with device
    batches (no D2H): the canvas of D*R frames repeats the last scaled frame,
    every packet decodes to the oracle's two-stage chain output."""
    from pixpath import avi, cli, io as pio
    rng = np.random.default_rng(31)
    frames = [synth.noise_frame(rng, po.YUV422P10LE, 320, 180) for _ in range(50)]
    seg, out = str(tmp_path / "seg.y4m"), str(tmp_path / "tmp_seg.avi")
    wr = pio.Y4MWriter(seg, "yuv422p10le", 320, 180, 60)
    wr.write(pio.join_planes(synth.batch(frames)))
    wr.close()
    assert cli.main(["avpvs", "-y", "--input", seg, "--size", "640x360", "--pix-fmt", "yuv422p10le", "--fps", "60",
                     "--duration", "1", "--overlay-yuv420", "--aopts=-an", "--gpu-ffv1", "--batch", "16", out]) == 0
    info, pk = avi.read_packets(out)
    assert len(pk) == 60
    for k in (0, 17, 49, 50, 59):
        f = frames[min(k, 49)]
        mid = po.scale(po.YUV422P10LE, f, po.YUV420P, 640, 360, po.SWS_BICUBIC)
        want = po.scale(po.YUV420P, mid, po.YUV422P10LE, 640, 360, po.SWS_BICUBIC)
        rc, dec = ref.decode_frame(info["extradata"], pk[k], 640, 360, 10, 1, 0)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], want[p])
    assert pk[50] == pk[59] == pk[49]


def test_writer_pool_reuses_encoder_across_pvses(gpu, tmp_path):
    """Two AVPVS writers in a row in one process (the reference's runner
    feeding several PVSes): the second takes the first's encoder from the
    pool, and both AVIs decode to their own frames (context states and slice
    buffers start clean for every batch)."""
    import torch
    from pixpath import avi, ffv1
    from pixpath.frames import FrameBatch
    rng = np.random.default_rng(77)
    w, h = 320, 180
    encs = []
    for k in range(2):
        frames = [synth.noise_frame(rng, po.YUV422P10LE, w, h) for _ in range(5)] if k == 0 else \
            [synth.smooth_frame(3 + i, po.YUV422P10LE, w, h) for i in range(7)]
        path = str(tmp_path / ("PVS%d.avi" % k))
        wr = ffv1.Ffv1AviWriter(path, "yuv422p10le", w, h, 60, slices=(4, 4), batch=8, device=gpu)
        encs.append(set(wr.encs))
        src = FrameBatch.interleaved("yuv422p10le", w, h, len(frames), device=gpu)
        for i, f in enumerate(frames):
            for p in range(3):
                src.view(p)[i].copy_(torch.from_numpy(f[p].astype(np.uint16)))
        wr.write_device(src)
        wr.close()
        info, pk = avi.read_packets(path)
        assert len(pk) == len(frames)
        for i, f in enumerate(frames):
            rc, dec = ref.decode_frame(info["extradata"], pk[i], w, h, 10, 1, 0)
            assert rc == 0
            for p in range(3):
                np.testing.assert_array_equal(dec[p], f[p], err_msg="PVS %d frame %d plane %d" % (k, i, p))
    assert encs[1] == encs[0]


@pytest.mark.parametrize("split", [1, 2, 3])
def test_writer_lanes_write_the_same_file(gpu, tmp_path, split):
    """The AVPVS writer's encoder lanes (split = K: the batch coded as K
    sub-batches on K encoders side by side, packets written in frame order):
    the AVI is byte-identical to the one-encoder writer's for 2.5 batches of
    frames fed in uneven pieces, and decodes to the input."""
    import torch
    from pixpath import avi, ffv1
    from pixpath.frames import FrameBatch
    w, h, n = 320, 180, 25
    frames = [synth.smooth_frame(i, po.YUV422P10LE, w, h) for i in range(n)]
    src = FrameBatch.interleaved("yuv422p10le", w, h, n, device=gpu)
    for i, f in enumerate(frames):
        for p in range(3):
            src.view(p)[i].copy_(torch.from_numpy(f[p].astype(np.uint16)))
    paths = []
    for k in (1, split):
        path = str(tmp_path / ("PVS_split%d_%d.avi" % (split, k)))
        wr = ffv1.Ffv1AviWriter(path, "yuv422p10le", w, h, 60, slices=(4, 4), batch=10, device=gpu, split=k)
        assert wr.K == k and len(wr.encs) == k
        for a, b in ((0, 3), (3, 11), (11, 12), (12, 25)):
            wr.write_device(FrameBatch.interleaved("yuv422p10le", w, h, b - a, device=gpu,
                                                   storage=src.storage[a:b]))
        wr.close()
        paths.append(path)
    assert open(paths[0], "rb").read() == open(paths[1], "rb").read()
    info, pk = avi.read_packets(paths[1])
    assert len(pk) == n
    for i in (0, 4, 9, 10, 17, 24):
        rc, dec = ref.decode_frame(info["extradata"], pk[i], w, h, 10, 1, 0)
        assert rc == 0
        for p in range(3):
            np.testing.assert_array_equal(dec[p], frames[i][p], err_msg="frame %d plane %d" % (i, p))


def test_writer_lanes_by_open_writers(gpu, tmp_path, monkeypatch):
    """writer_split: a writer opened alone on the device takes default_split()
    lanes, one opened while it is open takes one encoder of the whole batch,
    and once both are closed the next writer takes lanes again."""
    from pixpath import ffv1
    monkeypatch.delenv("PIXPATH_FFV1_SPLIT", raising=False)
    mk = lambda name: ffv1.Ffv1AviWriter(str(tmp_path / name), "yuv422p10le", 64, 32, 60, slices=(1, 1),
                                         batch=6, device=gpu)
    a = mk("a.avi")
    b = mk("b.avi")
    assert a.K == ffv1.default_split() == 2 and b.K == 1 and b.sub == 6 and a.sub == 3
    b.close()
    a.close()
    c = mk("c.avi")
    assert c.K == 2
    c.close()


def test_record_budget_split_keeps_the_bytes(gpu):
    """The per-slice renorm-record budget (pp_ffv1_encode_packets): a batch of
    mostly smooth frames with noise frames among them overflows the budget
    of a full launch, is re-coded in halves down to launches where every
    slice fits, and its packets are byte-identical to frame-by-frame encodes
    (max_frames=1: always the worst-case records) and to the C restatement."""
    from pixpath import ffv1
    w, h, grid = 640, 360, (4, 4)
    rng = np.random.default_rng(91)
    frames = [synth.smooth_frame(i, po.YUV422P10LE, w, h) for i in range(8)]
    frames[5] = synth.noise_frame(rng, po.YUV422P10LE, w, h)
    enc = ffv1.Ffv1Encoder("yuv422p10le", w, h, slices=grid, max_frames=8, device=gpu)
    pkts = enc.encode_to_host(_batch(gpu, "yuv422p10le", frames))
    assert enc.launches > 1
    one = ffv1.Ffv1Encoder("yuv422p10le", w, h, slices=grid, max_frames=1, device=gpu)
    for f, planes in enumerate(frames):
        assert pkts[f] == one.encode_to_host(_batch(gpu, "yuv422p10le", [planes]))[0], "frame %d" % f
    assert one.launches == 1
    for f in (4, 5):
        assert pkts[f] == ref.encode_frame(frames[f], 10, 1, 0, *grid)
    smooth = ffv1.Ffv1Encoder("yuv422p10le", w, h, slices=grid, max_frames=8, device=gpu)
    smooth.encode_to_host(_batch(gpu, "yuv422p10le", frames[:5]))
    assert smooth.launches == 1


def test_encoder_footprint(gpu):
    """A 600-frame 1080p yuv422p10le encoder (the AVPVS writer's) holds less
    than 18 GB of HBM: tokens 10 GB, renorm records ~5 GB, context states
    1.6 GB; the slice bytes are resolved in place over the records."""
    from pixpath import ffv1
    enc = ffv1.Ffv1Encoder("yuv422p10le", 1920, 1080, slices=(8, 8), max_frames=600, device=gpu)
    assert enc.memory_bytes < 18e9


def test_failed_writer_leaves_no_file_and_frees_its_encoder(gpu, tmp_path, monkeypatch):
    """An encode that fails inside the AVI writer: close() raises, neither the
    output nor its .part file remains, and the encoder is not pooled."""
    import os
    import torch
    from pixpath import ffv1
    from pixpath.frames import FrameBatch
    ffv1.clear_pool()
    path = str(tmp_path / "PVS.avi")
    wr = ffv1.Ffv1AviWriter(path, "yuv422p10le", 320, 180, 60, slices=(4, 4), batch=8, device=gpu)
    enc = wr.enc

    def boom(*a, **k):
        raise RuntimeError("injected encode failure")
    monkeypatch.setattr(enc, "encode_packets", boom)
    src = FrameBatch.interleaved("yuv422p10le", 320, 180, 3, device=gpu)
    src.storage.zero_()
    wr.write_device(src)
    with pytest.raises(RuntimeError, match="injected"):
        wr.close()
    assert not os.path.exists(path) and not os.path.exists(path + ".part")
    again = ffv1.acquire_encoder("yuv422p10le", 320, 180, slices=(4, 4), max_frames=8, device=gpu)
    assert again is not enc
    torch.cuda.synchronize()


WIDE = [(1920, 64, (1, 1), 3, 16), (5120, 16, (1, 1), 20, 15), (16384, 8, (1, 1), 6, 4),
        (1920, 1080, (1, 1), 1, 16), (1920, 1080, (2, 1), 2, 16), (1920, 1080, (2, 2), 2, 16),
        (3840, 2160, (2, 2), 1, 16)]


@pytest.mark.parametrize("name,fid,bits,hs,vs", [CASES[0], CASES[1]], ids=[CASES[0][0], CASES[1][0]])
@pytest.mark.parametrize("w,h,grid,n,lpw", WIDE, ids=["%dx%d-%dx%d" % (c[0], c[1], *c[2]) for c in WIDE])
def test_gpu_decoder_wide_slice_rows(gpu, name, fid, bits, hs, vs, w, h, grid, n, lpw):
    """Slice rows wider than 1,216 samples: the decoder sizes its
    slices per workgroup to the LDS line buffers -- 16 up to 4,912-sample rows,
    fewer beyond (5120 -> 15, 16384 -> 4, with frames spread over several
    workgroups, the last one partial).  GPU encode -> GPU decode returns the
    input; the C restatement's packets equal the GPU's and decode on the GPU."""
    from pixpath import ffv1
    rng = np.random.default_rng(w + h + n)
    frames = [synth.smooth_frame(i, fid, w, h) if i % 2 else synth.noise_frame(rng, fid, w, h) for i in range(n)]
    enc = ffv1.Ffv1Encoder(name, w, h, slices=grid, max_frames=n, device=gpu)
    pkts = enc.encode_to_host(_batch(gpu, name, frames))
    dec = ffv1.Ffv1Decoder(enc.extradata, w, h, max_frames=n, device=gpu)
    assert (dec.slices_per_workgroup, dec.row_cap) == (lpw, -(-(w // grid[0]) // 8) * 8)
    out = dec.decode(b"".join(pkts), [len(p) for p in pkts]).to_numpy()
    for f, planes in enumerate(frames):
        for p in range(3):
            np.testing.assert_array_equal(out[p][f], planes[p], err_msg="frame %d plane %d" % (f, p))
    for f in sorted({0, n - 1}):
        want = ref.encode_frame(frames[f], bits, hs, vs, *grid)
        assert pkts[f] == want, "frame %d: GPU packet differs from the C restatement's" % f
        out1 = dec.decode(want, [len(want)]).to_numpy()
        for p in range(3):
            np.testing.assert_array_equal(out1[p][0], frames[f][p])
