"""FFV1, host side.

* the CPU restatement (oracle/ffv1_oracle.c) decodes its own packets back to
  the input losslessly -- 8/10-bit, 4:2:0/4:2:2, noise / smooth / full-range
  extremes, several slice grids -- including FFmpeg's end-of-slice position
  check and the slice / record CRCs (the only pinning available: no FFV1
  decoder exists here, so parity against FFmpeg is unpinned);
* a corrupted byte is caught by the slice CRC;
* the configuration record the product builds on the host
  (pp_ffv1_encoder_create with no context) equals the oracle's byte for byte
  and parses to the documented fields.
"""
import numpy as np
import pytest

import ffv1_ref as ref
import pyoracle as po
import synth
from pixpath import ffv1

FMTS = [("yuv422p10le", po.YUV422P10LE, 10, 1, 0), ("yuv420p", po.YUV420P, 8, 1, 1),
        ("yuv420p10le", po.YUV420P10LE, 10, 1, 1), ("yuv422p", po.YUV422P, 8, 1, 0)]


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
@pytest.mark.parametrize("kind", ["noise", "smooth", "checker", "steps"])
@pytest.mark.parametrize("grid", [(1, 1), (2, 2), (4, 3)])
def test_oracle_round_trip(name, fid, bits, hs, vs, kind, grid):
    w, h = 192, 108
    rng = np.random.default_rng(hash((name, kind, grid)) & 0xffff)
    if kind == "noise":
        planes = synth.noise_frame(rng, fid, w, h)
    elif kind == "smooth":
        planes = synth.smooth_frame(7, fid, w, h)
    else:
        planes = synth.extreme_frame(kind, fid, w, h, seams_x=(50, 100), seams_y=(30,))
    extra = ref.extradata(bits, hs, vs, *grid)
    pkt = ref.encode_frame(planes, bits, hs, vs, *grid)
    rc, dec = ref.decode_frame(extra, pkt, w, h, bits, hs, vs)
    assert rc == 0
    for p in range(3):
        np.testing.assert_array_equal(dec[p], planes[p])


def test_slice_crc_catches_corruption():
    planes = synth.noise_frame(np.random.default_rng(5), po.YUV422P10LE, 128, 64)
    extra = ref.extradata(10, 1, 0, 2, 2)
    pkt = bytearray(ref.encode_frame(planes, 10, 1, 0, 2, 2))
    pkt[len(pkt) // 3] ^= 0x10
    rc, _ = ref.decode_frame(extra, bytes(pkt), 128, 64, 10, 1, 0)
    assert rc == -3


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
@pytest.mark.parametrize("grid", [(1, 1), (4, 4), (8, 6)])
def test_product_configuration_record(name, fid, bits, hs, vs, grid):
    enc = ffv1.Ffv1Encoder(name, 1920, 1080, slices=grid, host_only=True)
    x = enc.extradata
    assert x == ref.extradata(bits, hs, vs, *grid)
    rc, info = ref.parse_extradata(x)
    assert rc == 0 and info["crc_ok"] == 1
    assert (info["version"], info["micro_version"], info["coder_type"], info["ec"], info["intra"]) == (3, 4, 1, 1, 1)
    assert (info["bits"], info["hsub"], info["vsub"]) == (bits, hs, vs)
    assert (info["num_h_slices"], info["num_v_slices"], info["context_count"]) == (grid[0], grid[1], ref.pixpath_contexts(bits))
    assert ref.crc(x) == 0


@pytest.mark.parametrize("name,fid,bits,hs,vs", FMTS, ids=[f[0] for f in FMTS])
def test_product_decoder_reads_the_record(name, fid, bits, hs, vs):
    """pp_ffv1_decoder_create (host-only) accepts the oracle's record, reports
    the frame format, and refuses a record whose CRC parity is broken."""
    x = ref.extradata(bits, hs, vs, 8, 8)
    dec = ffv1.Ffv1Decoder(x, 1920, 1080, host_only=True)
    assert dec.fmt.name == name
    bad = bytearray(x)
    bad[3] ^= 0x04
    with pytest.raises(Exception, match="CRC"):
        ffv1.Ffv1Decoder(bytes(bad), 1920, 1080, host_only=True)


@pytest.mark.parametrize("w,grid,lpw,cap", [(1920, (8, 8), 16, 240), (1920, (1, 1), 16, 1920), (3840, (2, 2), 16, 1920),
                                            (4912, (1, 1), 16, 4912), (4992, (1, 1), 15, 4992), (5120, (1, 1), 15, 5120),
                                            (16384, (1, 1), 4, 16384), (1000, (3, 1), 16, 336)])
def test_decoder_geometry_fits_the_lds(w, grid, lpw, cap):
    """The decoder's slices per workgroup (pp_ffv1_decoder_geometry, host
    only): the widest slice row rounded to 8 samples, 2 B per sample per slice
    within the 156 KB of dynamic LDS less the record's quantisation tables
    (2.5 KB per set); 16 slices up to 4,912-sample rows, fewer beyond (the path
    tests/test_gpu_ffv1.py's wide-row cases run)."""
    x = ref.extradata(10, 1, 0, *grid)
    dec = ffv1.Ffv1Decoder(x, w, 64, host_only=True)
    assert (dec.slices_per_workgroup, dec.row_cap) == (lpw, cap)
    assert 2560 + lpw * cap * 2 <= 160 * 1024 - 4096


def test_encoder_refuses_grids_that_drop_chroma():
    """A slice at x0 covers chroma columns [x0 >> hsub, + ceil(width / 2)): with
    odd slice boundaries the last chroma row / column can fall in no slice
    (333x191 4:2:0 in 3x3 slices misses chroma row 95).  FFmpeg's encoder
    avoids such grids; pixpath's refuses them instead of dropping samples."""
    with pytest.raises(Exception, match="no slice"):
        ffv1.Ffv1Encoder("yuv420p", 333, 191, slices=(3, 3), host_only=True)
    ffv1.Ffv1Encoder("yuv422p", 333, 191, slices=(3, 3), host_only=True)   # no vertical subsampling
    ffv1.Ffv1Encoder("yuv420p", 333, 190, slices=(3, 2), host_only=True)   # odd width, covered
