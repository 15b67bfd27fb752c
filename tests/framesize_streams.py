"""Synthetic bitstreams for the p02 frame-size scanner parity tests
(lib/get_framesize.py).

Deterministic builders shared by tests/golden/gen_framesize_fixtures.py (which
runs the reference's own scanners on them) and tests/test_framesize_parity.py.
Small streams are also stored verbatim (base64) in the fixture; larger ones by
seed and SHA-256, so a drift of these builders shows up as a hash mismatch.
"""
import hashlib
import struct

import numpy as np

# H.264 NAL header bytes: SPS, PPS, SEI, AUD, IDR, non-IDR (ref), non-IDR (nonref),
# plus bytes a forbidden bit or a random payload could put after a start code
H264_HDR = [0x67, 0x68, 0x06, 0x09, 0x65, 0x41, 0x01, 0x21, 0x25, 0x45, 0x61, 0x05, 0x11, 0x15, 0x81, 0x85, 0x91]
# H.265 first header bytes: VPS, SPS, PPS, AUD, SEI, TRAIL_N/R, TSA, RASL, IDR_W_RADL, IDR_N_LP, CRA, reserved
H265_HDR = [0x40, 0x42, 0x44, 0x46, 0x4e, 0x00, 0x02, 0x04, 0x10, 0x12, 0x13, 0x14, 0x26, 0x28, 0x2a, 0x2b,
            0x2c, 0x20, 0x30, 0x3e]


def _payload(rng, n, emulation=True):
    """Random slice payload; with emulation prevention no 00 00 0x (x <= 3) occurs."""
    b = rng.integers(0, 256, n, dtype=np.uint8)
    b[rng.random(n) < 0.15] = 0  # bitstreams are zero-heavy
    if not emulation:
        return bytes(b)
    out = bytearray()
    z = 0
    for v in b.tolist():
        if z >= 2 and v <= 3:
            out.append(3)
            z = 0
        out.append(v)
        z = z + 1 if v == 0 else 0
    if out and out[-1] == 0:  # rbsp_trailing: never end on a zero
        out[-1] = 0x80
    return bytes(out)


def annexb(seed, codec, nal_units, mean_size=400, emulation=True, long_sc=0.5, trailing_zeros=0.1, lead=b""):
    rng = np.random.default_rng(seed)
    hdrs = H264_HDR if codec == "h264" else H265_HDR
    out = bytearray(lead)
    for _ in range(nal_units):
        if rng.random() < trailing_zeros:
            out += b"\x00" * int(rng.integers(1, 4))
        out += b"\x00\x00\x00\x01" if rng.random() < long_sc else b"\x00\x00\x01"
        out.append(int(hdrs[int(rng.integers(len(hdrs)))]))
        if codec == "h265":
            out.append(1)  # nuh_temporal_id_plus1
        out += _payload(rng, int(rng.exponential(mean_size)) + 1, emulation)
    return bytes(out)


def zero_heavy(seed, n, alphabet):
    """Dense random bytes over a small alphabet: start codes every few bytes."""
    rng = np.random.default_rng(seed)
    a = np.array(alphabet, dtype=np.uint8)
    return bytes(a[rng.integers(0, len(a), n)])


def ivf(seed, frames, mean_size=300, bad_marker=0.1, truncate=0, size_hi_byte=None):
    rng = np.random.default_rng(seed)
    out = bytearray(b"DKIF" + struct.pack("<HHIHHIIII", 0, 32, 0x30395056, 1920, 1080, 60, 1, frames, 0))
    for i in range(frames):
        n = int(rng.exponential(mean_size))
        if i % 7 == 3:
            n = int(rng.integers(0, 4))  # 0..3-byte frames
        data = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        if n:
            data[0] = (0x80 | (data[0] & 0x3f)) if rng.random() >= bad_marker else (data[0] & 0x7f)
        size_field = n | ((size_hi_byte << 24) if (size_hi_byte and i == frames // 2) else 0)
        out += struct.pack("<IQ", size_field, i) + data
    if truncate:
        out = out[:-truncate]
    return bytes(out)


def sha256(b):
    return hashlib.sha256(b).hexdigest()


def small_cases():
    """(name, codec, bytes) edge cases, stored verbatim in the fixture."""
    sc3, sc4 = b"\x00\x00\x01", b"\x00\x00\x00\x01"
    c = []
    for codec in ("h264", "h265"):
        f = 0x65 if codec == "h264" else 0x26
        c += [
            ("one_byte", codec, b"\x01"),
            ("sc_only", codec, sc3),
            ("sc_hdr", codec, sc3 + bytes([f])),
            ("sc4_hdr", codec, sc4 + bytes([f])),
            ("sc_at_end", codec, sc4 + bytes([f]) + b"\x11\x22" + sc3),
            ("no_leading_sc", codec, b"\x12\x34\x56" + sc3 + bytes([f]) + b"\x01\x02\x03" + sc4 + bytes([f, 9])),
            ("two_frames", codec, sc4 + bytes([f, 0x88, 0x99]) + sc4 + bytes([f, 1, 2, 3, 4])),
            ("zero_zero_sc", codec, sc3 + b"\x00" + sc3 + bytes([f]) + b"\x00\x00\x00\x00\x01" + bytes([f, 7])),
            ("nonframe_then_frame", codec, sc4 + b"\x67\x42" + sc3 + bytes([f, 0xaa]) + sc4 + b"\x68\x01"),
            ("hdr_after_zeros", codec, b"\x00\x00\x00\x00\x00\x01" + bytes([f]) + b"\x00\x00\x01\x01\x00\x00\x01"),
        ]
    c += [
        ("h264_a5_valueerror", "h264", sc4 + b"\x65\x10" + sc3 + b"\xa5\x00"),
        ("h264_b1_valueerror", "h264", sc3 + b"\xb1"),
        ("h264_c2_no_error", "h264", sc4 + b"\x65\x10" + sc3 + b"\xc2\x00" + sc3 + b"\x85"),
        ("h264_high_even", "h264", sc3 + b"\x81\x01\x02" + sc3 + b"\x91\x03" + sc3 + b"\x25"),
        ("h265_boundaries", "h265", b"".join(sc3 + bytes([h, 1, 0x55]) for h in
                                             (0x0f, 0x10, 0x13, 0x14, 0x1f, 0x20, 0x2b, 0x2c, 0x30))),
    ]
    return c


def medium_cases():
    """(name, codec, seed, builder) larger streams, stored by hash."""
    return [
        ("h264_stream", "h264", 264, lambda: annexb(264, "h264", 300)),
        ("h264_raw_scs", "h264", 265, lambda: annexb(265, "h264", 200, emulation=False)),
        ("h264_lead_garbage", "h264", 266, lambda: annexb(266, "h264", 120, lead=b"\x12\x00\x00\x00\x00")),
        ("h264_dense", "h264", 267, lambda: zero_heavy(267, 60000, [0, 0, 0, 1, 0x65, 0x41, 0x01, 0x09, 0x81, 0x7f])),
        ("h265_stream", "h265", 2650, lambda: annexb(2650, "h265", 300)),
        ("h265_raw_scs", "h265", 2651, lambda: annexb(2651, "h265", 200, emulation=False)),
        ("h265_dense", "h265", 2652, lambda: zero_heavy(2652, 60000, [0, 0, 0, 1, 0x26, 0x02, 0x40, 0x2b, 0x2c, 0xff])),
    ]


def ivf_cases():
    return [
        ("ivf_header_only", lambda: ivf(1, 0)),
        ("ivf_short", lambda: ivf(2, 0)[:20]),
        ("ivf_small", lambda: ivf(3, 12, mean_size=40)),
        ("ivf_stream", lambda: ivf(4, 300)),
        ("ivf_bad_markers", lambda: ivf(5, 80, bad_marker=0.5)),
        ("ivf_truncated", lambda: ivf(6, 40, truncate=7)),
        ("ivf_truncated_hdr", lambda: ivf(7, 40, mean_size=50)[:-(50 + 10)]),
        ("ivf_size_hi_byte", lambda: ivf(8, 30, mean_size=64, size_hi_byte=1)),
        ("ivf_random", lambda: bytes(np.random.default_rng(9).integers(0, 256, 5000, dtype=np.uint8))),
    ]


def vfi_cases():
    """delete_packets inputs: VP9 packet lists (index, dts, size) per segment."""
    def seg(n, t0, step=1 / 60, pairs=(), start_index=0):
        out = []
        for i in range(n):
            out.append({"index": start_index + i, "dts": round(t0 + i * step, 6), "size": 1000 + 17 * i})
            if i in pairs:
                out.append({"index": start_index + i + 1, "dts": round(t0 + i * step + 0.0005, 6), "size": 33 + i})
        return out

    def reindex(lst):  # ffprobe-like running index within a segment
        for i, p in enumerate(lst):
            p["index"] = i
        return lst

    return [
        ("no_superframes", seg(10, 0.0)),
        ("superframes", reindex(seg(12, 0.0, pairs=(2, 5, 9)))),
        ("two_segments", reindex(seg(8, 0.0, pairs=(1,))) + reindex(seg(8, 8 / 60, pairs=(3, 4)))),
        ("first_index_not_zero", seg(5, 0.0, start_index=3)),
        ("adjacent_pairs", reindex(seg(6, 0.0, pairs=(0, 1, 2)))),
    ]
