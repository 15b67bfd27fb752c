"""ctypes front of oracle/ffv1_oracle.c (TEST INFRASTRUCTURE ONLY: tests/,
bench.py's cpu_baseline).  FFV1 v3 restatement, parity unpinned against
FFmpeg (absent); see the C file's header."""
import ctypes
import os

import numpy as np

_LIB = os.environ.get("PIXORACLE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                         "libpixoracle.so")
_lib = None
INFO_KEYS = ("version", "micro_version", "coder_type", "colorspace", "bits", "chroma_planes", "hsub", "vsub",
             "extra_plane", "num_h_slices", "num_v_slices", "quant_table_sets", "ec", "intra", "context_count",
             "crc_ok")


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(_LIB)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.ffv1o_extradata.argtypes = [i32, i32, i32, i32, i32, vp, i64]
        L.ffv1o_extradata.restype = i64
        L.ffv1o_encode_frame.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, i64]
        L.ffv1o_encode_frame.restype = i64
        L.ffv1o_decode_frame.argtypes = [vp, i64, vp, i64, i32, i32, vp, vp]
        L.ffv1o_decode_frame.restype = i32
        L.ffv1o_parse_extradata.argtypes = [vp, i64, vp]
        L.ffv1o_crc.argtypes = [ctypes.c_uint32, vp, i64]
        L.ffv1o_crc.restype = ctypes.c_uint32
        L.ffv1o_state_tables.argtypes = [vp, vp]
        _lib = L
    return _lib


def _ptrs(planes):
    arr = (ctypes.c_void_p * 3)(*[p.ctypes.data for p in planes])
    ls = (ctypes.c_int64 * 3)(*[p.strides[0] for p in planes])
    return arr, ls


def extradata(bits, hsub, vsub, nh, nv):
    buf = np.zeros(4096, np.uint8)
    n = lib().ffv1o_extradata(bits, hsub, vsub, nh, nv, buf.ctypes.data, buf.size)
    if n < 0:
        raise RuntimeError("extradata")
    return buf[:n].tobytes()


def parse_extradata(x):
    info = (ctypes.c_int * 16)()
    b = np.frombuffer(x, np.uint8)
    rc = lib().ffv1o_parse_extradata(b.ctypes.data, b.size, info)
    return rc, dict(zip(INFO_KEYS, list(info)))


def encode_frame(planes, bits, hsub, vsub, nh, nv):
    """planes: 2-D numpy arrays (uint8 / uint16).  Returns the packet bytes."""
    planes = [np.ascontiguousarray(p) for p in planes]
    h, w = planes[0].shape
    cap = sum(p.nbytes for p in planes) * 2 + 4096 + 64 * nh * nv
    out = np.zeros(cap, np.uint8)
    arr, ls = _ptrs(planes)
    n = lib().ffv1o_encode_frame(arr, ls, w, h, bits, hsub, vsub, nh, nv, out.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("encode overflow")
    return out[:n].tobytes()


def decode_frame(extra, pkt, w, h, bits, hsub, vsub):
    """Returns (rc, planes)."""
    dt = np.uint16 if bits > 8 else np.uint8
    cw, ch = -(-w >> hsub), -(-h >> vsub)
    planes = [np.zeros((h, w), dt), np.zeros((ch, cw), dt), np.zeros((ch, cw), dt)]
    arr, ls = _ptrs(planes)
    x = np.frombuffer(extra, np.uint8)
    p = np.frombuffer(pkt, np.uint8)
    rc = lib().ffv1o_decode_frame(x.ctypes.data, x.size, p.ctypes.data, p.size, w, h, arr, ls)
    return rc, planes


def crc(data):
    b = np.frombuffer(bytes(data), np.uint8)
    return lib().ffv1o_crc(0, b.ctypes.data, b.size)


# ---- general FFV1 v3 streams (ffv1_oracle.c "General FFV1 version 3") -------
GEN_MAX_TABLES = 8


class Prof(ctypes.Structure):
    """ffv1o_prof: what an FFmpeg-like encoder puts in the record and slices."""
    _fields_ = [("bits", ctypes.c_int), ("hsub", ctypes.c_int), ("vsub", ctypes.c_int), ("nh", ctypes.c_int),
                ("nv", ctypes.c_int), ("micro", ctypes.c_int), ("coder", ctypes.c_int), ("ntables", ctypes.c_int),
                ("ec", ctypes.c_int), ("intra", ctypes.c_int), ("gop", ctypes.c_int), ("tidx", ctypes.c_int * 2),
                ("trans", ctypes.c_uint8 * 256), ("levels", ctypes.c_uint8 * (GEN_MAX_TABLES * 5 * 128)),
                ("has_init", ctypes.c_uint8 * GEN_MAX_TABLES), ("init", ctypes.c_void_p * GEN_MAX_TABLES)]


def _runs(bounds):
    """Level of d = 0..127 from the first d of each level >= 1."""
    lv = np.zeros(128, np.uint8)
    for k, b in enumerate(bounds, 1):
        lv[b:] = k
    return lv


# Tables of the shape FFmpeg's ffv1enc.c uses (quant11 / quant5 for 8 bits,
# quant9_10bit / quant5_10bit above): the level boundaries restated from its
# published tables, unpinned (FFmpeg is absent here)
QUANT11 = _runs([1, 2, 5, 12, 28])
QUANT5 = _runs([1, 4])
QUANT9_10 = _runs([2, 6, 16, 48])
QUANT5_10 = _runs([3, 64])
ZERO = np.zeros(128, np.uint8)
PIXPATH3 = _runs([1, 2, 4, 8, 16])  # round 4's pixpath quantiser (min(5, bit length), 666 contexts)


def pixpath_quant(bits):
    """The 3-input quantiser pixpath's encoder writes at a bit depth
    (ffv1host.cpp ffv1_default_quant, ffv1_oracle.c oracle_quant)."""
    return _runs([4, 32]) if bits > 8 else _runs([1, 3, 8])


def pixpath_contexts(bits):
    return 63 if bits > 8 else 172


def ffmpeg_context1_sets(bits):
    """`-context 1`'s two table sets (ffv1enc.c encode_init): set 0 the
    3-input model, set 1 the 5-input one (the slices use set 1)."""
    a, b = (QUANT11, QUANT5) if bits <= 8 else (QUANT9_10, QUANT5_10)
    return [[a, a, a, ZERO, ZERO], [a, a, b, b, b]]


def rac_one_state(factor, max_p):
    """ff_build_rac_states(c, factor * 2^32, max_p)'s one_state (rangecoder.c)."""
    one = 1 << 32
    f = int(factor * (1 << 32))
    st = [0] * 256
    p, last = one // 2, 0
    for _ in range(128):
        p8 = (256 * p + one // 2) >> 32
        if p8 <= last:
            p8 = last + 1
        if last and last < 256 and p8 <= max_p:
            st[last] = p8
        p += ((one - p) * f + one // 2) >> 32
        last = p8
    for i in range(256 - max_p, max_p + 1):
        if st[i]:
            continue
        p = (i * one + 128) >> 8
        p += ((one - p) * f + one // 2) >> 32
        p8 = (256 * p + one // 2) >> 32
        p8 = i + 1 if p8 <= i else min(p8, max_p)
        st[i] = p8
    return st


def custom_states():
    """A transmitted state table (coder_type 2) for the tests: the default
    construction at another adaptation rate (0.04, max 250) with its unset
    ends filled (read_extra_header requires 1..255 everywhere).  FFmpeg's own
    table (ffv1enc.c ver2_state) is not available here."""
    t = rac_one_state(0.04, 256 - 6)
    return [0] + [t[i] if t[i] else min(255, i + 1) for i in range(1, 256)]


def context_count(levels5):
    cc = 1
    for lv in levels5:
        cc *= 2 * (int(lv.max()) + 1) - 1
    return (cc + 1) // 2


def make_prof(bits, hsub, vsub, nh, nv, sets, tidx=(1, 1), coder=2, trans=None, init=None, gop=12, ec=1, micro=4):
    """A Prof (and the buffers it points at, kept on the object).  sets: list
    of 5-table level lists; init: {set: uint8 [context_count, 32]}."""
    pf = Prof()
    pf.bits, pf.hsub, pf.vsub, pf.nh, pf.nv, pf.micro, pf.coder = bits, hsub, vsub, nh, nv, micro, coder
    pf.ntables, pf.ec, pf.gop = len(sets), ec, gop
    pf.intra = 1 if gop == 1 else 0
    pf.tidx[0], pf.tidx[1] = tidx
    if coder == 2:
        t = trans if trans is not None else custom_states()
        for i in range(256):
            pf.trans[i] = t[i]
    lv = np.zeros((GEN_MAX_TABLES, 5, 128), np.uint8)
    for i, s in enumerate(sets):
        for k in range(5):
            lv[i, k] = s[k]
    ctypes.memmove(pf.levels, lv.ctypes.data, lv.nbytes)
    pf._keep = []
    for i, arr in (init or {}).items():
        a = np.ascontiguousarray(arr, np.uint8)
        assert a.shape == (context_count(sets[i]), 32)
        pf.has_init[i] = 1
        pf.init[i] = a.ctypes.data
        pf._keep.append(a)
    return pf


def _glib():
    L = lib()
    if not hasattr(L, "_gen"):
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.ffv1o_gen_extradata.argtypes = [ctypes.POINTER(Prof), vp, i64]
        L.ffv1o_gen_extradata.restype = i64
        L.ffv1o_gen_encoder_create.argtypes = [ctypes.POINTER(Prof), i32, i32]
        L.ffv1o_gen_encoder_create.restype = vp
        L.ffv1o_gen_encoder_destroy.argtypes = [vp]
        L.ffv1o_gen_encode_frame.argtypes = [vp, vp, vp, vp, i64]
        L.ffv1o_gen_encode_frame.restype = i64
        L.ffv1o_gen_decoder_create.argtypes = [vp, i64, i32, i32, vp]
        L.ffv1o_gen_decoder_create.restype = vp
        L.ffv1o_gen_decoder_destroy.argtypes = [vp]
        L.ffv1o_gen_decode_frame.argtypes = [vp, vp, i64, vp, vp, vp]
        L.ffv1o_gen_decode_frame.restype = i32
        L._gen = True
    return L


def gen_extradata(pf):
    buf = np.zeros(1 << 22, np.uint8)
    n = _glib().ffv1o_gen_extradata(ctypes.byref(pf), buf.ctypes.data, buf.size)
    if n < 0:
        raise RuntimeError("gen_extradata")
    return buf[:n].tobytes()


class GenEncoder:
    """The oracle's FFmpeg-like sequence encoder (states carried across a GOP)."""

    def __init__(self, pf, w, h):
        self.pf, self.w, self.h = pf, w, h
        self.h_ = _glib().ffv1o_gen_encoder_create(ctypes.byref(pf), w, h)
        if not self.h_:
            raise ValueError("bad profile")

    def __del__(self):
        if getattr(self, "h_", None):
            _glib().ffv1o_gen_encoder_destroy(self.h_)
            self.h_ = None

    def encode(self, planes):
        planes = [np.ascontiguousarray(p) for p in planes]
        cap = sum(p.nbytes for p in planes) * 2 + 4096 + 64 * self.pf.nh * self.pf.nv
        out = np.zeros(cap, np.uint8)
        arr, ls = _ptrs(planes)
        n = _glib().ffv1o_gen_encode_frame(self.h_, arr, ls, out.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("encode overflow")
        return out[:n].tobytes()


GEN_INFO = ("version", "micro_version", "coder_type", "bits", "hsub", "vsub", "num_h_slices", "num_v_slices",
            "quant_table_sets", "ec", "intra", "context_count0", "context_count1", "initial_states0",
            "initial_states1", "crc_ok")


class GenDecoder:
    def __init__(self, extra, w, h):
        self.w, self.h = w, h
        info = (ctypes.c_int * 16)()
        x = np.frombuffer(extra, np.uint8)
        self.h_ = _glib().ffv1o_gen_decoder_create(x.ctypes.data, x.size, w, h, info)
        self.info = dict(zip(GEN_INFO, list(info)))
        if not self.h_:
            raise ValueError("record refused: %r" % self.info)

    def __del__(self):
        if getattr(self, "h_", None):
            _glib().ffv1o_gen_decoder_destroy(self.h_)
            self.h_ = None

    def decode(self, pkt):
        """(rc, planes, keyframe) of the next packet of the sequence."""
        bits, hs, vs = self.info["bits"], self.info["hsub"], self.info["vsub"]
        dt = np.uint16 if bits > 8 else np.uint8
        cw, ch = -(-self.w >> hs), -(-self.h >> vs)
        planes = [np.zeros((self.h, self.w), dt), np.zeros((ch, cw), dt), np.zeros((ch, cw), dt)]
        arr, ls = _ptrs(planes)
        p = np.frombuffer(pkt, np.uint8)
        key = ctypes.c_int()
        rc = _glib().ffv1o_gen_decode_frame(self.h_, p.ctypes.data, p.size, arr, ls, ctypes.byref(key))
        return rc, planes, key.value
