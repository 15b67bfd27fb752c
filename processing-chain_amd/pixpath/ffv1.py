"""FFV1 encoder of the AVPVS intermediate on the MI355X (SURVEY.md section 8f
row 1): the pixel stage's output in the bitstream the reference's
`-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1`
(lib/ffmpeg.py:993, :1047) produces -- FFV1 version 3, range coder, slice
CRCs -- encoded by libpixpath's ffv1_slice_kernel (one lane per slice).

Bitstream choices that differ from ffmpeg's encoder and the parity status
(unpinned: no FFV1 decoder exists in this container or on the GPU box; the
CPU restatement oracle/ffv1_oracle.c decodes it losslessly) are in DESIGN.md.
"""
import ctypes
import os
import queue
import threading

import numpy as np
import torch

from . import formats
from ._native import PP_COPY_D2D, PP_COPY_D2H, check, lib
from .ops import _stream, context


class Ffv1Encoder:
    def __init__(self, fmt, w, h, slices=(8, 8), max_frames=600, device=None, host_only=False):
        self.fmt = formats.fmt(fmt)
        self.w, self.h = int(w), int(h)
        self.slices = (int(slices[0]), int(slices[1]))
        self.max_frames = int(max_frames)
        self.ctx = None if host_only else context(device)
        h_ = ctypes.c_void_p()
        check(lib().pp_ffv1_encoder_create(None if host_only else self.ctx.handle, self.fmt.id, self.w, self.h,
                                           self.slices[0], self.slices[1], self.max_frames, ctypes.byref(h_)))
        self.handle = h_
        self.stages = None  # the AVI writer's staging batches, pooled with the encoder

    def __del__(self):
        if getattr(self, "handle", None):
            try:
                lib().pp_ffv1_encoder_destroy(self.handle)
            except Exception:
                pass
            self.handle = None

    @property
    def extradata(self):
        """The configuration record (codec private data of the AVI/MKV stream)."""
        n = check(lib().pp_ffv1_extradata(self.handle, None, 0))
        buf = (ctypes.c_uint8 * n)()
        check(lib().pp_ffv1_extradata(self.handle, buf, n))
        return bytes(buf)

    @property
    def memory_bytes(self):
        """Device bytes this encoder holds (tokens, records, context states, packets)."""
        v = ctypes.c_int64()
        check(lib().pp_ffv1_encoder_memory(self.handle, ctypes.byref(v)))
        return v.value

    @property
    def launches(self):
        """Launches of the last encode: 1, or more when a slice needed more
        renorm records than the per-slice budget and the batch was re-coded
        in halves (pp_ffv1_encode_packets)."""
        v = ctypes.c_int()
        check(lib().pp_ffv1_encode_stats(self.handle, ctypes.byref(v)))
        return v.value

    def reserve(self, packet_bytes):
        """Size the device packet buffer and the pinned host buffer of
        encode_host for `packet_bytes` of packets now (pinning ~2 GB of host
        memory takes ~0.2 s: a writer does it before its first PVS)."""
        check(lib().pp_ffv1_encoder_reserve(self.handle, int(packet_bytes)))
        if getattr(self, "_host", None) is None or self._host.numel() < packet_bytes:
            self._host = torch.empty(max(int(packet_bytes), 1 << 20), dtype=torch.uint8).pin_memory()

    def encode_packets(self, src, stream=None):
        """Encode a FrameBatch into the encoder's own device packet buffer:
        (device pointer, total bytes, numpy int64 frame sizes).  The packets
        are valid until the next encode.  Synchronises the stream."""
        if (src.fmt.id, src.w, src.h) != (self.fmt.id, self.w, self.h):
            raise ValueError("batch does not match the encoder")
        sizes = np.zeros(src.n, np.int64)
        s = src.frames_struct()
        ptr = ctypes.c_void_p()
        total = check(lib().pp_ffv1_encode_packets(self.handle, ctypes.byref(s), src.n,
                                                   sizes.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ptr),
                                                   _stream(src.planes[0], stream)))
        return ptr.value, total, sizes

    def encode(self, src, stream=None):
        """Encode a FrameBatch; returns (device uint8 tensor of the packets back to back,
        numpy int64 frame sizes).  Synchronises the stream."""
        ptr, total, sizes = self.encode_packets(src, stream)
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=src.device)
        if total:
            st = _stream(src.planes[0], stream)
            check(lib().pp_copy_async(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr), total, PP_COPY_D2D, st))
            check(lib().pp_stream_synchronize(st))
        return out[:total], sizes

    def packets_to_host(self, ptr, n, stream):
        """One D2H of the last encode's n packet bytes (device pointer ptr) into
        the encoder's pinned host buffer on `stream`; returns its numpy view
        (valid until the next call)."""
        if getattr(self, "_host", None) is None or self._host.numel() < n:
            self._host = torch.empty(max(n + n // 4, 1 << 20), dtype=torch.uint8).pin_memory()
        if n:
            st = ctypes.c_void_p(stream if isinstance(stream, int) else stream.cuda_stream)
            check(lib().pp_copy_async(ctypes.c_void_p(self._host.data_ptr()), ctypes.c_void_p(ptr), n, PP_COPY_D2H,
                                      st))
            check(lib().pp_stream_synchronize(st))
        return self._host[:n].numpy()

    def packets_to_host_chunks(self, ptr, n, sizes, stream, chunk=128 << 20):
        """The last encode's packets D2H in packet-aligned chunks of about
        `chunk` bytes, all queued at once on `stream`; yields (numpy view,
        frame sizes) of each chunk as its copy lands, so the caller writes
        chunk k while chunk k + 1 is still in flight (the views stay valid
        until the next call)."""
        if getattr(self, "_host", None) is None or self._host.numel() < n:
            self._host = torch.empty(max(n + n // 4, 1 << 20), dtype=torch.uint8).pin_memory()
        st = ctypes.c_void_p(stream.cuda_stream)
        parts, i0, b0, acc = [], 0, 0, 0
        for i, k in enumerate(sizes.tolist()):
            acc += k
            if acc - b0 >= chunk or i == len(sizes) - 1:
                parts.append((i0, i + 1, b0, acc))
                i0, b0 = i + 1, acc
        evs = []
        for _, _, lo, hi in parts:
            if hi > lo:
                check(lib().pp_copy_async(ctypes.c_void_p(self._host.data_ptr() + lo), ctypes.c_void_p(ptr + lo),
                                          hi - lo, PP_COPY_D2H, st))
            ev = torch.cuda.Event()
            ev.record(stream)
            evs.append(ev)
        host = self._host.numpy()
        try:
            for (a, b, lo, hi), ev in zip(parts, evs):
                ev.synchronize()
                yield host[lo:hi], sizes[a:b]
        finally:  # a walk abandoned by a failed write leaves no copy in flight into _host
            stream.synchronize()

    def encode_host(self, src, stream=None):
        """(numpy uint8 view of the packets in a pinned host buffer, frame sizes):
        encode, then one D2H of the packets straight from the encoder's packet
        buffer (valid until the next call)."""
        ptr, n, sizes = self.encode_packets(src, stream)
        st = stream if stream is not None else torch.cuda.current_stream(src.device)
        return self.packets_to_host(ptr, n, st), sizes

    def encode_to_host(self, src, stream=None):
        """List of per-frame packets (bytes)."""
        data, sizes = self.encode_host(src, stream)
        out, off = [], 0
        for n in sizes.tolist():
            out.append(data[off:off + n].tobytes())
            off += n
        return out


def default_slices():
    """The AVPVS writers' slice grid: PIXPATH_FFV1_SLICES ("HxV"), else 8x8."""
    import os
    v = os.environ.get("PIXPATH_FFV1_SLICES", "8x8").lower().split("x")
    if len(v) != 2 or not all(t.isdigit() and int(t) > 0 for t in v):
        raise ValueError("PIXPATH_FFV1_SLICES must be HxV, e.g. 16x16")
    return int(v[0]), int(v[1])


_POOL_LOCK = threading.Lock()
_POOL = {}  # (fmt, w, h, slices, max_frames, device) -> [idle Ffv1Encoder]


def _pool_key(fmt, w, h, slices, max_frames, device):
    return (formats.fmt(fmt).id, int(w), int(h), tuple(int(v) for v in slices), int(max_frames), int(device))


def acquire_encoder(fmt, w, h, slices=(8, 8), max_frames=600, device=None):
    """An idle encoder of this geometry from the process's pool, else a new
    one.  An encoder of a 600-frame 1080p yuv422p10le batch holds ~17 GB of
    HBM (tokens 10 GB, renorm records 5 GB, context states 1.6 GB, packets),
    plus the writer's staging batch (5 GB) that is pooled with it; consecutive
    PVSes of one process reuse them instead of allocating per PVS."""
    key = _pool_key(fmt, w, h, slices, max_frames, context(device).device)
    with _POOL_LOCK:
        idle = _POOL.get(key)
        if idle:
            return idle.pop()
    return Ffv1Encoder(fmt, w, h, slices=slices, max_frames=max_frames, device=device)


def take_idle_encoder(fmt, w, h, slices=(8, 8), max_frames=600, device=None):
    """An idle pooled encoder of this geometry, or None (nothing is allocated)."""
    key = _pool_key(fmt, w, h, slices, max_frames, context(device).device)
    with _POOL_LOCK:
        idle = _POOL.get(key)
        return idle.pop() if idle else None


def release_encoder(enc, ok=True):
    """Return an encoder from acquire_encoder() to the pool; one that failed
    mid-encode (ok=False) is freed instead."""
    if not ok:
        enc.stages = None
        return
    key = _pool_key(enc.fmt, enc.w, enc.h, enc.slices, enc.max_frames, enc.ctx.device)
    with _POOL_LOCK:
        _POOL.setdefault(key, []).append(enc)


def reserve_encoders(fmt, w, h, count, slices=(8, 8), max_frames=600, device=None, stages=1):
    """Make the pool hold at least `count` idle encoders of this geometry, each
    with `stages` staging batches -- the writers of that many PVSes in flight
    then allocate nothing (`cli` and the bench call this before their first
    PVS).  Returns the number created."""
    from .frames import FrameBatch
    key = _pool_key(fmt, w, h, slices, max_frames, context(device).device)
    with _POOL_LOCK:
        have = len(_POOL.get(key, []))
    made = []
    for _ in range(max(0, count - have)):
        made.append(Ffv1Encoder(fmt, w, h, slices=slices, max_frames=max_frames, device=device))
    with _POOL_LOCK:
        idle = _POOL.setdefault(key, [])
        idle.extend(made)
        encs = list(idle)
    fb = formats.frame_bytes(formats.fmt(fmt), w, h)
    for enc in encs:
        st = getattr(enc, "stages", None) or []
        while len(st) < stages:
            st.append(FrameBatch.interleaved(enc.fmt, enc.w, enc.h, enc.max_frames,
                                             device=torch.device("cuda", enc.ctx.device)))
        enc.stages = st
        # packets of a full batch at 2:1 (video content codes at 2-5:1); a
        # batch that codes larger grows the buffers in its encode
        enc.reserve(enc.max_frames * fb // 2)
    return len(made)


def reserve_writers(fmt, w, h, count, slices=(8, 8), batch=600, device=None, split=None):
    """reserve_encoders for `count` AVPVS writers (Ffv1AviWriter) of `batch`
    frames in flight at once.  split = K: count x K encoders of ceil(batch / K)
    frames, one staging batch each.  split None (the writers' default, see
    writer_split): the first writer codes alone on the device and takes
    default_split() lanes, the other count - 1 open while it is still open and
    take one encoder of the whole batch; PIXPATH_FFV1_SPLIT set forces K for
    every writer."""
    made = 0
    if split is None and not os.environ.get("PIXPATH_FFV1_SPLIT"):
        k = default_split()
        made += reserve_encoders(fmt, w, h, k, slices=slices, max_frames=-(-int(batch) // k), device=device,
                                 stages=1)
        if count > 1:
            made += reserve_encoders(fmt, w, h, count - 1, slices=slices, max_frames=int(batch), device=device,
                                     stages=1)
        return made
    k = default_split() if split is None else max(1, int(split))
    sub = -(-int(batch) // k)
    return reserve_encoders(fmt, w, h, count * k, slices=slices, max_frames=sub, device=device, stages=1)


def clear_pool():
    """Free every idle pooled encoder (and its staging batches)."""
    with _POOL_LOCK:
        _POOL.clear()


class Ffv1Decoder:
    """FFV1 v3 decoder on the GPU (one lane per slice and GOP): the AVPVS read
    back for the CPVS stage -- pixpath's intra streams and FFmpeg's
    `-level 3 -coder 1 -context 1` ones (transmitted state table, 5-input
    context sets, GOPs with carried states).  ``decode(packets, sizes)`` takes
    consecutive frame packets back to back in host memory and returns a
    FrameBatch in HBM; a call that starts inside a GOP continues the previous
    call's states (``reset()`` after a seek)."""

    def __init__(self, extradata, w, h, max_frames=600, device=None, host_only=False):
        self.w, self.h, self.max_frames = int(w), int(h), int(max_frames)
        self.ctx = None if host_only else context(device)
        buf = (ctypes.c_uint8 * len(extradata)).from_buffer_copy(extradata)
        h_ = ctypes.c_void_p()
        check(lib().pp_ffv1_decoder_create(None if host_only else self.ctx.handle, buf, len(extradata), self.w,
                                           self.h, self.max_frames, ctypes.byref(h_)))
        self.handle = h_
        fid = check(lib().pp_ffv1_decoder_format(h_))
        self.fmt = formats.fmt(fid)
        nh, nv = ctypes.c_int(), ctypes.c_int()
        check(lib().pp_ffv1_decoder_slices(h_, ctypes.byref(nh), ctypes.byref(nv)))
        self.slices = (nh.value, nv.value)
        lpw, cap = ctypes.c_int(), ctypes.c_int()
        check(lib().pp_ffv1_decoder_geometry(h_, ctypes.byref(lpw), ctypes.byref(cap)))
        self.slices_per_workgroup, self.row_cap = lpw.value, cap.value
        info = (ctypes.c_int * 8)()
        n = check(lib().pp_ffv1_decoder_info(h_, info, 8))
        self.info = dict(zip(("micro_version", "coder_type", "quant_table_sets", "max_contexts", "intra", "ec",
                              "initial_states_mask", "pixpath_tables"), list(info)[:n]))

    def reset(self):
        """Forget the carried GOP states (the next decode must start at a keyframe)."""
        check(lib().pp_ffv1_decoder_reset(self.handle))

    def __del__(self):
        if getattr(self, "handle", None):
            try:
                lib().pp_ffv1_decoder_destroy(self.handle)
            except Exception:
                pass
            self.handle = None

    def decode(self, packets, sizes, dst=None, stream=None):
        from .frames import FrameBatch
        if isinstance(packets, np.ndarray):
            data = np.ascontiguousarray(packets, dtype=np.uint8)
        else:
            data = np.frombuffer(bytes(packets) if not isinstance(packets, (bytes, bytearray)) else packets, np.uint8)
        sizes = np.ascontiguousarray(sizes, dtype=np.int64)
        n = len(sizes)
        if dst is None:
            dst = FrameBatch(self.fmt, self.w, self.h, n, device=torch.device("cuda", self.ctx.device))
        s = dst.frames_struct()
        check(lib().pp_ffv1_decode(self.handle, data.ctypes.data_as(ctypes.c_void_p),
                                   sizes.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(s),
                                   _stream(dst.planes[0], stream)))
        return dst


def decode_group(decoders, packets, sizes, dst=None, stream=None):
    """One GPU launch over several streams of one configuration record
    (pp_ffv1_decode_group): decoders[k] decodes packets[k] (frame packets back
    to back in host memory, sizes[k] each) and keeps its own carried GOP
    states.  Returns the device FrameBatch of all streams' frames, stream k's
    at [sum(len(sizes[:k])), ...).  An FFmpeg-made AVPVS (GOP 12, 2x2 slices)
    has 200 slice chains per 600 frames, one GPU lane each, so one stream
    alone leaves the GPU almost idle; several side by side fill it."""
    from .frames import FrameBatch
    n = len(decoders)
    if n == 0 or len(packets) != n or len(sizes) != n:
        raise ValueError("decode_group: one packet buffer and size list per decoder")
    d0 = decoders[0]
    datas = []
    for pk in packets:
        if isinstance(pk, np.ndarray):
            datas.append(np.ascontiguousarray(pk, dtype=np.uint8))
        else:
            datas.append(np.frombuffer(bytes(pk) if not isinstance(pk, (bytes, bytearray)) else pk, np.uint8))
    szs = [np.ascontiguousarray(s_, dtype=np.int64) for s_ in sizes]
    counts = [len(s_) for s_ in szs]
    total = sum(counts)
    if dst is None:
        dst = FrameBatch(d0.fmt, d0.w, d0.h, total, device=torch.device("cuda", d0.ctx.device))
    elif dst.n < total:
        raise ValueError("decode_group: dst holds %d frames, the streams %d" % (dst.n, total))
    handles = (ctypes.c_void_p * n)(*[d.handle.value for d in decoders])
    pptr = (ctypes.c_void_p * n)(*[d_.ctypes.data for d_ in datas])
    sptr = (ctypes.c_void_p * n)(*[s_.ctypes.data for s_ in szs])
    nfr = (ctypes.c_int * n)(*counts)
    s = dst.frames_struct()
    check(lib().pp_ffv1_decode_group(handles, n, pptr, sptr, nfr, ctypes.byref(s), _stream(dst.planes[0], stream)))
    return dst


_DEV_LOCK = threading.Lock()
_DEV_STATE = {}  # device index -> (encode lock, encode stream, host-upload stream, packet D2H stream)


def _device_state(device):
    """One encode lock and one pair of streams per device and process, shared
    by every AVI writer: the writers' encodes run one at a time on one stream.
    Concurrent encodes from writer threads measured slower than serial ones
    beside a running scale pipeline (e2e_avpvs: 0.58 s per 600-frame encode
    when two overlap vs 0.19 s alone), and every extra stream shares one of
    the process's few hardware queues with the pipeline's."""
    with _DEV_LOCK:
        st = _DEV_STATE.get(device)
        if st is None:
            dev = torch.device("cuda", device)
            st = _DEV_STATE[device] = (threading.Lock(), torch.cuda.Stream(dev), torch.cuda.Stream(dev),
                                       torch.cuda.Stream(dev))
        return st


_SEMS = {}  # (device, lanes) -> semaphore of the encoder lanes' encodes


def _lane_semaphore(device, lanes):
    """At most `lanes` lane encodes at once on a device, over every writer of
    the process: the K sub-batches of one writer code side by side (K x 1/K of
    a batch is one batch's worth of slice chains), while the lanes of several
    writers queue as whole batches did under the shared encode lock
    (concurrent full-batch encodes measured slower than serial ones, see
    _device_state)."""
    with _DEV_LOCK:
        s = _SEMS.get((device, lanes))
        if s is None:
            s = _SEMS[(device, lanes)] = threading.BoundedSemaphore(lanes)
        return s


def provenance(slices):
    """The encoder tag written into the AVPVS (RIFF INFO ISFT) and echoed in
    the GPU command string p03 logs as `ffmpegCommand:` (p03_generateAvPvs.py:41-59)."""
    return "pixpath ffv1-gpu v3 intra %dx%d slices" % (int(slices[0]), int(slices[1]))


def default_split():
    """Encoders of an AVPVS writer that codes alone on its device (writer_split;
    PIXPATH_FFV1_SPLIT, default 2, forces it for every writer): the 600-frame
    batch of a PVS is coded as that many sub-batches, each on its own encoder,
    stream and worker thread, so the first half's encode starts while the
    pipeline still scales the second half, the halves code side by side (one
    600-frame encode leaves ~40 % of the SIMDs idle: 600 waves for 1,024), and
    the first half's packets are written to the AVI while the second half
    codes.  1 restores one encoder and one encode per batch."""
    v = os.environ.get("PIXPATH_FFV1_SPLIT", "2")
    if not v.isdigit() or not 1 <= int(v) <= 8:
        raise ValueError("PIXPATH_FFV1_SPLIT must be 1..8")
    return int(v)


_OPEN_LOCK = threading.Lock()
_OPEN = {}  # device -> AVPVS writers open on it


def writer_split(device, opened=None):
    """Encoder lanes for a new AVPVS writer on `device`: PIXPATH_FFV1_SPLIT when
    set, else default_split() when no other writer is open on the device (one
    PVS coding alone leaves SIMDs idle, which the lanes fill) and 1 when others
    are (their encodes fill the device already: on MI355X, 4 PVSes in flight
    code at 3.0k fps with one encoder each but 2.2-2.5k fps with two lanes each
    -- 8 encode streams on 4 hardware queues, profiles/r6/ab/README.md).
    `opened`: writers open on the device (default: the live count)."""
    if os.environ.get("PIXPATH_FFV1_SPLIT"):
        return default_split()
    if opened is None:
        with _OPEN_LOCK:
            opened = _OPEN.get(int(device), 0)
    return default_split() if opened == 0 else 1


class Ffv1AviWriter:
    """`cli avpvs --gpu-ffv1`: the AVPVS written as FFV1 encoded on the GPU in
    an AVI (pixpath.avi) -- the `-c:v ffv1 ... <pvs>.avi` of lib/ffmpeg.py:993
    without ffmpeg's encoder.

    Frames accumulate in HBM -- straight from the pipeline's device output
    (``write_device``: no D2H, no re-upload) or from host frames (``write``) --
    into batches of ``batch`` frames (default 600, a 10 s PVS at 60 fps: the
    encoder's parallelism is frames x slices).  With ``split`` = 1 a full batch
    is encoded by a worker thread on its own stream while the next batch fills
    (a second staging batch, allocated only when a PVS has more than one
    batch), its packets come back in one pinned D2H and go into the AVI.  With
    ``split`` = K > 1 (writer_split: 2 when the writer codes alone on the
    device) the batch is K sub-batches
    on K encoder LANES -- each lane its own encoder, staging batch, streams and
    worker thread -- submitted as each fills: the lanes' encodes overlap the
    pipeline and each other, and a lane writes its packets as soon as the
    lanes before it in frame order have written theirs.  The encoders and
    their staging batches come from the process's pool (acquire_encoder)."""

    def __init__(self, path, fmt, w, h, rate, slices=None, batch=600, device=None, shared=True, split=None):
        """slices: the FFV1 slice grid (default PIXPATH_FFV1_SLICES, else 8x8;
        16x16 encodes ~1.3x faster at ~7 % larger files).
        shared (split = 1 only): encode on the device's shared stream under
        its encode lock (_device_state); False gives the writer its own
        streams and lets its encodes overlap other writers' (bench comparison
        only).  split: encoder lanes (default writer_split(device))."""
        import time
        from . import avi
        t0 = time.perf_counter()
        if slices is None:
            slices = default_slices()
        self.fmt = formats.fmt(fmt)
        self._open_dev = None
        if split is None:
            split = writer_split(context(device).device)
        self.w, self.h = int(w), int(h)
        self.fb = formats.frame_bytes(self.fmt, w, h)
        self.batch = int(batch)
        self.K = max(1, min(int(split), self.batch))
        self.sub = -(-self.batch // self.K)  # frames per sub-batch (lane batch)
        self.encs = [acquire_encoder(self.fmt, w, h, slices=slices, max_frames=self.sub, device=device)
                     for _ in range(self.K)]
        self.enc = self.encs[0]
        self.device = torch.device("cuda", self.enc.ctx.device)
        for e in self.encs:
            if e.stages is None:
                e.stages = []
        # staging slots: split = 1 double-buffers on the one encoder (slots 0, 1),
        # else one slot per lane; slot s is coded by encoder lane_of[s]
        self.nslots = 2 if self.K == 1 else self.K
        self.lane_of = [0, 0] if self.K == 1 else list(range(self.K))
        self._stage(0)
        self.free = [threading.Event() for _ in range(self.nslots)]
        for e in self.free:
            e.set()
        self.cur, self.fill = 0, 0
        self.free[0].clear()
        self.claimed = True  # slot 0 is this writer's from the start
        if shared and self.K == 1:
            lock, st, self.put_stream, d2h = _device_state(self.device.index)
            self.lanes = [(lock, st, d2h)]
        else:
            self.put_stream = torch.cuda.Stream(self.device)  # host-frame uploads
            sem = _lane_semaphore(self.device.index, self.K) if shared else threading.BoundedSemaphore(self.K)
            self.lanes = [(sem, torch.cuda.Stream(self.device), torch.cuda.Stream(self.device))
                          for _ in range(self.K)]
        self.stream, self.d2h_stream = self.lanes[0][1], self.lanes[0][2]
        self.avi = avi.AviWriter(path, w, h, rate, extradata=self.enc.extradata,
                                 info={b"ISFT": provenance(self.enc.slices).encode()})
        self.frames = 0
        # worker-thread time per part; setup_s: encoder + staging + file open (0 allocations when pooled)
        self.stats = {"encode_s": 0.0, "write_s": 0.0, "bytes": 0, "launches": 0, "lanes": self.K,
                      "setup_s": time.perf_counter() - t0, "timeline": []}
        self.last_stream = self.put_stream
        self.seq = 0          # sub-batches submitted
        self.turn = 0         # the next sub-batch (in frame order) whose packets go into the AVI
        self.turn_cv = threading.Condition()
        self.err = []
        self.qs = [queue.Queue() for _ in range(self.K)]
        self.ths = [threading.Thread(target=self._work, args=(k,), daemon=True) for k in range(self.K)]
        for t in self.ths:
            t.start()
        with _OPEN_LOCK:  # counted open until close(): writers made meanwhile take one lane
            self._open_dev = self.device.index
            _OPEN[self._open_dev] = _OPEN.get(self._open_dev, 0) + 1

    def _stage(self, slot):
        from .frames import FrameBatch
        enc = self.encs[self.lane_of[slot]]
        k = slot if self.K == 1 else 0
        st = enc.stages
        while len(st) <= k:
            st.append(FrameBatch.interleaved(self.fmt, self.w, self.h, self.sub, device=self.device))
        return st[k]

    def _work(self, lane):
        import time
        from .frames import FrameBatch
        enc = self.encs[lane]
        lock, stream, d2h = self.lanes[lane]
        while True:
            item = self.qs[lane].get()
            if item is None:
                return
            slot, n, ev, t_q, seq = item
            mine = released = False
            try:
                if self.err:
                    # after a failure: still wait for this batch's copies into the
                    # staging batch (queued on the caller's stream) before close()
                    # drops the stages back to the allocator
                    ev.synchronize()
                else:
                    t_w = time.perf_counter()
                    stream.wait_event(ev)
                    ev.synchronize()  # the frames of this batch are in the staging batch
                    src = FrameBatch.interleaved(self.fmt, self.w, self.h, n, device=self.device,
                                                 storage=self._stage(slot).storage[:n])
                    # split = 1: the device's encodes one at a time, on its encode
                    # stream; lanes: at most K lane encodes at once on the device
                    with lock:
                        t0 = time.perf_counter()
                        with torch.cuda.stream(stream):
                            ptr, n, sizes = enc.encode_packets(src, stream=stream)
                    released = True  # the staging batch is read: the next sub-batch may fill it
                    self.free[slot].set()
                    # the packets leave on the D2H stream, outside the lock: the next
                    # writer's encode starts while this D2H runs, and no writer's host
                    # upload (put_stream, synchronised per upload) waits behind it
                    # (ADVICE r4); the D2H waits for the encode on its stream
                    d2h.wait_stream(stream)
                    t1 = time.perf_counter()
                    # the AVI takes the sub-batches in frame order
                    with self.turn_cv:
                        while self.turn != seq and not self.err:
                            self.turn_cv.wait()
                        mine = not self.err
                    if mine:
                        t_t = time.perf_counter()
                        # packets D2H in chunks, each written to the AVI as it lands
                        # (the copy of chunk k + 1 overlaps the write of chunk k)
                        for data, part in enc.packets_to_host_chunks(ptr, n, sizes, d2h):
                            self.avi.write_packets(data, part)
                        t2 = time.perf_counter()
                        self.stats["encode_s"] += t1 - t0
                        self.stats["write_s"] += t2 - t_t
                        self.stats["bytes"] += int(sizes.sum())
                        self.stats["launches"] += enc.launches
                        # timeline (perf_counter): batch queued, worker picked it up,
                        # its frames ready on the GPU, packets on the host, packets written
                        self.stats["timeline"].append((t_q, t_w, t0, t1, t2))
            except Exception as e:  # surfaced by the next write / close
                self.err.append(e)
                # a failed AVI write abandons packets_to_host_chunks with later
                # chunks' D2H copies still queued into the pinned buffer: drain
                # them before the encoder (and that buffer) can be released or
                # reused
                try:
                    d2h.synchronize()
                except Exception:
                    pass
            finally:
                if not released:  # once per item: the slot may already hold the next sub-batch
                    self.free[slot].set()
                with self.turn_cv:
                    if mine or self.err:
                        self.turn = max(self.turn, seq + 1)
                    self.turn_cv.notify_all()

    def _check(self):
        if self.err:
            raise self.err[0]

    def _submit(self, stream):
        import time
        ev = torch.cuda.Event()
        ev.record(stream)
        self.qs[self.lane_of[self.cur]].put((self.cur, self.fill, ev, time.perf_counter(), self.seq))
        self.seq += 1
        self.cur = (self.cur + 1) % self.nslots
        # the next slot is claimed when its first frames arrive (_claim), not
        # here: after a batch's last sub-batch the caller goes on (the next
        # PVS's pipeline) instead of waiting for lane 0's encode to free it
        self.claimed = False
        self.fill = 0
        self._check()

    def _claim(self):
        if not self.claimed:
            self.free[self.cur].wait()
            self.free[self.cur].clear()
            self.claimed = True
            self._check()

    def _put(self, rows, stream):
        """Append device frames (uint8 rows [k, frame_bytes]) on `stream`."""
        k, i = rows.shape[0], 0
        while i < k:
            self._claim()
            take = min(k - i, self.sub - self.fill)
            stage = self._stage(self.cur)
            with torch.cuda.stream(stream):
                stage.storage[self.fill:self.fill + take].copy_(rows[i:i + take], non_blocking=True)
            self.fill += take
            self.frames += take
            i += take
            self.last_stream = stream
            if self.fill == self.sub:
                self._submit(stream)
        if stream is self.put_stream:  # host uploads complete before any event on another stream
            stream.synchronize()

    def write_device(self, frames, stream=None, emit=None):
        """Append a device FrameBatch (interleaved) in order; ``emit[i]``: how
        many times frame i is written (vf_fps duplicates / drops)."""
        self._check()
        stream = stream or torch.cuda.current_stream(self.device)
        rows = frames.storage[:frames.n]
        if emit is None:
            self._put(rows, stream)
            return
        i, n = 0, len(emit)
        while i < n:  # runs of single frames go in one copy
            j = i
            while j < n and emit[j] == 1:
                j += 1
            if j > i:
                self._put(rows[i:j], stream)
                i = j
                continue
            for _ in range(emit[i]):
                self._put(rows[i:i + 1], stream)
            i += 1

    def write(self, frames_u8):
        """Append dense host frames."""
        data = np.frombuffer(memoryview(frames_u8).cast("B"), np.uint8)
        n = len(data) // self.fb
        if n == 0:
            return
        with torch.cuda.stream(self.put_stream):
            d = torch.from_numpy(data[:n * self.fb].reshape(n, self.fb)).to(self.device, non_blocking=False)
        self._put(d, self.put_stream)

    def release(self, ok=True):
        """After close(): the encoders and their staging batches go back to the
        pool (freed instead when the encode failed)."""
        for e in self.encs or []:
            release_encoder(e, ok=ok)
        self.encs = []
        self.enc = None

    def close(self):
        """Encode what is left, finish the AVI and rename it into place; on any
        failure the partial file is removed and the error re-raised."""
        ok = False
        try:
            if self.fill:
                import time
                ev = torch.cuda.Event()
                ev.record(self.last_stream)
                self.qs[self.lane_of[self.cur]].put((self.cur, self.fill, ev, time.perf_counter(), self.seq))
                self.seq += 1
                self.fill = 0
            for q in self.qs:
                q.put(None)
            for t in self.ths:
                t.join()
            self._check()
            self.avi.close()
            ok = True
            import time
            self.stats["closed_at"] = time.perf_counter()
        finally:
            if not ok:
                self.avi.abort()
                try:  # copies into the staging batch still queued on the caller's stream,
                    self.last_stream.synchronize()  # packet D2H copies on the D2H streams
                    for _, _, d2h in self.lanes:
                        d2h.synchronize()
                except Exception:
                    pass
            self.release(ok)
            self._closed()

    def _closed(self):
        dev, self._open_dev = self._open_dev, None
        if dev is not None:
            with _OPEN_LOCK:
                _OPEN[dev] = max(0, _OPEN.get(dev, 0) - 1)


class Ffv1AviReader:
    """`cli cpvs --gpu-ffv1`: an FFV1 AVI (as Ffv1AviWriter writes it) read
    back through the GPU decoder; the reader interface of pixpath.io.  Only
    the packet index is held (pixpath.avi.scan); each batch's packets are read
    from the file when that batch is decoded, so a long-test AVPVS of tens of
    GB never sits in host memory."""

    def __init__(self, path, batch=600, device=None, scanned=None):
        """batch: frames decoded per launch (the decoder's parallelism is
        frames x slices, so a whole 10-s PVS at once); scanned: avi.scan(path)
        when the caller already has it."""
        from . import avi
        info, self.index = scanned if scanned is not None else avi.scan(path)
        if info.get("fourcc") != b"FFV1":
            raise ValueError("%s: not an FFV1 AVI" % path)
        self.w, self.h, self.rate = info["w"], info["h"], info["rate"]
        self.batch = int(batch)
        self.dec = Ffv1Decoder(info["extradata"], self.w, self.h, max_frames=self.batch, device=device)
        self.fmt = self.dec.fmt
        self.pos = 0
        self.fh = open(path, "rb")
        self._cache, self._cpos = None, 0  # decoded frames not yet handed out (read_device)

    @property
    def frame_bytes(self):
        return formats.frame_bytes(self.fmt, self.w, self.h)

    def __len__(self):
        return len(self.index)

    def _pinned(self, n):
        """A page-locked host buffer of >= n bytes (reused): the decoder's H2D
        of the packets then runs at DMA speed instead of through the driver's
        pageable staging copy."""
        if getattr(self, "_pin", None) is None or self._pin.numel() < n:
            self._pin = torch.empty(max(int(n * 1.25), 1 << 20), dtype=torch.uint8).pin_memory()
        return self._pin.numpy()

    def _read(self, i, m):
        """Packets i..i+m-1 back to back (read straight into a pinned buffer)
        and their sizes."""
        ent = self.index[i:i + m]
        lo, hi = ent[0][0], ent[-1][0] + ent[-1][1]
        sizes = np.array([s for _, s in ent], np.int64)
        total = int(sizes.sum())
        buf = self._pinned(hi - lo)
        self.fh.seek(lo)
        got = self.fh.readinto(memoryview(buf)[:hi - lo])
        if got != hi - lo:
            raise ValueError("%s: truncated packet data" % self.fh.name)
        if hi - lo == total:
            return buf[:total], sizes
        # chunk headers between the packets: close the gaps in place (moving left)
        w = 0
        for o, s in ent:
            buf[w:w + s] = buf[o - lo:o - lo + s]
            w += s
        return buf[:total], sizes

    def read_device(self, n):
        """Up to n decoded frames as an interleaved device FrameBatch (None at
        the end).  Frames are decoded `batch` at a time into one device buffer
        and handed out as views of it: a view is valid until the next call."""
        from .frames import FrameBatch
        if self._cache is None or self._cpos >= self._cache.n:
            self._cache = self._decode(self.batch)
            self._cpos = 0
            if self._cache is None:
                return None
        k = min(n, self._cache.n - self._cpos)
        out = FrameBatch.interleaved(self.fmt, self.w, self.h, k, device=self._cache.device,
                                     storage=self._cache.storage[self._cpos:self._cpos + k])
        self._cpos += k
        return out

    def _decode(self, n):
        """Decode the next up to n packets into a (reused) device batch."""
        from .frames import FrameBatch
        k = min(n, len(self.index) - self.pos)
        if k <= 0:
            return None
        if getattr(self, "_dbuf", None) is None:
            self._dbuf = FrameBatch.interleaved(self.fmt, self.w, self.h, self.batch,
                                                device=torch.device("cuda", self.dec.ctx.device))
        out = FrameBatch.interleaved(self.fmt, self.w, self.h, k, device=self._dbuf.device,
                                     storage=self._dbuf.storage[:k])
        done = 0
        while done < k:
            m = min(self.batch, k - done)
            data, sizes = self._read(self.pos, m)
            part = FrameBatch.interleaved(self.fmt, self.w, self.h, m, device=out.device,
                                          storage=out.storage[done:done + m])
            self.dec.decode(data, sizes, dst=part)
            self.pos += m
            done += m
        return out

    def read_into(self, buf, n):
        """Decode up to n frames into the dense host array buf [n, frame_bytes]; returns the count."""
        done = 0
        while done < n:
            out = self.read_device(n - done)
            if out is None:
                break
            k = out.n
            buf[done:done + k] = out.storage[:k].cpu().numpy()
            done += k
        return done

    def close(self):
        self.fh.close()


def is_pixpath_ffv1(info):
    """True when an AVI's video stream (avi.scan info) is FFV1 with exactly the
    configuration record pixpath's encoder writes for its format, size and
    slice grid -- the streams the GPU decoder reads.  FFmpeg's own FFV1
    (`-coder 1 -context 1`: custom state table, 5-input contexts, inter
    frames) is not, and neither is any other record."""
    from ._native import PixpathError
    if info.get("fourcc") != b"FFV1" or not info.get("extradata") or "w" not in info:
        return False
    try:
        dec = Ffv1Decoder(info["extradata"], info["w"], info["h"], max_frames=1, host_only=True)
        probe = Ffv1Encoder(dec.fmt, info["w"], info["h"], slices=dec.slices, host_only=True)
    except (PixpathError, ValueError):
        return False
    return probe.extradata == info["extradata"]


def packet_is_keyframe(pkt):
    """The keyframe flag of an FFV1 frame packet: the first decision of its
    first slice's range coder at state 128 (ffv1dec.c decode_frame), i.e. the
    first two bytes as a 16-bit value (clamped to 0xFF00) >= 0x7F80."""
    low = (pkt[0] << 8) | pkt[1] if len(pkt) >= 2 else 0
    return min(low, 0xFF00) >= 0x7F80


def gpu_decodable(info):
    """True when the GPU decoder reads an AVI's video stream (avi.scan info):
    FFV1 whose configuration record pp_ffv1_decoder_create accepts -- pixpath's
    own, and FFmpeg's `-level 3 -coder 1 -context 1 -slicecrc 1` AVPVS
    (lib/ffmpeg.py:993, :1047) with its custom state table, 5-input contexts
    and GOPs, at 8 or 10 bits, 4:2:0 / 4:2:2 / 4:4:4."""
    from ._native import PixpathError
    if info.get("fourcc") != b"FFV1" or not info.get("extradata") or "w" not in info:
        return False
    try:
        Ffv1Decoder(info["extradata"], info["w"], info["h"], max_frames=1, host_only=True)
    except (PixpathError, ValueError):
        return False
    return True


def decoder_route(info, have_ffmpeg=None):
    """Which decoder reads an AVI's video stream (avi.scan info): "gpu" or
    "ffmpeg".

    - pixpath's own intra FFV1 (and any intra record the GPU decoder reads):
      the GPU -- frames x slices chains (38,400 per 600 frames at 8x8).
    - An FFmpeg-made FFV1 with GOPs (the reference's own AVPVS,
      `-threads 4 -level 3 -coder 1 -context 1`, lib/ffmpeg.py:993, :1047):
      one stream has 200 serial chains per 600 frames, one GPU lane each, and
      decodes slower on the GPU than on the host's cores (bench
      `reference_stream_decode`), so ffmpeg's decoder takes it when ffmpeg
      exists; the GPU otherwise.  Several such streams decoded together
      (decode_group) do fill the GPU.  Parity of the GPU path on FFmpeg's own
      files is unpinned (no FFmpeg-made FFV1 file exists here; the general
      decoder is checked against oracle/ffv1_oracle.c's general restatement).
    - PIXPATH_FFV1_DECODE=gpu|ffmpeg forces one for every stream the GPU
      decoder reads; PIXPATH_FFV1=ffmpeg (ffmpeg's FFV1 encoder in the gpu
      backend) also sends records not written by pixpath to ffmpeg.
    - Anything the GPU decoder refuses: ffmpeg."""
    import shutil
    if not gpu_decodable(info):
        return "ffmpeg"
    force = os.environ.get("PIXPATH_FFV1_DECODE", "").lower()
    if force in ("gpu", "ffmpeg"):
        return force
    own = is_pixpath_ffv1(info)
    if not own and os.environ.get("PIXPATH_FFV1", "").lower() == "ffmpeg":
        return "ffmpeg"
    if own:
        return "gpu"
    dec = Ffv1Decoder(info["extradata"], info["w"], info["h"], max_frames=1, host_only=True)
    if dec.info.get("intra"):
        return "gpu"
    if have_ffmpeg is None:
        have_ffmpeg = shutil.which("ffmpeg") is not None
    return "ffmpeg" if have_ffmpeg else "gpu"


def open_avpvs_reader(path, device=None, batch=600):
    """The reader of an AVPVS: the GPU FFV1 decoder (Ffv1AviReader) or
    ffmpeg's decoder through pixpath.io, as decoder_route decides."""
    from . import avi, io as pio
    if path.lower().endswith(".avi") and os.path.isfile(path):
        scanned = avi.scan(path)
        if decoder_route(scanned[0]) == "gpu":
            return Ffv1AviReader(path, batch=batch, device=device, scanned=scanned)
    return pio.open_reader(path)


def stall_avi(src_path, dst_path, buffer_events, skipping, spinner_path=None, black_frame=True, device=None):
    """PP-STALL-1 (the bufferer step, p03_generateAvPvs.py:236-243) on an
    all-intra FFV1 AVI written by Ffv1AviWriter, at the PACKET level: every
    output frame that is an input frame (pass-through, or a frozen copy with
    --skipping) is that frame's packet copied from the input file -- no decode,
    no encode; only the stall frames (frozen / black frame + spinner) are
    composed on the GPU, from the few source frames decoded for them, and
    FFV1-encoded with the input's own configuration.  Returns the output frame
    count, or None when the input's configuration record is not this
    encoder's (then the caller decodes and re-encodes every frame)."""
    from . import avi, ops, spinner, stall
    from .frames import FrameBatch
    info, index = avi.scan(src_path)
    if not is_pixpath_ffv1(info):
        return None
    rate, w, h = info["rate"], info["w"], info["h"]
    dec = Ffv1Decoder(info["extradata"], w, h, max_frames=1, device=device)
    delays = None
    if not skipping:
        anim, delays = spinner.load_apng(spinner_path)
    seq = stall.stall_schedule(buffer_events, rate, len(index), skipping, delays, black_frame)
    compose = [(s, sp) for s, sp in seq if sp >= 0 or s < 0]
    dev = torch.device("cuda", dec.ctx.device)
    packets = []
    with open(src_path, "rb") as fh:
        def packet(i):
            off, size = index[i]
            fh.seek(off)
            return fh.read(size)
        if compose:
            ops.spinner_upload(anim, dec.fmt, device=dev.index)
            srcs = sorted({s for s, _ in compose if s >= 0})
            pos = {s: k for k, s in enumerate(srcs)}
            sb = FrameBatch.interleaved(dec.fmt, w, h, max(1, len(srcs)), device=dev)
            for k, s in enumerate(srcs):  # one packet per distinct stall source (the frame before each stall)
                pk = packet(s)
                dec.decode(pk, [len(pk)], dst=FrameBatch.interleaved(dec.fmt, w, h, 1, device=dev,
                                                                      storage=sb.storage[k:k + 1]))
            # the process's idle pooled 600-frame encoder (the AVPVS writer's, when
            # the stall pass follows it in the same process) and its staging
            # batch; else an encoder sized to the stall frames (a `cli stall`
            # process composes a handful: ~22 GB for 600 frames would be wasted)
            enc = take_idle_encoder(dec.fmt, w, h, slices=dec.slices, max_frames=600, device=dev.index)
            pooled = enc is not None
            if not pooled:
                enc = Ffv1Encoder(dec.fmt, w, h, slices=dec.slices, max_frames=min(600, len(compose)),
                                  device=dev.index)
            B = enc.max_frames
            ok = False
            try:
                if not enc.stages:
                    enc.stages = [FrameBatch.interleaved(dec.fmt, w, h, B, device=dev)]
                out = enc.stages[0]
                for i in range(0, len(compose), B):
                    part = compose[i:i + B]
                    m = len(part)
                    dst = FrameBatch.interleaved(dec.fmt, w, h, m, device=dev, storage=out.storage[:m])
                    ops.stall_compose(sb, [pos[s] if s >= 0 else -1 for s, _ in part], [sp for _, sp in part],
                                      dst=dst)
                    data, sizes = enc.encode_host(dst)
                    o = 0
                    for k in sizes.tolist():
                        packets.append(data[o:o + k].tobytes())
                        o += k
                ok = True
            finally:
                if pooled:
                    release_encoder(enc, ok=ok)
        wr = avi.AviWriter(dst_path, w, h, rate, extradata=info["extradata"],
                           info={b"ISFT": provenance(dec.slices).encode()})
        try:
            j = 0
            for s, sp in seq:
                if sp >= 0 or s < 0:
                    wr.write_packet(packets[j])
                    j += 1
                else:
                    wr.write_packet(packet(s))
        except BaseException:
            wr.abort()
            raise
        wr.close()
    return len(seq)
