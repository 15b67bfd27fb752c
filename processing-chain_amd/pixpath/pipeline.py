"""Host<->device streaming pipeline: pinned double buffers + async copies.

decode pipe --read--> pinned_in[k%2] --H2D (h2d stream)--> dev_in[k%2]
   --kernels (compute stream)--> dev_out[k%2] --D2H (d2h stream)--> pinned_out[k%2]
   --write--> encode pipe

Reading batch k+1 and writing batch k-1 (host threads) overlap the H2D,
kernels and D2H of batch k.  H2D, compute and D2H are three HIP streams
ordered by events only where a buffer is reused, so the two PCIe directions
run concurrently (batch k+1's upload beside batch k-1's download) and both
overlap the kernels.  A writer with ``write_device(batch, stream)`` takes the
device output directly (the GPU FFV1 encoder): no D2H, no re-upload; a reader
with ``read_device(n)`` hands over frames already in HBM (the GPU FFV1
decoder): no host round trip, no H2D.  Frame layout everywhere is dense
Y|U|V per frame.
"""
import queue
import threading

import torch

from . import formats
from .frames import FrameBatch


class Stage:
    """A 1:1 per-frame transform on device batches: process(src, dst) enqueues kernels."""

    def __init__(self, in_fmt, in_w, in_h, out_fmt, out_w, out_h, process):
        self.in_fmt, self.in_w, self.in_h = formats.fmt(in_fmt), in_w, in_h
        self.out_fmt, self.out_w, self.out_h = formats.fmt(out_fmt), out_w, out_h
        self.process = process


class Pipeline:
    def __init__(self, stage, batch=32, device=None):
        self.stage = stage
        self.batch = int(batch)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        s = stage
        self.in_fb = formats.frame_bytes(s.in_fmt, s.in_w, s.in_h)
        self.out_fb = formats.frame_bytes(s.out_fmt, s.out_w, s.out_h)
        B = self.batch
        self.h_in = [torch.empty((B, self.in_fb), dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.h_out = [torch.empty((B, self.out_fb), dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.d_in = [FrameBatch.interleaved(s.in_fmt, s.in_w, s.in_h, B, device=self.device) for _ in range(2)]
        self.d_out = [FrameBatch.interleaved(s.out_fmt, s.out_w, s.out_h, B, device=self.device) for _ in range(2)]
        self.h2d_stream = torch.cuda.Stream(self.device)
        self.d2h_stream = torch.cuda.Stream(self.device)
        self.compute_stream = torch.cuda.Stream(self.device)
        self.frames_in = self.frames_out = 0

    def run(self, reader, writer, emit=None):
        """Stream all frames of `reader` through the stage into `writer`.
        ``emit(k_global, n)`` -> list of (batch-local index) to write for input frame k
        (fps maps duplicate / drop frames on the host); default: each frame once."""
        if hasattr(reader, "read_device"):
            return self._run_device_reader(reader, writer, emit)
        B = self.batch
        self.frames_in = self.frames_out = 0  # counts of this run
        rq = queue.Queue(maxsize=2)   # (slot, n) filled buffers
        free_in = queue.Queue()
        for i in range(2):
            free_in.put(i)
        err = []

        def read_loop():
            try:
                while True:
                    slot = free_in.get()
                    n = reader.read_into(self.h_in[slot].numpy(), B)
                    rq.put((slot, n))
                    if n < B:
                        return
            except Exception as e:  # surface reader failures in the main thread
                err.append(e)
                rq.put((None, 0))

        wq = queue.Queue(maxsize=2)

        def write_loop():
            try:
                while True:
                    item = wq.get()
                    if item is None:
                        return
                    slot, n, ev, base = item
                    ev.synchronize()
                    buf = self.h_out[slot].numpy()
                    if emit is None:
                        writer.write(buf[:n])
                    else:
                        for i in range(n):
                            for _ in range(emit(base + i)):
                                writer.write(buf[i:i + 1])
                    self.frames_out += n
                    out_free[slot].set()
            except Exception as e:  # e.g. the encoder died: release the producer and drain
                err.append(e)
                for ev in out_free:
                    ev.set()
                while wq.get() is not None:
                    pass

        out_free = [threading.Event(), threading.Event()]
        for e in out_free:
            e.set()
        comp_done, d2h_done = [None, None], [None, None]
        device_writer = hasattr(writer, "write_device")
        tr = threading.Thread(target=read_loop, daemon=True)
        tw = threading.Thread(target=write_loop, daemon=True)
        tr.start()
        tw.start()
        base = 0
        while True:
            slot, n = rq.get()
            if slot is None or n == 0 or err:
                if slot is not None:
                    free_in.put(slot)
                break
            out_free[slot].wait()
            if err:  # the writer failed while this slot was in use
                free_in.put(slot)
                break
            out_free[slot].clear()
            with torch.cuda.stream(self.h2d_stream):
                if comp_done[slot] is not None:  # batch k-2's kernels have read dev_in[slot]
                    self.h2d_stream.wait_event(comp_done[slot])
                self.d_in[slot].storage[:n].copy_(self.h_in[slot][:n], non_blocking=True)
                h2d_done = torch.cuda.Event()
                h2d_done.record(self.h2d_stream)
            self.compute_stream.wait_event(h2d_done)
            if d2h_done[slot] is not None:  # batch k-2's download has read dev_out[slot]
                self.compute_stream.wait_event(d2h_done[slot])
            with torch.cuda.stream(self.compute_stream):
                src = FrameBatch.interleaved(self.stage.in_fmt, self.stage.in_w, self.stage.in_h, n,
                                             device=self.device, storage=self.d_in[slot].storage[:n])
                dst = FrameBatch.interleaved(self.stage.out_fmt, self.stage.out_w, self.stage.out_h, n,
                                             device=self.device, storage=self.d_out[slot].storage[:n])
                self.stage.process(src, dst, self.compute_stream)
                comp_done[slot] = torch.cuda.Event()
                comp_done[slot].record(self.compute_stream)
            if device_writer:
                # the writer consumes the device batch on the compute stream (e.g. FFV1 encode)
                writer.write_device(dst, self.compute_stream, emit=None if emit is None else
                                    [emit(base + i) for i in range(n)])
                d2h_ev = torch.cuda.Event()
                d2h_ev.record(self.compute_stream)
                d2h_done[slot] = d2h_ev
                h2d_done.synchronize()
                free_in.put(slot)
                out_free[slot].set()
                self.frames_in += n
                self.frames_out += n
                base += n
                if n < B:
                    break
                continue
            self.d2h_stream.wait_event(comp_done[slot])
            with torch.cuda.stream(self.d2h_stream):
                self.h_out[slot][:n].copy_(self.d_out[slot].storage[:n], non_blocking=True)
                d2h_ev = torch.cuda.Event()
                d2h_ev.record(self.d2h_stream)
            d2h_done[slot] = d2h_ev
            # the input slot can be refilled once its H2D copy has finished
            h2d_done.synchronize()
            free_in.put(slot)
            wq.put((slot, n, d2h_ev, base))
            self.frames_in += n
            base += n
            if n < B:
                break
        wq.put(None)
        tw.join()
        if device_writer:
            self.compute_stream.synchronize()
        tr.join(timeout=1.0)
        if err:
            raise err[0]
        return self.frames_in

    def _run_device_reader(self, reader, writer, emit):
        """Frames come from the reader already in HBM (reader.read_device(n) ->
        interleaved FrameBatch or None); the stage runs on them in place of the
        H2D; outputs leave by D2H (or stay on the device for a device writer)."""
        B = self.batch
        self.frames_in = self.frames_out = 0
        device_writer = hasattr(writer, "write_device")
        base, slot = 0, 0
        d2h_done = [None, None]
        while True:
            src = reader.read_device(B)
            if src is None:
                break
            n = src.n
            self.compute_stream.wait_stream(torch.cuda.current_stream(self.device))  # the decode's stream
            if d2h_done[slot] is not None:
                d2h_done[slot].synchronize()  # h_out[slot] / d_out[slot] are free again
            with torch.cuda.stream(self.compute_stream):
                dst = FrameBatch.interleaved(self.stage.out_fmt, self.stage.out_w, self.stage.out_h, n,
                                             device=self.device, storage=self.d_out[slot].storage[:n])
                self.stage.process(src, dst, self.compute_stream)
            counts = None if emit is None else [emit(base + i) for i in range(n)]
            if device_writer:
                writer.write_device(dst, self.compute_stream, emit=counts)
                ev = torch.cuda.Event()
                ev.record(self.compute_stream)
                d2h_done[slot] = ev
            else:
                with torch.cuda.stream(self.compute_stream):
                    self.h_out[slot][:n].copy_(self.d_out[slot].storage[:n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.compute_stream)
                ev.synchronize()
                buf = self.h_out[slot].numpy()
                if counts is None:
                    writer.write(buf[:n])
                else:
                    for i, c in enumerate(counts):
                        for _ in range(c):
                            writer.write(buf[i:i + 1])
                d2h_done[slot] = None
            self.frames_in += n
            self.frames_out += n
            base += n
            slot ^= 1
            # the reader may overwrite its device frames on the next call: the
            # kernels that read them must be done
            self.compute_stream.synchronize()
            if n < B:
                break
        self.compute_stream.synchronize()
        return self.frames_in
