"""p02 frame-size scanners, a drop-in for
lib/get_framesize.py with the same names, arguments, return values, side
effects and failures.

  delete_packets(pvs_vfi)            :27-51   VP9 superframe merge (host logic)
  convert_file(filename, codec, force) :54-77 the same ffmpeg remux string
  remove_convFile(conv_filename)     :80-84
  get_framesize_vp9(filename, force) :87-141  -> pp_ivf_frame_sizes
  get_framesize_h264(filename, force) :144-201 -> pp_annexb_frame_sizes(H264)
  get_framesize_h265(filename, force) :204-263 -> pp_annexb_frame_sizes(H265)
  get_framesize_av1(filename, force=True) :266-274 the same ffprobe call

The byte loops run in libpixpath's host scanner (csrc/scan.cpp, memchr jumps
between start codes) instead of Python's per-byte hex() strings; results are
the reference's, pinned against its own outputs
(tests/golden/framesize_fixtures.json, tests/test_framesize_parity.py).
Reference behaviour kept on purpose:
  * an empty *_tmp file returns [] and is NOT removed (H.264/H.265);
  * an H.264 NAL header byte 0xa1..0xf5 with low digit 1/5 raises ValueError;
  * every VP9 frame failing the "10" frame-marker test prints
    "Frame misdeteciton! Aborting..." (and nothing aborts);
  * delete_packets raises UnboundLocalError when the first packet's index is
    not 0, and deletes at shifted indices exactly as the reference does.
"""
import ctypes
import json
import logging
import os.path
from os import remove

import numpy as np

from . import _native
from .probe import run_command

logger = logging.getLogger("main")


def delete_packets(pvs_vfi):
    """Merge packets whose dts differ by < 1.1 ms into the previous one."""
    last_dts = -10
    merged = 0
    to_delete = []
    for index, vf in enumerate(pvs_vfi):
        if pvs_vfi[index]["index"] == 0:
            merged_segment = 0
        if abs(vf["dts"] - last_dts) < 0.0011:
            pvs_vfi[index - 1]["size"] = int(pvs_vfi[index - 1]["size"]) + int(vf["size"])
            to_delete.append(index - merged)
            merged += 1
            merged_segment += 1  # noqa: F821 -- UnboundLocalError like the reference
            logger.debug("videoFrames merged!")
        else:
            pvs_vfi[index]["index"] = vf["index"] - merged_segment  # noqa: F821
        last_dts = vf["dts"]
    for i in to_delete:
        del pvs_vfi[i]


_SUFFIX = {"vp9": ("_tmp.ivf", ""), "h264": ("_tmp.h264", " -bsf:v h264_mp4toannexb"),
           "h265": ("_tmp.h265", " -bsf:v hevc_mp4toannexb")}


def convert_file(filename, codec, force):
    """Remux the segment's video into IVF / Annex B next to it (stream copy)."""
    add_y = " -y " if force else ""
    suffix, bsf = _SUFFIX["vp9" if codec == "vp9" else "h264" if codec == "h264" else "h265"]
    conv_filename = "".join([filename, suffix])
    cmd = "ffmpeg {} -i {} -vcodec copy -acodec copy".format(add_y, filename) + "{} {}".format(bsf, conv_filename)
    if os.path.isfile(conv_filename) and not force:
        return conv_filename
    run_command(cmd, "converting {} to {}".format(filename, conv_filename))
    return conv_filename


def remove_convFile(conv_filename):  # noqa: N802 -- reference name
    if os.path.isfile(conv_filename):
        remove(conv_filename)
    else:
        print("Tried to delete {conv_filename}, but it was not found!")


def _read(path):
    return np.fromfile(path, dtype=np.uint8)


def annexb_frame_sizes(data, codec):
    """Frame sizes of an Annex-B byte buffer (numpy uint8) as get_framesize_h264/h265 count them."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    L = _native.lib()
    ptr = data.ctypes.data_as(ctypes.c_void_p) if data.size else None
    nal = _native.PP_NAL_H264 if codec == "h264" else _native.PP_NAL_H265
    cap = max(16, data.size // 64)
    while True:  # a second call only when the frames outnumber the first guess
        out = np.zeros(cap, dtype=np.int64)
        n = L.pp_annexb_frame_sizes(ptr, data.size, nal, out.ctypes.data_as(ctypes.c_void_p), cap)
        if n < 0:
            msg = L.pp_last_error().decode(errors="replace")
            if msg.startswith("ValueError: "):
                raise ValueError(msg[len("ValueError: "):])
            _native.check(n)
        if n <= cap:
            return [int(v) for v in out[:n]]
        cap = n


def ivf_frame_sizes(data):
    """(sizes, misdetected frame count) of an IVF byte buffer as get_framesize_vp9 reads it."""
    mis = ctypes.c_int64(0)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    L = _native.lib()
    ptr = data.ctypes.data_as(ctypes.c_void_p) if data.size else None
    cap = max(16, data.size // 64)
    while True:
        out = np.zeros(cap, dtype=np.int64)
        n = _native.check(L.pp_ivf_frame_sizes(ptr, data.size, out.ctypes.data_as(ctypes.c_void_p), cap,
                                               ctypes.byref(mis)))
        if n <= cap:
            return [int(v) for v in out[:n]], int(mis.value)
        cap = n


def get_framesize_vp9(filename, force):
    conv_filename = convert_file(filename, "vp9", force)
    sizes, mis = ivf_frame_sizes(_read(conv_filename))
    for _ in range(mis):
        print("Frame misdeteciton! Aborting...")
    remove_convFile(conv_filename)
    return sizes


def _annexb(filename, force, codec):
    conv_filename = convert_file(filename, codec, force)
    data = _read(conv_filename)
    if data.size == 0:
        return []  # the reference returns before removing the empty temp file
    sizes = annexb_frame_sizes(data, codec)
    remove_convFile(conv_filename)
    return sizes


def get_framesize_h264(filename, force):
    return _annexb(filename, force, "h264")


def get_framesize_h265(filename, force):
    return _annexb(filename, force, "h265")


def get_framesize_av1(filename, force=True):
    cmd = "ffprobe -select_streams v -show_frames -of json '" + filename + "'"
    stdout, _ = run_command(cmd, name="get framesizes info for " + str(filename))
    info = json.loads(stdout)["frames"]
    return [int(ii["pkt_size"]) for ii in info]
