"""Host-side decisions of the pixel path.

Each function restates the reference function named in its docstring with the
same arguments, return values and error convention (logger.error + sys.exit(1)),
so it can be bound onto the reference's Pvs/Hrc/Segment objects or used
standalone.  Pinned by tests/golden/reference_fixtures.json.
"""
import logging
import sys
from fractions import Fraction

logger = logging.getLogger("main")


def calculate_avpvs_video_dimensions(SRC_width, SRC_height, postproc_enc_width, postproc_enc_height):
    """AVPVS [w, h] (reference lib/ffmpeg.py:33-58).

    The reference's first test is written ``SRC_width == postproc_enc_width &
    SRC_height == postproc_enc_height``; Python parses it as the chained
    comparison ``SRC_width == (postproc_enc_width & SRC_height) == postproc_enc_height``,
    which is kept here verbatim in meaning.
    """
    dims = [postproc_enc_width, postproc_enc_height]
    same = SRC_width == (postproc_enc_width & SRC_height) and (postproc_enc_width & SRC_height) == postproc_enc_height
    if not same:
        src_ar = SRC_width / SRC_height
        pp_ar = postproc_enc_width / postproc_enc_height
        if postproc_enc_width < SRC_width:  # mobile-like: keep the SRC aspect, even height
            if not (src_ar == pp_ar):
                h = int(float(postproc_enc_width) / src_ar)
                if h % 2 == 1:
                    h += 1
                dims[1] = h
        elif not (int(1000 * src_ar) == int(1000 * pp_ar)):
            dims[1] = SRC_height
    return dims


def set_pix_fmt(segment):
    """Segment.set_pix_fmt (reference lib/test_config.py:447-480): AVPVS/segment
    target pixel format from the SRC's, with 10-bit and coder overrides."""
    if segment.src.is_youtube:
        segment.target_pix_fmt = "yuv420p"
        return
    src_pix_fmt = segment.src.stream_info["pix_fmt"]
    if ("444" in src_pix_fmt) or ("422" in src_pix_fmt) or ("rgb" in src_pix_fmt):
        fmt = "yuv422p"
    elif "420" in src_pix_fmt:
        fmt = "yuv420p"
    else:
        logger.error("Unknown SRC pixel format: " + str(src_pix_fmt))
        sys.exit(1)
    if ("10" in src_pix_fmt) and (src_pix_fmt != "yuv410p"):
        fmt += "10le"
    if (segment.quality_level.video_codec == "h264") and (segment.video_coding.encoder.casefold() == "bitmovin"):
        fmt = "yuv420p"
    if segment.video_coding.forced_pix_fmt:
        fmt = segment.video_coding.forced_pix_fmt
    segment.target_pix_fmt = fmt


def get_pix_fmt_for_avpvs(pvs):
    """Pvs.get_pix_fmt_for_avpvs (reference lib/test_config.py:172-180)."""
    fmts = set(seg.target_pix_fmt for seg in pvs.segments)
    if len(fmts) > 1:
        logger.error("Segments for PVS " + str(pvs) + " use different target pixel formats!")
        sys.exit(1)
    return list(fmts)[0]


CPVS_FORMAT_MAP = {
    "yuv420p": ("rawvideo", "uyvy422"),
    "yuv422p": ("rawvideo", "uyvy422"),
    "yuv420p10le": ("v210", "yuv422p10le"),
    "yuv422p10le": ("v210", "yuv422p10le"),
}


def get_vcodec_and_pix_fmt_for_cpvs(pvs, rawvideo=False):
    """Pvs.get_vcodec_and_pix_fmt_for_cpvs (reference lib/test_config.py:188-227):
    8-bit AVPVS -> rawvideo uyvy422, 10-bit -> v210 (yuv422p10le); -a keeps the format."""
    avpvs_format = pvs.get_pix_fmt_for_avpvs()
    if rawvideo:
        return ("rawvideo", avpvs_format)
    if avpvs_format not in CPVS_FORMAT_MAP:
        logger.error("Cannot use input pixel format " + str(avpvs_format) + " for CPVS " + str(pvs))
        raise KeyError(avpvs_format)  # the reference indexes the map right after logging
    vcodec, pix = CPVS_FORMAT_MAP[avpvs_format]
    return (vcodec, pix)


def hrc_get_buff_events_media_time(hrc):
    """Hrc.get_buff_events_media_time (reference lib/test_config.py:312-333):
    stalls as [[media_time, duration], ...]; freezes as their sorted specs."""
    events = []
    if any(e.event_type == "freeze" for e in hrc.event_list):
        events = sorted(e.duration for e in hrc.event_list if e.event_type == "freeze")
    elif any(e.event_type in ("stall", "freeze") for e in hrc.event_list):
        t = 0
        for e in hrc.event_list:
            if e.event_type == "stall":
                events.append([t, e.duration])
            else:
                t += e.duration
    return events


def get_buff_events_media_time(pvs):
    """Pvs.get_buff_events_media_time (reference lib/test_config.py:158-162)."""
    return pvs.hrc.get_buff_events_media_time()


def buffer_string(events):
    """The bufferer `-b` argument: str(events) without spaces (p03_generateAvPvs.py:227)."""
    return str(events).replace(" ", "")


def get_fps(segment):
    """_get_fps (reference lib/ffmpeg.py:321-396): (fps filter spec or None, fps or None)."""
    spec = segment.quality_level.fps
    fps = None
    if spec in ("original", "auto"):
        fps = None
    elif spec == "24/25/30":
        orig = segment.src.get_fps()
        if orig in [24, 25, 30]:
            fps = None
        elif orig == 50:
            fps = 25
        elif orig in [60, 120]:
            fps = 30
        else:
            logger.error("SRC " + str(segment.src) + " has unsupported frame rate (" + str(orig) + ")")
            sys.exit(1)
    elif spec == "50/60":
        orig = segment.src.get_fps()
        if orig in [50, 60]:
            fps = None
        elif orig < 50:
            logger.error("fps for " + str(segment) + " were requested as 50/60 but SRC has only " + str(orig))
            sys.exit(1)
        elif orig == 120:
            fps = 60
        else:
            logger.error("SRC " + str(segment.src) + " has unsupported frame rate (" + str(orig) + ")")
            sys.exit(1)
    elif "/" in str(spec):
        fps = segment.src.get_fps() * float(Fraction(spec))
        if (fps > 60) or (fps < 12):
            logger.warning("fps for " + str(segment) + " were calculated as " + str(fps) + " which does not seem right")
    else:
        fps = int(spec)
    return (None if fps is None else "fps=fps=" + str(fps), fps)


# select patterns of encode_segment (reference lib/ffmpeg.py:806-831), keyed by int(100*out/in)
SELECT_PATTERNS = {
    50: "mod(n+1,2)",
    40: "not(mod(n,5))+not(mod(n-3,5))",
    33: "not(mod(n,3))",
    25: "not(mod(n,4))",
    80: "mod(n+1,5)",
    30: "not(mod(n,10)) + not(mod(n-3,10)) + not(mod(n-7,10))",
    60: "not(mod(n,5))+not(mod(n-3,5))+not(mod(n-2,5))",
}
SELECT_62_5 = "not(mod(n,8))+not(mod(n-3,8))+not(mod(n-2,8))+not(mod(n-5,8))+not(mod(n-6,8))"


def select_expression(orig_fps, fps):
    """select='...' pattern for a frame-rate reduction, or '' (no select), or raises SystemExit."""
    perc = 100 * fps / orig_fps
    if int(perc) == 100:
        return ""
    if int(perc) in SELECT_PATTERNS:
        return SELECT_PATTERNS[int(perc)]
    if perc == 62.5:
        return SELECT_62_5
    logger.error("Frame rate conversion from " + str(orig_fps) + " to " + str(fps) + " is not supported")
    sys.exit(1)


def eval_select(expr, n):
    """Evaluate one of the reference's select expressions for input frame n (0-based):
    keep the frame when the expression is non-zero (libavfilter select semantics)."""
    if expr == "":
        return True
    env = {"mod": lambda a, b: a - b * int(a / b) if b else 0, "n": n}
    env["not"] = None
    py = expr.replace("not(", "_not(")
    return bool(eval(py, {"__builtins__": {}}, {"mod": env["mod"], "n": n, "_not": lambda v: 0 if v else 1}))


def encode_segment_filter_chain(segment):
    """The -filter:v chain of encode_segment (reference lib/ffmpeg.py:794-837),
    quoted as the reference quotes it."""
    flist = ["scale={}:-2:flags=bicubic".format(segment.quality_level.width)]
    fps_cmd, fps = get_fps(segment)
    orig = float(Fraction(segment.src.stream_info["r_frame_rate"]))
    if fps_cmd:
        sel = select_expression(orig, fps)
        if sel:
            flist.append("select='" + sel + "'")
        flist.append("fps=fps=" + str(fps))
    else:
        flist.append("fps=fps=" + str(orig))
    return '"' + ",".join(flist) + '"'


def scale_height_keep_aspect(src_w, src_h, w, factor=2):
    """`scale=W:-2` output height (libavfilter scale_eval.c): av_rescale rounds to
    nearest, then a multiple of `factor`."""
    num, den = w * src_h, src_w * factor
    q = (2 * num + den) // (2 * den)  # av_rescale: round half away from zero (positive)
    return q * factor


def fps_index_map(n_in, in_rate, out_rate):
    """vf_fps output->input map (row a14): pure host function, same algorithm as
    the C-ABI pp_fps_map (so usable without the GPU library)."""
    a, b = Fraction(in_rate), Fraction(out_rate)
    N, D = a.denominator * b.numerator, a.numerator * b.denominator
    n_out = (n_in * N + D // 2) // D
    out, i = [], 0
    for k in range(n_out):
        while i + 1 < n_in and ((i + 1) * N * 2 + D) // (2 * D) <= k:
            i += 1
        out.append(i)
    return out


def _round_near(num, den):
    """av_rescale_rnd(..., AV_ROUND_NEAR_INF) for non-negative num / den."""
    return (2 * num + den) // (2 * den)


def select_fps_map(n_in, in_rate, out_rate, select_expr=""):
    """`select='expr',fps=fps=F` over n_in input frames at in_rate (row a14):
    the input frame shown at each output frame.

    select keeps frame n when the expression is non-zero and leaves its
    timestamp n / in_rate unchanged; vf_fps (libavfilter/vf_fps.c, rounding
    =near) converts each kept frame's timestamp to output frame units, starts
    at the first one, shows the newest kept frame whose converted timestamp is
    <= the output frame's, and stops at the end-of-stream timestamp
    n_in / in_rate.  Without a select this is fps_index_map."""
    a, b = Fraction(in_rate), Fraction(out_rate)
    N, D = a.denominator * b.numerator, a.numerator * b.denominator  # t_out = n * N / D
    kept = [n for n in range(n_in) if eval_select(select_expr, n)]
    if not kept:
        return []
    q = [_round_near(n * N, D) for n in kept]
    q_eof = _round_near(n_in * N, D)
    out, i = [], 0
    for j in range(q[0], q_eof):
        while i + 1 < len(q) and q[i + 1] <= j:
            i += 1
        out.append(kept[i])
    return out
