"""Drop-in for the pixel-path command builders of the reference's lib/ffmpeg.py.

Same function names, signatures, return convention (ONE whitespace-collapsed
shell string, or None when the output exists and overwrite is False) and error
convention (logger.error + sys.exit(1)) as the reference.

Two backends, chosen by ``set_backend()`` or the environment variable
PIXPATH_BACKEND:

* "ffmpeg" (default): the reference's strings, byte-identical (pinned by
  tests/golden/reference_fixtures.json) -- every pixel op runs inside ffmpeg.
* "gpu": the pixel work of a builder runs on the MI355X through
  ``python3 -m pixpath.cli`` (ffmpeg still decodes and encodes; frames cross
  PCIe once each way and every filter between decode and encode runs as HIP
  kernels).  The AVPVS intermediate is FFV1 coded on the GPU (PIXPATH_FFV1,
  default "gpu"; "ffmpeg" keeps the reference's `-coder 1 -context 1` encoder,
  the reference-faithful bitstream): then the long-test concat copies packets
  and the preview decodes on the GPU.  The audio mux stays a stream copy by
  ffmpeg; the mobile/tablet CPVS run their scale on the MI355X and keep x264
  (the tablet pad branch keeps the reference's string).

Reference functions mirrored (file:line in pnats2avhd/processing-chain):
  calculate_avpvs_video_dimensions  lib/ffmpeg.py:33
  encode_segment                    lib/ffmpeg.py:772 (p01; the encoder options stay the reference's)
  create_avpvs_short                lib/ffmpeg.py:940
  create_avpvs_segment              lib/ffmpeg.py:1003
  create_avpvs_long_concat          lib/ffmpeg.py:1058
  simple_encoding                   lib/ffmpeg.py:1108
  create_cpvs                       lib/ffmpeg.py:1149
  create_preview                    lib/ffmpeg.py:1250
  audio_mux                         lib/ffmpeg.py:1262
  bufferer_command                  p03_generateAvPvs.py:215-243 (inline there)
"""
import logging
import os
import shlex
import sys

from .chain import calculate_avpvs_video_dimensions  # noqa: F401  (re-export, a1)
from .chain import buffer_string, encode_segment_filter_chain  # noqa: F401

logger = logging.getLogger("main")

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FFV1_OPTS = "-c:v ffv1 -threads 4 -level 3 -coder 1 -context 1 -slicecrc 1"

_backend = os.environ.get("PIXPATH_BACKEND", "ffmpeg")


def set_backend(name):
    global _backend
    if name not in ("ffmpeg", "gpu"):
        raise ValueError("backend must be 'ffmpeg' or 'gpu'")
    _backend = name


def get_backend():
    return _backend


def _collapse(cmd):
    return " ".join(cmd.split())


def _skip_existing(output_file, overwrite):
    """(overwrite_spec, skip): the reference's -y / -n / None convention (lib/ffmpeg.py:964-970)."""
    if overwrite:
        return "-y", False
    if os.path.isfile(output_file):
        logger.warning("output " + output_file + " already exists, will not convert. Use --force to force overwriting.")
        return "-n", True
    return "-n", False


def ffv1_on_gpu():
    """The gpu backend's AVPVS codec: FFV1 coded on the GPU into pixpath's own
    AVI (default), or ffmpeg's FFV1 encoder fed through a
    pipe with PIXPATH_FFV1=ffmpeg."""
    v = os.environ.get("PIXPATH_FFV1", "gpu")
    if v not in ("gpu", "ffmpeg"):
        raise ValueError("PIXPATH_FFV1 must be 'gpu' or 'ffmpeg'")
    return v == "gpu"


def ffv1_slices():
    """The GPU FFV1 slice grid "HxV" (PIXPATH_FFV1_SLICES, default 8x8)."""
    v = os.environ.get("PIXPATH_FFV1_SLICES", "8x8").lower()
    t = v.split("x")
    if len(t) != 2 or not all(x.isdigit() and int(x) > 0 for x in t):
        raise ValueError("PIXPATH_FFV1_SLICES must be HxV, e.g. 16x16")
    return v


def _gpu_cli(sub, args):
    args = list(args)
    if ffv1_on_gpu():
        # FFV1 AVPVS coded on the GPU in pixpath's own AVI: the AVPVS writers
        # encode it, its readers (CPVS, stall, mobile scale) decode it there.
        # The codec and slice grid are part of the command, so p03's per-PVS
        # log (`ffmpegCommand:` lines, p03_generateAvPvs.py:41-59) records them;
        # with PIXPATH_FFV1=ffmpeg the command carries the reference's
        # `-c:v ffv1 ... -coder 1 -context 1` options instead.
        if sub == "avpvs" and FFV1_OPTS in args:
            args[-1:-1] = ["--gpu-ffv1", "--ffv1-slices", ffv1_slices()]
        elif sub == "avpvs":
            args.insert(-1, "--ffv1-input")
        elif sub in ("cpvs", "stall"):
            args.insert(-1, "--gpu-ffv1")
    return "PYTHONPATH={} python3 -m pixpath.cli {} {}".format(shlex.quote(PKG_DIR), sub,
                                                                " ".join(shlex.quote(str(a)) for a in args))


def encode_segment(segment, overwrite=False, video_encoder_command=None):
    """p01 segment encode (lib/ffmpeg.py:772-937): `-ss/-t` trim, then
    `scale=W:-2:flags=bicubic[,select='...'],fps=fps=F`, then the encoder.

    ``video_encoder_command(segment, current_pass=1, total_passes=1, logfile="")``
    is the reference's own _get_video_encoder_command (lib/ffmpeg.py:61-318):
    encoders are not part of the pixel path, so the drop-in takes it from the
    reference module.  In the ffmpeg backend the
    string is the reference's byte for byte.  In the gpu backend
    ``pixpath.cli encseg`` decodes the trimmed range, runs scale (+ the
    -pix_fmt conversion) on the MI355X and the select/fps frame choice on the
    host (pixpath.chain.select_fps_map), and hands the frames to the same
    encoder invocation(s) as Y4M (two-pass encodes read a temporary Y4M twice).
    """
    if video_encoder_command is None:
        raise TypeError("encode_segment needs the reference's _get_video_encoder_command "
                        "(video_encoder_command=...)")
    from fractions import Fraction

    from .chain import get_fps, select_expression
    test_config = segment.src.test_config
    input_file = segment.src.file_path
    output_file = os.path.join(test_config.get_video_segments_path(), segment.get_filename())
    if overwrite:
        overwrite_spec = "-y"
    else:
        overwrite_spec = "-n"
        if os.path.isfile(output_file):
            logger.warning("output " + output_file + " already exists, will not convert. Use --force to force overwriting.")
            return None
    nr_threads_opt = "" if segment.quality_level.video_codec == "av1" else " -threads 1"
    filters = encode_segment_filter_chain(segment)
    if test_config.type == "long":
        audio_encoder_cmd = "-c:a {} -b:a {}k".format(segment.audio_coding.encoder, segment.quality_level.audio_bitrate)
    else:
        audio_encoder_cmd = ""
    passes = segment.video_coding.passes
    if passes not in (1, 2) and not (segment.video_coding.crf or segment.video_coding.qp):
        logger.error("only 1 or 2 pass or crf encoding implemented")
        sys.exit(1)

    if _backend == "gpu":
        fps_cmd, fps = get_fps(segment)
        orig_fps = float(Fraction(segment.src.stream_info["r_frame_rate"]))
        sel = select_expression(orig_fps, fps) if fps_cmd else ""
        out_fps = fps if fps_cmd else orig_fps
        tmp = os.path.join(test_config.get_video_segments_path(),
                           ".pixpath_" + os.path.splitext(os.path.basename(output_file))[0] + ".y4m")
        dec = _gpu_cli("encseg", ["--input", input_file, "--start", segment.start_time, "--duration",
                                  segment.duration, "--width", segment.quality_level.width, "--flags", "bicubic",
                                  "--pix-fmt", segment.target_pix_fmt, "--select", sel, "--fps", out_fps,
                                  "--in-fps", segment.src.stream_info["r_frame_rate"], tmp if passes == 2 else "-"])
        # audio (long tests) from the trimmed SRC as in the reference command
        audio_in = ("-ss {} -t {} -i {} -map 0:v -map 1:a".format(segment.start_time, segment.duration, input_file)
                    if audio_encoder_cmd else "")
        if passes == 2:
            passlogfile = os.path.join(test_config.get_logs_path(),
                                       "passlogfile_" + os.path.splitext(os.path.basename(output_file))[0])
            output_format = {"mp4": "mp4", "mkv": "matroska"}.get(segment.ext)
            if output_format is None:
                logger.error("unknown segment extension " + segment.ext)
            common = "-nostdin -f yuv4mpegpipe -i {} {} -video_track_timescale 90000 {}".format(
                tmp, audio_in, audio_encoder_cmd)
            cmd = " ".join([dec, "&&", "ffmpeg -y", common,
                            video_encoder_command(segment, current_pass=1, total_passes=2, logfile=passlogfile),
                            "-f", str(output_format), "/dev/null", "&&", "ffmpeg", overwrite_spec, common,
                            video_encoder_command(segment, current_pass=2, total_passes=2, logfile=passlogfile),
                            output_file, ";", "rc=$?; rm -f", tmp, "; exit $rc"])
        else:
            cmd = " ".join([dec, "|", "ffmpeg -nostdin", overwrite_spec, "-f yuv4mpegpipe -i -", audio_in,
                            "-video_track_timescale 90000", video_encoder_command(segment), audio_encoder_cmd,
                            output_file])
        return _collapse(cmd)

    common_fmt = """
        -nostdin
        -ss {start} -i {input_file}
        {nr_threads_opt}
        -t {dur}
        -video_track_timescale 90000
        -filter:v {filters}
        {audio_encoder_cmd}
        """
    if passes == 2:
        common_opts = common_fmt.format(start=segment.start_time, dur=segment.duration, **locals())
        passlogfile = os.path.join(test_config.get_logs_path(),
                                   "passlogfile_" + os.path.splitext(os.path.basename(output_file))[0])
        if segment.ext == "mp4":
            output_format = "mp4"
        elif segment.ext == "mkv":
            output_format = "matroska"
        else:
            logger.error("unknown segment extension " + segment.ext)
        pass1 = " ".join(["ffmpeg", "-y", common_opts,
                          video_encoder_command(segment, current_pass=1, total_passes=2, logfile=passlogfile),
                          "-f", output_format, "/dev/null"])
        pass2 = " ".join(["ffmpeg", overwrite_spec, common_opts,
                          video_encoder_command(segment, current_pass=2, total_passes=2, logfile=passlogfile),
                          output_file])
        cmd = pass1 + " && " + pass2
    else:  # one pass, or crf/qp
        cmd = """
        ffmpeg -nostdin
        {overwrite_spec}
        -ss {start} -i {input_file}
        {nr_threads_opt}
        -t {dur}
        -video_track_timescale 90000
        -filter:v {filters}
        {video_encoder_cmd}
        {audio_encoder_cmd}
        {output_file}
        """.format(start=segment.start_time, dur=segment.duration, video_encoder_cmd=video_encoder_command(segment),
                   **locals())
    return _collapse(cmd)


def create_avpvs_short(pvs, overwrite=False, scale_avpvs_tosource=False, force_60_fps=False, post_proc_id=0):
    """Decode the first segment, upscale to the AVPVS size, FFV1 + FLAC (lib/ffmpeg.py:940-1000)."""
    test_config = pvs.test_config
    coding_width = test_config.post_processings[post_proc_id].coding_width
    coding_height = test_config.post_processings[post_proc_id].coding_height
    output_file = pvs.get_avpvs_wo_buffer_file_path() if pvs.has_buffering() else pvs.get_avpvs_file_path()

    fps_filter, fps = "", None
    if scale_avpvs_tosource:
        fps = pvs.src.get_fps()
        fps_filter = ",fps={src_framerate}"  # the reference never expands this placeholder
    elif force_60_fps:
        fps = 60.0
        fps_filter = ",fps={src_framerate}"

    overwrite_spec, skip = _skip_existing(output_file, overwrite)
    if skip:
        return None

    input_file = pvs.segments[0].get_segment_file_path()
    target_pix_fmt = pvs.get_pix_fmt_for_avpvs()
    w, h = calculate_avpvs_video_dimensions(pvs.src.stream_info["coded_width"], pvs.src.stream_info["coded_height"],
                                            coding_width, coding_height)
    ql = pvs.segments[0].quality_level
    if ql.height > h:  # the QL is taller than the AVPVS: use the QL size (lib/ffmpeg.py:981-986)
        w, h = ql.width, ql.height

    if _backend == "gpu":
        args = [overwrite_spec, "--input", input_file, "--size", "%dx%d" % (w, h), "--flags", "bicubic",
                "--pix-fmt", target_pix_fmt, "--vopts", FFV1_OPTS, "--aopts", "-c:a flac"]
        if fps is not None:
            # the reference passes the unexpanded placeholder `fps={src_framerate}`
            # to ffmpeg, which rejects it and the run fails (lib/ffmpeg.py:958-961);
            # the GPU backend hands over the same literal and fails the same way
            args += ["--fps", "{src_framerate}"]
        spinner = default_spinner_path()
        if pvs.has_buffering() and (pvs.has_framefreeze() or spinner):
            # p03's bufferer step composed in this same pass (section 8f-3):
            # `cli stall` later keeps the output when its arguments match
            # (bufferer_command with p03's default --spinner-path)
            args += ["--stall-output", pvs.get_avpvs_file_path(),
                     "--buffer", buffer_string(pvs.get_buff_events_media_time()), "--black-frame"]
            args += ["--skipping"] if pvs.has_framefreeze() else ["--spinner", spinner]
        return _collapse(_gpu_cli("avpvs", args + [output_file]))

    cmd = """
    ffmpeg -nostdin
    {overwrite_spec}
    -i {input_file}
    -filter:v scale={w}:{h}:flags=bicubic{fps_filter},setsar=1/1
    {FFV1_OPTS}
    -pix_fmt {target_pix_fmt} -c:a flac
    {output_file}""".format(FFV1_OPTS=FFV1_OPTS, **locals())
    return _collapse(cmd)


def create_avpvs_segment(seg, pvs, overwrite=False, scale_avpvs_tosource=False):
    """Long tests: one segment scaled onto a fixed-duration canvas (lib/ffmpeg.py:1003-1055).

    ffmpeg semantics reproduced by the GPU backend: scale to the AVPVS size in
    the overlay's yuv420p, fps to R, last frame repeated to D*R frames, then the
    -pix_fmt conversion to the AVPVS format."""
    test_config = pvs.test_config
    coding_height = test_config.post_processings[0].coding_height
    coding_width = test_config.post_processings[0].coding_width
    w, h = calculate_avpvs_video_dimensions(pvs.src.stream_info["coded_width"], pvs.src.stream_info["coded_height"],
                                            coding_width, coding_height)
    target_pix_fmt = pvs.get_pix_fmt_for_avpvs()
    input_file = seg.get_segment_file_path()
    output_file = seg.get_tmp_path()
    overwrite_spec, skip = _skip_existing(output_file, overwrite)
    if skip:
        return None
    src_framerate = pvs.src.get_fps() if scale_avpvs_tosource else 60.0
    segment_duration = seg.get_segment_duration()

    if _backend == "gpu":
        args = [overwrite_spec, "--input", input_file, "--size", "%dx%d" % (w, h), "--flags", "bicubic",
                "--pix-fmt", target_pix_fmt, "--fps", src_framerate, "--duration", segment_duration,
                "--overlay-yuv420", "--vopts", FFV1_OPTS, "--aopts", "-an"]
        return _collapse(_gpu_cli("avpvs", args + [output_file]))

    overlay = "-f lavfi -i nullsrc=s={w}x{h}:d={segment_duration}:r={src_framerate}".format(**locals())
    complex_filter = ("-filter_complex \"[0:v]scale={w}:{h}:flags=bicubic,fps={src_framerate},setsar=1/1[ol_0];"
                      "[1:v][ol_0]overlay[vout]\"").format(**locals())
    cmd = """
    ffmpeg -nostdin
    {overwrite_spec}
    -i {input_file}
    {overlay}
    {complex_filter}
    -map "[vout]" -t {segment_duration}
    {FFV1_OPTS}
    -pix_fmt {target_pix_fmt}
    {output_file}
    """.format(FFV1_OPTS=FFV1_OPTS, **locals())
    return _collapse(cmd)


def create_avpvs_long_concat(pvs, overwrite=False, scale_avpvs_tosource=False):
    """Stream-copy concat of the decoded segments (lib/ffmpeg.py:1058-1105); writes the
    concat file list as a side effect, like the reference.  No pixel work: the
    ffmpeg backend (and the gpu backend with PIXPATH_FFV1=ffmpeg) return the
    reference's string; with the segment canvases written as GPU-FFV1 AVIs the
    gpu backend copies their packets (`pixpath.cli concat`, same -t cut)."""
    output_file = pvs.get_tmp_wo_audio_path()
    overwrite_spec, skip = _skip_existing(output_file, overwrite)
    if skip:
        return None
    total = sum([int(s.get_segment_duration()) for s in pvs.segments])
    tmp_filelist = pvs.get_avpvs_file_list()
    with open(tmp_filelist, "w+") as fh:
        for s in pvs.segments:
            fh.write("file " + s.get_tmp_path() + "\n")
    if _backend == "gpu" and ffv1_on_gpu():
        return _collapse(_gpu_cli("concat", [overwrite_spec, "--filelist", tmp_filelist, "--duration", total,
                                             output_file]))
    cmd = """
    ffmpeg -nostdin
    {overwrite_spec}
    -f concat -safe 0
    -i {tmp_filelist}
    -c:v copy -t {total}
    {output_file}""".format(**locals())
    return _collapse(cmd)


def simple_encoding(pvs, overwrite, input_file, output_file, vopts, aopts="", filters=""):
    """lib/ffmpeg.py:1108-1146."""
    overwrite_spec, skip = _skip_existing(output_file, overwrite)
    if skip:
        return None
    cmd = """
    ffmpeg -nostdin
    {overwrite_spec}
    -i {input_file} {filters}
    {vopts} {aopts}
    {output_file}""".format(**locals())
    return _collapse(cmd)


def create_cpvs(pvs, post_processing, rawvideo=False, overwrite=False, nonraw_crf=17, mobile_vprofile="high",
                mobile_preset="fast"):
    """CPVS for the playback context (lib/ffmpeg.py:1149-1247).  PC/TV: fps, optional
    letterbox pad, uyvy422 rawvideo or v210 in AVI (GPU backend: fps map + pad +
    chroma conversion + packing on the MI355X).  Other contexts: x264 (ffmpeg)."""
    test_config = pvs.test_config
    input_file = pvs.get_avpvs_file_path()
    output_file = pvs.get_cpvs_file_path(context=post_processing.processing_type, rawvideo=rawvideo)
    w, h = calculate_avpvs_video_dimensions(pvs.src.stream_info["coded_width"], pvs.src.stream_info["coded_height"],
                                            post_processing.coding_width, post_processing.coding_height)
    aformat_normalize = ""
    if post_processing.processing_type in ["pc", "tv"]:
        vcodec, target_pix_fmt = pvs.get_vcodec_and_pix_fmt_for_cpvs(rawvideo=rawvideo)
        pad = h < post_processing.coding_height
        if test_config.is_short():
            pc_aopts = "-an"
        else:
            total_duration = str(pvs.hrc.get_long_hrc_duration())
            pc_aopts = "-ac 2 -c:a pcm_s16le -t {total_duration}".format(**locals())
        if _backend == "gpu":
            overwrite_spec, skip = _skip_existing(output_file, overwrite)
            if skip:
                return None
            args = [overwrite_spec, "--input", input_file, "--fps", post_processing.display_frame_rate,
                    "--vcodec", vcodec, "--pix-fmt", target_pix_fmt, "--aopts", "-af aresample=48000 " + pc_aopts]
            if pad:
                args += ["--pad", "%dx%d" % (post_processing.display_width, post_processing.display_height)]
            cmd = _collapse(_gpu_cli("cpvs", args + [output_file]))
        else:
            filters = "-af aresample=48000 -filter:v 'fps=fps={}".format(post_processing.display_frame_rate)
            if pad:
                filters += ",pad=width={}:height={}:x=(ow-iw)/2:y=(oh-ih)/2".format(
                    post_processing.display_width, post_processing.display_height) + "'"
            else:
                filters += "'"
            cmd = simple_encoding(pvs, overwrite, input_file, output_file,
                                  "-c:v " + vcodec + " -pix_fmt " + target_pix_fmt, pc_aopts, filters)
    else:
        mobile_vopts = ("-c:v libx264 -preset {mobile_preset} -pix_fmt yuv420p -crf {nonraw_crf} "
                        "-profile:v {mobile_vprofile} -movflags faststart").format(**locals())
        filters = "-filter:v '"
        if (post_processing.display_height != post_processing.coding_height) or (h < post_processing.coding_height):
            # the reference's leading comma (lib/ffmpeg.py:1210) is kept verbatim
            filters += ",pad=width={}:height={}:x=(ow-iw)/2:y=(oh-ih)/2".format(
                post_processing.display_width, post_processing.display_height) + "'"
        else:
            filters += "scale={}:{}:flags=bicubic,setsar=1/1".format(
                post_processing.display_width, post_processing.display_height) + "'"
        if test_config.is_short():
            mobile_aopts = "-an"
        else:
            total_duration = str(pvs.hrc.get_long_hrc_duration())
            aformat_normalize = "-c:a aac -b:a 512k"
            mobile_aopts = "-c:a aac -b:a 512k -t {total_duration}".format(**locals())
        if _backend == "gpu" and filters.startswith("-filter:v 'scale="):
            # `scale=DW:DH:flags=bicubic,setsar=1/1` into libx264's yuv420p: ffmpeg
            # negotiates one swscale context (resize + conversion), i.e. one plan on
            # the MI355X; the same x264 options encode the piped frames.  The pad
            # branch above keeps the reference's string (its leading comma makes
            # ffmpeg reject the graph, lib/ffmpeg.py:1206-1210; so does the drop-in).
            overwrite_spec, skip = _skip_existing(output_file, overwrite)
            if skip:
                return None
            cmd = _collapse(_gpu_cli("avpvs", [overwrite_spec, "--input", input_file, "--size", "%dx%d" % (
                post_processing.display_width, post_processing.display_height), "--flags", "bicubic",
                "--pix-fmt", "yuv420p", "--vopts", mobile_vopts, "--aopts", mobile_aopts, output_file]))
        else:
            cmd = simple_encoding(pvs, overwrite, input_file, output_file, mobile_vopts, mobile_aopts, filters)

    if test_config.is_long():
        if cmd is None:
            return
        cpvs_path = os.path.abspath(test_config.get_cpvs_path())
        cmd = " ".join([cmd, "&&", "TMP={cpvs_path}".format(**locals()),
                        "ffmpeg-normalize {output_file} -o {output_file} -f -nt rms {aformat_normalize}".format(
                            **locals())])
    return cmd


def create_preview(pvs, overwrite=False):
    """ProRes preview (lib/ffmpeg.py:1250-1259).  The encode is codec work
    (ffmpeg's ProRes in both backends); with the GPU FFV1 AVPVS the gpu backend
    decodes the AVPVS on the GPU (`pixpath.cli preview`) and pipes the frames
    to that encoder, so FFmpeg never decodes pixpath's FFV1 bitstream."""
    if _backend == "gpu" and ffv1_on_gpu():
        output_file = pvs.get_preview_file_path()
        overwrite_spec, skip = _skip_existing(output_file, overwrite)
        if skip:
            return None
        return _collapse(_gpu_cli("preview", [overwrite_spec, "--input", pvs.get_avpvs_file_path(), "--vopts",
                                              "-c:v prores", "--aopts", "-c:a aac", output_file]))
    return simple_encoding(pvs, overwrite, pvs.get_avpvs_file_path(), pvs.get_preview_file_path(), "-c:v prores",
                           "-c:a aac")


def audio_mux(pvs, overwrite=False):
    """Mux SRC audio as PCM (lib/ffmpeg.py:1262-1289); no pixel work."""
    input_file = pvs.get_tmp_wo_audio_path()
    audio_src = pvs.src.get_src_file_path()
    output_file = pvs.get_avpvs_wo_buffer_file_path() if pvs.has_buffering() else pvs.get_avpvs_file_path()
    overwrite_spec, skip = _skip_existing(output_file, overwrite)
    if skip:
        return None
    cmd = """
    ffmpeg -nostdin
    {overwrite_spec}
    -i {input_file}
    -i {audio_src}
    -c:v copy -ac 2 -c:a pcm_s16le -map 0:v -map 1:a
    {output_file}""".format(**locals())
    return _collapse(cmd)


def default_spinner_path():
    """p03's default --spinner-path (lib/parse_args.py:97-100:
    <reference>/util/spinner-128-white.png), from PIXPATH_SPINNER or the
    imported reference package; None when neither is known."""
    env = os.environ.get("PIXPATH_SPINNER")
    if env:
        return env
    mod = sys.modules.get("lib.parse_args") or sys.modules.get("lib.ffmpeg")
    if mod is not None and getattr(mod, "__file__", None):
        p = os.path.abspath(os.path.join(os.path.dirname(mod.__file__), "..", "util", "spinner-128-white.png"))
        if os.path.isfile(p):
            return p
    return None


def bufferer_command(pvs, spinner_path, force=False):
    """The stalling/freezing command p03 builds inline (p03_generateAvPvs.py:223-243).

    ffmpeg backend: the reference's bufferer string.  gpu backend: the PP-STALL-1
    compositor (frozen frame or black + centred spinner, or frame freezing with
    skipping) through pixpath.cli."""
    input_file = pvs.get_avpvs_wo_buffer_file_path()
    output_file = pvs.get_avpvs_file_path()
    bufferstring = buffer_string(pvs.get_buff_events_media_time())
    pix_fmt = pvs.get_pix_fmt_for_avpvs()
    overwrite_spec = "-f" if force else ""
    if pvs.has_framefreeze():
        stalling_type_options = "-e --skipping"
    else:
        stalling_type_options = "-s {}".format(spinner_path)
    if _backend == "gpu":
        args = ["-y" if force else "-n", "--input", input_file, "--buffer", bufferstring, "--pix-fmt", pix_fmt,
                "--black-frame", "--vopts", "-c:v ffv1", "--aopts", "-c:a pcm_s16le"]
        args += ["--skipping"] if pvs.has_framefreeze() else ["--spinner", spinner_path]
        return _collapse(_gpu_cli("stall", args + [output_file]))
    return ("bufferer -i {input_file} -o {output_file} -b {bufferstring} --force-framerate --black-frame"
            " -v ffv1 -a pcm_s16le -x {pix_fmt} {stalling_type_options} {overwrite_spec}").format(**locals())
