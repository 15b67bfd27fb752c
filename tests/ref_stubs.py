"""Duck-typed stand-ins for the reference's domain objects (lib/test_config.py
Pvs/Src/Hrc/Segment/QualityLevel/PostProcessing/TestConfig), carrying exactly
the attributes the lib/ffmpeg.py builders read.  Used both by
tests/golden/gen_reference_fixtures.py (to drive the reference builders) and by
the tests (to drive pixpath.ffmpeg) from the same scenario dicts, so a
fixture is (scenario -> reference output)."""
import os
import types


class PostProcessing:
    def __init__(self, ptype, dw, dh, cw=None, ch=None, rate=60):
        self.processing_type = ptype
        self.display_width, self.display_height = dw, dh
        self.coding_width = cw if cw is not None else dw
        self.coding_height = ch if ch is not None else dh
        self.display_frame_rate = rate


class TestConfig:
    def __init__(self, root, ttype, pps):
        self.root = root
        self.type = ttype
        self.post_processings = pps

    def is_short(self):
        return self.type == "short"

    def is_long(self):
        return self.type == "long"

    def get_avpvs_path(self):
        return os.path.join(self.root, "avpvs")

    def get_cpvs_path(self):
        return os.path.join(self.root, "cpvs")

    def get_video_segments_path(self):
        return os.path.join(self.root, "videoSegments")

    def get_logs_path(self):
        return os.path.join(self.root, "logs")

    def get_src_vid_path(self):
        return os.path.join(self.root, "srcVid")


class QualityLevel:
    def __init__(self, w, h, fps="original", codec="h264", ql_id="Q0"):
        self.width, self.height, self.fps, self.video_codec, self.ql_id = w, h, fps, codec, ql_id


class Src:
    def __init__(self, tc, w, h, pix_fmt="yuv420p", fps=60, name="SRC001.avi"):
        self.test_config = tc
        self.stream_info = {"coded_width": w, "coded_height": h, "width": w, "height": h,
                            "pix_fmt": pix_fmt, "r_frame_rate": str(fps)}
        self._fps = fps
        self.filename = name
        self.file_path = os.path.join(tc.get_src_vid_path(), name)
        self.is_youtube = False

    def get_fps(self):
        return float(self._fps)

    def get_src_file_path(self):
        return self.file_path

    def uses_10_bit(self):
        return ("10" in self.stream_info["pix_fmt"]) and (self.stream_info["pix_fmt"] != "yuv410p")


class Segment:
    def __init__(self, tc, src, ql, index, start, duration, target_pix_fmt, name=None):
        self.src, self.quality_level, self.index = src, ql, index
        self.start_time, self.duration = start, duration
        self.target_pix_fmt = target_pix_fmt
        name = name or "DB_%s_%s_VC01_%04d_%d-%d.mp4" % (src.filename.split(".")[0], ql.ql_id, index,
                                                          int(start), int(start + duration))
        self.filename = name
        self.file_path = os.path.join(tc.get_video_segments_path(), name)
        self.tmp_path = os.path.join(tc.get_avpvs_path(), "tmp_" + name + ".avi")

    def get_segment_file_path(self):
        return self.file_path

    def get_tmp_path(self):
        return self.tmp_path

    def get_segment_duration(self):
        return self.duration


class Event:
    def __init__(self, etype, duration):
        self.event_type, self.duration = etype, duration


class Hrc:
    def __init__(self, events):
        self.event_list = [Event(t, d) for t, d in events]

    def has_buffering(self):
        return any(e.event_type in ("stall", "freeze") for e in self.event_list)

    def has_framefreeze(self):
        return any(e.event_type == "freeze" for e in self.event_list)

    def get_long_hrc_duration(self):
        return sum(float(e.duration) for e in self.event_list)


class Pvs:
    def __init__(self, tc, pvs_id, src, hrc, segments):
        self.test_config, self.pvs_id, self.src, self.hrc, self.segments = tc, pvs_id, src, hrc, segments

    def has_buffering(self):
        return self.hrc.has_buffering()

    def has_framefreeze(self):
        return self.hrc.has_framefreeze()

    def get_avpvs_file_path(self):
        return os.path.join(self.test_config.get_avpvs_path(), self.pvs_id + ".avi")

    def get_avpvs_wo_buffer_file_path(self):
        return os.path.join(self.test_config.get_avpvs_path(), self.pvs_id + "_concat_wo_buffer.avi")

    def get_tmp_wo_audio_path(self):
        return os.path.join(self.test_config.get_avpvs_path(), self.pvs_id + "_concat_wo_audio.avi")

    def get_avpvs_file_list(self):
        return os.path.join(self.test_config.get_avpvs_path(), self.pvs_id + "_tmp_filelist.txt")

    def get_cpvs_file_path(self, context="pc", rawvideo=False):
        ext = (".mkv" if rawvideo else ".avi") if context == "pc" else ".mp4"
        return os.path.join(self.test_config.get_cpvs_path(), self.pvs_id + "_" + context[0:2].upper() + ext)

    def get_preview_file_path(self):
        return os.path.join(self.test_config.get_cpvs_path(), self.pvs_id + "_preview.mov")


def build(sc, root, pvs_methods):
    """Scenario dict -> (test_config, pvs, post_processings).  ``pvs_methods``
    provides get_pix_fmt_for_avpvs(pvs), get_vcodec_and_pix_fmt_for_cpvs(pvs,
    rawvideo), get_buff_events_media_time(pvs) and hrc_get_buff_events_media_time(hrc)
    -- the reference's (fixture generation) or pixpath's (tests)."""
    pps = [PostProcessing(*p) for p in sc["pps"]]
    tc = TestConfig(root, sc.get("type", "short"), pps)
    src = Src(tc, sc["src"][0], sc["src"][1], sc.get("src_pix_fmt", "yuv420p"), sc.get("src_fps", 60))
    segs = []
    t = 0
    for i, (qw, qh, dur) in enumerate(sc["segments"]):
        ql = QualityLevel(qw, qh, ql_id="Q%d" % i)
        segs.append(Segment(tc, src, ql, i, t, dur, sc["target_pix_fmt"]))
        t += dur
    hrc = Hrc(sc.get("events", [("quality_level", segs[0].duration)]))
    hrc.get_buff_events_media_time = types.MethodType(pvs_methods.hrc_get_buff_events_media_time, hrc)
    pvs = Pvs(tc, sc.get("pvs_id", "P2SXM00_SRC001_HRC001"), src, hrc, segs)
    pvs.get_pix_fmt_for_avpvs = types.MethodType(pvs_methods.get_pix_fmt_for_avpvs, pvs)
    pvs.get_vcodec_and_pix_fmt_for_cpvs = types.MethodType(pvs_methods.get_vcodec_and_pix_fmt_for_cpvs, pvs)
    pvs.get_buff_events_media_time = types.MethodType(pvs_methods.get_buff_events_media_time, pvs)
    return tc, pvs, pps
