"""ffprobe metadata exactly as the reference gathers it (SRC_analysis and
complexity hooks).

Mirrors, with the same ffprobe command strings and the same fallbacks:
  get_stream_size   lib/ffmpeg.py:399-417  (packet-size sum; reads <file>.yaml if present)
  get_src_info      lib/ffmpeg.py:566-633  (first video stream; r_frame_rate "a/b" ->
                                            str(int(a/b)), truncating: 60000/1001 -> "59")
  get_segment_info  lib/ffmpeg.py:433-563  (duration from the stream, else its DURATION
                                            tag, else the last packets' dts + durations;
                                            bitrates from bit_rate, else the stream size)
Pinned byte-for-byte against the reference's own outputs
(tests/golden/src_analysis_fixtures.json, tests/test_src_analysis_parity.py).

Deliberate difference: the reference's get_src_info, reached from analyse_src
with info_path=False, also stats and writes file descriptor 0
(open(False, 'w'), lib/ffmpeg.py:603, :627) -- printing a second YAML on a
terminal and closing stdin, so a second analyse_src in the same process fails
with EBADF.  pixpath writes only <src>.yaml.

Failure convention as the reference's cmd_utils.run_command (lib/cmd_utils.py:
132-148): a failing command logs its stdout/stderr and exits 1.
"""
import json
import logging
import os
import subprocess
import sys
from collections import OrderedDict
from fractions import Fraction

logger = logging.getLogger("main")


def run_command(cmd, name=""):
    """Shell command -> (stdout, stderr); on failure log and sys.exit(1)."""
    logger.debug("starting command: %s", cmd)
    x = subprocess.run(cmd, shell=True, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    out, err = str(x.stdout, "utf-8"), str(x.stderr, "utf-8")
    if x.returncode != 0:
        logger.error("Error running command: %s\nstdout: %s\nstderr: %s", cmd, out, err)
        sys.exit(1)
    return out, err


def _load_yaml(path):
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def get_stream_size(file_path, stream_type="video"):
    """Bytes of the video ("video") or audio stream: the sum of its packet sizes."""
    switch = "v" if stream_type == "video" else "a"
    if os.path.isfile(file_path + ".yaml"):
        return _load_yaml(file_path + ".yaml")["get_stream_size"][switch]
    cmd = ("ffprobe -loglevel error -select_streams " + switch +
           " -show_entries packet=size -of compact=p=0:nk=1  '" + file_path + "'")
    stdout, _ = run_command(cmd, name="get accumulated frame size for " + file_path)
    return sum(int(ll) for ll in stdout.split("\n") if ll != "")


def get_src_info(file_path):
    """ffprobe's first video stream (dict), r_frame_rate normalised to an integer string."""
    cmd = "ffprobe -loglevel error -select_streams v -show_streams -of json '" + file_path + "'"
    stdout, _ = run_command(cmd, name="get SRC info for " + file_path)
    info = json.loads(stdout)["streams"][0]
    if "/" in info["r_frame_rate"]:
        num, den = info["r_frame_rate"].split("/")
        info["r_frame_rate"] = str(int(int(num) / int(den)))
    return info


def _tag_duration(duration_str):
    hms, msec = duration_str.split(".")
    total = sum(int(x) * 60 ** i for i, x in enumerate(reversed(hms.split(":"))))
    return total + float("0." + msec)


def fix_video_profile_string(video_profile):
    """lib/ffmpeg.py:420-430."""
    for a, b in ((" ", ""), ("Profile", ""), ("High", "Hi"), (":", ""), ("Predictive", "P")):
        video_profile = video_profile.replace(a, b)
    return video_profile


def get_segment_info(file_path, filename="random", quality_level=None):
    """OrderedDict of segment_filename, file_size, video_* (and audio_*) keys."""
    size_cmd = ("stat -f '%z' '" if sys.platform == "darwin" else "stat -c '%s' '") + file_path + "'"
    stdout, _ = run_command(size_cmd, name="get segment size for " + file_path)
    segment_size = int(stdout.strip())
    stdout, _ = run_command("ffprobe -loglevel error -show_streams -of json '" + file_path + "'",
                            name="get segment video info for " + file_path)
    video_info = audio_info = None
    for st in json.loads(stdout)["streams"]:
        if st["codec_type"] == "video":
            video_info = st
        elif st["codec_type"] == "audio":
            audio_info = st
    if video_info is None:
        logger.error("No video stream found in segment " + file_path)
        sys.exit(1)

    if "duration" in video_info:
        video_duration = float(video_info["duration"])
    elif "DURATION" in video_info.get("tags", {}):
        video_duration = _tag_duration(video_info["tags"]["DURATION"])
    else:
        cmd = ("ffprobe -loglevel error -select_streams v -show_packets -show_entries "
               "packet=pts_time,dts_time,duration_time,size,flags -of json '" + file_path + "'")
        stdout, _ = run_command(cmd, name="get VFI for " + file_path)
        packets = json.loads(stdout)["packets"]
        index = -1
        while True:  # the last packet with both fields; the ones after it add one duration each
            pk = packets[index]
            if "dts_time" in pk and "duration_time" in pk:
                video_duration = float(pk["dts_time"]) + abs(index) * float(pk["duration_time"])
                break
            index -= 1
        logger.warning("Calculated duration of segment " + file_path + " manually. Might not be perfectly accurate.")
    if not video_duration:
        logger.error("Video duration of " + file_path + " was calculated as zero! "
                     "Make sure that the input file is correct.")
        sys.exit(1)

    if "bit_rate" in video_info:
        video_bitrate = round(float(video_info["bit_rate"]) / 1024.0, 2)
    else:
        video_bitrate = round((get_stream_size(file_path) * 8 / 1024.0) / video_duration, 2)
    target = quality_level.video_bitrate if quality_level is not None else 0
    profile = fix_video_profile_string(video_info["profile"]) if "profile" in video_info else ""
    ret = OrderedDict([
        ("segment_filename", filename), ("file_size", segment_size), ("video_duration", video_duration),
        ("video_frame_rate", float(Fraction(video_info["r_frame_rate"]))), ("video_bitrate", video_bitrate),
        ("video_target_bitrate", target), ("video_width", video_info["width"]),
        ("video_height", video_info["height"]), ("video_codec", video_info["codec_name"]),
        ("video_profile", profile)])
    if audio_info is not None:
        if "duration" in audio_info:
            audio_duration = float(audio_info["duration"])
        elif "DURATION" in audio_info.get("tags", {}):
            audio_duration = _tag_duration(audio_info["tags"]["DURATION"])
        elif "nb_frames" in audio_info:
            audio_duration = float(audio_info["nb_frames"]) / float(audio_info["sample_rate"])
        else:
            logger.error("Could not extract audio duration from " + file_path)
            sys.exit(1)
        if "bit_rate" in audio_info:
            audio_bitrate = round(float(audio_info["bit_rate"]) / 1024.0, 2)
        else:
            audio_bitrate = round((get_stream_size(file_path, stream_type="audio") * 8 / 1024.0) / audio_duration, 2)
        ret.update(OrderedDict([("audio_duration", audio_duration), ("audio_sample_rate", audio_info["sample_rate"]),
                                ("audio_codec", audio_info["codec_name"]), ("audio_bitrate", audio_bitrate)]))
    return ret
