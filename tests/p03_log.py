"""Provenance of the commands the drop-in builders return.

The reference writes every command of a PVS into `logs/<pvs>.log` as an
`ffmpegCommand:` line, with the segment, log and SRC directories stripped
(write_to_p03_logfile, p03_generateAvPvs.py:41-59).  The gpu backend's
commands go through the same function unchanged, so the log records what ran:
the `pixpath.cli` subcommand, and for the AVPVS writers the codec and slice
grid (`--gpu-ffv1 --ffv1-slices HxV`, pixpath.ffmpeg._gpu_cli), or with
PIXPATH_FFV1=ffmpeg the reference's own `-c:v ffv1 ... -coder 1 -context 1
-slicecrc 1` options.  The AVI itself carries the same tag (RIFF INFO ISFT,
pixpath.ffv1.provenance).

p03_log_line restates that line for the tests (test helper, not product code).
"""


def p03_log_line(cmd, video_segments_path, src_vid_path, logs_dir=None):
    """The `ffmpegCommand:` line p03 writes for `cmd` (p03_generateAvPvs.py:51-59)."""
    line = cmd.replace(video_segments_path + "/", "")
    if logs_dir is not None:
        line = line.replace(logs_dir + "/", "")
    for src in (src_vid_path if isinstance(src_vid_path, list) else [src_vid_path]):
        line = line.replace(src + "/", "")
    return "ffmpegCommand: " + line
