"""Stalling / freezing of an AVPVS (spec PP-STALL-1): the work of the external
`bufferer -i <wo_buffer.avi> -o <pvs>.avi -b <events> --force-framerate
--black-frame -v ffv1 -a pcm_s16le -x <pix_fmt> (-s <spinner> | -e --skipping)`
call of p03_generateAvPvs.py:215-260 (bufferer==0.22.1 is absent: parity
against it is unpinned, the rules below are this build's).

Video
  stall  [media_t, dur]: after input frame round(media_t*rate)-1, insert
         round(dur*rate) frames showing that frame (black when the stall is at
         t=0 and --black-frame is set) with the spinner centred and animated at
         its APNG frame delays (exact rational clock).
  freeze [t, dur] (--skipping): frames of [t, t+dur) are replaced by the frame
         before t (frame 0 when t=0); the length is unchanged.
Audio (pcm_s16le, as bufferer's -a)
  stall  the input audio is cut at each stall's media time and the stall's
         duration of silence (same rate and layout) is inserted, so audio and
         video stay aligned; freezes leave the audio unchanged.

`stall_schedule` is the whole output sequence for a known frame count (tests,
documentation); `StallStream` produces the same sequence while reading the
input once, holding only the last input frame (the AVPVS is never
materialised).
"""
from fractions import Fraction


def _spinner_clock(delays):
    ds = [Fraction(float(d)).limit_denominator(100000) for d in (delays if delays is not None else [0.0])]
    return ds, sum(ds)


def spinner_indices(k, rate, delays):
    """Spinner frame shown at each of the k stall frames (frame j at time j/rate)."""
    ds, period = _spinner_clock(delays)
    rate = Fraction(rate)
    out = []
    for j in range(k):
        ts = (Fraction(j) / rate) % period if period > 0 else Fraction(0)
        acc, si = Fraction(0), 0
        for si, dl in enumerate(ds):
            acc += dl
            if ts < acc:
                break
        out.append(si)
    return out


def stall_schedule(buffer_events, rate, n_in, skipping, spinner_delays=None, black_frame=True):
    """PP-STALL-1 output sequence for an AVPVS of n_in frames at `rate`: a list
    of (src_index, spinner_index); src_index -1 = black, spinner_index -1 = none."""
    rate = Fraction(rate)
    seq = [(i, -1) for i in range(n_in)]
    if skipping:
        for t, d in sorted(buffer_events):
            a = int(round(t * rate))
            b = min(n_in, int(round((t + d) * rate)))
            for i in range(a, b):
                seq[i] = (max(a - 1, 0), -1)
        return seq
    out, cursor = [], 0
    for t, d in sorted(buffer_events):
        at = min(n_in, int(round(t * rate)))
        out.extend(seq[cursor:at])
        cursor = at
        frozen = at - 1 if at > 0 else (-1 if black_frame else 0)
        out.extend((frozen, si) for si in spinner_indices(int(round(d * rate)), rate, spinner_delays))
    out.extend(seq[cursor:])
    return out


def stall_times(buffer_events, rate):
    """[(media time in s, duration in s)] of the inserted stalls, on the frame
    grid the video uses (at/rate, k/rate), sorted."""
    rate = Fraction(rate)
    return [(Fraction(int(round(t * rate))) / rate, Fraction(int(round(d * rate))) / rate)
            for t, d in sorted(buffer_events)]


class StallStream:
    """Streams an AVPVS through PP-STALL-1: ``run(frames, emit_input, emit_stall)``
    with ``frames`` an iterator of input frames in order; calls
    ``emit_input(frame)`` for an output frame that is an input frame (or a
    frozen copy) and ``emit_stall(frame_or_None, spinner_indices)`` for a run of
    stall frames (None = black).  The output equals stall_schedule's."""

    def __init__(self, buffer_events, rate, skipping, spinner_delays=None, black_frame=True):
        self.rate = Fraction(rate)
        self.skipping = skipping
        self.delays = spinner_delays
        self.black_frame = black_frame
        ev = sorted(buffer_events)
        if skipping:
            self.spans = [(int(round(t * self.rate)), int(round((t + d) * self.rate))) for t, d in ev]
        else:
            self.stalls = [(int(round(t * self.rate)), int(round(d * self.rate))) for t, d in ev]

    def run(self, frames, emit_input, emit_stall):
        p = self.pusher(emit_input, emit_stall)
        for f in frames:
            p.push(f)
        return p.close()

    def pusher(self, emit_input, emit_stall):
        """The same walk, frame by frame: ``push(frame)`` for every input frame
        in order, then ``close()`` (returns the input frame count).  Lets the
        AVPVS writer compose the stalled output while it writes the AVPVS.
        A pushed frame is referenced, not copied: it must stay valid until the
        next push (or close, for the last one); frames kept longer (freeze
        spans) are copied here."""
        return _FreezePush(self, emit_input) if self.skipping else _StallPush(self, emit_input, emit_stall)


class _StallPush:
    def __init__(self, s, emit_input, emit_stall):
        self.s, self.emit_input, self.emit_stall = s, emit_input, emit_stall
        self.last, self.i, self.k = None, 0, 0

    def push(self, f):
        s = self.s
        while self.k < len(s.stalls) and s.stalls[self.k][0] <= self.i:
            # a stall at t=0: black (--black-frame) or the first frame itself
            src = self.last if self.i > 0 else (None if s.black_frame else f)
            self.emit_stall(src, spinner_indices(s.stalls[self.k][1], s.rate, s.delays))
            self.k += 1
        self.emit_input(f)
        self.last, self.i = f, self.i + 1

    def close(self):
        s = self.s
        while self.k < len(s.stalls):  # stalls at or past the end show the last frame
            src = self.last if self.i > 0 else None
            self.emit_stall(src, spinner_indices(s.stalls[self.k][1], s.rate, s.delays))
            self.k += 1
        return self.i


class _FreezePush:
    def __init__(self, s, emit_input):
        self.s, self.emit_input = s, emit_input
        self.prev, self.i = None, 0
        self.held = {}  # span start a -> its frozen frame (the ORIGINAL frame a-1, or frame 0)

    def push(self, f):
        # the last span (in sorted order) covering i decides, as in stall_schedule
        owner = None
        for a, b in self.s.spans:
            if a <= self.i < b:
                owner = a
        for a, _ in self.s.spans:
            if a == self.i and a not in self.held:
                h = self.prev if a > 0 else f
                self.held[a] = h.copy() if hasattr(h, "copy") else h
        self.emit_input(f if owner is None else self.held[owner])
        self.prev, self.i = f, self.i + 1

    def close(self):
        return self.i


def stall_audio_graph(stalls, sample_rate, channel_layout):
    """ffmpeg -filter_complex graph on input 1's audio: cut at every stall's
    media time and insert that stall's duration of silence; output [aout].
    ``stalls``: stall_times() pairs.  None when there is nothing to insert."""
    stalls = [(t, d) for t, d in stalls if d > 0]
    if not stalls:
        return None
    n = len(stalls) + 1
    parts = ["[1:a]asplit=%d%s" % (n, "".join("[s%d]" % i for i in range(n)))]
    cat = []
    prev = Fraction(0)
    for i, (t, d) in enumerate(stalls):
        parts.append("[s%d]atrim=start=%s:end=%s,asetpts=PTS-STARTPTS[p%d]" % (i, _sec(prev), _sec(t), i))
        parts.append("anullsrc=r=%d:cl=%s,atrim=end=%s[z%d]" % (int(sample_rate), channel_layout, _sec(d), i))
        cat += ["[p%d]" % i, "[z%d]" % i]
        prev = t
    parts.append("[s%d]atrim=start=%s,asetpts=PTS-STARTPTS[p%d]" % (n - 1, _sec(prev), n - 1))
    cat.append("[p%d]" % (n - 1))
    parts.append("%sconcat=n=%d:v=0:a=1[aout]" % ("".join(cat), len(cat)))
    return ";".join(parts)


def _sec(x):
    """Seconds as a decimal ffmpeg accepts (exact for the frame grids used)."""
    x = Fraction(x)
    return ("%.9f" % float(x)).rstrip("0").rstrip(".") or "0"
