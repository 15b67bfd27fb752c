"""CPU oracle (TEST INFRASTRUCTURE ONLY -- imported by tests/ and bench.py's
cpu_baseline, never by the product) for the p02 frame-size scanners.

A byte-at-a-time restatement of lib/get_framesize.py's state machines on
integers instead of hex strings:
  annexb_sizes(data, "h264")  get_framesize_h264  lib/get_framesize.py:144-201
  annexb_sizes(data, "h265")  get_framesize_h265  lib/get_framesize.py:204-263
  ivf_sizes(data)             get_framesize_vp9   lib/get_framesize.py:87-141
Pinned against the reference's own outputs on the committed streams
(tests/golden/framesize_fixtures.json); the product scanner
(csrc/scan.cpp) is then fuzzed against it on random streams.
"""


def _h264_frame(b):
    # :180 -- hex(b)[-1] in '15' and (hex(b)[-2] == 'x' or int(hex(b)[-2]) % 2 == 0)
    s = hex(b)
    return (s[-1] == "5" or s[-1] == "1") and (s[-2] == "x" or int(s[-2]) % 2 == 0)


def _h265_frame(b):
    # :241
    s = hex(b)
    return s[-2] == "x" or (s[-2] == "1" and int(s[-1], 16) < 4) or (s[-2] == "2" and int(s[-1], 16) < 12)


def annexb_sizes(data, codec):
    test = _h264_frame if codec == "h264" else _h265_frame
    data = bytes(data)
    if not data:
        return []
    b = [None] * 5
    cur = 0
    is_frame = nal = False
    sizes = []
    for i, v in enumerate(data):
        b[0] = v
        cur += 1
        if b[0] == 1 and b[1] == 0 and b[2] == 0:
            nal = True
            if is_frame:
                sizes.append(cur - 5 if (b[3] == 0 and b[4] == 0) else cur - 3)
            is_frame = False
            cur = 0
        if nal and cur == 1:
            if test(b[0]):
                is_frame = True
            nal = False
        b[4], b[3], b[2], b[1] = b[3], b[2], b[1], b[0]
    if is_frame:
        sizes.append(cur + 3 if codec == "h264" else cur)
    return sizes


def ivf_sizes(data):
    """(sizes, frames whose first byte fails the '10' marker test)."""
    data = bytes(data)
    n = len(data)
    pos, sizes, mis = 32, [], 0
    while pos + 3 <= n:
        size = data[pos] | data[pos + 1] << 8 | data[pos + 2] << 16
        sizes.append(size)
        pos += 12
        got = max(0, min(3, n - pos))
        if got == 3 and data[pos] >> 6 != 2:
            mis += 1
        pos += got + size - 3
    return sizes, mis
