// p02 byte scanners: per-frame sizes of Annex-B H.264/H.265 and IVF (VP9)
// bitstreams, restating lib/get_framesize.py.
//
// The reference walks the file one byte at a time in Python, keeping the last
// five bytes as hex strings (get_framesize_h264 :144-201, get_framesize_h265
// :204-263) or seeking through the IVF frame headers (get_framesize_vp9
// :87-141).  Everything between two start codes only advances a counter, so
// the scan here jumps from one 0x01 byte to the next with memchr (SIMD in
// glibc) and evaluates the state machine only at start codes -- the output is
// the reference's, quirks included:
//   * a start code is 00 00 01; a frame's size runs from the byte after the
//     previous start code's 01 to 3 (or 5, when 00 00 00 01) bytes before the
//     next 01 -- i.e. leading zero_byte / trailing_zero bytes are attributed
//     like the reference does;
//   * the H.264 test is made on hex(byte): low digit 1 or 5 and, for bytes
//     >= 0x10, an even high digit -- which raises ValueError (int('a')) for
//     0xa1..0xf5 headers; reported as PP_ERR_INVALID with that message;
//   * the H.265 test keeps types 0..9 and 16..21 (bytes < 0x14, 0x20..0x2b);
//   * the last frame counts to the end of the file +3 (H.264) / +0 (H.265);
//   * IVF: only the low 24 bits of the 32-bit frame size are read, and the
//     "10" frame-marker check only counts misdetections (the reference prints
//     and carries on).
// Host-only code: no device work (a few MB per segment; the file read bounds it).
#include <cstring>

#include "common.hpp"

namespace {

// H.264 NAL header test of get_framesize_h264:180 on hex(b); -1 = ValueError
int h264_is_frame(unsigned b) {
    const unsigned lo = b & 15, hi = b >> 4;
    if (lo != 1 && lo != 5) return 0;
    if (b < 16) return 1;      // hex digit [-2] is 'x'
    if (hi >= 10) return -1;   // int('a'..'f') raises
    return hi % 2 == 0;
}

// H.265 NAL header test of get_framesize_h265:241 on hex(b)
int h265_is_frame(unsigned b) {
    const unsigned lo = b & 15, hi = b >> 4;
    return b < 16 || (hi == 1 && lo < 4) || (hi == 2 && lo < 12);
}

}  // namespace

extern "C" int64_t pp_annexb_frame_sizes(const uint8_t *buf, int64_t n, int codec, int64_t *sizes, int64_t cap) {
    if (n < 0 || cap < 0 || (n > 0 && !buf) || (cap > 0 && !sizes)) PP_FAIL(PP_ERR_INVALID, "null argument");
    if (codec != PP_NAL_H264 && codec != PP_NAL_H265) PP_FAIL(PP_ERR_INVALID, "codec %d", codec);
    int64_t cnt = 0;
    auto emit = [&](int64_t v) {
        if (cnt < cap) sizes[cnt] = v;
        ++cnt;
    };
    if (n == 0) return 0;
    int64_t r = -1;         // byte index where the reference's counter was last reset
    bool is_frame = false;
    int64_t k0 = 2;         // a start code ends at index >= 2
    while (k0 < n) {
        const void *hit = std::memchr(buf + k0, 1, (size_t)(n - k0));
        if (!hit) break;
        const int64_t k = static_cast<const uint8_t *>(hit) - buf;
        k0 = k + 1;
        if (buf[k - 1] != 0 || buf[k - 2] != 0) continue;
        const int64_t cur = k - r;
        if (is_frame) emit(k >= 4 && buf[k - 3] == 0 && buf[k - 4] == 0 ? cur - 5 : cur - 3);
        is_frame = false;
        r = k;
        if (k + 1 < n) {  // the NAL header byte, read while the counter is 1
            const unsigned h = buf[k + 1];
            const int f = codec == PP_NAL_H264 ? h264_is_frame(h) : h265_is_frame(h);
            if (f < 0) PP_FAIL(PP_ERR_INVALID, "ValueError: invalid literal for int() with base 10: '%c'", "0123456789abcdef"[h >> 4]);
            is_frame = f != 0;
        }
    }
    if (is_frame) {
        const int64_t cur = (n - 1) - r;
        emit(codec == PP_NAL_H264 ? cur + 3 : cur);
    }
    return cnt;
}

extern "C" int64_t pp_ivf_frame_sizes(const uint8_t *buf, int64_t n, int64_t *sizes, int64_t cap,
                                      int64_t *misdetected) {
    if (n < 0 || cap < 0 || (n > 0 && !buf) || (cap > 0 && !sizes)) PP_FAIL(PP_ERR_INVALID, "null argument");
    int64_t cnt = 0, mis = 0;
    int64_t pos = 32;  // IVF file header
    while (pos + 3 <= n) {
        const int64_t size = (int64_t)buf[pos] | ((int64_t)buf[pos + 1] << 8) | ((int64_t)buf[pos + 2] << 16);
        if (cnt < cap) sizes[cnt] = size;
        ++cnt;
        pos += 3 + 9;  // rest of the 12-byte frame header
        const int64_t got = pos >= n ? 0 : (n - pos < 3 ? n - pos : 3);
        if (got == 3 && (buf[pos] >> 6) != 2) ++mis;  // frame_marker "10"
        pos += got + size - 3;
    }
    if (misdetected) *misdetected = mis;
    return cnt;
}
