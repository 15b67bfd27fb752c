// Host-side fuzzer of libpixpath's parsers of untrusted bytes (SURVEY.md
// section 5: sanitizer builds of the host code).  Built by `make sanitize`
// with g++ -fsanitize=address,undefined and no GPU code; run by
// tests/test_host_sanitize.py.  Every input comes from a seeded generator:
//
//   * FFV1 configuration records (ffv1host.cpp ffv1_parse_record): pixpath's
//     own records for every format / slice grid, then bit flips, byte
//     overwrites, truncations, extensions and random buffers -- a valid record
//     must parse back to what was written, a corrupt one may fail but must
//     never read outside its buffer;
//   * FFV1 frame packets (ffv1_slice_table, the footer walk the decoder's host
//     side does on every packet of an AVPVS file): frames with valid 24-bit
//     slice-size footers, then corrupt footers, sizes (negative, zero, larger
//     than the buffer) -- on success every slice lies inside its frame and the
//     slices tile it;
//   * the p02 bitstream scanners (scan.cpp pp_annexb_frame_sizes,
//     pp_ivf_frame_sizes) on random and start-code-laden buffers;
//   * the swscale filter construction (filters.cpp FilterBank::build /
//     compact) for random sizes, flags and parameters.
//
//   * general FFV1 records given as seeds (file of u32-LE-length-prefixed
//     records: the oracle's FFmpeg-like records with transmitted state
//     tables, 5-input table sets and initial states) -- each must parse, then
//     its mutations must never read outside the buffer.
//
// usage: fuzz_host [iterations (default 20000)] [seed] [seed-record file]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ffv1host.hpp"
#include "filters.hpp"

namespace pp {
// the library's error sink (api.cpp in the product build)
void set_error(const char *fmt, ...) { (void)fmt; }
}  // namespace pp

extern "C" int64_t pp_annexb_frame_sizes(const uint8_t *buf, int64_t n, int codec, int64_t *sizes, int64_t cap);
extern "C" int64_t pp_ivf_frame_sizes(const uint8_t *buf, int64_t n, int64_t *sizes, int64_t cap,
                                      int64_t *misdetected);

namespace {

using namespace pp;

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
    uint64_t next() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    }
    int below(int n) { return n > 0 ? (int)(next() % (uint64_t)n) : 0; }
};

int g_fail = 0;
#define CHECK(cond, ...)                                        \
    do {                                                        \
        if (!(cond)) {                                          \
            std::fprintf(stderr, "CHECK failed: " __VA_ARGS__); \
            std::fprintf(stderr, "\n");                         \
            ++g_fail;                                           \
        }                                                       \
    } while (0)

// a heap copy of exactly n bytes, so ASan flags any read past the end
std::vector<uint8_t> exact(const std::vector<uint8_t> &v) { return std::vector<uint8_t>(v.begin(), v.end()); }

void mutate(Rng &r, std::vector<uint8_t> &b) {
    const int kind = r.below(6);
    if (b.empty() || kind == 5) {
        b.resize(r.below(64));
        for (auto &x : b) x = (uint8_t)r.next();
        return;
    }
    switch (kind) {
    case 0: b[r.below((int)b.size())] ^= (uint8_t)(1u << r.below(8)); break;  // bit flip
    case 1: b[r.below((int)b.size())] = (uint8_t)r.next(); break;              // byte overwrite
    case 2: b.resize(r.below((int)b.size())); break;                            // truncation
    case 3:                                                                     // extension
        for (int k = r.below(16) + 1; k; --k) b.push_back((uint8_t)r.next());
        break;
    default:                                                                    // several flips
        for (int k = r.below(8) + 2; k; --k) b[r.below((int)b.size())] ^= (uint8_t)r.next();
    }
}

long fuzz_records(Rng &r, int iters) {
    static const int fmts[][3] = {{8, 1, 1}, {8, 1, 0}, {10, 1, 1}, {10, 1, 0}};
    long n = 0;
    for (int it = 0; it < iters; ++it) {
        const int *f = fmts[r.below(4)];
        const int nh = 1 + r.below(16), nv = 1 + r.below(16);
        const int w = 64 * (1 + r.below(30)), h = 64 * (1 + r.below(17));
        std::vector<uint8_t> rec = ffv1_write_record(f[0], f[1], f[2], nh, nv, ffv1_default_quant(f[0]));
        pp::Ffv1Record out;
        std::string err;
        if (it % 8 == 0) {  // the valid record round trips
            std::vector<uint8_t> b = exact(rec);
            const int rc = ffv1_parse_record(b.data(), (int)b.size(), w, h, &out, &err);
            CHECK(rc == 0 && out.bits == f[0] && out.hsub == f[1] && out.vsub == f[2] && out.nh == nh &&
                      out.nv == nv && out.ec == 1 && out.ntables == 1 && out.ctx_count[0] == ffv1_default_quant(f[0]).contexts() && out.intra == 1 &&
                      out.coder == 1,
                  "record %d/%d/%d %dx%d did not round trip: %d %s", f[0], f[1], f[2], nh, nv, rc, err.c_str());
        }
        std::vector<uint8_t> m = rec;
        for (int k = 1 + r.below(3); k; --k) mutate(r, m);
        std::vector<uint8_t> b = exact(m);
        (void)ffv1_parse_record(b.empty() ? nullptr : b.data(), (int)b.size(), w, h, &out, &err);
        ++n;
    }
    return n;
}

long fuzz_seed_records(Rng &r, int iters, const char *path) {
    std::vector<std::vector<uint8_t>> seeds;
    if (FILE *f = std::fopen(path, "rb")) {
        uint8_t hdr[4];
        while (std::fread(hdr, 1, 4, f) == 4) {
            const uint32_t n = hdr[0] | hdr[1] << 8 | hdr[2] << 16 | (uint32_t)hdr[3] << 24;
            std::vector<uint8_t> b(n);
            if (std::fread(b.data(), 1, n, f) != n) break;
            seeds.push_back(std::move(b));
        }
        std::fclose(f);
    }
    CHECK(!seeds.empty(), "no seed records in %s", path);
    long n = 0;
    for (size_t k = 0; k < seeds.size(); ++k) {
        pp::Ffv1Record out;
        std::string err;
        std::vector<uint8_t> b = exact(seeds[k]);
        const int rc = ffv1_parse_record(b.data(), (int)b.size(), 1920, 1080, &out, &err);
        CHECK(rc == 0, "seed record %zu refused: %s", k, err.c_str());
    }
    for (int it = 0; it < iters && !seeds.empty(); ++it) {
        std::vector<uint8_t> m = seeds[r.below((int)seeds.size())];
        for (int k = 1 + r.below(3); k; --k) mutate(r, m);
        std::vector<uint8_t> b = exact(m);
        pp::Ffv1Record out;
        std::string err;
        (void)ffv1_parse_record(b.empty() ? nullptr : b.data(), (int)b.size(), 1920, 1080, &out, &err);
        ++n;
    }
    return n;
}

long fuzz_packets(Rng &r, int iters) {
    long n = 0;
    for (int it = 0; it < iters; ++it) {
        const int per = 1 + r.below(16), nframes = 1 + r.below(4), ec = r.below(2);
        const int trailer = 3 + 5 * ec;
        std::vector<uint8_t> pk;
        std::vector<int64_t> sizes;
        for (int f = 0; f < nframes; ++f) {
            const size_t base = pk.size();
            for (int s = 0; s < per; ++s) {
                const int len = r.below(200);
                for (int k = 0; k < len; ++k) pk.push_back((uint8_t)r.next());
                for (int k = 0; k < trailer - 3; ++k) pk.push_back((uint8_t)r.next());
                pk.push_back((uint8_t)(len >> 16));
                pk.push_back((uint8_t)(len >> 8));
                pk.push_back((uint8_t)len);
            }
            sizes.push_back((int64_t)(pk.size() - base));
        }
        // mutate footers, payload bytes or the frame sizes
        const int kind = r.below(5);
        if (kind == 1 && !pk.empty()) {
            for (int k = 1 + r.below(4); k; --k) pk[r.below((int)pk.size())] = (uint8_t)r.next();
        } else if (kind == 2) {
            sizes[r.below(nframes)] += r.below(41) - 20;
        } else if (kind == 3) {
            sizes[r.below(nframes)] = -(int64_t)r.below(1000) - 1;
        } else if (kind == 4 && !pk.empty()) {
            pk.resize(r.below((int)pk.size()));
            int64_t tot = 0;
            for (auto &s : sizes) {  // frame sizes past the truncation are cut to what is left
                s = std::max<int64_t>(0, std::min<int64_t>(s, (int64_t)pk.size() - tot));
                tot += s;
            }
        }
        int64_t total_sz = 0;
        bool sizes_ok = true;
        for (int64_t s : sizes) {
            sizes_ok = sizes_ok && s >= 0;
            total_sz += s;
        }
        if (!sizes_ok || total_sz > (int64_t)pk.size()) {
            // a caller hands over its own buffer of the sizes it claims: skip
            // lies about the buffer length, keep negative sizes (must be refused)
            if (sizes_ok) continue;
        }
        std::vector<uint8_t> b = exact(pk);
        std::vector<int64_t> soff((size_t)nframes * per, -1), slen((size_t)nframes * per, -1);
        int64_t total = -1;
        std::string err;
        const int rc = ffv1_slice_table(b.empty() ? nullptr : b.data(), sizes.data(), nframes, per, ec,
                                        soff.data(), slen.data(), &total, &err);
        ++n;
        if (rc == 0) {
            int64_t base = 0;
            for (int f = 0; f < nframes; ++f) {
                int64_t at = base;
                for (int s = 0; s < per; ++s) {
                    const int64_t o = soff[(size_t)f * per + s], l = slen[(size_t)f * per + s];
                    CHECK(o == at && l >= trailer && o + l <= base + sizes[f], "slice %d of frame %d outside", s, f);
                    at = o + l;
                }
                CHECK(at == base + sizes[f], "frame %d slices do not tile it", f);
                base += sizes[f];
            }
            CHECK(total == base, "total %lld != %lld", (long long)total, (long long)base);
        } else {
            CHECK(!err.empty(), "failure without a message");
        }
    }
    return n;
}

long fuzz_scanners(Rng &r, int iters) {
    long n = 0;
    for (int it = 0; it < iters; ++it) {
        std::vector<uint8_t> buf(r.below(4096));
        for (auto &x : buf) x = (uint8_t)(r.below(4) ? r.below(3) : r.next());  // many 0x00 / 0x01 bytes
        if (it % 3 == 0 && buf.size() > 32) {  // an IVF-like header
            std::memcpy(buf.data(), "DKIF", 4);
            buf[6] = 32;
        }
        std::vector<uint8_t> b = exact(buf);
        std::vector<int64_t> sizes(r.below(64));
        int64_t mis = 0;
        const uint8_t *p = b.empty() ? nullptr : b.data();
        (void)pp_annexb_frame_sizes(p, (int64_t)b.size(), 1 + r.below(2), sizes.empty() ? nullptr : sizes.data(),
                                    (int64_t)sizes.size());
        (void)pp_ivf_frame_sizes(p, (int64_t)b.size(), sizes.empty() ? nullptr : sizes.data(), (int64_t)sizes.size(),
                                 &mis);
        n += 2;
    }
    return n;
}

long fuzz_filters(Rng &r, int iters) {
    static const int flags[] = {PP_SWS_BICUBIC, PP_SWS_LANCZOS, PP_SWS_BILINEAR};
    long n = 0;
    for (int it = 0; it < iters; ++it) {
        const int src = 4 + r.below(r.below(2) ? 64 : 4096), dst = 1 + r.below(r.below(2) ? 64 : 4096);
        const int xinc = (int)((((int64_t)src << 16) + (dst >> 1)) / dst);
        pp::FilterBank fb;
        std::string err;
        const double p0 = r.below(4) ? PP_SWS_PARAM_DEFAULT : (double)r.below(10);
        if (fb.build(xinc, src, dst, r.below(2) ? 4 : 2, r.below(2) ? 1 << 14 : 1 << 12, flags[r.below(3)], p0,
                     PP_SWS_PARAM_DEFAULT, pp::local_pos(r.below(2)), pp::local_pos(r.below(2)), &err) == 0) {
            pp::FilterBank::Compact c;
            if (fb.compact(src, 1 + r.below(8), &c, &err) == 0) {
                // a window wider than the plane starts at 0 (the kernel zero-fills
                // past the edge); every non-zero tap reads inside the plane
                for (int i = 0; i < dst; ++i) {
                    CHECK(c.pos[i] >= 0 && (c.pos[i] + c.taps <= src || c.pos[i] == 0), "window %d at %d", i,
                          c.pos[i]);
                    for (int k = 0; k < c.taps; ++k)
                        if (c.coef[(size_t)i * c.taps + k])
                            CHECK(c.pos[i] + k < src, "tap %d of output %d outside [0, %d)", k, i, src);
                }
            }
        }
        ++n;
    }
    return n;
}

}  // namespace

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    const uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1;
    Rng r(seed);
    const long a = fuzz_records(r, iters);
    const long b = fuzz_packets(r, iters);
    const long c = fuzz_scanners(r, iters / 4);
    const long d = fuzz_filters(r, iters / 20);
    const long e = argc > 3 ? fuzz_seed_records(r, iters, argv[3]) : 0;
    std::printf("records %ld packets %ld scans %ld filters %ld seeded %ld failures %d\n", a, b, c, d, e, g_fail);
    return g_fail ? 1 : 0;
}
