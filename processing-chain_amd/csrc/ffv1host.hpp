// Host side of the FFV1 codec: the range-coder
// state tables, the CRC, the configuration record (written by the encoder,
// parsed and checked by the decoder) and the walk of a frame packet's slice
// footers.  Plain C++ with no HIP dependency, so it also builds on its own
// under ASan / UBSan (`make sanitize`, csrc/fuzz_host.cpp) and is fuzzed with
// corrupt records and packets -- every byte it reads comes from a file.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace pp {

constexpr int kFfv1CtxBytes = 32;  // state bytes per context
constexpr int kFfv1MaxCtx = 16384; // (32768 + 1) / 2: read_quant_tables' bound on one set
constexpr int kFfv1MaxTables = 8;  // MAX_QUANT_TABLES

// ff_build_rac_states(c, 0.05 * 2^32, 256 - 8): the default state-transition table
void rac_states(uint8_t zero[256], uint8_t one[256]);
// AV_CRC_32_IEEE: polynomial 0x04C11DB7, MSB first, initial 0, no final xor
void crc_table(uint32_t t[256]);
// A 3-input threshold quantiser: the level of |d| (d = 0..127) is the number
// of thresholds <= |d|, odd-mirrored for d = 128..255 (read_quant_table's
// shape; every FFV1 input quantiser has it).  Ffv1Quant() is thresholds 1, 2,
// 4, 8, 16 = min(5, bit length |d|): 11 levels, (11^3 + 1) / 2 = 666 contexts
// (pixpath's encoder up to round 5); the encoder now writes ffv1_default_quant.
struct Ffv1Quant {
    int n = 5;
    int thr[5] = {1, 2, 4, 8, 16};
    int levels() const { return 2 * n + 1; }
    int contexts() const { return (levels() * levels() * levels() + 1) / 2; }
};
int ffv1_quant(int i, const Ffv1Quant &q);
// The quantiser pixpath's encoder writes for a bit depth (oracle/ffv1_oracle.c
// oracle_quant restates the same rule).
Ffv1Quant ffv1_default_quant(int depth);

// The configuration record (RFC 9043 4.2, ffv1enc.c write_extradata) of
// pixpath's encoder: version 3, range coder with the default table, one
// 3-input quantisation set (q), slice CRCs, intra; CRC-32 parity appended.
std::vector<uint8_t> ffv1_write_record(int depth, int hsub, int vsub, int slices_h, int slices_v,
                                       const Ffv1Quant &q);

// What the decoder needs from a configuration record (RFC 9043 4.2,
// ffv1dec.c read_extra_header): version 3, range coder with the default
// (coder_type 1) or a transmitted (2) state-transition table, YCbCr with
// chroma planes and no alpha, 8..10 bits, 4:2:0 / 4:2:2 / 4:4:4, up to 8
// quantisation table sets of up to 5 inputs, optional initial context states
// per set, slice CRCs or not, intra or inter.
struct Ffv1Record {
    int bits = 8, hsub = 1, vsub = 1, nh = 1, nv = 1, ec = 0, intra = 1, micro = 0, coder = 1;
    int ntables = 0;
    int ctx_count[kFfv1MaxTables] = {};
    int max_ctx = 0;                            // largest set: the decoder's per-plane state slots
    int16_t quant[kFfv1MaxTables][5][256];      // scaled, mirrored (read_quant_tables)
    uint8_t zero_state[256], one_state[256];    // the slice coders' table
    std::vector<uint8_t> init[kFfv1MaxTables];  // [ctx_count][32] when transmitted, else empty (128s)
};

// Parse and check a configuration record for a w x h stream: 0 (PP_OK), or a
// negative PP_ERR_* with *err set.  Never reads outside extra[0, size).
int ffv1_parse_record(const uint8_t *extra, int size, int w, int h, Ffv1Record *rec, std::string *err);

// The keyframe flag of a frame packet: the first range-coded decision of
// its first slice (at state 128, before any table is involved).
int ffv1_keyframe_bit(const uint8_t *slice0, int64_t n);

// The slice table of `nframes` packets held back to back (frame_sizes[f]
// bytes each): every frame's slice footers walked backwards from the packet
// end (ffv1dec.c decode_frame), slice i of frame f at soff[f * per + i] with
// slen bytes (footer included).  0, or a negative PP_ERR_* with *err set.
int ffv1_slice_table(const uint8_t *packets, const int64_t *frame_sizes, int nframes, int per, int ec,
                     int64_t *soff, int64_t *slen, int64_t *total, std::string *err);

}  // namespace pp
