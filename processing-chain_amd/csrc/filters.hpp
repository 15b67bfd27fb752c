// Polyphase filter banks (FFmpeg initFilter restatement) -- see filters.cpp.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/pixpath.h"

namespace pp {

struct FilterBank {
    int n = 0;                 // outputs
    int size = 0;              // taps per output (FFmpeg layout, aligned)
    std::vector<int32_t> pos;  // first source sample per output
    std::vector<int16_t> coef; // n * size, sums to `one`

    struct Compact {
        int taps = 0;
        std::vector<int32_t> pos;
        std::vector<int16_t> coef; // n * taps
    };

    // xinc: 16.16 step; align: x86 filterAlign; one: 1<<14 (H) or 1<<12 (V);
    // src_pos/dst_pos: get_local_pos() chroma siting (128 = centre).
    int build(int xinc, int src_n, int dst_n, int align, int one, int flags, double p0, double p1,
              int src_pos, int dst_pos, std::string *err);
    // Re-window for the GPU: drop zero taps, width >= bucket_min, all windows in [0, src_n).
    int compact(int src_n, int bucket_min, Compact *out, std::string *err) const;
};

// get_local_pos() of libswscale/utils.c for the default (-513) siting.
inline int local_pos(int chr_subsample) {
    int pos = (128 << chr_subsample) - 128;
    pos += 128;
    return pos >> chr_subsample;
}

}  // namespace pp
