// strip_kernel instances for 16-bit (9/10-bit) source samples: chain plans
// (FUSE 8 / 10, create_avpvs_segment) and packed uyvy422 output (FUSE 1).
#include "strip.hpp"

namespace pp {

KernelFn pick_strip_chain_u16(int out2, int hw, int vtm) {
    if (out2 == 8) {
        PP_STRIP_HW_F(uint16_t, 8, 8)
    }
    PP_STRIP_HW_F(uint16_t, 8, 10)
}

KernelFn pick_strip_packed_u16(int hw, int vtm) {
    PP_STRIP_HW_F(uint16_t, 8, 1)
}

}  // namespace pp
