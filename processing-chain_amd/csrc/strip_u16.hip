// strip_kernel instances for 16-bit (9/10-bit) source samples (see strip.hpp).
#include "strip.hpp"

namespace pp {

KernelFn pick_strip_u16(int outb, int hw, int vtm, int tw) {
    if (outb == 8) {
        PP_STRIP_HW(uint16_t, 8)
    }
    PP_STRIP_HW(uint16_t, 10)
}

int strip_vtm_bucket(int vtp) { return strip_vtm_bucket_impl(vtp); }

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
