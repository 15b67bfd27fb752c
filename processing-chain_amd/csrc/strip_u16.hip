// strip_kernel instances for 16-bit (9/10-bit) source samples, plain plans (see
// strip.hpp); the chain and packed instances are in strip_u16_chain.hip, so the
// two units compile in parallel.
#include "strip.hpp"

namespace pp {

KernelFn pick_strip_u16(int outb, int hw, int vtm, int tw) {
    if (outb == 8) {
        PP_STRIP_HW(uint16_t, 8)
    }
    PP_STRIP_HW(uint16_t, 10)
}

int strip_vtm_bucket(int vtp) { return strip_vtm_bucket_impl(vtp); }

}  // namespace pp
