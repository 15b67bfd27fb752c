// strip_kernel instances for 8-bit source samples, plain plans (see
// strip.hpp); the chain and packed instances are in strip_u8_chain.hip, so the
// two units compile in parallel.
#include "strip.hpp"

namespace pp {

KernelFn pick_strip_u8(int outb, int hw, int vtm, int tw) {
    if (outb == 8) {
        PP_STRIP_HW(uint8_t, 8)
    }
    PP_STRIP_HW(uint8_t, 10)
}

}  // namespace pp
