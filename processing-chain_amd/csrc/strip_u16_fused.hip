// strip_kernel instances for 16-bit (9/10-bit) source samples: the two launches of a
// 10-bit chain plan (create_avpvs_segment into yuv422p10le), each on an
// instance without the other's code -- FUSE 9 the luma launch (fuse 1), FUSE
// 11 the chroma launch (fuse 2).  Narrow H windows only (the upscale plans);
// other windows return nullptr and take the FUSE 10 chain instance.
#include "strip.hpp"

namespace pp {

#define PP_STRIP_HW_NARROW_F(ST, OUTB, FUSE)                                 \
    switch (hw) {                                                            \
    case 3: PP_STRIP_VTM(ST, OUTB, 3, FUSE, 256)                             \
    case 4: PP_STRIP_VTM(ST, OUTB, 4, FUSE, 256)                             \
    case 5: PP_STRIP_VTM(ST, OUTB, 5, FUSE, 256)                             \
    case 6: PP_STRIP_VTM(ST, OUTB, 6, FUSE, 256)                             \
    default: return nullptr;                                                 \
    }

KernelFn pick_strip_luma_u16(int hw, int vtm) {
    PP_STRIP_HW_NARROW_F(uint16_t, 8, 9)
}

KernelFn pick_strip_chroma_u16(int hw, int vtm) {
    PP_STRIP_HW_NARROW_F(uint16_t, 8, 11)
}

}  // namespace pp
