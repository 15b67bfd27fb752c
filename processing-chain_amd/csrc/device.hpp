// Device-side helpers shared by the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pp {

// Raw buffer resource over [base, base + nbytes): loads at or past nbytes read
// 0 without touching memory (a 16-B load that straddles nbytes reads 0 as a
// whole).  The inputs are wave-uniform by construction; readfirstlane makes
// that explicit, otherwise the compiler can lose track of it and wrap every
// load in a waterfall loop.
__device__ inline __amdgpu_buffer_rsrc_t uniform_rsrc(const void *base, int nbytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
    void *p = reinterpret_cast<void *>((static_cast<uint64_t>(hi) << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
}

constexpr int kOobOff = 0x7ffffff0;  // a buffer offset past any nbytes: reads 0, no memory access

}  // namespace pp
