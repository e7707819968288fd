// ptx_launch.h -- host-side launch wrappers exported by ptx_kernels.hip to ptx_api.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include "ptx_device.h"

namespace ptx {

constexpr int kTile = 16;
constexpr int kBlock = 256;

// dynamic LDS bytes for a traversal stack of `depth` entries per thread
inline size_t stack_lds_bytes(uint32_t depth) { return (size_t)depth * kBlock * sizeof(uint32_t); }

hipError_t launch_gbuffer(const Scene &sc, uint4 *gbuf, uint32_t stack_depth, hipStream_t s);
hipError_t launch_init(const Scene &sc, const uint4 *gbuf, uint4 *reservoir, uint32_t stack_depth, hipStream_t s);
hipError_t launch_final(const Scene &sc, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                        uint32_t stack_depth, hipStream_t s);
hipError_t launch_mcpt(const Scene &sc, float4 *accum, uint32_t stack_depth, hipStream_t s);

// persistent-lane variants (ptx_persist.hip); ctr = a zeroed u32 pixel-queue counter
hipError_t launch_init_persistent(const Scene &sc, const uint4 *gbuf, uint4 *reservoir, unsigned int *ctr,
                                  uint32_t stack_depth, hipStream_t s);
hipError_t launch_final_persistent(const Scene &sc, const uint4 *gbuf, const uint4 *reservoir, float4 *accum,
                                   unsigned int *ctr, uint32_t stack_depth, hipStream_t s);
hipError_t launch_mcpt_persistent(const Scene &sc, float4 *accum, unsigned int *ctr, uint32_t stack_depth,
                                  hipStream_t s);

}  // namespace ptx
