// Occupancy calibration of the SQ PMC counters (trace_queue read 1.36 waves/SIMD
// from 4 * SQ_WAVE_CYCLES / cycles / 1024 while the wave timeline showed 4 resident).
// Launches a kernel whose waves are all resident for the whole dispatch -- exactly W waves per
// SIMD (W = 1, 2, 4), each spinning on a VALU chain for a fixed count -- so that
// tools/pmc_summary.py's formula must read W.  Run under
//   rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -- ./occ_calib
// build: hipcc -O3 --offload-arch=gfx950 tools/cl/occ_calib.hip -o tools/cl/occ_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void spin(float *out, int iters) {
    float a = (float)threadIdx.x, b = 1.0001f;
    for (int i = 0; i < iters; ++i) a = a * b + 0.5f;
    if (a == 12345.0f) out[blockIdx.x] = a;  // never true: keeps the chain live
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0)) return 2;
    const int cus = p.multiProcessorCount;
    float *d = nullptr;
    if (hipMalloc(&d, 1 << 20)) return 2;
    for (int w : {1, 2, 4}) {
        // 256-thread workgroups = 4 waves = one per SIMD; w workgroups per CU = w waves per SIMD
        hipLaunchKernelGGL(spin, dim3(cus * w), dim3(256), 0, 0, d, 400000);
        if (hipDeviceSynchronize()) return 3;
        printf("launched %d workgroups (%d CUs x %d): %d waves per SIMD\n", cus * w, cus, w, w);
    }
    (void)hipFree(d);
    return 0;
}
