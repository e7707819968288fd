// Standalone GPU check of the DPP wave scan (ptx_device.h wave_incl_scan / wave_excl_sum)
// against a serial prefix sum, run before any pipeline test uses it.
// build: hipcc -O3 --offload-arch=gfx950 -I pathtracerdemo_amd/csrc tools/cl/dpp_scan_check.hip -o tools/cl/dpp_scan_check
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "ptx_device.h"

__global__ void scan_kernel(const uint32_t *in, uint32_t *excl, uint32_t *tot) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t total;
    excl[i] = ptx::wave_excl_sum(in[i], total);
    tot[i] = total;
}

int main() {
    const int waves = 4096, n = waves * 64;
    std::vector<uint32_t> in(n), ex(n), to(n);
    srand(7);
    for (int i = 0; i < n; ++i) {
        const int w = i / 64;
        in[i] = w % 3 == 0 ? (uint32_t)(rand() & 1) : w % 3 == 1 ? (uint32_t)(rand() % 128) : (uint32_t)rand() % 100000u;
    }
    uint32_t *d_in, *d_ex, *d_to;
    if (hipMalloc(&d_in, n * 4) || hipMalloc(&d_ex, n * 4) || hipMalloc(&d_to, n * 4)) return 2;
    if (hipMemcpy(d_in, in.data(), n * 4, hipMemcpyHostToDevice)) return 2;
    hipLaunchKernelGGL(scan_kernel, dim3(n / 256), dim3(256), 0, 0, d_in, d_ex, d_to);
    if (hipDeviceSynchronize()) return 3;
    if (hipMemcpy(ex.data(), d_ex, n * 4, hipMemcpyDeviceToHost) || hipMemcpy(to.data(), d_to, n * 4, hipMemcpyDeviceToHost)) return 2;
    long bad = 0;
    for (int w = 0; w < waves; ++w) {
        uint32_t s = 0;
        for (int l = 0; l < 64; ++l) {
            if (ex[w * 64 + l] != s) ++bad;
            s += in[w * 64 + l];
        }
        for (int l = 0; l < 64; ++l)
            if (to[w * 64 + l] != s) ++bad;
    }
    printf("dpp scan check: %ld mismatches over %d waves\n", bad, waves);
    return bad ? 1 : 0;
}
