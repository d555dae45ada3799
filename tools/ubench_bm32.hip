// Exhaustive error of the fp32 Box-Muller pieces against the fp64 ones the
// draw defines (tpe_device.h bm_radius / sincos_turn32): every one of the
// 2^32 radius words y and angle words w.  Prints the largest relative error
// of the radius and the largest absolute error of cos and sin -- the
// constants behind the fp32 draw's rigorous error bound (tpe_device.h
// kBm32RadRel / kBm32TrigAbs).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_bm32 tools/ubench_bm32.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../hyperopt_amd/csrc/tpe_device.h"

using namespace tpe;

#define CHK(x)                                                                    \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
            return 1;                                                             \
        }                                                                         \
    } while (0)

// out[0]: max |rad32 - rad64| / rad64 (rad64 > 0), out[1]: max |rad32 - rad64|
// where rad64 == 0, out[2]: max |c32 - c64|, out[3]: max |s32 - s64|, as the
// bit patterns of non-negative doubles (ordered like the values)
__global__ __launch_bounds__(256) void k_sweep(unsigned long long* __restrict__ out) {
    __shared__ double lt[kLogTabLen], ct[kCosTabLen];
    stage_bm_tables(ct, lt);
    __syncthreads();
    double er = 0.0, ez = 0.0, ec = 0.0, es = 0.0;
    const uint64_t n = 1ull << 32;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t v = (uint32_t)i;
        const double r64 = bm_radius(v, lt);
        const double r32 = (double)bm_radius32(v);
        if (r64 > 0.0) er = fmax(er, fabs(r32 - r64) / r64);
        else ez = fmax(ez, fabs(r32 - r64));
        double c64, s64;
        sincos_turn32(v, c64, s64, ct);
        float c32, s32;
        sincos_turn32f(v, c32, s32);
        ec = fmax(ec, fabs((double)c32 - c64));
        es = fmax(es, fabs((double)s32 - s64));
    }
    const double m[4] = {er, ez, ec, es};
    for (int k = 0; k < 4; ++k) {
        double x = m[k];
        for (int off = 32; off > 0; off >>= 1) x = fmax(x, __shfl_xor(x, off));
        if ((threadIdx.x & 63) == 0) atomicMax(out + k, (unsigned long long)__double_as_longlong(x));
    }
}

int main() {
    unsigned long long* d;
    CHK(hipMalloc(&d, 4 * sizeof(unsigned long long)));
    CHK(hipMemset(d, 0, 4 * sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_sweep, dim3(8192), dim3(256), 0, 0, d);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    unsigned long long h[4];
    CHK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    double v[4];
    for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<double*>(&h[k]);
    printf("{\"words\": 4294967296, \"rad_rel_max\": %.6e, \"rad_abs_max_at_zero\": %.6e, "
           "\"cos_abs_max\": %.6e, \"sin_abs_max\": %.6e, \"bound_rad_rel\": %.6e, \"bound_trig_abs\": %.6e}\n",
           v[0], v[1], v[2], v[3], (double)kBm32RadRel, (double)kBm32TrigAbs);
    printf("%s\n", (v[0] <= kBm32RadRel && v[1] == 0.0 && v[2] <= kBm32TrigAbs && v[3] <= kBm32TrigAbs)
                       ? "BOUNDS HOLD" : "BOUNDS VIOLATED");
    CHK(hipFree(d));
    return 0;
}
