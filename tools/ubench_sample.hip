// Microbenchmark of the below-mixture sampler's pieces (tpe_device.h
// sample_raw) on one GPU: Philox alone, + component search, + Box-Muller,
// the full bounded GMM1 draw, and candidate variants.  Prints ns per
// candidate for 2^28 draws.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_sample tools/ubench_sample.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#include "../hyperopt_amd/csrc/tpe_device.h"

using namespace tpe;

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int V>
__global__ __launch_bounds__(256) void k_bench(const DLabel* __restrict__ Lp, const SampRec* __restrict__ s,
                                               int64_t n, double* __restrict__ out) {
    const DLabel L = *Lp;
    double acc = 0.0;
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (int64_t)gridDim.x * 256) {
        const uint32_t k0 = 1234u, k1 = 0u;
        if constexpr (V == 0) {   // Philox alone
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            acc += (double)(r.x ^ r.y ^ r.z ^ r.w);
        } else if constexpr (V == 1) {   // + binary cdf search
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            const int k = cdf_search(s, L.ns, (double)r.x * 0x1.0p-32);
            acc += s[k].mu + (double)(r.y ^ r.z ^ r.w);
        } else if constexpr (V == 2) {   // + Box-Muller
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            const int k = cdf_search(s, L.ns, (double)r.x * 0x1.0p-32);
            const double u1 = u01_open0(r.y, r.z);
            const double rad = sqrt(-2.0 * log(u1));
            const double nrm = rad * cospi(2.0 * ((double)r.w * 0x1.0p-32));
            acc += s[k].mu + s[k].sigma * nrm;
        } else if constexpr (V == 3) {   // the full draw (bounded GMM1)
            double v;
            sample_raw<DENSE_GMM>(L, s, 1234u, 7u, (uint32_t)g, v);
            acc += v;
        } else if constexpr (V == 4) {   // Box-Muller without the search
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            const double u1 = u01_open0(r.y, r.z);
            const double rad = sqrt(-2.0 * log(u1));
            const double nrm = rad * cospi(2.0 * ((double)r.w * 0x1.0p-32));
            acc += nrm + (double)r.x;
        } else if constexpr (V == 5) {   // log only
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            acc += log(u01_open0(r.y, r.z)) + (double)(r.x ^ r.w);
        } else if constexpr (V == 6) {   // cospi only
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            acc += cospi(2.0 * ((double)r.w * 0x1.0p-32)) + (double)(r.x ^ r.y ^ r.z);
        } else if constexpr (V == 7) {   // fast log only
            const U4 r = philox4x32_10(U4{(uint32_t)g, 0u, 3u, 7u}, k0, k1);
            acc += flog(u01_open0(r.y, r.z)) + (double)(r.x ^ r.w);
        } else if constexpr (V == 9 || V == 10) {   // 4 slots through sample_slots (10: unbounded)
            if ((g & 3) == 0) {
                uint32_t rk[4] = {7u, 7u, 7u, 7u}, gg[4] = {(uint32_t)g, (uint32_t)g + 1, (uint32_t)g + 2, (uint32_t)g + 3};
                double o[4] = {0, 0, 0, 0};
                DLabel L2 = L;
                if (V == 10) L2.flags = 0;
                sample_slots<DENSE_GMM, 4>(L2, SampGlobal{s, L2.ns}, 1234u, rk, gg, 15u, o);
                acc += o[0] + o[1] + o[2] + o[3];
            }
        } else if constexpr (V == 8) {   // Philox with 64-bit products
            U4 c{(uint32_t)g, 0u, 3u, 7u};
            uint32_t a0 = k0, a1 = k1;
#pragma unroll
            for (int i = 0; i < 10; ++i) {
                const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
                c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ a0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ a1,
                       (uint32_t)p0};
                a0 += 0x9E3779B9u;
                a1 += 0xBB67AE85u;
            }
            acc += (double)(c.x ^ c.y ^ c.z ^ c.w);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// max |flog(x) - log(x)| in ulps of log(x), x over many decades
__global__ void k_flog_err(int64_t n, unsigned long long* worst, unsigned long long* mism) {
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (int64_t)gridDim.x * 256) {
        const U4 r = philox4x32_10(U4{(uint32_t)g, 1u, 5u, 9u}, 77u, 0u);
        const double m = 1.0 + (double)(((uint64_t)r.x << 20) ^ r.y) * 0x1.0p-52;
        const int e = (int)(r.z % 2000u) - 1000;
        const double x = ldexp(m, e);
        const double a = flog(x), b = log(x);
        if (a != b) atomicAdd(mism, 1ull);
        const double ulp = fabs(b) > 0 ? fabs(nextafter(b, 2.0 * b) - b) : 0x1.0p-1074;
        const double err = fabs(a - b) / ulp;
        atomicMax(worst, (unsigned long long)(err * 1000.0));
    }
}

int main() {
    {
        unsigned long long *dw, *dm, hw = 0, hm = 0;
        CHK(hipMalloc(&dw, 8));
        CHK(hipMalloc(&dm, 8));
        CHK(hipMemset(dw, 0, 8));
        CHK(hipMemset(dm, 0, 8));
        hipLaunchKernelGGL(k_flog_err, dim3(4096), dim3(256), 0, 0, (int64_t)1 << 26, dw, dm);
        CHK(hipMemcpy(&hw, dw, 8, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(&hm, dm, 8, hipMemcpyDeviceToHost));
        printf("flog vs log: worst %.3f ulp (of the library log), %llu of 2^26 differ\n", hw / 1000.0, hm);
    }
    const int K = 26;
    std::vector<SampRec> hs(K);
    // 25 observations (sigma 0.4, linear-forgetting-like weights) and the
    // prior (mu 0, sigma 10) at weight 1/26, in mu order
    {
        double w[K], tot = 0.0;
        for (int k = 0; k < K; ++k) {
            w[k] = (k == 12) ? 1.0 : 0.5 + 0.5 * k / K;
            tot += w[k];
        }
        double c = 0.0;
        for (int k = 0; k < K; ++k) {
            c += w[k] / tot;
            hs[k] = SampRec{c, k == 12 ? 0.0 : -4.8 + 9.6 * k / K, k == 12 ? 10.0 : 0.4, 0.0};
        }
        hs[K - 1].cdf = 1.0;
    }
    DLabel hl{};
    hl.mode = DENSE_GMM;
    hl.flags = 3;
    hl.low = -5.0;
    hl.high = 5.0;
    hl.ns = K;
    SampRec* ds;
    DLabel* dl;
    double* dout;
    const int grid = 256 * 32;
    CHK(hipMalloc(&ds, K * sizeof(SampRec)));
    CHK(hipMalloc(&dl, sizeof(DLabel)));
    CHK(hipMalloc(&dout, (size_t)grid * 256 * sizeof(double)));
    CHK(hipMemcpy(ds, hs.data(), K * sizeof(SampRec), hipMemcpyHostToDevice));
    CHK(hipMemcpy(dl, &hl, sizeof(DLabel), hipMemcpyHostToDevice));
    const int64_t n = (int64_t)1 << 28;
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const char* names[] = {"philox", "+cdf_search", "+box-muller", "sample_raw bounded", "philox+box-muller",
                           "philox+log", "philox+cospi", "philox+flog", "philox 64-bit mul",
                           "sample_slots x4 bnd", "sample_slots x4 unb"};
    for (int v = 0; v < 11; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipEventRecord(a));
            switch (v) {
                case 0: hipLaunchKernelGGL(k_bench<0>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 1: hipLaunchKernelGGL(k_bench<1>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 2: hipLaunchKernelGGL(k_bench<2>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 3: hipLaunchKernelGGL(k_bench<3>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 4: hipLaunchKernelGGL(k_bench<4>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 5: hipLaunchKernelGGL(k_bench<5>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 6: hipLaunchKernelGGL(k_bench<6>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 7: hipLaunchKernelGGL(k_bench<7>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 8: hipLaunchKernelGGL(k_bench<8>, dim3(grid), dim3(256), 0, 0, dl, ds, n, dout); break;
                case 9: hipLaunchKernelGGL(k_bench<9>, dim3(grid), dim3(256), 0, 0, dl, ds, n * 4, dout); break;
                case 10: hipLaunchKernelGGL(k_bench<10>, dim3(grid), dim3(256), 0, 0, dl, ds, n * 4, dout); break;
            }
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("%-22s %8.3f ms per 2^28  (%.3f ms per 335.5M)\n", names[v], ms, ms * 1.25);
        }
    }
    return 0;
}
