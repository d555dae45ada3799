// Issue cost of the VALU instruction classes in the draw kernel (k_hot_bx)
// and the fp64 lpdf kernel (k_round<double>) on one MI355X: cycles per
// wave64 instruction per SIMD, measured with 1, 2, 4 and 8 waves per SIMD
// (every CU busy).  Each kernel runs 8 independent register chains of one
// instruction.  Every wave stamps the shader clock (clock64) and the 100 MHz
// real-time clock (wall_clock64) around its loop; the host takes the clock
// the chip held (shader ticks / real time, median over waves) and the span
// from the first wave's start to the last wave's end, so
//   cycles per instruction per SIMD = span x clock / (instructions / SIMDs)
// does not depend on how the launch staggered the waves; with enough waves
// per SIMD it is the issue cost (dependency latency hidden).  bench.py /
// tools/pmc_summary.py weight the PMC instruction counts with these costs
// (the cycle-weighted issue model).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_issue tools/ubench_issue.hip
//   tools/ubench_issue > profiles/<tag>_issue_costs.json
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr int kIters = 2048;   // loop trips; 8 chains x 4 unrolled per trip
constexpr int kPerTrip = 32;

// one chain step of each instruction class (inline asm: the exact opcode)
#define STEP_F64(op) asm volatile(op " %0, %0, %1" : "+v"(d[c]) : "v"(db))
#define STEP_F64_3(op) asm volatile(op " %0, %0, %1, %2" : "+v"(d[c]) : "v"(db), "v"(dc))
#define STEP_F64_1(op) asm volatile(op " %0, %0" : "+v"(d[c]))
#define STEP_F32_3(op) asm volatile(op " %0, %0, %1, %2" : "+v"(f[c]) : "v"(fb), "v"(fc))
#define STEP_F32_1(op) asm volatile(op " %0, %0" : "+v"(f[c]))
#define STEP_U32_2(op) asm volatile(op " %0, %0, %1" : "+v"(u[c]) : "v"(ub))

enum Op {
    FMA_F64, MUL_F64, ADD_F64, LDEXP_F64, SQRT_F64, RCP_F64, RNDNE_F64, MAX_F64, CVT_F64_U32,
    MAD_U64_U32, BITOP3, ADD_U32, XOR_B32, LSHL_B32, CNDMASK, MOV_B64, CMP_U64, MUL_LO_U32,
    FMA_F32, PK_FMA_F32, EXP_F32, LOG_F32, CVT_I32_F64, FRACT_F64, N_OPS
};
static const char* kNames[N_OPS] = {
    "v_fma_f64", "v_mul_f64", "v_add_f64", "v_ldexp_f64", "v_sqrt_f64", "v_rcp_f64", "v_rndne_f64",
    "v_max_f64", "v_cvt_f64_u32", "v_mad_u64_u32", "v_bitop3_b32", "v_add_u32", "v_xor_b32",
    "v_lshlrev_b32", "v_cndmask_b32", "v_mov_b64", "v_cmp_gt_u64", "v_mul_lo_u32", "v_fma_f32",
    "v_pk_fma_f32", "v_exp_f32", "v_log_f32", "v_cvt_i32_f64", "v_fract_f64"};

template <int OP>
__device__ __forceinline__ void step(double* d, float* f, uint32_t* u, uint64_t* w, double db, double dc,
                                     float fb, float fc, uint32_t ub, int c) {
    if constexpr (OP == FMA_F64) STEP_F64_3("v_fma_f64");
    else if constexpr (OP == MUL_F64) STEP_F64("v_mul_f64");
    else if constexpr (OP == ADD_F64) STEP_F64("v_add_f64");
    else if constexpr (OP == LDEXP_F64) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[c]) : "v"(ub));
    else if constexpr (OP == SQRT_F64) STEP_F64_1("v_sqrt_f64");
    else if constexpr (OP == RCP_F64) STEP_F64_1("v_rcp_f64");
    else if constexpr (OP == RNDNE_F64) STEP_F64_1("v_rndne_f64");
    else if constexpr (OP == MAX_F64) STEP_F64("v_max_f64");
    else if constexpr (OP == CVT_F64_U32) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[c]) : "v"(u[c]));
    else if constexpr (OP == MAD_U64_U32)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[c]) : "v"(ub), "v"(u[c]) : "vcc");
    else if constexpr (OP == BITOP3)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(u[c]) : "v"(ub), "v"(fb));
    else if constexpr (OP == ADD_U32) STEP_U32_2("v_add_u32");
    else if constexpr (OP == XOR_B32) STEP_U32_2("v_xor_b32");
    else if constexpr (OP == LSHL_B32) STEP_U32_2("v_lshlrev_b32");
    else if constexpr (OP == CNDMASK)
        asm volatile("v_cmp_gt_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(ub) : "vcc");
    else if constexpr (OP == MOV_B64) asm volatile("v_mov_b64 %0, %1" : "=v"(w[c]) : "v"(d[c]));
    else if constexpr (OP == CMP_U64)
        asm volatile("v_cmp_gt_u64 vcc, %0, %2\n\tv_cndmask_b32 %1, %1, %3, vcc"
                     : "+v"(w[c]), "+v"(u[c]) : "v"(w[(c + 1) & 7]), "v"(ub) : "vcc");
    else if constexpr (OP == MUL_LO_U32) STEP_U32_2("v_mul_lo_u32");
    else if constexpr (OP == FMA_F32) STEP_F32_3("v_fma_f32");
    else if constexpr (OP == PK_FMA_F32)
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(w[c]) : "v"(w[(c + 3) & 7]), "v"(w[(c + 5) & 7]));
    else if constexpr (OP == EXP_F32) STEP_F32_1("v_exp_f32");
    else if constexpr (OP == LOG_F32) STEP_F32_1("v_log_f32");
    else if constexpr (OP == CVT_I32_F64) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(u[c]) : "v"(d[c]));
    else if constexpr (OP == FRACT_F64) STEP_F64_1("v_fract_f64");
}

template <int OP>
__global__ __launch_bounds__(256) void k_issue(uint64_t* __restrict__ stamps, double* __restrict__ sink) {
    double d[8];
    float f[8];
    uint32_t u[8];
    uint64_t w[8];
    for (int c = 0; c < 8; ++c) {
        d[c] = 1.0 + threadIdx.x * 1e-3 + c;
        f[c] = 1.0f + threadIdx.x * 1e-3f + c;
        u[c] = threadIdx.x * 77u + c;
        w[c] = (uint64_t)threadIdx.x * 12345u + c;
    }
    const double db = 0.999999, dc = 1e-9;
    const float fb = 0.9999f, fc = 1e-6f;
    const uint32_t ub = 3u + (threadIdx.x & 1);
    __syncthreads();
    const uint64_t r0 = wall_clock64();
    const uint64_t t0 = clock64();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int r = 0; r < kPerTrip / 8; ++r)
#pragma unroll
            for (int c = 0; c < 8; ++c) step<OP>(d, f, u, w, db, dc, fb, fc, ub, c);
    }
    const uint64_t t1 = clock64();
    const uint64_t r1 = wall_clock64();
    double s = 0.0;
    for (int c = 0; c < 8; ++c) s += d[c] + f[c] + (double)u[c] + (double)w[c];
    if (s == 12345.678) sink[threadIdx.x] = s;   // (keeps the chains live)
    if ((threadIdx.x & 63) == 0) {
        uint64_t* st = stamps + 4 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
        st[0] = t0;
        st[1] = t1;
        st[2] = r0;
        st[3] = r1;
    }
}

template <int OP>
int run(int n_cu, uint64_t* d_st, double* d_sink, std::vector<uint64_t>& h) {
    printf("  \"%s\": {", kNames[OP]);
    double ghz_all = 0.0;
    for (int wps = 1; wps <= 8; wps *= 2) {
        const int blocks = n_cu * wps;   // 256 threads = 4 waves (one per SIMD) per workgroup
        const int waves = blocks * 4;
        hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, d_st, d_sink);   // (warm)
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(256), 0, 0, d_st, d_sink);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h.data(), d_st, (size_t)waves * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        std::vector<double> ghz;
        uint64_t rmin = UINT64_MAX, rmax = 0;
        for (int w = 0; w < waves; ++w) {
            const uint64_t* st = h.data() + 4 * (size_t)w;
            if (st[3] > st[2]) ghz.push_back((double)(st[1] - st[0]) / (double)(st[3] - st[2]) * 0.1);
            rmin = std::min(rmin, st[2]);
            rmax = std::max(rmax, st[3]);
        }
        std::sort(ghz.begin(), ghz.end());
        const double clk = ghz.empty() ? 0.0 : ghz[ghz.size() / 2];   // GHz (real-time clock: 100 MHz)
        const double span_cycles = (double)(rmax - rmin) * 10.0 * clk;  // ns x GHz
        const double n_instr = (double)kIters * kPerTrip * (OP == CNDMASK || OP == CMP_U64 ? 2 : 1);
        const double per_simd = n_instr * waves / (4.0 * n_cu);
        printf("%s\"%d\": %.3f", wps > 1 ? ", " : "", wps, span_cycles / per_simd);
        ghz_all = clk;
    }
    printf(", \"ghz\": %.3f}%s\n", ghz_all, OP + 1 < N_OPS ? "," : "");
    return 0;
}

template <int OP>
int run_all(int n_cu, uint64_t* d_cyc, double* d_sink, std::vector<uint64_t>& h) {
    if (run<OP>(n_cu, d_cyc, d_sink, h)) return 1;
    if constexpr (OP + 1 < N_OPS) return run_all<OP + 1>(n_cu, d_cyc, d_sink, h);
    return 0;
}

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int n_cu = prop.multiProcessorCount;
    uint64_t* d_cyc;
    double* d_sink;
    CHK(hipMalloc(&d_cyc, (size_t)n_cu * 8 * 4 * 4 * sizeof(uint64_t)));
    CHK(hipMalloc(&d_sink, 256 * sizeof(double)));
    std::vector<uint64_t> h((size_t)n_cu * 8 * 4 * 4);
    printf("{\"device\": \"%s\", \"cus\": %d, \"note\": \"shader cycles per wave64 instruction per SIMD "
           "at 1/2/4/8 waves per SIMD over the launch's span at the clock the chip held (ghz: the "
           "8-wave run's, shader ticks over the 100 MHz real-time clock); 8 independent chains per "
           "wave; v_cndmask_b32 and v_cmp_gt_u64 are measured in pairs with a compare / select and "
           "counted per instruction\",\n",
           prop.gcnArchName, n_cu);
    printf(" \"cycles_per_instr_per_simd\": {\n");
    if (run_all<0>(n_cu, d_cyc, d_sink, h)) return 1;
    printf(" }}\n");
    CHK(hipFree(d_cyc));
    CHK(hipFree(d_sink));
    return 0;
}
