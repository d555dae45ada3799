// tpe_device.h -- device-side building blocks of the gfx950 TPE engine:
// Philox4x32-10 counter RNG, the truncated-mixture samplers, the
// log-sum-exp / quantized-mass scorers and the broadcast_best comparator.
//
// Reference semantics are cited per function (mvanveen/hyperopt,
// hyperopt/tpe.py).  Everything here is wave64 VALU code: one candidate per
// lane (R per thread), mixture components are wave-uniform and are read
// through the scalar unit (s_load into SGPRs), so no LDS is needed for them.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tpe_bm_table.h"
#include "tpe_exp_table.h"

namespace tpe {

constexpr double kEps = 1e-12;  // tpe.py:31

enum Mode : int { DENSE_GMM = 0, DENSE_LGMM = 1, QUANT_GMM = 2, QUANT_LGMM = 3, CAT = 4 };
// kernel-template only (never a label's mode): one launch over the dense
// GMM1 and LGMM1 labels together, the family read from each label
constexpr int DENSE_ANY = 8;

// One resident label, prepared on the host by tpe_set_posterior.
struct DLabel {
    int32_t mode;
    int32_t flags;      // TPE_HAS_LOW | TPE_HAS_HIGH | TPE_HAS_Q
    double low, high, q;
    double exp_low, exp_high;   // LGMM1 quantized bounds in sample space
    double shift_b, shift_a;    // dense: LSE shift M (max_k log coef_k)
    double centre;              // dense fp64: origin of the recentred records
    double logpacc_b, logpacc_a;// quantized: log(p_accept) per mixture
    int64_t comp_b, comp_a;     // record offsets into the component arrays
    int32_t nb, na;
    int64_t samp_off;           // offset of the below mixture's sampling records
    int32_t ns;
    int32_t stream;             // Philox stream id (label position, or the spec's TPE_HAS_STREAM id)
    float amax_b, amax_a;       // dense: largest fp32 record scale a per mixture (screen_err)
};

// Component record.  dense fp64: (m = (mu - centre) a, a = sqrt(K/2)/max(sigma,EPS),
// c = K (log coef - M), w) so that z = x' a - m with x' = x - centre (one FMA);
// dense fp32: the same form in log2 units (a = sqrt(log2(e)/2)/max(sigma,EPS),
// c = log2(e) (log coef - M)).  quantized: (mu, a = 1/max(sqrt(2)
// sigma, EPS), -, w).  categorical: c = log p.
template <typename T>
struct alignas(4 * sizeof(T)) Comp {
    T mu, a, c, w;
};

// Sampling record of the below mixture: cumulative weight, raw mu and sigma.
struct alignas(32) SampRec {
    double cdf, mu, sigma, pad;
};

struct Partial {
    uint64_t key;
    int64_t idx;
    double value, lb, la;
};

// -------------------------------------------------------------- fast log ----
// Natural log of a positive normal fp64 number in ~30 VALU operations (the
// library log takes ~85 issue slots): x = m 2^k with m in [sqrt(1/2),
// sqrt(2)), f = m - 1 (exact), s = f / (2 + f), z = s^2,
//   log(1 + f) = f - hf + s (hf + R(z)),  hf = f^2 / 2,
// R a degree-7 minimax polynomial of 2 atanh(s)/s - 2 (the classic fdlibm
// reduction and coefficients; < 1 ulp), plus k ln 2 in two parts.  Zero,
// negatives, subnormals, infinities and NaN take the library log.  Every
// kernel that logs a candidate or a sum uses this one function, so the
// screen and the fp64 round agree bit for bit.
__device__ __forceinline__ double flog(double x) {
    if (!(x >= 0x1.0p-1022 && x < __builtin_inf())) return log(x);
    int k;
    double m = frexp(x, &k);   // [0.5, 1)
    if (m < 0.70710678118654752440) {
        m *= 2.0;
        --k;
    }
    const double f = m - 1.0;
    const double s = f / (2.0 + f), z = s * s;
    const double R =
        z * fma(fma(fma(fma(fma(fma(1.479819860511658591e-01, z, 1.531383769920937332e-01), z,
                                1.818357216161805012e-01), z, 2.222219843214978396e-01), z,
                        2.857142874366239149e-01), z, 3.999999999940941908e-01), z,
                6.666666666666735130e-01);
    const double hf = 0.5 * f * f;
    const double dk = (double)k;
    return dk * 6.93147180369123816490e-01 - ((hf - (s * (hf + R) + dk * 1.90821492927058770002e-10)) - f);
}

// ---------------------------------------------------------------- Philox ----
struct U4 {
    uint32_t x, y, z, w;
};

// a ^ b ^ k in ONE VALU operation: gfx950's three-input bit operation
// (truth table 0x96 = odd parity); k wave-uniform (an SGPR operand).  The
// compiler forms two v_xor_b32 from the C expression.
__device__ __forceinline__ uint32_t xor3_vvs(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
    // one 32x32 -> 64-bit product per multiplier (v_mad_u64_u32) instead of
    // separate low and high multiplies: the same words, a third faster.  The
    // keys pass through an empty asm, so the 20 round keys are recomputed by
    // the scalar unit per call instead of being hoisted out of the caller's
    // loops -- held there, they spilled and came back by v_readlane (VALU).
    asm volatile("" : "+s"(k0), "+s"(k1));
    {   // round 1: the counter's y, z, w words are uniform in every caller
        // (attempt, stream, round): the compiler keeps their part scalar
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    {   // round 2: y = the low product of round 1's uniform z, still scalar
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, xor3_vvs((uint32_t)(p0 >> 32), c.w, k1),
               (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    // rounds 3..10: every word per lane; the two 3-input xors per round as
    // v_bitop3 (6 -> 4 VALU operations per round, the same words)
#pragma unroll
    for (int i = 2; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = U4{xor3_vvs((uint32_t)(p1 >> 32), c.y, k0), (uint32_t)p1, xor3_vvs((uint32_t)(p0 >> 32), c.w, k1),
               (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// 32-bit uniform in [2^-32, 1] (never 0: Box-Muller takes its log): 1 -
// y 2^-32, exact.  (The radius sqrt(-2 log u) then reaches 6.66 sigma: the
// draws are normals truncated there, a probability of 2.7e-11 per draw.)
__device__ __forceinline__ double u01_open0(uint32_t y) { return 1.0 - (double)y * 0x1.0p-32; }

// first k with cdf[k] > u (cdf[n-1] == 1 exactly, u < 1).
__device__ __forceinline__ int cdf_search(const SampRec* __restrict__ s, int n, double u) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid].cdf > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// One attempt of the below mixture's draw for global candidate g: component
// ~ weights (inverse cdf), x = mu + sigma N(0, 1) by Box-Muller, before any
// truncation test.  The counter is (g, attempt, label stream, round).
constexpr uint32_t kMaxAttempts = 1u << 16;

// Component lookup of the draw: the first k with cdf[k] > u.  SampGlobal
// searches the records in global memory; SampShared (a workgroup's copy in
// LDS, stage_samp, padded to 64 entries) starts from a 256-cell guide
// (gd[j] = the first k with cdf[k] > j / 256, j = the top 8 bits of u's
// 32-bit word) and takes at most `steps` more comparisons -- the most
// cumulative weights any cell holds, 1 for mixtures without weights below
// 1/256 -- else a branch-free lower bound over all 64; the categorical tile
// kernel walks the 64-entry guide table (guide[j] = the first k with
// cdf[k] > j / 64).  All return the same component.
// The uniform is the Philox word w (u = w 2^-32, exact): SampShared
// compares w with integer thresholds thr[k] = ceil(cdf[k] 2^32), and
// cdf[k] <= u  <=>  cdf[k] 2^32 <= w  <=>  thr[k] <= w (w an integer, the
// scaling exact) -- the same component without the conversion to double.
struct SampGlobal {
    const SampRec* __restrict__ s;
    int ns;
    __device__ __forceinline__ const double* cos_tab() const { return kCosSinTab; }
    __device__ __forceinline__ const double* log_tab() const { return kLogTab; }
    __device__ __forceinline__ void pick(uint32_t w, double& mu, double& sg) const {
        const double u = (double)w * 0x1.0p-32;
        const int k = cdf_search(s, ns, u);
        mu = s[k].mu;
        sg = s[k].sigma;
    }
};

constexpr int kSampLds = 64;     // below components staged in LDS (K_b <= 26 in practice)
constexpr int kGuideSteps = 3;   // guided picks take at most this many comparisons
struct SampLds {
    double cdf[kSampLds], mu[kSampLds], sg[kSampLds];
    uint64_t thr[kSampLds];   // ceil(cdf 2^32)
    float mu32[kSampLds], sg32[kSampLds];   // fp32 copies (k_hot_bx's fp32 draw)
    uint8_t guide[64];
    uint8_t gd[256];
    int steps;
};

struct SampShared {
    const SampLds* __restrict__ t;
    // Box-Muller's tables: the constant ones, or a workgroup's LDS copies
    // (stage_bm_tables: a per-lane gather from LDS instead of through the
    // vector memory path)
    const double* cs = kCosSinTab;
    const double* lg = kLogTab;
    int steps = -1;   // t->steps read once by the caller (-1: read per pick)
    __device__ __forceinline__ const double* cos_tab() const { return cs; }
    __device__ __forceinline__ const double* log_tab() const { return lg; }
    __device__ __forceinline__ int pick_index(uint32_t w) const {
        // (steps is the same for the whole workgroup: a scalar branch)
        const int st = steps >= 0 ? steps : __builtin_amdgcn_readfirstlane(t->steps);
        int k;
        if (st <= kGuideSteps) {
            k = t->gd[w >> 24];
#pragma unroll
            for (int s = 0; s < kGuideSteps; ++s)
                if (s < st) k += t->thr[k] <= w ? 1 : 0;   // (k <= ns - 1 throughout: thr[ns - 1] = 2^32 > w)
        } else {   // branch-free lower bound over the 64 (padded with 2.0: thr 2^33)
            k = 0;
#pragma unroll
            for (int step = kSampLds / 2; step > 0; step >>= 1) k = t->thr[k + step - 1] <= w ? k + step : k;
        }
        return k;
    }
    __device__ __forceinline__ void pick(uint32_t w, double& mu, double& sg) const {
        const int k = pick_index(w);
        mu = t->mu[k];
        sg = t->sg[k];
    }
};

// a workgroup's LDS copy of label L's below sampling records (false, and
// nothing staged, when K_b > kSampLds); every thread must call it
__device__ __forceinline__ bool stage_samp(const DLabel& L, const SampRec* __restrict__ samp, SampLds* t) {
    if (L.ns > kSampLds || L.ns < 1) return false;
    for (int k = threadIdx.x; k < kSampLds; k += blockDim.x) {
        if (k < L.ns) {
            const SampRec r = samp[L.samp_off + k];
            t->cdf[k] = r.cdf;
            t->thr[k] = (uint64_t)ceil(r.cdf * 0x1.0p32);   // (exact: a power-of-two scaling, cdf in [0, 1])
            t->mu[k] = r.mu;
            t->sg[k] = r.sigma;
            t->mu32[k] = (float)r.mu;
            t->sg32[k] = (float)r.sigma;
        } else {   // padding: never picked (u < 1 <= cdf[ns - 1])
            t->cdf[k] = 2.0;
            t->thr[k] = 1ull << 33;
            t->mu[k] = 0.0;
            t->sg[k] = 0.0;
            t->mu32[k] = 0.0f;
            t->sg32[k] = 0.0f;
        }
    }
    if (threadIdx.x == 0) t->steps = 0;
    __syncthreads();
    if (threadIdx.x < 64) {
        const double v = (double)threadIdx.x / 64.0;
        int k = 0;
        while (k < L.ns - 1 && t->cdf[k] <= v) ++k;
        t->guide[threadIdx.x] = (uint8_t)k;
    }
    for (int j = threadIdx.x; j < 256; j += blockDim.x) {
        // the first k with cdf[k] > j / 256, and the cumulative weights
        // inside [j / 256, (j + 1) / 256): the comparisons a pick in the
        // cell may need
        const double v0 = (double)j / 256.0, v1 = (double)(j + 1) / 256.0;
        int k0 = 0, k1 = 0;
        for (int k = 0; k < L.ns - 1; ++k) {
            k0 += t->cdf[k] <= v0 ? 1 : 0;
            k1 += t->cdf[k] < v1 ? 1 : 0;
        }
        t->gd[j] = (uint8_t)k0;
        if (k1 > k0) atomicMax(&t->steps, k1 - k0);
    }
    __syncthreads();
    return true;
}

// a workgroup's LDS copies of Box-Muller's cos/sin and log tables (every
// thread must call it; a barrier before use -- stage_samp's serves)
constexpr int kCosTabLen = 2 * (1 << kCosTabBits), kLogTabLen = 2 * (1 << kLogTabBits);
__device__ __forceinline__ void stage_bm_tables(double* cs, double* lg) {
    for (int i = threadIdx.x; i < kCosTabLen; i += blockDim.x) cs[i] = kCosSinTab[i];
    for (int i = threadIdx.x; i < kLogTabLen; i += blockDim.x) lg[i] = kLogTab[i];
}

// (cos, sin)(2 pi w / 2^32): the top 8 bits' angle a from a 256-entry
// table (tpe_bm_table.h), the residual t = 2 pi (w mod 2^24) / 2^32 <
// 2 pi / 256 by its Taylor polynomials (t^10 / 10! < 1e-22), then
// cos(a + t) = cos a cos t - sin a sin t, sin(a + t) = sin a cos t + cos a
// sin t -- ~17 VALU operations and one 16-byte load instead of the library
// sincospi's ~80.
__device__ __forceinline__ void sincos_turn32(uint32_t w, double& c, double& s,
                                              const double* __restrict__ tab) {
    const int k = (int)(w >> 24);
    const double t = (double)(w & 0xFFFFFFu) * (6.283185307179586 * 0x1.0p-32);
    const double t2 = t * t;
    const double ct = fma(fma(fma(fma(1.0 / 40320.0, t2, -1.0 / 720.0), t2, 1.0 / 24.0), t2, -0.5), t2, 1.0);
    const double st = t * fma(fma(fma(-1.0 / 5040.0, t2, 1.0 / 120.0), t2, -1.0 / 6.0), t2, 1.0);
    const double ca = tab[2 * k], sa = tab[2 * k + 1];
    c = fma(ca, ct, -sa * st);
    s = fma(sa, ct, ca * st);
}

// -log(u) for the Box-Muller uniform u in [2^-52, 1]: u = 2^e m, m in [1,
// 2); the 7-bit interval j of m gives a 24-bit reciprocal inv ~ 1 / c_j
// and log(1 / inv) (tpe_bm_table.h), r = m inv - 1 (|r| < 2^-8) and log1p(r)
// by its degree-7 Taylor polynomial (r^8 / 8 < 2^-67) -- ~10 fp64
// operations instead of flog's ~28 (its division); ~1 ulp.  (Only the
// draw's radius uses it: every log of a candidate or a sum stays flog.)
__device__ __forceinline__ double bm_neglog(double u, const double* __restrict__ tab) {
    const uint64_t b = __builtin_bit_cast(uint64_t, u);
    const int e = (int)(b >> 52) - 1023;
    const int j = (int)((b >> 45) & 127u);
    const double m = __builtin_bit_cast(double, (b & 0xFFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
    const double r = fma(m, tab[2 * j], -1.0);
    double q = fma(1.0 / 7.0, r, -1.0 / 6.0);
    q = fma(q, r, 0.2);
    q = fma(q, r, -0.25);
    q = fma(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    q = fma(q, r, 1.0);
    return -fma((double)e, 6.93147180559945286e-01, fma(r, q, tab[2 * j + 1]));
}

// Box-Muller's radius sqrt(-2 log u) from word y (lt: kLogTab or its LDS copy)
__device__ __forceinline__ double bm_radius(uint32_t y, const double* __restrict__ lt) {
    return __builtin_amdgcn_sqrt(fmax(0.0, 2.0 * bm_neglog(u01_open0(y), lt)));
}

// ---------------------------------------------------- fp32 Box-Muller ----
// The same radius and angle in fp32 with the hardware transcendentals
// (v_log_f32 = log2, v_sqrt_f32, v_sin_f32 / v_cos_f32 of revolutions):
// about a third of the fp64 sequences' issue cycles (fp64 runs at half rate
// on CDNA4 and the fp64 log / sincos are ~25 operations each).  Their error
// against the fp64 functions above is measured EXHAUSTIVELY -- every one of
// the 2^32 words, tools/ubench_bm32.hip (profiles/r5*_bm32_sweep.txt) -- and
// the bounds below cover the largest error found with a margin (r5d: radius
// 2.48e-7 relative, cos / sin 1.88e-7 absolute; x1.6); k_hot_bx's
// fp32 draw carries them into a per-candidate bound on |x32 - x64|.
constexpr float kBm32RadRel = 4.0e-7f;    // |rad32 - rad64| <= kBm32RadRel rad64 (and 0 at rad64 = 0)
constexpr float kBm32TrigAbs = 3.0e-7f;   // |cos32 - cos64|, |sin32 - sin64| <= kBm32TrigAbs

// -ln(u) for u = 1 - y 2^-32 (u01_open0's uniform) in fp32: for u <= 1/2
// the exact integer m = 2^32 - y gives u = m 2^-32 (one fp32 rounding) and
// -ln u = -log2(u) ln 2; above 1/2, -ln(1 - t) with t = y 2^-32 by Kahan's
// log1p form (the rounding of w = 1 - t corrected by t / (1 - w))
__device__ __forceinline__ float bm_neglog32(uint32_t y) {
    constexpr float kLn2f = 0.6931471805599453f;
    if (y >= 0x80000000u) {
        const float u = (float)(0u - y) * 0x1.0p-32f;   // (y > 0: 2^32 - y in [1, 2^31])
        return -__builtin_amdgcn_logf(u) * kLn2f;
    }
    const float t = (float)y * 0x1.0p-32f;
    const float w = 1.0f - t;
    if (w == 1.0f) return t;
    return (-__builtin_amdgcn_logf(w) * kLn2f) * (t * __builtin_amdgcn_rcpf(1.0f - w));
}

__device__ __forceinline__ float bm_radius32(uint32_t y) {
    return __builtin_amdgcn_sqrtf(2.0f * bm_neglog32(y));
}

// (cos, sin)(2 pi w 2^-32) in fp32: w - 2^31 as a signed turn fraction in
// [-1/2, 1/2) (half the input rounding of [0, 1)), cos(2 pi (x + 1/2)) =
// -cos(2 pi x), likewise sin
__device__ __forceinline__ void sincos_turn32f(uint32_t w, float& c, float& s) {
    const float x = (float)(int32_t)(w ^ 0x80000000u) * 0x1.0p-32f;
    c = -__builtin_amdgcn_cosf(x);
    s = -__builtin_amdgcn_sinf(x);
}

// Candidates 2p and 2p + 1 share one Philox4x32-10 call per attempt: the
// counter is (p, attempt, label stream, round); word x picks candidate 2p's
// component ~ weights, word z candidate 2p + 1's, word y gives the
// Box-Muller radius and word w the angle, and the pair's normals are rad cos
// and rad sin (independent N(0, 1)).  draw_pair draws both, draw_attempt one
// of them -- the same arithmetic, so the same bits.
template <typename Src>
__device__ __forceinline__ void draw_pair(const DLabel& L, const Src& src, uint32_t k0, uint32_t k1, uint32_t p,
                                          uint32_t it, uint32_t round, double& d0, double& d1) {
    const U4 r = philox4x32_10(U4{p, it, (uint32_t)L.stream, round}, k0, k1);
    double mu0, sg0, mu1, sg1;
    src.pick(r.x, mu0, sg0);
    src.pick(r.z, mu1, sg1);
    const double rad = bm_radius(r.y, src.log_tab());
    double c, s;
    sincos_turn32(r.w, c, s, src.cos_tab());
    d0 = fma(sg0, rad * c, mu0);
    d1 = fma(sg1, rad * s, mu1);
}

template <typename Src>
__device__ __forceinline__ double draw_attempt(const DLabel& L, const Src& src, uint32_t k0, uint32_t k1,
                                               uint32_t g, uint32_t it, uint32_t round) {
    const U4 r = philox4x32_10(U4{g >> 1, it, (uint32_t)L.stream, round}, k0, k1);
    const bool h = (g & 1u) != 0;
    double mu, sg;
    src.pick(h ? r.z : r.x, mu, sg);
    const double rad = bm_radius(r.y, src.log_tab());
    double c, s;
    sincos_turn32(r.w, c, s, src.cos_tab());
    return fma(sg, rad * (h ? s : c), mu);
}

// Slot r of thread t in a tile of R x nthreads candidates (R even): slots
// r, r + 1 are one Box-Muller pair, candidates 2 ((r / 2) nthreads + t) and
// the next one
__device__ __host__ __forceinline__ uint32_t tile_cand(int r, uint32_t t, uint32_t nthreads) {
    return 2u * ((uint32_t)(r >> 1) * nthreads + t) + (uint32_t)(r & 1);
}

// LGMM1 sample value of an accepted log-space draw (tpe.py:255: np.exp);
// RAW sample_slots leave this step to the caller
__device__ __forceinline__ double lgmm_value(double draw) { return exp(draw); }

// Draw one sample of the below posterior for global candidate g, BEFORE
// quantization (LGMM1: after the exp).
// GMM1 / LGMM1 (tpe.py:68-99 / 222-256): component ~ weights, x ~ N(mu, sigma),
// bounded: retry until low <= x < high (re-selecting the component, exactly as
// the reference loop does), LGMM1 then exp(x).
// categorical (stochastic.py:109-147): index ~ p.
// Returns false if the truncation interval was not reached within the cap.
template <int MODE>
__device__ __forceinline__ bool sample_raw(const DLabel& L, const SampRec* __restrict__ s,
                                           uint64_t seed, uint32_t round, uint32_t g,
                                           double& out) {
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    if constexpr (MODE == CAT) {
        const U4 r = philox4x32_10(U4{g, 0u, (uint32_t)L.stream, round}, k0, k1);
        out = (double)cdf_search(s, L.ns, (double)r.x * 0x1.0p-32);
        return true;
    } else {
        const bool bounded = (L.flags & 3) == 3;
        for (uint32_t it = 0; it < kMaxAttempts; ++it) {
            const double draw = draw_attempt(L, SampGlobal{s, L.ns}, k0, k1, g, it, round);
            if (!bounded || (L.low <= draw && draw < L.high)) {
                out = (MODE == DENSE_LGMM || MODE == QUANT_LGMM) ? lgmm_value(draw) : draw;
                return true;
            }
        }
        out = __builtin_nan("");
        return false;
    }
}

// sample_raw for the R slots of a thread (bit for bit the same draws): the
// lane keeps a queue of its pending slots (bit mask) and spends every
// attempt of the rejection loop on the first of them, so a wave runs ~R +
// (the largest excess of one lane) attempts instead of R times the largest
// attempt count of each slot -- with a prior component reaching far out of
// [low, high), nearly every wave has a lane that retries.  Slots outside
// `pend` keep their value.  Returns false if a slot hit the attempt cap
// (its value is NaN).
template <int MODE, int R, typename Src, bool RAW = false>
__device__ __forceinline__ bool sample_slots(const DLabel& L, const Src& src, uint64_t seed,
                                             const uint32_t (&rk)[R], const uint32_t (&g)[R], uint32_t pend,
                                             double (&out)[R]) {
    static_assert(MODE != CAT, "categorical slots draw once each");
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const bool bounded = (L.flags & 3) == 3;
    const uint32_t mask0 = pend;
    bool ok = true;
    // attempt 0 of every pending slot, straight-line; the queue below takes
    // the rejected ones from attempt 1 (the same attempt sequence per slot)
    // (every slot is drawn, pending or not: no branch, so with a branch-free
    // pick the slots' sequences can interleave)
    uint32_t rej = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double draw = draw_attempt(L, src, k0, k1, g[r], 0u, rk[r]);
        const bool p = (pend >> r) & 1u;
        out[r] = p ? draw : out[r];
        if (p && bounded && !(L.low <= draw && draw < L.high)) rej |= 1u << r;
    }
    pend = rej;
    uint32_t it = 1;
    while (pend) {
        const int cur = __builtin_ctz(pend);
        uint32_t gg = g[0], rr = rk[0];
#pragma unroll
        for (int r = 1; r < R; ++r)
            if (cur == r) {
                gg = g[r];
                rr = rk[r];
            }
        const double draw = draw_attempt(L, src, k0, k1, gg, it, rr);
        const bool acc = !bounded || (L.low <= draw && draw < L.high);
        if (acc || it + 1 >= kMaxAttempts) {
            const double v = acc ? draw : __builtin_nan("");
            ok = ok && acc;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (cur == r) out[r] = v;
            pend &= pend - 1;
            it = 1;
        } else {
            ++it;
        }
    }
    if constexpr ((MODE == DENSE_LGMM || MODE == QUANT_LGMM) && !RAW) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((mask0 >> r) & 1u) out[r] = lgmm_value(out[r]);
    }
    return ok;
}

// set bits of a wave mask below this lane (v_mbcnt_lo + v_mbcnt_hi)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The workgroup-cooperative form of sample_slots for tile kernels (every
// thread of the workgroup calls it, uniform control flow): attempt 0 of
// every slot straight-line; the rejected slots go to an LDS list and the
// whole workgroup retries them together, each list entry walking its own
// attempts 1, 2, .. -- so a rejection costs one lane-attempt instead of a
// wave-wide queue iteration (the same draws, bit for bit).  Slot r of
// thread t holds candidate g0 + tile_cand(r, t, blockDim): slots r, r + 1 are
// a Box-Muller pair, drawn by one Philox call (draw_pair) when g0 is even.
// The accepted values come back through CAP entries at a time (the
// rejected slots of one tile are a few per cent of R * 256 with bounded
// labels: one pass; more take several, each retrying the next CAP entries).
// A smaller value array leaves LDS for more workgroups per CU.
//
// The list: each wave appends to its own segment of R * 64 entries, in
// slot order, at the running count it keeps in a scalar register -- the
// rejection mask of a slot IS its comparison's wave mask, so a slot costs
// two v_mbcnt and an add (round 3: one LDS atomic and ~17 VALU operations
// per slot); after the barrier the segments are read as one list in wave
// order through their counts.
constexpr int kTileWaves = 4;   // sample_tile: 256-thread workgroups
template <int R, int CAP = R * 256>
struct RetryLds {
    int wn[kTileWaves];       // per wave: its rejected slots of this tile
    uint16_t slot[R * 256];   // per wave a segment of R * 64: candidate offset within the tile
    double val[CAP];
};

// (every thread of the workgroup calls it, blockDim.x == 256; no workgroup
// barrier: each wave retries its own rejected slots -- `par` is unused, kept
// for the callers.
// Slots outside `pend` receive unspecified values: both callers read the
// pending slots only.)
template <int MODE, int R, typename Src, bool RAW = false, int CAP = R * 256>
__device__ __forceinline__ bool sample_tile(const DLabel& L, const Src& src, uint64_t seed, uint32_t rk,
                                            uint32_t g0, uint32_t pend, double (&out)[R], RetryLds<R, CAP>& q,
                                            int par) {
    static_assert(MODE != CAT, "categorical slots draw once each");
    static_assert(R * 256 <= 65536, "tile offsets are 16-bit");
    (void)par;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const bool bounded = (L.flags & 3) == 3;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint16_t* __restrict__ seg = q.slot + wave * (R * 64);
    constexpr int kAccepted = 1 << 20;   // pos of an accepted slot: past any list
    int pos[R];     // this lane's slots in its wave's segment (kAccepted: not listed)
    int run = 0;    // the wave's rejected slots so far (uniform)
    static_assert(R % 2 == 0, "sample_tile draws Box-Muller pairs");
    const bool paired = (g0 & 1u) == 0;   // (an odd first index: each slot on its own, the same bits)
#pragma unroll
    for (int r = 0; r < R; r += 2) {
        const uint32_t c0 = tile_cand(r, threadIdx.x, blockDim.x);
        double dd[2];
        if (paired) {
            draw_pair(L, src, k0, k1, (g0 + c0) >> 1, 0u, rk, dd[0], dd[1]);
        } else {
            dd[0] = draw_attempt(L, src, k0, k1, g0 + c0, 0u, rk);
            dd[1] = draw_attempt(L, src, k0, k1, g0 + c0 + 1u, 0u, rk);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const double draw = dd[h];
            const bool p = (pend >> (r + h)) & 1u;
            out[r + h] = draw;
            const bool rej = p && bounded && !(L.low <= draw && draw < L.high);
            const uint64_t m = __ballot(rej);
            pos[r + h] = rej ? run + (int)lanes_below(m) : kAccepted;
            if (rej) seg[pos[r + h]] = (uint16_t)(c0 + (uint32_t)h);
            run += (int)__popcll(m);
        }
    }
    bool ok = true;
    if (bounded && run > 0) {   // (a label without both bounds never rejects: no list)
        // the wave retries its own rejected slots -- no workgroup barrier:
        // its segment and its share of val are its own, and LDS operations
        // of one wave complete in order (the wave barriers only keep the
        // compiler from moving them); a retry is the slot's own attempts 1,
        // 2, .. either way, so the values are the cooperative retry's
        constexpr int WC = CAP / kTileWaves;
        double* __restrict__ wval = q.val + wave * WC;
        for (int c0 = 0; c0 < run; c0 += WC) {
            const int c1 = min(run, c0 + WC);
            __builtin_amdgcn_wave_barrier();
            for (int e = c0 + lane; e < c1; e += 64) {
                const uint32_t gg = g0 + (uint32_t)seg[e];
                double v = __builtin_nan("");
                for (uint32_t it = 1; it < kMaxAttempts; ++it) {
                    const double draw = draw_attempt(L, src, k0, k1, gg, it, rk);
                    if (L.low <= draw && draw < L.high) {
                        v = draw;
                        break;
                    }
                }
                ok = ok && v == v;
                wval[e - c0] = v;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < R; ++r) {   // (segment entry pos in [c0, c1); kAccepted never is)
                const uint32_t k = (uint32_t)(pos[r] - c0);
                if (k < (uint32_t)(c1 - c0)) out[r] = wval[k];
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if constexpr ((MODE == DENSE_LGMM || MODE == QUANT_LGMM) && !RAW) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((pend >> r) & 1u) out[r] = lgmm_value(out[r]);
    }
    return ok;
}

// sample_tile's draws in fp32 with a rigorous bound, for k_hot_bx (RAW,
// dense GMM1 / LGMM1, every thread of the 256-thread workgroup calls it):
// slot r gets xf[r] and ef[r]: ef >= 0 -- the draw's attempt 0 was accepted
// and |xf - x64| <= ef, x64 being the value the fp64 draw (draw_attempt /
// draw_pair) gives the same candidate; ef = -a <= 0 -- the fp64 draw decided
// (attempt a accepted) and xf is its value rounded to fp32.  k_screen_hot re-draws
// a listed candidate in fp64 from (index, attempt), so every value that is
// scored is the fp64 draw's, bit for bit.
//   attempt 0: Philox as draw_pair; the component picked by the same
//     integer thresholds (the same component); radius and angle by the fp32
//     functions above; x = fma(sg, rad cos|sin, mu) in fp32.  The bound (the
//     measured kBm32RadRel / kBm32TrigAbs, the fp32 roundings of mu, sigma,
//     the products and the fma, and the fp64 draw's own rounding):
//       ef = 1.001 (sg rad (eps_r + eps_t + 2^-23) + 2^-23 (|mu| + |x|))
//   truncation: x64 in [low, high) is decided by xf +- ef where the
//     interval clears a bound; where it straddles one (or xf is NaN) the
//     slot joins the rejected ones, flagged to start from attempt 0 --
//     so the accepted attempt of every slot is the fp64 draw's;
//   those slots: sample_tile's cooperative fp64 retries (exact values),
//     recording the accepted attempt.
// escale > 1 widens every bound (tests: TPE_OPT_HOT32 = 2 sends many more
// slots through the fp64 decisions and the margins; the round is the same).
// Returns false if a slot hit the attempt cap.
template <int R>
struct RetryLds32 {
    int wn[kTileWaves];
    uint16_t slot[R * 256];
    double val[R * 256 / 2];   // (a pass holds up to R * 128 retried slots)
    int32_t att[R * 256 / 2];
};

__device__ __forceinline__ float f32_step(float f, bool up) {   // the adjacent float (f finite)
    const uint32_t u = __float_as_uint(f);
    if (f == 0.0f) return __uint_as_float(up ? 1u : 0x80000001u);
    return __uint_as_float((f > 0.0f) == up ? u + 1u : u - 1u);
}
__device__ __forceinline__ float f32_up(double v) {   // the smallest float >= v
    const float f = (float)v;
    return (double)f >= v ? f : f32_step(f, true);
}
__device__ __forceinline__ float f32_dn(double v) {   // the largest float <= v
    const float f = (float)v;
    return (double)f <= v ? f : f32_step(f, false);
}

template <int R, typename Src>
__device__ __forceinline__ bool sample_tile32(const DLabel& L, const Src& src, uint64_t seed, uint32_t rk,
                                              uint32_t g0, uint32_t pend, float (&xf)[R], float (&ef)[R],
                                              RetryLds32<R>& q, float escale = 1.0f) {
    static_assert(R % 2 == 0, "Box-Muller pairs");
    static_assert(R * 256 <= 32768, "tile offsets are 15-bit (bit 15: start at attempt 0)");
    constexpr int CAP = R * 256 / 2;
    constexpr uint16_t kFrom0 = 0x8000;   // list entry flag: decide attempt 0 in fp64 too
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const bool bounded = (L.flags & 3) == 3;
    // the bounds as floats that keep the decisions exact (f32_up / f32_dn)
    const float lo_up = f32_up(L.low), lo_dn = f32_dn(L.low), hi_up = f32_up(L.high), hi_dn = f32_dn(L.high);
    constexpr float kEpsDraw = kBm32RadRel + kBm32TrigAbs + 0x1.0p-23f;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint16_t* __restrict__ seg = q.slot + wave * (R * 64);
    constexpr int kAccepted = 1 << 20;
    int pos[R];
    int run = 0;
    const bool paired = (g0 & 1u) == 0;
#pragma unroll
    for (int r = 0; r < R; r += 2) {
        const uint32_t c0 = tile_cand(r, threadIdx.x, blockDim.x);
        float x2[2], e2[2];
        bool ex2[2] = {false, false};   // exact fp64 values (the odd-start tile)
        if (paired) {
            const U4 w = philox4x32_10(U4{(g0 + c0) >> 1, 0u, (uint32_t)L.stream, rk}, k0, k1);
            const int ka = src.pick_index(w.x), kb = src.pick_index(w.z);
            const float rad = bm_radius32(w.y);
            float c, s;
            sincos_turn32f(w.w, c, s);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = h ? kb : ka;
                const float mu = src.t->mu32[k], sg = src.t->sg32[k];
                const float x = __builtin_fmaf(sg, rad * (h ? s : c), mu);
                x2[h] = x;
                e2[h] = escale * 1.001f *
                        (sg * rad * kEpsDraw + 0x1.0p-23f * (__builtin_fabsf(mu) + __builtin_fabsf(x)));
            }
        } else {   // (an odd first index, uniform: no shared pair -- each slot's fp64 draw)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const double d = draw_attempt(L, src, k0, k1, g0 + c0 + (uint32_t)h, 0u, rk);
                x2[h] = (float)d;
                e2[h] = 0.0f;
                ex2[h] = !bounded || (L.low <= d && d < L.high);   // (accepted: exact)
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool p = (pend >> (r + h)) & 1u;
            const float x = x2[h], e = e2[h];
            bool list = false;
            uint16_t flag = 0;
            if (p && bounded && !ex2[h]) {
                if (!paired) {
                    list = true;   // rejected at attempt 0 (exactly)
                } else {
                    const float e2u = e + 0x1.0p-22f * __builtin_fabsf(x);   // (+ the roundings of x -+ e)
                    const bool acc_sure = x - e2u >= lo_up && x + e2u < hi_dn;
                    const bool rej_sure = x + e2u < lo_dn || x - e2u >= hi_up;
                    // straddling a bound (or NaN): the fp64 draw decides from attempt 0
                    list = !acc_sure;
                    flag = rej_sure ? 0 : kFrom0;
                }
            }
            xf[r + h] = x;
            ef[r + h] = e;
            const uint64_t m = __ballot(list);
            pos[r + h] = list ? run + (int)lanes_below(m) : kAccepted;
            if (list) seg[pos[r + h]] = (uint16_t)((c0 + (uint32_t)h) | flag);
            run += (int)__popcll(m);
        }
    }
    bool ok = true;
    if (bounded) {
        if (lane == 0) q.wn[wave] = run;
        __syncthreads();
        int b[kTileWaves + 1];
        b[0] = 0;
#pragma unroll
        for (int w = 0; w < kTileWaves; ++w) b[w + 1] = b[w] + q.wn[w];
        const int n = b[kTileWaves];
        const int mine = b[wave];
        if (n == 0) __syncthreads();
        for (int c0 = 0; c0 < n; c0 += CAP) {
            const int c1 = min(n, c0 + CAP);
            for (int e = c0 + (int)threadIdx.x; e < c1; e += blockDim.x) {
                int w = 0;
#pragma unroll
                for (int k = 1; k < kTileWaves; ++k) w += e >= b[k] ? 1 : 0;
                int bw = b[0];
#pragma unroll
                for (int k = 1; k < kTileWaves; ++k) bw = w == k ? b[k] : bw;
                const uint16_t ent = q.slot[w * (R * 64) + (e - bw)];
                const uint32_t gg = g0 + (uint32_t)(ent & 0x7FFFu);
                double v = __builtin_nan("");
                int32_t a = -1;
                for (uint32_t it = (ent & kFrom0) ? 0u : 1u; it < kMaxAttempts; ++it) {
                    const double draw = draw_attempt(L, src, k0, k1, gg, it, rk);
                    if (L.low <= draw && draw < L.high) {
                        v = draw;
                        a = (int32_t)it;
                        break;
                    }
                }
                ok = ok && v == v;
                q.val[e - c0] = v;
                q.att[e - c0] = a;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t k = (uint32_t)(pos[r] + (mine - c0));
                if (k < (uint32_t)(c1 - c0)) {
                    // the fp64 draw's value and accepted attempt a, carried as
                    // ef = -a (the cap: NaN value, ef = -1 -- k_hot_bx32 raises
                    // the error flag through the return value)
                    xf[r] = (float)q.val[k];
                    ef[r] = q.att[k] < 0 ? -1.0f : -(float)q.att[k];
                }
            }
            if (c1 < n) __syncthreads();
        }
    }
    return ok;
}

// np.round(x / q) * q (round half to even), tpe.py:99 / :255
__device__ __forceinline__ double quantize(double v, double q) { return rint(v / q) * q; }

template <int MODE>
__device__ __forceinline__ bool sample_below(const DLabel& L, const SampRec* __restrict__ s,
                                             uint64_t seed, uint32_t round, uint32_t g,
                                             double& out) {
    const bool ok = sample_raw<MODE>(L, s, seed, round, g, out);
    if (MODE != CAT && (L.flags & 4)) out = quantize(out, L.q);
    return ok;
}

// numpy minimum/maximum: NaN propagates.
__device__ __forceinline__ double np_min(double a, double b) { return (a != a || a < b) ? a : b; }
__device__ __forceinline__ double np_max(double a, double b) { return (a != a || a > b) ? a : b; }

// ------------------------------------------------------------ dense LSE ----
// log sum_k exp(-z_k^2 + c_k) + M with z_k = (x - mu_k) a_k; tpe.py:144-150 and
// 284-287 (+ logsum_rows :259-262).  c_k <= 0 after the host shift by M, so the
// one-pass sum cannot overflow; if it underflows (candidate ~ > 36 sigma from
// every component) or is NaN, the lane recomputes the reference's two-pass
// form (row max first).
//
// fp64 records are pre-scaled by K = N/ln 2 (N = 4096, tpe_exp_table.h) on
// the host (a' = a sqrt(K), c' = (c - M) K), so the fma that forms the
// exponent directly yields u = K t <= 0, and exp(t) = 2^(u/N) is evaluated as
//   k = rint(u), f = u - k (exact, |f| <= 1/2),
//   2^(f/N) by the degree-3 Taylor polynomial 1 + c1 f + c2 f^2 + c3 f^3
//   (|f ln2/N| <= 8.5e-5: 2e-18 truncation, tools/gen_exp_table.py),
//   times 2^((k mod N)/N) from an N-entry LDS table, scaled by 2^(k div N)
// -- 10 fp64 + 3 integer VALU operations per (candidate, component) pair
// instead of ~23 fp64 (plus range selects) for a general exp; within ~3 ulp
// of exp per term (test_device_math).  Rounds 1-3 used a degree-2 minimax
// (2.5e-14 relative per term): round 4 spends the FMA so that a near-tie's
// fp64 score is as close to numpy's as numpy's is to the exact one.
// The table costs 32 KB of LDS per workgroup (4 workgroups = 4 waves/SIMD per
// CU, the same occupancy the kernel's 105 VGPRs allow); a wave's 32-lane
// groups hit ~3.5-way bank conflicts on it whatever its size.
__device__ __forceinline__ void load_exp_table(double* lds) {
    for (int i = threadIdx.x; i < kExpTabSize; i += blockDim.x) lds[i] = kExp2Tab[i];
    __syncthreads();
}

// 2^(f/N) for |f| <= 1/2 (Horner, kExpDeg fp64 FMAs)
static_assert(kExpDeg == 2 || kExpDeg == 3, "tpe_exp_table.h: degree 2 or 3");
__device__ __forceinline__ double exp_poly(double f) {
    if constexpr (kExpDeg == 2)
        return fma(fma(kExpC2, f, kExpC1), f, 1.0);
    else
        return fma(fma(fma(kExpC3, f, kExpC2), f, kExpC1), f, 1.0);
}

// exp(u / K) for u <= 0 (NaN / -inf propagate to NaN and trigger the fallback)
__device__ __forceinline__ double exp_scaled(double u, const double* __restrict__ tab) {
    const double k = rint(u);
    const double f = u - k;
    const double p = exp_poly(f);
    const int ki = (int)k;
    return ldexp(p * tab[ki & (kExpTabSize - 1)], ki >> kExpTabBits);
}

// acc + exp_scaled(u): the power of two is applied to the polynomial first so
// the table product and the accumulation fuse into one FMA.
__device__ __forceinline__ double exp_scaled_acc(double u, const double* __restrict__ tab,
                                                 double acc) {
    const double k = rint(u);
    const double f = u - k;
    const double p = exp_poly(f);
    const int ki = (int)k;
    return fma(ldexp(p, ki >> kExpTabBits), tab[ki & (kExpTabSize - 1)], acc);
}

// x: recentred candidate (x - centre), records as documented at Comp.
__device__ __forceinline__ double lse_twopass(const Comp<double>* __restrict__ c, int n, double x) {
    double m = -__builtin_inf();
    for (int k = 0; k < n; ++k) {
        const double z = fma(x, c[k].a, -c[k].mu);
        m = fmax(m, fma(-z, z, c[k].c));
    }
    if (!(m > -__builtin_inf())) return __builtin_nan("");  // all -inf or NaN: reference gives NaN
    double s = 0.0;
    for (int k = 0; k < n; ++k) {
        const double z = fma(x, c[k].a, -c[k].mu);
        s += exp((fma(-z, z, c[k].c) - m) * kExpScaleInv);
    }
    return log(s) + m * kExpScaleInv;
}

// fp32 records: (m = (mu - centre) a, a, c, w) in log2 units, x recentred
__device__ __forceinline__ float lse_twopass(const Comp<float>* __restrict__ c, int n, float x) {
    float m = -__builtin_inff();
    for (int k = 0; k < n; ++k) {
        const float z = fmaf(x, c[k].a, -c[k].mu);
        m = fmaxf(m, fmaf(-z, z, c[k].c));
    }
    if (!(m > -__builtin_inff())) return __builtin_nanf("");
    float s = 0.0f;
    for (int k = 0; k < n; ++k) {
        const float z = fmaf(x, c[k].a, -c[k].mu);
        s += __builtin_amdgcn_exp2f(fmaf(-z, z, c[k].c) - m);
    }
    return (__builtin_log2f(s) + m) * 0.69314718055994531f;  // back to natural log
}

// acc[r] += sum_{k < n} exp_scaled(-z_k^2 + c_k) for the recentred x[r].
//
// The records are wave-uniform and come through the scalar cache,
// double-buffered in batches of U (A/B, no register copies).  Scalar and LDS
// loads share lgkmcnt and scalar loads return out of order, so the wait for
// a batch's exp-table reads also waits for every scalar load in flight: the
// next batch's loads are issued right after the current batch's exponents
// are formed (its first use of its records), ~10 VALU per evaluation before
// that wait.  The plain loop issued them just before it (config 3: 97 ->
// 98 % of the issue rate; config 5: +25 %).
template <int R>
__device__ __forceinline__ void lse_acc_run(const Comp<double>* __restrict__ c, int n,
                                            const double (&x)[R], double (&acc)[R],
                                            const double* __restrict__ tab) {
    if (n <= 0) return;
    constexpr int U = R >= 2 ? 4 : 8;
    const int nbat = n / U, nfull = nbat * U;
    double Am[U], Aa[U], Ac[U], Bm[U], Ba[U], Bc[U], t[U][R];
    // batch at record k0; a prefetch past the last full batch re-reads it
    auto load = [&](double (&m)[U], double (&a)[U], double (&cc)[U], int k0) {
        const Comp<double>* p = c + min(k0, nfull - U);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            m[u] = p[u].mu;
            a[u] = p[u].a;
            cc[u] = p[u].c;
        }
    };
    auto expo = [&](const double (&m)[U], const double (&a)[U], const double (&cc)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const double z = fma(x[r], a[u], -m[u]);
                t[u][r] = fma(-z, z, cc[u]);
            }
    };
    auto accum = [&]() {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = exp_scaled_acc(t[u][r], tab, acc[r]);
    };
    if (nbat > 0) load(Am, Aa, Ac, 0);
    int b = 0;
    for (; b + 2 <= nbat; b += 2) {
        expo(Am, Aa, Ac);
        __builtin_amdgcn_sched_barrier(0);
        load(Bm, Ba, Bc, (b + 1) * U);
        __builtin_amdgcn_sched_barrier(0);
        accum();
        expo(Bm, Ba, Bc);
        __builtin_amdgcn_sched_barrier(0);
        load(Am, Aa, Ac, (b + 2) * U);
        __builtin_amdgcn_sched_barrier(0);
        accum();
    }
    if (b < nbat) {
        expo(Am, Aa, Ac);
        accum();
    }
    for (int k = nfull; k < n; ++k) {
        const double m = c[k].mu, a = c[k].a, cc = c[k].c;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double z = fma(x[r], a, -m);
            acc[r] = exp_scaled_acc(fma(-z, z, cc), tab, acc[r]);
        }
    }
}

// The fp64 summation order of a dense mixture, shared by every fp64 kernel
// (tile, split-K and packed maps, the re-scores): slices of kSumSlice
// consecutive components, each summed in order from 0, the slice sums
// added in order to acc.  Fixing it lets a sum be split across waves by
// slices (k_score_slices, k_rescore_slices) with the same bits.
constexpr int kSumSlice = 256;

template <int R>
__device__ __forceinline__ void lse_acc(const Comp<double>* __restrict__ c, int n,
                                        const double (&x)[R], double (&acc)[R],
                                        const double* __restrict__ tab) {
    for (int k0 = 0; k0 < n; k0 += kSumSlice) {
        double part[R];
#pragma unroll
        for (int r = 0; r < R; ++r) part[r] = 0.0;
        lse_acc_run<R>(c + k0, min(kSumSlice, n - k0), x, part, tab);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] += part[r];
    }
}

// A term of exp_scaled_acc is exactly +0.0 once u < -kZeroU: ldexp(p, e)
// with p < 2 and e = floor(rint(u) / 4096) <= -1076 is below 2^-1075 and
// rounds to 0.  (u = c' - z^2 with z = x' a' - m', so a component's term can
// be nonzero only where |x' a' - m'| <= sqrt(c' + kZeroU), kZeroU with a
// margin for the roundings of z and u.)
constexpr double kZeroU = 4403201.5 + 64.0;

// log(acc) + shift, or the two-pass form when the sum underflowed / is NaN
__device__ __forceinline__ double lse_finish(const Comp<double>* __restrict__ c, int n, double acc,
                                             double xr, double shift) {
    double v = flog(acc);
    if (!(acc >= 1e-290)) v = lse_twopass(c, n, xr);  // rare: underflow / NaN
    return v + shift;
}

template <int R>
__device__ __forceinline__ void lse_dense(const Comp<double>* __restrict__ c, int n, double shift,
                                          double centre, const double (&xin)[R],
                                          double (&out)[R], const double* __restrict__ tab) {
    double acc[R], x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        acc[r] = 0.0;
        x[r] = xin[r] - centre;
    }
    lse_acc<R>(c, n, x, acc, tab);
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = lse_finish(c, n, acc[r], x[r], shift);
}

// fp32 path: records (m, a, c) pre-scaled by log2(e) and recentred like the
// fp64 ones, so z = fma(x', a, -m), t = fma(-z, z, c) and the hardware
// v_exp_f32 (exp2) is used directly; the shift is in natural-log units.
// Candidates go in pairs through packed fp32 (v_pk_fma_f32 on a float2, the
// component constants broadcast from SGPRs): 2 packed FMAs + 2 v_exp_f32 +
// one packed add per two evaluations.  The 8 terms of a record batch are
// added as a tree, 16 batch sums into a mid sum, and the mid sums into the
// running sum, which keeps the summation error bound at (K/128 + 27) u
// instead of K u (screen_err).
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int R>
__device__ __forceinline__ void lse_acc(const Comp<float>* __restrict__ c, int n,
                                        const float (&xf)[R], float (&out)[R]) {
    // candidate pairs through packed fp32, an odd one scalar; the record
    // stream double-buffered as in the fp64 lse_acc (no LDS here, but a use
    // of a scalar-loaded record while the next batch is in flight still
    // waits for all of it: the loads go out after the batch's exponents)
    constexpr int P = R / 2;
    constexpr bool kOdd = R % 2 != 0;
    constexpr int PP = P > 0 ? P : 1;
    f32x2 x2[PP], acc2[PP];
    float x1 = kOdd ? xf[R - 1] : 0.0f, acc1 = 0.0f;
#pragma unroll
    for (int p = 0; p < PP; ++p) {
        x2[p] = P > 0 ? f32x2{xf[2 * p], xf[2 * p + 1]} : f32x2{0.0f, 0.0f};
        acc2[p] = f32x2{0.0f, 0.0f};
    }
    if (n > 0) {
        constexpr int U = 8;
        const int nbat = n / U, nfull = nbat * U;
        float Am[U], Aa[U], Ac[U], Bm[U], Ba[U], Bc[U], t1[U];
        f32x2 t2[U][PP];
        auto load = [&](float (&m)[U], float (&a)[U], float (&cc)[U], int k0) {
            const Comp<float>* q = c + min(k0, nfull - U);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                m[u] = q[u].mu;
                a[u] = q[u].a;
                cc[u] = q[u].c;
            }
        };
        auto expo = [&](const float (&m)[U], const float (&a)[U], const float (&cc)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const f32x2 z = __builtin_elementwise_fma(x2[p], f32x2{a[u], a[u]},
                                                              f32x2{-m[u], -m[u]});
                    t2[u][p] = __builtin_elementwise_fma(-z, z, f32x2{cc[u], cc[u]});
                }
                if constexpr (kOdd) {
                    const float z = fmaf(x1, a[u], -m[u]);
                    t1[u] = fmaf(-z, z, cc[u]);
                }
            }
        };
        // batch trees go into mid sums, flushed into the running sums every
        // 16 batches (128 records)
        f32x2 mid2[PP];
        float mid1 = 0.0f;
#pragma unroll
        for (int p = 0; p < PP; ++p) mid2[p] = f32x2{0.0f, 0.0f};
        auto accum = [&]() {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                f32x2 e[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    e[u] = f32x2{__builtin_amdgcn_exp2f(t2[u][p].x), __builtin_amdgcn_exp2f(t2[u][p].y)};
                mid2[p] += ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
            }
            if constexpr (kOdd) {
                float e[U];
#pragma unroll
                for (int u = 0; u < U; ++u) e[u] = __builtin_amdgcn_exp2f(t1[u]);
                mid1 += ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
            }
        };
        auto flush = [&]() {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                acc2[p] += mid2[p];
                mid2[p] = f32x2{0.0f, 0.0f};
            }
            if constexpr (kOdd) {
                acc1 += mid1;
                mid1 = 0.0f;
            }
        };
        if (nbat > 0) load(Am, Aa, Ac, 0);
        int b = 0;
        for (; b + 2 <= nbat; b += 2) {
            expo(Am, Aa, Ac);
            __builtin_amdgcn_sched_barrier(0);
            load(Bm, Ba, Bc, (b + 1) * U);
            __builtin_amdgcn_sched_barrier(0);
            accum();
            expo(Bm, Ba, Bc);
            __builtin_amdgcn_sched_barrier(0);
            load(Am, Aa, Ac, (b + 2) * U);
            __builtin_amdgcn_sched_barrier(0);
            accum();
            if (((b + 2) & 15) == 0) flush();
        }
        if (b < nbat) {
            expo(Am, Aa, Ac);
            accum();
        }
        flush();
        for (int k = nfull; k < n; ++k) {
            const float m = c[k].mu, a = c[k].a, cc = c[k].c;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const f32x2 z = __builtin_elementwise_fma(x2[p], f32x2{a, a}, f32x2{-m, -m});
                const f32x2 t = __builtin_elementwise_fma(-z, z, f32x2{cc, cc});
                acc2[p] += f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
            }
            if constexpr (kOdd) {
                const float z = fmaf(x1, a, -m);
                acc1 += __builtin_amdgcn_exp2f(fmaf(-z, z, cc));
            }
        }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
        out[2 * p] = acc2[p].x;
        out[2 * p + 1] = acc2[p].y;
    }
    if constexpr (kOdd) out[R - 1] = acc1;
}

// x: recentred candidate (y - centre) in fp32
__device__ __forceinline__ double lse_finish(const Comp<float>* __restrict__ c, int n, float acc,
                                             float x, double shift) {
    float v = __builtin_log2f(acc) * 0.69314718055994531f;
    if (!(acc >= 1e-30f)) v = lse_twopass(c, n, x);
    return (double)v + shift;
}

template <int R>
__device__ __forceinline__ void lse_dense(const Comp<float>* __restrict__ c, int n, double shift,
                                          double centre, const double (&xd)[R], double (&out)[R],
                                          const double* __restrict__) {
    float acc[R], xf[R];
#pragma unroll
    for (int r = 0; r < R; ++r) xf[r] = (float)(xd[r] - centre);
    lse_acc<R>(c, n, xf, acc);
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = lse_finish(c, n, acc[r], xf[r], shift);
}

// -------------------------------------------------------- fp32 screen ----
// The exact fp64 round screens every candidate with the fp32 sums above and
// re-scores in fp64 only those that can still win.  screen_err bounds
// |lpdf32 - lpdf| of ONE mixture (natural-log units) for a candidate at
// recentred x' (|x'| = X, |fl32(x') - x'| = dx), rigorously, from the fp32
// arithmetic (u = 2^-24), with S32 its fp32 sum (log2 S32 = l2):
//  * split the terms at an exponent cut -T (log2 units), T chosen per
//    candidate so that the terms below it are negligible:
//    T = (43 + log2(2K) - l2) / 0.9997, clamped to [16, 125] (so relevant
//    terms stay normal fp32 numbers);
//  * a "relevant" term has exact t = c' - z^2 >= -T; since c' <= 0 then
//    |z| <= sqrt(T) and |c'| <= T;
//  * z = fma(x32, a32, -m32): |z32 - z| <= zeta = dx amax + (2 X amax +
//    2 sqrt(T)) u (x32 rounded, a32 rounded, |m| <= X a + sqrt(T) for a
//    relevant term, one rounding of the fma);
//  * t = fma(-z, z, c32): |t32 - t| <= dt = (2 T + 1) u + zeta (2 sqrt(T)
//    + zeta);
//  * v_exp_f32: 2 ulp (2^-22) relative; so a relevant term is within
//    rho = 0.7 dt + 2.5e-7 relative (dt <= 0.01);
//  * the sum of positive terms: (K/128 + 27) u relative (tree of 8, mid sum
//    of 16 batches, running sum, a tail of < 8 terms added one by one);
//  * the other terms: exact < 2^-T, computed < 2^-0.9997T (dt <= 0.01 keeps
//    |z32| within 1e-4 relative of |z|), at most 2 K 2^-0.9997T / S <=
//    2^-42 relative (S >= S32 / 1.01);
//  * v_log_f32: 2^-22 (|log2 S| + 1) absolute.
// Uncertified (S < 2^-60, NaN, dt > 0.01) returns +inf: the candidate is
// always re-scored, which also keeps the reference's NaN-greatest order.
constexpr float kScreenMinAcc = 0x1.0p-60f;

// Kc: the longest run of terms one fp32 running sum adds (K, or a chunk's
// length when the mixture is summed in chunks whose fp32 sums are added in
// fp64 -- that addition adds nch 2^-53, inside the 2^-41 slack)
//
// skip: the relative mass of terms left out of the sum altogether (the
// windowed screen, below): a bound B of their sum over S, B / S <= B 1.01 /
// S32.
__device__ __forceinline__ double screen_err(float amax, int K, int Kc, double X, double dx,
                                             float acc, float l2, double skip = 0.0) {
    if (!(acc >= kScreenMinAcc) || !(acc <= 0x1.0p+100f) || !(X <= 1e30)) return __builtin_inf();
    if (!(skip <= 0.01)) return __builtin_inf();
    constexpr double u = 0x1.0p-24;
    const double T = fmin(125.0, fmax(16.0, (43.0 + log2(2.0 * (double)K) - (double)l2) / 0.9997));
    const double sqT = sqrt(T) * (1.0 + 1e-12);
    const double A = (double)amax * 1.001;
    const double zeta = (dx * A + (2.0 * X * A + 2.0 * sqT) * u) * 1.001;
    const double dt = (2.0 * T + 1.0) * u + zeta * (2.0 * sqT + zeta);
    if (!(dt <= 0.01)) return __builtin_inf();
    const double rho = 0.7 * dt + 2.5e-7;
    const double gsum = ((double)(Kc / 128) + 28.0) * u * 1.01;
    const double rel = rho + gsum + skip + 0x1.0p-41;
    return 1.02 * rel + 0x1.0p-22 * 0.6931471805599453 * (fabs((double)l2) + 1.0);
}

// ------------------------------------------------------ windowed screen ----
// Parzen components are narrow (sigma >= prior_sigma / min(100, N + 1),
// tpe.py:404-477) and sorted by mu, so a candidate's above sum is decided by
// the components near it: at config 3, 14 % of the (candidate, component)
// terms are above 2^-64 of the largest.  The windowed screen sorts a round's
// candidates by a coarse bin of x', and sums each tile of 2048 neighbouring
// candidates only over the window of components whose term can reach
// 2^-T for some candidate of the tile, plus the "wide" components
// (always summed).  Every term left out is exactly < 2^-T (log2 units,
// relative to the LSE shift); their total, bounded per bin of x'
// (tpe_window.hip k_win_skip), enters screen_err as skip.  The fp64 re-score
// of the survivors still sums every component.
constexpr int kWinTDefault = 16;   // TPE_OPT_WIN_T: the cut T, in [8, 62]
constexpr int kWinBinBits = 11;
constexpr int kWinBins = 1 << kWinBinBits;

struct WinLabel {
    double xlo, inv_bw;   // bin of x': floor((x' - xlo) inv_bw), clamped to [0, kWinBins)
    int32_t n_wide;       // wide components (listed at the label's comp_a in win_wide)
    int32_t pad;
};

__device__ __host__ __forceinline__ int win_bin(const WinLabel& W, double x) {
    const double f = (x - W.xlo) * W.inv_bw;
    if (!(f >= 1.0)) return 0;   // also NaN
    if (!(f < (double)(kWinBins - 1))) return kWinBins - 1;
    return (int)f;
}

// ----------------------------------------------------- expansion screen ----
// Past ~100 observations most above components share one sigma: the gaps
// between sorted observations are narrower than prior_sigma / min(100, N +
// 1), so adaptive_parzen_normal clips them all to it (tpe.py:404-477).  For
// those "clipped" components (fp64 record scale a' = a*) the above sum over
// a bin of x' with centre x_b, x' = x_b + delta, is
//   sum_k exp(c_k - kappa (x' - mu_k)^2)
//     = exp(-kappa delta^2) sum_n delta^n A_n,
//   A_n = sum_k g_k (2 kappa d_k)^n / n!,  g_k = exp(c_k - kappa d_k^2),
//   d_k = mu_k - x_b,  kappa = a*^2 / K (natural-log curvature),
// a Taylor series in delta whose coefficients are per bin, not per
// candidate.  tpe_expand.hip tabulates A_0..A_{P-1} per bin (in fp64, with a
// rigorous absolute bound of truncation + rounding) and lists, per bin, the
// other ("unclipped") components that can reach it; k_screen_bx scores a
// candidate with the below mixture in full fp64 (the fp64 round's own code,
// so lpdf_below is bit-identical), the above mixture as the bin's
// polynomial plus its list, and a bound ~1e-12 wide: only near-ties of the
// best score are re-scored.
constexpr int kBxP = 15;          // Taylor coefficients per bin
constexpr int kBxRow = 16;        // doubles per bin row (one 128-B line): A_0..A_14, Eabs
// components left out of a bin's window stay below 2^-T of the largest
// term (T per index, BxLabel.tcut): 64 for tile rounds through the hot-bin
// prefilter (narrower windows, fewer bins: config 3's index 0.53 -> 0.45 ms
// with the same re-scores, r5t) and, since the packed map re-scores a few
// near-ties by slices, for the packed map's rounds too (96 certified every
// value-only cell of config 5, 64 leaves ~14 near-ties per step to the fp64
// re-score: index 4.42 -> 3.55 ms, step 8.7 -> 7.8 ms, r5aj)
constexpr double kBxT = 64.0;
constexpr double kBxTTile = 64.0;

struct BxLabel {
    double xlo, inv_bw, bw;   // bin b = floor((x' - xlo) inv_bw), centre xlo + (b + 1/2) bw
    double rmax;              // largest |delta| the bin's bound covers
    double astar, kappa;      // clipped record scale, its curvature a*^2 / K
    double dwin;              // window half-width: clipped components beyond never reach 2^-T
    double rP;                // rmax^P
    int64_t tab_off;          // first row of the label in bx_tab
    int64_t cnt_off;          // first of its nbins list counts in bx_loff
    int64_t list_off;         // first of its nbins slots of n_nc entries in bx_list
    int32_t nbins, n_nc;      // bins; unclipped components (listed at comp_a in bx_nc)
    double inv_sbw;           // kBxSub / bw: sub-bin of x' = floor((x' - xlo) inv_sbw)
    int64_t sb_off;           // first of its nbins kBxSub sub-bins in bx_sb / bx_sbp
    double tcut;              // the window's cut T: components left out stay below 2^-T
};

// Hot-bin prefilter of the expansion screen.  Each bin is cut into kBxSub
// sub-bins, and tpe_expand.hip (k_bx_bounds) stores for each a rigorous
// interval [L, U] of the fp64 round's score over every x' in it (both
// mixtures bounded term by term / through the bin's polynomial, fp64 rounding
// and the fp64 round's own error inside a generous margin), plus the below
// mixture's sampling mass p of the sub-bin.  A round first draws every
// candidate and reads only its sub-bin's (U, L) (k_hot_bx): tau = the largest
// L over the candidates is a lower bound of the best fp64 score, so a
// candidate with U < tau can never win (its score is strictly below the
// candidate that attains tau).  tau is not known while drawing, so the
// candidates are listed against tau0 = max L over the sub-bins (or short
// runs of them) a round of n candidates fills with near certainty (mass p >=
// kHotFill / n; the run's smallest L); the round checks
// tau >= tau0 afterwards (then every candidate with U >= tau was listed) and
// otherwise re-runs the plain expansion screen -- the filter never changes a
// winner, tau0 only decides how often that fallback runs.  Only the listed
// candidates go through the expansion screen (k_screen_hot).
constexpr int kBxSubBits = 4;
constexpr int kBxSub = 1 << kBxSubBits;
constexpr double kHotFill = 16.0;   // P(a run of that mass stays empty) <= e^-16

__device__ __host__ __forceinline__ int bx_bin(const BxLabel& B, double x) {
    const double f = (x - B.xlo) * B.inv_bw;
    if (!(f >= 0.0) || !(f < (double)B.nbins)) return -1;   // also NaN
    return (int)f;
}

__device__ __forceinline__ float float_up(double v) {   // smallest float >= v (finite v)
    float f = (float)v;
    if ((double)f < v) {
        uint32_t b = __float_as_uint(f);
        b = f > 0.0f ? b + 1u : (f < 0.0f ? b - 1u : 1u);
        f = __uint_as_float(b);
    }
    return f;
}

__device__ __forceinline__ float float_down(double v) {   // largest float <= v (finite v)
    return -float_up(-v);
}

// |lpdf64 - lpdf| of the fp64 path (tpe_device.h lse_acc<double>): a
// sequential sum of K terms, each within ~2.5e-14 + 2 ulp
__device__ __forceinline__ double fp64_err(int K, double mag) {
    return ((double)K + 64.0) * 0x1.0p-52 + 1e-13 + mag * 0x1.0p-50;
}

// ------------------------------------------------------- quantized mass ----
// GMM1_lpdf q != None (tpe.py:151-166) and LGMM1_lpdf q != None (:288-305):
// prob = sum_k [w_k Phi(ub) - w_k Phi(lb)] accumulated sequentially over k in
// linear space, exactly like the reference (no FMA contraction here, so the
// cancellation behaves the same); lpdf = log(prob) - log(p_accept).
template <bool LOG>
__device__ __forceinline__ double quant_lpdf(const Comp<double>* __restrict__ c, int n,
                                             double ub, double lb, double logpacc) {
#pragma clang fp contract(off)
    double prob = 0.0;
    for (int k = 0; k < n; ++k) {
        const double mu = c[k].mu, a = c[k].a, w = c[k].w;
        double pu, pl;
        if (LOG) {  // lognormal_cdf: .5 + .5 * erf(z)     tpe.py:194
            pu = 0.5 + 0.5 * erf((ub - mu) * a);
            pl = 0.5 + 0.5 * erf((lb - mu) * a);
        } else {    // normal_cdf: 0.5 * (1 + erf(z))      tpe.py:107
            pu = 0.5 * (1.0 + erf((ub - mu) * a));
            pl = 0.5 * (1.0 + erf((lb - mu) * a));
        }
        double inc = w * pu;
        inc -= w * pl;
        prob += inc;
    }
    return flog(prob) - logpacc;
}

// Integration interval of a quantized candidate x (tpe.py:154-161 / 292-300);
// for LGMM1 the lognormal_cdf log(max(v, EPS)) is applied here, once per
// candidate, so the per-component loop is identical for both families.
template <int MODE>
__device__ __forceinline__ void quant_bounds(const DLabel& L, double x, double& ub, double& lb,
                                             bool& negative) {
    const double half = L.q / 2.0;
    ub = x + half;
    lb = x - half;
    negative = false;
    if constexpr (MODE == QUANT_GMM) {
        if (L.flags & 2) ub = np_min(ub, L.high);
        if (L.flags & 1) lb = np_max(lb, L.low);
    } else {
        if (L.flags & 2) ub = np_min(ub, L.exp_high);
        if (L.flags & 1) lb = np_max(lb, L.exp_low);
        lb = np_max(0.0, lb);
        negative = ub < 0.0;  // tpe.py:187-188 raises
        ub = flog(np_max(ub, kEps));
        lb = flog(np_max(lb, kEps));
    }
}

// Lane-strided share of prob = sum_k [w Phi(ub) - w Phi(lb)] (components
// k = lane, lane+64, ...); the wave sums the 64 shares afterwards.
template <bool LOG, int STRIDE = 64>
__device__ __forceinline__ double quant_share(const Comp<double>* __restrict__ c, int n, double ub,
                                              double lb, int lane) {
#pragma clang fp contract(off)
    double prob = 0.0;
    for (int k = lane; k < n; k += STRIDE) {
        const double mu = c[k].mu, a = c[k].a, w = c[k].w;
        double pu, pl;
        if (LOG) {
            pu = 0.5 + 0.5 * erf((ub - mu) * a);
            pl = 0.5 + 0.5 * erf((lb - mu) * a);
        } else {
            pu = 0.5 * (1.0 + erf((ub - mu) * a));
            pl = 0.5 * (1.0 + erf((lb - mu) * a));
        }
        double inc = w * pu;
        inc -= w * pl;
        prob += inc;
    }
    return prob;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// -------------------------------------------------------- broadcast_best ----
// np.argmax over score = below - above: NaN is greatest (first NaN wins),
// -0 == +0, and ties go to the lowest index.  Encoded as a total order key.
__device__ __host__ __forceinline__ uint64_t order_key(double s) {
    if (s != s) return ~0ull;
    if (s == 0.0) s = 0.0;
    uint64_t b;
    __builtin_memcpy(&b, &s, 8);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ bool better(uint64_t ka, int64_t ia, uint64_t kb, int64_t ib) {
    return ka > kb || (ka == kb && ia < ib);
}

}  // namespace tpe
