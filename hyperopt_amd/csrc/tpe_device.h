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

// Sampling record of one component of the below mixture: the pick's
// cumulative weight and the component's inverse-CDF draw of its normal
// truncated to [low, high) -- folded on the device for every posterior
// (samp_fold_block: host-uploaded and device-built posteriors draw the same
// bits).
struct alignas(64) SampRec {
    double cdf;         // cumulative normalised w_k m_k (the component pick)
    double mu, sigma;   // the component
    double wd;          // w_k / sum_i w_i m_i: the truncated mixture's density is sum_k wd_k phi_k(x) in [low, high)
    double ssg;         // sigma, or -sigma when the interval is mirrored (the mean at or below low)
    double p0, q0;      // Phi(a'), Phi(-b'): the normal's mass below / above the (mirrored) interval [a', b')
    double m;           // the interval's mass (0: never picked)
};

// The expansion index's per-record bound terms of an above record (k_bx_terms,
// once per index; k_bx_bounds reads them for its bins' lists): c = c'/K, kap
// = a'^2 / K, mu = m'/a', ec = 1e-15 (64 + |c|) + 3e-14, es = 64e-15
// sqrt(kap); ec < 0 marks a weighted unusable record, c = -inf one without a
// term
struct alignas(16) BxTerm {
    double c, kap, mu, ec, es, pad;
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

// ------------------------------------------------ the inverse-CDF draw ----
// AS241 (Wichura 1988, "PPND16"): the lower-tail normal quantile
// z = Phi^-1(t) for t in (0, 1/2] -- rational approximations in three
// regions, ~7e-16 relative against 40-digit arithmetic over uniform t and
// t down to 1e-300 (checked when this was written).  One function for every
// kernel, so every kernel draws the same bits.
// a constant materialised in SGPRs where it is used: without it the
// compiler hoists ndtri_lower's 48 fp64 coefficients out of the callers'
// loops into VGPRs (k_hot_bx: 150 VGPRs, spills); fp64 FMA takes one SGPR
// operand, and the scalar unit's moves issue beside the VALU
__device__ __forceinline__ double sk(double c) {
    asm volatile("" : "+s"(c));
    return c;
}

__device__ __forceinline__ double ndtri_lower(double t) {
    const double q = t - 0.5;   // (exact: t in [1/4, 1/2] by Sterbenz, the product below rounds once)
    if (q >= -0.425) {
        const double r = 0.180625 - q * q;
        const double num =
            fma(fma(fma(fma(fma(fma(fma(sk(2.5090809287301226727e+3), r, sk(3.3430575583588128105e+4)), r,
                                    sk(6.7265770927008700853e+4)), r, sk(4.5921953931549871457e+4)), r,
                            sk(1.3731693765509461125e+4)), r, sk(1.9715909503065514427e+3)), r,
                    sk(1.3314166789178437745e+2)), r, sk(3.3871328727963666080e0));
        const double den =
            fma(fma(fma(fma(fma(fma(fma(sk(5.2264952788528545610e+3), r, sk(2.8729085735721942674e+4)), r,
                                    sk(3.9307895800092710610e+4)), r, sk(2.1213794301586595867e+4)), r,
                            sk(5.3941960214247511077e+3)), r, sk(6.8718700749205790830e+2)), r,
                    sk(4.2313330701600911252e+1)), r, 1.0);
        return q * num / den;
    }
    double r = sqrt(-flog(t));
    if (r <= 5.0) {
        r -= 1.6;
        const double num =
            fma(fma(fma(fma(fma(fma(fma(sk(7.74545014278341407640e-4), r, sk(2.27238449892691845833e-2)), r,
                                    sk(2.41780725177450611770e-1)), r, sk(1.27045825245236838258e0)), r,
                            sk(3.64784832476320460504e0)), r, sk(5.76949722146069140550e0)), r,
                    sk(4.63033784615654529590e0)), r, sk(1.42343711074968357734e0));
        const double den =
            fma(fma(fma(fma(fma(fma(fma(sk(1.05075007164441684324e-9), r, sk(5.47593808499534494600e-4)), r,
                                    sk(1.51986665636164571966e-2)), r, sk(1.48103976427480074590e-1)), r,
                            sk(6.89767334985100004550e-1)), r, sk(1.67638483018380384940e0)), r,
                    sk(2.05319162663775882187e0)), r, 1.0);
        return -(num / den);
    }
    r -= 5.0;
    const double num =
        fma(fma(fma(fma(fma(fma(fma(sk(2.01033439929228813265e-7), r, sk(2.71155556874348757815e-5)), r,
                                sk(1.24266094738807843860e-3)), r, sk(2.65321895265761230930e-2)), r,
                        sk(2.96560571828504891230e-1)), r, sk(1.78482653991729133580e0)), r,
                sk(5.46378491116411436990e0)), r, sk(6.65790464350110377720e0));
    const double den =
        fma(fma(fma(fma(fma(fma(fma(sk(2.04426310338993978564e-15), r, sk(1.42151175831644588870e-7)), r,
                                sk(1.84631831751005468180e-5)), r, sk(7.86869131145613259100e-4)), r,
                        sk(1.48753612908506148525e-2)), r, sk(1.36929880922735805310e-1)), r,
                sk(5.99832206555887937690e-1)), r, 1.0);
    return -(num / den);
}

// The component data a draw needs (SampRec's fields, or a workgroup's LDS
// copy): mean, signed sigma, the interval's cut masses and mass, and the
// pick's threshold interval [tlo, thi) of the component (integers,
// thr = ceil(cdf 2^32)) with iw = 1 / (thi - tlo).
struct DrawComp {
    double mu, ssg, p0, q0, m, iw;
    uint64_t tlo, thi;
};

// One candidate from its two Philox words: wp picked the component (its
// threshold interval holds wp), wu is the uniform.
//   v = (wu + r) 2^-32 in (0, 1): r = (wp - tlo + 1/2) / (thi - tlo) is wp's
//     position inside the picked component's interval -- uniform and
//     independent of the component and of wu (~log2(w 2^32) more bits, so
//     the tails reach ~9 sigma); 1 - v is formed the same way from the other
//     end, exactly;
//   p = p0 + m v and q = q0 + m (1 - v): the normal's CDF at the draw and its
//     complement, each accurate where it is small;
//   z = Phi^-1(p) (lower tail of p or of q), x = mu + ssg z;
//   bounded labels: x clamped into [low, high) -- a rounding at an end of
//     the interval, ~1e-16 of the draws.
// A component of zero mass (m = 0: the mixture's truncated mass is zero,
// k_samp_fold) returns NaN -- the callers raise the sampler error.
__device__ __forceinline__ double icdf_draw(const DLabel& L, const DrawComp& c, uint32_t wp, uint32_t wu) {
    const double r = ((double)(wp - (uint32_t)c.tlo) + 0.5) * c.iw;
    const double rb = ((double)((uint32_t)(c.thi - 1 - c.tlo) - (wp - (uint32_t)c.tlo)) + 0.5) * c.iw;
    const double v = ((double)wu + r) * 0x1.0p-32;
    const double vb = ((double)(0xFFFFFFFFu - wu) + rb) * 0x1.0p-32;
    const double p = fma(c.m, v, c.p0), q = fma(c.m, vb, c.q0);
    const double z = p <= 0.5 ? ndtri_lower(p) : -ndtri_lower(q);
    double x = fma(c.ssg, z, c.mu);
    if ((L.flags & 3) == 3) {
        x = x < L.low ? L.low : x;
        x = x >= L.high ? nextafter(L.high, -__builtin_inf()) : x;
    }
    return c.m > 0.0 ? x : __builtin_nan("");
}

// first k with cdf[k] > u (cdf[n-1] == 1 exactly, u < 1).
__device__ __forceinline__ int cdf_search(const SampRec* __restrict__ s, int n, double u) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid].cdf > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// The pick's integer threshold of cumulative weight c: ceil(c 2^32) (exact: a
// power-of-two scaling, c in [0, 1]); cdf[k] <= u = w 2^-32  <=>  thr[k] <= w
__device__ __forceinline__ uint64_t pick_thr(double c) { return (uint64_t)ceil(c * 0x1.0p32); }

// Component lookup of the draw: the first k with thr[k] > w.  SampGlobal
// searches the records in global memory; SampShared (a workgroup's copy in
// LDS, stage_samp, padded to 64 entries) starts from a 256-cell guide
// (gd[j] = the first k with cdf[k] > j / 256, j = the top 8 bits of w) and
// takes at most `steps` more comparisons -- the most cumulative weights any
// cell holds, 1 for mixtures without weights below 1/256 -- else a
// branch-free lower bound over all 64; the categorical tile kernel walks
// the 64-entry guide table (guide[j] = the first k with cdf[k] > j / 64).
// All return the same component and the same DrawComp bits.
struct SampGlobal {
    const SampRec* __restrict__ s;
    int ns;
    __device__ __forceinline__ DrawComp comp(uint32_t w) const {
        const int k = cdf_search(s, ns, (double)w * 0x1.0p-32);
        const SampRec r = s[k];
        DrawComp c;
        c.mu = r.mu;
        c.ssg = r.ssg;
        c.p0 = r.p0;
        c.q0 = r.q0;
        c.m = r.m;
        c.tlo = k ? pick_thr(s[k - 1].cdf) : 0;
        c.thi = pick_thr(r.cdf);
        c.iw = 1.0 / (double)(c.thi - c.tlo);
        return c;
    }
};

constexpr int kSampLds = 64;     // below components staged in LDS (K_b <= 26 in practice)
constexpr int kGuideSteps = 3;   // guided picks take at most this many comparisons
struct alignas(16) SampLds {
    double cdf[kSampLds], mu[kSampLds], ssg[kSampLds], p0[kSampLds], q0[kSampLds], m[kSampLds], iw[kSampLds];
    uint64_t thr[kSampLds];   // ceil(cdf 2^32)
    uint32_t thr1[kSampLds];  // thr - 1 (thr >= 1 wherever the guided pick compares: thr <= w <=> thr1 < w)
    uint8_t guide[64];
    uint8_t gd[256];
    int steps;
};

struct SampShared {
    const SampLds* __restrict__ t;
    int steps = -1;   // t->steps read once by the caller (-1: read per pick)
    __device__ __forceinline__ int pick_index(uint32_t w) const {
        // (steps is the same for the whole workgroup: a scalar branch)
        const int st = steps >= 0 ? steps : __builtin_amdgcn_readfirstlane(t->steps);
        int k;
        if (st <= kGuideSteps) {
            // (from the guide on, cdf[k] > (w >> 24) 2^-8 >= 0: thr[k] >= 1, so
            // the 32-bit thr1 compare is the 64-bit one)
            k = t->gd[w >> 24];
#pragma unroll
            for (int s = 0; s < kGuideSteps; ++s)
                if (s < st) k += t->thr1[k] < w ? 1 : 0;   // (k <= ns - 1 throughout: thr[ns - 1] = 2^32 > w)
        } else {   // branch-free lower bound over the 64 (padded with 2.0: thr 2^33)
            k = 0;
#pragma unroll
            for (int step = kSampLds / 2; step > 0; step >>= 1) k = t->thr[k + step - 1] <= w ? k + step : k;
        }
        return k;
    }
    __device__ __forceinline__ DrawComp comp_at(int k) const {
        DrawComp c;
        c.mu = t->mu[k];
        c.ssg = t->ssg[k];
        c.p0 = t->p0[k];
        c.q0 = t->q0[k];
        c.m = t->m[k];
        c.iw = t->iw[k];
        c.tlo = k ? t->thr[k - 1] : 0;
        c.thi = t->thr[k];
        return c;
    }
    __device__ __forceinline__ DrawComp comp(uint32_t w) const { return comp_at(pick_index(w)); }
};

// a workgroup's LDS copy of label L's below sampling records (false, and
// nothing staged, when K_b > kSampLds); every thread must call it
__device__ __forceinline__ bool stage_samp(const DLabel& L, const SampRec* __restrict__ samp, SampLds* t) {
    if (L.ns > kSampLds || L.ns < 1) return false;
    for (int k = threadIdx.x; k < kSampLds; k += blockDim.x) {
        if (k < L.ns) {
            const SampRec r = samp[L.samp_off + k];
            const uint64_t thi = pick_thr(r.cdf), tlo = k ? pick_thr(samp[L.samp_off + k - 1].cdf) : 0;
            t->cdf[k] = r.cdf;
            t->thr[k] = thi;
            t->thr1[k] = (uint32_t)(thi - 1);   // (thi = 0: never compared by the guided pick)
            t->mu[k] = r.mu;
            t->ssg[k] = r.ssg;
            t->p0[k] = r.p0;
            t->q0[k] = r.q0;
            t->m[k] = r.m;
            t->iw[k] = 1.0 / (double)(thi - tlo);   // (SampGlobal::comp's expression: the same bits)
        } else {   // padding: never picked (u < 1 <= cdf[ns - 1])
            t->cdf[k] = 2.0;
            t->thr[k] = 1ull << 33;
            t->thr1[k] = 0xffffffffu;   // (never reached: thr[ns - 1] = 2^32 stops the pick)
            t->mu[k] = 0.0;
            t->ssg[k] = 0.0;
            t->p0[k] = 0.0;
            t->q0[k] = 0.0;
            t->m[k] = 0.0;
            t->iw[k] = 0.0;
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

// stage_samp's LDS image kept in global memory (k_samp_image, once per
// posterior): a workgroup that only needs the staged table copies it with
// 16-byte loads instead of rebuilding the thresholds and guides
constexpr int kSampImgVec = (int)((sizeof(SampLds) + 15) / 16);
__device__ __forceinline__ void stage_samp_image(const uint4* __restrict__ img, SampLds* t) {
    uint4* d = reinterpret_cast<uint4*>(t);
    for (int k = threadIdx.x; k < kSampImgVec; k += blockDim.x) d[k] = img[k];
    __syncthreads();
}

// Phi(x) = erfc(-x / sqrt 2) / 2 (accurate in both tails)
__device__ __forceinline__ double ncdf(double x) { return 0.5 * erfc(-x * 0.70710678118654752440); }

// The truncated-normal terms of one sampling component (SampRec.ssg, p0,
// q0, m).  tpe.py:88-93 retries (component ~ w, x ~ N(mu, sigma)) until low
// <= x < high: component k is accepted with probability m_k, its mass in the
// bounds, so the accepted draw takes k with probability w_k m_k / sum w m
// and x ~ N(mu_k, sigma_k) restricted to the bounds.  With a = (low - mu) /
// sigma, b = (high - mu) / sigma: a component whose mean is at or below low
// (a >= 0) is mirrored (z -> -z: [a', b') = [-b, -a), ssg = -sigma) so that
// a' < 0 always and p0 = Phi(a'), q0 = Phi(-b') are both accurate; m =
// Phi(b') - p0 when b' <= 0, else 1 - p0 - q0.  Labels without both bounds
// (and categorical ones): m = 1, p0 = q0 = 0.
__device__ __forceinline__ void samp_trunc(const DLabel& L, SampRec& s) {
#pragma clang fp contract(off)
    s.ssg = s.sigma;
    s.p0 = 0.0;
    s.q0 = 0.0;
    s.m = 1.0;
    if (L.mode == CAT || (L.flags & 3) != 3) return;
    if (!(s.sigma > 0.0 && s.sigma < __builtin_inf())) {   // (a point mass, or no distribution)
        s.ssg = 0.0;
        s.m = (L.low <= s.mu && s.mu < L.high) ? 1.0 : 0.0;
        return;
    }
    const double a = (L.low - s.mu) / s.sigma, b = (L.high - s.mu) / s.sigma;
    const bool flip = a >= 0.0;
    const double a2 = flip ? -b : a, b2 = flip ? -a : b;
    s.ssg = flip ? -s.sigma : s.sigma;
    s.p0 = ncdf(a2);
    s.q0 = ncdf(-b2);
    const double m = b2 <= 0.0 ? ncdf(b2) - s.p0 : (1.0 - s.p0) - s.q0;
    s.m = m > 0.0 ? m : 0.0;
}

// The below mixture's sampling records of one label, folded in place by
// every thread of one block (k_fold for device builds, k_samp_fold for
// host-uploaded posteriors: one function, so both draw the same bits).  On
// entry s[k] holds mu, sigma and wd = the raw weight w_k; on exit the pick's
// cumulative weights cdf_k = sum_{i<=k} w_i m_i / Z (summed in order by one
// thread; cdf_{ns-1} = 1 exactly), wd_k = w_k / Z and the truncation terms.
// Z = 0 (the bounds hold none of the mixture's mass: the reference's loop
// would never end) leaves every m = 0, so every draw fails loudly.  Returns
// (thread 0) whether sum w > 0.
__device__ __forceinline__ bool samp_fold_block(const DLabel& L, SampRec* __restrict__ s, int ns) {
#pragma clang fp contract(off)
    for (int k = threadIdx.x; k < ns; k += blockDim.x) {
        SampRec r = s[k];
        samp_trunc(L, r);
        s[k] = r;
    }
    __syncthreads();
    // the cumulative sums in order on one thread, from LDS copies when the
    // mixture fits (a dependent global load per step cost ~40 us per build)
    constexpr int kFoldLds = 64;
    __shared__ double fw[kFoldLds], fm[kFoldLds], fc[kFoldLds];
    __shared__ bool fok;
    const bool lds = ns <= kFoldLds;
    if (lds)
        for (int k = threadIdx.x; k < ns; k += blockDim.x) {
            fw[k] = s[k].wd;
            fm[k] = s[k].m;
        }
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0, Z = 0.0;
        for (int k = 0; k < ns; ++k) {
            const double w = lds ? fw[k] : s[k].wd, m = lds ? fm[k] : s[k].m;
            tot += w;
            Z += w * m;
        }
        fok = tot > 0.0;
        const bool zero = !(Z > 0.0);
        double run = 0.0;
        for (int k = 0; k < ns; ++k) {
            const double w = lds ? fw[k] : s[k].wd, m = lds ? fm[k] : s[k].m;
            run += w * m;
            const double c = (k == ns - 1 || zero) ? 1.0 : run / Z;
            if (lds) {
                fc[k] = c;
                fw[k] = zero ? 0.0 : w / Z;
                fm[k] = zero ? 0.0 : m;
            } else {
                s[k].cdf = c;
                s[k].wd = zero ? 0.0 : w / Z;
                if (zero) s[k].m = 0.0;
            }
        }
    }
    __syncthreads();
    if (lds)
        for (int k = threadIdx.x; k < ns; k += blockDim.x) {
            s[k].cdf = fc[k];
            s[k].wd = fw[k];
            s[k].m = fm[k];
        }
    __syncthreads();
    return fok;
}

// Candidates 2p and 2p + 1 share one Philox4x32-10 call: the counter is (p,
// 0, label stream, round); words x, y are candidate 2p's pick and uniform,
// words z, w candidate 2p + 1's.  draw_pair draws both, draw_one one of
// them -- the same arithmetic, so the same bits.  The value is the draw
// space's (LGMM1: log space, before the exp).
template <typename Src>
__device__ __forceinline__ void draw_pair(const DLabel& L, const Src& src, uint32_t k0, uint32_t k1, uint32_t p,
                                          uint32_t round, double& d0, double& d1) {
    const U4 r = philox4x32_10(U4{p, 0u, (uint32_t)L.stream, round}, k0, k1);
    d0 = icdf_draw(L, src.comp(r.x), r.x, r.y);
    d1 = icdf_draw(L, src.comp(r.z), r.z, r.w);
}

template <typename Src>
__device__ __forceinline__ double draw_one(const DLabel& L, const Src& src, uint32_t k0, uint32_t k1, uint32_t g,
                                           uint32_t round) {
    const U4 r = philox4x32_10(U4{g >> 1, 0u, (uint32_t)L.stream, round}, k0, k1);
    const bool h = (g & 1u) != 0;
    const uint32_t wp = h ? r.z : r.x, wu = h ? r.w : r.y;
    return icdf_draw(L, src.comp(wp), wp, wu);
}

// the Philox words of candidate g (pick, uniform): k_hot_bx's prefilter
// decides most candidates from them alone
__device__ __forceinline__ void draw_words(const DLabel& L, uint32_t k0, uint32_t k1, uint32_t g, uint32_t round,
                                           uint32_t& wp, uint32_t& wu) {
    const U4 r = philox4x32_10(U4{g >> 1, 0u, (uint32_t)L.stream, round}, k0, k1);
    const bool h = (g & 1u) != 0;
    wp = h ? r.z : r.x;
    wu = h ? r.w : r.y;
}

// Slot r of thread t in a tile of R x nthreads candidates (R even): slots
// r, r + 1 are one Philox pair, candidates 2 ((r / 2) nthreads + t) and
// the next one
__device__ __host__ __forceinline__ uint32_t tile_cand(int r, uint32_t t, uint32_t nthreads) {
    return 2u * ((uint32_t)(r >> 1) * nthreads + t) + (uint32_t)(r & 1);
}

// LGMM1 sample value of a log-space draw (tpe.py:255: np.exp); RAW
// sample_slots leave this step to the caller
__device__ __forceinline__ double lgmm_value(double draw) { return exp(draw); }

// Draw one sample of the below posterior for global candidate g, BEFORE
// quantization (LGMM1: after the exp).
// GMM1 / LGMM1 (tpe.py:68-99 / 222-256): the reference draws component ~
// weights and x ~ N(mu, sigma), retrying both until low <= x < high; the
// accepted draw is component k with probability w_k m_k / sum w m (m_k: the
// component's mass inside the bounds) and x ~ N(mu_k, sigma_k) restricted to
// [low, high) -- drawn here directly by the inverse CDF (icdf_draw), no
// retries.  LGMM1 then exp(x).
// categorical (stochastic.py:109-147): index ~ p.
// Returns false when the bounds hold no mass (NaN: the reference's loop
// would never end).
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
        const double draw = draw_one(L, SampGlobal{s, L.ns}, k0, k1, g, round);
        out = (MODE == DENSE_LGMM || MODE == QUANT_LGMM) ? lgmm_value(draw) : draw;
        return draw == draw;
    }
}

// sample_raw for the R slots of a thread (bit for bit the same draws).
// Slots outside `pend` keep their value.  Returns false if a slot's draw
// failed (NaN).
template <int MODE, int R, typename Src, bool RAW = false>
__device__ __forceinline__ bool sample_slots(const DLabel& L, const Src& src, uint64_t seed,
                                             const uint32_t (&rk)[R], const uint32_t (&g)[R], uint32_t pend,
                                             double (&out)[R]) {
    static_assert(MODE != CAT, "categorical slots draw once each");
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    bool ok = true;
    // (every slot is drawn, pending or not: no branch)
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double draw = draw_one(L, src, k0, k1, g[r], rk[r]);
        const bool p = (pend >> r) & 1u;
        out[r] = p ? draw : out[r];
        ok = ok && (!p || draw == draw);
    }
    if constexpr ((MODE == DENSE_LGMM || MODE == QUANT_LGMM) && !RAW) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((pend >> r) & 1u) out[r] = lgmm_value(out[r]);
    }
    return ok;
}

// set bits of a wave mask below this lane (v_mbcnt_lo + v_mbcnt_hi)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// sample_slots for tile kernels: slot r of thread t holds candidate g0 +
// tile_cand(r, t, blockDim): slots r, r + 1 are a Philox pair, drawn by one
// call (draw_pair) when g0 is even.  Slots outside `pend` receive
// unspecified values (the callers read the pending slots only).
template <int MODE, int R, typename Src, bool RAW = false>
__device__ __forceinline__ bool sample_tile(const DLabel& L, const Src& src, uint64_t seed, uint32_t rk,
                                            uint32_t g0, uint32_t pend, double (&out)[R]) {
    static_assert(MODE != CAT, "categorical slots draw once each");
    static_assert(R % 2 == 0, "sample_tile draws Philox pairs");
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const bool paired = (g0 & 1u) == 0;   // (an odd first index: each slot on its own, the same bits)
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; r += 2) {
        const uint32_t c0 = tile_cand(r, threadIdx.x, blockDim.x);
        if (paired) {
            draw_pair(L, src, k0, k1, (g0 + c0) >> 1, rk, out[r], out[r + 1]);
        } else {
            out[r] = draw_one(L, src, k0, k1, g0 + c0, rk);
            out[r + 1] = draw_one(L, src, k0, k1, g0 + c0 + 1u, rk);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) ok = ok && (!((pend >> (r + h)) & 1u) || out[r + h] == out[r + h]);
    }
    if constexpr ((MODE == DENSE_LGMM || MODE == QUANT_LGMM) && !RAW) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((pend >> r) & 1u) out[r] = lgmm_value(out[r]);
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
constexpr int kSumSlice = 64;

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
