// tpe_expand.hip -- the index of the expansion screen (tpe_device.h,
// "expansion screen"): per dense label of the resident posterior, bins of
// the candidate range with the Taylor coefficients of the clipped above
// components and the list of the other above components that reach each
// bin.  Built once per posterior, lazily, before the first large sampled
// round (bx_prepare); k_screen_bx (tpe_engine.hip) uses it.
//
//   k_bx_scan     per label: candidate range, a* (the largest above record
//                 scale = the clipped sigma's), unclipped count
//   (host)        bins per label from kappa and the cut T: the Taylor argument
//                 2 kappa |d| |delta| stays <= ~0.5, so 15 terms leave a
//                 truncation ~4e-17 of the bin's mass
//   k_bx_compact  per label: the unclipped components in record order
//   k_bx_count    per bin: unclipped components whose term can reach 2^-T in it
//   k_bx_offsets  per label: their exclusive scan (list offsets), the total
//   k_bx_fill     per bin: the list
//   k_bx_table    per bin (one wave): A_0..A_14 over the clipped components within the
//                 window, and the absolute bound Eabs of truncation + rounding
//
// Bounds (natural-log units, records as tpe_device.h Comp: c'/K = log coef -
// M <= 0, a'^2 / K = 1 / (2 sigma^2)): a clipped component farther than
// dwin = sqrt(T ln 2 / kappa) + rmax from a bin centre has every term below
// 2^-T in the bin, and so has an unclipped one left off the bin's list
// (reach test with a one-nat margin); the k_screen_bx bound adds na 2^-T for
// them.  Per clipped component in the window, with y = 2 kappa |d| rmax:
//   truncation   g y^P / P! e^y                          (Lagrange remainder)
//   rounding     g e^y ((3P + 10 + 4 |arg|) 2^-53        (g and the n-th term)
//                       + 2 kappa (|d| + r)(|mu'| + |d| + r) 2^-51)
//                                                         (mu' = m'/a', d, delta)
// and per bin (W + 6 + 2P + 8) 2^-53 G for the sums (per lane, then the
// butterfly) and the Horner evaluation
// (sum_n |A_n| |delta|^n <= G = sum_k g e^y), x 1.02.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>

#include "../../include/hyperopt_tpe.h"
#include "tpe_ctx.h"
#include "tpe_device.h"

using namespace tpe;
using tpe_rt::kBlock;

namespace {

constexpr double kInf = __builtin_inf();
constexpr double kLn2 = 0.6931471805599453;
constexpr double kU = 0x1.0p-53;
constexpr int kScanFields = 6;   // xlo, xhi, a*, unclipped, clipped, pad
constexpr int32_t kMaxUnclipped = 16384;
constexpr int32_t kMaxBins = 1 << 16;
constexpr int32_t kMinBins = 64;

__device__ double blk_max(double v, double* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh[0];
    for (int w = 1; w < kBlock / 64; ++w) r = fmax(r, sh[w]);
    __syncthreads();
    return r;
}

__device__ double blk_min(double v, double* sh) { return -blk_max(-v, sh); }

__device__ int blk_sum(int v, int* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int r = 0;
    for (int w = 0; w < kBlock / 64; ++w) r += sh[w];
    __syncthreads();
    return r;
}

// exclusive prefix of v over the block (thread order) and the total
__device__ int blk_prefix(int v, int* sh, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
    }
    if (lane == 63) sh[wave] = inc;
    __syncthreads();
    int before = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
        if (w < wave) before += sh[w];
        tot += sh[w];
    }
    __syncthreads();
    total = tot;
    return before + inc - v;
}

__device__ __forceinline__ bool usable(const Comp<double>& r) {
    return r.a > 0.0 && r.a < kInf && fabs(r.mu) < kInf;
}

// grid (dense labels): range, a*, counts -> scan[y * kScanFields ...]
__global__ __launch_bounds__(kBlock) void k_bx_scan(const DLabel* __restrict__ labels,
                                                    const int32_t* __restrict__ grp,
                                                    const Comp<double>* __restrict__ comps64,
                                                    const SampRec* __restrict__ samp,
                                                    double* __restrict__ scan) {
    const int y = blockIdx.x;
    const DLabel L = labels[grp[y]];
    __shared__ double shd[kBlock / 64];
    __shared__ int shi[kBlock / 64];
    double lo = kInf, hi = -kInf;
    if ((L.flags & 3) == 3) {   // (LGMM1: the bounds are in log space)
        lo = L.low;
        hi = L.high;
    } else {
        for (int k = threadIdx.x; k < L.ns; k += kBlock) {
            const SampRec s = samp[L.samp_off + k];
            lo = fmin(lo, s.mu - 8.0 * s.sigma);
            hi = fmax(hi, s.mu + 8.0 * s.sigma);
        }
        lo = blk_min(lo, shd);
        hi = blk_max(hi, shd);
    }
    const Comp<double>* c = comps64 + L.comp_a;
    double am = 0.0;
    for (int k = threadIdx.x; k < L.na; k += kBlock)
        if (usable(c[k])) am = fmax(am, c[k].a);
    am = blk_max(am, shd);
    int nc = 0, ncl = 0;
    for (int k = threadIdx.x; k < L.na; k += kBlock) {
        const bool cl = c[k].a == am;
        nc += !cl;
        ncl += cl;
    }
    nc = blk_sum(nc, shi);
    ncl = blk_sum(ncl, shi);
    if (threadIdx.x == 0) {
        double* o = scan + (size_t)y * kScanFields;
        o[0] = lo - L.centre;
        o[1] = hi - L.centre;
        o[2] = am;
        o[3] = (double)nc;
        o[4] = (double)ncl;
        o[5] = 0.0;
    }
}

// grid (dense labels): the unclipped above components' indices, record order
__global__ __launch_bounds__(kBlock) void k_bx_compact(const DLabel* __restrict__ labels,
                                                       const int32_t* __restrict__ grp,
                                                       const Comp<double>* __restrict__ comps64,
                                                       const BxLabel* __restrict__ bx,
                                                       int32_t* __restrict__ nc) {
    const int li = grp[blockIdx.x];
    const DLabel L = labels[li];
    const double am = bx[li].astar;
    __shared__ int shi[kBlock / 64];
    int base = 0;
    for (int k0 = 0; k0 < L.na; k0 += kBlock) {
        const int k = k0 + threadIdx.x;
        const bool f = k < L.na && comps64[L.comp_a + k].a != am;
        int tot;
        const int pos = blk_prefix((int)f, shi, tot);
        if (f) nc[L.comp_a + base + pos] = k;
        base += tot;
    }
}

// can unclipped record r have a term >= 2^-(T + 1.44) anywhere in bin b?
__device__ __forceinline__ bool reaches(const Comp<double>& r, const BxLabel& B, int b) {
    if (!(r.c > -kInf)) return false;              // never a term
    if (!usable(r)) return true;                   // let the direct term decide
    const double mu = r.mu / r.a, kap = r.a * r.a * kExpScaleInv;
    const double e0 = B.xlo + (double)b * B.bw, e1 = e0 + B.bw;
    const double slack = (fabs(e0) + fabs(e1) + B.bw) * 1e-12;
    const double dist = fmax(0.0, fmax(e0 - slack - mu, mu - e1 - slack)) * (1.0 - 1e-9);
    return r.c * kExpScaleInv - kap * dist * dist >= -(kBxT * kLn2 + 1.0);
}

// grid (ceil(max bins / 256), dense labels): per bin the count of reaching
// unclipped components (fill = false) or their list (fill = true)
template <bool FILL>
__global__ __launch_bounds__(kBlock) void k_bx_list(const DLabel* __restrict__ labels,
                                                    const int32_t* __restrict__ grp,
                                                    const Comp<double>* __restrict__ comps64,
                                                    const BxLabel* __restrict__ bx,
                                                    const int32_t* __restrict__ nc,
                                                    int32_t* __restrict__ loff,
                                                    int32_t* __restrict__ list) {
    const int li = grp[blockIdx.y];
    const DLabel L = labels[li];
    const BxLabel B = bx[li];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B.nbins) return;
    const Comp<double>* c = comps64 + L.comp_a;
    const int32_t* ncl = nc + L.comp_a;
    int cnt = 0;
    int32_t* out = FILL ? list + B.list_off + loff[B.cnt_off + b] : nullptr;
    for (int j = 0; j < B.n_nc; ++j) {
        const int k = ncl[j];
        if (reaches(c[k], B, b)) {
            if (FILL) out[cnt] = k;
            ++cnt;
        }
    }
    if (!FILL) loff[B.cnt_off + b] = cnt;
}

// grid (dense labels): counts -> exclusive offsets (nbins + 1 entries), total
__global__ __launch_bounds__(kBlock) void k_bx_offsets(const int32_t* __restrict__ grp,
                                                       const BxLabel* __restrict__ bx,
                                                       int32_t* __restrict__ loff,
                                                       int64_t* __restrict__ total) {
    const BxLabel B = bx[grp[blockIdx.x]];
    __shared__ int shi[kBlock / 64];
    int32_t* o = loff + B.cnt_off;
    int64_t base = 0;
    for (int b0 = 0; b0 < B.nbins; b0 += kBlock) {
        const int b = b0 + threadIdx.x;
        const int v = b < B.nbins ? o[b] : 0;
        int tot;
        const int pos = blk_prefix(v, shi, tot);
        if (b < B.nbins) o[b] = (int32_t)(base + pos);
        base += tot;
    }
    if (threadIdx.x == 0) {
        o[B.nbins] = (int32_t)base;
        total[blockIdx.x] = base;
    }
}

// 1 / n!, n <= kBxP
__constant__ double kInvFact[kBxP + 1] = {
    1.0, 1.0, 1.0 / 2, 1.0 / 6, 1.0 / 24, 1.0 / 120, 1.0 / 720, 1.0 / 5040, 1.0 / 40320, 1.0 / 362880,
    1.0 / 3628800, 1.0 / 39916800, 1.0 / 479001600, 1.0 / 6227020800.0, 1.0 / 87178291200.0,
    1.0 / 1307674368000.0};


// first record index k in [0, n) with mu'_k >= v (mu' = m'/a', sorted by mu)
__device__ __forceinline__ int lower_mu(const Comp<double>* __restrict__ c, int n, double v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const Comp<double> r = c[mid];
        const double mu = r.a > 0.0 ? r.mu / r.a : -kInf;
        if (mu >= v) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// grid (ceil(max bins / 4), dense labels): one wave per bin, its lanes
// striding over the window's clipped components, the partial sums added by a
// butterfly at the end (a bin's window holds thousands of components: one
// thread per bin left the chip ~0.6 waves per SIMD)
__global__ __launch_bounds__(kBlock) void k_bx_table(const DLabel* __restrict__ labels,
                                                     const int32_t* __restrict__ grp,
                                                     const Comp<double>* __restrict__ comps64,
                                                     const BxLabel* __restrict__ bx,
                                                     double* __restrict__ tab) {
    const int li = grp[blockIdx.y];
    const DLabel L = labels[li];
    const BxLabel B = bx[li];
    __shared__ double exp_tab[kExpTabSize];
    load_exp_table(exp_tab);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (b >= B.nbins) return;   // whole waves (after the table's barrier)
    const Comp<double>* c = comps64 + L.comp_a;
    const double xb = B.xlo + ((double)b + 0.5) * B.bw;
    const double r = B.rmax, kap = B.kappa;
    const double D = B.dwin * (1.0 + 1e-9) + (fabs(xb) + B.dwin) * 1e-12;
    // the window: records sorted by mu, so the clipped ones within D of xb
    // are a contiguous index range (margins cover mu' = m'/a' rounding)
    const int k0 = lower_mu(c, L.na, xb - D), k1 = lower_mu(c, L.na, xb + D);
    double A[kBxP];
#pragma unroll
    for (int n = 0; n < kBxP; ++n) A[n] = 0.0;
    double Rb = 0.0, G = 0.0, ERR = 0.0, W = 0.0;
    // mu' = m' (1 / a*): <= 1.5 ulp (inside the 2^-51 allowance below);
    // g = exp(arg) through the fp64 round's table exp (<= 2.6e-14 relative,
    // added to the rounding term); the powers g (2 kappa d)^n by one
    // multiply each, A_n += that / n! (one rounding each, inside 3P + 10)
    const double inv_a = 1.0 / B.astar;
    for (int k = k0 + lane; k < k1; k += 64) {
        const Comp<double> rec = c[k];
        if (rec.a != B.astar) continue;
        const double mu = rec.mu * inv_a, d = mu - xb;
        const double arg = rec.c * kExpScaleInv - kap * d * d;
        if (!(arg > -740.0)) continue;   // below 2^-1067 in the whole bin: in the skip term
        const double g = exp_scaled(fmin(arg * kExpScale, 0.0), exp_tab), two = 2.0 * kap * d;
        // e^y only enters the bounds: 1 + y + y^2 >= e^y for 0 <= y <= 1.79
        const double yv = fabs(two) * r, ey = yv <= 1.5 ? fma(yv, yv, 1.0 + yv) : exp(yv) * 1.000001;
        double t = g;
        A[0] += t;
#pragma unroll
        for (int n = 1; n < kBxP; ++n) {
            t *= two;
            A[n] = fma(t, kInvFact[n], A[n]);
        }
        const double tP = fabs(t * two) * kInvFact[kBxP];   // g |2 kappa d|^P / P!
        const double gy = g * ey;
        Rb += tP * B.rP * ey;
        G += gy;
        ERR += gy * ((3.0 * kBxP + 10.0 + 4.0 * fabs(arg)) * kU + 2.6e-14 +
                     2.0 * kap * (fabs(d) + r) * (fabs(mu) + fabs(d) + r) * 0x1.0p-51);
        W += 1.0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int n = 0; n < kBxP; ++n) A[n] += __shfl_xor(A[n], off);
        Rb += __shfl_xor(Rb, off);
        G += __shfl_xor(G, off);
        ERR += __shfl_xor(ERR, off);
        W += __shfl_xor(W, off);
    }
    if (lane != 0) return;
    double* row = tab + (size_t)(B.tab_off + b) * kBxRow;
#pragma unroll
    for (int n = 0; n < kBxP; ++n) row[n] = A[n];
    // sums: each lane's sequential part (<= W terms) then 6 butterfly levels
    row[kBxP] = 1.02 * (Rb + ERR + (W + 6.0 + 2.0 * kBxP + 8.0) * kU * G) + 1e-300;
}

// lo += the smallest, hi += the largest value of one component's term
// exp(c - kappa (x' - mu)^2) over x' in [e0, e1] (the term is unimodal in
// x'); eps covers the rounding of mu = m'/a', of the distances and of the
// exponent, generously
// (the exps through the fp64 round's LDS table: exp_scaled is within
// 2.6e-14 relative of exp, so 3e-14 more in eps keeps both sides rigorous)
__device__ __forceinline__ void gauss_bounds(const Comp<double>& r, double e0, double e1, double& lo,
                                             double& hi, const double* __restrict__ etab) {
    const double c = r.c * kExpScaleInv;
    if (!(c > -kInf)) return;   // zero weight: no term
    const double kap = r.a * r.a * kExpScaleInv, mu = r.mu / r.a;
    const double dn = mu < e0 ? e0 - mu : (mu > e1 ? mu - e1 : 0.0);
    const double df = fmax(fabs(e0 - mu), fabs(e1 - mu));
    const double eps = 1e-15 * (64.0 + 64.0 * sqrt(kap) * (fabs(e0) + fabs(e1) + fabs(mu)) + fabs(c)) + 3e-14;
    hi += exp_scaled((c - kap * dn * dn + eps) * kExpScale, etab);
    const double ul = (c - kap * df * df - eps) * kExpScale;
    lo += ul > -4.0e6 ? exp_scaled(ul, etab) : 0.0;   // (below ~2^-980: 0 is a lower bound)
}

// P(a0 <= draw < a1) of one sampling component N(mu, sg) (draw space), in
// fp32: the mass only steers tau0, never a bound
__device__ __forceinline__ double normal_mass(double mu, double sg, double a0, double a1) {
    const double s = 1.0 / (sg * 1.4142135623730951);
    const float z0 = (float)((a0 - mu) * s), z1 = (float)((a1 - mu) * s);
    return z0 > 0.0f ? 0.5 * (double)(erfcf(z0) - erfcf(z1)) : 0.5 * (double)(erfcf(-z1) - erfcf(-z0));
}

// grid (ceil(max sub-bins / 256), dense labels): one sub-bin per thread --
// the hot-bin prefilter's [L, U] of the fp64 score over the sub-bin (float,
// rounded outward) and the sampling mass p of the sub-bin (tpe_device.h,
// "hot-bin prefilter").  Below mixture: every component bounded term by
// term.  Above mixture: the bin's polynomial Taylor-shifted to the sub-bin
// centre (|A(dc + t) - A_0'| <= sum_n>0 |A_n'| h^n), +- its Eabs, times the
// range of exp(-kappa delta^2); the bin's list term by term; the skipped
// components' na 2^-T on the upper side.  U, L: log ratio of the bounds plus
// the shift difference, widened by 1e-7 (1 + |v|) and the fp64 round's own
// error; +inf / -inf where a sum is not safely inside the normal range or a
// record is unusable.
__global__ __launch_bounds__(kBlock) void k_bx_bounds(const DLabel* __restrict__ labels,
                                                      const int32_t* __restrict__ grp,
                                                      const Comp<double>* __restrict__ comps64,
                                                      const SampRec* __restrict__ samp,
                                                      const BxLabel* __restrict__ bx,
                                                      const double* __restrict__ tab,
                                                      const int32_t* __restrict__ loff,
                                                      const int32_t* __restrict__ list,
                                                      float2* __restrict__ sb, float* __restrict__ sbp) {
    const int li = grp[blockIdx.y];
    const DLabel L = labels[li];
    const BxLabel B = bx[li];
    __shared__ double etab[kExpTabSize];
    load_exp_table(etab);
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= nsb) return;
    const int b = (int)(j >> kBxSubBits);
    const double sw = B.bw / kBxSub;
    const double e0n = B.xlo + (double)j * sw, e1n = e0n + sw;
    // slack: the rounding of a candidate's sub-bin index, and (LGMM1: k_hot_bx
    // bins the raw draw) |log(exp(draw)) - draw| <= ~4e-16 (2 + |draw|)
    const double slack = 2e-10 * B.bw + 1e-15 * (fabs(e0n) + fabs(e1n) + fabs(L.centre) + 2.0);
    const double e0 = e0n - slack, e1 = e1n + slack;
    // sampling mass (steers tau0 only: nominal edges, bounded labels cut)
    double p = 0.0;
    {
        double a0 = L.centre + e0n, a1 = L.centre + e1n;
        if ((L.flags & 3) == 3) {
            a0 = fmax(a0, L.low);
            a1 = fmin(a1, L.high);
        }
        double prev = 0.0;
        for (int k = 0; k < L.ns && a1 > a0; ++k) {
            const SampRec s = samp[L.samp_off + k];
            const double w = s.cdf - prev;
            prev = s.cdf;
            if (w > 0.0 && s.sigma > 0.0 && s.sigma < kInf) p += w * normal_mass(s.mu, s.sigma, a0, a1);
        }
    }
    bool ok = true;
    double blo = 0.0, bhi = 0.0;
    for (int k = 0; k < L.nb; ++k) {
        const Comp<double> r = comps64[L.comp_b + k];
        if (!usable(r)) {
            ok = ok && !(r.c > -kInf);
            continue;
        }
        gauss_bounds(r, e0, e1, blo, bhi, etab);
    }
    // clipped above components: the bin's polynomial around the sub-bin centre
    const double xb = B.xlo + ((double)b + 0.5) * B.bw;
    const double dc = 0.5 * (e0 + e1) - xb, h = 0.5 * (e1 - e0);
    if (!(fabs(dc) + h <= B.rmax)) ok = false;
    const double* rw = tab + (size_t)(B.tab_off + b) * kBxRow;
    double c[kBxP];
    double G = 0.0, rp = 1.0;
#pragma unroll
    for (int n = 0; n < kBxP; ++n) {
        c[n] = rw[n];
        G += fabs(c[n]) * rp;
        rp *= fabs(dc) + h;
    }
    // Taylor shift: c <- coefficients of A(dc + t)
#pragma unroll
    for (int i = 0; i < kBxP - 1; ++i)
#pragma unroll
        for (int k = kBxP - 2; k >= i; --k) c[k] = fma(dc, c[k + 1], c[k]);
    double dev = 0.0, hp = h;
#pragma unroll
    for (int n = 1; n < kBxP; ++n) {
        dev += fabs(c[n]) * hp;
        hp *= h;
    }
    const double eabs = rw[kBxP];
    const double alo = c[0] - dev - 1e-13 * G - eabs, ahi = c[0] + dev + 1e-13 * G + eabs;
    const double d0 = dc - h, d1 = dc + h;
    const double dmin = (d0 <= 0.0 && d1 >= 0.0) ? 0.0 : fmin(fabs(d0), fabs(d1));
    const double dmax = fmax(fabs(d0), fabs(d1));
    const double emax = exp(-B.kappa * dmin * dmin) * (1.0 + 1e-14);
    const double emin = exp(-B.kappa * dmax * dmax) * (1.0 - 1e-14);
    double slo = alo > 0.0 ? emin * alo : 0.0, shi = ahi > 0.0 ? emax * ahi : 0.0;
    const Comp<double>* ca = comps64 + L.comp_a;
    const int j0 = loff[B.cnt_off + b], j1 = loff[B.cnt_off + b + 1];
    for (int jj = j0; jj < j1; ++jj) {
        const Comp<double> r = ca[list[B.list_off + jj]];
        if (!usable(r)) {
            ok = ok && !(r.c > -kInf);
            continue;
        }
        gauss_bounds(r, e0, e1, slo, shi, etab);
    }
    shi += (double)L.na * exp2(-kBxT);
    const double dsh = L.shift_b - L.shift_a;
    const double mag = fabs(L.shift_b) + fabs(L.shift_a) + 2.0 * (fabs(L.centre) + fabs(e0) + fabs(e1)) + 64.0;
    const double fe = (double)(L.nb + L.na + 64) * 0x1.0p-50 + mag * 0x1.0p-48;
    double U = kInf, Lo = -kInf;
    if (ok && bhi >= 1e-280 && slo >= 1e-280) {
        const double v = log(bhi) - log(slo) + dsh;
        if (v == v) U = v + 1e-7 * (1.0 + fabs(v)) + fe;
    }
    if (ok && blo >= 1e-280 && shi > 0.0 && shi < kInf) {
        const double v = log(blo) - log(shi) + dsh;
        if (v == v) Lo = v - 1e-7 * (1.0 + fabs(v)) - fe;
    }
    if (!(U == U) || !(Lo == Lo) || U < Lo) {
        U = kInf;
        Lo = -kInf;
    }
    sb[B.sb_off + j] = make_float2(float_up(U), float_down(Lo));
    sbp[B.sb_off + j] = (float)p;
}

}  // namespace

int tpe_rt::bx_prepare(tpe_ctx* ctx) {
    tpe_rt::Posterior& P = *ctx->P;
    if (P.bx_ready) return TPE_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = bx_build(ctx);
    if (rc == TPE_OK && ctx->timing) {   // the build's wall time, kernels included
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        ctx->prep_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return rc;
}

// the tables, lists and sub-bin bounds of every dense label (bx_prepare)
int tpe_rt::bx_build(tpe_ctx* ctx) {
    tpe_rt::Posterior& P = *ctx->P;
    P.bx_ok = false;
    const std::vector<int32_t>& gg = P.h_group[DENSE_GMM];
    const std::vector<int32_t>& gl = P.h_group[DENSE_LGMM];
    const int nl = (int)(gg.size() + gl.size());
    if (nl == 0) {
        P.bx_ready = true;
        return TPE_OK;
    }
    const int32_t* grp = P.groups.p + P.group_off[DENSE_GMM];
    HIPCHK(ctx, P.bx_scan.reserve((size_t)nl * kScanFields));
    hipLaunchKernelGGL(k_bx_scan, dim3(nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p,
                       P.samp.p, P.bx_scan.p);
    HIPCHK(ctx, hipGetLastError());
    std::vector<double> sc((size_t)nl * kScanFields);
    HIPCHK(ctx, hipMemcpyAsync(sc.data(), P.bx_scan.p, sc.size() * sizeof(double), hipMemcpyDeviceToHost,
                               ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    // bins per label
    P.bx_h.assign(P.n_labels, BxLabel{});
    bool ok = true;
    int64_t rows = 0, cnts = 0;
    int32_t bins_max = 0;
    for (int y = 0; y < nl; ++y) {
        const int li = y < (int)gg.size() ? gg[y] : gl[y - gg.size()];
        const double* s = sc.data() + (size_t)y * kScanFields;
        const double xlo = s[0], xhi = s[1], am = s[2];
        const int32_t n_nc = (int32_t)s[3], n_cl = (int32_t)s[4];
        BxLabel B{};
        const double kap = am * am * kExpScaleInv;
        if (!(am > 0.0) || !(kap > 0.0 && kap < 1e300) || !(xhi > xlo) || !std::isfinite(xhi - xlo) ||
            n_nc > kMaxUnclipped || n_cl < 1) {
            ok = false;
            break;
        }
        const double d0 = std::sqrt(kBxT * kLn2 / kap);
        const double r_target = 0.25 / (kap * d0);   // Taylor argument 2 kappa |d| r <= ~0.5
        const double want = (xhi - xlo) / (2.0 * r_target);
        if (!(want <= (double)kMaxBins)) {
            ok = false;
            break;
        }
        int32_t nb = kMinBins;
        while ((double)nb < want) nb <<= 1;
        if ((int64_t)nb * std::max(n_nc, 1) > ((int64_t)1 << 27)) {   // list build cost
            ok = false;
            break;
        }
        B.xlo = xlo;
        B.bw = (xhi - xlo) / nb;
        B.inv_bw = 1.0 / B.bw;
        B.rmax = 0.5 * B.bw * (1.0 + 1e-9);
        B.astar = am;
        B.kappa = kap;
        B.dwin = d0 + B.rmax;
        B.rP = std::pow(B.rmax, (double)kBxP) * (1.0 + 1e-12);
        B.nbins = nb;
        B.n_nc = n_nc;
        B.inv_sbw = (double)kBxSub / B.bw;
        B.sb_off = rows * kBxSub;
        B.tab_off = rows;
        B.cnt_off = cnts;
        rows += nb;
        cnts += nb + 1;
        bins_max = std::max(bins_max, nb);
        P.bx_h[li] = B;
    }
    if (!ok) {
        P.bx_ready = true;   // not eligible: the windowed screen runs
        return TPE_OK;
    }
    HIPCHK(ctx, P.bx.reserve(P.n_labels));
    HIPCHK(ctx, P.bx_tab.reserve((size_t)rows * kBxRow));
    HIPCHK(ctx, P.bx_loff.reserve((size_t)cnts));
    HIPCHK(ctx, P.bx_nc.reserve(P.comps64.cap));
    HIPCHK(ctx, hipMemcpyAsync(P.bx.p, P.bx_h.data(), P.n_labels * sizeof(BxLabel), hipMemcpyHostToDevice,
                               ctx->stream));
    const dim3 gb((unsigned)((bins_max + kBlock - 1) / kBlock), nl);
    hipLaunchKernelGGL(k_bx_compact, dim3(nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p,
                       P.bx.p, P.bx_nc.p);
    hipLaunchKernelGGL(k_bx_list<false>, gb, dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p,
                       P.bx.p, P.bx_nc.p, P.bx_loff.p, nullptr);
    int64_t* tot = reinterpret_cast<int64_t*>(P.bx_scan.p);   // the scan is read: reuse it
    hipLaunchKernelGGL(k_bx_offsets, dim3(nl), dim3(kBlock), 0, ctx->stream, grp, P.bx.p, P.bx_loff.p, tot);
    HIPCHK(ctx, hipGetLastError());
    std::vector<int64_t> tot_h(nl);
    HIPCHK(ctx, hipMemcpyAsync(tot_h.data(), tot, nl * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    int64_t lsum = 0;
    for (int y = 0; y < nl; ++y) {
        const int li = y < (int)gg.size() ? gg[y] : gl[y - gg.size()];
        if (tot_h[y] > ((int64_t)1 << 30)) return ctx->fail(TPE_ERR_ARG, "expansion screen: lists too long");
        P.bx_h[li].list_off = lsum;
        lsum += tot_h[y];
    }
    HIPCHK(ctx, P.bx_list.reserve((size_t)std::max<int64_t>(lsum, 1)));
    HIPCHK(ctx, hipMemcpyAsync(P.bx.p, P.bx_h.data(), P.n_labels * sizeof(BxLabel), hipMemcpyHostToDevice,
                               ctx->stream));
    hipLaunchKernelGGL(k_bx_list<true>, gb, dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p,
                       P.bx.p, P.bx_nc.p, P.bx_loff.p, P.bx_list.p);
    const dim3 gt((unsigned)((bins_max + kBlock / 64 - 1) / (kBlock / 64)), nl);
    hipLaunchKernelGGL(k_bx_table, gt, dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p, P.bx.p,
                       P.bx_tab.p);
    HIPCHK(ctx, P.bx_sb.reserve((size_t)rows * kBxSub));
    HIPCHK(ctx, P.bx_sbp.reserve((size_t)rows * kBxSub));
    P.bx_sb_max = (int64_t)bins_max * kBxSub;
    static uint64_t gen_counter = 0;   // unique over every posterior of the process
    P.bx_gen = __atomic_add_fetch(&gen_counter, 1, __ATOMIC_RELAXED);
    const dim3 gs((unsigned)((P.bx_sb_max + kBlock - 1) / kBlock), nl);
    hipLaunchKernelGGL(k_bx_bounds, gs, dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p, P.samp.p,
                       P.bx.p, P.bx_tab.p, P.bx_loff.p, P.bx_list.p, P.bx_sb.p, P.bx_sbp.p);
    HIPCHK(ctx, hipGetLastError());
    P.bx_ok = true;
    P.bx_ready = true;
    return TPE_OK;
}
