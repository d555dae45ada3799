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
//                 truncation ~4e-17 of the bin's mass.  (Bins twice as wide,
//                 argument <= ~1, were measured in round 5: the index 0.63 ->
//                 0.49 ms, but the screen certified only 70-80 % of the
//                 candidates -- the bound's e^y and cancellation terms -- and
//                 the round re-scored 419k near-ties instead of 186: 1.48 ->
//                 4.37 ms, r5g.)
//   k_bx_compact  per label: the unclipped components in record order
//   k_bx_list     per bin: the unclipped components whose term can reach 2^-T
//                 in it, into the bin's slot of n_nc entries, and their count
//   k_bx_table    per bin (one thread): A_0..A_14 over the clipped components
//                 within the window, and the absolute bound Eabs of truncation
//                 + rounding
//   k_bx_bounds   per sub-bin: the hot-bin prefilter's [L, U] and sampling mass
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
#include <cstring>
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

// grid (dense labels): range, a*, counts -> scan[y * kScanFields ...].
// The candidate range of a label without both bounds covers each sampling
// component k to z_k sigma_k with w_k Q(z_k) <= kRangeTail (at most 8 sigma):
// a candidate outside the bins is always listed and scored in fp64 (exact,
// only slower), and at 2^24 candidates per round that happens ~1e-3 times per
// label; a one-sided bound cuts the range on its side.
constexpr double kRangeTail = 1e-10;
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
            const double w = s.wd;   // (no bounds here: the pick's weight)
            // Q(z) <= exp(-z^2 / 2) / 2: z = sqrt(2 ln(w / tail)) suffices
            const double z = w > kRangeTail ? fmin(8.0, sqrt(2.0 * log(w / kRangeTail))) : 0.0;
            lo = fmin(lo, s.mu - z * s.sigma);
            hi = fmax(hi, s.mu + z * s.sigma);
        }
        lo = blk_min(lo, shd);
        hi = blk_max(hi, shd);
        if (L.flags & 1) lo = fmax(lo, L.low);
        if (L.flags & 2) hi = fmin(hi, L.high);
    }
    const Comp<double>* c = comps64 + L.comp_a;
    // (kScanU records per thread loaded before use: a dependent load per
    // record left the 10k-record passes latency-bound)
    constexpr int kScanU = 8;
    double am = 0.0;
    for (int k0 = threadIdx.x; k0 < L.na; k0 += kBlock * kScanU) {
        Comp<double> r[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const int k = k0 + u * kBlock;
            r[u] = k < L.na ? c[k] : Comp<double>{0.0, 0.0, 0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u)
            if (k0 + u * kBlock < L.na && usable(r[u])) am = fmax(am, r[u].a);
    }
    am = blk_max(am, shd);
    int nc = 0, ncl = 0;
    for (int k0 = threadIdx.x; k0 < L.na; k0 += kBlock * kScanU) {
        double a[kScanU];
#pragma unroll
        for (int u = 0; u < kScanU; ++u) {
            const int k = k0 + u * kBlock;
            a[u] = k < L.na ? c[k].a : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kScanU; ++u)
            if (k0 + u * kBlock < L.na) {
                const bool cl = a[u] == am;
                nc += !cl;
                ncl += cl;
            }
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
    // kCompactU consecutive records per thread (record order kept): one
    // block scan per kBlock x kCompactU records (per kBlock, the 40 scans
    // of a 10k-record label took ~20 us)
    constexpr int kCompactU = 8;
    int base = 0;
    for (int k0 = 0; k0 < L.na; k0 += kBlock * kCompactU) {
        const int kt = k0 + (int)threadIdx.x * kCompactU;
        bool f[kCompactU];
        int mine = 0;
#pragma unroll
        for (int u = 0; u < kCompactU; ++u) {
            f[u] = kt + u < L.na && comps64[L.comp_a + kt + u].a != am;
            mine += f[u];
        }
        int tot;
        int at = base + blk_prefix(mine, shi, tot);
#pragma unroll
        for (int u = 0; u < kCompactU; ++u)
            if (f[u]) nc[L.comp_a + at++] = kt + u;
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
    return r.c * kExpScaleInv - kap * dist * dist >= -(B.tcut * kLn2 + 1.0);
}

// grid (ceil(max bins / 256), dense labels): per bin the unclipped
// components that reach it, in record order, into the bin's slot of n_nc
// entries (list_off + b n_nc), their count into cnt[cnt_off + b]
__global__ __launch_bounds__(kBlock) void k_bx_list(const DLabel* __restrict__ labels,
                                                    const int32_t* __restrict__ grp,
                                                    const Comp<double>* __restrict__ comps64,
                                                    const BxLabel* __restrict__ bx,
                                                    const int32_t* __restrict__ nc,
                                                    int32_t* __restrict__ cnt,
                                                    int32_t* __restrict__ list) {
    const int li = grp[blockIdx.y];
    const BxLabel B = bx[li];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if ((int)(blockIdx.x * kBlock) >= B.nbins) return;   // (the whole workgroup)
    const DLabel L = labels[li];
    const Comp<double>* c = comps64 + L.comp_a;
    const int32_t* ncl = nc + L.comp_a;
    // the unclipped records staged kBlock at a time in LDS (every lane reads
    // every record: walked in global memory they were two dependent loads
    // per record, ~45 us a launch)
    __shared__ Comp<double> sc[kBlock];
    __shared__ int32_t sk[kBlock];
    int m = 0;
    int32_t* out = list + B.list_off + (int64_t)b * B.n_nc;
    for (int j0 = 0; j0 < B.n_nc; j0 += kBlock) {
        const int nj = min(kBlock, B.n_nc - j0);
        __syncthreads();   // (the previous chunk read by every lane)
        if ((int)threadIdx.x < nj) {
            const int k = ncl[j0 + threadIdx.x];
            sk[threadIdx.x] = k;
            sc[threadIdx.x] = c[k];
        }
        __syncthreads();
        if (b < B.nbins)
            for (int j = 0; j < nj; ++j)
                if (reaches(sc[j], B, b)) out[m++] = sk[j];
    }
    if (b < B.nbins) cnt[B.cnt_off + b] = m;
}

// 1 / n!, n <= kBxP
__constant__ double kInvFact[kBxP + 1] = {
    1.0, 1.0, 1.0 / 2, 1.0 / 6, 1.0 / 24, 1.0 / 120, 1.0 / 720, 1.0 / 5040, 1.0 / 40320, 1.0 / 362880,
    1.0 / 3628800, 1.0 / 39916800, 1.0 / 479001600, 1.0 / 6227020800.0, 1.0 / 87178291200.0,
    1.0 / 1307674368000.0};


__device__ __forceinline__ double rec_mu(const Comp<double>& r) { return r.a > 0.0 ? r.mu / r.a : -kInf; }

// The wave's first record index with mu' >= v0 (-> k0) and with mu' >= v1
// (-> k1) over records [0, n) sorted by mu (mu' = m'/a'): lanes 0..31 search
// v0, lanes 32..63 v1, each half probing 32 evenly spaced records per step
// (~4 dependent loads for 10k records instead of 13)
__device__ __forceinline__ void wave_window(const Comp<double>* __restrict__ c, int n, double v0, double v1,
                                            int& k0, int& k1) {
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const double v = half ? v1 : v0;
    int lo = 0, hi = n;   // the answer lies in [lo, hi]
    while (__ballot(hi > lo)) {
        const int span = hi - lo;
        const int step = (span + 31) >> 5;
        const int q = lo + l32 * step;
        bool ge = true;
        if (span > 0 && q < hi) ge = rec_mu(c[q]) >= v;
        const uint32_t mh = (uint32_t)(__ballot(ge) >> (half * 32));
        if (span > 0) {
            if (mh == 0u) {
                lo += 31 * step + 1;
            } else {
                const int i = __builtin_ctz(mh);
                if (i == 0) {
                    hi = lo;
                } else {
                    hi = min(lo + i * step, hi);
                    lo += (i - 1) * step + 1;
                }
            }
        }
    }
    k0 = __builtin_amdgcn_readlane(lo, 0);
    k1 = __builtin_amdgcn_readlane(lo, 32);
}

// grid (the labels' 64-bin blocks, flat): 64 consecutive bins per
// workgroup, 16 per wave; a wave's union window of clipped components
// (wave_window over its 16 bins) in batches of 64 records, loaded coalesced
// into the wave's LDS slot as (mu', c') pairs and read back by lane groups
// of 16 at 4 addresses a step (LDS broadcasts: one ds_read_b128 per
// component instead of four v_readlane VALU operations and their SGPR
// hazards -- round 3 measured the kernel at 0.33 VALU busy); each lane adds
// every 4th component within its own bin's window, branch-free, to its
// A_0..A_14, and the 4 groups' sums meet by shuffles at the end (round 6;
// one bin per lane over the 64 bins' union window, 4 waves splitting it,
// before).  The bound (module comment) per lane: with |d| <= D for every
// summed component, e^y <= e^Y (Y = 2 kappa D rmax), so the per-component
// terms of the bound are accumulated as four sums and combined at the end
// (each term at least what the per-component form gives).
//
// Split window (grid z = nsplit > 1, for occupancy): workgroup z sums the
// z-th 64-aligned part of each wave's window and stores its sums in part
// (split-major, [z][sum][row]); k_bx_table_fin adds the parts in z order
// and writes the rows.  The bound counts the nsplit - 1 extra additions.
constexpr int kTabSums = kBxP + 3;   // A_0..A_14, S0, S1, S3
constexpr int kPartSums = kTabSums + 1;   // + the window size W
constexpr int kBxChains = 4;   // components per step of k_bx_table (independent chains)
constexpr int kBxMaxSplit = 8;

__device__ __forceinline__ double bin_reach(const BxLabel& B, double x) {
    return B.dwin * (1.0 + 1e-9) + (fabs(x) + B.dwin) * 1e-12;
}

// a bin's row: A_0..A_14 and Eabs from its sums (module comment)
__device__ __forceinline__ void table_row(const BxLabel& B, int b, const double* A, double S0, double S1,
                                          double S3, double W, int nsplit, double* __restrict__ tab) {
    const double r = B.rmax, kap = B.kappa;
    const double xb = B.xlo + ((double)b + 0.5) * B.bw, D = bin_reach(B, xb);
    // every summed component has |d| <= D: |mu'| <= |xb| + D, and at most
    // the window's W of them were summed
    const double S2 = (fabs(xb) + D) * S0 * (1.0 + 1e-15);   // >= sum g |mu'|
    // e^y <= 1 + y + y^2 for 0 <= y <= 1.79, else exp(y) (1 + 1e-6)
    const double Y = 2.0 * kap * D * r, eY = Y <= 1.5 ? fma(Y, Y, 1.0 + Y) : exp(Y) * 1.000001;
    const double G = eY * S0;                                  // sum_k g e^y
    const double Rb = eY * B.rP * kInvFact[kBxP] * S3;         // truncation (Lagrange)
    const double ERR = eY * (((3.0 * kBxP + 10.0) * kU + 2.6e-14) * S0 + 4.0 * kU * S1 +
                             2.0 * kap * (D + r) * (S2 + (D + r) * S0) * 0x1.0p-51);
    double* row = tab + (size_t)(B.tab_off + b) * kBxRow;
#pragma unroll
    for (int n = 0; n < kBxP; ++n) row[n] = A[n];
    // the sums: each lane group's sequential sum, then 2 additions (of <= W
    // terms; 6 counted, from the 4-wave form),
    // then nsplit - 1 more (split window)
    row[kBxP] = 1.02 * (Rb + ERR + (W + 6.0 + (double)(nsplit - 1) + 2.0 * kBxP + 8.0) * kU * G) + 1e-300;
}

__global__ __launch_bounds__(kBlock) void k_bx_table(const DLabel* __restrict__ labels,
                                                     const int32_t* __restrict__ grp,
                                                     const Comp<double>* __restrict__ comps64,
                                                     const BxLabel* __restrict__ bx,
                                                     double* __restrict__ tab, int nsplit,
                                                     double* __restrict__ part, int64_t rows,
                                                     const int2* __restrict__ blocks) {
    // (the grid numbers the labels' 64-bin blocks flat: a grid of the
    // largest label's blocks per label left most of the others' empty)
    const int2 blk = blocks[blockIdx.x];   // (dense label position, first bin)
    const int li = grp[blk.x];
    const BxLabel B = bx[li];
    const int b0 = blk.y;             // the workgroup's first bin (nbins: a multiple of 64)
    const DLabel L = labels[li];
    __shared__ double lds[kExpTabSize];   // the exp table
    __shared__ double2 stage[kBlock / 64][64];   // per wave: its batch's (mu', c')
    load_exp_table(lds);
    // wave w: the 16 bins b0 + 16 w .. + 15; lane = (component group g,
    // bin bl): each lane sums every 4th component of its wave's window for
    // its bin, the 4 groups added at the end (round 6: the 64 bins' union
    // window over all 64 lanes evaluated ~1.36x the (bin, component) pairs
    // that can reach a bin at T = 64; 16 bins' union ~1.09x)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int bl = lane & 15, g = lane >> 4;
    const int bw0 = b0 + 16 * wave, b = bw0 + bl;
    const double kap = B.kappa;
    auto centre = [&](int i) { return B.xlo + ((double)i + 0.5) * B.bw; };
    auto reach = [&](double x) { return bin_reach(B, x); };
    const double xb = centre(b), D = reach(xb);
    // (the wave's window: records sorted by mu, so the clipped ones within D
    // of any of its bins are a contiguous index range; margins cover mu' =
    // m'/a' rounding)
    const double xf = centre(bw0), xl = centre(bw0 + 15);
    int k0, k1;
    wave_window(comps64 + L.comp_a, L.na, xf - reach(xf), xl + reach(xl), k0, k1);
    const Comp<double>* c = comps64 + L.comp_a;
    double A[kBxP];
#pragma unroll
    for (int n = 0; n < kBxP; ++n) A[n] = 0.0;
    double S0 = 0.0, S1 = 0.0, S3 = 0.0;   // sum g, g |arg|, |g (2 kappa d)^P|
    // mu' = m' (1 / a*): <= 1.5 ulp (inside the 2^-51 allowance below);
    // g = exp(arg) through the fp64 round's table exp (<= 2.6e-14 relative,
    // added to the rounding term); the powers g (2 kappa d)^n by one
    // multiply each, A_n += that / n! (one rounding each, inside 3P + 10)
    const double inv_a = 1.0 / B.astar;
    // this workgroup's part of the wave's window: [ks, ke)
    const int chunk = ((k1 - k0 + nsplit - 1) / nsplit + 63) & ~63;
    const int ks = min(k1, k0 + (int)blockIdx.z * chunk), ke = min(k1, ks + chunk);
    for (int kc = ks; kc < ke; kc += 64) {
        const int k = kc + lane;
        double mu_l = 0.0, c_l = -kInf;
        if (k < ke) {
            const Comp<double> rec = c[k];
            if (rec.a == B.astar) {
                mu_l = rec.mu * inv_a;
                c_l = rec.c * kExpScaleInv;
            }
        }
        const int cnt = min(64, ke - kc);
        __builtin_amdgcn_wave_barrier();   // (the previous batch's reads come first: LDS is in order per wave)
        stage[wave][lane] = double2{mu_l, c_l};
        __builtin_amdgcn_wave_barrier();
        // kBxChains components per lane per step (independent exp and power
        // chains): lane group g takes components j + g + 4 q
        for (int j = 0; j < cnt; j += 4 * kBxChains) {
            double cj[kBxChains], dj[kBxChains], aj[kBxChains], mj[kBxChains];
            bool any = false;
#pragma unroll
            for (int q = 0; q < kBxChains; ++q) {
                const int jj = j + g + 4 * q;
                const double2 v = stage[wave][min(jj, 63)];   // (4 addresses per wave: LDS broadcasts)
                cj[q] = jj < cnt ? v.y : -kInf;
                mj[q] = v.x;
                any = any || cj[q] > -kInf;
            }
            if (!__ballot(any)) continue;   // unclipped or weightless (wave-uniform)
            double t[kBxChains], y[kBxChains];
#pragma unroll
            for (int q = 0; q < kBxChains; ++q) {
                dj[q] = mj[q] - xb;
                aj[q] = fmax(cj[q] - kap * dj[q] * dj[q], -745.0);
                // outside the bin's window, or below 2^-1067 in the whole bin
                // (in the skip term): g = 0, so every sum below is unchanged
                const bool in = fabs(dj[q]) <= D && aj[q] > -740.0;
                const double e = exp_scaled(fmin(aj[q] * kExpScale, 0.0), lds);
                t[q] = in ? e : 0.0;
                y[q] = 2.0 * kap * dj[q];
            }
#pragma unroll
            for (int q = 0; q < kBxChains; ++q) {
                S0 += t[q];
                S1 = fma(t[q], fabs(aj[q]), S1);
                A[0] += t[q];
            }
#pragma unroll
            for (int n = 1; n < kBxP; ++n)
#pragma unroll
                for (int q = 0; q < kBxChains; ++q) {
                    t[q] *= y[q];
                    A[n] = fma(t[q], kInvFact[n], A[n]);
                }
#pragma unroll
            for (int q = 0; q < kBxChains; ++q) S3 += fabs(t[q] * y[q]);
        }
    }
    // the 4 groups' sums per bin: (g0 + g2) + (g1 + g3) into lanes 0..15
    auto fold = [&](double v) {
        v += __shfl_down(v, 32);
        v += __shfl_down(v, 16);
        return v;
    };
#pragma unroll
    for (int n = 0; n < kBxP; ++n) A[n] = fold(A[n]);
    S0 = fold(S0);
    S1 = fold(S1);
    S3 = fold(S3);
    if (g != 0) return;
    if (nsplit > 1) {   // (coalesced over the bins: [z][sum][row])
        double* q = part + (size_t)blockIdx.z * kPartSums * rows + B.tab_off + b;
#pragma unroll
        for (int n = 0; n < kBxP; ++n) q[(size_t)n * rows] = A[n];
        q[(size_t)(kBxP + 0) * rows] = S0;
        q[(size_t)(kBxP + 1) * rows] = S1;
        q[(size_t)(kBxP + 2) * rows] = S3;
        q[(size_t)(kBxP + 3) * rows] = (double)(k1 - k0);
        return;
    }
    table_row(B, b, A, S0, S1, S3, (double)(k1 - k0), 1, tab);
}

// grid (ceil(max bins / 256), dense labels): a split window's parts added in
// z order, the rows written
__global__ __launch_bounds__(kBlock) void k_bx_table_fin(const int32_t* __restrict__ grp,
                                                         const BxLabel* __restrict__ bx,
                                                         double* __restrict__ tab, int nsplit,
                                                         const double* __restrict__ part, int64_t rows) {
    const BxLabel B = bx[grp[blockIdx.y]];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B.nbins) return;
    double A[kBxP], S[3];
    const double* q = part + B.tab_off + b;
#pragma unroll
    for (int n = 0; n < kBxP; ++n) A[n] = q[(size_t)n * rows];
#pragma unroll
    for (int n = 0; n < 3; ++n) S[n] = q[(size_t)(kBxP + n) * rows];
    const double W = q[(size_t)(kBxP + 3) * rows];
    for (int z = 1; z < nsplit; ++z) {
        const double* qz = q + (size_t)z * kPartSums * rows;
#pragma unroll
        for (int n = 0; n < kBxP; ++n) A[n] += qz[(size_t)n * rows];
#pragma unroll
        for (int n = 0; n < 3; ++n) S[n] += qz[(size_t)(kBxP + n) * rows];
    }
    table_row(B, b, A, S[0], S[1], S[2], W, nsplit, tab);
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

// A below component, folded once per workgroup for gauss_bounds' arithmetic
// (the same expressions, evaluated once instead of per sub-bin): c = c'/K,
// kap = a'^2 / K, mu = m'/a', and eps = ec + es (|e0| + |e1| + |mu|) with
// ec = 1e-15 (64 + |c|) + 3e-14, es = 64e-15 sqrt(kap)
struct BelowTerm {
    double c, kap, mu, ec, es;
};
constexpr int kStageBelow = 64;   // below components staged in LDS (more: read per sub-bin)
constexpr int64_t kBoundsWgs = (int64_t)1 << 30;   // k_bx_bounds' workgroups over the labels, at most
// (4096 -- each workgroup striding over several blocks -- measured 127 -> 144 us at config 3, r6x)

__device__ __forceinline__ void term_bounds(const BelowTerm& t, double e0, double e1, double& lo, double& hi,
                                            const double* __restrict__ etab) {
    const double dn = t.mu < e0 ? e0 - t.mu : (t.mu > e1 ? t.mu - e1 : 0.0);
    const double df = fmax(fabs(e0 - t.mu), fabs(e1 - t.mu));
    const double eps = fma(t.es, fabs(e0) + fabs(e1) + fabs(t.mu), t.ec);
    hi += exp_scaled((t.c - t.kap * dn * dn + eps) * kExpScale, etab);
    const double ul = (t.c - t.kap * df * df - eps) * kExpScale;
    lo += ul > -4.0e6 ? exp_scaled(ul, etab) : 0.0;   // (below ~2^-980: 0 is a lower bound)
}

// grid (ceil(max above records / 256), dense labels): each above record's
// bound terms (BxTerm), the per-record part of gauss_bounds evaluated once
// instead of per sub-bin of every bin whose list holds the record
__global__ __launch_bounds__(kBlock) void k_bx_terms(const DLabel* __restrict__ labels,
                                                     const int32_t* __restrict__ grp,
                                                     const Comp<double>* __restrict__ comps64,
                                                     BxTerm* __restrict__ terms) {
    const DLabel L = labels[grp[blockIdx.y]];
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= L.na) return;
    const Comp<double> r = comps64[L.comp_a + k];
    BxTerm t{-kInf, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (usable(r)) {
        t.c = r.c * kExpScaleInv;
        t.kap = r.a * r.a * kExpScaleInv;
        t.mu = r.mu / r.a;
        t.ec = 1e-15 * (64.0 + fabs(t.c)) + 3e-14;
        t.es = 1e-15 * 64.0 * sqrt(t.kap);
    } else if (r.c > -kInf) {
        t.ec = -1.0;   // a weighted unusable record: no bound anywhere
    }
    terms[L.comp_a + k] = t;
}

// grid (blocks of 256 sub-bins strided, dense labels): one sub-bin per thread --
// the hot-bin prefilter's [L, U] of the fp64 score over the sub-bin (float,
// rounded outward) and the sampling mass p of the sub-bin (tpe_device.h,
// "hot-bin prefilter").  Below mixture: every component bounded term by
// term.  Above mixture: the bin's polynomial Taylor-shifted to the sub-bin
// centre (|A(dc + t) - A_0'| <= sum_n>0 |A_n'| h^n), +- its Eabs, times the
// range of exp(-kappa delta^2); the bin's list term by term; the skipped
// components' na 2^-T on the upper side.  U, L: log ratio of the bounds plus
// the shift difference, widened by 1e-7 (1 + |v|) and the fp64 round's own
// error; +inf / -inf where a sum is not safely inside the normal range or a
// record is unusable.  The mass only steers tau0, never a bound: the
// below mixture's density at the sub-bin's midpoint times its width (fp32;
// a sub-bin is < 1/100 of the narrowest sampling sigma, so the midpoint
// rule is within ~1e-5 relative).
__global__ __launch_bounds__(kBlock) void k_bx_bounds(const DLabel* __restrict__ labels,
                                                      const int32_t* __restrict__ grp,
                                                      const Comp<double>* __restrict__ comps64,
                                                      const SampRec* __restrict__ samp,
                                                      const BxLabel* __restrict__ bx,
                                                      const double* __restrict__ tab,
                                                      const int32_t* __restrict__ cnt,
                                                      const int32_t* __restrict__ list,
                                                      const BxTerm* __restrict__ terms,
                                                      float2* __restrict__ sb, float* __restrict__ sbp) {
    const int li = grp[blockIdx.y];
    const BxLabel B = bx[li];
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    if ((int64_t)blockIdx.x * kBlock >= nsb) return;   // the whole workgroup
    const DLabel L = labels[li];
    __shared__ double etab[kExpTabSize];
    __shared__ BelowTerm bt[kStageBelow];
    __shared__ float4 sm[kStageBelow];   // sampling: mu, 1 / sigma, w / (sigma sqrt(2 pi)), -
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    for (int i = threadIdx.x; i < kExpTabSize; i += kBlock) etab[i] = kExp2Tab[i];
    __syncthreads();
    const bool staged_b = L.nb <= kStageBelow, staged_s = L.ns <= kStageBelow;
    if (staged_b && threadIdx.x < L.nb) {
        const Comp<double> r = comps64[L.comp_b + threadIdx.x];
        BelowTerm t{-kInf, 0.0, 0.0, 0.0, 0.0};
        if (usable(r)) {
            t.c = r.c * kExpScaleInv;
            t.kap = r.a * r.a * kExpScaleInv;
            t.mu = r.mu / r.a;
            t.ec = 1e-15 * (64.0 + fabs(t.c)) + 3e-14;
            t.es = 1e-15 * 64.0 * sqrt(t.kap);
        } else if (r.c > -kInf) {
            atomicOr(&bad, 1);   // a weighted unusable record: no bound anywhere
        }
        bt[threadIdx.x] = t;
    }
    if (staged_s && threadIdx.x < L.ns) {
        const SampRec s = samp[L.samp_off + threadIdx.x];
        const double w = s.wd;   // (the truncated mixture's density weight, k_samp_fold)
        const bool ok = w > 0.0 && s.sigma > 0.0 && s.sigma < kInf;
        sm[threadIdx.x] = ok ? make_float4((float)(s.mu - L.centre), (float)(1.0 / s.sigma),
                                           (float)(w / (s.sigma * 2.5066282746310002)), 0.0f)
                             : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    __syncthreads();
    // (blocks of the label strided over the grid when it is capped)
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < nsb; j += (int64_t)gridDim.x * kBlock) {
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
        double a0 = e0n, a1 = e1n;   // recentred draw space
        if ((L.flags & 3) == 3) {
            a0 = fmax(a0, L.low - L.centre);
            a1 = fmin(a1, L.high - L.centre);
        }
        if (a1 > a0) {
            const float xm = (float)(0.5 * (a0 + a1));
            float dens = 0.0f;
            if (staged_s) {
                for (int k = 0; k < L.ns; ++k) {
                    const float4 q = sm[k];
                    const float z = (xm - q.x) * q.y;
                    dens = fmaf(q.z, __expf(-0.5f * z * z), dens);
                }
            } else {
                for (int k = 0; k < L.ns; ++k) {
                    const SampRec s = samp[L.samp_off + k];
                    const double w = s.wd;
                    if (!(w > 0.0 && s.sigma > 0.0 && s.sigma < kInf)) continue;
                    const float z = (float)((xm - (s.mu - L.centre)) / s.sigma);
                    dens += (float)(w / (s.sigma * 2.5066282746310002)) * __expf(-0.5f * z * z);
                }
            }
            p = (double)dens * (a1 - a0);
        }
    }
    bool ok = bad == 0;
    double blo = 0.0, bhi = 0.0;
    if (staged_b) {
        for (int k = 0; k < L.nb; ++k) {
            const BelowTerm t = bt[k];
            if (t.c > -kInf) term_bounds(t, e0, e1, blo, bhi, etab);
        }
    } else {
        for (int k = 0; k < L.nb; ++k) {
            const Comp<double> r = comps64[L.comp_b + k];
            if (!usable(r)) {
                ok = ok && !(r.c > -kInf);
                continue;
            }
            gauss_bounds(r, e0, e1, blo, bhi, etab);
        }
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
    const BxTerm* ta = terms + L.comp_a;
    const int32_t* lst = list + B.list_off + (int64_t)b * B.n_nc;
    const int m = cnt[B.cnt_off + b];
    for (int jj = 0; jj < m; ++jj) {
        const BxTerm q = ta[lst[jj]];
        if (q.ec < 0.0) ok = false;
        else if (q.c > -kInf) term_bounds(BelowTerm{q.c, q.kap, q.mu, q.ec, q.es}, e0, e1, slo, shi, etab);
    }
    shi += (double)L.na * exp2(-B.tcut);
    const double dsh = L.shift_b - L.shift_a;
    const double mag = fabs(L.shift_b) + fabs(L.shift_a) + 2.0 * (fabs(L.centre) + fabs(e0) + fabs(e1)) + 64.0;
    const double fe = (double)(L.nb + L.na + 64) * 0x1.0p-50 + mag * 0x1.0p-48;
    double U = kInf, Lo = -kInf;
    // (flog: <= 1 ulp, far inside the 1e-7 widening)
    if (ok && bhi >= 1e-280 && slo >= 1e-280) {
        const double v = flog(bhi) - flog(slo) + dsh;
        if (v == v) U = v + 1e-7 * (1.0 + fabs(v)) + fe;
    }
    if (ok && blo >= 1e-280 && shi > 0.0 && shi < kInf) {
        const double v = flog(blo) - flog(shi) + dsh;
        if (v == v) Lo = v - 1e-7 * (1.0 + fabs(v)) - fe;
    }
    if (!(U == U) || !(Lo == Lo) || U < Lo) {
        U = kInf;
        Lo = -kInf;
    }
    sb[B.sb_off + j] = make_float2(float_up(U), float_down(Lo));
    sbp[B.sb_off + j] = (float)p;
    }
}

// grid (dense labels of the snapshot): any byte of a dense label's DLabel,
// records or sampling records that differs from the snapshot -> *diff = 1
__global__ __launch_bounds__(kBlock) void k_bx_compare(const int32_t* __restrict__ grp,
                                                       const DLabel* __restrict__ lab, const DLabel* __restrict__ lab0,
                                                       const Comp<double>* __restrict__ c,
                                                       const Comp<double>* __restrict__ c0,
                                                       const SampRec* __restrict__ sr, const SampRec* __restrict__ sr0,
                                                       int64_t c_cap, int64_t s_cap, int32_t* __restrict__ diff) {
    const int li = grp[blockIdx.x];
    const uint32_t* a = reinterpret_cast<const uint32_t*>(lab + li);
    const uint32_t* b = reinterpret_cast<const uint32_t*>(lab0 + li);
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    if (threadIdx.x < sizeof(DLabel) / 4 && a[threadIdx.x] != b[threadIdx.x]) bad = 1;
    __syncthreads();
    if (bad) {
        if (threadIdx.x == 0) atomicOr(diff, 1);
        return;
    }
    const DLabel L = lab[li];
    if (L.comp_b + L.nb > c_cap || L.comp_a + L.na > c_cap || L.samp_off + L.ns > s_cap) {
        if (threadIdx.x == 0) atomicOr(diff, 1);
        return;
    }
    bool d = false;
    auto same = [](const Comp<double>& x, const Comp<double>& y) {
        return __double_as_longlong(x.mu) == __double_as_longlong(y.mu) &&
               __double_as_longlong(x.a) == __double_as_longlong(y.a) &&
               __double_as_longlong(x.c) == __double_as_longlong(y.c) &&
               __double_as_longlong(x.w) == __double_as_longlong(y.w);
    };
    for (int k = threadIdx.x; k < L.nb; k += kBlock) d |= !same(c[L.comp_b + k], c0[L.comp_b + k]);
    for (int k = threadIdx.x; k < L.na; k += kBlock) d |= !same(c[L.comp_a + k], c0[L.comp_a + k]);
    for (int k = threadIdx.x; k < L.ns; k += kBlock) {
        const SampRec x = sr[L.samp_off + k], y = sr0[L.samp_off + k];
        d |= __double_as_longlong(x.cdf) != __double_as_longlong(y.cdf) ||
             __double_as_longlong(x.mu) != __double_as_longlong(y.mu) ||
             __double_as_longlong(x.sigma) != __double_as_longlong(y.sigma);
    }
    if (d) atomicOr(diff, 1);
}

}  // namespace

int tpe_rt::bx_keep_check(tpe_ctx* ctx) {
    tpe_rt::Posterior& P = *ctx->P;
    ctx->pin[0].bx_diff = 1;
    if (!P.bx_ready || P.bx_snap_nl <= 0) return TPE_OK;
    HIPCHK(ctx, P.bx_diff.reserve(1));
    HIPCHK(ctx, hipMemsetAsync(P.bx_diff.p, 0, sizeof(int32_t), ctx->stream));
    hipLaunchKernelGGL(k_bx_compare, dim3(P.bx_snap_nl), dim3(kBlock), 0, ctx->stream, P.bx_snap_g.p, P.labels.p,
                       P.bx_snap_l.p, P.comps64.p, P.bx_snap_c.p, P.samp.p, P.bx_snap_s.p,
                       (int64_t)std::min(P.comps64.cap, P.bx_snap_c.cap),
                       (int64_t)std::min(P.samp.cap, P.bx_snap_s.cap), P.bx_diff.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(&ctx->pin[0].bx_diff, P.bx_diff.p, sizeof(int32_t), hipMemcpyDeviceToHost,
                               ctx->stream));
    return TPE_OK;
}

bool tpe_rt::bx_keep_after(tpe_ctx* ctx, bool groups_changed) {
    tpe_rt::Posterior& P = *ctx->P;
    return P.bx_ready && P.bx_snap_nl > 0 && !groups_changed && ctx->pin[0].bx_diff == 0;
}

int tpe_rt::bx_prescan(tpe_ctx* ctx, hipStream_t st, bool* queued) {
    tpe_rt::Posterior& P = *ctx->P;
    *queued = false;
    const int nl = (int)(P.h_group[DENSE_GMM].size() + P.h_group[DENSE_LGMM].size());
    if (nl == 0 || !P.groups.p) return TPE_OK;
    HIPCHK(ctx, P.bx_scan.reserve((size_t)nl * kScanFields));
    HIPCHK(ctx, P.bx_scan_h.resize((size_t)nl * kScanFields));
    hipLaunchKernelGGL(k_bx_scan, dim3(nl), dim3(kBlock), 0, st, P.labels.p, P.groups.p + P.group_off[DENSE_GMM],
                       P.comps64.p, P.samp.p, P.bx_scan.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(P.bx_scan_h.data(), P.bx_scan.p, (size_t)nl * kScanFields * sizeof(double),
                               hipMemcpyDeviceToHost, st));
    *queued = true;
    return TPE_OK;
}

// unique over every posterior of the process (an index built here or
// imported, tpe_share.hip): the hot-bin caches are keyed by it
uint64_t tpe_rt::next_bx_gen() {
    static uint64_t gen_counter = 0;
    return __atomic_add_fetch(&gen_counter, 1, __ATOMIC_RELAXED);
}

// The index is queued on the context's stream without waiting for it (one
// short round trip for the layout): a caller can overlap it with host work
// (tpe_prepare).  Its device time is bracketed by events and read when asked.
int tpe_rt::bx_prepare(tpe_ctx* ctx) {
    tpe_rt::Posterior& P = *ctx->P;
    if (P.bx_ready) return TPE_OK;
    const bool timed = ctx->timing && ctx->ev_prep[0];
    if (timed) HIPCHK(ctx, hipEventRecord(ctx->ev_prep[0], ctx->stream));
    const int rc = bx_build(ctx);
    if (rc == TPE_OK && timed) {
        HIPCHK(ctx, hipEventRecord(ctx->ev_prep[1], ctx->stream));
        ctx->prep_pending = true;
    }
    return rc;
}

// the tables, lists and sub-bin bounds of every dense label (bx_prepare):
// one host round trip (the per-label scan decides the bins and the layout)
int tpe_rt::bx_build(tpe_ctx* ctx) {
    tpe_rt::Posterior& P = *ctx->P;
    P.bx_ok = false;
    const std::vector<int32_t>& gg = P.h_group[DENSE_GMM];
    const std::vector<int32_t>& gl = P.h_group[DENSE_LGMM];
    const int nl = (int)(gg.size() + gl.size());
    P.bx_snap_nl = 0;
    if (nl == 0) {
        P.bx_ready = true;
        return TPE_OK;
    }
    const int32_t* grp = P.groups.p + P.group_off[DENSE_GMM];
    std::vector<double> sc((size_t)nl * kScanFields);
    if (P.bx_prescan_ok && P.bx_scan_h.n == sc.size()) {
        // (the build queued the scan and its read-back before its own sync)
        std::memcpy(sc.data(), P.bx_scan_h.data(), sc.size() * sizeof(double));
    } else {
        HIPCHK(ctx, P.bx_scan.reserve((size_t)nl * kScanFields));
        hipLaunchKernelGGL(k_bx_scan, dim3(nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p,
                           P.samp.p, P.bx_scan.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(sc.data(), P.bx_scan.p, sc.size() * sizeof(double), hipMemcpyDeviceToHost,
                                   ctx->stream));
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    }
    P.bx_prescan_ok = false;
    // bins per label: the fewest (a multiple of 64) whose half-width keeps
    // the Taylor argument 2 kappa |d| r <= ~0.5 over the window
    P.bx_h.assign(P.n_labels, BxLabel{});
    // the window's cut: forced (TPE_OPT_BX_T), else what the coming rounds
    // need (tile rounds through the hot-bin prefilter: kBxTTile)
    const double T = ctx->bx_t_force > 0 ? (double)ctx->bx_t_force : ctx->bx_t_next;
    bool ok = true;
    int64_t rows = 0, lsum = 0;
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
        const double d0 = std::sqrt(T * kLn2 / kap);
        const double r_target = 0.25 / (kap * d0);   // Taylor argument 2 kappa |d| r <= ~0.5
        const double want = (xhi - xlo) / (2.0 * r_target);
        if (!(want <= (double)kMaxBins)) {
            ok = false;
            break;
        }
        const int32_t nb = std::max<int32_t>(kMinBins, ((int32_t)std::ceil(want) + 63) / 64 * 64);
        if ((int64_t)nb * n_nc > ((int64_t)1 << 27)) {   // list build cost
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
        B.tcut = T;
        B.sb_off = rows * kBxSub;   // (nb a multiple of 64: a multiple of 32, as k_hot_bx needs)
        B.tab_off = rows;
        B.cnt_off = rows;           // one list count per bin
        B.list_off = lsum;          // nb slots of n_nc entries
        rows += nb;
        lsum += (int64_t)nb * n_nc;
        bins_max = std::max(bins_max, nb);
        P.bx_h[li] = B;
    }
    if (ok && lsum > ((int64_t)1 << 28)) ok = false;   // > 1 GB of list slots
    if (!ok) {
        P.bx_ready = true;   // not eligible: the windowed screen runs
        return TPE_OK;
    }
    HIPCHK(ctx, P.bx.reserve(P.n_labels));
    HIPCHK(ctx, P.bx_tab.reserve((size_t)rows * kBxRow));
    HIPCHK(ctx, P.bx_loff.reserve((size_t)rows));
    HIPCHK(ctx, P.bx_list.reserve((size_t)std::max<int64_t>(lsum, 1)));
    HIPCHK(ctx, P.bx_nc.reserve(P.comps64.cap));
    HIPCHK(ctx, P.bx_sb.reserve((size_t)rows * kBxSub));
    HIPCHK(ctx, P.bx_sbp.reserve((size_t)rows * kBxSub));
    // (through a pinned copy: from pageable memory the copy was staged
    // synchronously, ~15 us of the host between the build and the index)
    HIPCHK(ctx, P.bx_up_h.resize(P.n_labels));
    std::memcpy(P.bx_up_h.data(), P.bx_h.data(), P.n_labels * sizeof(BxLabel));
    HIPCHK(ctx, hipMemcpyAsync(P.bx.p, P.bx_up_h.data(), P.n_labels * sizeof(BxLabel), hipMemcpyHostToDevice,
                               ctx->stream));
    hipLaunchKernelGGL(k_bx_compact, dim3(nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p,
                       P.bx.p, P.bx_nc.p);
    const dim3 gb((unsigned)((bins_max + kBlock - 1) / kBlock), nl);
    hipLaunchKernelGGL(k_bx_list, gb, dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p, P.bx.p,
                       P.bx_nc.p, P.bx_loff.p, P.bx_list.p);
    // the window split: ~8192 workgroups (4 per CU at a time, LDS-bound; the
    // heavy dense-region blocks split too, so the tail shortens -- config 3's
    // ~2000 blocks: split 1 / 2 / 4 / 8 -> 0.538 / 0.492 / 0.469 / 0.503 ms in
    // one process, r5be); past 4096 blocks in 3 parts -- config 5's ~6000:
    // 1 / 2 / 3 / 4 -> 3.36 / 3.13 / 3.03 / 3.05 ms, r5bf (unsplit until the
    // quantized labels' rebuild beside it stopped holding the host, r5z)
    const int64_t wgs = (rows + 63) / 64;
    // (round 6, 16 bins per wave: config 3 split 1 / 2 / 4 / 8 -> 0.364 /
    // 0.361 / 0.354 / 0.382 ms index, config 5 1 / 2 / 3 / 4 / 6 -> 2.97 /
    // 2.73 / 2.68 / 2.67 / 2.75 ms, r6ag: at most 4 parts)
    const int nsplit = ctx->bx_split > 0 ? std::min(ctx->bx_split, kBxMaxSplit)
                       : wgs >= 4096     ? 3
                                         : (int)std::max<int64_t>(1, std::min<int64_t>(4, 8192 / std::max<int64_t>(wgs, 1)));
    if (nsplit > 1) HIPCHK(ctx, P.bx_part.reserve((size_t)nsplit * kPartSums * rows));
    {   // the labels' 64-bin blocks, numbered flat (the previous index's
        // copy out of the pinned buffer is done: bx_build's scan read-back
        // or the build's report synchronised the stream since)
        HIPCHK(ctx, P.bx_blocks_h.resize((size_t)((rows + 63) / 64)));
        int64_t n = 0;
        for (int y = 0; y < nl; ++y) {
            const int li = y < (int)gg.size() ? gg[y] : gl[y - gg.size()];
            for (int b0 = 0; b0 < P.bx_h[li].nbins; b0 += 64) P.bx_blocks_h.data()[n++] = make_int2(y, b0);
        }
        P.bx_blocks_h.n = (size_t)n;
        HIPCHK(ctx, P.bx_blocks.reserve((size_t)n));
        HIPCHK(ctx, hipMemcpyAsync(P.bx_blocks.p, P.bx_blocks_h.data(), (size_t)n * sizeof(int2),
                                   hipMemcpyHostToDevice, ctx->stream));
    }
    hipLaunchKernelGGL(k_bx_table, dim3((unsigned)P.bx_blocks_h.n, 1, nsplit), dim3(kBlock), 0,
                       ctx->stream, P.labels.p, grp, P.comps64.p, P.bx.p, P.bx_tab.p, nsplit, P.bx_part.p, rows,
                       P.bx_blocks.p);
    if (nsplit > 1)
        hipLaunchKernelGGL(k_bx_table_fin, dim3((unsigned)((bins_max + kBlock - 1) / kBlock), nl), dim3(kBlock), 0,
                           ctx->stream, grp, P.bx.p, P.bx_tab.p, nsplit, P.bx_part.p, rows);
    P.bx_sb_max = (int64_t)bins_max * kBxSub;
    P.bx_gen = tpe_rt::next_bx_gen();
    int32_t na_max = 1;
    for (int y = 0; y < nl; ++y)
        na_max = std::max(na_max, P.h_labels[y < (int)gg.size() ? gg[y] : gl[y - gg.size()]].na);
    HIPCHK(ctx, P.bx_terms.reserve(P.comps64.cap));
    hipLaunchKernelGGL(k_bx_terms, dim3((unsigned)((na_max + kBlock - 1) / kBlock), nl), dim3(kBlock), 0,
                       ctx->stream, P.labels.p, grp, P.comps64.p, P.bx_terms.p);
    const dim3 gs((unsigned)std::min<int64_t>((P.bx_sb_max + kBlock - 1) / kBlock,
                                              std::max<int64_t>(1, kBoundsWgs / nl)), nl);
    hipLaunchKernelGGL(k_bx_bounds, gs, dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.comps64.p, P.samp.p,
                       P.bx.p, P.bx_tab.p, P.bx_loff.p, P.bx_list.p, P.bx_terms.p, P.bx_sb.p, P.bx_sbp.p);
    HIPCHK(ctx, hipGetLastError());
    // the snapshot a later rebuild is compared with (bx_keep_check)
    int64_t c_ext = 0, s_ext = 0;
    for (int y = 0; y < nl; ++y) {
        const DLabel& d = P.h_labels[y < (int)gg.size() ? gg[y] : gl[y - gg.size()]];
        c_ext = std::max<int64_t>({c_ext, (int64_t)d.comp_b + d.nb, (int64_t)d.comp_a + d.na});
        s_ext = std::max<int64_t>(s_ext, (int64_t)d.samp_off + d.ns);
    }
    HIPCHK(ctx, P.bx_snap_l.reserve(P.n_labels));
    HIPCHK(ctx, P.bx_snap_c.reserve(std::max<int64_t>(c_ext, 1)));
    HIPCHK(ctx, P.bx_snap_s.reserve(std::max<int64_t>(s_ext, 1)));
    HIPCHK(ctx, P.bx_snap_g.reserve(nl));
    {   // (one launch: four copies before)
        const tpe_rt::CopySpec cs[4] = {{P.bx_snap_l.p, P.labels.p, (int64_t)P.n_labels * (int64_t)sizeof(DLabel)},
                                        {P.bx_snap_c.p, P.comps64.p, c_ext * (int64_t)sizeof(Comp<double>)},
                                        {P.bx_snap_s.p, P.samp.p, s_ext * (int64_t)sizeof(SampRec)},
                                        {P.bx_snap_g.p, grp, (int64_t)nl * (int64_t)sizeof(int32_t)}};
        const int rc = tpe_rt::copy_batch(ctx, ctx->stream, cs, 4);
        if (rc) return rc;
    }
    P.bx_snap_nl = nl;
    P.bx_ok = true;
    P.bx_ready = true;
    return TPE_OK;
}
