// tpe_window.hip -- the windowed fp32 screen of large sampled rounds
// (tpe_device.h, "windowed screen").
//
// The plain screen (tpe_engine.hip k_screen) sums every candidate over every
// component of both mixtures.  But the above mixture's Parzen components are
// narrow and sorted by mu (adaptive_parzen_normal, tpe.py:404-477: sigma >=
// prior_sigma / min(100, N + 1)), so only the components near a candidate can
// move its sum.  Here:
//
//   per posterior (k_win_hist, k_win_seg, k_win_carry, k_win_bins, k_win_skip;
//   once, lazily):
//     each above component's interval [lo, hi] of recentred x' where its term
//     can reach 2^-(T + 1) (from its fp32 record; the extra 1 covers the
//     records' rounding), the prefix max of hi and the suffix min of lo over
//     the narrow components in record order, the list of wide components
//     (interval longer than 4x the label's median or half its candidate
//     range, or too far from the centre for the rounding margin), and for
//     each of kWinBins bins of the candidate range the window [k_lo, k_hi) of
//     record indices outside which no narrow component reaches 2^-T
//     anywhere in the bin;
//
//   per round (k_win_key, a stable radix sort, k_screen_win):
//     every candidate keyed by (round, label, bin of x') and sorted with its
//     (x' fp32, index) value, so a workgroup's 2048 candidates are neighbours;
//     the tile's window is [k_lo(bin of its min), k_hi(bin of its max)), the
//     below mixture and the wide components outside the window are summed in
//     full, and the bound (screen_err) grows by the skipped mass relative to
//     the sum, bounded per bin of the candidate (k_win_skip).
//
// The selection (k_select) and the fp64 re-score (k_rescore, every
// component) are the plain screen's, so winners and lpdfs are bit-identical
// to the fp64 round's; only the set of re-scored candidates can differ.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "../../include/hyperopt_tpe.h"
#include "tpe_ctx.h"
#include "tpe_device.h"

using namespace tpe;
using tpe_rt::kBlock;

namespace {

constexpr int kSegR = 8;
constexpr int kSeg = kSegR * kBlock;     // components per prep workgroup
constexpr int kKeyR = 4;                 // candidates per thread, k_win_key
constexpr int kWinR = 8;                 // candidates per thread, k_screen_win (tile 2048)
constexpr double kInf = __builtin_inf();
constexpr int kCoarseBits = 8;                    // per-cell sort key: bin >> 3
constexpr int64_t kCellSortMin = (int64_t)1 << 20;

// ---------------------------------------------------------- block helpers ----
struct MaxOp {
    __device__ double operator()(double a, double b) const { return a > b ? a : b; }
};
struct MinOp {
    __device__ double operator()(double a, double b) const { return a < b ? a : b; }
};
struct AddOp {
    __device__ int operator()(int a, int b) const { return a + b; }
};

// exclusive prefix (in thread order) of v under op, and the block total;
// sh: kBlock / 64 entries
template <typename T, typename Op>
__device__ T block_prefix(T v, T id, Op op, T* sh, T& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T o = __shfl_up(inc, off);
        if (lane >= off) inc = op(inc, o);
    }
    T excl = __shfl_up(inc, 1);
    if (lane == 0) excl = id;
    if (lane == 63) sh[wave] = inc;
    __syncthreads();
    T before = id, tot = id;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        if (w < wave) before = op(before, sh[w]);
        tot = op(tot, sh[w]);
    }
    __syncthreads();
    total = tot;
    return op(before, excl);
}

// exclusive suffix (over the threads after this one) of v under op
template <typename T, typename Op>
__device__ T block_suffix(T v, T id, Op op, T* sh) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T o = __shfl_down(inc, off);
        if (lane + off < 64) inc = op(inc, o);
    }
    T excl = __shfl_down(inc, 1);
    if (lane == 63) excl = id;
    if (lane == 0) sh[wave] = inc;
    __syncthreads();
    T after = id;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w)
        if (w > wave) after = op(after, sh[w]);
    __syncthreads();
    return op(after, excl);
}

template <typename T, typename Op>
__device__ T block_reduce(T v, Op op, T* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    T r = sh[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) r = op(r, sh[w]);
    __syncthreads();
    return r;
}

// ------------------------------------------------------------- the index ----
// The label's candidate range, recentred: [low, high) for a bounded label
// (sample_raw's acceptance interval), else the below mixture's mu +- 8 sigma
// hull.  Only the bins' placement depends on it (candidates outside fall in
// the end bins, whose windows are open-ended).
__device__ void label_range(const DLabel& L, const SampRec* __restrict__ samp, double& xlo,
                            double& xhi, double* sh) {
    double lo = kInf, hi = -kInf;
    if ((L.flags & 3) == 3) {
        lo = L.low;
        hi = L.high;
    } else {
        for (int k = threadIdx.x; k < L.ns; k += kBlock) {
            const SampRec s = samp[L.samp_off + k];
            lo = fmin(lo, s.mu - 8.0 * s.sigma);
            hi = fmax(hi, s.mu + 8.0 * s.sigma);
        }
        lo = block_reduce(lo, MinOp{}, sh);
        hi = block_reduce(hi, MaxOp{}, sh);
    }
    xlo = lo - L.centre;
    xhi = hi - L.centre;
    if (!(fabs(xlo) < 1e300)) xlo = 0.0;
    if (!(xhi > xlo) || !(fabs(xhi) < 1e300)) xhi = xlo + 1.0;
}

struct Interval {
    double lo, hi;
    bool wide;
};

// Wide components: an interval longer than kWideF times the label's median
// (a few edge or sparse-region components, whose long reach would flatten
// the prefix max / suffix min for every bin after / before them), or longer
// than half the candidate range (the prior component).  The median comes from
// a histogram of log2 widths (kWidthBins half-octave bins, k_win_hist), so
// the threshold is kWideF x the upper edge of the median's bin.
constexpr double kWideF = 4.0;
constexpr int kWidthBins = 256;          // log2 width in [-64, 64), half octaves

__device__ __forceinline__ int width_bin(double w) {
    const double b = 2.0 * (log2(w) + 64.0);
    if (!(b >= 0.0)) return 0;
    if (!(b < (double)(kWidthBins - 1))) return kWidthBins - 1;
    return (int)b;
}

// Where component r's term can reach 2^-(T + 1): |x' a - m| <= s with
// s = sqrt(c + T + 1) (log2 units, c <= 0).  Outside it, the exact term
// (from the unrounded a, m, c) stays below 2^-T as long as the records'
// rounding moves z by less than sqrt(c + T + 1) - sqrt(c + T) >= 1 / (2
// sqrt(T + 1)) ~ 0.07, i.e. (|x' a| + |m|) 2^-23 < 0.07 for every x' near the
// interval: |m| < 2^17 suffices; records beyond that are always summed.
// Never-relevant components (c < -(T + 1), also c = -inf) get an empty
// interval and no wide flag.
__device__ __forceinline__ Interval comp_interval(const Comp<float>& r, double span, double thr,
                                                 double T) {
    Interval v{kInf, -kInf, false};
    const double m = r.mu, a = r.a, cc = (double)r.c + (T + 1.0);
    if (cc < 0.0) return v;
    if (!(cc <= 1e30) || !(a > 0.0) || !(a < 1e30) || !(fabs(m) < 131072.0)) {
        v.wide = true;
        return v;
    }
    const double s = sqrt(cc) * (1.0 + 1e-9);
    double lo = (m - s) / a, hi = (m + s) / a;
    lo -= fabs(lo) * 1e-12 + 1e-300;
    hi += fabs(hi) * 1e-12 + 1e-300;
    if (hi - lo > 0.5 * span || hi - lo > thr) {
        v.wide = true;
        return v;
    }
    v.lo = lo;
    v.hi = hi;
    return v;
}

// grid (segments, dense labels): histogram of the narrow-candidate
// intervals' log2 widths (everything but never-relevant components)
__global__ __launch_bounds__(kBlock) void k_win_hist(const DLabel* __restrict__ labels,
                                                     const int32_t* __restrict__ grp,
                                                     const Comp<float>* __restrict__ comps32,
                                                     const SampRec* __restrict__ samp,
                                                     int32_t* __restrict__ hist, double T) {
    const int y = blockIdx.y, li = grp[y];
    const DLabel L = labels[li];
    __shared__ double shd[kBlock / 64];
    __shared__ int h[kWidthBins];
    double xlo, xhi;
    label_range(L, samp, xlo, xhi, shd);
    for (int b = threadIdx.x; b < kWidthBins; b += kBlock) h[b] = 0;
    __syncthreads();
    const int64_t k0 = (int64_t)blockIdx.x * kSeg;
    const Comp<float>* c = comps32 + L.comp_a;
    for (int j = 0; j < kSegR; ++j) {
        const int64_t k = k0 + j * kBlock + threadIdx.x;
        if (k >= L.na) break;
        const Interval v = comp_interval(c[k], xhi - xlo, kInf, T);
        if (v.hi >= v.lo) atomicAdd(&h[width_bin(v.hi - v.lo)], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kWidthBins; b += kBlock)
        if (h[b]) atomicAdd(&hist[(size_t)y * kWidthBins + b], h[b]);
}

// kWideF x the upper edge of the median width's bin (+inf without data)
__device__ double wide_threshold(const int32_t* __restrict__ hist_row, int* sh) {
    static_assert(kWidthBins == kBlock, "one bin per thread");
    const int v = hist_row[threadIdx.x];
    int tot;
    const int before = block_prefix(v, 0, AddOp{}, sh, tot);
    __shared__ int med;
    if (threadIdx.x == 0) med = kWidthBins;
    __syncthreads();
    // the bin holding the (tot + 1) / 2-th width
    if (tot > 0 && before < (tot + 1) / 2 && before + v >= (tot + 1) / 2) med = threadIdx.x;
    __syncthreads();
    const int m = med;
    __syncthreads();
    if (m >= kWidthBins) return kInf;
    return kWideF * exp2(0.5 * (double)(m + 1) - 64.0);
}

// grid (segments, dense labels): per kSeg components the segment-local
// prefix max of hi and suffix min of lo (wide and dropped components are
// neutral), and the segment's max hi, min lo and wide count
__global__ __launch_bounds__(kBlock) void k_win_seg(const DLabel* __restrict__ labels,
                                                    const int32_t* __restrict__ grp,
                                                    const Comp<float>* __restrict__ comps32,
                                                    const SampRec* __restrict__ samp, int32_t nseg,
                                                    const int32_t* __restrict__ hist,
                                                    WinLabel* __restrict__ win, double* __restrict__ P,
                                                    double* __restrict__ Q, double* __restrict__ seg,
                                                    double T) {
    const int y = blockIdx.y, li = grp[y];
    const DLabel L = labels[li];
    __shared__ double shd[kBlock / 64];
    __shared__ int shi[kBlock / 64];
    double xlo, xhi;
    label_range(L, samp, xlo, xhi, shd);
    const double thr = wide_threshold(hist + (size_t)y * kWidthBins, shi);
    const int s = blockIdx.x;
    if (s == 0 && threadIdx.x == 0) win[li] = WinLabel{xlo, (double)kWinBins / (xhi - xlo), 0, 0};
    double* sg = seg + ((size_t)y * nseg + s) * 3;
    const int64_t k0 = (int64_t)s * kSeg;
    if (k0 >= L.na) {
        if (threadIdx.x == 0) {
            sg[0] = -kInf;
            sg[1] = kInf;
            sg[2] = 0.0;
        }
        return;
    }
    const Comp<float>* c = comps32 + L.comp_a;
    double lo[kSegR], hi[kSegR];
    int nw = 0;
#pragma unroll
    for (int j = 0; j < kSegR; ++j) {
        const int64_t k = k0 + threadIdx.x * kSegR + j;
        Interval v{kInf, -kInf, false};
        if (k < L.na) v = comp_interval(c[k], xhi - xlo, thr, T);
        lo[j] = v.lo;
        hi[j] = v.hi;
        nw += v.wide;
    }
    double pm[kSegR], run = -kInf;
#pragma unroll
    for (int j = 0; j < kSegR; ++j) {
        run = hi[j] > run ? hi[j] : run;
        pm[j] = run;
    }
    double tot_hi;
    const double before = block_prefix(run, -kInf, MaxOp{}, shd, tot_hi);
    double sm[kSegR];
    run = kInf;
#pragma unroll
    for (int j = kSegR - 1; j >= 0; --j) {
        run = lo[j] < run ? lo[j] : run;
        sm[j] = run;
    }
    const double after = block_suffix(run, kInf, MinOp{}, shd);
    const double tot_lo = block_reduce(run, MinOp{}, shd);
    int tot_w;
    (void)block_prefix(nw, 0, AddOp{}, shi, tot_w);
#pragma unroll
    for (int j = 0; j < kSegR; ++j) {
        const int64_t k = k0 + threadIdx.x * kSegR + j;
        if (k < L.na) {
            P[L.comp_a + k] = pm[j] > before ? pm[j] : before;
            Q[L.comp_a + k] = sm[j] < after ? sm[j] : after;
        }
    }
    if (threadIdx.x == 0) {
        sg[0] = tot_hi;
        sg[1] = tot_lo;
        sg[2] = (double)tot_w;
    }
}

// grid (segments, dense labels): carry the other segments into P and Q, and
// list the wide components in record order (record .w = index bits)
__global__ __launch_bounds__(kBlock) void k_win_carry(const DLabel* __restrict__ labels,
                                                      const int32_t* __restrict__ grp,
                                                      const Comp<float>* __restrict__ comps32,
                                                      const SampRec* __restrict__ samp, int32_t nseg,
                                                      const int32_t* __restrict__ hist,
                                                      WinLabel* __restrict__ win, double* __restrict__ P,
                                                      double* __restrict__ Q,
                                                      const double* __restrict__ seg,
                                                      Comp<float>* __restrict__ wide,
                                                      uint8_t* __restrict__ wflag, double T) {
    const int y = blockIdx.y, li = grp[y];
    const DLabel L = labels[li];
    __shared__ double shd[kBlock / 64];
    __shared__ int shi[kBlock / 64];
    double xlo, xhi;
    label_range(L, samp, xlo, xhi, shd);
    const double thr = wide_threshold(hist + (size_t)y * kWidthBins, shi);
    const int s = blockIdx.x;
    const int64_t k0 = (int64_t)s * kSeg;
    if (k0 >= L.na) return;
    const int nseg_l = (int)((L.na + kSeg - 1) / kSeg);
    const double* sg = seg + (size_t)y * nseg * 3;
    double cp = -kInf, cq = kInf;
    int woff = 0;
    for (int t = 0; t < s; ++t) {
        cp = sg[3 * t] > cp ? sg[3 * t] : cp;
        woff += (int)sg[3 * t + 2];
    }
    for (int t = s + 1; t < nseg_l; ++t) cq = sg[3 * t + 1] < cq ? sg[3 * t + 1] : cq;
    const Comp<float>* c = comps32 + L.comp_a;
    bool fl[kSegR];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < kSegR; ++j) {
        const int64_t k = k0 + threadIdx.x * kSegR + j;
        fl[j] = false;
        if (k < L.na) {
            const size_t at = L.comp_a + k;
            P[at] = P[at] > cp ? P[at] : cp;
            Q[at] = Q[at] < cq ? Q[at] : cq;
            fl[j] = comp_interval(c[k], xhi - xlo, thr, T).wide;
            wflag[at] = fl[j];
        }
        cnt += fl[j];
    }
    int tot;
    int at = woff + block_prefix(cnt, 0, AddOp{}, shi, tot);
#pragma unroll
    for (int j = 0; j < kSegR; ++j)
        if (fl[j]) {
            const int k = (int)(k0 + threadIdx.x * kSegR + j);
            Comp<float> r = c[k];
            r.w = __int_as_float(k);
            wide[L.comp_a + at++] = r;
        }
    if (s == nseg_l - 1 && threadIdx.x == 0) win[li].n_wide = woff + tot;
}

// the recentred interval of bin b (open-ended at both ends), widened so that
// every x' with win_bin(x') == b lies inside despite the bin arithmetic's
// rounding
__device__ __forceinline__ void bin_edges(const WinLabel& W, int b, double& elo, double& ehi) {
    const double bw = 1.0 / W.inv_bw;
    elo = b == 0 ? -kInf : W.xlo + b * bw;
    ehi = b == kWinBins - 1 ? kInf : W.xlo + (b + 1) * bw;
    const double slack = (fabs(W.xlo) + bw * kWinBins) * 1e-12;
    elo -= slack;
    ehi += slack;
}

// grid (kWinBins / kBlock, dense labels): per bin the window [k_lo, k_hi):
// components before k_lo have hi < the bin's lower edge (P[k] < edge), those
// from k_hi on have lo > its upper edge (Q[k] > edge)
__global__ __launch_bounds__(kBlock) void k_win_bins(const DLabel* __restrict__ labels,
                                                     const int32_t* __restrict__ grp,
                                                     const WinLabel* __restrict__ win,
                                                     const double* __restrict__ P,
                                                     const double* __restrict__ Q,
                                                     int2* __restrict__ bins) {
    const int li = grp[blockIdx.y];
    const DLabel L = labels[li];
    const WinLabel W = win[li];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= kWinBins) return;
    double elo, ehi;
    bin_edges(W, b, elo, ehi);
    const double* p = P + L.comp_a;
    const double* q = Q + L.comp_a;
    int lo = 0, hi = L.na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (p[mid] >= elo) hi = mid; else lo = mid + 1;
    }
    const int klo = lo;
    lo = 0;
    hi = L.na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (q[mid] > ehi) hi = mid; else lo = mid + 1;
    }
    bins[(size_t)li * kWinBins + b] = int2{klo, lo > klo ? lo : klo};
}

// grid (kWinBins / kBlock, dense labels): per bin an upper bound of the
// skipped mass, sum over the narrow (and never-relevant) components outside
// the bin's window of the largest exact term they reach anywhere in the bin
// (widened by the candidates' fp32 rounding, 2^-22 relative).  A tile's
// window contains the window of every bin its candidates fall in, and its
// wide components are summed, so this bounds the mass the tile leaves out
// for each of its candidates.  Per component, from its fp32 record (m, a, c,
// log2 units): distance d of the centre m/a from the bin, |z| >= d a - delta
// with delta covering the record's rounding ((|x'| a + |m|) 2^-23), term <=
// 2^(c + |c| 2^-22 - z^2); fp32 exp2 (2 ulp), summed in fp64, x 1.01, plus
// na 2^-126 for the terms fp32 flushes.
//
// grid (kWinBins / kBlock, dense labels, component chunks of kSkipChunk):
// each chunk's partial sum per bin into part[(y nchunk + chunk) kWinBins + b];
// k_win_skip_sum adds the chunks in order (deterministic).
constexpr int kSkipChunk = 1024;

__global__ __launch_bounds__(kBlock) void k_win_skip(const DLabel* __restrict__ labels,
                                                     const int32_t* __restrict__ grp,
                                                     const Comp<float>* __restrict__ comps32,
                                                     const WinLabel* __restrict__ win,
                                                     const int2* __restrict__ bins,
                                                     const uint8_t* __restrict__ wflag,
                                                     double* __restrict__ part) {
    const int li = grp[blockIdx.y];
    const DLabel L = labels[li];
    const WinLabel W = win[li];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    const bool on = b < kWinBins;
    double elo, ehi;
    bin_edges(W, on ? b : 0, elo, ehi);
    const double wl = fmax(fabs(elo) < kInf ? fabs(elo) : 0.0, fabs(ehi) < kInf ? fabs(ehi) : 0.0);
    elo -= wl * 0x1.0p-22;
    ehi += wl * 0x1.0p-22;
    const int2 w = on ? bins[(size_t)li * kWinBins + b] : int2{0, 0};
    const Comp<float>* c = comps32 + L.comp_a;
    const uint8_t* fl = wflag + L.comp_a;
    double acc = 0.0;
    const int k0 = blockIdx.z * kSkipChunk, k1 = min(L.na, k0 + kSkipChunk);
    for (int k = k0; k < k1; ++k) {
        if (fl[k]) continue;                       // wide: summed by every tile
        if (k >= w.x && k < w.y) continue;         // in the bin's window
        const Comp<float> r = c[k];
        const double a = r.a, m = r.mu, cc = r.c;
        const double ctr = m / a;
        const double d = fmax(0.0, fmax(elo - ctr, ctr - ehi));
        const double xmax = fabs(ctr) + d;
        const double zl = fmax(0.0, d * a * (1.0 - 1e-9) - ((xmax * a + fabs(m)) * 0x1.0p-23 + 1e-9));
        const double t = cc + fabs(cc) * 0x1.0p-22 + 1e-9 - zl * zl;
        if (t > -126.0) acc += (double)__builtin_amdgcn_exp2f((float)(t + 1e-6 * (1.0 + fabs(t))));
    }
    if (on) part[((size_t)blockIdx.y * gridDim.z + blockIdx.z) * kWinBins + b] = acc;
}

__global__ __launch_bounds__(kBlock) void k_win_skip_sum(const DLabel* __restrict__ labels,
                                                         const int32_t* __restrict__ grp, int32_t nchunk,
                                                         const double* __restrict__ part,
                                                         double* __restrict__ skipm) {
    const int li = grp[blockIdx.y];
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= kWinBins) return;
    const int nc = (labels[li].na + kSkipChunk - 1) / kSkipChunk;
    double acc = 0.0;
    for (int c = 0; c < nc; ++c) acc += part[((size_t)blockIdx.y * nchunk + c) * kWinBins + b];
    skipm[(size_t)li * kWinBins + b] = acc * 1.01 + (double)labels[li].na * 0x1.0p-126;
}

// ------------------------------------------------------------- per round ----
// grid (ceil(n / 1024), labels, rounds of the batch): key (round, label, bin)
// and value (x' fp32 bits << 32 | candidate index) of every candidate, at
// position ((z - z0) nl + y) n + i.  The candidates are drawn exactly as the
// plain screen and the fp64 round draw them.
// Packed (cpack = C > 0, grid.z = 1): one cell per label, candidate j = z C
// + i of round z0 + z, value index j.  keys8: cells of >= kCellSortMin
// candidates are sorted one by one on a coarse 8-bit bin (one radix pass;
// the windows still come from the fine bins of each tile's min and max).
template <bool SAMPLE>
__global__ __launch_bounds__(kBlock) void k_win_key(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ grp,
    const SampRec* __restrict__ samp, const WinLabel* __restrict__ win,
    const double* __restrict__ cand_in, int64_t ncell, int32_t cpack, int64_t cand_offset,
    uint64_t seed, const uint32_t* __restrict__ rounds, int32_t z0, int32_t nl,
    uint32_t* __restrict__ keys, uint8_t* __restrict__ keys8, uint64_t* __restrict__ vals,
    int32_t* __restrict__ err) {
    const int y = blockIdx.y, li = grp[y];
    const DLabel L = labels[li];
    const WinLabel W = win[li];
    const bool lgmm = L.mode == DENSE_LGMM;
    const uint32_t cell = blockIdx.z * (uint32_t)nl + y;
#pragma unroll
    for (int r = 0; r < kKeyR; ++r) {
        const int64_t j = (int64_t)blockIdx.x * (kKeyR * kBlock) + r * kBlock + threadIdx.x;
        if (j >= ncell) continue;
        int64_t i = j, z = z0 + blockIdx.z;
        if (cpack) {
            z = z0 + j / cpack;
            i = j - (j / cpack) * cpack;
        }
        double v;
        if constexpr (SAMPLE) {
            const uint32_t g = (uint32_t)(cand_offset + i), rk = rounds[z];
            const bool ok = lgmm ? sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rk, g, v)
                                 : sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rk, g, v);
            if (!ok) atomicOr(err, 1);
        } else {
            v = cand_in[i];
        }
        const double xr = (lgmm ? flog(v) : v) - L.centre;
        const size_t pos = (size_t)cell * ncell + j;
        const uint32_t bin = (uint32_t)win_bin(W, xr);
        if (keys8) keys8[pos] = (uint8_t)(bin >> (kWinBinBits - kCoarseBits));
        else keys[pos] = (cell << kWinBinBits) | bin;
        vals[pos] = ((uint64_t)__float_as_uint((float)xr) << 32) | (uint32_t)j;
    }
}

// grid (ceil(n / 2048), labels, rounds of the batch): one tile of 2048
// sorted neighbours; see the file comment.  PROBE: per candidate index the
// fp32 score and its bound (tests).
template <bool PROBE>
__global__ __launch_bounds__(kBlock) void k_screen_win(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ grp,
    const Comp<float>* __restrict__ comps32, const WinLabel* __restrict__ win,
    const int2* __restrict__ bins, const Comp<float>* __restrict__ wide,
    const double* __restrict__ skipm,
    const uint64_t* __restrict__ vals, int64_t n, int32_t z0, int32_t nl, int32_t y0, int32_t nl_all,
    float* __restrict__ hi_out,
    unsigned long long* __restrict__ lbkey, unsigned long long* __restrict__ terms,
    double* __restrict__ s_out, double* __restrict__ e_out, float2* __restrict__ lohi) {
    constexpr int R = kWinR;
    const int y = blockIdx.y, li = grp[y];
    const DLabel L = labels[li];
    const WinLabel W = win[li];
    const size_t bcell = (size_t)blockIdx.z * nl + y;
    const size_t gcell = (size_t)(z0 + blockIdx.z) * nl_all + y0 + y;   // the whole round's cell
    const uint64_t* vrow = vals + bcell * n;
    const int64_t t0 = (int64_t)blockIdx.x * (R * kBlock);
    float xf[R];
    uint32_t ci[R];
    bool valid[R];
    double mn = kInf, mx = -kInf;
    int nv = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t p = t0 + r * kBlock + threadIdx.x;
        valid[r] = p < n;
        const uint64_t v = valid[r] ? vrow[p] : 0ull;
        xf[r] = __uint_as_float((uint32_t)(v >> 32));
        ci[r] = (uint32_t)v;
        if (valid[r]) {
            mn = fmin(mn, (double)xf[r]);
            mx = fmax(mx, (double)xf[r]);
            ++nv;
        } else {
            xf[r] = 0.0f;
        }
    }
    __shared__ double shd[kBlock / 64];
    __shared__ int shi[kBlock / 64];
    mn = block_reduce(mn, MinOp{}, shd);
    mx = block_reduce(mx, MaxOp{}, shd);
    int nvt;
    (void)block_prefix(nv, 0, AddOp{}, shi, nvt);
    // the true x' lies within 2^-24 |x'f| of the stored fp32 value
    const int b1 = win_bin(W, mn - fabs(mn) * 0x1.0p-23 - 0x1.0p-149);
    const int b2 = win_bin(W, mx + fabs(mx) * 0x1.0p-23 + 0x1.0p-149);
    const int2 w1 = bins[(size_t)li * kWinBins + b1], w2 = bins[(size_t)li * kWinBins + b2];
    const int klo = __builtin_amdgcn_readfirstlane(w1.x);
    const int khi = __builtin_amdgcn_readfirstlane(w2.y > w1.x ? w2.y : w1.x);
    float ab[R], aa[R];
    lse_acc<R>(comps32 + L.comp_b, L.nb, xf, ab);
    lse_acc<R>(comps32 + L.comp_a + klo, khi - klo, xf, aa);
    // the wide components outside the window, one by one
    float aw[R];
#pragma unroll
    for (int r = 0; r < R; ++r) aw[r] = 0.0f;
    int nout = 0;
    const Comp<float>* wl = wide + L.comp_a;
    for (int j = 0; j < W.n_wide; ++j) {
        const Comp<float> rec = wl[j];
        const int k = __float_as_int(rec.w);
        if (k >= klo && k < khi) continue;
        ++nout;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float z = fmaf(xf[r], rec.a, -rec.mu);
            aw[r] += __builtin_amdgcn_exp2f(fmaf(-z, z, rec.c));
        }
    }
    const int nwin = khi - klo;
    // summation error: the window's run (nwin / 128 + 28) u, the wide run
    // nout u, one more addition
    const int Kc = nwin + 128 * (nout + 1);
    uint64_t bk = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!valid[r]) continue;
        aa[r] += aw[r];
        const float l2b = __builtin_log2f(ab[r]), l2a = __builtin_log2f(aa[r]);
        const double lb = (double)l2b * 0.6931471805599453 + L.shift_b;
        const double la = (double)l2a * 0.6931471805599453 + L.shift_a;
        const double s = lb - la;
        const double X = fabs((double)xf[r]) * (1.0 + 0x1.0p-23);
        const double dx = X * 0x1.0p-24 + 0x1.0p-149;
        // the mass left out, bounded per bin of the candidate's own x'
        const double skip = skipm[(size_t)li * kWinBins + win_bin(W, (double)xf[r])] * 1.01 / (double)aa[r];
        const double E = 1.25 * (screen_err(L.amax_b, L.nb, L.nb, X, dx, ab[r], l2b) +
                                 screen_err(L.amax_a, L.na, Kc, X, dx, aa[r], l2a, skip) +
                                 fp64_err(L.nb + L.na, fabs(lb) + fabs(la) + X + fabs(L.centre)));
        if constexpr (PROBE) {
            s_out[ci[r]] = s;
            e_out[ci[r]] = E;
            continue;
        }
        const bool cert = E <= 1e30 && s == s;
        if (lohi) {   // packed: per candidate, selected per round by k_pick_win
            lohi[bcell * n + ci[r]] = cert ? float2{float_down(s - E), float_up(s + E)}
                                           : float2{-__builtin_inff(), __builtin_inff()};
            continue;
        }
        float h = __builtin_inff();
        if (cert) {
            h = float_up(s + E);
            const uint64_t key = order_key(s - E);
            bk = key > bk ? key : bk;
        }
        hi_out[gcell * n + t0 + r * kBlock + threadIdx.x] = h;
    }
    if (threadIdx.x == 0 && terms)
        atomicAdd(terms, (unsigned long long)nvt * (unsigned long long)(L.nb + nwin + nout));
    if (PROBE || lohi) return;
    __shared__ unsigned long long shk[kBlock / 64];
    struct KMax {
        __device__ unsigned long long operator()(unsigned long long a, unsigned long long b) const {
            return a > b ? a : b;
        }
    };
    const unsigned long long m = block_reduce((unsigned long long)bk, KMax{}, shk);
    if (threadIdx.x == 0 && m) atomicMax(lbkey + gcell, m);
}

}  // namespace

// ------------------------------------------------------------------ host ----
int64_t tpe_rt::win_rounds_per_batch(int64_t n, int32_t nl) {
    // the sort takes an int count: batches of at most 2^30 candidates
    const int64_t per = std::max<int64_t>(1, n * (int64_t)nl);
    return std::max<int64_t>(1, ((int64_t)1 << 30) / per);
}

int tpe_rt::win_prepare(tpe_ctx* ctx) {
    tpe_rt::Posterior& P = *ctx->P;
    if (P.win_ready && P.win_t == ctx->win_t) return TPE_OK;
    P.win_t = ctx->win_t;
    const double T = (double)ctx->win_t;
    const int nl = (int)(P.h_group[DENSE_GMM].size() + P.h_group[DENSE_LGMM].size());
    if (nl == 0) {
        P.win_ready = true;
        return TPE_OK;
    }
    int32_t na_max = 1;
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : P.h_group[m]) na_max = std::max(na_max, P.h_labels[li].na);
    const int nseg = (na_max + kSeg - 1) / kSeg;
    HIPCHK(ctx, P.win.reserve(P.n_labels));
    HIPCHK(ctx, P.win_p.reserve(P.comps32.cap));
    HIPCHK(ctx, P.win_q.reserve(P.comps32.cap));
    HIPCHK(ctx, P.win_wide.reserve(P.comps32.cap));
    HIPCHK(ctx, P.win_bins.reserve((size_t)P.n_labels * kWinBins));
    HIPCHK(ctx, P.win_seg.reserve((size_t)nl * nseg * 3));
    HIPCHK(ctx, P.win_hist.reserve((size_t)nl * kWidthBins));
    HIPCHK(ctx, P.win_flag.reserve(P.comps32.cap));
    HIPCHK(ctx, P.win_skip.reserve((size_t)P.n_labels * kWinBins));
    HIPCHK(ctx, hipMemsetAsync(P.win_hist.p, 0, (size_t)nl * kWidthBins * sizeof(int32_t), ctx->stream));
    const int32_t* grp = P.groups.p + P.group_off[DENSE_GMM];
    hipLaunchKernelGGL(k_win_hist, dim3(nseg, nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp,
                       P.comps32.p, P.samp.p, P.win_hist.p, T);
    hipLaunchKernelGGL(k_win_seg, dim3(nseg, nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp,
                       P.comps32.p, P.samp.p, nseg, P.win_hist.p, P.win.p, P.win_p.p, P.win_q.p,
                       P.win_seg.p, T);
    hipLaunchKernelGGL(k_win_carry, dim3(nseg, nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp,
                       P.comps32.p, P.samp.p, nseg, P.win_hist.p, P.win.p, P.win_p.p, P.win_q.p,
                       P.win_seg.p, P.win_wide.p, P.win_flag.p, T);
    hipLaunchKernelGGL(k_win_bins, dim3(kWinBins / kBlock, nl), dim3(kBlock), 0, ctx->stream,
                       P.labels.p, grp, P.win.p, P.win_p.p, P.win_q.p, P.win_bins.p);
    const int nchunk = (na_max + kSkipChunk - 1) / kSkipChunk;
    HIPCHK(ctx, P.win_skip_part.reserve((size_t)nl * nchunk * kWinBins));
    hipLaunchKernelGGL(k_win_skip, dim3(kWinBins / kBlock, nl, nchunk), dim3(kBlock), 0, ctx->stream,
                       P.labels.p, grp, P.comps32.p, P.win.p, P.win_bins.p, P.win_flag.p,
                       P.win_skip_part.p);
    hipLaunchKernelGGL(k_win_skip_sum, dim3(kWinBins / kBlock, nl), dim3(kBlock), 0, ctx->stream,
                       P.labels.p, grp, nchunk, P.win_skip_part.p, P.win_skip.p);
    HIPCHK(ctx, hipGetLastError());
    P.win_ready = true;
    return TPE_OK;
}

namespace {
struct Shape {
    int64_t ncell, cells;
    size_t total;
};
Shape shape_of(const tpe_rt::WinScreenArgs& a) {
    // candidates per cell; cells: (round, label), or one per label packed
    Shape sh;
    sh.ncell = a.cpack ? (int64_t)a.nz * a.cpack : a.n;
    sh.cells = a.cpack ? a.nl : (int64_t)a.nz * a.nl;
    sh.total = (size_t)sh.cells * sh.ncell;
    return sh;
}
int end_bit_of(int64_t cells) {
    int cell_bits = 0;
    while (((int64_t)1 << cell_bits) < cells) ++cell_bits;
    return kWinBinBits + cell_bits;
}
}  // namespace

int tpe_rt::win_reserve(tpe_ctx* ctx, size_t total, int64_t cells, int nslots) {
    if (total > ((size_t)1 << 30)) return ctx->fail(TPE_ERR_ARG, "windowed screen batch too large");
    const int64_t ncell = (int64_t)(total / (size_t)std::max<int64_t>(cells, 1));
    const bool per_cell = ncell >= kCellSortMin;
    for (int k = 0; k < nslots; ++k) {
        HIPCHK(ctx, ctx->win_vals[k].reserve(total));
        HIPCHK(ctx, ctx->win_vals2[k].reserve(total));
        size_t bytes = 0;
        if (per_cell) {
            HIPCHK(ctx, ctx->win_keys8[k].reserve(total));
            HIPCHK(ctx, ctx->win_keys8b[k].reserve(total));
            hipcub::DoubleBuffer<uint8_t> kb(ctx->win_keys8[k].p, ctx->win_keys8b[k].p);
            hipcub::DoubleBuffer<uint64_t> vb(ctx->win_vals[k].p, ctx->win_vals2[k].p);
            HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kb, vb, (int)ncell, 0,
                                                             kCoarseBits, ctx->stream));
        } else {
            HIPCHK(ctx, ctx->win_keys[k].reserve(total));
            HIPCHK(ctx, ctx->win_keys2[k].reserve(total));
            hipcub::DoubleBuffer<uint32_t> kb(ctx->win_keys[k].p, ctx->win_keys2[k].p);
            hipcub::DoubleBuffer<uint64_t> vb(ctx->win_vals[k].p, ctx->win_vals2[k].p);
            HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kb, vb, (int)total, 0,
                                                             end_bit_of(cells), ctx->stream));
        }
        HIPCHK(ctx, ctx->win_tmp[k].reserve(std::max<size_t>(bytes, 1)));
    }
    return TPE_OK;
}

int tpe_rt::win_sort(tpe_ctx* ctx, const WinScreenArgs& a, hipStream_t st, const uint64_t** sorted) {
    tpe_rt::Posterior& P = *ctx->P;
    const Shape sh = shape_of(a);
    const int k = a.slot;
    const bool per_cell = sh.ncell >= kCellSortMin;
    if (sh.total > ctx->win_vals[k].cap || sh.total > ((size_t)1 << 30) ||
        sh.total > (per_cell ? ctx->win_keys8[k].cap : ctx->win_keys[k].cap))
        return ctx->fail(TPE_ERR_ARG, "windowed screen: slot buffers not reserved");
    uint32_t* keys = per_cell ? nullptr : ctx->win_keys[k].p;
    uint8_t* keys8 = per_cell ? ctx->win_keys8[k].p : nullptr;
    const dim3 gk((unsigned)((sh.ncell + kKeyR * kBlock - 1) / (kKeyR * kBlock)), a.nl,
                  a.cpack ? 1 : a.nz);
    if (a.cand_in)
        hipLaunchKernelGGL(k_win_key<false>, gk, dim3(kBlock), 0, st, P.labels.p, a.grp, P.samp.p,
                           P.win.p, a.cand_in, sh.ncell, 0, a.cand_offset, a.seed, ctx->rounds.p, a.z0,
                           a.nl, keys, keys8, ctx->win_vals[k].p, ctx->errflag.p);
    else
        hipLaunchKernelGGL(k_win_key<true>, gk, dim3(kBlock), 0, st, P.labels.p, a.grp, P.samp.p,
                           P.win.p, nullptr, sh.ncell, a.cpack, a.cand_offset, a.seed, ctx->rounds.p,
                           a.z0, a.nl, keys, keys8, ctx->win_vals[k].p, ctx->errflag.p);
    HIPCHK(ctx, hipGetLastError());
    if (per_cell) {   // one single-pass sort per cell, all ending in the same buffer
        const uint64_t* out = nullptr;
        for (int64_t c = 0; c < sh.cells; ++c) {
            const size_t off = (size_t)c * sh.ncell;
            hipcub::DoubleBuffer<uint8_t> kb(ctx->win_keys8[k].p + off, ctx->win_keys8b[k].p + off);
            hipcub::DoubleBuffer<uint64_t> vb(ctx->win_vals[k].p + off, ctx->win_vals2[k].p + off);
            size_t bytes = ctx->win_tmp[k].cap;
            HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(ctx->win_tmp[k].p, bytes, kb, vb, (int)sh.ncell,
                                                             0, kCoarseBits, st));
            const uint64_t* base = vb.Current() - off;
            if (out && base != out) return ctx->fail(TPE_ERR_HIP, "windowed screen: sort buffers diverged");
            out = base;
        }
        *sorted = out;
        return TPE_OK;
    }
    hipcub::DoubleBuffer<uint32_t> kb(ctx->win_keys[k].p, ctx->win_keys2[k].p);
    hipcub::DoubleBuffer<uint64_t> vb(ctx->win_vals[k].p, ctx->win_vals2[k].p);
    size_t bytes = ctx->win_tmp[k].cap;
    HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(ctx->win_tmp[k].p, bytes, kb, vb, (int)sh.total, 0,
                                                     end_bit_of(sh.cells), st));
    *sorted = vb.Current();
    return TPE_OK;
}

int tpe_rt::win_tiles(tpe_ctx* ctx, const WinScreenArgs& a, const uint64_t* sorted, hipStream_t st) {
    tpe_rt::Posterior& P = *ctx->P;
    const Shape sh = shape_of(a);
    const dim3 gs((unsigned)((sh.ncell + kWinR * kBlock - 1) / (kWinR * kBlock)), a.nl,
                  a.cpack ? 1 : a.nz);
    const int32_t nl_all = a.nl_all ? a.nl_all : a.nl;
    if (a.cand_in)
        hipLaunchKernelGGL(k_screen_win<true>, gs, dim3(kBlock), 0, st, P.labels.p, a.grp, P.comps32.p,
                           P.win.p, P.win_bins.p, P.win_wide.p, P.win_skip.p, sorted, sh.ncell, a.z0,
                           a.nl, a.y0, nl_all, nullptr, nullptr, nullptr, a.s_out, a.e_out, nullptr);
    else
        hipLaunchKernelGGL(k_screen_win<false>, gs, dim3(kBlock), 0, st, P.labels.p, a.grp, P.comps32.p,
                           P.win.p, P.win_bins.p, P.win_wide.p, P.win_skip.p, sorted, sh.ncell, a.z0,
                           a.nl, a.y0, nl_all, a.hi, a.lbkey, ctx->win_evals.p, nullptr, nullptr, a.lohi);
    return ctx->hip(hipGetLastError(), "k_screen_win launch");
}

int tpe_rt::win_screen(tpe_ctx* ctx, const WinScreenArgs& a, const uint64_t** sorted_vals) {
    const Shape sh = shape_of(a);
    int rc = win_reserve(ctx, sh.total, sh.cells, 1);
    if (rc) return rc;
    WinScreenArgs b = a;
    b.slot = 0;
    if ((rc = win_sort(ctx, b, ctx->stream, sorted_vals))) return rc;
    const bool timed = ctx->timing && !a.cand_in;
    if (timed) HIPCHK(ctx, hipEventRecord(ctx->evs[0], ctx->stream));
    if ((rc = win_tiles(ctx, b, *sorted_vals, ctx->stream))) return rc;
    if (timed) HIPCHK(ctx, hipEventRecord(ctx->evs[1], ctx->stream));
    return TPE_OK;
}
