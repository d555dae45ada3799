// tpe_engine.hip -- gfx950 kernels + C ABI (include/hyperopt_tpe.h) of the
// TPE suggestion hot path (mvanveen/hyperopt hyperopt/tpe.py:651-916).
//
// Layout in HBM (resident per context, replaced by tpe_set_posterior):
//   labels   : DLabel[L]                  per-label mode, bounds, shifts, offsets
//   comps64  : Comp<double>[records]      below then above mixture of each label
//   comps32  : Comp<float>[records]       fp32 copy of the dense records (TPE_F32)
//   samp     : SampRec[sum K_b]           cumulative weights + mu/sigma of l(x)
// Per round:
//   partials : Partial[rounds][L][tiles]  per-workgroup winners
//   results  : tpe_label_result[rounds][L]
//   qj       : int64[rounds][Lq][C]       grid index of every quantized candidate
//   qtab     : double2[sum G]             lpdf pair per distinct grid value
//   chunk_part: double[labels][chunks + 2][gx][R * 256]  chunked packed map sums
// Kernels
//   k_round<T, MODE, SAMPLE>  sample -> lpdf under l and g -> block maxloc
//                             (dense families, categorical, supplied candidates)
//   k_round_chunk / k_finish_chunks
//                             packed rounds with the above mixture cut into
//                             chunks along grid.z, then in-order sum -> maxloc
//   k_sample_small / k_score_slices / k_finish_slices
//                             split-K map of small rounds (C * rounds <= 2048)
//   k_qsample<MODE>           quantized families: draw, store grid index j, min/max
//   k_qtable<MODE>            one workgroup per distinct grid value: lpdf pair
//   k_qscan<MODE>             per candidate: table lookup -> block maxloc
//   k_reduce / k_emit         per (round, label) winner over the partials
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hyperopt_tpe.h"
#include "tpe_ctx.h"
#include "tpe_device.h"

using namespace tpe;
using namespace tpe_rt;

namespace {

constexpr int kR = 4;                 // candidates per thread, tile map
constexpr int kRGroup = 3;            // candidates per thread, packed map with C <= 768
constexpr int kTile = kBlock * kR;    // candidates per workgroup, tile map

thread_local std::string g_create_error;


// ---------------------------------------------------------- block maxloc ----
// broadcast_best (tpe.py:769-778) over one workgroup's candidates: per-thread
// best of its R, wave64 butterfly, then the 4 waves through LDS.
// `sh` is the calling kernel's kBlock/64-entry LDS array (declared in the
// kernel, so every kernel owns exactly the LDS it declares).
__device__ __forceinline__ void block_maxloc(uint64_t bk, int64_t bi, double bv, double bl,
                                             double ba, Partial* __restrict__ dst,
                                             Partial* __restrict__ sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t ok = __shfl_xor(bk, off);
        const int64_t oi = __shfl_xor(bi, off);
        const double ov = __shfl_xor(bv, off), ol = __shfl_xor(bl, off), oa = __shfl_xor(ba, off);
        if (better(ok, oi, bk, bi)) {
            bk = ok;
            bi = oi;
            bv = ov;
            bl = ol;
            ba = oa;
        }
    }
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) sh[tid >> 6] = Partial{bk, bi, bv, bl, ba};
    __syncthreads();
    if (tid == 0) {
        Partial best = sh[0];
        for (int w = 1; w < kBlock / 64; ++w)
            if (better(sh[w].key, sh[w].idx, best.key, best.idx)) best = sh[w];
        *dst = best;
    }
}

// ------------------------------------------------------------ slot maps ----
// Where slot r of a thread lives.
//  * Tile map (cpack == 0): one round per grid.z, that round's candidates
//    spread over the grid (large C).
//  * Packed map (cpack == C < 256 R): rpb = floor(256 R / C) whole rounds per
//    workgroup, rounds along grid.x -- batched rounds with small C (e.g. 4096
//    new_ids x 24 candidates) keep the lanes busy; the per-round maxloc goes
//    through LDS.
struct Slots {
    int32_t cpack;      // candidates per round in the packed map, 0 = tile map
    int32_t rpb;        // rounds per workgroup (packed map)
    int32_t n_rounds;

    template <int R>
    __device__ __forceinline__ void at(int r, int64_t n, int64_t& z, int64_t& i,
                                       bool& valid) const {
        if (cpack == 0) {
            z = blockIdx.z;
            i = (int64_t)blockIdx.x * (R * kBlock) + r * kBlock + threadIdx.x;
            valid = i < n;
        } else {
            const int local = r * kBlock + threadIdx.x;
            const int zr = local / cpack;
            z = (int64_t)blockIdx.x * rpb + zr;
            i = local - zr * cpack;
            valid = zr < rpb && z < n_rounds;
        }
    }
};

// packed map with kRGroup slots per thread (else kR: tile map, or packed
// rounds spread over kR * 256 slots)
__host__ __device__ inline bool narrow(const Slots& S) {
    return S.cpack != 0 && (int64_t)S.rpb * S.cpack <= kBlock * kRGroup;
}

// broadcast_best epilogue for either map: block maxloc into the tile's
// partial, or, packed, one winner per round: every slot posts its key to
// LDS, a reducer per round picks the best slot (slots of a round are in
// candidate order, so the lowest slot among equal keys is the lowest index),
// and the owner of that slot writes the round's record.
template <int R>
__device__ __forceinline__ void finish_slots(const Slots& S, const double (&x)[R],
                                             const double (&lb)[R], const double (&la)[R],
                                             const bool (&valid)[R], const int64_t (&z)[R],
                                             const int64_t (&gi)[R], int li, int32_t n_labels,
                                             int32_t tiles, Partial* __restrict__ partials,
                                             void* lds_scratch, Partial* __restrict__ sh) {
    if (S.cpack == 0) {
        uint64_t bk = 0;
        int64_t bi = INT64_MAX;
        double bv = 0.0, bl = 0.0, ba = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!valid[r]) continue;
            const uint64_t key = order_key(lb[r] - la[r]);
            if (better(key, gi[r], bk, bi)) {
                bk = key;
                bi = gi[r];
                bv = x[r];
                bl = lb[r];
                ba = la[r];
            }
        }
        block_maxloc(bk, bi, bv, bl, ba,
                     partials + ((size_t)blockIdx.z * n_labels + li) * tiles + blockIdx.x, sh);
        return;
    }
    // scratch: R*256 keys + R*256 winners (12 KB at R = 4), aliased on the
    // exp table, which every wave has finished reading at the barrier
    static_assert(R * kBlock * (sizeof(uint64_t) + sizeof(int32_t)) <=
                  kExpTabSize * sizeof(double), "packed scratch exceeds the LDS table");
    __syncthreads();
    uint64_t* keys = reinterpret_cast<uint64_t*>(lds_scratch);
    int32_t* win = reinterpret_cast<int32_t*>(keys + R * kBlock);
    uint64_t key[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        key[r] = valid[r] ? order_key(lb[r] - la[r]) : 0;
        keys[r * kBlock + threadIdx.x] = key[r];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < S.rpb; t += kBlock) {
        const int s0 = t * S.cpack;
        int best = s0;
        uint64_t bk = keys[s0];
        for (int c = 1; c < S.cpack; ++c)
            if (keys[s0 + c] > bk) {
                bk = keys[s0 + c];
                best = s0 + c;
            }
        win[t] = best;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!valid[r]) continue;
        const int local = r * kBlock + threadIdx.x;
        if (win[local / S.cpack] == local)
            partials[(size_t)z[r] * n_labels + li] = Partial{key[r], gi[r], x[r], lb[r], la[r]};
    }
}

// --------------------------------------------------------------- kernels ----

// The candidates of a thread's R slots: drawn from the below mixture (the
// label's Philox stream, round key, candidate index) or read from cand_in.
// RAW: LGMM1 slots keep the accepted log-space draw (no exp; the caller
// applies lgmm_value where it needs the sample itself)
template <int MODE, bool SAMPLE, int R, bool RAW = false>
__device__ __forceinline__ void draw_slots(const DLabel& L, const Slots& S, bool lgmm,
                                           const SampRec* __restrict__ samp,
                                           const double* __restrict__ cand_in, int64_t n,
                                           int64_t cand_offset, uint64_t seed,
                                           const uint32_t* __restrict__ rounds,
                                           int32_t* __restrict__ err, double (&x)[R],
                                           int64_t (&z)[R], int64_t (&ci)[R], int64_t (&gi)[R],
                                           bool (&valid)[R], const SampLds* sl = nullptr) {
    uint32_t g32[R], rk[R], pend = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        S.template at<R>(r, n, z[r], ci[r], valid[r]);
        gi[r] = cand_offset + ci[r];
        g32[r] = (uint32_t)gi[r];
        rk[r] = 0;
        x[r] = lgmm ? 1.0 : 0.0;
        if (valid[r]) {
            pend |= 1u << r;
            if constexpr (SAMPLE) rk[r] = rounds[z[r]];
            else x[r] = cand_in[ci[r]];
        }
    }
    if constexpr (SAMPLE) {
        if constexpr (MODE == CAT) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (valid[r]) (void)sample_below<CAT>(L, samp + L.samp_off, seed, rk[r], g32[r], x[r]);
        } else {
            bool ok;
            if (sl) {
                const SampShared src{sl};
                if constexpr (MODE == DENSE_ANY)
                    ok = lgmm ? sample_slots<DENSE_LGMM, R, SampShared, RAW>(L, src, seed, rk, g32, pend, x)
                              : sample_slots<DENSE_GMM, R, SampShared, RAW>(L, src, seed, rk, g32, pend, x);
                else
                    ok = sample_slots<MODE, R, SampShared, RAW>(L, src, seed, rk, g32, pend, x);
            } else {
                const SampGlobal src{samp + L.samp_off, L.ns};
                if constexpr (MODE == DENSE_ANY)
                    ok = lgmm ? sample_slots<DENSE_LGMM, R, SampGlobal, RAW>(L, src, seed, rk, g32, pend, x)
                              : sample_slots<DENSE_GMM, R, SampGlobal, RAW>(L, src, seed, rk, g32, pend, x);
                else
                    ok = sample_slots<MODE, R, SampGlobal, RAW>(L, src, seed, rk, g32, pend, x);
            }
            if (!ok) atomicOr(err, 1);
            if (L.flags & 4) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (valid[r]) x[r] = quantize(x[r], L.q);
            }
        }
    }
}

template <typename T, int MODE, bool SAMPLE, int R>
__global__ __launch_bounds__(kBlock) void k_round(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<T>* __restrict__ comps, const Comp<double>* __restrict__ comps64,
    const SampRec* __restrict__ samp, const double* __restrict__ cand_in, int64_t n,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, int32_t n_labels,
    int32_t tiles, Partial* __restrict__ partials, double* __restrict__ out_lb,
    double* __restrict__ out_la, int32_t* __restrict__ err, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    __shared__ double exp_tab[kExpTabSize];
    constexpr bool kDense = MODE == DENSE_GMM || MODE == DENSE_LGMM || MODE == DENSE_ANY;
    if constexpr (kDense) load_exp_table(exp_tab);
    // LGMM1 label? (compile-time, or per label -- uniform over the workgroup)
    const bool lgmm = MODE == DENSE_LGMM || MODE == QUANT_LGMM ||
                      (MODE == DENSE_ANY && L.mode == DENSE_LGMM);

    double x[R], lb[R], la[R];
    int64_t z[R], ci[R], gi[R];
    bool valid[R];
    draw_slots<MODE, SAMPLE, R>(L, S, lgmm, samp, cand_in, n, cand_offset, seed, rounds, err, x, z,
                                ci, gi, valid);

    if constexpr (kDense) {
        double y[R];
        if (lgmm) {
#pragma unroll
            for (int r = 0; r < R; ++r) y[r] = flog(x[r]);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) y[r] = x[r];
        }
        lse_dense<R>(comps + L.comp_b, L.nb, L.shift_b, L.centre, y, lb, exp_tab);
        lse_dense<R>(comps + L.comp_a, L.na, L.shift_a, L.centre, y, la, exp_tab);
        if (lgmm) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                lb[r] -= y[r];
                la[r] -= y[r];
            }
        }
    } else if constexpr (MODE == QUANT_GMM || MODE == QUANT_LGMM) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double ub, lo;
            bool neg;
            quant_bounds<MODE>(L, x[r], ub, lo, neg);
            if (valid[r] && neg) atomicOr(err, 2);
            lb[r] = quant_lpdf<MODE == QUANT_LGMM>(comps64 + L.comp_b, L.nb, ub, lo, L.logpacc_b);
            la[r] = quant_lpdf<MODE == QUANT_LGMM>(comps64 + L.comp_a, L.na, ub, lo, L.logpacc_a);
        }
    } else {  // CAT: categorical_lpdf = log(p[sample])   tpe.py:56-63
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t s = (int64_t)x[r];
            if (valid[r] && (s < 0 || s >= L.nb || (double)s != x[r])) atomicOr(err, 4);
            const int64_t sc = s < 0 ? 0 : (s >= L.nb ? L.nb - 1 : s);
            lb[r] = comps64[L.comp_b + sc].c;
            la[r] = comps64[L.comp_a + sc].c;
        }
    }

    if (out_lb) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (valid[r]) {
                const size_t row = ((size_t)z[r] * n_labels + li) * (size_t)n;
                out_lb[row + ci[r]] = lb[r];
                out_la[row + ci[r]] = la[r];
            }
    }
    __shared__ Partial sh[kBlock / 64];
    finish_slots<R>(S, x, lb, la, valid, z, gi, li, n_labels, tiles, partials, exp_tab, sh);
}

// ------------------------------------------------- chunked packed map ----
// Batched sampled rounds with small C (e.g. 512 new_ids x 24 candidates)
// give the packed map only gx * labels workgroups -- for config 5 that is
// ~1200, one generation of workgroups with a long tail.  The above mixture's components are then cut into `nch`
// chunks along grid.z: each workgroup draws the same slots (Philox is
// stateless), sums its chunk relative to the label's LSE shift (chunk 0 also
// the below mixture) and stores the raw sums; k_finish_chunks adds the
// chunks in order, takes the logs and does the per-round maxloc.
//
// part layout per (label position y, plane p, workgroup x): R * 256 slots,
// planes 0 = candidate, 1 = below sum, 2 + c = above sum of chunk c.
__device__ __forceinline__ size_t chunk_plane(int y, int p, int nch, int x, int gx, int R) {
    return (((size_t)y * (nch + 2) + p) * gx + x) * (size_t)(R * kBlock);
}

template <typename T, int R>
__global__ __launch_bounds__(kBlock) void k_round_chunk(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<T>* __restrict__ comps, const SampRec* __restrict__ samp, int64_t n,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, int32_t chunk,
    double* __restrict__ part, int32_t* __restrict__ err, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    constexpr bool kTab = sizeof(T) == 8;
    __shared__ double exp_tab[kTab ? kExpTabSize : 1];
    if constexpr (kTab) load_exp_table(exp_tab);
    const bool lgmm = L.mode == DENSE_LGMM;
    const int nch = gridDim.z, c = blockIdx.z;
    double x[R], y[R];
    int64_t z[R], ci[R], gi[R];
    bool valid[R];
    draw_slots<DENSE_ANY, true, R>(L, S, lgmm, samp, nullptr, n, cand_offset, seed, rounds, err, x,
                                   z, ci, gi, valid);
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = lgmm ? flog(x[r]) : x[r];
    const int k0 = min(c * chunk, L.na), k1 = min(k0 + chunk, L.na);
    double sb[R], sa[R];
    if constexpr (kTab) {
        double xr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            xr[r] = y[r] - L.centre;
            sb[r] = 0.0;
            sa[r] = 0.0;
        }
        if (c == 0) lse_acc<R>(comps + L.comp_b, L.nb, xr, sb, exp_tab);
        lse_acc<R>(comps + L.comp_a + k0, k1 - k0, xr, sa, exp_tab);
    } else {
        float fb[R], fa[R], xf[R];
#pragma unroll
        for (int r = 0; r < R; ++r) xf[r] = (float)(y[r] - L.centre);
        if (c == 0) lse_acc<R>(comps + L.comp_b, L.nb, xf, fb);
        lse_acc<R>(comps + L.comp_a + k0, k1 - k0, xf, fa);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            sb[r] = c == 0 ? (double)fb[r] : 0.0;
            sa[r] = (double)fa[r];
        }
    }
    const int gx = gridDim.x, bx = blockIdx.x, by = blockIdx.y;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int s = r * kBlock + threadIdx.x;
        if (c == 0) {
            part[chunk_plane(by, 0, nch, bx, gx, R) + s] = x[r];
            part[chunk_plane(by, 1, nch, bx, gx, R) + s] = sb[r];
        }
        part[chunk_plane(by, 2 + c, nch, bx, gx, R) + s] = sa[r];
    }
}

template <typename T, int R>
__global__ __launch_bounds__(kBlock) void k_finish_chunks(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<T>* __restrict__ comps, int64_t n, int64_t cand_offset, int32_t n_labels,
    int32_t tiles, int32_t nch, const double* __restrict__ part, Partial* __restrict__ partials,
    double* __restrict__ out_lb, double* __restrict__ out_la, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int gx = gridDim.x, bx = blockIdx.x, by = blockIdx.y;
    double x[R], lb[R], la[R];
    int64_t z[R], gi[R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int64_t ci;
        S.template at<R>(r, n, z[r], ci, valid[r]);
        gi[r] = cand_offset + ci;
        const int s = r * kBlock + threadIdx.x;
        x[r] = part[chunk_plane(by, 0, nch, bx, gx, R) + s];
        const double sb = part[chunk_plane(by, 1, nch, bx, gx, R) + s];
        double sa = 0.0;
        for (int c = 0; c < nch; ++c) sa += part[chunk_plane(by, 2 + c, nch, bx, gx, R) + s];
        const double y = lgmm ? flog(x[r]) : x[r];
        if constexpr (sizeof(T) == 8) {
            lb[r] = lse_finish(comps + L.comp_b, L.nb, sb, y - L.centre, L.shift_b);
            la[r] = lse_finish(comps + L.comp_a, L.na, sa, y - L.centre, L.shift_a);
        } else {
            lb[r] = lse_finish(comps + L.comp_b, L.nb, (float)sb, (float)(y - L.centre), L.shift_b);
            la[r] = lse_finish(comps + L.comp_a, L.na, (float)sa, (float)(y - L.centre), L.shift_a);
        }
        if (lgmm) {
            lb[r] -= y;
            la[r] -= y;
        }
        if (out_lb && valid[r]) {
            const size_t row = ((size_t)z[r] * n_labels + li) * (size_t)n;
            out_lb[row + ci] = lb[r];
            out_la[row + ci] = la[r];
        }
    }
    __shared__ uint64_t scratch[R * kBlock * 3 / 2];   // finish_slots: keys + winners
    __shared__ Partial sh[kBlock / 64];
    finish_slots<R>(S, x, lb, la, valid, z, gi, li, n_labels, tiles, partials, scratch, sh);
}

// ------------------------------------------------ fp32 screen (tile map) ----
// The exact fp64 round of the dense labels in three kernels:
//   k_screen   every candidate in packed fp32 (3.5 issue slots per eval
//              instead of 12.25): an upper bound hi = s32 + E of its score
//              and, per (round, label), the largest lower bound s32 - E
//              (E: screen_err + fp64_err, tpe_device.h, x 1.25);
//   k_select   compacts the candidates with hi >= that lower bound -- the
//              only ones whose fp64 score can reach the fp64 maximum;
//   k_rescore  draws them again (Philox is stateless) and scores them with
//              the fp64 code of k_round, so the winner, its value and its
//              lpdfs are bit-identical to the unscreened round's.
// Scores are per (round, label) rows of n candidates; hi and the compacted
// indices use the label's position in the dense group (blockIdx.y).
__device__ __forceinline__ uint64_t block_max_key(uint64_t k, uint64_t* __restrict__ sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(k, off);
        k = o > k ? o : k;
    }
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = k;
    __syncthreads();
    uint64_t m = sh[0];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) m = sh[w] > m ? sh[w] : m;
    return m;
}

// SAMPLE = false (tpe_screen_probe, tests): candidates from cand_in, and the
// fp32 score and its error bound written per candidate instead
template <int R, bool SAMPLE>
__global__ __launch_bounds__(kBlock) void k_screen(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<float>* __restrict__ comps32, const SampRec* __restrict__ samp, int64_t n,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, int32_t nl,
    float* __restrict__ hi, unsigned long long* __restrict__ lbkey, int32_t* __restrict__ err,
    Slots S, const double* __restrict__ cand_in, double* __restrict__ s_out,
    double* __restrict__ e_out) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const bool lgmm = L.mode == DENSE_LGMM;
    double x[R];
    int64_t z[R], ci[R], gi[R];
    bool valid[R];
    draw_slots<DENSE_ANY, SAMPLE, R>(L, S, lgmm, samp, cand_in, n, cand_offset, seed, rounds, err,
                                     x, z, ci, gi, valid);
    double y[R], X[R], dx[R];
    float xf[R], ab[R], aa[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        y[r] = lgmm ? flog(x[r]) : x[r];
        const double xr = y[r] - L.centre;
        xf[r] = (float)xr;
        X[r] = fabs(xr);
        dx[r] = fabs((double)xf[r] - xr);
    }
    lse_acc<R>(comps32 + L.comp_b, L.nb, xf, ab);
    lse_acc<R>(comps32 + L.comp_a, L.na, xf, aa);
    const size_t row = ((size_t)blockIdx.z * nl + blockIdx.y) * (size_t)n;
    uint64_t bk = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!valid[r]) continue;
        const float l2b = __builtin_log2f(ab[r]), l2a = __builtin_log2f(aa[r]);
        const double lb = (double)l2b * 0.6931471805599453 + L.shift_b;
        const double la = (double)l2a * 0.6931471805599453 + L.shift_a;
        const double s = lb - la;
        const double E = 1.25 * (screen_err(L.amax_b, L.nb, L.nb, X[r], dx[r], ab[r], l2b) +
                                 screen_err(L.amax_a, L.na, L.na, X[r], dx[r], aa[r], l2a) +
                                 fp64_err(L.nb + L.na, fabs(lb) + fabs(la) + fabs(y[r])));
        if constexpr (!SAMPLE) {
            s_out[ci[r]] = s;
            e_out[ci[r]] = E;
            continue;
        }
        float h = __builtin_inff();
        if (E <= 1e30 && s == s) {
            h = float_up(s + E);
            const uint64_t k = order_key(s - E);
            bk = k > bk ? k : bk;
        }
        hi[row + ci[r]] = h;
    }
    if constexpr (!SAMPLE) return;
    __shared__ uint64_t sh[kBlock / 64];
    bk = block_max_key(bk, sh);
    if (threadIdx.x == 0 && bk) atomicMax(lbkey + (size_t)blockIdx.z * nl + blockIdx.y, bk);
}

// The expansion screen (tpe_device.h "expansion screen", index from
// tpe_expand.hip): per candidate the below mixture through the fp64 round's
// own code (lpdf_below bit-identical to it), the above mixture as its bin's
// Taylor polynomial (clipped components) plus the bin's list of unclipped
// components (direct fp64 terms), and a rigorous bound E of |s - s64|:
//   |S - S_exact| <= Eabs_bin (truncation + rounding of the table)
//                  + 8 u S_clip (exp(-kappa delta^2)) + na 2^-T (left out)
//                  + (3e-14 + (n_list + 4) u) S_list + 2 u S,
//   eps = that / S, |log S - log S_exact| <= 1.001 eps + 2u (|log S| + 1),
//   E = 1.25 (that + fp64_err), the fp64 round's own distance from exact.
// Candidates outside the bins, with S < 1e-280 or eps > 1e-6, or NaN, get
// s = NaN, E = +inf (always re-scored).  E is ~1e-12, far below an fp32
// rounding of the score.  Returns the terms the R candidates summed
// directly (nb + list each).
constexpr int kListU = 4;   // bin-list entries loaded per step (bx_score)
template <int R>
__device__ __forceinline__ int bx_score(const DLabel& L, const BxLabel& B,
                                        const Comp<double>* __restrict__ comps64,
                                        const double* __restrict__ tab, const int32_t* __restrict__ loff,
                                        const int32_t* __restrict__ list, const double* __restrict__ exp_tab,
                                        const double (&x)[R], const bool (&valid)[R], double (&s)[R],
                                        double (&E)[R]) {
    const bool lgmm = L.mode == DENSE_LGMM;
    double y[R], xr[R], acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        y[r] = lgmm ? flog(x[r]) : x[r];
        xr[r] = y[r] - L.centre;
        acc[r] = 0.0;
    }
    // below: the fp64 round's lse_dense, term for term
    lse_acc<R>(comps64 + L.comp_b, L.nb, xr, acc, exp_tab);
    // (lb itself is not needed: s = log(acc_b / S) + shift_b - shift_a, one
    // log instead of two; candidates whose below sum underflows -- the fp64
    // round's two-pass fallback -- are uncertified)
    const Comp<double>* ca = comps64 + L.comp_a;
    const double skip_abs = (double)L.na * exp2(-B.tcut);
    int nterms = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        s[r] = __builtin_nan("");
        E[r] = __builtin_inf();
        if (!valid[r]) continue;
        const int b = bx_bin(B, xr[r]);
        if (b < 0) continue;
        const double delta = xr[r] - (B.xlo + ((double)b + 0.5) * B.bw);
        const double* rw = tab + (size_t)(B.tab_off + b) * kBxRow;
        double poly = rw[kBxP - 1];
#pragma unroll
        for (int k = kBxP - 2; k >= 0; --k) poly = fma(poly, delta, rw[k]);
        const double eabs = rw[kBxP];
        // exp(-t), t = kappa delta^2 <= kappa rmax^2 <= 0.0625 / (T ln 2) < 3e-3 (T >= 32):
        // degree 5 leaves t^6 / 720 < 2e-21 (inside the 8 u S_clip term)
        const double t = B.kappa * delta * delta;
        const double et = fma(fma(fma(fma(fma(-1.0 / 120.0, t, 1.0 / 24.0), t, -1.0 / 6.0), t, 0.5), t,
                                  -1.0), t, 1.0);
        const double sclip = et * poly;
        const int j0 = 0, j1 = loff[B.cnt_off + b];   // the bin's count, its slot of n_nc entries
        const int32_t* lst = list + B.list_off + (int64_t)b * B.n_nc;
        double snc = 0.0;
        // the list walked kListU entries at a time: their indices, then
        // their records, loaded before the terms are added in order (one
        // entry per step was two dependent loads per term: the screen's
        // latency, r6r)
        for (int j = j0; j < j1; j += kListU) {
            int32_t kk[kListU];
#pragma unroll
            for (int u = 0; u < kListU; ++u) kk[u] = lst[min(j + u, j1 - 1)];
            Comp<double> rr[kListU];
#pragma unroll
            for (int u = 0; u < kListU; ++u) rr[u] = ca[kk[u]];
#pragma unroll
            for (int u = 0; u < kListU; ++u)
                if (j + u < j1) {
                    const double zz = fma(xr[r], rr[u].a, -rr[u].mu);
                    snc = exp_scaled_acc(fma(-zz, zz, rr[u].c), exp_tab, snc);
                }
        }
        nterms += L.nb + (j1 - j0);
        const double sum = sclip + snc;
        const double ea = eabs + 8.0 * 0x1.0p-53 * fabs(sclip) + skip_abs +
                          (3e-14 + (double)(j1 - j0 + 4) * 0x1.0p-53) * snc + 0x1.0p-52 * sum;
        // 1 / sum: hardware reciprocal + one Newton step (relative error
        // ~2^-50), and 1.0001 on top: eps only bounds
        const double r0 = __builtin_amdgcn_rcp(sum);
        const double rs = fma(fma(-sum, r0, 1.0), r0, r0);
        const double eps = ea * rs * 1.0001;
        const double ab = acc[r];
        if (fabs(delta) <= B.rmax && t <= 2e-3 && sum >= 1e-280 && ab >= 1e-290 && eps <= 1e-6) {
            // s = (log acc_b + shift_b) - (log S + shift_a): one log of the
            // ratio; the fp64 round's own logs, shifts and (LGMM) - y terms
            // add at most mag 2^-50 (fp64_err), mag from the exponents
            const double lq = flog(ab / sum);
            s[r] = lq + (L.shift_b - L.shift_a);
            const double mag = (double)(abs(ilogb(ab)) + abs(ilogb(sum)) + 2) * 0.6931471805599453 +
                               fabs(L.shift_b) + fabs(L.shift_a) + 2.0 * fabs(y[r]) + fabs(L.centre);
            E[r] = 1.25 * (1.001 * eps + 0x1.0p-52 * (fabs(lq) + 1.0) + fp64_err(L.nb + L.na, mag));
        }
    }
    return nterms;
}

// Every candidate of the workgroup whose upper bound hv reaches the
// workgroup's best lower bound bk (every one the round's best lower bound
// can select is among them) is appended to the cell's list (idx, hi) with one
// atomic per workgroup; bk goes to lbkey[cell], the terms to *terms.  Every
// thread of the workgroup must call it.
template <int R>
__device__ __forceinline__ void bx_append(const double (&hv)[R], const bool (&valid)[R],
                                          const int64_t (&ci)[R], uint64_t bk, int nterms, size_t cell,
                                          int64_t stride, double* __restrict__ hi,
                                          unsigned long long* __restrict__ lbkey, int32_t* __restrict__ cnt,
                                          int32_t* __restrict__ idx, unsigned long long* __restrict__ terms) {
    __shared__ uint64_t sh[kBlock / 64];
    bk = block_max_key(bk, sh);
    if (threadIdx.x == 0 && bk) atomicMax(lbkey + cell, bk);
    bool take[R];
    int mine = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        take[r] = valid[r] && order_key(hv[r]) >= bk;
        mine += take[r];
    }
    __shared__ int shc[kBlock / 64], shb;
    int tw = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(tw, off);
        if ((threadIdx.x & 63) >= off) tw += o;
    }
    if ((threadIdx.x & 63) == 63) shc[threadIdx.x >> 6] = tw;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += shc[w];
        shb = tot ? atomicAdd(cnt + cell, tot) : 0;
    }
    __syncthreads();
    int at = shb + tw - mine;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) at += shc[w];
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (take[r]) {
            idx[cell * (size_t)stride + at] = (int32_t)ci[r];
            hi[cell * (size_t)stride + at] = hv[r];
            ++at;
        }
    __shared__ int shn[kBlock / 64];
    int t = nterms;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if ((threadIdx.x & 63) == 0) shn[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0 && terms) {
        unsigned long long tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += (unsigned long long)shn[w];
        atomicAdd(terms, tot);
    }
    __syncthreads();   // the LDS above may be reused by the caller's next pass
}

// upper bound of a certified candidate (+inf otherwise); bk: the largest
// order key of a certified lower bound
template <int R>
__device__ __forceinline__ void bx_bounds(const double (&s)[R], const double (&E)[R], const bool (&valid)[R],
                                          double (&hv)[R], uint64_t& bk) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        hv[r] = __builtin_inf();
        if (valid[r] && E[r] <= 1e30 && s[r] == s[r]) {
            hv[r] = s[r] + E[r];
            const uint64_t k = order_key(s[r] - E[r]);
            bk = k > bk ? k : bk;
        }
    }
}

// The expansion screen over every candidate of the round (drawn here), or
// (SAMPLE = false) over caller-supplied candidates -> s_out / e_out.  lohi:
// packed map, (lower, upper) per candidate, picked per round.
template <int R, bool SAMPLE>
__global__ __launch_bounds__(kBlock) void k_screen_bx(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp,
    const BxLabel* __restrict__ bx, const double* __restrict__ tab, const int32_t* __restrict__ loff,
    const int32_t* __restrict__ list, int64_t n, int64_t cand_offset, uint64_t seed,
    const uint32_t* __restrict__ rounds, int32_t nl, double* __restrict__ hi,
    unsigned long long* __restrict__ lbkey, int32_t* __restrict__ cnt, int32_t* __restrict__ idx,
    unsigned long long* __restrict__ terms,
    int32_t* __restrict__ err, Slots S, const double* __restrict__ cand_in,
    double* __restrict__ s_out, double* __restrict__ e_out, double2* __restrict__ lohi, int64_t stride) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const BxLabel B = bx[li];
    __shared__ double exp_tab[kExpTabSize];
    __shared__ SampLds sl;
    load_exp_table(exp_tab);
    const bool staged = SAMPLE && stage_samp(L, samp, &sl);
    const bool lgmm = L.mode == DENSE_LGMM;
    double x[R];
    int64_t z[R], ci[R], gi[R];
    bool valid[R];
    draw_slots<DENSE_ANY, SAMPLE, R>(L, S, lgmm, samp, cand_in, n, cand_offset, seed, rounds, err,
                                     x, z, ci, gi, valid, staged ? &sl : nullptr);
    double s[R], E[R];
    const int nterms = bx_score<R>(L, B, comps64, tab, loff, list, exp_tab, x, valid, s, E);
    if constexpr (!SAMPLE) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (valid[r]) {
                s_out[ci[r]] = s[r];
                e_out[ci[r]] = E[r];
            }
        return;
    } else {
        if (lohi) {   // packed map: (lower, upper) per candidate; one atomic per wave
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!valid[r]) continue;
                const bool cert = E[r] <= 1e30 && s[r] == s[r];
                lohi[((size_t)blockIdx.y * S.n_rounds + z[r]) * n + ci[r]] =
                    cert ? make_double2(s[r] - E[r], s[r] + E[r])
                         : make_double2(-__builtin_inf(), __builtin_inf());
            }
            int t = nterms;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
            if ((threadIdx.x & 63) == 0 && terms) atomicAdd(terms, (unsigned long long)t);
            return;
        }
        double hv[R];
        uint64_t bk = 0;
        bx_bounds<R>(s, E, valid, hv, bk);
        bx_append<R>(hv, valid, ci, bk, nterms, (size_t)blockIdx.z * nl + blockIdx.y, stride, hi, lbkey, cnt, idx,
                     terms);
    }
}

// ------------------------------------------------------ hot-bin prefilter ----
// (tpe_device.h "hot-bin prefilter")  tau0 per label position: over runs
// of 1, 2, 4, .. kHotRun consecutive sub-bins whose sampling mass reaches
// pmin together (a candidate lands in the run with near certainty, and then
// its L is at least the run's smallest), the largest smallest L (0 = no
// such run: every candidate is listed).  grid (blocks of 256 sub-bins strided,
// dense labels), one run start per thread, atomicMax into tau0 (zeroed).
constexpr int kHotRun = 32;
constexpr int64_t kHotPrepWgs = (int64_t)1 << 30;   // k_hot_tau0 / k_hot_bits: workgroups over the labels, at most
// (2048 measured 30 -> 34 us for k_hot_tau0 at config 3, r6x)
__global__ __launch_bounds__(kBlock) void k_hot_tau0(const int32_t* __restrict__ group,
                                                     const BxLabel* __restrict__ bx,
                                                     const float2* __restrict__ sb,
                                                     const float* __restrict__ sbp, float pmin,
                                                     unsigned long long* __restrict__ tau0) {
    const BxLabel B = bx[group[blockIdx.y]];
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    // per block of the label (strided over the grid when it is capped) its
    // sub-bins and the kHotRun after them, staged in LDS with coalesced
    // loads (a run walked in global memory was one dependent load per step)
    __shared__ float tp[kBlock + kHotRun], tl[kBlock + kHotRun];
    uint64_t k = 0;
    for (int64_t j0 = (int64_t)blockIdx.x * kBlock; j0 < nsb; j0 += (int64_t)gridDim.x * kBlock) {
        __syncthreads();   // (the previous block's reads)
        for (int t = threadIdx.x; t < kBlock + kHotRun; t += kBlock)
            if (j0 + t < nsb) {
                tp[t] = sbp[B.sb_off + j0 + t];
                tl[t] = sb[B.sb_off + j0 + t].y;
            }
        __syncthreads();
        const int64_t j = j0 + threadIdx.x;
        if (j < nsb) {
            float p = 0.0f, lmin = __builtin_inff();
            for (int w = 0; w < kHotRun && j + w < nsb; ++w) {
                p += tp[threadIdx.x + w];
                lmin = fminf(lmin, tl[threadIdx.x + w]);
                if (p >= pmin) {
                    const uint64_t v = order_key((double)lmin);
                    k = v > k ? v : k;
                    break;
                }
            }
        }
    }
    __shared__ uint64_t sh[kBlock / 64];
    k = block_max_key(k, sh);
    if (threadIdx.x == 0 && k) atomicMax(tau0 + blockIdx.y, k);
}


// per label position: bit j of the label's words = (order key of U_j >=
// tau0); grid (blocks of 256 sub-bins strided, dense labels), one sub-bin per
// thread (coalesced), a wave's 64 bits written as two words
__global__ __launch_bounds__(kBlock) void k_hot_bits(const int32_t* __restrict__ group,
                                                     const BxLabel* __restrict__ bx,
                                                     const float2* __restrict__ sb,
                                                     const unsigned long long* __restrict__ tau0,
                                                     uint32_t* __restrict__ hbits) {
    const BxLabel B = bx[group[blockIdx.y]];
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    const uint64_t t0 = tau0[blockIdx.y];
    const int lane = threadIdx.x & 63;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j - lane < nsb; j += (int64_t)gridDim.x * kBlock) {
        const int64_t jw = j - lane;   // the wave's first sub-bin (a multiple of 64; the loop wave-uniform)
        const bool set = j < nsb && order_key((double)sb[B.sb_off + j].x) >= t0;
        const uint64_t m = __ballot(set);
        if (lane == 0) hbits[(B.sb_off >> 5) + (jw >> 5)] = (uint32_t)m;
        if (lane == 32 && jw + 32 < nsb) hbits[(B.sb_off >> 5) + (jw >> 5) + 1] = (uint32_t)(m >> 32);
    }
}

// Draw every candidate of the round (the same draws as k_screen_bx) and
// test its sub-bin's bit (U >= tau0, k_hot_bits: 4 KB per label at config 3,
// staged in LDS when it fits): the candidates whose bit is set (and those
// outside the sub-bins) are listed with their draw -- (hidx, hx)[cell
// hstride + position], hcnt[cell].  The largest L of the cell is taken over
// the LISTED candidates (k_screen_hot): a candidate left out has L <= U <
// tau0, so the cell's largest L reaches tau0 iff a listed candidate's does.
//
// Most candidates are decided from their Philox words alone (round 6): the
// draw is x = mu_k + ssg_k Phi^-1(p0_k + m_k v), monotone in v = (wu + r)
// 2^-32 within the picked component k, so each component's uniform is cut
// into kHotCells u-cells (the top bits of wu) and a cell is marked
// (k_hot_ucells, once per posterior and n) when the x-range of its v-range
// can touch a set bit or leave the bins.  A candidate in an unmarked cell
// cannot be listed; the others (~1 %) go to a mark list per cell and are
// drawn in fp64 by k_hot_draw (icdf_draw, the exact draw of every kernel)
// and tested against the sub-bin bits -- so the list is exactly the one the
// full draw gives.
constexpr int kHotCellBits = 11;
constexpr int kHotCells = 1 << kHotCellBits;   // u-cells per sampling component
constexpr int kHotCellWords = kHotCells / 32;

// per dense label position: stage_samp's LDS table written out (the draw
// kernels copy it instead of rebuilding it per workgroup)
__global__ __launch_bounds__(kBlock) void k_samp_image(const DLabel* __restrict__ labels,
                                                       const int32_t* __restrict__ group,
                                                       const SampRec* __restrict__ samp, uint4* __restrict__ img) {
    __shared__ SampLds sl;
    (void)stage_samp(labels[group[blockIdx.x]], samp, &sl);   // (launched for ns <= kSampLds only)
    const uint4* s = reinterpret_cast<const uint4*>(&sl);
    for (int k = threadIdx.x; k < kSampImgVec; k += kBlock) img[(size_t)blockIdx.x * kSampImgVec + k] = s[k];
}

// per dense label position: the set bits of the label's sub-bin words
// before each word (exclusive prefix), one workgroup per label
__global__ __launch_bounds__(1024) void k_hot_prefix(const int32_t* __restrict__ group,
                                                     const BxLabel* __restrict__ bx,
                                                     const uint32_t* __restrict__ hbits,
                                                     int32_t* __restrict__ pc) {
    const BxLabel B = bx[group[blockIdx.x]];
    const int64_t nw = ((int64_t)B.nbins * kBxSub + 31) / 32;
    const uint32_t* wd = hbits + (B.sb_off >> 5);
    int32_t* out = pc + (B.sb_off >> 5);
    const int64_t per = (nw + 1023) / 1024;
    const int64_t w0 = (int64_t)threadIdx.x * per, w1 = min(nw, w0 + per);
    int32_t v = 0;
    for (int64_t w = w0; w < w1; ++w) v += __popc(wd[w]);
    __shared__ int32_t wsum[16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int32_t run = x - v;
    for (int u = 0; u < wv; ++u) run += wsum[u];
    for (int64_t w = w0; w < w1; ++w) {
        out[w] = run;
        run += __popc(wd[w]);
    }
}

// the x an edge of u-cells meets: v = e / kHotCells exactly (1 - v too),
// then icdf_draw's own arithmetic (p, q, z, x, the clamp); p or q = 0 at an
// unbounded tail: -inf / +inf
__device__ __forceinline__ double hot_edge_x(const DLabel& L, const DrawComp& c, int e) {
    const double v = (double)e * (1.0 / kHotCells), vb = (double)(kHotCells - e) * (1.0 / kHotCells);
    const double p = fma(c.m, v, c.p0), q = fma(c.m, vb, c.q0);
    double z;
    if (p <= 0.5) z = p > 0.0 ? ndtri_lower(p) : -__builtin_inf();
    else z = q > 0.0 ? -ndtri_lower(q) : __builtin_inf();
    double x = fma(c.ssg, z, c.mu);
    if ((L.flags & 3) == 3) {
        x = x < L.low ? L.low : x;
        x = x >= L.high ? nextafter(L.high, -__builtin_inf()) : x;
    }
    return x;
}

// set bits of the label's words at sub-bins < j (prefix pc)
__device__ __forceinline__ int64_t hot_bits_before(const uint32_t* __restrict__ wd, const int32_t* __restrict__ pc,
                                                   int64_t j) {
    const int64_t w = j >> 5;
    const int b = (int)(j & 31);
    return (int64_t)pc[w] + __popc(wd[w] & ((1u << b) - 1u));
}

// The u-cells of every sampling component of every dense label: bit c of
// component k is set when some v in [c, c + 1) / kHotCells can draw x (any
// r, with the rounding of the draw and of the candidate's sub-bin index:
// ~1e-12 relative of slack) into a sub-bin whose bit is set, or outside the
// bins.  Grid (kHotCells / 256, kSampLds, dense labels); layout
// ucell[((y kSampLds + k) kHotCellWords + word].
__global__ __launch_bounds__(kBlock) void k_hot_ucells(const DLabel* __restrict__ labels,
                                                       const int32_t* __restrict__ group,
                                                       const SampRec* __restrict__ samp,
                                                       const BxLabel* __restrict__ bx,
                                                       const uint32_t* __restrict__ hbits,
                                                       const int32_t* __restrict__ pc,
                                                       uint32_t* __restrict__ ucell) {
    const int li = group[blockIdx.z];
    const DLabel L = labels[li];
    const int k = blockIdx.y;
    if (k >= L.ns) return;   // (the whole workgroup)
    const BxLabel B = bx[li];
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    const SampRec r = samp[L.samp_off + k];
    DrawComp c{};
    c.mu = r.mu;
    c.ssg = r.ssg;
    c.p0 = r.p0;
    c.q0 = r.q0;
    c.m = r.m;
    const int cell = (int)blockIdx.x * kBlock + (int)threadIdx.x;
    bool hot = true;
    if (c.m > 0.0) {
        const double x0 = hot_edge_x(L, c, cell), x1 = hot_edge_x(L, c, cell + 1);
        const double xa = fmin(x0, x1), xb = fmax(x0, x1);
        if (xa == xa && xb == xb && fabs(xa) < __builtin_inf() && fabs(xb) < __builtin_inf()) {
            const double slop = 1e-12 * (fabs(c.mu) + fabs(xa - c.mu) + fabs(xb - c.mu) + fabs(c.ssg));
            double f0 = (xa - slop - L.centre - B.xlo) * B.inv_sbw;
            double f1 = (xb + slop - L.centre - B.xlo) * B.inv_sbw;
            f0 -= 1e-6 + 1e-12 * fabs(f0);
            f1 += 1e-6 + 1e-12 * fabs(f1);
            if (f0 >= 0.0 && f1 < (double)nsb) {
                const int64_t j0 = (int64_t)f0, j1 = (int64_t)f1;
                const uint32_t* wd = hbits + (B.sb_off >> 5);
                const int32_t* pp = pc + (B.sb_off >> 5);
                const int64_t n1 = hot_bits_before(wd, pp, j1) + ((wd[j1 >> 5] >> (j1 & 31)) & 1u);
                hot = n1 - hot_bits_before(wd, pp, j0) > 0;
            }
        }
    }
    const uint64_t m = __ballot(hot);
    const int lane = threadIdx.x & 63;
    uint32_t* o = ucell + ((size_t)blockIdx.z * kSampLds + k) * kHotCellWords + (cell >> 5);
    if (lane == 0) o[0] = (uint32_t)m;
    if (lane == 32) o[0] = (uint32_t)(m >> 32);
}

// the work items of k_screen_hot: per cell ceil(min(count, stride) / per)
// passes of `per` listed candidates, pre[c] their exclusive prefix (pre[cells]
// = the total), *next (its item counter) zeroed; every thread of a B-thread
// workgroup calls it
template <int B>
__device__ __forceinline__ void hot_items_body(const int32_t* __restrict__ hcnt, int64_t cells, int64_t hstride,
                                               int64_t per, int32_t* __restrict__ pre, int32_t* __restrict__ next) {
    __shared__ int32_t wsum[B / 64];
    __shared__ int32_t carry;
    if (threadIdx.x == 0) {
        carry = 0;
        *next = 0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t c0 = 0; c0 < cells; c0 += B) {
        const int64_t c = c0 + threadIdx.x;
        int32_t v = 0;
        if (c < cells) v = (int32_t)((min((int64_t)hcnt[c], hstride) + per - 1) / per);
        int32_t x = v;   // inclusive scan over the wave
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int32_t wp = carry;
        for (int u = 0; u < w; ++u) wp += wsum[u];
        if (c < cells) pre[c] = wp + x - v;
        __syncthreads();   // (carry and wsum read by every thread)
        if (threadIdx.x == B - 1) carry = wp + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) pre[cells] = carry;
}

// The draw kernel, in two launches (round 6).  k_hot_bx (tile map only:
// workgroups stride over the cell's tiles of R * 256 candidates, Philox
// pairs per thread, the label's staged sampling table (k_samp_image) and
// u-cells copied once per workgroup): per candidate the Philox words, the
// component pick and one u-cell bit; the marked candidates' indices (~0.8 %,
// r6h) gather in a buffer per WAVE in LDS and go to the workgroup's own
// segment of the mark list (an LDS counter: no global atomics -- a counter
// per cell shared by every workgroup serialised the flushes, r6i).  No fp64
// in it: ~54 VGPRs, 8 waves per SIMD.  k_hot_draw then draws the marked
// candidates by the inverse CDF in fp64 and lists those whose sub-bin's bit
// is set (or that fall outside the bins) -- exactly the list the full draw
// gives.
constexpr int kMarkBuf = 128;     // marked indices per wave

template <int R>
__global__ __launch_bounds__(kBlock, 8) void k_hot_bx(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group, const uint4* __restrict__ img,
    const uint32_t* __restrict__ ucell, int64_t n, int64_t cand_offset, uint64_t seed,
    const uint32_t* __restrict__ rounds, int32_t nl, int32_t* __restrict__ mseg, int32_t* __restrict__ midx,
    int64_t mcap, int32_t* __restrict__ hflag) {
    static_assert(R % 2 == 0, "Philox pairs");
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    __shared__ SampLds sl;
    extern __shared__ uint32_t ucw[];   // (dynamic: the largest label's ns x kHotCellWords)
    __shared__ int32_t buf[kBlock / 64][kMarkBuf];
    __shared__ int32_t wg_n;
    {
        const uint32_t* uc = ucell + (size_t)blockIdx.y * kSampLds * kHotCellWords;
        for (int w = threadIdx.x; w < L.ns * kHotCellWords; w += kBlock) ucw[w] = uc[w];
        if (threadIdx.x == 0) wg_n = 0;
    }
    stage_samp_image(img + (size_t)blockIdx.y * kSampImgVec, &sl);   // (its barrier publishes the stage above)
    const size_t cell = (size_t)blockIdx.z * nl + blockIdx.y;
    const size_t seg = cell * gridDim.x + blockIdx.x;
    int32_t* __restrict__ out = midx + seg * (size_t)mcap;
    const uint32_t rk = rounds[blockIdx.z];
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    constexpr int64_t per = (int64_t)R * kBlock;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const SampShared src{&sl, __builtin_amdgcn_readfirstlane(sl.steps)};
    // one wave's buffered indices (count c, wave-uniform) to the segment;
    // past mcap it overflows: hflag bit 2 (below)
    auto flush = [&](int c) {
        int gb = 0;
        if (lane == 0) gb = atomicAdd(&wg_n, c);
        gb = __builtin_amdgcn_readfirstlane(__shfl(gb, 0));
        __builtin_amdgcn_wave_barrier();
        for (int k = lane; k < c; k += 64)
            if (gb + k < mcap) out[gb + k] = buf[wv][k];
        __builtin_amdgcn_wave_barrier();
    };
    int wn = 0;   // this wave's buffered indices (wave-uniform)
    // the tile loop, its guided pick's step count (uniform over the
    // workgroup: the label's) a compile-time constant -- the candidates'
    // pick chains then interleave, without a branch per step
    auto tiles = [&](auto st_c) {
        constexpr int ST = decltype(st_c)::value;
        for (int64_t base = (int64_t)blockIdx.x * per; base < n; base += (int64_t)gridDim.x * per) {
            const uint32_t g0 = (uint32_t)(cand_offset + base);
            const bool paired = (g0 & 1u) == 0;   // (uniform)
            // the tile's words, picks and u-cell bits for all R slots at once
            // (independent chains: their LDS lookups overlap)
            uint32_t wp[R], wu[R];
            if (paired) {   // (one uniform branch per tile: the pairs' chains interleave)
#pragma unroll
                for (int r = 0; r < R; r += 2) {
                    const uint32_t c0 = tile_cand(r, threadIdx.x, kBlock);
                    const U4 W = philox4x32_10(U4{(g0 + c0) >> 1, 0u, (uint32_t)L.stream, rk}, k0, k1);
                    wp[r] = W.x;
                    wu[r] = W.y;
                    wp[r + 1] = W.z;
                    wu[r + 1] = W.w;
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; r += 2) {
                    const uint32_t c0 = tile_cand(r, threadIdx.x, kBlock);
                    draw_words(L, k0, k1, g0 + c0, rk, wp[r], wu[r]);
                    draw_words(L, k0, k1, g0 + c0 + 1u, rk, wp[r + 1], wu[r + 1]);
                }
            }
            uint32_t mark = 0;
            auto mark_one = [&](int r) {
                int k;
                if constexpr (ST >= 0) {   // the guided pick with its step count fixed: no branch per step
                    k = sl.gd[wp[r] >> 24];
#pragma unroll
                    for (int t = 0; t < ST; ++t) k += sl.thr1[k] < wp[r] ? 1 : 0;
                } else {
                    k = src.pick_index(wp[r]);
                }
                const uint32_t uc = wu[r] >> (32 - kHotCellBits);
                return (bool)((ucw[k * kHotCellWords + (uc >> 5)] >> (uc & 31)) & 1u);
            };
            if (base + per <= n) {   // (uniform: a whole tile, no range check per candidate)
#pragma unroll
                for (int r = 0; r < R; ++r) mark |= (uint32_t)mark_one(r) << r;
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    mark |= (uint32_t)(base + (int64_t)tile_cand(r, threadIdx.x, kBlock) < n && mark_one(r)) << r;
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const bool m = (mark >> r) & 1u;
                const uint64_t bal = __ballot(m);
                if (!bal) continue;
                const int c = (int)__popcll(bal);
                if (wn + c > kMarkBuf) {   // (wave-uniform)
                    flush(wn);
                    wn = 0;
                }
                if (m) buf[wv][wn + (int)lanes_below(bal)] = (int32_t)(base + (int64_t)tile_cand(r, threadIdx.x, kBlock));
                wn += c;
            }
        }
    };
    switch (src.steps) {
    case 0: tiles(std::integral_constant<int, 0>{}); break;
    case 1: tiles(std::integral_constant<int, 1>{}); break;
    case 2: tiles(std::integral_constant<int, 2>{}); break;
    case 3: tiles(std::integral_constant<int, 3>{}); break;
    default: tiles(std::integral_constant<int, -1>{}); break;
    }
    if (wn > 0) flush(wn);
    __syncthreads();
    if (threadIdx.x == 0) {
        mseg[seg] = wg_n;
        if (wg_n > mcap) atomicOr(hflag, 2);
    }
}

// The marked candidates of every (round, dense label) cell: the words
// again (one Philox call each), the inverse-CDF draw in fp64 and the sub-bin
// test; listed ones -- bit set, or outside the bins (or NaN) -- gather in
// LDS and go to the cell's hot list (hidx, hx) with one global atomic per
// workgroup (per kDrawBuf listed).  Grid (workgroups per cell, cells): each
// workgroup takes a contiguous run of the cell's mark segments and numbers
// their entries flat (full lanes).
constexpr int kDrawBuf = 1024;
constexpr int kDrawSegs = 64;     // mark segments per k_hot_draw workgroup, at most
__global__ __launch_bounds__(kBlock) void k_hot_draw(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group, const uint4* __restrict__ img,
    const BxLabel* __restrict__ bx, const uint32_t* __restrict__ hbits, int64_t cand_offset, uint64_t seed,
    const uint32_t* __restrict__ rounds, int32_t nl, const int32_t* __restrict__ mseg, int32_t nseg,
    const int32_t* __restrict__ midx, int64_t mcap, int32_t* __restrict__ hcnt, int32_t* __restrict__ hidx,
    double* __restrict__ hx, int32_t* __restrict__ err, int64_t hstride, int32_t* __restrict__ hflag) {
    const size_t cell = blockIdx.y;
    const int li = group[cell % (size_t)nl];
    const DLabel L = labels[li];
    const BxLabel B = bx[li];
    __shared__ SampLds sl;
    __shared__ int32_t lidx[kDrawBuf];
    __shared__ double lx[kDrawBuf];
    __shared__ int32_t ln, lbase;
    if (threadIdx.x == 0) ln = 0;
    stage_samp_image(img + (cell % (size_t)nl) * kSampImgVec, &sl);
    const SampShared src{&sl, __builtin_amdgcn_readfirstlane(sl.steps)};
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    const uint32_t* __restrict__ gbits = hbits + (B.sb_off >> 5);
    const uint32_t rk = rounds[cell / (size_t)nl];
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const int lane = threadIdx.x & 63;
    // the buffered entries to the cell's list (every thread; uniform)
    auto flush = [&]() {
        __syncthreads();
        const int c = ln;
        if (threadIdx.x == 0) {
            lbase = atomicAdd(hcnt + cell, c);
            if (lbase + c > hstride) atomicOr(hflag, 2);   // (the round screens every candidate instead)
        }
        __syncthreads();
        const int64_t b = lbase;
        for (int k = threadIdx.x; k < c; k += kBlock)
            if (b + k < hstride) {
                hidx[cell * (size_t)hstride + b + k] = lidx[k];
                hx[cell * (size_t)hstride + b + k] = lx[k];
            }
        __syncthreads();
        if (threadIdx.x == 0) ln = 0;
        __syncthreads();
    };
    // this workgroup's mark segments [s0, s1) of the cell, numbered flat
    // (full lanes: a segment holds ~100-300 marks)
    __shared__ int32_t spre[kDrawSegs + 1];
    const int s0 = (int)((int64_t)blockIdx.x * nseg / gridDim.x);
    const int s1 = (int)((int64_t)(blockIdx.x + 1) * nseg / gridDim.x);   // (s1 - s0 <= kDrawSegs: the launch)
    if (threadIdx.x == 0) {
        int32_t t = 0;
        for (int k = s0; k < s1; ++k) {
            spre[k - s0] = t;
            t += (int32_t)min((int64_t)mseg[cell * (size_t)nseg + k], mcap);
        }
        spre[s1 - s0] = t;
    }
    __syncthreads();
    const int32_t total = spre[s1 - s0];
    bool bad = false;
    for (int32_t j0 = 0; j0 < total; j0 += kBlock) {
        if (ln > kDrawBuf - kBlock) flush();   // (ln read by every thread after a barrier: uniform)
        const int32_t j = j0 + (int32_t)threadIdx.x;
        bool take = false;
        int32_t ci = 0;
        double x = 0.0;
        if (j < total) {
            int k = 0;
            while (spre[k + 1] <= j) ++k;   // (the segment holding flat entry j)
            ci = midx[(cell * (size_t)nseg + s0 + k) * (size_t)mcap + (j - spre[k])];
            uint32_t wp, wu;
            draw_words(L, k0, k1, (uint32_t)(cand_offset + ci), rk, wp, wu);
            x = icdf_draw(L, src.comp(wp), wp, wu);
            bad = bad || x != x;
            const double f = (x - L.centre - B.xlo) * B.inv_sbw;
            if (f >= 0.0 && f < (double)nsb) {
                const int64_t sb = (int64_t)f;
                take = (gbits[sb >> 5] >> (sb & 31)) & 1u;
            } else {
                take = true;   // outside the bins (or NaN): always listed
            }
        }
        const uint64_t bal = __ballot(take);
        if (bal) {
            int gb = 0;
            if (lane == 0) gb = atomicAdd(&ln, (int)__popcll(bal));
            gb = __builtin_amdgcn_readfirstlane(__shfl(gb, 0));
            if (take) {
                const int at = gb + (int)lanes_below(bal);
                lidx[at] = ci;
                lx[at] = x;
            }
        }
        __syncthreads();   // (ln settled before the next chunk's check)
    }
    flush();
    if (bad) atomicOr(err, 1);
}

// k_screen_hot's work items numbered from the hot lists' counts (one
// workgroup).  A launch of its own: the last-workgroup pattern in
// k_hot_draw cost every workgroup a device-scope release + acquire -- an L2
// write-back and invalidate each (r6m: 2046 of them, 76 us for a shard's
// ~0.5M draws)
__global__ __launch_bounds__(1024) void k_hot_items(const int32_t* __restrict__ hcnt, int64_t cells, int64_t hstride,
                                                   int64_t per, int32_t* __restrict__ items) {
    hot_items_body<1024>(hcnt, cells, hstride, per, items, items + cells + 1);
}


// The expansion screen over the listed candidates only, one pass of R * 256
// listed candidates per work item (numbered by k_hot_items): one workgroup
// per item, the grid the most items the lists can hold (the ones past the
// round's items exit at once).  Round 4-6's persistent grid took items from
// a counter and staged the exp table once per workgroup, but its loop let
// the compiler hoist ~80 VGPRs of per-thread addresses out of it: 192 VGPRs,
// two waves per SIMD, against 111 and four without the loop (r6ad).  The
// same scores, bounds and appends as k_screen_bx (the passes are the same
// R * 256-aligned slices of each cell's list).
template <int R>
__global__ __launch_bounds__(kBlock) void k_screen_hot(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const BxLabel* __restrict__ bx, const double* __restrict__ tab,
    const int32_t* __restrict__ loff, const int32_t* __restrict__ list, int64_t n, int32_t nl, int64_t cells,
    const int32_t* __restrict__ pre, int32_t* __restrict__ next,
    const int32_t* __restrict__ hcnt, const int32_t* __restrict__ hidx, const double* __restrict__ hx,
    double* __restrict__ hi, unsigned long long* __restrict__ lbkey, int32_t* __restrict__ cnt,
    int32_t* __restrict__ idx, unsigned long long* __restrict__ terms, const float2* __restrict__ sb,
    unsigned long long* __restrict__ tkey, int64_t hstride) {
    constexpr int64_t per = (int64_t)R * kBlock;
    __shared__ double exp_tab[kExpTabSize];
    __shared__ uint64_t shk[kBlock / 64];
    const int32_t total = pre[cells];
    const int32_t item = (int32_t)blockIdx.x;
    if (item >= total) return;   // (uniform: a workgroup past the items stages nothing)
    load_exp_table(exp_tab);
    // the item's cell: the last c with pre[c] <= item (empty cells share
    // their successor's start)
    int64_t lo = 0, up = cells;
    while (up - lo > 1) {
        const int64_t mid = (lo + up) >> 1;
        if (pre[mid] <= item) lo = mid; else up = mid;
    }
    const size_t cell = (size_t)__builtin_amdgcn_readfirstlane((int)lo);   // (uniform: scalar loads below)
    const int64_t m = min((int64_t)hcnt[cell], hstride);   // (an overflowed list falls back anyway)
    const int64_t j0 = (int64_t)(item - pre[cell]) * per;
    const int li = __builtin_amdgcn_readfirstlane(group[cell % (size_t)nl]);
    const DLabel L = labels[li];
    const BxLabel B = bx[li];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int64_t nsb = (int64_t)B.nbins * kBxSub;
    uint64_t kl = 0;   // the largest sub-bin L of the listed candidates
    double x[R];
    int64_t ci[R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = j0 + r * kBlock + threadIdx.x;
        valid[r] = j < m;
        const double d = valid[r] ? hx[cell * (size_t)hstride + j] : 0.0;   // the raw draw
        x[r] = lgmm ? lgmm_value(d) : d;
        ci[r] = valid[r] ? hidx[cell * (size_t)hstride + j] : 0;
        const double f = (d - L.centre - B.xlo) * B.inv_sbw;   // k_hot_bx's sub-bin
        if (valid[r] && f >= 0.0 && f < (double)nsb) {
            const uint64_t k = order_key((double)sb[B.sb_off + (int64_t)f].y);
            kl = k > kl ? k : kl;
        }
    }
    double s[R], E[R], hv[R];
    const int nterms = bx_score<R>(L, B, comps64, tab, loff, list, exp_tab, x, valid, s, E);
    uint64_t bk = 0;
    bx_bounds<R>(s, E, valid, hv, bk);
    bx_append<R>(hv, valid, ci, bk, nterms, cell, hstride, hi, lbkey, cnt, idx, terms);
    kl = block_max_key(kl, shk);
    if (threadIdx.x == 0 && kl) atomicMax(tkey + cell, kl);
}

// tpe_hot_probe: the sub-bin (U, L) of caller-supplied candidates of one
// label, read exactly as k_hot_bx reads them
__global__ __launch_bounds__(kBlock) void k_hot_probe(const DLabel* __restrict__ labels,
                                                      const BxLabel* __restrict__ bx,
                                                      const float2* __restrict__ sb,
                                                      const float* __restrict__ sbp, int32_t label,
                                                      const double* __restrict__ cand, int64_t n,
                                                      double* __restrict__ u_out, double* __restrict__ l_out,
                                                      double* __restrict__ p_out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const DLabel L = labels[label];
    const BxLabel B = bx[label];
    const double y = L.mode == DENSE_LGMM ? flog(cand[i]) : cand[i];
    const double f = (y - L.centre - B.xlo) * B.inv_sbw;
    double u = __builtin_inf(), l = -__builtin_inf(), pm = 0.0;
    if (f >= 0.0 && f < (double)((int64_t)B.nbins * kBxSub)) {
        const float2 v = sb[B.sb_off + (int64_t)f];
        u = v.x;
        l = v.y;
        pm = sbp[B.sb_off + (int64_t)f];
    }
    u_out[i] = u;
    l_out[i] = l;
    p_out[i] = pm;
}


// Each workgroup owns a contiguous slice of its (round, label) row: it
// counts its takers, reserves their places with ONE atomic (a per-wave
// atomic on the row's counter serialised ~1.3M same-address atomics at
// config 3: 12.5 ms), then writes them.
// The windowed screen (tpe_window.hip) leaves hi in sorted order: vmap (the
// unit of rounds from z0 on and labels from position y0 on, nl_unit of them)
// gives each sorted position's candidate index.
template <typename H>
__global__ __launch_bounds__(kBlock) void k_select(const H* __restrict__ hi, int64_t n, int32_t nl,
                                                   const unsigned long long* __restrict__ lbkey,
                                                   int32_t* __restrict__ cnt, int32_t* __restrict__ idx,
                                                   int32_t z0, int32_t y0, int32_t nl_unit,
                                                   const uint64_t* __restrict__ vmap) {
    const size_t cell = (size_t)(z0 + blockIdx.z) * nl + y0 + blockIdx.y;
    const size_t row = cell * (size_t)n;
    const uint64_t* vrow =
        vmap ? vmap + ((size_t)blockIdx.z * nl_unit + blockIdx.y) * (size_t)n : nullptr;
    const uint64_t lb = lbkey[cell];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t span = ((n + gridDim.x - 1) / gridDim.x + kBlock - 1) / kBlock * kBlock;
    const int64_t lo = (int64_t)blockIdx.x * span, hi_end = min(n, lo + span);
    int mine = 0;   // this wave's takers (lane 0's copy is authoritative)
    for (int64_t i0 = lo; i0 < hi_end; i0 += kBlock) {
        const int64_t i = i0 + threadIdx.x;
        const bool take = i < hi_end && order_key((double)hi[row + i]) >= lb;
        mine += (int)__popcll(__ballot(take));
    }
    __shared__ int wcount[kBlock / 64], wbase[kBlock / 64];
    if (lane == 0) wcount[wave] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += wcount[w];
        int base = tot ? atomicAdd(cnt + cell, tot) : 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            wbase[w] = base;
            base += wcount[w];
        }
    }
    __syncthreads();
    if (!wcount[wave]) return;   // wave-uniform; no barrier below
    int at = wbase[wave];
    for (int64_t i0 = lo; i0 < hi_end; i0 += kBlock) {
        const int64_t i = i0 + threadIdx.x;
        const bool take = i < hi_end && order_key((double)hi[row + i]) >= lb;
        const uint64_t m = __ballot(take);
        if (take)
            idx[row + at + __popcll(m & ((1ull << lane) - 1ull))] =
                vrow ? (int32_t)(uint32_t)vrow[i] : (int32_t)i;
        at += (int)__popcll(m);
    }
}

// empty partials for the rows (round blockIdx.z, label group[blockIdx.y])

// One workgroup per kRescoreR * 256 re-scored candidates of one (round,
// label) (chunk table from the host: cell = round * nl + label position);
// each writes its block maxloc to res[chunk], and k_rescore_merge keeps
// each cell's best.  Sized after the counts are read back, so the hardware
// scheduler balances the chunks over the chip.
using RescoreChunk = tpe_rt::RescoreChunkH;

// candidates per thread in k_rescore: config 3 re-scores ~24k candidates
// per (round, label), ~3k workgroups at 2 per thread (4: 3.75 ms at ~2
// workgroups per CU)
#ifndef TPE_RESCORE_R
#define TPE_RESCORE_R 2
#endif
constexpr int kRescoreR = TPE_RESCORE_R;
// at most this many candidates to re-score in a round: split by slices
constexpr int64_t kSlicedRescoreMax = 1 << 16;
constexpr int kRsW = 64;   // candidates per sliced re-score entry (one per lane)

// candidates per thread in k_screen (its own tile width): the component's
// m shared by more candidates costs fewer v_mov_b64 per eval
#ifndef TPE_SCREEN_R
#define TPE_SCREEN_R 8
#endif
constexpr int kScreenR = TPE_SCREEN_R;

// candidates per thread in k_screen_bx (the below mixture's records shared
// by R candidates; the above part is per candidate)
#ifndef TPE_BX_R
#define TPE_BX_R 4
#endif
constexpr int kBxR = TPE_BX_R;

// candidates per thread and tile in k_hot_bx (Philox words, pick and u-cell
// bit each), and the workgroups per cell striding over the listed
// candidates in k_screen_hot
#ifndef TPE_HOT_R
#define TPE_HOT_R 8
#endif
constexpr int kHotR = TPE_HOT_R;
#ifndef TPE_HOT_WGS
#define TPE_HOT_WGS 16384
#endif
constexpr int64_t kHotWgs = TPE_HOT_WGS;
#ifndef TPE_HOT_BX_WGS
#define TPE_HOT_BX_WGS 8192   // (the two draw kernels: 2048 0.54 ms, 4096 0.52, 8192 0.48, r6j)
#endif
constexpr int64_t kHotBxWgs = TPE_HOT_BX_WGS;   // k_hot_bx's workgroups over a round, at most
constexpr int64_t kHotFillWgs = 2560;           //   at least (two passes of the resident workgroups)
constexpr int64_t kHotMinTiles = 6;             //   tiles per workgroup, at least (unless filling)
#ifndef TPE_HOT_DRAW_WGS
#define TPE_HOT_DRAW_WGS 2048
#endif
constexpr int64_t kHotDrawWgs = TPE_HOT_DRAW_WGS;   // k_hot_draw's workgroups over a round, about
constexpr int kQR = 8;   // candidates per thread, k_qfused_tiles
constexpr int kQLdsKeys = 1024;   // grid values whose keys k_qfused_tiles stages in LDS
constexpr int kCatR = 8;  // candidates per thread, k_cat_tiles

// The re-score's work table, built on the device from the cells' counts --
// no read-back in the middle of a round (the mid-round sync was
// fixed latency of every round).  total = the sum of the counts; the
// re-score is `sliced` (one wave per kRsW candidates and summation slice)
// when total <= kSlicedRescoreMax, otherwise chunks of `per_full` candidates
// per workgroup (packed map: always chunks).  Per cell: its range of entries
// (first << 32 | count) and the offset of its candidates in the cell order
// (eoff[cells] = total); the entries {cell, j} in cell order.  One workgroup
// of kPlanBlock threads; the re-score kernels read `plan` and stride over
// its entries with grids sized for the largest table.
using RescorePlan = tpe_rt::RescorePlanH;
constexpr int kPlanBlock = 1024;
// (every thread of a B-thread workgroup calls it)
template <int B>
__device__ __forceinline__ void rescore_plan_body(const int32_t* __restrict__ cnt, int64_t cells, int32_t per_full,
                                                  int64_t sliced_max, int64_t cap, RescoreChunk* __restrict__ chunks,
                                                  int64_t* __restrict__ range, int64_t* __restrict__ eoff,
                                                  RescorePlan* __restrict__ plan) {
    constexpr int kPlanBlock = B;
    constexpr int W = kPlanBlock / 64;
    __shared__ int64_t wsum[W];
    __shared__ int64_t tot_sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t t = 0;
    for (int64_t c = threadIdx.x; c < cells; c += kPlanBlock) t += cnt[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) wsum[wave] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t a = 0;
        for (int w = 0; w < W; ++w) a += wsum[w];
        tot_sh = a;
    }
    __syncthreads();
    const int64_t total = tot_sh;
    if (total > cap) {   // more than the buffers hold: no entries, the host re-runs the round
        if (threadIdx.x == 0) *plan = RescorePlan{total, 0, 0, 1, 0};
        return;
    }
    const bool sliced = sliced_max > 0 && total <= sliced_max;
    const int64_t per = sliced ? (int64_t)kRsW : (int64_t)per_full;
    int64_t carry = 0, ecarry = 0;   // entries and candidates before this block of cells
    for (int64_t c0 = 0; c0 < cells; c0 += kPlanBlock) {
        __syncthreads();   // (wsum reuse)
        const int64_t c = c0 + threadIdx.x;
        const int64_t k = c < cells ? (int64_t)cnt[c] : 0;
        const int64_t nc = (k + per - 1) / per;
        // inclusive scans of (entries, candidates) over the block
        int64_t se = nc, sk = k;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t oe = __shfl_up(se, o), ok = __shfl_up(sk, o);
            if (lane >= o) {
                se += oe;
                sk += ok;
            }
        }
        __shared__ int64_t wk[W];
        if (lane == 63) {
            wsum[wave] = se;
            wk[wave] = sk;
        }
        __syncthreads();
        int64_t be = 0, bk = 0, te = 0, tk = 0;
        for (int w = 0; w < W; ++w) {
            if (w < wave) {
                be += wsum[w];
                bk += wk[w];
            }
            te += wsum[w];
            tk += wk[w];
        }
        if (c < cells) {
            const int64_t first = carry + be + se - nc;
            range[c] = (first << 32) | nc;
            if (eoff) eoff[c] = ecarry + bk + sk - k;
            for (int64_t j = 0; j < nc; ++j) chunks[first + j] = RescoreChunk{(int32_t)c, (int32_t)j};
        }
        carry += te;
        ecarry += tk;
    }
    if (threadIdx.x == 0) {
        if (eoff) eoff[cells] = ecarry;
        *plan = RescorePlan{total, (int32_t)carry, sliced ? 1 : 0, 0, 0};
    }
}

// The expansion screen's per-cell lists (candidate index, upper bound) hold
// every candidate whose bound reached its workgroup's best lower bound;
// keep those that reach the cell's (the round's) best, compacted in place.
// One workgroup per cell; chunks in order, so writes never pass reads.
// Fused into the same launch (round 6: two launches fewer on every round's
// critical path): the hot-bin prefilter's check of the cell (tkey: its
// largest listed L against tau0 -> the fallback flag; nullptr without the
// prefilter), and, by the workgroup that finishes last (done: a counter the
// round's fills zero), the re-score plan over every cell's count.
__global__ __launch_bounds__(kBlock) void k_select_plan(const double* __restrict__ hi, int64_t stride,
                                                        const unsigned long long* __restrict__ lbkey,
                                                        int32_t* __restrict__ cnt, int32_t* __restrict__ idx,
                                                        const unsigned long long* __restrict__ tkey,
                                                        const unsigned long long* __restrict__ tau0, int32_t nl,
                                                        int32_t* __restrict__ hflag, uint32_t* __restrict__ done,
                                                        int32_t per_full, int64_t sliced_max, int64_t cap,
                                                        RescoreChunk* __restrict__ chunks,
                                                        int64_t* __restrict__ range, RescorePlan* __restrict__ plan) {
    const size_t cell = blockIdx.x;
    const uint64_t lb = lbkey[cell];
    const int len = cnt[cell];
    int32_t* il = idx + cell * (size_t)stride;
    const double* hl = hi + cell * (size_t)stride;
    __shared__ int shc[kBlock / 64];
    __shared__ bool last;
    int out = 0;
    for (int j0 = 0; j0 < len; j0 += kBlock) {
        const int j = j0 + threadIdx.x;
        const bool keep = j < len && order_key(hl[j]) >= lb;
        const int32_t v = j < len ? il[j] : 0;
        const uint64_t m = __ballot(keep);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0) shc[wave] = __popcll(m);
        __syncthreads();   // every read of this chunk is done
        int at = out + __popcll(m & ((1ull << lane) - 1ull));
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            if (w < wave) at += shc[w];
            tot += shc[w];
        }
        if (keep) il[at] = v;
        out += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        cnt[cell] = out;
        if (tkey && tkey[cell] < tau0[cell % (size_t)nl]) atomicOr(hflag, 1);
        __threadfence();   // (the count and the list before the counter)
        last = atomicAdd(done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;   // (uniform)
    __threadfence();     // (acquire: every cell's count and list)
    rescore_plan_body<kBlock>(cnt, (int64_t)gridDim.x, per_full, sliced_max, cap, chunks, range, nullptr, plan);
}

__global__ __launch_bounds__(kPlanBlock) void k_rescore_plan(const int32_t* __restrict__ cnt, int64_t cells,
                                                             int32_t per_full, int64_t sliced_max, int64_t cap,
                                                             RescoreChunk* __restrict__ chunks,
                                                             int64_t* __restrict__ range, int64_t* __restrict__ eoff,
                                                             RescorePlan* __restrict__ plan) {
    rescore_plan_body<kPlanBlock>(cnt, cells, per_full, sliced_max, cap, chunks, range, eoff, plan);
}

template <int R>
__global__ __launch_bounds__(kBlock) void k_rescore(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp, int64_t stride,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, int32_t nl,
    int32_t n_labels, int32_t tiles, const int32_t* __restrict__ cnt, const int32_t* __restrict__ idx,
    const RescoreChunk* __restrict__ chunks, const RescorePlan* __restrict__ plan, Partial* __restrict__ res) {
    if (plan->sliced) return;   // (uniform: the sliced kernels take this round)
    const int32_t ne = plan->ne;
    if ((int32_t)blockIdx.x >= ne) return;
    __shared__ double exp_tab[kExpTabSize];
    load_exp_table(exp_tab);
    for (int32_t e = blockIdx.x; e < ne; e += gridDim.x) {
    const RescoreChunk ch = chunks[e];
    const int32_t z = ch.cell / nl, y = ch.cell % nl;
    const int li = group[y];
    const int64_t count = cnt[ch.cell];
    constexpr int64_t per = (int64_t)R * kBlock;
    const int64_t base = (int64_t)ch.j * per;
    const DLabel L = labels[li];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int32_t* list = idx + (size_t)ch.cell * (size_t)stride;
    const uint32_t rk = rounds[z];
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
    double bv = 0.0, bl = 0.0, ba = 0.0;
    double x[R], yv[R], lb[R], la[R];
    int64_t gi[R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = base + r * kBlock + threadIdx.x;
        valid[r] = j < count;
        gi[r] = cand_offset + (valid[r] ? list[j] : 0);
        double v = lgmm ? 1.0 : 0.0;
        if (valid[r]) {
            if (lgmm) (void)sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rk, (uint32_t)gi[r], v);
            else (void)sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rk, (uint32_t)gi[r], v);
        }
        x[r] = v;
        yv[r] = lgmm ? flog(v) : v;
    }
    lse_dense<R>(comps64 + L.comp_b, L.nb, L.shift_b, L.centre, yv, lb, exp_tab);
    lse_dense<R>(comps64 + L.comp_a, L.na, L.shift_a, L.centre, yv, la, exp_tab);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (lgmm) {
            lb[r] -= yv[r];
            la[r] -= yv[r];
        }
        if (!valid[r]) continue;
        const uint64_t key = order_key(lb[r] - la[r]);
        if (better(key, gi[r], bk, bi)) {
            bk = key;
            bi = gi[r];
            bv = x[r];
            bl = lb[r];
            ba = la[r];
        }
    }
    __shared__ Partial sh[kBlock / 64];
    block_maxloc(bk, bi, bv, bl, ba, res + e, sh);
    __syncthreads();   // (sh is read by thread 0 before the next entry writes it)
    (void)z;
    }
}

// The re-score of a few candidates per (round, dense label) -- the
// expansion screen leaves a handful of near-ties -- split by summation
// slices so it fills the chip instead of one wave per label walking 10k
// components: k_rescore_slices re-draws an entry's candidates and sums one
// kSumSlice slice of one mixture for the 64 candidates of the entry per
// wave, and k_rescore_fin adds the slices in
// order (lse_acc's order: the bits of the fp64 round) and keeps the entry's
// best.  Entry = RescoreChunk{cell, j}: candidates [64 j, 64 j + 64) of the
// cell's list.  part: [entry][s_max slices][64].  The entries come from
// k_rescore_plan; the kernels stride over them (grids sized for the largest
// table) and leave a round whose plan is not sliced to k_rescore.

// acc + p[0] + p[stride] + ... + p[(n-1) stride], added in that order, the
// loads issued 8 at a time (the slice sums of a sliced re-score: one
// dependent L2 round trip per slice took ~50 us for 200 slices, r5ag)
__device__ __forceinline__ double ordered_sum(const double* __restrict__ p, int n, size_t stride, double acc) {
    int s = 0;
    for (; s + 8 <= n; s += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(s + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; s < n; ++s) acc += p[(size_t)s * stride];
    return acc;
}

// The entry's candidate of this lane (the round's draw, re-drawn from its
// index): value and global index, NaN / -1 past the cell's count
__device__ __forceinline__ void rescore_cand(const DLabel& L, const SampRec* __restrict__ samp, int64_t stride,
                                             int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds,
                                             int32_t nl, const int32_t* __restrict__ cnt,
                                             const int32_t* __restrict__ idx, const RescoreChunk& ch, int lane,
                                             double& v, int64_t& g) {
    const int32_t z = ch.cell / nl;
    const int64_t j = (int64_t)ch.j * kRsW + lane;
    v = __builtin_nan("");
    g = -1;
    if (j < cnt[ch.cell]) {
        g = cand_offset + idx[(size_t)ch.cell * (size_t)stride + j];
        if (L.mode == DENSE_LGMM) (void)sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rounds[z], (uint32_t)g, v);
        else (void)sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rounds[z], (uint32_t)g, v);
    }
}

// One wave per (entry of kRsW candidates, summation slice): each wave
// re-draws its entry's candidates (round 6: the draw kernel before it was a
// launch of its own) and sums its slice in order; the first slice's wave
// also stores the candidates for k_rescore_fin.  Grid (slice groups,
// entries strided).
__global__ __launch_bounds__(kBlock) void k_rescore_slices(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp, int64_t stride,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, int32_t nl,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ idx, const RescoreChunk* __restrict__ chunks,
    const RescorePlan* __restrict__ plan, double* __restrict__ xbuf, int64_t* __restrict__ gbuf, int32_t s_max,
    double* __restrict__ part) {
    if (!plan->sliced) return;
    const int32_t ne = plan->ne;
    if ((int32_t)blockIdx.y >= ne) return;   // (uniform, before the table's barrier)
    __shared__ double exp_tab[kExpTabSize];
    load_exp_table(exp_tab);   // (every wave takes part before any leaves)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int e = blockIdx.y; e < ne; e += gridDim.y) {
    const RescoreChunk ch = chunks[e];
    const DLabel L = labels[group[ch.cell % nl]];
    const int nsb = (L.nb + kSumSlice - 1) / kSumSlice, nsa = (L.na + kSumSlice - 1) / kSumSlice;
    const int slice = blockIdx.x * (kBlock / 64) + wave;
    if (slice >= nsb + nsa) continue;   // (no barrier below)
    double x;
    int64_t g;
    rescore_cand(L, samp, stride, cand_offset, seed, rounds, nl, cnt, idx, ch, lane, x, g);
    if (slice == 0) {
        xbuf[(size_t)e * kRsW + lane] = x;
        gbuf[(size_t)e * kRsW + lane] = g;
    }
    const bool above = slice >= nsb;
    const int k0 = (above ? slice - nsb : slice) * kSumSlice;
    const int k1 = min(k0 + kSumSlice, above ? L.na : L.nb);
    const double xr[1] = {(L.mode == DENSE_LGMM ? flog(x) : x) - L.centre};
    double acc[1] = {0.0};
    lse_acc_run<1>(comps64 + (above ? L.comp_a : L.comp_b) + k0, k1 - k0, xr, acc, exp_tab);
    part[((size_t)e * s_max + slice) * kRsW + lane] = acc[0];
    }
}

// k_rescore_fin's workgroups: every one pays a device-scope release (an L2
// write-back) for the last-workgroup merge, and a round re-scores a few
// dozen entries (256 before round 6's measurements of that fence)
constexpr int64_t kRsFinWgs = 64;

// The re-score's end: per entry (one wave each, entries strided) the slice
// sums added in order, the logs and the entry's maxloc into res[entry];
// then the workgroup that finishes last (done: zeroed by the round's fills)
// keeps each (round, dense label) cell's best entry in the row's first
// partial slot -- an empty record when the cell listed nothing -- which is
// all k_reduce reads of a dense row on this path (round 6: k_rescore_merge
// and k_fill_empty were launches of their own).  The chunked re-score
// (k_rescore, a plan past kSlicedRescoreMax) runs before this kernel and
// leaves its entries' records in res too.
__global__ __launch_bounds__(kRsW) void k_rescore_fin(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, int32_t nl, const RescoreChunk* __restrict__ chunks,
    const RescorePlan* __restrict__ plan, const double* __restrict__ xbuf, const int64_t* __restrict__ gbuf,
    int32_t s_max, const double* __restrict__ part, Partial* __restrict__ res, uint32_t* __restrict__ done,
    int64_t cells, int32_t n_labels, int32_t tiles, const int64_t* __restrict__ range,
    Partial* __restrict__ partials) {
    const bool sliced = plan->sliced != 0;
    const int32_t ne = plan->ne;
    const int lane = threadIdx.x;
    for (int e = blockIdx.x; sliced && e < ne; e += gridDim.x) {
    const RescoreChunk ch = chunks[e];
    const DLabel L = labels[group[ch.cell % nl]];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int nsb = (L.nb + kSumSlice - 1) / kSumSlice, nsa = (L.na + kSumSlice - 1) / kSumSlice;
    const double x = xbuf[(size_t)e * kRsW + lane];
    const int64_t g = gbuf[(size_t)e * kRsW + lane];
    const double* p = part + (size_t)e * s_max * kRsW + lane;
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
    double bv = 0.0, bl = 0.0, ba = 0.0;
    if (g >= 0) {   // (padding lanes would take lse_finish's two-pass fallback)
        const double sb = ordered_sum(p, nsb, kRsW, 0.0);
        const double sa = ordered_sum(p + (size_t)nsb * kRsW, nsa, kRsW, 0.0);
        const double y = lgmm ? flog(x) : x;
        double lb = lse_finish(comps64 + L.comp_b, L.nb, sb, y - L.centre, L.shift_b);
        double la = lse_finish(comps64 + L.comp_a, L.na, sa, y - L.centre, L.shift_a);
        if (lgmm) {
            lb -= y;
            la -= y;
        }
        bk = order_key(lb - la);
        bi = g;
        bv = x;
        bl = lb;
        ba = la;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t ok = __shfl_xor(bk, off);
        const int64_t oi = __shfl_xor(bi, off);
        const double ov = __shfl_xor(bv, off), ol = __shfl_xor(bl, off), oa = __shfl_xor(ba, off);
        if (better(ok, oi, bk, bi)) {
            bk = ok;
            bi = oi;
            bv = ov;
            bl = ol;
            ba = oa;
        }
    }
    if (lane == 0) res[e] = Partial{bk, bi, bv, bl, ba};
    }
    __shared__ bool last;
    if (lane == 0) {
        __threadfence();   // (this workgroup's records before the counter)
        last = atomicAdd(done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;   // (uniform)
    __threadfence();     // (acquire: every entry's record)
    const bool over = plan->overflow != 0;   // (no table: every cell empty -- cannot happen on the tile map)
    for (int64_t c = lane; c < cells; c += kRsW) {
        const int64_t first = over ? 0 : range[c] >> 32, count = over ? 0 : range[c] & 0xffffffffll;
        Partial best{0, INT64_MAX, 0.0, 0.0, 0.0};
        for (int64_t j = 0; j < count; ++j)
            if (better(res[first + j].key, res[first + j].idx, best.key, best.idx)) best = res[first + j];
        const int64_t z = c / nl;
        partials[((size_t)z * n_labels + group[c % nl]) * tiles] = best;
    }
}

// ---------------------------------------- fp32 screen (packed map) ----
// Batched rounds with small C (config 5: 4096 new_ids x 24 candidates)
// keep their whole rounds inside one workgroup, so the screen needs no
// atomics for the bound: k_round_chunk<float> writes the fp32 sums (per
// chunk of the above mixture, as the fp64 chunked map does), k_pick_packed
// forms s32 and its bound per slot, takes the per-round largest lower
// bound in LDS and compacts the slots that can still win -- about one per
// (round, label) -- into a per-label list, with each round's [first, count)
// range; k_rescore_packed re-draws them and runs the fp64 arithmetic of the
// unscreened packed map (below sum, above sum chunk by chunk added in order,
// lse_finish), and k_pick_rounds keeps each round's best.  The winners and
// their lpdfs are those of the unscreened packed round, bit for bit.
struct RoundSel {
    int32_t first, count;
};

// entries per packed re-score block: kRP * 256 (a label's ~3k entries at
// config 5 leave less of the last block idle than with kR)
constexpr int kRP = 2;

template <int R>
__global__ __launch_bounds__(kBlock) void k_pick_packed(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group, int64_t n, int32_t nl,
    int32_t nch, int32_t chunk, const double* __restrict__ part, int32_t* __restrict__ cnt,
    int64_t* __restrict__ list, int64_t cap, RoundSel* __restrict__ rsel, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int gx = gridDim.x, bx = blockIdx.x, by = blockIdx.y;
    constexpr int NS = R * kBlock;
    __shared__ uint64_t lo_key[NS];
    __shared__ uint64_t hi_key[NS];
    __shared__ uint64_t round_lb[NS];
    __shared__ int16_t round_cnt[NS], round_first[NS];   // <= R * 256 slots per workgroup
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int64_t z, ci;
        bool valid;
        S.template at<R>(r, n, z, ci, valid);
        const int s = r * kBlock + threadIdx.x;
        const double x = part[chunk_plane(by, 0, nch, bx, gx, R) + s];
        const double sb = part[chunk_plane(by, 1, nch, bx, gx, R) + s];
        double sa = 0.0;
        for (int c = 0; c < nch; ++c) sa += part[chunk_plane(by, 2 + c, nch, bx, gx, R) + s];
        const double y = lgmm ? flog(x) : x;
        const double xr = y - L.centre;
        const float xf = (float)xr;
        const double X = fabs(xr), dx = fabs((double)xf - xr);
        const double lb = flog(sb) + L.shift_b, la = flog(sa) + L.shift_a;
        const double s32 = lb - la;
        const double E = 1.25 * (screen_err(L.amax_b, L.nb, L.nb, X, dx, (float)sb, (float)log2(sb)) +
                                 screen_err(L.amax_a, L.na, chunk, X, dx, (float)sa, (float)log2(sa)) +
                                 fp64_err(L.nb + L.na, fabs(lb) + fabs(la) + fabs(y)));
        const bool cert = valid && E <= 1e30 && s32 == s32;
        lo_key[s] = cert ? order_key(s32 - E) : 0ull;
        hi_key[s] = !valid ? 0ull : (cert ? order_key(s32 + E) : ~0ull);
    }
    __syncthreads();
    // one thread per round of this workgroup: its largest lower bound
    for (int t = threadIdx.x; t < S.rpb; t += kBlock) {
        uint64_t m = 0;
        for (int c = 0; c < S.cpack; ++c) m = lo_key[t * S.cpack + c] > m ? lo_key[t * S.cpack + c] : m;
        round_lb[t] = m;
        int k = 0;
        for (int c = 0; c < S.cpack; ++c) k += (hi_key[t * S.cpack + c] >= m && hi_key[t * S.cpack + c]);
        round_cnt[t] = k;
    }
    __syncthreads();
    __shared__ int base;
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int t = 0; t < S.rpb; ++t) {
            round_first[t] = (int16_t)tot;
            tot += round_cnt[t];
        }
        base = tot ? atomicAdd(cnt + by, tot) : 0;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < S.rpb; t += kBlock) {
        const int64_t z = (int64_t)bx * S.rpb + t;
        if (z >= S.n_rounds) continue;
        const uint64_t m = round_lb[t];
        int at = base + round_first[t];
        rsel[(size_t)z * nl + by] = RoundSel{at, round_cnt[t]};
        for (int c = 0; c < S.cpack; ++c) {
            const uint64_t h = hi_key[t * S.cpack + c];
            if (h && h >= m) list[(size_t)by * cap + at++] = (z << 32) | (int64_t)c;
        }
    }
}

// The windowed packed screen (tpe_window.hip) leaves each candidate's
// (lower, upper) score bound in lohi[y n_rounds C + z C + i]: one thread per
// (round, label) takes the round's largest lower bound and lists, in
// candidate order, the candidates whose upper bound reaches it -- the same
// list and per-round ranges k_pick_packed makes.
// value_only (TPE_OPT_VALUE_ONLY): a round whose selection is ONE candidate
// whose lower bound clears every other candidate's upper bound by at least
// kValueMargin (relative) is decided: it is the argmax under any fp64
// evaluation of the reference's formulas (the HIP round's, numpy's --
// rounding moves a score by ~1e-12 at most), so its lpdfs are not computed
// (rsel = {candidate, -1}; k_pick_rounds re-draws its value, lpdfs NaN).
constexpr double kValueMargin = 1e-9;
template <typename P2>
__global__ __launch_bounds__(kBlock) void k_pick_win(const P2* __restrict__ lohi, int32_t n_rounds,
                                                     int32_t C, int32_t* __restrict__ cnt,
                                                     int64_t* __restrict__ list, int64_t cap,
                                                     RoundSel* __restrict__ rsel, int32_t nl, int32_t value_only) {
    using V = decltype(lohi->x);
    const int y = blockIdx.y;
    const int64_t z = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool valid = z < n_rounds;
    const P2* row = lohi + ((size_t)y * n_rounds + (valid ? z : 0)) * C;
    V m = -(V)__builtin_inf();
    int k = 0, single = -1;
    if (valid) {
        for (int c = 0; c < C; ++c) m = row[c].x > m ? row[c].x : m;
        for (int c = 0; c < C; ++c) k += row[c].y >= m;
        if (value_only && k == 1) {
            double second = -__builtin_inf();
            int cs = -1;
            for (int c = 0; c < C; ++c) {
                if (row[c].y >= m) cs = c;
                else second = fmax(second, (double)row[c].y);
            }
            const double md = (double)m;
            if (md - second >= kValueMargin * fmax(1.0, fabs(md))) single = cs;   // (NaN: not decided)
        }
        if (single >= 0) k = 0;   // nothing to re-score
    }
    __shared__ int sh[kBlock / 64 + 1];
    // exclusive prefix of the counts over the workgroup's rounds
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int inc = k;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
    }
    if (lane == 63) sh[wave] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const int t = sh[w];
            sh[w] = tot;
            tot += t;
        }
        sh[kBlock / 64] = tot ? atomicAdd(cnt + y, tot) : 0;
    }
    __syncthreads();
    if (!valid) return;
    int at = sh[kBlock / 64] + sh[wave] + inc - k;
    if (single >= 0) {
        rsel[(size_t)z * nl + y] = RoundSel{single, -1};
        return;
    }
    rsel[(size_t)z * nl + y] = RoundSel{at, k};
    for (int c = 0; c < C; ++c)
        if (row[c].y >= m) list[(size_t)y * cap + at++] = (z << 32) | (int64_t)c;
}

// Re-score work item (label position, block j of kR * 256 entries) x chunk:
// blockIdx.y = c sums the above mixture's chunk c (c = 0 also the below
// mixture and the candidate) from zero -- the chunked map's own per-chunk
// sums -- into plane 2 + c (0: below, 1: x) at the entry's place off[y] + e
// of the compacted order; k_finish_rescore adds the chunks in order.
// Per dense label (grid.x = label position), over its above records in
// order.  A record's fp64 term can be nonzero only for x' in [lo, hi]
// (zero_reach, kZeroU); "wide" records (half-width above 1.5x the clipped
// sigma's: the prior and the sparse tails' components) are listed
// (zwide[comp_a + j], count zn[label]); over the others zhi[k] = the
// prefix max of hi, zlo[k] = the suffix min of lo (+-inf for wide records
// and records that are 0 everywhere).  For x' in [xa, xb] every nonzero
// term is a wide record or lies in [first k with zhi[k] >= xa, first k with
// zlo[k] > xb).  Thread t scans a contiguous segment; thread 0 scans the
// segment totals (once per posterior).
__device__ __forceinline__ void zero_reach(const Comp<double>& c, double& lo, double& hi) {
    const double t = c.c + kZeroU;
    if (t < 0.0) {   // 0 everywhere
        lo = __builtin_inf();
        hi = -__builtin_inf();
        return;
    }
    const double mu = c.mu / c.a, w = sqrt(t) / c.a;
    const double slack = 1e-9 * (fabs(mu) + w + 1.0);
    lo = mu - w - slack;
    hi = mu + w + slack;
    if (!(c.a > 0.0) || !(lo <= hi) || !(t >= 0.0)) {   // NaN / unusable: nonzero anywhere (a wide record)
        lo = -__builtin_inf();
        hi = __builtin_inf();
    }
}

constexpr int kZwBlock = 1024;
// (skipped when the round's device-planned re-score holds nothing: a
// value-only round that certified every cell needs no windows; the host
// marks them built only when the plan was not empty)
__global__ __launch_bounds__(kZwBlock) void k_zero_windows(const RescorePlan* __restrict__ plan,
                                                           const DLabel* __restrict__ labels,
                                                           const int32_t* __restrict__ group,
                                                           const Comp<double>* __restrict__ comps64,
                                                           double* __restrict__ zhi, double* __restrict__ zlo,
                                                           int32_t* __restrict__ zwide, int32_t* __restrict__ zn) {
    if (plan->total == 0 || plan->sliced) return;   // (uniform; the sliced re-score sums every slice)
    const int li = group[blockIdx.x];
    const DLabel L = labels[li];
    const Comp<double>* c = comps64 + L.comp_a;
    double* ph = zhi + L.comp_a;
    double* pl = zlo + L.comp_a;
    int32_t* pw = zwide + L.comp_a;
    const int n = L.na, seg = (n + kZwBlock - 1) / kZwBlock, tid = threadIdx.x;
    const int k0 = min(n, tid * seg), k1 = min(n, k0 + seg);
    __shared__ double sh[kZwBlock], sl[kZwBlock];
    __shared__ int32_t sw[kZwBlock];
    __shared__ double wmax;
    // the clipped sigma's half-width: the largest record scale a'
    double am = 0.0;
    for (int k = k0; k < k1; ++k) am = fmax(am, c[k].a);
    sh[tid] = am;
    __syncthreads();
    if (tid == 0) {
        double m = 0.0;
        for (int t = 0; t < kZwBlock; ++t) m = fmax(m, sh[t]);
        wmax = m > 0.0 ? 1.5 * sqrt(kZeroU) / m : __builtin_inf();
    }
    __syncthreads();
    const double W = wmax;
    auto reach = [&](int k, double& lo, double& hi) -> bool {   // true: wide
        zero_reach(c[k], lo, hi);
        const bool wide = hi - lo > 2.0 * W;   // (+inf - -inf: an unusable record is wide)
        if (wide) {
            lo = __builtin_inf();
            hi = -__builtin_inf();
        }
        return wide;
    };
    double mh = -__builtin_inf(), ml = __builtin_inf();
    int nw = 0;
    for (int k = k0; k < k1; ++k) {
        double lo, hi;
        nw += reach(k, lo, hi) ? 1 : 0;
        mh = fmax(mh, hi);
        ml = fmin(ml, lo);
    }
    sh[tid] = mh;
    sl[tid] = ml;
    sw[tid] = nw;
    __syncthreads();
    if (tid == 0) {   // exclusive prefix max / suffix min / prefix sum of the segments
        double run = -__builtin_inf();
        int cnt = 0;
        for (int t = 0; t < kZwBlock; ++t) {
            const double v = sh[t];
            sh[t] = run;
            run = fmax(run, v);
            const int w = sw[t];
            sw[t] = cnt;
            cnt += w;
        }
        zn[li] = cnt;
        run = __builtin_inf();
        for (int t = kZwBlock - 1; t >= 0; --t) {
            const double v = sl[t];
            sl[t] = run;
            run = fmin(run, v);
        }
    }
    __syncthreads();
    double run = sh[tid];
    int at = sw[tid];
    for (int k = k0; k < k1; ++k) {
        double lo, hi;
        if (reach(k, lo, hi)) pw[at++] = k;
        run = fmax(run, hi);
        ph[k] = run;
    }
    run = sl[tid];
    for (int k = k1 - 1; k >= k0; --k) {
        double lo, hi;
        (void)reach(k, lo, hi);
        run = fmin(run, lo);
        pl[k] = run;
    }
}

// lse_acc over components [k0, k1) of the label's above records c (slices
// from k0, as lse_acc(c + k0, k1 - k0)) summing only the narrow window [wlo,
// whi) and the wide records wide[0..nw) (sorted): every other term is
// exactly +0.0 at the wave's candidates, and skipping +0.0 terms and slice
// sums leaves every partial sum -- hence the result -- bit-identical.  All
// bounds wave-uniform.
template <int R>
__device__ __forceinline__ void lse_acc_zero_window(const Comp<double>* __restrict__ c, int k0, int k1, int wlo,
                                                    int whi, const int32_t* __restrict__ wide, int nw,
                                                    const double (&x)[R], double (&acc)[R],
                                                    const double* __restrict__ tab) {
    int p = 0;   // first wide record >= k0
    {
        int lo = 0, hi = nw;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (wide[mid] < k0) lo = mid + 1; else hi = mid;
        }
        p = lo;
    }
    for (int s = k0; s < k1; s += kSumSlice) {
        const int b = min(s + kSumSlice, k1);
        const int ra = max(s, wlo), rb = min(b, whi);
        const bool wide_here = p < nw && wide[p] < b;
        if (ra >= rb && !wide_here) continue;   // the slice sums to +0.0
        double part[R];
#pragma unroll
        for (int r = 0; r < R; ++r) part[r] = 0.0;
        for (; p < nw && wide[p] < min(b, wlo); ++p) lse_acc_run<R>(c + wide[p], 1, x, part, tab);
        if (ra < rb) lse_acc_run<R>(c + ra, rb - ra, x, part, tab);
        for (; p < nw && wide[p] < min(b, whi); ++p) {}   // (inside the window: summed above)
        for (; p < nw && wide[p] < b; ++p) lse_acc_run<R>(c + wide[p], 1, x, part, tab);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] += part[r];
    }
}

// first k in [0, n) with v[k] > t (strict) or >= t; v non-decreasing
__device__ __forceinline__ int first_above(const double* __restrict__ v, int n, double t, bool strict) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const bool past = strict ? v[mid] > t : v[mid] >= t;
        if (past) hi = mid; else lo = mid + 1;
    }
    return lo;
}

template <int R>
__global__ __launch_bounds__(kBlock) void k_rescore_packed(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, int32_t chunk,
    const int32_t* __restrict__ cnt, const int64_t* __restrict__ list, int64_t cap,
    const RescoreChunk* __restrict__ chunks, const int64_t* __restrict__ off, const RescorePlan* __restrict__ plan,
    int64_t total, double* __restrict__ planes, const double* __restrict__ zhi, const double* __restrict__ zlo,
    const int32_t* __restrict__ zwide, const int32_t* __restrict__ zn) {
    if (plan->overflow || plan->sliced) return;
    const int32_t ne = plan->ne;
    if ((int32_t)blockIdx.x >= ne) return;   // (uniform, before the table's barrier)
    __shared__ double exp_tab[kExpTabSize];
    load_exp_table(exp_tab);
    for (int32_t ei = blockIdx.x; ei < ne; ei += gridDim.x) {
    const RescoreChunk ch = chunks[ei];
    const int y = ch.cell, c = blockIdx.y;
    const DLabel L = labels[group[y]];
    const int64_t count = cnt[y];
    constexpr int64_t per = (int64_t)R * kBlock;
    const bool lgmm = L.mode == DENSE_LGMM;
    double x[R], xr[R], sb[R], sa[R];
    int64_t e[R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        e[r] = (int64_t)ch.j * per + r * kBlock + threadIdx.x;
        valid[r] = e[r] < count;
        const int64_t ent = valid[r] ? list[(size_t)y * cap + e[r]] : 0;
        const int64_t z = ent >> 32, i = ent & 0xffffffffll;
        double v = lgmm ? 1.0 : 0.0;
        if (valid[r]) {
            const uint32_t rk = rounds[z], gi = (uint32_t)(cand_offset + i);
            if (lgmm) (void)sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rk, gi, v);
            else (void)sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rk, gi, v);
        }
        x[r] = v;
        xr[r] = (lgmm ? flog(v) : v) - L.centre;
        sb[r] = 0.0;
        sa[r] = 0.0;
    }
    if (c == 0) lse_acc<R>(comps64 + L.comp_b, L.nb, xr, sb, exp_tab);
    const int k0 = min(c * chunk, L.na), k1 = min(k0 + chunk, L.na);
    if (zhi) {
        // the wave's candidates span [xa, xb]: the above records outside
        // the window have terms of exactly +0.0 at all of them
        double xa = __builtin_inf(), xb = -__builtin_inf();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (valid[r]) {
                xa = fmin(xa, xr[r]);
                xb = fmax(xb, xr[r]);
            }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            xa = fmin(xa, __shfl_xor(xa, o));
            xb = fmax(xb, __shfl_xor(xb, o));
        }
        if (!(xa <= xb)) {   // no valid lane (or NaN): the whole chunk, as lse_acc
            lse_acc<R>(comps64 + L.comp_a + k0, k1 - k0, xr, sa, exp_tab);
        } else {
            const int wlo = __builtin_amdgcn_readfirstlane(first_above(zhi + L.comp_a, L.na, xa, false));
            const int whi = __builtin_amdgcn_readfirstlane(first_above(zlo + L.comp_a, L.na, xb, true));
            lse_acc_zero_window<R>(comps64 + L.comp_a, k0, k1, wlo, whi, zwide + L.comp_a, zn[group[y]], xr,
                                   sa, exp_tab);
        }
    } else {
        lse_acc<R>(comps64 + L.comp_a + k0, k1 - k0, xr, sa, exp_tab);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!valid[r]) continue;
        const size_t g = (size_t)(off[y] + e[r]);
        if (c == 0) {
            planes[g] = sb[r];
            planes[(size_t)total + g] = x[r];
        }
        planes[(size_t)(2 + c) * total + g] = sa[r];
    }
    }
}

__global__ __launch_bounds__(kBlock) void k_finish_rescore(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, int64_t cand_offset, int32_t nch,
    const int32_t* __restrict__ cnt, const int64_t* __restrict__ list, int64_t cap,
    const RescoreChunk* __restrict__ chunks, const int64_t* __restrict__ off, const RescorePlan* __restrict__ plan,
    int64_t total, const double* __restrict__ planes, Partial* __restrict__ res) {
    if (plan->overflow || plan->sliced) return;
    const int32_t ne = plan->ne;
    for (int32_t ei = blockIdx.x; ei < ne; ei += gridDim.x) {
    const RescoreChunk ch = chunks[ei];
    const int y = ch.cell;
    const DLabel L = labels[group[y]];
    const bool lgmm = L.mode == DENSE_LGMM;
    constexpr int64_t per = (int64_t)kRP * kBlock;
    for (int r = 0; r < kRP; ++r) {
        const int64_t e = (int64_t)ch.j * per + r * kBlock + threadIdx.x;
        if (e >= cnt[y]) continue;
        const size_t g = (size_t)(off[y] + e);
        const double sb = planes[g], x = planes[(size_t)total + g];
        double sa = 0.0;
        for (int c = 0; c < nch; ++c) sa += planes[(size_t)(2 + c) * total + g];
        const double yv = lgmm ? flog(x) : x;
        double lb = lse_finish(comps64 + L.comp_b, L.nb, sb, yv - L.centre, L.shift_b);
        double la = lse_finish(comps64 + L.comp_a, L.na, sa, yv - L.centre, L.shift_a);
        if (lgmm) {
            lb -= yv;
            la -= yv;
        }
        const int64_t i = list[(size_t)y * cap + e] & 0xffffffffll;
        res[g] = Partial{order_key(lb - la), cand_offset + i, x, lb, la};
    }
    }
}

// The packed map's re-score of a few listed candidates (plan->sliced: at most
// TPE_OPT_PK_SLICED, 8192 by default).  k_rescore_packed gives each listed candidate one
// thread walking its chunk of the above mixture -- config 5 lists ~1
// candidate in some rounds, and that one thread's chain of ~7k dependent
// fp64 terms took 1.6 ms (r5ac).  Here one wave sums one kSumSlice slice for
// kRsW listed candidates of a label (entry {label, j}), in the packed map's
// order: the below mixture's slices from record 0, the above mixture's per
// chunk of `chunk` records (slices from the chunk's start, spc per chunk),
// each chunk's slice sums added in order and the chunk sums added in order
// (k_round_chunk / k_finish_chunks / k_rescore_packed: the same bits).
// Slices outside the wave's zero window are exactly +0.0 and skipped.
// part: [entry][s_max][kRsW], s_max = below slices + nch * spc.

__global__ __launch_bounds__(kBlock) void k_rescore_draw_packed(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group, const SampRec* __restrict__ samp,
    int64_t cand_offset, uint64_t seed, const uint32_t* __restrict__ rounds, const RescorePlan* __restrict__ plan,
    const int32_t* __restrict__ cnt, const int64_t* __restrict__ list, int64_t cap,
    const RescoreChunk* __restrict__ chunks, double* __restrict__ xbuf, int64_t* __restrict__ gbuf,
    const double* __restrict__ zhi, const double* __restrict__ zlo, int32_t* __restrict__ win) {
    if (plan->overflow || !plan->sliced) return;
    const int32_t ne = plan->ne;
    const int lane = threadIdx.x % kRsW;
    for (int e = blockIdx.x * (kBlock / kRsW) + threadIdx.x / kRsW; e < ne; e += gridDim.x * (kBlock / kRsW)) {
    const RescoreChunk ch = chunks[e];
    const DLabel L = labels[group[ch.cell]];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int64_t j = (int64_t)ch.j * kRsW + lane;
    double v = lgmm ? 1.0 : 0.0;
    int64_t g = -1;
    if (j < cnt[ch.cell]) {
        const int64_t ent = list[(size_t)ch.cell * cap + j];
        const uint32_t rk = rounds[ent >> 32], gi = (uint32_t)(cand_offset + (ent & 0xffffffffll));
        if (lgmm) (void)sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rk, gi, v);
        else (void)sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rk, gi, v);
        g = j;
    }
    xbuf[(size_t)e * kRsW + lane] = v;
    gbuf[(size_t)e * kRsW + lane] = g;
    if (zhi) {
        // the entry's zero window (the posterior's windows built by an
        // earlier round): the above records whose terms can be nonzero at
        // some candidate of the entry
        const double xr = (lgmm ? flog(v) : v) - L.centre;
        double xa = g >= 0 ? xr : __builtin_inf(), xb = g >= 0 ? xr : -__builtin_inf();
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            xa = fmin(xa, __shfl_xor(xa, o));
            xb = fmax(xb, __shfl_xor(xb, o));
        }
        if (lane == 0) {
            const bool any = xa <= xb;
            win[2 * e] = any ? first_above(zhi + L.comp_a, L.na, xa, false) : 0;
            win[2 * e + 1] = any ? first_above(zlo + L.comp_a, L.na, xb, true) : L.na;
        }
    }
    }
}

__global__ __launch_bounds__(kBlock) void k_rescore_slices_packed(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group, const Comp<double>* __restrict__ comps64,
    const RescoreChunk* __restrict__ chunks, const RescorePlan* __restrict__ plan, const double* __restrict__ xbuf,
    int32_t s_max, int32_t chunk, int32_t spc, double* __restrict__ part, const int32_t* __restrict__ win,
    const int32_t* __restrict__ zwide, const int32_t* __restrict__ zn) {
    if (plan->overflow || !plan->sliced) return;
    const int32_t ne = plan->ne;
    if ((int32_t)blockIdx.y >= ne) return;   // (uniform, before the table's barrier)
    __shared__ double exp_tab[kExpTabSize];
    load_exp_table(exp_tab);   // (every wave takes part before any leaves)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slice = blockIdx.x * (kBlock / 64) + wave;
    if (slice >= s_max) return;   // (no barrier below)
    for (int e = blockIdx.y; e < ne; e += gridDim.y) {
    const RescoreChunk ch = chunks[e];
    const DLabel L = labels[group[ch.cell]];
    const int nsb = (L.nb + kSumSlice - 1) / kSumSlice;
    const double x = xbuf[(size_t)e * kRsW + lane];
    const double xr[1] = {(L.mode == DENSE_LGMM ? flog(x) : x) - L.centre};
    double acc[1] = {0.0};
    if (slice < nsb) {
        const int k0 = slice * kSumSlice, k1 = min(k0 + kSumSlice, L.nb);
        lse_acc_run<1>(comps64 + L.comp_b + k0, k1 - k0, xr, acc, exp_tab);
    } else {
        const int s = slice - nsb, c = s / spc;
        const int kb = min((c + 1) * chunk, L.na);
        const int k0 = c * chunk + (s - c * spc) * kSumSlice, k1 = min(k0 + kSumSlice, kb);
        if (k0 < k1) {
            if (win) {
                const int wlo = __builtin_amdgcn_readfirstlane(win[2 * e]);
                const int whi = __builtin_amdgcn_readfirstlane(win[2 * e + 1]);
                lse_acc_zero_window<1>(comps64 + L.comp_a, k0, k1, wlo, whi, zwide + L.comp_a,
                                       zn[group[ch.cell]], xr, acc, exp_tab);
            } else {
                lse_acc_run<1>(comps64 + L.comp_a + k0, k1 - k0, xr, acc, exp_tab);
            }
        }
    }
    part[((size_t)e * s_max + slice) * kRsW + lane] = acc[0];
    }
}

__global__ __launch_bounds__(kRsW) void k_rescore_fin_packed(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group, const Comp<double>* __restrict__ comps64,
    int64_t cand_offset, int32_t nch, int32_t spc, const int64_t* __restrict__ list, int64_t cap,
    const RescoreChunk* __restrict__ chunks, const int64_t* __restrict__ off, const RescorePlan* __restrict__ plan,
    const double* __restrict__ xbuf, const int64_t* __restrict__ gbuf, int32_t s_max,
    const double* __restrict__ part, Partial* __restrict__ res) {
    if (plan->overflow || !plan->sliced) return;
    const int32_t ne = plan->ne;
    const int lane = threadIdx.x;
    for (int e = blockIdx.x; e < ne; e += gridDim.x) {
    const RescoreChunk ch = chunks[e];
    const int y = ch.cell;
    const DLabel L = labels[group[y]];
    const bool lgmm = L.mode == DENSE_LGMM;
    const int64_t j = gbuf[(size_t)e * kRsW + lane];
    if (j < 0) continue;
    const int nsb = (L.nb + kSumSlice - 1) / kSumSlice;
    const double x = xbuf[(size_t)e * kRsW + lane];
    const double* p = part + (size_t)e * s_max * kRsW + lane;
    const double sb = ordered_sum(p, nsb, kRsW, 0.0);
    double sa = 0.0;
    for (int c = 0; c < nch; ++c) sa += ordered_sum(p + (size_t)(nsb + c * spc) * kRsW, spc, kRsW, 0.0);
    const double yv = lgmm ? flog(x) : x;
    double lb = lse_finish(comps64 + L.comp_b, L.nb, sb, yv - L.centre, L.shift_b);
    double la = lse_finish(comps64 + L.comp_a, L.na, sa, yv - L.centre, L.shift_a);
    if (lgmm) {
        lb -= yv;
        la -= yv;
    }
    const int64_t i = list[(size_t)y * cap + j] & 0xffffffffll;
    res[off[y] + j] = Partial{order_key(lb - la), cand_offset + i, x, lb, la};
    }
}

// one thread per (round, dense label): the best re-scored candidate of the
// round (its entries are in candidate order) -> the round's partial
// (a value-only cell, rs.count = -1: its one candidate rs.first is re-drawn,
// its lpdfs left NaN)
__global__ __launch_bounds__(kBlock) void k_pick_rounds(const DLabel* __restrict__ labels,
                                                        const int32_t* __restrict__ group, int32_t nl,
                                                        int32_t n_rounds, int32_t n_labels,
                                                        const RoundSel* __restrict__ rsel,
                                                        const Partial* __restrict__ res,
                                                        const int64_t* __restrict__ off,
                                                        const RescorePlan* __restrict__ plan,
                                                        const SampRec* __restrict__ samp, int64_t cand_offset,
                                                        uint64_t seed, const uint32_t* __restrict__ rounds,
                                                        Partial* __restrict__ partials) {
    const int64_t cell = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (cell >= (int64_t)n_rounds * nl || plan->overflow) return;
    const int64_t z = cell / nl;
    const int y = (int)(cell % nl);
    const RoundSel rs = rsel[cell];
    if (rs.count < 0) {
        const DLabel L = labels[group[y]];
        const uint32_t gi = (uint32_t)(cand_offset + rs.first);
        double v = 0.0;
        if (L.mode == DENSE_LGMM) (void)sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rounds[z], gi, v);
        else (void)sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rounds[z], gi, v);
        partials[(size_t)z * n_labels + group[y]] =
            Partial{order_key(0.0), cand_offset + rs.first, v, __builtin_nan(""), __builtin_nan("")};
        return;
    }
    Partial best{0, INT64_MAX, 0.0, 0.0, 0.0};
    for (int k = 0; k < rs.count; ++k) {
        const Partial& p = res[(size_t)(off[y] + rs.first + k)];
        if (better(p.key, p.idx, best.key, best.idx)) best = p;
    }
    partials[(size_t)z * n_labels + group[y]] = best;
}

// ------------------------------------------------------- split-K map ----
// Small candidate sets (tpe.suggest's default n_EI_candidates = 24, one
// round): one workgroup per label would walk all K components serially and
// leave the chip idle, so the component loop is split instead -- each wave
// sums one slice of kSlice components of one mixture for every candidate of
// the round (partial sums relative to the same LSE shift, or partial
// probabilities for quantized labels), and a finishing kernel adds the
// slices in order, takes the log and does the broadcast_best maxloc.
constexpr int kSlice = kSumSlice;   // dense (the fp64 sum order, tpe_device.h): ~12 VALU per component
constexpr int kSliceQ = 64;      // quantized: two erf per component
constexpr int kSliceWaves = kBlock / 64;

__host__ __device__ constexpr int slice_len(int mode) {
    return (mode == QUANT_GMM || mode == QUANT_LGMM) ? kSliceQ : kSlice;
}

// candidates of one (round, label): the same Philox draws as k_round / k_qsample
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_sample_small(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const SampRec* __restrict__ samp, int64_t n, int64_t cand_offset, uint64_t seed,
    const uint32_t* __restrict__ rounds, int32_t n_rounds, int32_t n_labels,
    double* __restrict__ xs, int32_t* __restrict__ err) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= (int64_t)n_rounds * n) return;
    const int64_t z = s / n, i = s - z * n;
    double v;
    bool ok;
    if constexpr (MODE == DENSE_ANY)
        ok = L.mode == DENSE_LGMM
                 ? sample_below<DENSE_LGMM>(L, samp + L.samp_off, seed, rounds[z], (uint32_t)(cand_offset + i), v)
                 : sample_below<DENSE_GMM>(L, samp + L.samp_off, seed, rounds[z], (uint32_t)(cand_offset + i), v);
    else
        ok = sample_below<MODE>(L, samp + L.samp_off, seed, rounds[z], (uint32_t)(cand_offset + i), v);
    if (!ok) atomicOr(err, 1);
    xs[((size_t)z * n_labels + li) * n + i] = v;
}

// one slice [k0, k1) of a mixture for candidate x (dense: sum of exp terms
// relative to the mixture's shift; quantized: partial probability)
template <typename T, int MODE>
__device__ __forceinline__ double slice_sum(const DLabel& L, const Comp<T>* __restrict__ c,
                                            const Comp<double>* __restrict__ c64, int k0, int k1,
                                            double x, const double* __restrict__ tab) {
    if constexpr (MODE == DENSE_GMM || MODE == DENSE_LGMM || MODE == DENSE_ANY) {
        const bool lgmm = MODE == DENSE_LGMM || (MODE == DENSE_ANY && L.mode == DENSE_LGMM);
        const double v = lgmm ? flog(x) : x;
        if constexpr (sizeof(T) == 8) {
            const double xr[1] = {v - L.centre};
            double acc[1] = {0.0};
            lse_acc<1>(c + k0, k1 - k0, xr, acc, tab);
            return acc[0];
        } else {
            const float xv[1] = {(float)(v - L.centre)};
            float acc[1];
            lse_acc<1>(c + k0, k1 - k0, xv, acc);
            return (double)acc[0];
        }
    } else {
#pragma clang fp contract(off)
        double ub, lb;
        bool neg;
        quant_bounds<MODE>(L, x, ub, lb, neg);
        double prob = 0.0;
        for (int k = k0; k < k1; ++k) {
            const double mu = c64[k].mu, a = c64[k].a, w = c64[k].w;
            double pu, pl;
            if (MODE == QUANT_LGMM) {
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
}

// grid (slice groups, labels, rounds); wave w of workgroup b takes slice
// b * kSliceWaves + w: below slices first, then above slices.
template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void k_score_slices(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<T>* __restrict__ comps, const Comp<double>* __restrict__ comps64, int64_t n,
    int32_t n_labels, int32_t s_max, const double* __restrict__ xs, double* __restrict__ part) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const int64_t z = blockIdx.z;
    constexpr bool kTab =
        (MODE == DENSE_GMM || MODE == DENSE_LGMM || MODE == DENSE_ANY) && sizeof(T) == 8;
    __shared__ double exp_tab[kTab ? kExpTabSize : 1];
    if constexpr (kTab) load_exp_table(exp_tab);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int S = slice_len(MODE);
    const int nsb = (L.nb + S - 1) / S, nsa = (L.na + S - 1) / S;
    const int slice = blockIdx.x * kSliceWaves + wave;
    if (slice >= nsb + nsa) return;
    const bool above = slice >= nsb;
    const int k0 = (above ? slice - nsb : slice) * S;
    const int k1 = min(k0 + S, above ? L.na : L.nb);
    const int64_t base = above ? L.comp_a : L.comp_b;
    const double* xrow = xs + ((size_t)z * n_labels + li) * n;
    double* prow = part + (((size_t)z * n_labels + li) * s_max + slice) * n;
    for (int64_t c = lane; c < n; c += 64)
        prow[c] = slice_sum<T, MODE>(L, comps + base, comps64 + base, k0, k1, xrow[c], exp_tab);
}

// per (label, round): add the slices in order, log / shift, broadcast_best
template <typename T, int MODE>
__global__ __launch_bounds__(kBlock) void k_finish_slices(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<T>* __restrict__ comps, int64_t n, int64_t cand_offset, int32_t n_labels,
    int32_t s_max, const double* __restrict__ xs, const double* __restrict__ part,
    Partial* __restrict__ partials, int32_t* __restrict__ err) {
    const int li = group[blockIdx.x];
    const DLabel L = labels[li];
    const int64_t z = blockIdx.y;
    constexpr int S = slice_len(MODE);
    const int nsb = (L.nb + S - 1) / S, nsa = (L.na + S - 1) / S;
    const double* xrow = xs + ((size_t)z * n_labels + li) * n;
    const double* prow = part + ((size_t)z * n_labels + li) * s_max * n;
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
    double bv = 0.0, bl = 0.0, ba = 0.0;
    // the slices of one mixture, added in order (loads issued 8 ahead)
    auto add_slices = [&](int s0, int ns, int64_t c) {
        double acc = 0.0;
        int s = 0;
        for (; s + 8 <= ns; s += 8) {
            double v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = prow[(size_t)(s0 + s + j) * n + c];
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += v[j];
        }
        for (; s < ns; ++s) acc += prow[(size_t)(s0 + s) * n + c];
        return acc;
    };
    for (int64_t c = threadIdx.x; c < n; c += kBlock) {
        const double x = xrow[c];
        const double sb = add_slices(0, nsb, c), sa = add_slices(nsb, nsa, c);
        double lb, la;
        if constexpr (MODE == DENSE_GMM || MODE == DENSE_LGMM || MODE == DENSE_ANY) {
            const bool lgmm = MODE == DENSE_LGMM || (MODE == DENSE_ANY && L.mode == DENSE_LGMM);
            const double y = lgmm ? flog(x) : x;
            if constexpr (sizeof(T) == 8) {
                lb = lse_finish(comps + L.comp_b, L.nb, sb, y - L.centre, L.shift_b);
                la = lse_finish(comps + L.comp_a, L.na, sa, y - L.centre, L.shift_a);
            } else {
                lb = lse_finish(comps + L.comp_b, L.nb, (float)sb, (float)(y - L.centre), L.shift_b);
                la = lse_finish(comps + L.comp_a, L.na, (float)sa, (float)(y - L.centre), L.shift_a);
            }
            if (lgmm) {
                lb -= y;
                la -= y;
            }
        } else {
            double ub, lo;
            bool neg;
            quant_bounds<MODE>(L, x, ub, lo, neg);
            if (neg) atomicOr(err, 2);
            lb = flog(sb) - L.logpacc_b;
            la = flog(sa) - L.logpacc_a;
        }
        const int64_t gi = cand_offset + c;
        const uint64_t key = order_key(lb - la);
        if (better(key, gi, bk, bi)) {
            bk = key;
            bi = gi;
            bv = x;
            bl = lb;
            ba = la;
        }
    }
    __shared__ Partial sh[kBlock / 64];
    block_maxloc(bk, bi, bv, bl, ba, partials + (size_t)z * n_labels + li, sh);
}

// Quantized families, pass 1: draw every candidate, keep its grid index
// j = rint(v / q) (so x = j * q exactly as np.round(v / q) * q), and the
// per-(round, label) min/max of j (order-preserving biased unsigned).
template <int MODE, int R>
__global__ __launch_bounds__(kBlock) void k_qsample(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const SampRec* __restrict__ samp, int64_t n, int64_t cand_offset, uint64_t seed,
    const uint32_t* __restrict__ rounds, int32_t nq, int32_t qbase, int64_t* __restrict__ qj,
    unsigned long long* __restrict__ qmin, unsigned long long* __restrict__ qmax,
    int32_t* __restrict__ err, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    // grid window of the label (all rounds of this launch share one table
    // window): thread -> wave -> workgroup, then one atomic pair per workgroup
    unsigned long long mn = ~0ull, mx = 0ull;
    int64_t zs[R], is[R];
    bool vs[R];
    uint32_t g32[R], rk[R], pend = 0;
    double xs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        S.template at<R>(r, n, zs[r], is[r], vs[r]);
        g32[r] = (uint32_t)(cand_offset + is[r]);
        rk[r] = vs[r] ? rounds[zs[r]] : 0u;
        xs[r] = 0.0;
        if (vs[r]) pend |= 1u << r;
    }
    __shared__ SampLds sl;
    bool ok;
    if (stage_samp(L, samp, &sl)) ok = sample_slots<MODE, R>(L, SampShared{&sl}, seed, rk, g32, pend, xs);
    else ok = sample_slots<MODE, R>(L, SampGlobal{samp + L.samp_off, L.ns}, seed, rk, g32, pend, xs);
    if (!ok) atomicOr(err, 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t z = zs[r], i = is[r];
        if (vs[r]) {
            const double v = xs[r];
            const double jd = rint(v / L.q);
            int64_t j = 0;
            if (jd >= -0x1.0p52 && jd <= 0x1.0p52) j = (int64_t)jd;
            else atomicOr(err, 8);
            qj[((size_t)z * nq + qbase + blockIdx.y) * (size_t)n + i] = j;
            const unsigned long long key = (unsigned long long)j ^ 0x8000000000000000ull;
            mn = key < mn ? key : mn;
            mx = key > mx ? key : mx;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long a = __shfl_xor(mn, off), b = __shfl_xor(mx, off);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    __shared__ unsigned long long wmn[kBlock / 64], wmx[kBlock / 64];
    if ((threadIdx.x & 63) == 0) {
        wmn[threadIdx.x >> 6] = mn;
        wmx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) {
            mn = wmn[w] < mn ? wmn[w] : mn;
            mx = wmx[w] > mx ? wmx[w] : mx;
        }
        if (mn <= mx) {
            atomicMin(qmin + qbase + blockIdx.y, mn);
            atomicMax(qmax + qbase + blockIdx.y, mx);
        }
    }
}

// Quantized families, pass 2: one workgroup per distinct grid value x = j * q
// (a wave each left config 5's ~2.6k waves at 0.59 VALU busy), thread-strided
// component sums for both mixtures, written once to the table.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_qtable(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const QInfo* __restrict__ qinfo, int32_t nq,
    int32_t qbase, double2* __restrict__ tab, unsigned long long* __restrict__ qkmax,
    const Comp<double>* __restrict__ qcomp, const int32_t* __restrict__ qc_n) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    const QInfo Q = qinfo[qbase + blockIdx.y];
    const int64_t s = blockIdx.x;
    if (s >= Q.G) return;   // uniform over the workgroup
    const double x = (double)(Q.jmin + s) * L.q;
    double ub, lo;
    bool neg;
    quant_bounds<MODE>(L, x, ub, lo, neg);
    constexpr bool kLog = MODE == QUANT_LGMM;
    double pb = wave_sum(quant_share<kLog, kBlock>(comps64 + L.comp_b, L.nb, ub, lo, threadIdx.x));
    // the above mixture as its runs of equal (mu, a): a quantized label's
    // observations take few distinct values (k_qcompress)
    double pa = wave_sum(quant_share<kLog, kBlock>(qcomp + L.comp_a, qc_n[li], ub, lo, threadIdx.x));
    __shared__ double2 wp[kBlock / 64];
    if ((threadIdx.x & 63) == 0) wp[threadIdx.x >> 6] = make_double2(pb, pa);
    __syncthreads();
    if (threadIdx.x == 0) {
        pb = wp[0].x;
        pa = wp[0].y;
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) {
            pb += wp[w].x;
            pa += wp[w].y;
        }
        const double2 v = make_double2(flog(pb) - L.logpacc_b, flog(pa) - L.logpacc_a);
        tab[Q.tab_off + s] = v;
        const int64_t j = Q.jmin + s;
        if (qkmax && j >= Q.jlo && j <= Q.jhi) atomicMax(qkmax + qbase + blockIdx.y, order_key(v.x - v.y));
    }
}

// The quantized labels' above mixtures as runs of equal (mu, a) -- records
// sorted by mu, the ties of a quantized label's observations adjacent (the
// run's interior shares the clipped minimum sigma): each run becomes one
// record carrying the run's total weight, so k_qtable sums ~(distinct values
// x 3) erf pairs per grid value instead of one per observation (config 5:
// 50k -> a few hundred).  prob = sum_k w_k (Phi_u - Phi_l) regrouped as
// sum_runs W_run (Phi_u - Phi_l), W_run a difference of the label's weight
// prefix sums (~1e-16 of the total weight each): inside the quantized lpdf
// bar (relative 1e-9, absolute 1e-13 on the probability).  One workgroup per
// quantized label position, chunks of 4096 records (4 per thread): the run
// starts and the prefix by block scans; a start stores the prefix before
// it, the run's end (after a barrier) the difference.
constexpr int kQcBlock = 1024;
constexpr int kQcU = 4;   // records per thread per chunk
__global__ __launch_bounds__(kQcBlock) void k_qcompress(const DLabel* __restrict__ labels,
                                                        const int32_t* __restrict__ group,
                                                        const Comp<double>* __restrict__ comps64,
                                                        Comp<double>* __restrict__ qcomp,
                                                        int32_t* __restrict__ qc_n) {
    const int li = group[blockIdx.x];
    const DLabel L = labels[li];
    const Comp<double>* c = comps64 + L.comp_a;
    Comp<double>* out = qcomp + L.comp_a;
    const int n = L.na, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ int32_t wcnt[kQcBlock / 64];
    __shared__ double wsum[kQcBlock / 64];
    __shared__ int32_t runs;
    __shared__ double pre;
    if (threadIdx.x == 0) {
        runs = 0;
        pre = 0.0;
    }
    __syncthreads();
    // kQcU consecutive records per thread per chunk (one chunk of kQcBlock
    // was three barriers and a dependent round of loads per 1024 records:
    // ~70 us for a 7.5k-record label); the thread's records and the two
    // around them loaded first
    for (int c0 = 0; c0 < n; c0 += kQcBlock * kQcU) {
        const int kb = c0 + (int)threadIdx.x * kQcU;
        double mu[kQcU + 2], av[kQcU + 2], wv[kQcU], cv[kQcU];
#pragma unroll
        for (int i = 0; i < kQcU + 2; ++i) {
            const int k = kb - 1 + i;
            const bool ok = k >= 0 && k < n;
            mu[i] = ok ? c[k].mu : 0.0;
            av[i] = ok ? c[k].a : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kQcU; ++u) {
            const bool ok = kb + u < n;
            wv[u] = ok ? c[kb + u].w : 0.0;
            cv[u] = ok ? c[kb + u].c : 0.0;
        }
        auto differ = [&](int i, int j) {   // (bit-unequal mu or a)
            return __double_as_longlong(mu[i]) != __double_as_longlong(mu[j]) ||
                   __double_as_longlong(av[i]) != __double_as_longlong(av[j]);
        };
        bool st[kQcU], en[kQcU];
        double loc[kQcU];
        double run = 0.0;
        int nst = 0;
#pragma unroll
        for (int u = 0; u < kQcU; ++u) {
            const int k = kb + u;
            const bool in = k < n;
            st[u] = in && (k == 0 || differ(u + 1, u));
            en[u] = in && (k == n - 1 || differ(u + 2, u + 1));
            loc[u] = run;   // the thread's weight before record u
            run += wv[u];
            nst += st[u];
        }
        // inclusive scans over the wave: the threads' weights and starts
        double x = run;
        int xs = nst;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const double y = __shfl_up(x, off);
            const int ys = __shfl_up(xs, off);
            if (lane >= off) {
                x += y;
                xs += ys;
            }
        }
        if (lane == 63) {
            wsum[w] = x;
            wcnt[w] = xs;
        }
        __syncthreads();
        double e0 = pre;   // the weight before this thread's first record
        int32_t r0 = runs;
        for (int u = 0; u < w; ++u) {
            e0 += wsum[u];
            r0 += wcnt[u];
        }
        e0 += x - run;
        r0 += xs - nst;   // the starts before this thread's first record
        int32_t rr[kQcU];
        double ek[kQcU];
        int32_t sc = 0;
#pragma unroll
        for (int u = 0; u < kQcU; ++u) {
            sc += st[u];
            rr[u] = r0 + sc - 1;   // the run holding record u
            ek[u] = e0 + loc[u];
            if (st[u]) out[rr[u]] = Comp<double>{mu[u + 1], av[u + 1], cv[u], ek[u]};
        }
        __syncthreads();   // every start of this chunk written (and the shared sums read)
#pragma unroll
        for (int u = 0; u < kQcU; ++u)
            if (en[u]) out[rr[u]].w = (ek[u] + wv[u]) - out[rr[u]].w;
        if (threadIdx.x == kQcBlock - 1) {   // the chunk's totals onward
            double t = pre;
            int32_t q = runs;
            for (int u = 0; u < kQcBlock / 64; ++u) {
                t += wsum[u];
                q += wcnt[u];
            }
            pre = t;
            runs = q;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) qc_n[li] = runs;
}

// Quantized families, pass 3: per candidate look up its grid value's lpdf
// pair (direct evaluation when the label's window was too wide for a table),
// then the same block maxloc as k_round.
template <int MODE, int R>
__global__ __launch_bounds__(kBlock) void k_qscan(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const int64_t* __restrict__ qj,
    const QInfo* __restrict__ qinfo, const double2* __restrict__ tab, int64_t n,
    int64_t cand_offset, int32_t nq, int32_t qbase, int32_t n_labels, int32_t tiles,
    Partial* __restrict__ partials, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    double x[R], lb[R], la[R];
    int64_t z[R], ci[R], gi[R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        S.template at<R>(r, n, z[r], ci[r], valid[r]);
        gi[r] = cand_offset + ci[r];
        const QInfo Q = qinfo[qbase + blockIdx.y];         // window shared by all rounds
        const size_t slot = (size_t)(valid[r] ? z[r] : 0) * nq + qbase + blockIdx.y;
        const int64_t j = valid[r] ? qj[slot * (size_t)n + ci[r]] : Q.jmin;
        x[r] = (double)j * L.q;
        const int64_t s = j - Q.jmin;
        if (s >= 0 && s < Q.G) {
            const double2 t = tab[Q.tab_off + s];
            lb[r] = t.x;
            la[r] = t.y;
        } else {
            double ub, lo;
            bool neg;
            quant_bounds<MODE>(L, x[r], ub, lo, neg);
            lb[r] = quant_lpdf<MODE == QUANT_LGMM>(comps64 + L.comp_b, L.nb, ub, lo, L.logpacc_b);
            la[r] = quant_lpdf<MODE == QUANT_LGMM>(comps64 + L.comp_a, L.na, ub, lo, L.logpacc_a);
        }
    }
    __shared__ double scratch[R * kBlock * 3 / 2];
    __shared__ Partial sh[kBlock / 64];
    finish_slots<R>(S, x, lb, la, valid, z, gi, li, n_labels, tiles, partials, scratch, sh);
}

// Bounded quantized labels whose grid window is known before sampling
// (launch_quantized: [low, high] / q): the tables are built first and one
// kernel draws, maps to the grid (k_qsample's arithmetic), looks up and
// reduces -- no index array, no window round trip.  Same values as
// k_qsample + k_qscan.
template <int MODE, int R>
__global__ __launch_bounds__(kBlock) void k_qfused(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp,
    const QInfo* __restrict__ qinfo, const double2* __restrict__ tab, int64_t n, int64_t cand_offset,
    uint64_t seed, const uint32_t* __restrict__ rounds, int32_t qbase, int32_t n_labels, int32_t tiles,
    Partial* __restrict__ partials, int32_t* __restrict__ err, Slots S) {
    const int li = group[blockIdx.y];
    const DLabel L = labels[li];
    __shared__ SampLds sl;
    const bool staged = stage_samp(L, samp, &sl);
    const QInfo Q = qinfo[qbase + blockIdx.y];
    double x[R], lb[R], la[R], v[R];
    int64_t z[R], ci[R], gi[R];
    bool valid[R];
    uint32_t g32[R], rk[R], pend = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        S.template at<R>(r, n, z[r], ci[r], valid[r]);
        gi[r] = cand_offset + ci[r];
        g32[r] = (uint32_t)gi[r];
        rk[r] = valid[r] ? rounds[z[r]] : 0u;
        v[r] = 0.0;
        if (valid[r]) pend |= 1u << r;
    }
    const bool ok = staged ? sample_slots<MODE, R>(L, SampShared{&sl}, seed, rk, g32, pend, v)
                           : sample_slots<MODE, R>(L, SampGlobal{samp + L.samp_off, L.ns}, seed, rk, g32, pend, v);
    if (!ok) atomicOr(err, 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double jd = rint(v[r] / L.q);
        int64_t j = Q.jmin;
        if (valid[r]) {
            if (jd >= -0x1.0p52 && jd <= 0x1.0p52) j = (int64_t)jd;
            else atomicOr(err, 8);
        }
        x[r] = (double)j * L.q;
        const int64_t s = j - Q.jmin;
        if (s >= 0 && s < Q.G) {
            const double2 t = tab[Q.tab_off + s];
            lb[r] = t.x;
            la[r] = t.y;
        } else {
            double ub, lo;
            bool neg;
            quant_bounds<MODE>(L, x[r], ub, lo, neg);
            lb[r] = quant_lpdf<MODE == QUANT_LGMM>(comps64 + L.comp_b, L.nb, ub, lo, L.logpacc_b);
            la[r] = quant_lpdf<MODE == QUANT_LGMM>(comps64 + L.comp_a, L.na, ub, lo, L.logpacc_a);
        }
    }
    __shared__ double scratch[R * kBlock * 3 / 2];
    __shared__ Partial sh[kBlock / 64];
    finish_slots<R>(S, x, lb, la, valid, z, gi, li, n_labels, tiles, partials, scratch, sh);
}

// both quantized lpdfs of one candidate evaluated directly (scalar
// arguments: the call spills nothing outside its own branch)
template <bool LOG>
__device__ __noinline__ double2 quant_pair_direct(const Comp<double>* __restrict__ cb, int nb, double lpb,
                                                  const Comp<double>* __restrict__ ca, int na, double lpa,
                                                  double ub, double lo) {
    return make_double2(quant_lpdf<LOG>(cb, nb, ub, lo, lpb), quant_lpdf<LOG>(ca, na, ub, lo, lpa));
}

// Exact early exit of a round whose scores take few values (quantized and
// categorical labels): kmax = the best score key any drawable candidate can
// have.  Once a candidate of index f holds kmax, no candidate after f can win
// (a later equal score loses the tie), so a workgroup stops at the first tile
// starting past found[cell] = the smallest such f reported so far; every
// candidate before the true first kmax index is still processed (its tile
// starts before any reported f), so the block maxloc over what was
// processed is the np.argmax winner.  found only decreases; a stale read
// only costs work.  The stop test is made uniform over the workgroup.
__device__ __forceinline__ bool tile_stop(const int64_t* __restrict__ found, int64_t gbase, int64_t* sh) {
    if (threadIdx.x == 0) *sh = __hip_atomic_load(found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool stop = *sh <= gbase;
    __syncthreads();
    return stop;
}

// A workgroup of an early-exit launch whose first tile already lies past the
// cell's find does nothing but empty its partial slot (and its share of the
// slots after the launch's): the second phase's grid costs little once the
// first phase has found the winner.  Uniform over the workgroup.
__device__ __forceinline__ bool early_out(const int64_t* __restrict__ fcell, int64_t gfirst, Partial* prow,
                                          int32_t slot, int32_t tiles, int32_t empty_from, int64_t* sh) {
    if (threadIdx.x == 0) *sh = __hip_atomic_load(fcell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*sh > gfirst) return false;
    for (int64_t t = (int64_t)empty_from + blockIdx.x + (int64_t)threadIdx.x * gridDim.x; t < tiles;
         t += (int64_t)kBlock * gridDim.x)
        prow[t] = Partial{0, INT64_MAX, 0.0, 0.0, 0.0};
    if (threadIdx.x == 0) prow[slot] = Partial{0, INT64_MAX, 0.0, 0.0, 0.0};
    return true;
}

// k_qfused for the tile map with workgroups striding over the tiles of
// R * 256 candidates from candidate i0 on (the sampling records staged once
// per workgroup, a running best per thread): the block's winner goes to
// partial slot slot_base + blockIdx.x, and the workgroups empty the slots from
// empty_from on, so k_reduce sees every tile slot.  Same candidates, values
// and winner as k_qfused; with kmax (bounded labels, qkmax) the early exit
// above.
template <int MODE, int R>
__global__ __launch_bounds__(kBlock, 4) void k_qfused_tiles(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp,
    const QInfo* __restrict__ qinfo, const double2* __restrict__ tab, int64_t n, int64_t cand_offset,
    uint64_t seed, const uint32_t* __restrict__ rounds, int32_t qbase, int32_t n_labels, int32_t tiles,
    Partial* __restrict__ partials, int32_t* __restrict__ err, const unsigned long long* __restrict__ qkmax,
    int64_t* __restrict__ found, int64_t i0, int32_t slot_base, int32_t empty_from,
    unsigned long long* __restrict__ drawn) {
    const int li = group[blockIdx.y];
    constexpr int64_t per = (int64_t)R * kBlock;
    __shared__ int64_t sfound;
    Partial* prow = partials + ((size_t)blockIdx.z * n_labels + li) * tiles;
    int64_t* fcell = found ? found + (size_t)blockIdx.z * n_labels + li : nullptr;
    if (fcell && early_out(fcell, cand_offset + i0 + (int64_t)blockIdx.x * per, prow, slot_base + blockIdx.x, tiles,
                           empty_from, &sfound))
        return;
    const DLabel L = labels[li];
    __shared__ SampLds sl;
    const bool staged = stage_samp(L, samp, &sl);
    const QInfo Q = qinfo[qbase + blockIdx.y];
    const uint32_t rk = rounds[blockIdx.z];
    // the window's scores as order keys in LDS when they fit: per candidate
    // one LDS read; the winner's lpdfs are read from the table at the end
    __shared__ unsigned long long skey[kQLdsKeys];
    const bool lds_keys = Q.G > 0 && Q.G <= kQLdsKeys;
    if (lds_keys)
        for (int t = threadIdx.x; t < (int)Q.G; t += kBlock) {
            const double2 v = tab[Q.tab_off + t];
            skey[t] = order_key(v.x - v.y);
        }
    __syncthreads();
    const bool early = found && Q.G > 0 && Q.jlo <= Q.jhi;
    const uint64_t kmax = early ? qkmax[qbase + blockIdx.y] : 0;
    __syncthreads();
    bool reported = false;
    int64_t ndrawn = 0;
    uint64_t bk = 0;
    int64_t bi = INT64_MAX, bj = 0;
    bool bdirect = false;
    double bl = 0.0, ba = 0.0;
    for (int64_t base = i0 + (int64_t)blockIdx.x * per; base < n; base += (int64_t)gridDim.x * per) {
        if (early && tile_stop(fcell, cand_offset + base, &sfound)) break;
        ndrawn += min(per, n - base);
        double v[R];
        uint32_t pend = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            v[r] = 0.0;
            if (base + tile_cand(r, threadIdx.x, kBlock) < n) pend |= 1u << r;
        }
        const uint32_t g0 = (uint32_t)(cand_offset + base);
        const bool ok = staged ? sample_tile<MODE, R>(L, SampShared{&sl}, seed, rk, g0, pend, v)
                               : sample_tile<MODE, R>(L, SampGlobal{samp + L.samp_off, L.ns}, seed, rk, g0, pend, v);
        if (!ok) atomicOr(err, 1);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!((pend >> r) & 1u)) continue;
            const double jd = rint(v[r] / L.q);
            int64_t j = Q.jmin;
            if (jd >= -0x1.0p52 && jd <= 0x1.0p52) j = (int64_t)jd;
            else atomicOr(err, 8);
            const int64_t sidx = j - Q.jmin;
            const int64_t gi = cand_offset + base + tile_cand(r, threadIdx.x, kBlock);
            if (lds_keys && sidx >= 0 && sidx < Q.G) {
                const uint64_t key = skey[sidx];
                if (better(key, gi, bk, bi)) {
                    bk = key;
                    bi = gi;
                    bj = j;
                    bdirect = false;
                }
                continue;
            }
            const double x = (double)j * L.q;
            double lb, la;
            if (sidx >= 0 && sidx < Q.G) {
                const double2 t = tab[Q.tab_off + sidx];
                lb = t.x;
                la = t.y;
            } else {   // outside the table window (out of line: rare, register-heavy)
                double ub, lo;
                bool neg;
                quant_bounds<MODE>(L, x, ub, lo, neg);
                const double2 pr = quant_pair_direct<MODE == QUANT_LGMM>(
                    comps64 + L.comp_b, L.nb, L.logpacc_b, comps64 + L.comp_a, L.na, L.logpacc_a, ub, lo);
                lb = pr.x;
                la = pr.y;
            }
            const uint64_t key = order_key(lb - la);
            if (better(key, gi, bk, bi)) {
                bk = key;
                bi = gi;
                bj = j;
                bdirect = true;
                bl = lb;
                ba = la;
            }
        }
        if (early && !reported && bk == kmax && bi != INT64_MAX) {
            atomicMin((unsigned long long*)fcell, (unsigned long long)bi);
            reported = true;
        }
    }
    if (bi != INT64_MAX && !bdirect) {   // the winner came from the LDS keys
        const double2 t = tab[Q.tab_off + (bj - Q.jmin)];
        bl = t.x;
        ba = t.y;
    }
    const double bv = (double)bj * L.q;
    if (drawn && threadIdx.x == 0) atomicAdd(drawn, (unsigned long long)ndrawn);
    for (int64_t t = (int64_t)empty_from + blockIdx.x + (int64_t)threadIdx.x * gridDim.x; t < tiles;
         t += (int64_t)kBlock * gridDim.x)
        prow[t] = Partial{0, INT64_MAX, 0.0, 0.0, 0.0};
    __shared__ Partial sh[kBlock / 64];
    block_maxloc(bk, bi, bv, bl, ba, prow + slot_base + blockIdx.x, sh);
}

// Sampled categorical labels, tile map, workgroups striding over the tiles
// of R * 256 candidates from candidate i0 on (sample_below<CAT>'s draws: the
// first category whose cumulative weight exceeds the Philox word, here from
// the workgroup's LDS copy of the weights when they fit), log p lookup
// (tpe.py:56-63), running best per thread; partial slots and the early exit
// as k_qfused_tiles, kmax over the categories a draw can return (those of
// positive weight, and the last, which also takes a rounding overshoot of
// the cumulative weights).  Same winner as k_round<CAT>.
template <int R>
__global__ __launch_bounds__(kBlock) void k_cat_tiles(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ group,
    const Comp<double>* __restrict__ comps64, const SampRec* __restrict__ samp, int64_t n, int64_t cand_offset,
    uint64_t seed, const uint32_t* __restrict__ rounds, int32_t n_labels, int32_t tiles,
    Partial* __restrict__ partials, int64_t* __restrict__ found, int64_t i0, int32_t slot_base,
    int32_t empty_from, unsigned long long* __restrict__ drawn) {
    const int li = group[blockIdx.y];
    constexpr int64_t per = (int64_t)R * kBlock;
    __shared__ int64_t sfound;
    Partial* prow = partials + ((size_t)blockIdx.z * n_labels + li) * tiles;
    int64_t* fcell = found ? found + (size_t)blockIdx.z * n_labels + li : nullptr;
    if (fcell && early_out(fcell, cand_offset + i0 + (int64_t)blockIdx.x * per, prow, slot_base + blockIdx.x, tiles,
                           empty_from, &sfound))
        return;
    const DLabel L = labels[li];
    __shared__ SampLds sl;
    const bool staged = stage_samp(L, samp, &sl);
    const uint32_t rk = rounds[blockIdx.z];
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    __shared__ uint64_t shk[kBlock / 64];
    uint64_t km = 0;
    for (int k = threadIdx.x; k < L.nb; k += kBlock) {
        const double w = k < L.ns ? samp[L.samp_off + k].cdf - (k ? samp[L.samp_off + k - 1].cdf : 0.0) : 1.0;
        if (w > 0.0 || k == L.nb - 1 || k == L.ns - 1) {
            const uint64_t key = order_key(comps64[L.comp_b + k].c - comps64[L.comp_a + k].c);
            km = key > km ? key : km;
        }
    }
    const uint64_t kmax = block_max_key(km, shk);
    const bool early = found != nullptr;
    bool reported = false;
    int64_t ndrawn = 0;
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
    double bv = 0.0, bl = 0.0, ba = 0.0;
    for (int64_t base = i0 + (int64_t)blockIdx.x * per; base < n; base += (int64_t)gridDim.x * per) {
        if (early && tile_stop(fcell, cand_offset + base, &sfound)) break;
        ndrawn += min(per, n - base);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t ci = base + r * kBlock + threadIdx.x;
            if (ci >= n) continue;
            const int64_t gi = cand_offset + ci;
            const U4 w = philox4x32_10(U4{(uint32_t)gi, 0u, (uint32_t)L.stream, rk}, k0, k1);
            const double u = (double)w.x * 0x1.0p-32;
            int k;
            if (staged) {
                k = sl.guide[(int)(u * 64.0)];
                while (sl.cdf[k] <= u) ++k;
            } else {
                k = cdf_search(samp + L.samp_off, L.ns, u);
            }
            const int sc = k >= L.nb ? L.nb - 1 : k;
            const double lb = comps64[L.comp_b + sc].c, la = comps64[L.comp_a + sc].c;
            const uint64_t key = order_key(lb - la);
            if (better(key, gi, bk, bi)) {
                bk = key;
                bi = gi;
                bv = (double)k;
                bl = lb;
                ba = la;
            }
        }
        if (early && !reported && bk == kmax && bi != INT64_MAX) {
            atomicMin((unsigned long long*)fcell, (unsigned long long)bi);
            reported = true;
        }
    }
    if (drawn && threadIdx.x == 0) atomicAdd(drawn, (unsigned long long)ndrawn);
    for (int64_t t = (int64_t)empty_from + blockIdx.x + (int64_t)threadIdx.x * gridDim.x; t < tiles;
         t += (int64_t)kBlock * gridDim.x)
        prow[t] = Partial{0, INT64_MAX, 0.0, 0.0, 0.0};
    __shared__ Partial sh[kBlock / 64];
    block_maxloc(bk, bi, bv, bl, ba, prow + slot_base + blockIdx.x, sh);
}

__device__ __forceinline__ tpe_label_result to_result(const Partial& p, int li) {
    tpe_label_result r;
    r.value = p.value;
    r.score = p.lb - p.la;
    r.lpdf_below = p.lb;
    r.lpdf_above = p.la;
    r.index = p.idx != INT64_MAX ? p.idx : -1;
    r.label = li;
    // a value-only cell (k_pick_rounds: key of 0.0, both lpdfs NaN; a real
    // NaN score carries the NaN key, the greatest) has no score to merge by
    r.status = (p.key == order_key(0.0) && p.lb != p.lb && p.la != p.la) ? TPE_STATUS_VALUE_ONLY : 0;
    return r;
}

// per (label, round): the maxloc over its tiles' partials.  1024 threads, four
// independent running bests per thread over the (key, idx) words only (16 of
// the 40 bytes), the winning tile's record fetched once at the end: one
// workgroup per label streams up to 8192 partials at full memory parallelism
// instead of one dependent 40-byte load chain per thread.
constexpr int kReduceBlock = 1024;
// (dense_one: the dense labels' rows hold their winner in the first slot
// only -- the screened tile map's k_rescore_fin -- and the rest is not read)
__global__ __launch_bounds__(kReduceBlock) void k_reduce(const Partial* __restrict__ partials,
                                                         int32_t tiles_all, int32_t n_labels,
                                                         tpe_label_result* __restrict__ out,
                                                         const DLabel* __restrict__ labels, int32_t dense_one) {
    const int li = blockIdx.x, rz = blockIdx.y, tid = threadIdx.x;
    const Partial* p = partials + ((size_t)rz * n_labels + li) * tiles_all;
    int32_t tiles = tiles_all;
    if (dense_one) {
        const int32_t mode = labels[li].mode;
        if (mode == DENSE_GMM || mode == DENSE_LGMM) tiles = 1;
    }
    uint64_t bk[4] = {0, 0, 0, 0};
    int64_t bi[4] = {INT64_MAX, INT64_MAX, INT64_MAX, INT64_MAX};
    int32_t bt[4] = {-1, -1, -1, -1};
    for (int t0 = tid; t0 < tiles; t0 += 4 * kReduceBlock) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = t0 + u * kReduceBlock;
            if (t < tiles) {
                const uint64_t k = p[t].key;
                const int64_t i = p[t].idx;
                if (better(k, i, bk[u], bi[u])) {
                    bk[u] = k;
                    bi[u] = i;
                    bt[u] = t;
                }
            }
        }
    }
#pragma unroll
    for (int u = 1; u < 4; ++u)
        if (better(bk[u], bi[u], bk[0], bi[0])) {
            bk[0] = bk[u];
            bi[0] = bi[u];
            bt[0] = bt[u];
        }
    uint64_t k = bk[0];
    int64_t i = bi[0];
    int32_t t = bt[0];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t ok = __shfl_xor(k, off);
        const int64_t oi = __shfl_xor(i, off);
        const int32_t ot = __shfl_xor(t, off);
        if (better(ok, oi, k, i)) {
            k = ok;
            i = oi;
            t = ot;
        }
    }
    __shared__ uint64_t shk[kReduceBlock / 64];
    __shared__ int64_t shi[kReduceBlock / 64];
    __shared__ int32_t sht[kReduceBlock / 64];
    if ((tid & 63) == 0) {
        shk[tid >> 6] = k;
        shi[tid >> 6] = i;
        sht[tid >> 6] = t;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kReduceBlock / 64; ++w)
            if (better(shk[w], shi[w], k, i)) {
                k = shk[w];
                i = shi[w];
                t = sht[w];
            }
        const Partial best = t >= 0 ? p[t] : Partial{0, INT64_MAX, 0.0, 0.0, 0.0};
        out[(size_t)rz * n_labels + li] = to_result(best, li);
    }
}

// A round's small read-backs in one copy: each was its own hipMemcpyAsync
// (a blit launch of ~4 us on the device and ~7 us of host API time each, 5-7
// per round, on the round's critical path); now defer_read registers them,
// flush_reads packs them with one launch (k_pack_reads) into one block and
// copies it with one D2H, unpack_reads scatters it after the round's sync.
constexpr int kPackMax = 8;
struct PackArgs {
    const uint32_t* src[kPackMax];
    int64_t off[kPackMax];   // (32-bit words)
    int64_t words[kPackMax];
    int32_t n;
};
__global__ __launch_bounds__(kBlock) void k_pack_reads(PackArgs a, uint32_t* __restrict__ out) {
    for (int t = 0; t < a.n; ++t)
        for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.words[t]; i += (int64_t)gridDim.x * kBlock)
            out[a.off[t] + i] = a.src[t][i];
}

int defer_read(tpe_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    if (bytes <= 0) return TPE_OK;
    if ((bytes & 3) || ((uintptr_t)src & 3) || bytes > (1 << 16))   // (large or odd: its own copy)
        return ctx->hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream), "read-back");
    ctx->rep.push_back(tpe_ctx::RepTask{src, dst, bytes});
    return TPE_OK;
}

// A round's results from the pinned staging buffer into the caller's array:
// config 5's batched round returns 25 MB (4096 rounds x 128 labels x 48 B),
// which one thread copies (first touch of the caller's fresh pages included)
// in about as long as the round's kernels take; 2 MB slices over up to 8
// threads (4.20 -> 3.80 ms per config-5 round, r5ab).
static void copy_out(void* dst, const void* src, size_t bytes) {
    constexpr size_t kSlice = (size_t)2 << 20;
    const int nt = (int)std::min<size_t>(8, bytes / kSlice);
    if (nt < 2) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const size_t per = (bytes / nt + 63) & ~(size_t)63;
    auto part = [&](int t) {
        const size_t a = std::min(bytes, (size_t)t * per), b = std::min(bytes, a + per);
        if (b > a) std::memcpy((char*)dst + a, (const char*)src + a, b - a);
    };
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int t = 1; t < nt; ++t) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
}

int flush_reads(tpe_ctx* ctx) {
    if (ctx->rep.empty()) return TPE_OK;
    int64_t total = 0, mx = 1;
    for (const auto& r : ctx->rep) {
        total += r.bytes;
        mx = std::max(mx, r.bytes / 4);
    }
    HIPCHK(ctx, ctx->rep_d.reserve(total));
    HIPCHK(ctx, ctx->rep_h.resize(total));
    int64_t off = 0;
    for (size_t i = 0; i < ctx->rep.size(); i += kPackMax) {
        PackArgs a{};
        a.n = (int32_t)std::min<size_t>(kPackMax, ctx->rep.size() - i);
        for (int t = 0; t < a.n; ++t) {
            const auto& r = ctx->rep[i + t];
            a.src[t] = (const uint32_t*)r.src;
            a.off[t] = off / 4;
            a.words[t] = r.bytes / 4;
            off += r.bytes;
        }
        hipLaunchKernelGGL(k_pack_reads, dim3((unsigned)std::min<int64_t>((mx + kBlock - 1) / kBlock, 16)),
                           dim3(kBlock), 0, ctx->stream, a, (uint32_t*)ctx->rep_d.p);
        HIPCHK(ctx, hipGetLastError());
    }
    return ctx->hip(hipMemcpyAsync(ctx->rep_h.data(), ctx->rep_d.p, total, hipMemcpyDeviceToHost, ctx->stream),
                    "packed read-back");
}

// after the stream's sync
void unpack_reads(tpe_ctx* ctx) {
    int64_t off = 0;
    for (const auto& r : ctx->rep) {
        std::memcpy(r.dst, ctx->rep_h.data() + off, r.bytes);
        off += r.bytes;
    }
    ctx->rep.clear();
}

// Several small fills in one launch (per-round counters, flags and
// thresholds): grid.y = the fill, 32-bit words.  A hipMemsetAsync each would
// cost a host API call and a queue slot apiece -- a round's resets used to be
// ~10 of them between its kernels.
constexpr int kMaxFills = 8;
struct FillSet {
    uint32_t* p[kMaxFills];
    int64_t n[kMaxFills];
    uint32_t v[kMaxFills];
    int32_t count;
};
__global__ __launch_bounds__(kBlock) void k_fill_words(FillSet f) {
    const int j = blockIdx.y;
    uint32_t* p = f.p[j];
    const int64_t n = f.n[j];
    const uint32_t v = f.v[j];
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) p[i] = v;
}

// one partial per (round, label) -- packed and split-K maps: a thread each
__global__ __launch_bounds__(kBlock) void k_emit(const Partial* __restrict__ partials, int64_t n,
                                                 int32_t n_labels,
                                                 tpe_label_result* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < n) out[j] = to_result(partials[j], (int)(j % n_labels));
}

// argmax of below - above over caller arrays (tpe_broadcast_best)
__global__ __launch_bounds__(kBlock) void k_argmax(const double* __restrict__ b,
                                                   const double* __restrict__ a, int64_t n,
                                                   Partial* __restrict__ partials) {
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const uint64_t k = order_key(b[i] - a[i]);
        if (better(k, i, bk, bi)) {
            bk = k;
            bi = i;
        }
    }
    __shared__ Partial sh[kBlock / 64];
    block_maxloc(bk, bi, 0.0, 0.0, 0.0, partials + blockIdx.x, sh);
}

// sample-only kernel (tpe_*_sample): one draw per thread, no scoring
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_sample_only(const DLabel* __restrict__ labels,
                                                        const SampRec* __restrict__ samp,
                                                        int64_t n, int64_t offset, uint64_t seed,
                                                        const uint32_t* __restrict__ rounds,
                                                        double* __restrict__ out,
                                                        int32_t* __restrict__ err) {
    const DLabel L = labels[0];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    double v;
    if (!sample_below<MODE>(L, samp + L.samp_off, seed, rounds[0], (uint32_t)(offset + i), v))
        atomicOr(err, 1);
    out[i] = v;
}

// ------------------------------------------------------------ host side ----

inline bool host_better(uint64_t ka, int64_t ia, uint64_t kb, int64_t ib) {
    return ka > kb || (ka == kb && ia < ib);
}

// numpy-style pairwise summation (what np.sum does for float64 vectors)
double np_pairwise_sum_impl(const double* a, size_t n) {
    if (n < 8) {
        double r = 0.0;
        for (size_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        size_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    size_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sum_impl(a, n2) + np_pairwise_sum_impl(a + n2, n - n2);
}

// normal_cdf, tpe.py:102-107
double host_normal_cdf(double x, double mu, double sigma) {
    const double bottom = std::max(std::sqrt(2.0) * sigma, kEps);
    return 0.5 * (1.0 + std::erf((x - mu) / bottom));
}


}  // namespace


namespace {

// Fold one GMM1/LGMM1 mixture into device records (host fp64, reference
// formulas).  Returns the LSE shift (dense) or log p_accept (quantized).
struct Folded {
    double shift = 0.0, logpacc = 0.0, amax = 0.0;
};

Folded fold_mixture(int kind, bool quant, int flags, double low, double high, double centre,
                    const double* w, const double* mu, const double* sg, int n,
                    Comp<double>* out64, Comp<float>* out32) {
    Folded f;
    const bool bounded = (flags & 3) != 0;
    double p_accept = 1.0;
    if (bounded) {  // tpe.py:139-142 / 279-282
        std::vector<double> t(n);
        for (int k = 0; k < n; ++k)
            t[k] = w[k] * (host_normal_cdf(high, mu[k], sg[k]) - host_normal_cdf(low, mu[k], sg[k]));
        p_accept = tpe_rt::np_pairwise_sum(t.data(), n);
    }
    if (quant) {
        f.logpacc = std::log(p_accept);
        for (int k = 0; k < n; ++k) {
            const double a = 1.0 / std::max(std::sqrt(2.0) * sg[k], kEps);
            out64[k] = Comp<double>{mu[k], a, 0.0, w[k]};
            if (out32) out32[k] = Comp<float>{(float)mu[k], (float)a, 0.f, (float)w[k]};
        }
        return f;
    }
    std::vector<double> c(n);
    std::vector<double> a(n);
    for (int k = 0; k < n; ++k) {
        if (kind == TPE_GMM1) {  // log(w / sqrt(2 pi sigma^2) / p_accept), tpe.py:148-150
            const double Z = std::sqrt(2.0 * M_PI * (sg[k] * sg[k]));
            c[k] = std::log(w[k] / Z / p_accept);
            a[k] = std::sqrt(0.5) / std::max(sg[k], kEps);
        } else {  // log w - log(max(sigma,EPS) sqrt(2 pi)); -log x per candidate, tpe.py:199-208
            const double s = std::max(sg[k], kEps);
            c[k] = std::log(w[k]) - std::log(s * std::sqrt(2.0 * M_PI));
            a[k] = std::sqrt(0.5) / s;
        }
    }
    double M = -INFINITY;
    for (int k = 0; k < n; ++k)
        if (c[k] > M) M = c[k];
    if (!std::isfinite(M)) M = 0.0;
    f.shift = M;
    const double l2e = 1.4426950408889634;
    const double sK = std::sqrt(kExpScale);
    for (int k = 0; k < n; ++k) {
        // fp64 records in exp_scaled units (see tpe_device.h: u = K t)
        out64[k] = Comp<double>{(mu[k] - centre) * (a[k] * sK), a[k] * sK, (c[k] - M) * kExpScale,
                                w[k]};
        if (out32) {
            const double a2 = a[k] * std::sqrt(l2e);
            out32[k] = Comp<float>{(float)((mu[k] - centre) * a2), (float)a2,
                                   (float)((c[k] - M) * l2e), (float)w[k]};
            f.amax = std::max(f.amax, (double)out32[k].a);
        }
    }
    return f;
}

int validate_mixture(tpe_ctx* ctx, int32_t k, int32_t flags, double low, double high,
                     bool sampler_checks) {
    if (k <= 0) return ctx->fail(TPE_ERR_TYPE, "need vector of weights (empty mixture)");
    if ((flags & 3) == 1 || (flags & 3) == 2)
        return ctx->fail(TPE_ERR_TYPE, "low and high must both be given or both be None");
    if (sampler_checks && (flags & 3) == 3 && !(low < high))  // GMM1/LGMM1 only, tpe.py:86
        return ctx->fail(TPE_ERR_VALUE, "low >= high");
    return TPE_OK;
}

struct Groups {
    const int32_t* dev[kNumModes];   // device pointers to label ids per mode
    int32_t count[kNumModes];
};

struct RoundArgs {
    int64_t n, cand_offset;
    uint64_t seed;
    int32_t n_rounds, tiles;   // tiles: partials per (round, label)
    const double* cand_in;
    double *olb, *ola;
    Slots S;                   // slot map (tile or grouped)
    uint32_t gx, gz;           // grid.x / grid.z of the per-candidate kernels
    // the whole problem when this context runs one shard of it (multi-device
    // contexts, tpe_multi.hip): decisions that change a summation order --
    // chunking, table vs direct quantized scoring -- follow the whole
    // problem, so every sharding gives bit-identical winners
    int64_t total_slots;       // candidates x rounds over all shards
    uint32_t gx_whole;         // grid.x the whole problem would use
};

// The launches of an early-exit tile round (k_qfused_tiles, k_cat_tiles):
// a first phase of at most kEarlyTiles tiles per label (where the best
// drawable score almost always turns up), then -- if the round is longer --
// the rest with the full grid, whose workgroups stop as soon as they see the
// first phase's find.  Partial slots: phase 1 [0, g1), phase 2 [g1, g1 + g2),
// the last launch empties the slots after its own.
constexpr int64_t kEarlyTiles = 64;
struct EarlyPhase {
    unsigned grid;
    int64_t i0, n;
    int32_t slot_base, empty_from;
};

// the second phase's workgroups over all its (label, round) cells: they
// stride over the tiles, so a smaller grid costs nothing when the first
// phase found the winner (every workgroup exits at once) and still fills the
// chip when it did not
constexpr int64_t kEarlyWgs2 = 2048;

std::vector<EarlyPhase> early_phases(const RoundArgs& a, int64_t per, unsigned grid, bool early,
                                     int64_t cells) {
    const int64_t tiles_n = (a.n + per - 1) / per;
    const int64_t g1 = std::min<int64_t>({tiles_n, kEarlyTiles, (int64_t)a.tiles - 1});
    if (!early || g1 < 1 || g1 >= tiles_n || (int64_t)a.tiles - g1 < 1)
        return {EarlyPhase{grid, 0, a.n, 0, (int32_t)grid}};
    const unsigned g2 = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>({(int64_t)grid, (int64_t)a.tiles - g1, kEarlyWgs2 / std::max<int64_t>(1, cells)}));
    return {EarlyPhase{(unsigned)g1, 0, g1 * per, 0, a.tiles},
            EarlyPhase{g2, g1 * per, a.n, (int32_t)g1, (int32_t)(g1 + g2)}};
}

// queue a fill of `bytes` (a multiple of 4) with the 32-bit pattern v
void add_fill(FillSet& f, void* p, size_t bytes, uint32_t v) {
    if (!bytes) return;
    f.p[f.count] = (uint32_t*)p;
    f.n[f.count] = (int64_t)(bytes / 4);
    f.v[f.count] = v;
    ++f.count;
}

int run_fills(tpe_ctx* ctx, FillSet& f) {
    if (!f.count) return TPE_OK;
    int64_t mx = 1;
    for (int j = 0; j < f.count; ++j) mx = std::max(mx, f.n[j]);
    hipLaunchKernelGGL(k_fill_words, dim3((unsigned)std::min<int64_t>((mx + kBlock - 1) / kBlock, 1024), f.count),
                       dim3(kBlock), 0, ctx->stream, f);
    f.count = 0;
    return ctx->hip(hipGetLastError(), "fill launch");
}

// the per-(round, label) first-find indices (reset at the round's start,
// run_round; nullptr: early exit off)
int64_t* early_found(tpe_ctx* ctx) { return ctx->early ? ctx->xfound.p : nullptr; }

// The candidates an early-exit tile round of one family drew, counted the
// same way whatever order the workgroups ran in: per
// (round, label) cell every tile that starts at or before the cell's first
// index holding its best drawable score (found, exact), or all n when it was
// never found (or the early exit is off) -- the work a scan in index order
// must do.  The workgroups' own counts also include the tiles they drew
// before another's find reached them, which depends on the interleaving
// (with TPE_OPT_AUX_FAMILIES: on the dense draw beside them).
__global__ __launch_bounds__(kBlock) void k_early_drawn(const int64_t* __restrict__ found,
                                                        const int32_t* __restrict__ group, int32_t nl,
                                                        int32_t nz, int32_t n_labels, int64_t n,
                                                        int64_t cand_offset, int64_t per,
                                                        unsigned long long* __restrict__ drawn) {
    const int64_t cell = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    unsigned long long c = 0;
    if (cell < (int64_t)nl * nz) {
        const int64_t z = cell / nl;
        const int y = (int)(cell % nl);
        const int64_t f = found ? found[(size_t)z * n_labels + group[y]] : INT64_MAX;
        const int64_t i = f - cand_offset;
        c = (unsigned long long)((f == INT64_MAX || i < 0 || i >= n) ? n : std::min<int64_t>(n, (i / per + 1) * per));
    }
    // one atomic per wave
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(drawn, c);
}

void launch_early_drawn(tpe_ctx* ctx, const int32_t* group, int nl, const RoundArgs& a, int64_t* found,
                        int64_t per, unsigned long long* drawn) {
    const int64_t cells = (int64_t)nl * a.gz;
    hipLaunchKernelGGL(k_early_drawn, dim3((unsigned)((cells + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       found, group, nl, (int32_t)a.gz, ctx->P->n_labels, a.n, a.cand_offset, per, drawn);
}

void bracket(tpe_ctx* ctx, int mode, int which) {
    ctx->mode_ran[mode] = true;
    if (ctx->timing) (void)hipEventRecord(ctx->evm[mode][which], ctx->stream);
}

template <typename T, int MODE, bool SAMPLE>
void launch_round(tpe_ctx* ctx, const Groups& g, const RoundArgs& a) {
    const int nl = g.count[MODE];
    if (nl == 0 || a.tiles == 0) return;
    bracket(ctx, MODE, 0);
    if constexpr (MODE == CAT && SAMPLE) {
        if (a.S.cpack == 0 && a.olb == nullptr && a.cand_in == nullptr) {   // tile map: persistent
            const unsigned cgx = (unsigned)std::max<int64_t>(
                1, std::min<int64_t>({(int64_t)a.gx, (a.n + kCatR * kBlock - 1) / (kCatR * kBlock),
                                      kHotWgs / std::max<int64_t>(1, (int64_t)nl * a.gz)}));
            int64_t* found = early_found(ctx);
            ctx->cat_early = true;
            for (const EarlyPhase& ph :
                 early_phases(a, (int64_t)kCatR * kBlock, cgx, found != nullptr, (int64_t)nl * a.gz))
                hipLaunchKernelGGL((k_cat_tiles<kCatR>), dim3(ph.grid, nl, a.gz), dim3(kBlock), 0, ctx->stream,
                                   ctx->P->labels.p, g.dev[MODE], ctx->P->comps64.p, ctx->P->samp.p, ph.n,
                                   a.cand_offset, a.seed, ctx->rounds.p, ctx->P->n_labels, a.tiles,
                                   ctx->partials.p, found, ph.i0, ph.slot_base, ph.empty_from, nullptr);
            launch_early_drawn(ctx, g.dev[MODE], nl, a, found, (int64_t)kCatR * kBlock, ctx->xdrawn.p + 1);
            bracket(ctx, MODE, 1);
            return;
        }
    }
    const Comp<T>* comps;
    if constexpr (sizeof(T) == 8) comps = ctx->P->comps64.p; else comps = ctx->P->comps32.p;
    if (narrow(a.S))
        hipLaunchKernelGGL((k_round<T, MODE, SAMPLE, kRGroup>), dim3(a.gx, nl, a.gz), dim3(kBlock),
                           0, ctx->stream, ctx->P->labels.p, g.dev[MODE], comps, ctx->P->comps64.p,
                           ctx->P->samp.p, a.cand_in, a.n, a.cand_offset, a.seed, ctx->rounds.p,
                           ctx->P->n_labels, a.tiles, ctx->partials.p, a.olb, a.ola, ctx->errflag.p,
                           a.S);
    else
        hipLaunchKernelGGL((k_round<T, MODE, SAMPLE, kR>), dim3(a.gx, nl, a.gz), dim3(kBlock), 0,
                           ctx->stream, ctx->P->labels.p, g.dev[MODE], comps, ctx->P->comps64.p,
                           ctx->P->samp.p, a.cand_in, a.n, a.cand_offset, a.seed, ctx->rounds.p,
                           ctx->P->n_labels, a.tiles, ctx->partials.p, a.olb, a.ola, ctx->errflag.p,
                           a.S);
    bracket(ctx, MODE, 1);
}

// Chunks of the above mixtures for a packed sampled round: a fixed length
// of kChunkLen components (round 6; the count followed the workgroups of the
// round before), so a label's summation order -- chunk sums added in order
// -- depends on the label alone and a label-sharded multi-device context
// (or a label-shard rank) returns the one-context bits.  Config 5 (50k
// above components): 7 chunks, as the workgroup rule picked there.
// TPE_OPT_CHUNKS forces a count (tests): chunk = ceil(na_max / count).
constexpr int32_t kChunkLen = 8192;

int dense_chunks(const tpe_ctx* ctx) {
    int32_t na_max = 1;
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : ctx->P->h_group[m]) na_max = std::max(na_max, ctx->P->h_labels[li].na);
    if (ctx->chunks_forced) return ctx->chunks_forced;
    return (int)((na_max + kChunkLen - 1) / kChunkLen);
}

int32_t dense_chunk_len(const tpe_ctx* ctx, int nch) {
    int32_t na_max = 1;
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : ctx->P->h_group[m]) na_max = std::max(na_max, ctx->P->h_labels[li].na);
    return ctx->chunks_forced ? (na_max + nch - 1) / nch : kChunkLen;
}

// nb + na summed over the dense labels: the terms an unwindowed screen sums
// per candidate index (one candidate per dense label)
int64_t dense_terms(const tpe_ctx* ctx) {
    int64_t t = 0;
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : ctx->P->h_group[m]) t += ctx->P->h_labels[li].nb + ctx->P->h_labels[li].na;
    return t;
}

// tile-map rounds with at least this many candidates use the windowed screen
constexpr int64_t kWinMinN = 8192;
// TPE_OPT_WIN_GROUPS > 1 splits a batch into label groups, each sorted on
// the aux stream while the previous group is screened.  Off by default: the
// chip is busy either way (config 3: 47.6 ms in one group, 47.1 in 2, 47.1
// in 4, 47.2 in 8), and one group keeps k_screen_win's own time clean.

// Packed-map sampled rounds of the dense labels, screened (see
// k_pick_packed): fp32 chunk sums, per-round selection, fp64 re-score with
// the chunked map's summation order, per-round pick.
int launch_screen_packed(tpe_ctx* ctx, const int32_t* grp, int nl, int nch, const RoundArgs& a) {
    const int32_t chunk = dense_chunk_len(ctx, nch);
    // the fp32 pass and the pick use their own, wider slot map: kScreenR
    // candidates per thread (whole rounds per workgroup, as the packed map);
    // the chunks stay those of the fp64 packed map, which the re-score repeats
    Slots S8{(int32_t)a.n, (int32_t)((kScreenR * kBlock) / a.n), a.n_rounds};
    const uint32_t gx8 = (uint32_t)((a.n_rounds + S8.rpb - 1) / S8.rpb);
    const size_t planes = (size_t)nl * (nch + 2) * gx8 * (kScreenR * kBlock);
    const int64_t cap = (int64_t)a.n_rounds * a.n;   // candidate slots per label
    HIPCHK(ctx, ctx->scr_list.reserve((size_t)nl * cap));
    HIPCHK(ctx, ctx->scr_rsel.reserve((size_t)a.n_rounds * nl));
    HIPCHK(ctx, ctx->scr_cnt.reserve(nl));
    HIPCHK(ctx, hipMemsetAsync(ctx->scr_cnt.p, 0, nl * sizeof(int32_t), ctx->stream));
    RoundSel* rsel = reinterpret_cast<RoundSel*>(ctx->scr_rsel.p);
    bool use_bx = false;
    if (ctx->expand && cap >= kWinMinN && a.n <= kBxR * kBlock) {
        ctx->bx_t_next = kBxT;   // (the packed map: value-only certification)
        int rc = tpe_rt::bx_prepare(ctx);
        if (rc) return rc;
        use_bx = ctx->P->bx_ok;
    }
    if (use_bx) {
        // expansion screen: fp64 (lower, upper) bounds per candidate over a
        // packed slot map of kBxR candidates per thread, then the per-round
        // selection -- ~1 candidate per (round, label) left to re-score
        tpe_rt::Posterior& P = *ctx->P;
        ctx->screen_mode = 3;
        HIPCHK(ctx, ctx->win_evals.reserve(1));
        HIPCHK(ctx, hipMemsetAsync(ctx->win_evals.p, 0, sizeof(unsigned long long), ctx->stream));
        HIPCHK(ctx, ctx->bx_lohi.reserve((size_t)nl * cap));
        const Slots Sb{(int32_t)a.n, (int32_t)((kBxR * kBlock) / a.n), a.n_rounds};
        const uint32_t gxb = (uint32_t)((a.n_rounds + Sb.rpb - 1) / Sb.rpb);
        if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[0], ctx->stream));
        hipLaunchKernelGGL((k_screen_bx<kBxR, true>), dim3(gxb, nl, 1), dim3(kBlock), 0, ctx->stream,
                           P.labels.p, grp, P.comps64.p, P.samp.p, P.bx.p, P.bx_tab.p, P.bx_loff.p,
                           P.bx_list.p, a.n, a.cand_offset, a.seed, ctx->rounds.p, nl, nullptr, nullptr,
                           nullptr, nullptr, ctx->win_evals.p, ctx->errflag.p, Sb, nullptr, nullptr, nullptr,
                           ctx->bx_lohi.p, (int64_t)0);
        if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[1], ctx->stream));
        hipLaunchKernelGGL(k_pick_win<double2>, dim3((unsigned)((a.n_rounds + kBlock - 1) / kBlock), nl),
                           dim3(kBlock), 0, ctx->stream, ctx->bx_lohi.p, a.n_rounds, (int32_t)a.n,
                           ctx->scr_cnt.p, ctx->scr_list.p, cap, rsel, nl, ctx->value_only ? 1 : 0);
        HIPCHK(ctx, hipMemcpyAsync(&ctx->pin[0].screen_exec, ctx->win_evals.p, sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, ctx->stream));
        ctx->screen_exec_pending = true;
    } else if (ctx->window && cap >= kWinMinN && (int64_t)nl * cap <= ((int64_t)1 << 30)) {
        // windowed: every round's candidates of a label sorted together into
        // tiles of neighbours (tpe_window.hip), bounds per candidate, then
        // the per-round selection
        int rc = tpe_rt::win_prepare(ctx);
        if (rc) return rc;
        HIPCHK(ctx, ctx->win_evals.reserve(1));
        HIPCHK(ctx, hipMemsetAsync(ctx->win_evals.p, 0, sizeof(unsigned long long), ctx->stream));
        HIPCHK(ctx, ctx->win_lohi.reserve((size_t)nl * cap));
        const uint64_t* sorted = nullptr;
        tpe_rt::WinScreenArgs wa{grp, nl, a.n, a.cand_offset, a.seed, 0, a.n_rounds, nullptr,
                                 nullptr, nullptr, nullptr, nullptr, (int32_t)a.n, ctx->win_lohi.p};
        if ((rc = tpe_rt::win_screen(ctx, wa, &sorted))) return rc;
        hipLaunchKernelGGL(k_pick_win<float2>, dim3((unsigned)((a.n_rounds + kBlock - 1) / kBlock), nl),
                           dim3(kBlock), 0, ctx->stream, ctx->win_lohi.p, a.n_rounds, (int32_t)a.n,
                           ctx->scr_cnt.p, ctx->scr_list.p, cap, rsel, nl, ctx->value_only ? 1 : 0);
        HIPCHK(ctx, hipMemcpyAsync(&ctx->pin[0].screen_exec, ctx->win_evals.p, sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, ctx->stream));
        ctx->screen_exec_pending = true;
    } else {
        HIPCHK(ctx, ctx->chunk_part.reserve(planes));
        if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[0], ctx->stream));
        hipLaunchKernelGGL((k_round_chunk<float, kScreenR>), dim3(gx8, nl, nch), dim3(kBlock), 0,
                           ctx->stream, ctx->P->labels.p, grp, ctx->P->comps32.p, ctx->P->samp.p, a.n,
                           a.cand_offset, a.seed, ctx->rounds.p, chunk, ctx->chunk_part.p, ctx->errflag.p,
                           S8);
        if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[1], ctx->stream));
        hipLaunchKernelGGL((k_pick_packed<kScreenR>), dim3(gx8, nl), dim3(kBlock), 0, ctx->stream,
                           ctx->P->labels.p, grp, a.n, nl, nch, chunk, ctx->chunk_part.p, ctx->scr_cnt.p,
                           ctx->scr_list.p, cap, rsel, S8);
        ctx->screen_exec += (int64_t)a.n_rounds * a.n * dense_terms(ctx);
    }
    // the re-score planned on the device (no mid-round read-back): per
    // label chunks of kRP * 256 listed candidates, buffers for pk_cap of
    // them (a round listing more runs again with larger ones)
    HIPCHK(ctx, ctx->scr_cnt_h.resize(nl));
    HIPCHK(ctx, hipMemcpyAsync(ctx->scr_cnt_h.data(), ctx->scr_cnt.p, nl * sizeof(int32_t),
                               hipMemcpyDeviceToHost, ctx->stream));
    constexpr int64_t per = (int64_t)kRP * kBlock;
    const int64_t pcap = std::max<int64_t>(1, std::min<int64_t>(ctx->pk_cap, (int64_t)nl * cap));
    const int64_t ne_max = nl + (pcap + per - 1) / per;
    // a few listed candidates: sliced (k_rescore_slices_packed), entries of
    // kRsW candidates, s_max slices each
    const int64_t sl_max = std::min<int64_t>(ctx->pk_sliced, pcap);
    const int64_t ne_sl = sl_max > 0 ? nl + (sl_max + kRsW - 1) / kRsW : 0;
    const int32_t spc = (chunk + kSumSlice - 1) / kSumSlice;
    int32_t s_max = 0;
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : ctx->P->h_group[m])
            s_max = std::max(s_max, (ctx->P->h_labels[li].nb + kSumSlice - 1) / kSumSlice + nch * spc);
    HIPCHK(ctx, ctx->scr_res.reserve(pcap));
    HIPCHK(ctx, ctx->scr_off.reserve(nl + 1));
    HIPCHK(ctx, ctx->scr_chunks.reserve(std::max(ne_max, ne_sl)));
    if (ne_sl > 0) {
        HIPCHK(ctx, ctx->rs_x.reserve((size_t)ne_sl * kRsW));
        HIPCHK(ctx, ctx->rs_g.reserve((size_t)ne_sl * kRsW));
        HIPCHK(ctx, ctx->rs_part.reserve((size_t)ne_sl * s_max * kRsW));
    }
    HIPCHK(ctx, ctx->scr_range.reserve(nl));
    HIPCHK(ctx, ctx->scr_planes.reserve((size_t)(nch + 2) * pcap));
    HIPCHK(ctx, ctx->rs_plan.reserve(3));
    RescoreChunk* tabd = reinterpret_cast<RescoreChunk*>(ctx->scr_chunks.p);
    RescorePlan* plan = reinterpret_cast<RescorePlan*>(ctx->rs_plan.p);
    hipLaunchKernelGGL(k_rescore_plan, dim3(1), dim3(kPlanBlock), 0, ctx->stream, ctx->scr_cnt.p, (int64_t)nl,
                       (int32_t)per, sl_max, pcap, tabd, ctx->scr_range.p, ctx->scr_off.p, plan);
    HIPCHK(ctx, hipMemcpyAsync(&ctx->pin[0].plan, plan, sizeof(RescorePlan), hipMemcpyDeviceToHost, ctx->stream));
    ctx->pk_plan_pending = true;
    {
        tpe_rt::Posterior& P = *ctx->P;
        if (ctx->zero_win && !P.zw_ready) {   // once per posterior
            HIPCHK(ctx, P.zw_hi.reserve(P.comps64.cap));
            HIPCHK(ctx, P.zw_lo.reserve(P.comps64.cap));
            HIPCHK(ctx, P.zw_wide.reserve(P.comps64.cap));
            HIPCHK(ctx, P.zw_n.reserve(std::max(P.n_labels, 1)));
            // every dense label of the posterior (the GMM1 and LGMM1 groups are adjacent)
            const int nd = (int)(P.h_group[DENSE_GMM].size() + P.h_group[DENSE_LGMM].size());
            hipLaunchKernelGGL(k_zero_windows, dim3((unsigned)nd), dim3(kZwBlock), 0, ctx->stream, plan, P.labels.p,
                               P.groups.p + P.group_off[DENSE_GMM], P.comps64.p, P.zw_hi.p, P.zw_lo.p,
                               P.zw_wide.p, P.zw_n.p);
            ctx->zw_pending = true;   // built iff the plan was chunked (read after the round's sync)
        }
        if (ne_sl > 0) {
            // (zero windows only when an earlier round of this posterior
            // built them: k_zero_windows skips a sliced plan -- 0.67 ms at
            // config 5, more than the slices it would let a re-score skip)
            const bool zw = ctx->zero_win && P.zw_ready;
            HIPCHK(ctx, ctx->rs_win.reserve((size_t)2 * ne_sl));
            const unsigned g_sl = (unsigned)std::min<int64_t>(ne_sl, 1024);
            hipLaunchKernelGGL(k_rescore_draw_packed, dim3((unsigned)((ne_sl + kBlock / kRsW - 1) / (kBlock / kRsW))),
                               dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.samp.p, a.cand_offset, a.seed,
                               ctx->rounds.p, plan, ctx->scr_cnt.p, ctx->scr_list.p, cap, tabd, ctx->rs_x.p,
                               ctx->rs_g.p, zw ? P.zw_hi.p : nullptr, zw ? P.zw_lo.p : nullptr, ctx->rs_win.p);
            hipLaunchKernelGGL(k_rescore_slices_packed, dim3((unsigned)((s_max + 3) / 4), g_sl), dim3(kBlock), 0,
                               ctx->stream, P.labels.p, grp, P.comps64.p, tabd, plan, ctx->rs_x.p, s_max, chunk,
                               spc, ctx->rs_part.p, zw ? ctx->rs_win.p : nullptr, P.zw_wide.p, P.zw_n.p);
            hipLaunchKernelGGL(k_rescore_fin_packed, dim3(g_sl), dim3(kRsW), 0, ctx->stream, P.labels.p, grp,
                               P.comps64.p, a.cand_offset, nch, spc, ctx->scr_list.p, cap, tabd, ctx->scr_off.p,
                               plan, ctx->rs_x.p, ctx->rs_g.p, s_max, ctx->rs_part.p, ctx->scr_res.p);
        }
        const unsigned g = (unsigned)std::min<int64_t>(ne_max, 2048);
        hipLaunchKernelGGL((k_rescore_packed<kRP>), dim3(g, nch), dim3(kBlock), 0,
                           ctx->stream, ctx->P->labels.p, grp, ctx->P->comps64.p, ctx->P->samp.p,
                           a.cand_offset, a.seed, ctx->rounds.p, chunk, ctx->scr_cnt.p,
                           ctx->scr_list.p, cap, tabd, ctx->scr_off.p, plan, pcap, ctx->scr_planes.p,
                           ctx->zero_win ? P.zw_hi.p : nullptr, ctx->zero_win ? P.zw_lo.p : nullptr,
                           P.zw_wide.p, P.zw_n.p);
        hipLaunchKernelGGL(k_finish_rescore, dim3(g), dim3(kBlock), 0, ctx->stream,
                           ctx->P->labels.p, grp, ctx->P->comps64.p, a.cand_offset, nch, ctx->scr_cnt.p,
                           ctx->scr_list.p, cap, tabd, ctx->scr_off.p, plan, pcap, ctx->scr_planes.p,
                           ctx->scr_res.p);
    }
    const int64_t cells = (int64_t)a.n_rounds * nl;
    hipLaunchKernelGGL(k_pick_rounds, dim3((unsigned)((cells + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, ctx->P->labels.p, grp, nl, a.n_rounds, ctx->P->n_labels, rsel, ctx->scr_res.p,
                       ctx->scr_off.p, plan, ctx->P->samp.p, a.cand_offset, a.seed, ctx->rounds.p,
                       ctx->partials.p);
    ctx->screen_total += cells * a.n;
    ctx->screen_pending = true;
    return ctx->hip(hipGetLastError(), "packed screen launch");
}

// Sampled rounds: the dense GMM1 and LGMM1 labels in ONE launch (their
// groups are adjacent), so both families fill the chip together instead of
// leaving each other's tail idle.  Timed and counted in the DENSE_GMM slot.
// the expansion screen over every candidate of a sampled tile-map round
void screen_bx_all(tpe_ctx* ctx, const int32_t* grp, int nl, const RoundArgs& a) {
    tpe_rt::Posterior& P = *ctx->P;
    const unsigned bgx = (unsigned)((a.n + kBxR * kBlock - 1) / (kBxR * kBlock));
    hipLaunchKernelGGL((k_screen_bx<kBxR, true>), dim3(bgx, nl, a.gz), dim3(kBlock), 0, ctx->stream, P.labels.p,
                       grp, P.comps64.p, P.samp.p, P.bx.p, P.bx_tab.p, P.bx_loff.p, P.bx_list.p, a.n,
                       a.cand_offset, a.seed, ctx->rounds.p, nl, ctx->scr_hid.p, ctx->scr_lb.p, ctx->scr_cnt.p,
                       ctx->scr_idx.p, ctx->win_evals.p, ctx->errflag.p, a.S, nullptr, nullptr, nullptr, nullptr,
                       a.n);
}

// The hot-bin prefilter's listing threshold tau0 and its sub-bin bits for
// rounds of n candidates per label: a function of the posterior's index and
// n only, kept across rounds (and built ahead by tpe_prepare).
int hot_tau_prepare(tpe_ctx* ctx, int64_t n) {
    tpe_rt::Posterior& P = *ctx->P;
    const int nl = (int)(P.h_group[DENSE_GMM].size() + P.h_group[DENSE_LGMM].size());
    if (nl == 0 || !P.bx_ok || !P.bx_sb.p) return TPE_OK;
    const int32_t* grp = P.groups.p + P.group_off[DENSE_GMM];
    if (ctx->hot_tau0.cap < (size_t)nl) ctx->hot_tau0_gen = 0;   // (re)allocated: recompute
    HIPCHK(ctx, ctx->hot_tau0.reserve(nl));
    if (ctx->hot_tau0_gen == P.bx_gen && ctx->hot_tau0_n == n && ctx->hot != 2) return TPE_OK;
    HIPCHK(ctx, ctx->hot_bits.reserve((size_t)(P.bx_sb.cap + 31) / 32));
    HIPCHK(ctx, hipMemsetAsync(ctx->hot_tau0.p, 0, nl * sizeof(unsigned long long), ctx->stream));
    const unsigned sbw = (unsigned)std::min<int64_t>((P.bx_sb_max + kBlock - 1) / kBlock,
                                                     std::max<int64_t>(1, kHotPrepWgs / nl));
    hipLaunchKernelGGL(k_hot_tau0, dim3(sbw, nl), dim3(kBlock), 0,
                       ctx->stream, grp, P.bx.p, P.bx_sb.p, P.bx_sbp.p, (float)(kHotFill / (double)n),
                       ctx->hot_tau0.p);
    if (ctx->hot == 2)   // test mode: a threshold no candidate reaches -> the fallback
        HIPCHK(ctx, hipMemsetAsync(ctx->hot_tau0.p, 0xff, nl * sizeof(unsigned long long), ctx->stream));
    hipLaunchKernelGGL(k_hot_bits, dim3(sbw, nl), dim3(kBlock), 0,
                       ctx->stream, grp, P.bx.p, P.bx_sb.p, ctx->hot_tau0.p, ctx->hot_bits.p);
    // the sampling components' u-cells (k_hot_bx decides most candidates from them)
    HIPCHK(ctx, ctx->hot_pc.reserve((size_t)(P.bx_sb.cap + 31) / 32));
    HIPCHK(ctx, ctx->hot_ucell.reserve((size_t)nl * kSampLds * kHotCellWords));
    hipLaunchKernelGGL(k_hot_prefix, dim3((unsigned)nl), dim3(1024), 0, ctx->stream, grp, P.bx.p, ctx->hot_bits.p,
                       ctx->hot_pc.p);
    int32_t ns_max = 1;   // (workgroups past a label's ns exit at once; none past the largest)
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : P.h_group[m]) ns_max = std::max(ns_max, std::min(P.h_labels[li].ns, kSampLds));
    hipLaunchKernelGGL(k_hot_ucells, dim3(kHotCells / kBlock, ns_max, nl), dim3(kBlock), 0, ctx->stream, P.labels.p,
                       grp, P.samp.p, P.bx.p, ctx->hot_bits.p, ctx->hot_pc.p, ctx->hot_ucell.p);
    bool staged = true;   // (k_hot_bx runs only when every dense label's records fit in LDS)
    for (int m : {DENSE_GMM, DENSE_LGMM})
        for (int li : P.h_group[m]) staged = staged && P.h_labels[li].ns >= 1 && P.h_labels[li].ns <= kSampLds;
    if (staged) {
        HIPCHK(ctx, ctx->samp_img.reserve((size_t)nl * kSampImgVec));
        hipLaunchKernelGGL(k_samp_image, dim3((unsigned)nl), dim3(kBlock), 0, ctx->stream, P.labels.p, grp, P.samp.p,
                           ctx->samp_img.p);
    }
    ctx->hot_tau0_gen = ctx->hot == 2 ? 0 : P.bx_gen;
    ctx->hot_tau0_n = n;
    return ctx->hip(hipGetLastError(), "hot-bin threshold launch");
}

// Per-cell capacity of the hot-bin prefilter's lists (and of the expansion
// screen's appends from them): a fraction of the round, grown after an
// overflow (which makes that round screen every candidate instead)
constexpr int64_t kHotMinCap = 1 << 12;
int64_t hot_stride(const tpe_ctx* ctx, int64_t n) {
    return std::min<int64_t>(n, std::max<int64_t>(kHotMinCap, (int64_t)((double)n / ctx->hot_cap_div)));
}

// the re-score's table, plan and sliced buffers for `cells` lists of up
// to lst candidates
int rescore_reserve(tpe_ctx* ctx, size_t cells, int64_t lst, int32_t s_max) {
    const int64_t per_full = (int64_t)kRescoreR * kBlock;
    const int64_t ne_sliced = (int64_t)cells + kSlicedRescoreMax / kRsW;
    const int64_t ne_full = (int64_t)cells + ((int64_t)cells * lst + per_full - 1) / per_full;
    const int64_t ne_cap = std::max(ne_sliced, ne_full);
    HIPCHK(ctx, ctx->scr_chunks.reserve(ne_cap));
    HIPCHK(ctx, ctx->scr_res.reserve(ne_cap));
    HIPCHK(ctx, ctx->scr_off.reserve(cells));
    HIPCHK(ctx, ctx->rs_plan.reserve(3));   // (RescorePlan: 24 B)
    HIPCHK(ctx, ctx->rs_x.reserve((size_t)ne_sliced * kRsW));
    HIPCHK(ctx, ctx->rs_g.reserve((size_t)ne_sliced * kRsW));
    HIPCHK(ctx, ctx->rs_part.reserve((size_t)ne_sliced * s_max * kRsW));
    return TPE_OK;
}

template <typename T>
int launch_dense(tpe_ctx* ctx, const Groups& g, const RoundArgs& a) {
    const int nl = g.count[DENSE_GMM] + g.count[DENSE_LGMM];
    if (nl == 0 || a.tiles == 0) return TPE_OK;
    bracket(ctx, DENSE_GMM, 0);
    const Comp<T>* comps;
    if constexpr (sizeof(T) == 8) comps = ctx->P->comps64.p; else comps = ctx->P->comps32.p;
    const int32_t* grp = ctx->P->groups.p + ctx->P->group_off[DENSE_GMM];
    const int nch = a.S.cpack ? dense_chunks(ctx) : 1;
    if (sizeof(T) == 8 && ctx->screen && a.S.cpack == 0) {   // fp32 screen + fp64 re-score
        const size_t cells = (size_t)a.n_rounds * nl;
        bool use_bx = false, hot = false, plan_done = false;
        ctx->hot_ran = false;
        ctx->hot_listed = 0;
        ctx->hot_fallback = 0;
        if (ctx->expand && a.n >= kWinMinN && a.cand_in == nullptr) {
            ctx->bx_t_next = kBxTTile;   // (tile rounds: the hot-bin prefilter)
            int rc = tpe_rt::bx_prepare(ctx);
            if (rc) return rc;
            use_bx = ctx->P->bx_ok;
        }
        hot = use_bx && ctx->hot != 0 && ctx->P->bx_sb.p != nullptr && !ctx->hot_redo;
        for (int m : {DENSE_GMM, DENSE_LGMM})   // k_hot_bx stages every label's sampling records
            for (int li : ctx->P->h_group[m]) hot = hot && ctx->P->h_labels[li].ns >= 1 && ctx->P->h_labels[li].ns <= kSampLds;
        // the expansion screen's appends: a cell's hot list at most (the
        // prefilter), else any candidate of the round
        int64_t lst = hot ? hot_stride(ctx, a.n) : a.n;
        if (use_bx) HIPCHK(ctx, ctx->scr_hid.reserve(cells * lst));
        else HIPCHK(ctx, ctx->scr_hi.reserve(cells * a.n));
        HIPCHK(ctx, ctx->scr_idx.reserve(cells * lst));
        HIPCHK(ctx, ctx->scr_lb.reserve(cells));
        HIPCHK(ctx, ctx->scr_cnt.reserve(cells));
        FillSet fs{};
        add_fill(fs, ctx->scr_lb.p, cells * sizeof(unsigned long long), 0);
        add_fill(fs, ctx->scr_cnt.p, cells * sizeof(int32_t), 0);
        // the tail's last-workgroup counters (k_select_plan, k_rescore_fin)
        // and the hot list's item counter (k_hot_bx's last workgroup)
        HIPCHK(ctx, ctx->rs_done.reserve(4));
        add_fill(fs, ctx->rs_done.p, 4 * sizeof(uint32_t), 0);
        // the re-score's buffers, planned on the device from the counts:
        // sliced for a few near-ties, chunks of kRescoreR * 256 otherwise
        // (sized for the largest table either plan can make)
        int32_t s_max = 1;
        for (int m : {DENSE_GMM, DENSE_LGMM})
            for (int li : ctx->P->h_group[m]) {
                const DLabel& d = ctx->P->h_labels[li];
                s_max = std::max(s_max, (d.nb + kSumSlice - 1) / kSumSlice + (d.na + kSumSlice - 1) / kSumSlice);
            }
        const unsigned sx = (unsigned)std::min<int64_t>((a.n + 8 * kBlock - 1) / (8 * kBlock), 1024);
        ctx->screen_mode = use_bx ? 3 : (ctx->window && a.n >= kWinMinN && a.cand_in == nullptr) ? 2 : 1;
        if (!use_bx) {   // the expansion screen adds its own resets to the same launch
            const int rc = run_fills(ctx, fs);
            if (rc) return rc;
        }
        if (use_bx) {
            // expansion screen: no sort, ~1e-12 bounds, near-ties re-scored
            tpe_rt::Posterior& P = *ctx->P;
            HIPCHK(ctx, ctx->win_evals.reserve(1));
            add_fill(fs, ctx->win_evals.p, sizeof(unsigned long long), 0);
            if (hot) {
                HIPCHK(ctx, ctx->hot_x.reserve(cells * lst));
                HIPCHK(ctx, ctx->hot_i.reserve(cells * lst));
                HIPCHK(ctx, ctx->hot_cnt.reserve(cells));
                HIPCHK(ctx, ctx->hot_t.reserve(cells));
                HIPCHK(ctx, ctx->hot_flag.reserve(1));
                add_fill(fs, ctx->hot_cnt.p, cells * sizeof(int32_t), 0);
                add_fill(fs, ctx->hot_t.p, cells * sizeof(unsigned long long), 0);
                add_fill(fs, ctx->hot_flag.p, sizeof(int32_t), 0);
            }
            {
                const int rc = run_fills(ctx, fs);
                if (rc) return rc;
            }
            if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[0], ctx->stream));
            if (hot) {
                // hot-bin prefilter: draw + sub-bin bounds, then the
                // expansion screen over the listed candidates only
                {
                    const int rc = hot_tau_prepare(ctx, a.n);
                    if (rc) return rc;
                }
                const int64_t cells_l = (int64_t)nl * a.gz;
                // workgroups per cell (tiles strided): at most one per tile and
                // kHotBxWgs over the round; at least kHotMinTiles tiles each
                // (a workgroup stages its tables first: a label shard's few
                // cells at one or two tiles per workgroup ran 0.54 ms instead
                // of 0.46) unless the chip needs more to fill it
                const int64_t hr = kHotR;
                const int64_t tiles_c = (a.n + hr * kBlock - 1) / (hr * kBlock);
                const int64_t per_cell = std::min<int64_t>(
                    {tiles_c, kHotBxWgs / cells_l,
                     std::max<int64_t>((kHotFillWgs + cells_l - 1) / cells_l, tiles_c / kHotMinTiles)});
                const dim3 hg((unsigned)std::max<int64_t>(1, per_cell), nl, a.gz);
                HIPCHK(ctx, ctx->hot_items.reserve((size_t)cells + 2));
                int32_t ns_max = 1;
                for (int m : {DENSE_GMM, DENSE_LGMM})
                    for (int li : ctx->P->h_group[m]) ns_max = std::max(ns_max, ctx->P->h_labels[li].ns);
                const size_t ucw_bytes = (size_t)ns_max * kHotCellWords * sizeof(uint32_t);
                // the mark lists: a segment per k_hot_bx workgroup, sized like
                // the hot lists (n / hot_cap_div of its candidates; marked ~1.2x
                // listed)
                const int64_t segs = (int64_t)hg.x;
                const int64_t mcap = std::max<int64_t>(
                    1024, (int64_t)((double)((tiles_c + segs - 1) / segs * hr * kBlock) / ctx->hot_cap_div));
                HIPCHK(ctx, ctx->hot_mi.reserve(cells * segs * mcap));
                HIPCHK(ctx, ctx->hot_mcnt.reserve(cells * segs));
                hipLaunchKernelGGL((k_hot_bx<kHotR>), hg, dim3(kBlock), ucw_bytes, ctx->stream, P.labels.p, grp,
                                   ctx->samp_img.p, ctx->hot_ucell.p, a.n, a.cand_offset, a.seed, ctx->rounds.p, nl,
                                   ctx->hot_mcnt.p, ctx->hot_mi.p, mcap, ctx->hot_flag.p);
                // (the screen's bracket: the mark kernel alone -- the roofline's kernel)
                if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[1], ctx->stream));
                // the exact draw of the marked: a workgroup per mark segment, at
                // most kHotDrawWgs over the round
                const int64_t dw = std::max<int64_t>(
                    (segs + kDrawSegs - 1) / kDrawSegs,
                    std::max<int64_t>(1, std::min<int64_t>(segs, kHotDrawWgs / (int64_t)cells)));
                hipLaunchKernelGGL(k_hot_draw, dim3((unsigned)dw, (unsigned)cells), dim3(kBlock), 0, ctx->stream,
                                   P.labels.p, grp, ctx->samp_img.p, P.bx.p, ctx->hot_bits.p, a.cand_offset, a.seed,
                                   ctx->rounds.p, nl, ctx->hot_mcnt.p, (int32_t)segs, ctx->hot_mi.p, mcap,
                                   ctx->hot_cnt.p, ctx->hot_i.p, ctx->hot_x.p, ctx->errflag.p, lst, ctx->hot_flag.p);
                hipLaunchKernelGGL(k_hot_items, dim3(1), dim3(1024), 0, ctx->stream, ctx->hot_cnt.p, (int64_t)cells, lst,
                                   (int64_t)kBxR * kBlock, ctx->hot_items.p);
                const int64_t items_max = (int64_t)cells * ((lst + (int64_t)kBxR * kBlock - 1) / ((int64_t)kBxR * kBlock));
                hipLaunchKernelGGL((k_screen_hot<kBxR>), dim3((unsigned)std::max<int64_t>(1, items_max)), dim3(kBlock), 0,
                                   ctx->stream,
                                   P.labels.p, grp, P.comps64.p, P.bx.p, P.bx_tab.p, P.bx_loff.p, P.bx_list.p, a.n,
                                   nl, (int64_t)cells, ctx->hot_items.p, ctx->hot_items.p + cells + 1,
                                   ctx->hot_cnt.p, ctx->hot_i.p, ctx->hot_x.p, ctx->scr_hid.p, ctx->scr_lb.p,
                                   ctx->scr_cnt.p, ctx->scr_idx.p, ctx->win_evals.p, P.bx_sb.p, ctx->hot_t.p, lst);
            } else {
                screen_bx_all(ctx, grp, nl, a);
                if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[1], ctx->stream));
            }
            {
                const int rc = rescore_reserve(ctx, cells, lst, s_max);
                if (rc) return rc;
            }
            hipLaunchKernelGGL(k_select_plan, dim3((unsigned)cells), dim3(kBlock), 0, ctx->stream, ctx->scr_hid.p,
                               lst, ctx->scr_lb.p, ctx->scr_cnt.p, ctx->scr_idx.p, hot ? ctx->hot_t.p : nullptr,
                               ctx->hot_tau0.p, nl, ctx->hot_flag.p, ctx->rs_done.p, (int32_t)(kRescoreR * kBlock),
                               kSlicedRescoreMax, (int64_t)cells * lst,
                               reinterpret_cast<RescoreChunk*>(ctx->scr_chunks.p), ctx->scr_off.p,
                               reinterpret_cast<RescorePlan*>(ctx->rs_plan.p));
            plan_done = true;
            if (hot) {
                HIPCHK(ctx, ctx->hot_cnt_h.resize(cells));
                int rc = defer_read(ctx, ctx->hot_cnt_h.data(), ctx->hot_cnt.p, cells * sizeof(int32_t));
                if (!rc) rc = defer_read(ctx, &ctx->pin[0].hot_flag, ctx->hot_flag.p, sizeof(int32_t));
                if (rc) return rc;
            }
            {
                const int rc = defer_read(ctx, &ctx->pin[0].screen_exec, ctx->win_evals.p, sizeof(unsigned long long));
                if (rc) return rc;
            }
            ctx->screen_exec_pending = true;
        } else if (ctx->window && a.n >= kWinMinN && a.cand_in == nullptr) {
            // windowed: units of (batch of rounds, group of labels); with
            // several units each is keyed and sorted on the aux stream into
            // one of two buffer slots while the main stream screens and
            // selects the previous one
            int rc = tpe_rt::win_prepare(ctx);
            if (rc) return rc;
            HIPCHK(ctx, ctx->win_evals.reserve(1));
            HIPCHK(ctx, hipMemsetAsync(ctx->win_evals.p, 0, sizeof(unsigned long long), ctx->stream));
            struct Unit {
                int32_t z0, nz, y0, ny;
            };
            std::vector<Unit> units;
            const int32_t zb = (int32_t)tpe_rt::win_rounds_per_batch(a.n, nl);
            // label groups only when a batch is big enough to hide its sort
            const int32_t ng = ctx->win_groups > 0 ? std::min<int32_t>(ctx->win_groups, nl) : 1;
            size_t max_total = 0;
            int64_t max_cells = 1;
            for (int32_t z0 = 0; z0 < a.n_rounds; z0 += zb)
                for (int32_t g = 0; g < ng; ++g) {
                    const int32_t y0 = (int32_t)((int64_t)nl * g / ng), y1 = (int32_t)((int64_t)nl * (g + 1) / ng);
                    const Unit u{z0, std::min(zb, a.n_rounds - z0), y0, y1 - y0};
                    units.push_back(u);
                    max_total = std::max(max_total, (size_t)u.nz * u.ny * a.n);
                    max_cells = std::max<int64_t>(max_cells, (int64_t)u.nz * u.ny);
                }
            const int nslots = units.size() > 1 ? 2 : 1;
            if ((rc = tpe_rt::win_reserve(ctx, max_total, max_cells, nslots))) return rc;
            const size_t nev = 2 * units.size();
            while (ctx->evw.size() < nev) {
                hipEvent_t e;
                HIPCHK(ctx, hipEventCreate(&e));
                ctx->evw.push_back(e);
            }
            ctx->evw_used = ctx->timing ? (int32_t)units.size() : 0;
            const bool pipe = units.size() > 1;
            if (pipe) {   // the aux stream starts after this round's setup on the main one
                HIPCHK(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
                HIPCHK(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
            }
            for (size_t ui = 0; ui < units.size(); ++ui) {
                const Unit& u = units[ui];
                const int slot = (int)(ui & 1);
                tpe_rt::WinScreenArgs wa{grp + u.y0, u.ny, a.n, a.cand_offset, a.seed, u.z0, u.nz, nullptr,
                                         ctx->scr_hi.p, ctx->scr_lb.p, nullptr, nullptr};
                wa.y0 = u.y0;
                wa.nl_all = nl;
                wa.slot = slot;
                const uint64_t* sorted = nullptr;
                if (pipe) {
                    // the slot's previous unit must be screened and selected first
                    if (ui >= 2) HIPCHK(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_done[slot], 0));
                    if ((rc = tpe_rt::win_sort(ctx, wa, ctx->aux, &sorted))) return rc;
                    HIPCHK(ctx, hipEventRecord(ctx->ev_sorted[slot], ctx->aux));
                    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_sorted[slot], 0));
                } else if ((rc = tpe_rt::win_sort(ctx, wa, ctx->stream, &sorted))) {
                    return rc;
                }
                if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evw[2 * ui], ctx->stream));
                if ((rc = tpe_rt::win_tiles(ctx, wa, sorted, ctx->stream))) return rc;
                if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evw[2 * ui + 1], ctx->stream));
                hipLaunchKernelGGL(k_select<float>, dim3(sx, u.ny, u.nz), dim3(kBlock), 0, ctx->stream, ctx->scr_hi.p,
                                   a.n, nl, ctx->scr_lb.p, ctx->scr_cnt.p, ctx->scr_idx.p, u.z0, u.y0, u.ny,
                                   sorted);
                if (pipe) HIPCHK(ctx, hipEventRecord(ctx->ev_done[slot], ctx->stream));
            }
            {
                const int rc = defer_read(ctx, &ctx->pin[0].screen_exec, ctx->win_evals.p, sizeof(unsigned long long));
                if (rc) return rc;
            }
            ctx->screen_exec_pending = true;
        } else {
            if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[0], ctx->stream));
            const unsigned sgx = (unsigned)((a.n + kScreenR * kBlock - 1) / (kScreenR * kBlock));
            hipLaunchKernelGGL((k_screen<kScreenR, true>), dim3(sgx, nl, a.gz), dim3(kBlock), 0, ctx->stream,
                               ctx->P->labels.p, grp, ctx->P->comps32.p, ctx->P->samp.p, a.n,
                               a.cand_offset, a.seed, ctx->rounds.p, nl, ctx->scr_hi.p, ctx->scr_lb.p,
                               ctx->errflag.p, a.S, nullptr, nullptr, nullptr);
            if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->evs[1], ctx->stream));
            hipLaunchKernelGGL(k_select<float>, dim3(sx, nl, a.gz), dim3(kBlock), 0, ctx->stream, ctx->scr_hi.p,
                               a.n, nl, ctx->scr_lb.p, ctx->scr_cnt.p, ctx->scr_idx.p, 0, 0, nl, nullptr);
            ctx->screen_exec += (int64_t)a.n_rounds * a.n * dense_terms(ctx);
        }
        HIPCHK(ctx, ctx->scr_cnt_h.resize(cells));
        {
            const int rc = defer_read(ctx, ctx->scr_cnt_h.data(), ctx->scr_cnt.p, cells * sizeof(int32_t));
            if (rc) return rc;
        }
        if (hot) {
            ctx->hot_ran = true;   // (its lists and flag are read after the round's one sync)
            ctx->hot_cells = (int64_t)cells;
        }
        const int64_t per_full = (int64_t)kRescoreR * kBlock;
        const int64_t ne_sliced = (int64_t)cells + kSlicedRescoreMax / kRsW;
        const int64_t ne_full = (int64_t)cells + ((int64_t)cells * lst + per_full - 1) / per_full;
        RescoreChunk* chp = reinterpret_cast<RescoreChunk*>(ctx->scr_chunks.p);
        RescorePlan* plan = reinterpret_cast<RescorePlan*>(ctx->rs_plan.p);
        if (!plan_done) {   // (the windowed and fp32 screens' k_select: the plan on its own)
            const int rc = rescore_reserve(ctx, cells, lst, s_max);
            if (rc) return rc;
            chp = reinterpret_cast<RescoreChunk*>(ctx->scr_chunks.p);
            plan = reinterpret_cast<RescorePlan*>(ctx->rs_plan.p);
            hipLaunchKernelGGL(k_rescore_plan, dim3(1), dim3(kPlanBlock), 0, ctx->stream, ctx->scr_cnt.p,
                               (int64_t)cells, (int32_t)per_full, kSlicedRescoreMax, (int64_t)cells * lst, chp,
                               ctx->scr_off.p, nullptr, plan);
        }
        // the chunked re-score (a plan past kSlicedRescoreMax; returns at once
        // otherwise), then the sliced one, whose end keeps each cell's best in
        // the row's first partial slot (k_rescore_fin); the grids stride over
        // the entries -- a round lists a few dozen near-ties
        hipLaunchKernelGGL((k_rescore<kRescoreR>), dim3((unsigned)std::min<int64_t>(ne_full, 512)), dim3(kBlock), 0,
                           ctx->stream, ctx->P->labels.p, grp, ctx->P->comps64.p, ctx->P->samp.p, lst,
                           a.cand_offset, a.seed, ctx->rounds.p, nl, ctx->P->n_labels, a.tiles,
                           ctx->scr_cnt.p, ctx->scr_idx.p, chp, plan, ctx->scr_res.p);
        hipLaunchKernelGGL(k_rescore_slices, dim3((unsigned)((s_max + 3) / 4), (unsigned)std::min<int64_t>(ne_sliced, 64)),
                           dim3(kBlock), 0, ctx->stream, ctx->P->labels.p, grp, ctx->P->comps64.p, ctx->P->samp.p, lst,
                           a.cand_offset, a.seed, ctx->rounds.p, nl, ctx->scr_cnt.p, ctx->scr_idx.p, chp, plan,
                           ctx->rs_x.p, ctx->rs_g.p, s_max, ctx->rs_part.p);
        hipLaunchKernelGGL(k_rescore_fin, dim3((unsigned)std::min<int64_t>(ne_sliced, kRsFinWgs)), dim3(kRsW), 0, ctx->stream,
                           ctx->P->labels.p, grp, ctx->P->comps64.p, nl, chp, plan, ctx->rs_x.p, ctx->rs_g.p, s_max,
                           ctx->rs_part.p, ctx->scr_res.p, ctx->rs_done.p + 1, (int64_t)cells, ctx->P->n_labels,
                           a.tiles, ctx->scr_off.p, ctx->partials.p);
        ctx->dense_one = true;   // (k_reduce reads a dense row's first slot only)
        ctx->screen_total += (int64_t)cells * a.n;
        ctx->screen_pending = true;
        bracket(ctx, DENSE_GMM, 1);
        return ctx->hip(hipGetLastError(), "screen launch");
    }
    if (sizeof(T) == 8 && ctx->screen && a.S.cpack != 0) {   // packed map, screened
        const int rc = launch_screen_packed(ctx, grp, nl, nch, a);
        bracket(ctx, DENSE_GMM, 1);
        return rc;
    }
    if (nch > 1) {
        const int32_t chunk = dense_chunk_len(ctx, nch);
        const size_t planes = (size_t)nl * (nch + 2) * a.gx * (kR * kBlock);
        HIPCHK(ctx, ctx->chunk_part.reserve(planes));
#define TPE_CHUNKED(RR)                                                                          \
    hipLaunchKernelGGL((k_round_chunk<T, RR>), dim3(a.gx, nl, nch), dim3(kBlock), 0, ctx->stream, \
                       ctx->P->labels.p, grp, comps, ctx->P->samp.p, a.n, a.cand_offset, a.seed,    \
                       ctx->rounds.p, chunk, ctx->chunk_part.p, ctx->errflag.p, a.S);              \
    hipLaunchKernelGGL((k_finish_chunks<T, RR>), dim3(a.gx, nl), dim3(kBlock), 0, ctx->stream,   \
                       ctx->P->labels.p, grp, comps, a.n, a.cand_offset, ctx->P->n_labels, a.tiles, \
                       nch, ctx->chunk_part.p, ctx->partials.p, a.olb, a.ola, a.S)
        if (narrow(a.S)) {
            TPE_CHUNKED(kRGroup);
        } else {
            TPE_CHUNKED(kR);
        }
#undef TPE_CHUNKED
    } else if (narrow(a.S))
        hipLaunchKernelGGL((k_round<T, DENSE_ANY, true, kRGroup>), dim3(a.gx, nl, a.gz), dim3(kBlock),
                           0, ctx->stream, ctx->P->labels.p, grp, comps, ctx->P->comps64.p,
                           ctx->P->samp.p, a.cand_in, a.n, a.cand_offset, a.seed, ctx->rounds.p,
                           ctx->P->n_labels, a.tiles, ctx->partials.p, a.olb, a.ola, ctx->errflag.p,
                           a.S);
    else
        hipLaunchKernelGGL((k_round<T, DENSE_ANY, true, kR>), dim3(a.gx, nl, a.gz), dim3(kBlock), 0,
                           ctx->stream, ctx->P->labels.p, grp, comps, ctx->P->comps64.p,
                           ctx->P->samp.p, a.cand_in, a.n, a.cand_offset, a.seed, ctx->rounds.p,
                           ctx->P->n_labels, a.tiles, ctx->partials.p, a.olb, a.ola, ctx->errflag.p,
                           a.S);
    bracket(ctx, DENSE_GMM, 1);
    return TPE_OK;
}

// Quantized families in a sampled round: qsample (both families) -> host
// decides each label's table window -> qtable + qscan per family.
int launch_quantized(tpe_ctx* ctx, const Groups& g, const RoundArgs& a, int64_t* evals_q) {
    const int nqg = g.count[QUANT_GMM], nql = g.count[QUANT_LGMM];
    const int nq = nqg + nql;
    evals_q[0] = evals_q[1] = 0;
    if (nq == 0 || a.tiles == 0) return TPE_OK;
    if (!ctx->P->qc_ready) {   // the above mixtures' runs (k_qtable), once per posterior
        const int rc = tpe_rt::qc_launch(ctx, ctx->stream);
        if (rc) return rc;
    }
    // bounded labels: the grid window from [low, high] / q before sampling
    // (a margin of one step each side); fused when every label has one
    {
        std::vector<QInfo> qi(nq);
        int64_t tab = 0, maxG = 0;
        bool fused = ctx->dedup;
        const int64_t total = a.total_slots;
        for (int qpos = 0; qpos < nq && fused; ++qpos) {
            const int li = qpos < nqg ? ctx->P->h_group[QUANT_GMM][qpos] : ctx->P->h_group[QUANT_LGMM][qpos - nqg];
            const DLabel& d = ctx->P->h_labels[li];
            const bool lg = qpos >= nqg;
            const double lo = lg ? d.exp_low : d.low, hi = lg ? d.exp_high : d.high;
            if ((d.flags & 3) != 3 || !(d.q > 0.0) || !std::isfinite(lo / d.q) || !std::isfinite(hi / d.q) ||
                std::fabs(lo / d.q) > 0x1.0p50 || std::fabs(hi / d.q) > 0x1.0p50) {
                fused = false;
                break;
            }
            const int64_t jmin = (int64_t)std::floor(lo / d.q) - 1, jmax = (int64_t)std::ceil(hi / d.q) + 1;
            const int64_t G = jmax - jmin + 1;
            if (G < 1 || 2 * G > total) {
                fused = false;
                break;
            }
            // the grid indices a draw can take: x in [lo, hi) (LGMM1: exp of a
            // log-space draw, within an ulp), j = rint(x / q) is monotone in x
            const double xl = lg ? lo * (1.0 - 0x1.0p-50) : lo, xh = lg ? hi * (1.0 + 0x1.0p-50) : hi;
            const int64_t jlo = std::max(jmin, (int64_t)std::nearbyint(xl / d.q));
            const int64_t jhi = std::min(jmax, (int64_t)std::nearbyint(xh / d.q));
            qi[qpos] = QInfo{jmin, G, tab, jlo, jhi, 0};
            tab += G;
            maxG = std::max(maxG, G);
            evals_q[lg ? 1 : 0] += G * (int64_t)(d.nb + d.na);
        }
        if (fused) {
            HIPCHK(ctx, ctx->qinfo.reserve(nq));
            HIPCHK(ctx, ctx->qtab.reserve(std::max<int64_t>(tab, 1)));
            HIPCHK(ctx, ctx->qkmax.reserve(nq));
            HIPCHK(ctx, hipMemcpyAsync(ctx->qinfo.p, qi.data(), nq * sizeof(QInfo), hipMemcpyHostToDevice,
                                       ctx->stream));
            FillSet fs{};
            add_fill(fs, ctx->qkmax.p, nq * sizeof(unsigned long long), 0);
            {
                const int rc = run_fills(ctx, fs);
                if (rc) return rc;
            }
            int64_t* found = a.S.cpack == 0 ? early_found(ctx) : nullptr;
            for (int fam = 0; fam < 2; ++fam) {
                const int mode = fam ? QUANT_LGMM : QUANT_GMM;
                const int cnt = fam ? nql : nqg;
                const int qbase = fam ? nqg : 0;
                if (!cnt) continue;
                bracket(ctx, mode, 0);
                dim3 tg((unsigned)maxG, cnt, 1);
                if (fam)
                    hipLaunchKernelGGL(k_qtable<QUANT_LGMM>, tg, dim3(kBlock), 0, ctx->stream, ctx->P->labels.p,
                                       g.dev[mode], ctx->P->comps64.p, ctx->qinfo.p, nq, qbase, ctx->qtab.p,
                                       ctx->qkmax.p, ctx->P->qcomp.p, ctx->P->qc_n.p);
                else
                    hipLaunchKernelGGL(k_qtable<QUANT_GMM>, tg, dim3(kBlock), 0, ctx->stream, ctx->P->labels.p,
                                       g.dev[mode], ctx->P->comps64.p, ctx->qinfo.p, nq, qbase, ctx->qtab.p,
                                       ctx->qkmax.p, ctx->P->qcomp.p, ctx->P->qc_n.p);
                dim3 sg(a.gx, cnt, a.gz);
#define TPE_QFUSED(M, RR)                                                                          \
    hipLaunchKernelGGL((k_qfused<M, RR>), sg, dim3(kBlock), 0, ctx->stream, ctx->P->labels.p,         \
                       g.dev[mode], ctx->P->comps64.p, ctx->P->samp.p, ctx->qinfo.p, ctx->qtab.p, a.n,  \
                       a.cand_offset, a.seed, ctx->rounds.p, qbase, ctx->P->n_labels, a.tiles,          \
                       ctx->partials.p, ctx->errflag.p, a.S)
                // tile map: workgroups stride over the tiles (a.gx slots)
                const unsigned qgx = (unsigned)std::max<int64_t>(
                    1, std::min<int64_t>({(int64_t)a.gx, (a.n + kQR * kBlock - 1) / (kQR * kBlock),
                                          kHotWgs / std::max<int64_t>(1, (int64_t)cnt * a.gz)}));
#define TPE_QTILES(M)                                                                                   \
    do {                                                                                                \
    for (const EarlyPhase& ph : early_phases(a, (int64_t)kQR * kBlock, qgx, found != nullptr,           \
                                             (int64_t)cnt * a.gz))                                     \
        hipLaunchKernelGGL((k_qfused_tiles<M, kQR>), dim3(ph.grid, cnt, a.gz), dim3(kBlock), 0,         \
                           ctx->stream, ctx->P->labels.p, g.dev[mode], ctx->P->comps64.p, ctx->P->samp.p, \
                           ctx->qinfo.p, ctx->qtab.p, ph.n, a.cand_offset, a.seed, ctx->rounds.p, qbase,  \
                           ctx->P->n_labels, a.tiles, ctx->partials.p, ctx->errflag.p, ctx->qkmax.p, found, \
                           ph.i0, ph.slot_base, ph.empty_from, nullptr);                                \
    launch_early_drawn(ctx, g.dev[mode], cnt, a, found, (int64_t)kQR * kBlock, ctx->xdrawn.p);          \
    } while (0)
                if (fam) {
                    if (a.S.cpack == 0) TPE_QTILES(QUANT_LGMM);
                    else if (narrow(a.S)) TPE_QFUSED(QUANT_LGMM, kRGroup);
                    else TPE_QFUSED(QUANT_LGMM, kR);
                } else {
                    if (a.S.cpack == 0) TPE_QTILES(QUANT_GMM);
                    else if (narrow(a.S)) TPE_QFUSED(QUANT_GMM, kRGroup);
                    else TPE_QFUSED(QUANT_GMM, kR);
                }
#undef TPE_QTILES
#undef TPE_QFUSED
                bracket(ctx, mode, 1);
            }
            return ctx->hip(hipGetLastError(), "fused quantized launch");
        }
        evals_q[0] = evals_q[1] = 0;
    }
    const size_t slots = (size_t)a.n_rounds * nq;   // candidate rows
    HIPCHK(ctx, ctx->qj.reserve(slots * (size_t)a.n));
    HIPCHK(ctx, ctx->qmm.reserve(2 * (size_t)nq));
    HIPCHK(ctx, ctx->qinfo.reserve(nq));
    // the first quantized family's timing bracket covers the shared sampling
    // pass and the window round trip as well
    const int first_mode = nqg ? QUANT_GMM : QUANT_LGMM;
    bracket(ctx, first_mode, 0);
    HIPCHK(ctx, hipMemsetAsync(ctx->qmm.p, 0xFF, nq * sizeof(unsigned long long), ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->qmm.p + nq, 0, nq * sizeof(unsigned long long), ctx->stream));
#define TPE_QSAMPLE(M, CNT, BASE, RR)                                                         \
    hipLaunchKernelGGL((k_qsample<M, RR>), dim3(a.gx, CNT, a.gz), dim3(kBlock), 0, ctx->stream, \
                       ctx->P->labels.p, g.dev[M], ctx->P->samp.p, a.n, a.cand_offset, a.seed,      \
                       ctx->rounds.p, nq, BASE, ctx->qj.p, ctx->qmm.p, ctx->qmm.p + nq,        \
                       ctx->errflag.p, a.S)
    if (nqg) {
        if (narrow(a.S)) TPE_QSAMPLE(QUANT_GMM, nqg, 0, kRGroup);
        else TPE_QSAMPLE(QUANT_GMM, nqg, 0, kR);
    }
    if (nql) {
        if (narrow(a.S)) TPE_QSAMPLE(QUANT_LGMM, nql, nqg, kRGroup);
        else TPE_QSAMPLE(QUANT_LGMM, nql, nqg, kR);
    }
#undef TPE_QSAMPLE
    HIPCHK(ctx, hipGetLastError());
    std::vector<unsigned long long> mm(2 * (size_t)nq);
    HIPCHK(ctx, hipMemcpyAsync(mm.data(), ctx->qmm.p, 2 * nq * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->qx) {   // one shard of a multi-device round: the window of the whole set
        int rc = ctx->qx->exchange(ctx, mm);
        if (rc) return rc;
    }
    // one table per label, shared by every round (the posterior does not
    // depend on the round); worth it when the label's grid window is smaller
    // than half its candidates over all rounds (each slot costs one
    // candidate's work)
    std::vector<QInfo> qi(nq);
    int64_t tab = 0, maxG = 0;
    const int64_t total = a.total_slots;
    for (int qpos = 0; qpos < nq; ++qpos) {
        const int64_t jmin = (int64_t)(mm[qpos] ^ 0x8000000000000000ull);
        const int64_t jmax = (int64_t)(mm[nq + qpos] ^ 0x8000000000000000ull);
        const int64_t G = (mm[qpos] <= mm[nq + qpos]) ? jmax - jmin + 1 : 0;
        qi[qpos] = QInfo{jmin, (ctx->dedup && G > 0 && 2 * G <= total) ? G : 0, tab, 1, 0, 0};
        tab += qi[qpos].G;
        maxG = std::max(maxG, qi[qpos].G);
        const int li = qpos < nqg ? ctx->P->h_group[QUANT_GMM][qpos] : ctx->P->h_group[QUANT_LGMM][qpos - nqg];
        const DLabel& d = ctx->P->h_labels[li];
        evals_q[qpos < nqg ? 0 : 1] += (qi[qpos].G ? qi[qpos].G : total) * (int64_t)(d.nb + d.na);
    }
    HIPCHK(ctx, ctx->qtab.reserve(std::max<int64_t>(tab, 1)));
    HIPCHK(ctx, hipMemcpyAsync(ctx->qinfo.p, qi.data(), nq * sizeof(QInfo),
                               hipMemcpyHostToDevice, ctx->stream));
    for (int fam = 0; fam < 2; ++fam) {
        const int mode = fam ? QUANT_LGMM : QUANT_GMM;
        const int cnt = fam ? nql : nqg;
        const int qbase = fam ? nqg : 0;
        if (!cnt) continue;
        if (mode != first_mode) bracket(ctx, mode, 0);
        if (maxG > 0) {
            dim3 tg((unsigned)maxG, cnt, 1);
            if (fam)
                hipLaunchKernelGGL(k_qtable<QUANT_LGMM>, tg, dim3(kBlock), 0, ctx->stream,
                                   ctx->P->labels.p, g.dev[mode], ctx->P->comps64.p, ctx->qinfo.p, nq,
                                   qbase, ctx->qtab.p, nullptr, ctx->P->qcomp.p, ctx->P->qc_n.p);
            else
                hipLaunchKernelGGL(k_qtable<QUANT_GMM>, tg, dim3(kBlock), 0, ctx->stream,
                                   ctx->P->labels.p, g.dev[mode], ctx->P->comps64.p, ctx->qinfo.p, nq,
                                   qbase, ctx->qtab.p, nullptr, ctx->P->qcomp.p, ctx->P->qc_n.p);
        }
        dim3 sg(a.gx, cnt, a.gz);
#define TPE_QSCAN(M, RR)                                                                      \
    hipLaunchKernelGGL((k_qscan<M, RR>), sg, dim3(kBlock), 0, ctx->stream, ctx->P->labels.p,     \
                       g.dev[mode], ctx->P->comps64.p, ctx->qj.p, ctx->qinfo.p, ctx->qtab.p, a.n, \
                       a.cand_offset, nq, qbase, ctx->P->n_labels, a.tiles, ctx->partials.p, a.S)
        if (fam) {
            if (narrow(a.S)) TPE_QSCAN(QUANT_LGMM, kRGroup);
            else TPE_QSCAN(QUANT_LGMM, kR);
        } else {
            if (narrow(a.S)) TPE_QSCAN(QUANT_GMM, kRGroup);
            else TPE_QSCAN(QUANT_GMM, kR);
        }
#undef TPE_QSCAN
        bracket(ctx, mode, 1);
    }
    HIPCHK(ctx, hipGetLastError());
    return TPE_OK;
}

// Split-K map (small sampled candidate sets): sample -> slice sums ->
// finish, per family.  Returns the evaluations executed.
constexpr int64_t kSplitKMaxSlots = 2048;   // n * n_rounds per label

inline int slices_of(const DLabel& d) {
    const int S = slice_len(d.mode);
    return (d.nb + S - 1) / S + (d.na + S - 1) / S;
}

// MODE = DENSE_ANY: the GMM1 and LGMM1 labels in one chain (their groups are
// adjacent), timed in the DENSE_GMM slot
template <typename T, int MODE>
int launch_splitk(tpe_ctx* ctx, const Groups& g, const RoundArgs& a, int32_t s_max) {
    constexpr bool kAny = MODE == DENSE_ANY;
    const int nl = kAny ? g.count[DENSE_GMM] + g.count[DENSE_LGMM] : g.count[MODE];
    if (nl == 0) return TPE_OK;
    const int32_t* grp = kAny ? ctx->P->groups.p + ctx->P->group_off[DENSE_GMM] : g.dev[MODE];
    int32_t s_mode = 0;
    for (int m : {kAny ? DENSE_GMM : MODE, kAny ? DENSE_LGMM : MODE})
        for (int li : ctx->P->h_group[m]) s_mode = std::max(s_mode, slices_of(ctx->P->h_labels[li]));
    const Comp<T>* comps;
    if constexpr (sizeof(T) == 8) comps = ctx->P->comps64.p; else comps = ctx->P->comps32.p;
    const int32_t L = ctx->P->n_labels;
    const int slot = kAny ? DENSE_GMM : MODE;
    bracket(ctx, slot, 0);
    const unsigned sb = (unsigned)((a.n * a.n_rounds + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_sample_small<MODE>, dim3(sb, nl), dim3(kBlock), 0, ctx->stream,
                       ctx->P->labels.p, grp, ctx->P->samp.p, a.n, a.cand_offset, a.seed,
                       ctx->rounds.p, a.n_rounds, L, ctx->xs.p, ctx->errflag.p);
    hipLaunchKernelGGL((k_score_slices<T, MODE>),
                       dim3((unsigned)((s_mode + kSliceWaves - 1) / kSliceWaves), nl, a.n_rounds),
                       dim3(kBlock), 0, ctx->stream, ctx->P->labels.p, grp, comps,
                       ctx->P->comps64.p, a.n, L, s_max, ctx->xs.p, ctx->slice_part.p);
    hipLaunchKernelGGL((k_finish_slices<T, MODE>), dim3(nl, a.n_rounds), dim3(kBlock), 0,
                       ctx->stream, ctx->P->labels.p, grp, comps, a.n, a.cand_offset, L, s_max,
                       ctx->xs.p, ctx->slice_part.p, ctx->partials.p, ctx->errflag.p);
    bracket(ctx, slot, 1);
    return ctx->hip(hipGetLastError(), "split-K launch");
}

int run_round(tpe_ctx* ctx, uint64_t seed, const uint32_t* rounds_h, int32_t n_rounds, int64_t n,
              int64_t cand_offset, const double* cand_in_dev, double* olb, double* ola,
              tpe_label_result* out, int32_t only_label) {
    if (ctx->P->n_labels == 0) return ctx->fail(TPE_ERR_ARG, "no posterior set (tpe_set_posterior)");
    if (n < 0 || n_rounds <= 0) return ctx->fail(TPE_ERR_ARG, "bad candidate/round count");
    if (cand_offset < 0 || cand_offset + n > (int64_t)UINT32_MAX)
        return ctx->fail(TPE_ERR_ARG, "candidate indices must stay below 2^32");
    // a deferred subset rebuild (TPE_OPT_DEFER_REPORT: quantized /
    // categorical labels on the second stream) is settled after the dense
    // labels' kernels are queued when this round takes the side families to
    // the second stream; first thing otherwise
    if (!(ctx->build.pending && only_label < 0 && cand_in_dev == nullptr && n > 0 && ctx->aux_families &&
          ctx->aux && !ctx->qx))
        TPE_SETTLE(ctx);
    // slot map: packed (whole rounds per workgroup) for candidate sets smaller
    // than a tile, tiled otherwise
    Slots S{0, 0, n_rounds};
    int32_t tiles;
    uint32_t gx, gz;
    if (n > 0 && n < kTile) {
        const int per_block = n <= kBlock * kRGroup ? kBlock * kRGroup : kTile;
        S.cpack = (int32_t)n;
        S.rpb = per_block / (int32_t)n;
        tiles = 1;
        gx = (uint32_t)((n_rounds + S.rpb - 1) / S.rpb);
        gz = 1;
    } else {
        tiles = (int32_t)((n + kTile - 1) / kTile);
        gx = (uint32_t)tiles;
        gz = (uint32_t)n_rounds;
    }
    const int32_t L = ctx->P->n_labels;
    ctx->rep.clear();   // (an earlier round that failed between its reads and its flush)
    HIPCHK(ctx, ctx->partials.reserve((size_t)n_rounds * L * std::max(tiles, 1)));
    HIPCHK(ctx, ctx->results.reserve((size_t)n_rounds * L));
    HIPCHK(ctx, ctx->rounds.reserve(n_rounds));
    HIPCHK(ctx, ctx->errflag.reserve(1));
    HIPCHK(ctx, hipMemcpyAsync(ctx->rounds.p, rounds_h, n_rounds * sizeof(uint32_t),
                               hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, ctx->xdrawn.reserve(2));
    {
        FillSet f{};
        add_fill(f, ctx->errflag.p, sizeof(int32_t), 0);
        add_fill(f, ctx->xdrawn.p, 2 * sizeof(unsigned long long), 0);
        if (ctx->early && S.cpack == 0 && cand_in_dev == nullptr) {   // early_found: no find yet
            HIPCHK(ctx, ctx->xfound.reserve((size_t)n_rounds * L));
            add_fill(f, ctx->xfound.p, (size_t)n_rounds * L * sizeof(int64_t), 0x7f7f7f7fu);
        }
        const int rc = run_fills(ctx, f);
        if (rc) return rc;
    }
    // the families this round launches (TPE_OPT_MODE_MASK); the others keep
    // their statistics from the round that last ran them, and their result
    // entries are unspecified
    const int32_t fam = only_label >= 0 ? 31 : ctx->mode_mask;
    const bool dense_on = (fam & 3) != 0;
    Groups g;
    for (int m = 0; m < kNumModes; ++m) {
        g.dev[m] = ctx->P->groups.p + ctx->P->group_off[m];
        g.count[m] = (fam >> m) & 1 ? (int32_t)ctx->P->h_group[m].size() : 0;
        if (!((fam >> m) & 1)) continue;
        ctx->mode_ran[m] = false;
        ctx->mode_ms[m] = 0.f;
        ctx->mode_evals[m] = 0;
    }
    if (only_label >= 0) {  // tpe_score: launch the one label's mode only
        HIPCHK(ctx, ctx->one_group.reserve(1));
        HIPCHK(ctx, hipMemcpyAsync(ctx->one_group.p, &only_label, sizeof(int32_t),
                                   hipMemcpyHostToDevice, ctx->stream));
        for (int m = 0; m < kNumModes; ++m) g.count[m] = 0;
        const int m = ctx->P->h_labels[only_label].mode;
        g.dev[m] = ctx->one_group.p;
        g.count[m] = 1;
    }
    // the whole problem (ctx->hint_*: set by a multi-device context for its shards)
    const int64_t n_whole =
        ctx->hint_n > 0 ? ctx->hint_n : (ctx->opt_whole_n > 0 ? ctx->opt_whole_n : n);
    const int32_t rounds_whole = ctx->hint_rounds > 0
                                     ? ctx->hint_rounds
                                     : (ctx->opt_whole_rounds > 0 ? ctx->opt_whole_rounds : n_rounds);
    const uint32_t gx_whole =
        S.cpack ? (uint32_t)((rounds_whole + S.rpb - 1) / S.rpb) : gx;
    RoundArgs a{n, cand_offset, seed, n_rounds, tiles, cand_in_dev, olb, ola, S, gx, gz,
                n_whole * rounds_whole, gx_whole};
    if (dense_on) {
        ctx->screen_total = ctx->screen_rescored = 0;
        ctx->hot_ran = false;
        ctx->hot_listed = 0;
        ctx->hot_fallback = 0;
        ctx->screen_mode = 0;
        ctx->screen_exec = 0;
        ctx->screen_rescore_terms = 0;
    }
    if (fam & (1 << CAT)) ctx->cat_early = false;
    ctx->dense_one = false;
    ctx->pk_plan_pending = false;
    ctx->zw_pending = false;
    ctx->evw_used = 0;
    ctx->screen_pending = false;
    ctx->screen_exec_pending = false;
    const bool sample = cand_in_dev == nullptr;
    int64_t evals_q[2] = {0, 0};
    if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    // split-K for small sampled rounds (packed map, one tile per label)
    const bool splitk = sample && ctx->splitk && n > 0 && S.cpack != 0 &&
                        a.total_slots <= kSplitKMaxSlots;
    if (splitk) {
        TPE_SETTLE(ctx);
        int32_t s_max = 1;
        for (int m = 0; m < CAT; ++m)
            for (int li : ctx->P->h_group[m]) s_max = std::max(s_max, slices_of(ctx->P->h_labels[li]));
        HIPCHK(ctx, ctx->xs.reserve((size_t)n_rounds * L * n));
        HIPCHK(ctx, ctx->slice_part.reserve((size_t)n_rounds * L * s_max * n));
        int rc;
        if (ctx->precision == TPE_F32) {
            if ((rc = launch_splitk<float, DENSE_ANY>(ctx, g, a, s_max))) return rc;
        } else {
            if ((rc = launch_splitk<double, DENSE_ANY>(ctx, g, a, s_max))) return rc;
        }
        if ((rc = launch_splitk<double, QUANT_GMM>(ctx, g, a, s_max))) return rc;
        if ((rc = launch_splitk<double, QUANT_LGMM>(ctx, g, a, s_max))) return rc;
        for (int q = 0; q < 2; ++q)
            for (int li : ctx->P->h_group[q ? QUANT_LGMM : QUANT_GMM]) {
                const DLabel& d = ctx->P->h_labels[li];
                evals_q[q] += n * (int64_t)n_rounds * (d.nb + d.na);
            }
        launch_round<double, CAT, true>(ctx, g, a);
    } else if (sample) {
        // the quantized and categorical labels (short kernels) on the second
        // stream, beside the dense draw: their own partial rows, early-exit
        // slots, tables and draw counters; forked after the round's resets,
        // joined before the reduction.  (A multi-device shard's quantized
        // window exchange stays on the main stream.)
        const bool side = ctx->aux_families && ctx->aux && !ctx->qx && a.tiles > 0 &&
                          g.count[CAT] + g.count[QUANT_GMM] + g.count[QUANT_LGMM] > 0;
        int rc = TPE_OK;
        bool dense_done = false;
        if (side) {
            HIPCHK(ctx, hipEventRecord(ctx->ev_cat[0], ctx->stream));
            if (ctx->build.pending) {
                // the deferred rebuild: the dense labels' kernels first (they
                // read none of its labels' records), then its report (the
                // host waits for the second stream), then the side families
                // after it on that stream
                rc = ctx->precision == TPE_F32 ? launch_dense<float>(ctx, g, a) : launch_dense<double>(ctx, g, a);
                if (rc) return rc;
                dense_done = true;
                TPE_SETTLE(ctx);
            }
            HIPCHK(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_cat[0], 0));
            std::swap(ctx->stream, ctx->aux);   // (every launch below on the second stream)
            rc = launch_quantized(ctx, g, a, evals_q);
            if (rc == TPE_OK) launch_round<double, CAT, true>(ctx, g, a);
            std::swap(ctx->stream, ctx->aux);
            const hipError_t e = hipEventRecord(ctx->ev_cat[1], ctx->aux);
            if (rc == TPE_OK && e != hipSuccess) rc = ctx->hip(e, "second-stream join");
        } else {
            TPE_SETTLE(ctx);
            rc = launch_quantized(ctx, g, a, evals_q);
        }
        if (rc == TPE_OK && !dense_done)
            rc = ctx->precision == TPE_F32 ? launch_dense<float>(ctx, g, a) : launch_dense<double>(ctx, g, a);
        if (side) HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_cat[1], 0));
        if (rc) return rc;
        if (!side) launch_round<double, CAT, true>(ctx, g, a);
    } else {
        launch_round<double, QUANT_GMM, false>(ctx, g, a);
        launch_round<double, QUANT_LGMM, false>(ctx, g, a);
        if (ctx->precision == TPE_F32) {
            launch_round<float, DENSE_GMM, false>(ctx, g, a);
            launch_round<float, DENSE_LGMM, false>(ctx, g, a);
        } else {
            launch_round<double, DENSE_GMM, false>(ctx, g, a);
            launch_round<double, DENSE_LGMM, false>(ctx, g, a);
        }
        launch_round<double, CAT, false>(ctx, g, a);
    }
    HIPCHK(ctx, hipGetLastError());
    TPE_SETTLE(ctx);   // (every path above settled it; a guard)
    if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    if (tiles == 1) {
        const int64_t nr = (int64_t)n_rounds * L;
        hipLaunchKernelGGL(k_emit, dim3((unsigned)((nr + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           ctx->stream, ctx->partials.p, nr, L, ctx->results.p);
        HIPCHK(ctx, hipGetLastError());
    } else if (tiles > 1) {
        hipLaunchKernelGGL(k_reduce, dim3(L, n_rounds), dim3(kReduceBlock), 0, ctx->stream,
                           ctx->partials.p, tiles, L, ctx->results.p, ctx->P->labels.p, ctx->dense_one ? 1 : 0);
        HIPCHK(ctx, hipGetLastError());
    }
    if (ctx->timing) HIPCHK(ctx, hipEventRecord(ctx->ev2, ctx->stream));
    PinScalars& pin = ctx->pin[0];
    const size_t n_res = (size_t)n_rounds * L;
    if (tiles > 0 && ctx->dev_out)
        HIPCHK(ctx, hipMemcpyAsync(ctx->dev_out, ctx->results.p, n_res * sizeof(tpe_label_result),
                                   hipMemcpyDeviceToDevice, ctx->stream));
    // large results (config 5: 25 MB) come back in pieces, each copied into
    // the caller's array as soon as it lands, under the next piece's transfer
    const size_t res_bytes = n_res * sizeof(tpe_label_result);
    const int pieces = (tiles > 0 && out && res_bytes >= ((size_t)8 << 20)) ? tpe_ctx::kResPieces : 0;
    const size_t piece = ((res_bytes + std::max(pieces, 1) - 1) / std::max(pieces, 1) + 4095) & ~(size_t)4095;
    {
        int rc = defer_read(ctx, &pin.err, ctx->errflag.p, sizeof(int32_t));
        if (!rc) rc = defer_read(ctx, pin.xdrawn, ctx->xdrawn.p, 2 * sizeof(unsigned long long));
        if (!rc && tiles > 0 && out) HIPCHK(ctx, ctx->res_h.resize(n_res));
        if (!rc && pieces) {
            for (int k = 0; k < pieces; ++k) {
                const size_t a0 = std::min(res_bytes, k * piece), a1 = std::min(res_bytes, a0 + piece);
                if (!ctx->ev_res[k])
                    HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_res[k], hipEventDisableTiming));
                if (a1 > a0)
                    HIPCHK(ctx, hipMemcpyAsync((char*)ctx->res_h.data() + a0, (const char*)ctx->results.p + a0,
                                               a1 - a0, hipMemcpyDeviceToHost, ctx->stream));
                HIPCHK(ctx, hipEventRecord(ctx->ev_res[k], ctx->stream));
            }
        } else if (!rc && tiles > 0 && out) {
            rc = defer_read(ctx, ctx->res_h.data(), ctx->results.p, res_bytes);
        }
        if (!rc) rc = flush_reads(ctx);
        if (rc) return rc;
    }
    for (int k = 0; k < pieces; ++k) {
        const size_t a0 = std::min(res_bytes, k * piece), a1 = std::min(res_bytes, a0 + piece);
        HIPCHK(ctx, hipEventSynchronize(ctx->ev_res[k]));
        if (a1 > a0) copy_out((char*)out + a0, (const char*)ctx->res_h.data() + a0, a1 - a0);
    }
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    unpack_reads(ctx);
    if (tiles > 0 && out && !pieces) copy_out(out, ctx->res_h.data(), res_bytes);
    if (tiles == 0 && out) std::memset(out, 0, res_bytes);   // (no candidates: empty records; the caller's array is uninitialised)
    if (ctx->zw_pending) {
        ctx->P->zw_ready = pin.plan.total > 0 && !pin.plan.sliced;
        ctx->zw_pending = false;
    }
    if (ctx->pk_plan_pending && pin.plan.overflow && !ctx->pk_redo) {
        // the packed re-score listed more candidates than its buffers hold:
        // nothing was re-scored; the round again with buffers for them all
        ctx->pk_cap = pin.plan.total + pin.plan.total / 4 + 1024;
        ctx->pk_redo = true;
        const int rc = run_round(ctx, seed, rounds_h, n_rounds, n, cand_offset, cand_in_dev, olb, ola, out,
                                 only_label);
        ctx->pk_redo = false;
        return rc;
    }
    const int32_t errh = pin.err;
    ctx->xdrawn_h[0] = pin.xdrawn[0];
    ctx->xdrawn_h[1] = pin.xdrawn[1];
    if (dense_on) ctx->screen_ms = 0.f;
    if (ctx->screen_exec_pending) {
        ctx->screen_exec += (int64_t)ctx->pin[0].screen_exec;
        ctx->screen_exec_pending = false;
    }
    if (ctx->screen_pending) {
        // cell = round x (dense GMM1 labels, then dense LGMM1 labels)
        const std::vector<int32_t>& gg = ctx->P->h_group[DENSE_GMM];
        const std::vector<int32_t>& gl = ctx->P->h_group[DENSE_LGMM];
        const size_t nld = gg.size() + gl.size();
        for (size_t c = 0; c < ctx->scr_cnt_h.size(); ++c) {
            const int32_t cnt = ctx->scr_cnt_h[c];
            const size_t y = c % nld;
            const DLabel& d = ctx->P->h_labels[y < gg.size() ? gg[y] : gl[y - gg.size()]];
            ctx->screen_rescored += cnt;
            ctx->screen_rescore_terms += (int64_t)cnt * (d.nb + d.na);
        }
        ctx->screen_pending = false;
        if (ctx->timing && ctx->evw_used > 0) {   // windowed tile rounds: the units' k_screen_win
            for (int32_t u = 0; u < ctx->evw_used; ++u) {
                float ms = 0.f;
                HIPCHK(ctx, hipEventElapsedTime(&ms, ctx->evw[2 * u], ctx->evw[2 * u + 1]));
                ctx->screen_ms += ms;
            }
        } else if (ctx->timing) {
            HIPCHK(ctx, hipEventElapsedTime(&ctx->screen_ms, ctx->evs[0], ctx->evs[1]));
        }
    }
    if (ctx->timing) {
        HIPCHK(ctx, hipEventElapsedTime(&ctx->score_ms, ctx->ev0, ctx->ev1));
        HIPCHK(ctx, hipEventElapsedTime(&ctx->round_ms, ctx->ev0, ctx->ev2));
    } else {
        ctx->score_ms = ctx->round_ms = 0.f;
    }
    for (int m = 0; m < kNumModes; ++m)
        if (ctx->mode_ran[m])
            if (ctx->timing)
                HIPCHK(ctx, hipEventElapsedTime(&ctx->mode_ms[m], ctx->evm[m][0], ctx->evm[m][1]));
    int64_t evals = 0;
    for (int32_t l = 0; l < L; ++l) {
        if (only_label >= 0 && l != only_label) continue;
        const DLabel& d = ctx->P->h_labels[l];
        if (!((fam >> d.mode) & 1)) continue;   // not launched (TPE_OPT_MODE_MASK)
        if (sample && (d.mode == QUANT_GMM || d.mode == QUANT_LGMM)) continue;  // counted below
        if (d.mode == CAT && ctx->cat_early) continue;   // counted below: the candidates drawn
        const int64_t e = ((d.mode == CAT) ? 2 * n : n * (int64_t)(d.nb + d.na)) * n_rounds;
        evals += e;
        // sampled rounds time both dense families in one launch (chain)
        const bool merged = sample && d.mode == DENSE_LGMM;
        ctx->mode_evals[merged ? DENSE_GMM : d.mode] += e;
    }
    ctx->mode_evals[QUANT_GMM] += evals_q[0];
    ctx->mode_evals[QUANT_LGMM] += evals_q[1];
    if (ctx->cat_early) {   // 2 lookups per categorical candidate actually drawn
        ctx->mode_evals[CAT] += 2 * (int64_t)ctx->xdrawn_h[1];
        evals += 2 * (int64_t)ctx->xdrawn_h[1];
    }
    ctx->evals = evals + evals_q[0] + evals_q[1];
    if (tiles == 0 && out) {
        for (int32_t j = 0; j < n_rounds * L; ++j)
            out[j] = tpe_label_result{NAN, NAN, NAN, NAN, -1, j % L, 0};
    }
    if (dense_on && ctx->hot_ran) {
        for (int64_t c = 0; c < ctx->hot_cells; ++c) ctx->hot_listed += ctx->hot_cnt_h[c];
        const int32_t hf = pin.hot_flag;
        if (hf && !ctx->hot_redo && errh == 0) {
            // a cell's best lower bound stayed below tau0 (bit 1: its list may
            // miss a winner) or a list overflowed (bit 2): the dense labels run
            // again with every candidate through the expansion screen (the
            // same draws; their results replace these), and later rounds list
            // more after an overflow.  Only the dense families re-run
            // (TPE_OPT_MODE_MASK): the quantized and categorical labels'
            // partial rows, draw counts and evaluations stay this run's, and
            // the reduction reads them again.  tpe_last_hot reports the
            // fallback (bench: hot_fallbacks), which no test or bench has seen
            // outside the forced TPE_OPT_HOT = 2
            if ((hf & 2) && ctx->hot_cap_div > 1.0) ctx->hot_cap_div = std::max(1.0, ctx->hot_cap_div / 4.0);
            const int64_t listed = ctx->hot_listed;
            int64_t side_evals = 0;
            for (int m = QUANT_GMM; m <= CAT; ++m)
                if ((fam >> m) & 1) side_evals += ctx->mode_evals[m];
            const unsigned long long drawn0 = ctx->xdrawn_h[0], drawn1 = ctx->xdrawn_h[1];
            const bool cat_early = ctx->cat_early;
            const int32_t mask = ctx->mode_mask;
            ctx->mode_mask = fam & ((1 << DENSE_GMM) | (1 << DENSE_LGMM));
            ctx->hot_redo = true;
            const int rc = run_round(ctx, seed, rounds_h, n_rounds, n, cand_offset, cand_in_dev, olb, ola, out,
                                     only_label);
            ctx->hot_redo = false;
            ctx->mode_mask = mask;
            ctx->hot_ran = true;
            ctx->hot_fallback = hf;
            ctx->hot_listed = listed;
            ctx->evals += side_evals;
            ctx->xdrawn_h[0] = drawn0;
            ctx->xdrawn_h[1] = drawn1;
            ctx->cat_early = cat_early;
            return rc;
        }
    }
    if (errh & 1) return ctx->fail(TPE_ERR_SAMPLE, "truncated sampler: interval [low, high) not reached");
    if (errh & 2) return ctx->fail(TPE_ERR_VALUE, "negative arg to lognormal_cdf");
    if (errh & 4) return ctx->fail(TPE_ERR_VALUE, "categorical sample out of range");
    if (errh & 8) return ctx->fail(TPE_ERR_VALUE, "quantized sample beyond 2^52 grid steps");
    return TPE_OK;
}

// the sampling records of a host-uploaded posterior: one block per label,
// the device build's fold (samp_fold_block)
__global__ __launch_bounds__(64) void k_samp_fold(const DLabel* __restrict__ labels, SampRec* __restrict__ samp) {
    const DLabel L = labels[blockIdx.x];
    (void)samp_fold_block(L, samp + L.samp_off, L.ns);
}

void launch_sample_only(tpe_ctx* ctx, int mode, int64_t n, int64_t offset, uint64_t seed,
                        double* out) {
    const int blocks = (int)((n + kBlock - 1) / kBlock);
#define TPE_SO(M)                                                                             \
    hipLaunchKernelGGL(k_sample_only<M>, dim3(blocks), dim3(kBlock), 0, ctx->stream,         \
                       ctx->P->labels.p, ctx->P->samp.p, n, offset, seed, ctx->rounds.p, out,       \
                       ctx->errflag.p)
    switch (mode) {
        case DENSE_GMM: TPE_SO(DENSE_GMM); break;
        case DENSE_LGMM: TPE_SO(DENSE_LGMM); break;
        case QUANT_GMM: TPE_SO(QUANT_GMM); break;
        case QUANT_LGMM: TPE_SO(QUANT_LGMM); break;
        default: TPE_SO(CAT); break;
    }
#undef TPE_SO
}

int set_posterior_impl(tpe_ctx* ctx, const tpe_label_desc* labels, int32_t n_labels,
                       const double* weights, const double* mus, const double* sigmas,
                       int64_t n_components, bool sampler_checks) {
    if (!ctx) return TPE_ERR_ARG;
    if (ctx->P == &ctx->resident) ctx->build.n_labels = 0;   // no built mixtures resident
    ctx->P->bx_prescan_ok = false;   // (a build's pre-scan is of that build's posterior)
    if (n_labels <= 0 || !labels || !weights) return ctx->fail(TPE_ERR_ARG, "empty posterior");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    std::vector<DLabel> dl(n_labels);
    std::vector<Comp<double>> c64;
    std::vector<Comp<float>> c32;
    std::vector<SampRec> sr;
    std::vector<int32_t> grp[kNumModes];
    for (int32_t l = 0; l < n_labels; ++l) {
        const tpe_label_desc& d = labels[l];
        DLabel& o = dl[l];
        std::memset(&o, 0, sizeof(o));
        const bool quant = (d.flags & TPE_HAS_Q) != 0;
        if (d.kind == TPE_CATEGORICAL) o.mode = CAT;
        else if (d.kind == TPE_GMM1) o.mode = quant ? QUANT_GMM : DENSE_GMM;
        else if (d.kind == TPE_LGMM1) o.mode = quant ? QUANT_LGMM : DENSE_LGMM;
        else return ctx->fail(TPE_ERR_ARG, "label " + std::to_string(l) + ": unknown kind");
        if (d.n_below <= 0 || d.n_above <= 0 || d.below_off < 0 || d.above_off < 0 ||
            d.below_off + d.n_below > n_components || d.above_off + d.n_above > n_components)
            return ctx->fail(TPE_ERR_ARG, "label " + std::to_string(l) + ": component range");
        if (d.kind == TPE_CATEGORICAL && d.n_below != d.n_above)
            return ctx->fail(TPE_ERR_ARG, "categorical: below/above sizes differ");
        if (d.kind != TPE_CATEGORICAL) {
            if (!mus || !sigmas) return ctx->fail(TPE_ERR_ARG, "mus/sigmas required");
            int rc = validate_mixture(ctx, d.n_below, d.flags, d.low, d.high, sampler_checks);
            if (rc) return rc;
            if (quant && !(d.q > 0) && !(d.q < 0)) return ctx->fail(TPE_ERR_VALUE, "q must be non-zero");
        }
        o.flags = d.flags;
        o.low = d.low;
        o.high = d.high;
        o.q = d.q;
        o.exp_low = std::exp(d.low);
        o.exp_high = std::exp(d.high);
        o.nb = d.n_below;
        o.na = d.n_above;
        o.stream = l;
        if (d.kind != TPE_CATEGORICAL && !quant) {
            // recentre both mixtures on the middle of their means: keeps
            // (mu - centre) a small, so z = x' a - m loses nothing to rounding
            double lo = INFINITY, hi = -INFINITY;
            for (int side = 0; side < 2; ++side) {
                const int64_t off = side ? d.above_off : d.below_off;
                const int32_t n = side ? d.n_above : d.n_below;
                for (int k = 0; k < n; ++k) {
                    lo = std::min(lo, mus[off + k]);
                    hi = std::max(hi, mus[off + k]);
                }
            }
            o.centre = (std::isfinite(lo) && std::isfinite(hi)) ? 0.5 * lo + 0.5 * hi : 0.0;
        }
        for (int side = 0; side < 2; ++side) {
            const int64_t off = side ? d.above_off : d.below_off;
            const int32_t n = side ? d.n_above : d.n_below;
            const int64_t at = (int64_t)c64.size();
            c64.resize(at + n);
            c32.resize(at + n);
            if (d.kind == TPE_CATEGORICAL) {
                for (int k = 0; k < n; ++k) {
                    const double lp = std::log(weights[off + k]);
                    c64[at + k] = Comp<double>{0.0, 0.0, lp, weights[off + k]};
                    c32[at + k] = Comp<float>{0.f, 0.f, (float)lp, (float)weights[off + k]};
                }
            } else {
                Folded f = fold_mixture(d.kind, quant, d.flags, d.low, d.high, o.centre, weights + off,
                                        mus + off, sigmas + off, n, c64.data() + at, c32.data() + at);
                (side ? o.shift_a : o.shift_b) = f.shift;
                (side ? o.logpacc_a : o.logpacc_b) = f.logpacc;
                (side ? o.amax_a : o.amax_b) = (float)f.amax;
            }
            (side ? o.comp_a : o.comp_b) = at;
        }
        // sampling records of the below mixture: the components and their raw
        // weights, folded on the device after the upload (k_samp_fold: the
        // device build's own fold, so both posteriors draw the same bits)
        o.samp_off = (int64_t)sr.size();
        o.ns = d.n_below;
        double tot = 0.0;
        for (int k = 0; k < d.n_below; ++k) tot += weights[d.below_off + k];
        if (!(tot > 0) && sampler_checks) return ctx->fail(TPE_ERR_VALUE, "below weights sum to zero");
        for (int k = 0; k < d.n_below; ++k) {
            SampRec s{};
            s.mu = d.kind == TPE_CATEGORICAL ? 0.0 : mus[d.below_off + k];
            s.sigma = d.kind == TPE_CATEGORICAL ? 0.0 : sigmas[d.below_off + k];
            s.wd = weights[d.below_off + k];
            sr.push_back(s);
        }
        grp[o.mode].push_back(l);
    }
    std::vector<int32_t> cat;
    for (int m = 0; m < kNumModes; ++m) {
        ctx->P->group_off[m] = (int32_t)cat.size();
        cat.insert(cat.end(), grp[m].begin(), grp[m].end());
        ctx->P->h_group[m] = grp[m];
    }
    HIPCHK(ctx, ctx->P->labels.reserve(n_labels));
    HIPCHK(ctx, ctx->P->comps64.reserve(c64.size()));
    HIPCHK(ctx, ctx->P->comps32.reserve(c32.size()));
    HIPCHK(ctx, ctx->P->samp.reserve(sr.size()));
    HIPCHK(ctx, ctx->P->groups.reserve(cat.size()));
    HIPCHK(ctx, hipMemcpy(ctx->P->labels.p, dl.data(), dl.size() * sizeof(DLabel), hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->P->comps64.p, c64.data(), c64.size() * sizeof(Comp<double>), hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->P->comps32.p, c32.data(), c32.size() * sizeof(Comp<float>), hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->P->samp.p, sr.data(), sr.size() * sizeof(SampRec), hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->P->groups.p, cat.data(), cat.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_samp_fold, dim3((unsigned)n_labels), dim3(64), 0, ctx->stream, ctx->P->labels.p,
                       ctx->P->samp.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->P->groups_h = cat;
    ctx->P->h_labels = dl;
    ctx->P->win_ready = false;
    ctx->P->zw_ready = false;
    ctx->P->qc_ready = false;
    ctx->P->bx_ready = false;
    ctx->P->n_labels = n_labels;
    return TPE_OK;
}

}  // namespace

// np.sum: numpy reduces in chunks of its 8192-element buffer, accumulated in
// order from 0.0, each chunk summed pairwise
double tpe_rt::np_pairwise_sum(const double* a, size_t n) {
    double r = 0.0;
    for (size_t c = 0; c < n; c += 8192) r += np_pairwise_sum_impl(a + c, std::min<size_t>(8192, n - c));
    return r;
}

int tpe_rt::qc_launch(tpe_ctx* ctx, hipStream_t st) {
    tpe_rt::Posterior& P = *ctx->P;
    const int nall = (int)(P.h_group[QUANT_GMM].size() + P.h_group[QUANT_LGMM].size());
    if (nall > 0) {
        HIPCHK(ctx, P.qcomp.reserve(P.comps64.cap));
        HIPCHK(ctx, P.qc_n.reserve(std::max(P.n_labels, 1)));
        hipLaunchKernelGGL(k_qcompress, dim3((unsigned)nall), dim3(kQcBlock), 0, st, P.labels.p,
                           P.groups.p + P.group_off[QUANT_GMM], P.comps64.p, P.qcomp.p, P.qc_n.p);
        HIPCHK(ctx, hipGetLastError());
    }
    P.qc_ready = true;
    return TPE_OK;
}

// ================================================================ C ABI ====
namespace {
// one thread per result: the best of the parts, tpe_merge_results' order
__global__ __launch_bounds__(kBlock) void k_merge_results(const tpe_label_result* __restrict__ parts,
                                                          int32_t n_parts, int32_t n,
                                                          tpe_label_result* __restrict__ out,
                                                          int32_t* __restrict__ err) {
    const int32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    for (int32_t p = 0; p < n_parts; ++p) {
        const tpe_label_result* c = parts + (size_t)p * n + j;
        if (c->index >= 0 && c->status == TPE_STATUS_VALUE_ONLY) *err = 1;   // no score to merge by
    }
    // the winning part's index is tracked and its record copied once (a
    // per-field select of whole records, round 4's first form, came out
    // mixing the value of one part with the rest of another)
    int32_t bp = 0;
    int64_t bi = parts[j].index;
    uint64_t bk = order_key(parts[j].score);
    for (int32_t p = 1; p < n_parts; ++p) {
        const tpe_label_result* c = parts + (size_t)p * n + j;
        const int64_t ci = c->index;
        if (ci < 0) continue;
        const uint64_t ck = order_key(c->score);
        if (bi < 0 || better(ck, ci, bk, bi)) {
            bp = p;
            bi = ci;
            bk = ck;
        }
    }
    out[j] = parts[(size_t)bp * n + j];
}

}  // namespace

extern "C" {

int tpe_abi_version(void) { return TPE_ABI_VERSION; }

// Hash of the sources this library was compiled from (hyperopt_amd/_build.py
// passes it; the "TPE_SOURCE_HASH=" prefix lets the build script find it in
// the file without loading the library).
#ifndef TPE_SOURCE_HASH
#define TPE_SOURCE_HASH "unstamped000000"
#endif
static const char kSourceStamp[] __attribute__((used)) = "TPE_SOURCE_HASH=" TPE_SOURCE_HASH;
const char* tpe_source_hash(void) { return kSourceStamp + 16; }

int tpe_ctx_create(int device, int precision, tpe_ctx** out) {
    if (!out) return TPE_ERR_ARG;
    *out = nullptr;
    if (precision != TPE_F64 && precision != TPE_F32) {
        g_create_error = "precision must be TPE_F64 or TPE_F32";
        return TPE_ERR_ARG;
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || device < 0 || device >= ndev) {
        g_create_error = std::string("no HIP device ") + std::to_string(device) + " (" +
                         (e == hipSuccess ? "count " + std::to_string(ndev) : hipGetErrorString(e)) + ")";
        return TPE_ERR_HIP;
    }
    e = hipSetDevice(device);
    if (e != hipSuccess) {
        g_create_error = hipGetErrorString(e);
        return TPE_ERR_HIP;
    }
    tpe_ctx* c = new tpe_ctx();
    c->device = device;
    c->precision = precision;
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreate(&c->ev0) == hipSuccess && hipEventCreate(&c->ev1) == hipSuccess &&
              hipEventCreate(&c->ev2) == hipSuccess;
    for (int m = 0; m < kNumModes; ++m)
        ok = ok && hipEventCreate(&c->evm[m][0]) == hipSuccess &&
             hipEventCreate(&c->evm[m][1]) == hipSuccess;
    ok = ok && hipEventCreate(&c->evs[0]) == hipSuccess && hipEventCreate(&c->evs[1]) == hipSuccess;
    ok = ok && hipEventCreate(&c->ev_prep[0]) == hipSuccess && hipEventCreate(&c->ev_prep[1]) == hipSuccess;
    // the second stream at the device's highest priority: its short
    // kernels (a deferred rebuild's tail, the side families) get workgroup
    // slots as the dense draw's free up instead of after its whole grid
    // (config 3 2.42 -> 2.37 ms, config 5 6.93 -> 6.71, r5au)
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    ok = ok && hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, prio_hi) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_cat[0], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&c->ev_cat[1], hipEventDisableTiming) == hipSuccess;
    for (int j = 0; j < 2; ++j)
        ok = ok && hipEventCreateWithFlags(&c->ev_sorted[j], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_done[j], hipEventDisableTiming) == hipSuccess;
    ok = ok && c->pin.resize(1) == hipSuccess;
    if (ok) c->pin[0] = PinScalars{};
    if (!ok) {
        g_create_error = "stream/event creation failed";
        tpe_ctx_destroy(c);
        return TPE_ERR_HIP;
    }
    *out = c;
    return TPE_OK;
}

TPE_DEV void tpe1_ctx_destroy(tpe_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    c->resident.release();
    c->single.release();
    c->partials.release();
    c->results.release();
    c->rounds.release();
    c->errflag.release();
    c->build_err.release();
    c->cand.release();
    c->out_lb.release();
    c->out_la.release();
    c->one_group.release();
    c->qj.release();
    c->qmm.release();
    c->qinfo.release();
    c->qtab.release();
    c->xs.release();
    c->slice_part.release();
    c->build.release();
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    for (int m = 0; m < kNumModes; ++m)
        for (int j = 0; j < 2; ++j)
            if (c->evm[m][j]) (void)hipEventDestroy(c->evm[m][j]);
    for (int j = 0; j < 2; ++j) {
        if (c->evs[j]) (void)hipEventDestroy(c->evs[j]);
        if (c->ev_prep[j]) (void)hipEventDestroy(c->ev_prep[j]);
    }
    for (hipEvent_t& e : c->ev_res)
        if (e) (void)hipEventDestroy(e);
    c->scr_hi.release();
    c->scr_idx.release();
    c->scr_range.release();
    c->rs_plan.release();
    c->scr_lb.release();
    c->scr_cnt.release();
    c->scr_chunks.release();
    c->scr_list.release();
    c->scr_res.release();
    c->scr_rsel.release();
    c->scr_off.release();
    c->scr_planes.release();
    c->chunk_part.release();
    for (int j = 0; j < 2; ++j) {
        c->win_keys[j].release();
        c->win_keys2[j].release();
        c->win_keys8[j].release();
        c->win_keys8b[j].release();
        c->win_vals[j].release();
        c->win_vals2[j].release();
        c->win_tmp[j].release();
        if (c->ev_sorted[j]) (void)hipEventDestroy(c->ev_sorted[j]);
        if (c->ev_done[j]) (void)hipEventDestroy(c->ev_done[j]);
    }
    c->win_evals.release();
    c->win_lohi.release();
    for (hipEvent_t e : c->evw) (void)hipEventDestroy(e);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    for (hipEvent_t e : c->ev_cat)
        if (e) (void)hipEventDestroy(e);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* tpe_last_error(const tpe_ctx* c) {
    return c ? c->err.c_str() : g_create_error.c_str();
}

TPE_DEV int tpe1_set_posterior(tpe_ctx* ctx, const tpe_label_desc* labels, int32_t n_labels,
                      const double* weights, const double* mus, const double* sigmas,
                      int64_t n_components) {
    TPE_SETTLE(ctx);
    return set_posterior_impl(ctx, labels, n_labels, weights, mus, sigmas, n_components, true);
}

TPE_DEV int tpe1_suggest(tpe_ctx* ctx, uint64_t seed, uint32_t round, int64_t n_candidates,
                int64_t cand_offset, tpe_label_result* out) {
    if (!ctx || !out) return TPE_ERR_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    return run_round(ctx, seed, &round, 1, n_candidates, cand_offset, nullptr, nullptr, nullptr,
                     out, -1);
}

TPE_DEV int tpe1_suggest_batch(tpe_ctx* ctx, uint64_t seed, const uint32_t* rounds, int32_t n_rounds,
                      int64_t n_candidates, int64_t cand_offset, tpe_label_result* out) {
    if (!ctx || !out || !rounds) return TPE_ERR_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    return run_round(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, nullptr, nullptr,
                     nullptr, out, -1);
}

TPE_DEV int tpe1_score(tpe_ctx* ctx, int32_t label, const double* cand, int64_t n, double* lpdf_below,
                       double* lpdf_above, tpe_label_result* out) {
    if (!ctx || (!cand && n > 0)) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (label < 0 || label >= ctx->P->n_labels) return ctx->fail(TPE_ERR_ARG, "label out of range");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    // host-side argument checks that the reference raises before computing
    const DLabel& d = ctx->P->h_labels[label];
    if (d.mode == QUANT_LGMM) {
        for (int64_t i = 0; i < n; ++i) {
            double ub = cand[i] + d.q / 2.0;
            if ((d.flags & 2) && ub > d.exp_high) ub = d.exp_high;
            if (ub < 0) return ctx->fail(TPE_ERR_VALUE, "negative arg to lognormal_cdf");
        }
    }
    if (d.mode == CAT) {
        for (int64_t i = 0; i < n; ++i)
            if (!(cand[i] >= 0 && cand[i] < d.nb) || cand[i] != std::floor(cand[i]))
                return ctx->fail(TPE_ERR_VALUE, "categorical sample out of range");
    }
    const size_t rows = (size_t)ctx->P->n_labels * std::max<int64_t>(n, 1);
    HIPCHK(ctx, ctx->cand.reserve(std::max<int64_t>(n, 1)));
    HIPCHK(ctx, ctx->out_lb.reserve(rows));
    HIPCHK(ctx, ctx->out_la.reserve(rows));
    if (n > 0)
        HIPCHK(ctx, hipMemcpyAsync(ctx->cand.p, cand, n * sizeof(double), hipMemcpyHostToDevice,
                                   ctx->stream));
    std::vector<tpe_label_result> all(ctx->P->n_labels);
    uint32_t round = 0;
    int rc = run_round(ctx, 0, &round, 1, n, 0, ctx->cand.p, ctx->out_lb.p, ctx->out_la.p,
                       all.data(), label);
    if (rc) return rc;
    const size_t row = (size_t)label * n;
    if (lpdf_below && n > 0)
        HIPCHK(ctx, hipMemcpy(lpdf_below, ctx->out_lb.p + row, n * sizeof(double), hipMemcpyDeviceToHost));
    if (lpdf_above && n > 0)
        HIPCHK(ctx, hipMemcpy(lpdf_above, ctx->out_la.p + row, n * sizeof(double), hipMemcpyDeviceToHost));
    if (out) {
        *out = all[label];
        if (n == 0) *out = tpe_label_result{NAN, NAN, NAN, NAN, -1, label, 0};
    }
    return TPE_OK;
}

int tpe_hot_probe(tpe_ctx* ctx, int32_t label, const double* cand, int64_t n, double* upper, double* lower,
                  double* mass) {
    if (!ctx || (n > 0 && (!cand || !upper || !lower || !mass))) return TPE_ERR_ARG;
    TPE_NOT_LSHARD(ctx);
    TPE_SETTLE(ctx);
    if (label < 0 || label >= ctx->P->n_labels) return ctx->fail(TPE_ERR_ARG, "label out of range");
    const DLabel& d = ctx->P->h_labels[label];
    if (d.mode != DENSE_GMM && d.mode != DENSE_LGMM)
        return ctx->fail(TPE_ERR_ARG, "hot probe: label is not a dense GMM1/LGMM1 label");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    ctx->bx_t_next = kBxTTile;   // (the probes check the tile rounds' index)
    int rc = tpe_rt::bx_prepare(ctx);
    if (rc) return rc;
    tpe_rt::Posterior& P = *ctx->P;
    if (!P.bx_ok) return ctx->fail(TPE_ERR_ARG, "hot probe: the posterior has no expansion index");
    if (n == 0) return TPE_OK;
    HIPCHK(ctx, ctx->cand.reserve(n));
    HIPCHK(ctx, ctx->out_lb.reserve(n));
    HIPCHK(ctx, ctx->out_la.reserve(n));
    HIPCHK(ctx, ctx->xs.reserve(n));
    HIPCHK(ctx, hipMemcpyAsync(ctx->cand.p, cand, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_hot_probe, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       P.labels.p, P.bx.p, P.bx_sb.p, P.bx_sbp.p, label, ctx->cand.p, n, ctx->out_lb.p,
                       ctx->out_la.p, ctx->xs.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(upper, ctx->out_lb.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(lower, ctx->out_la.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(mass, ctx->xs.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return TPE_OK;
}

int tpe_screen_probe(tpe_ctx* ctx, int32_t label, const double* cand, int64_t n, double* score32,
                     double* err_bound) {
    if (!ctx || (n > 0 && (!cand || !score32 || !err_bound))) return TPE_ERR_ARG;
    TPE_NOT_LSHARD(ctx);
    TPE_SETTLE(ctx);
    if (label < 0 || label >= ctx->P->n_labels) return ctx->fail(TPE_ERR_ARG, "label out of range");
    const DLabel& d = ctx->P->h_labels[label];
    if (d.mode != DENSE_GMM && d.mode != DENSE_LGMM)
        return ctx->fail(TPE_ERR_ARG, "screen probe: label is not a dense GMM1/LGMM1 label");
    if (n == 0) return TPE_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, ctx->cand.reserve(n));
    HIPCHK(ctx, ctx->out_lb.reserve(n));
    HIPCHK(ctx, ctx->out_la.reserve(n));
    HIPCHK(ctx, ctx->one_group.reserve(1));
    HIPCHK(ctx, ctx->rounds.reserve(1));
    HIPCHK(ctx, ctx->errflag.reserve(1));
    HIPCHK(ctx, hipMemcpyAsync(ctx->one_group.p, &label, sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->cand.p, cand, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    bool use_bx = false;
    if (ctx->expand && n >= 2048) {
        ctx->bx_t_next = kBxTTile;
        int rc = tpe_rt::bx_prepare(ctx);
        if (rc) return rc;
        use_bx = ctx->P->bx_ok;
    }
    if (use_bx) {   // the expansion screen's per-candidate score and bound
        tpe_rt::Posterior& P = *ctx->P;
        const unsigned bgx = (unsigned)((n + kBxR * kBlock - 1) / (kBxR * kBlock));
        hipLaunchKernelGGL((k_screen_bx<kBxR, false>), dim3(bgx, 1, 1), dim3(kBlock), 0, ctx->stream,
                           P.labels.p, ctx->one_group.p, P.comps64.p, P.samp.p, P.bx.p, P.bx_tab.p,
                           P.bx_loff.p, P.bx_list.p, n, 0, 0, ctx->rounds.p, 1, nullptr, nullptr, nullptr,
                           nullptr, nullptr, ctx->errflag.p, Slots{0, 0, 1}, ctx->cand.p, ctx->out_lb.p,
                           ctx->out_la.p, nullptr, (int64_t)0);
    } else if (ctx->window && n >= 2048) {   // the windowed screen's tiles of sorted neighbours
        int rc = tpe_rt::win_prepare(ctx);
        if (rc) return rc;
        if (n > ((int64_t)1 << 30)) return ctx->fail(TPE_ERR_ARG, "screen probe: too many candidates");
        const uint64_t* sorted = nullptr;
        tpe_rt::WinScreenArgs wa{ctx->one_group.p, 1, n, 0, 0, 0, 1, ctx->cand.p,
                                 nullptr, nullptr, ctx->out_lb.p, ctx->out_la.p};
        if ((rc = tpe_rt::win_screen(ctx, wa, &sorted))) return rc;
    } else {
        const uint32_t tiles = (uint32_t)((n + kTile - 1) / kTile);
        hipLaunchKernelGGL((k_screen<kR, false>), dim3(tiles, 1, 1), dim3(kBlock), 0, ctx->stream,
                           ctx->P->labels.p, ctx->one_group.p, ctx->P->comps32.p, ctx->P->samp.p, n, 0,
                           0, ctx->rounds.p, 1, nullptr, nullptr, ctx->errflag.p, Slots{0, 0, 1},
                           ctx->cand.p, ctx->out_lb.p, ctx->out_la.p);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(score32, ctx->out_lb.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(err_bound, ctx->out_la.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return TPE_OK;
}

int tpe_suggest_batch_device(tpe_ctx* ctx, uint64_t seed, const uint32_t* rounds, int32_t n_rounds,
                             int64_t n_candidates, int64_t cand_offset, tpe_label_result* d_out,
                             tpe_label_result* out) {
    if (!ctx || !d_out || !rounds) return TPE_ERR_ARG;
    TPE_NOT_LSHARD(ctx);
    if (!ctx->peers.empty()) return ctx->fail(TPE_ERR_ARG, "device results: single-device contexts only");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (n_candidates <= 0) return ctx->fail(TPE_ERR_ARG, "device results need candidates");
    ctx->dev_out = d_out;
    const int rc = run_round(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, nullptr, nullptr, nullptr, out,
                             -1);
    ctx->dev_out = nullptr;
    return rc;
}

int tpe_merge_results_device(tpe_ctx* ctx, const tpe_label_result* d_parts, int32_t n_parts, int32_t n,
                             tpe_label_result* d_out) {
    if (!ctx || !d_parts || !d_out || n_parts <= 0 || n < 0) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);   // (a pending deferred rebuild first, as every entry point but a round)
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (n == 0) return TPE_OK;
    HIPCHK(ctx, ctx->errflag.reserve(1));
    HIPCHK(ctx, ctx->pin.resize(1));
    ctx->pin[0].err = 0;
    HIPCHK(ctx, hipMemsetAsync(ctx->errflag.p, 0, sizeof(int32_t), ctx->stream));
    hipLaunchKernelGGL(k_merge_results, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       d_parts, n_parts, n, d_out, ctx->errflag.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(&ctx->pin[0].err, ctx->errflag.p, sizeof(int32_t), hipMemcpyDeviceToHost,
                               ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->pin[0].err)
        return ctx->fail(TPE_ERR_ARG, "tpe_merge_results_device: a part holds a value-only record "
                                      "(TPE_OPT_VALUE_ONLY): it has no score to merge by");
    return TPE_OK;
}

int tpe_merge_results(const tpe_label_result* parts, int32_t n_parts, int32_t n,
                      tpe_label_result* out) {
    if (!parts || !out || n_parts <= 0 || n < 0) return TPE_ERR_ARG;
    for (int64_t j = 0; j < (int64_t)n_parts * n; ++j)
        if (parts[j].index >= 0 && parts[j].status == TPE_STATUS_VALUE_ONLY) return TPE_ERR_ARG;
    for (int32_t j = 0; j < n; ++j) {
        tpe_label_result best = parts[j];
        for (int32_t p = 1; p < n_parts; ++p) {
            const tpe_label_result& c = parts[(size_t)p * n + j];
            if (c.index < 0) continue;
            if (best.index < 0 ||
                host_better(order_key(c.score), c.index, order_key(best.score), best.index))
                best = c;
        }
        out[j] = best;
    }
    return TPE_OK;
}

int tpe_last_timing(const tpe_ctx* ctx, float* score_ms, float* round_ms) {
    if (!ctx) return TPE_ERR_ARG;
    if (score_ms) *score_ms = ctx->score_ms;
    if (round_ms) *round_ms = ctx->round_ms;
    return TPE_OK;
}

int64_t tpe_last_evals(const tpe_ctx* ctx) { return ctx ? ctx->evals : -1; }

int tpe_last_screen(const tpe_ctx* ctx, int64_t* screened, int64_t* rescored, float* screen_ms) {
    if (!ctx) return TPE_ERR_ARG;
    if (screened) *screened = ctx->screen_total;
    if (rescored) *rescored = ctx->screen_rescored;
    if (screen_ms) *screen_ms = ctx->screen_ms;
    return TPE_OK;
}

int tpe_last_screen_terms(const tpe_ctx* ctx, int64_t* terms) {
    if (!ctx) return TPE_ERR_ARG;
    if (terms) *terms = ctx->screen_exec;
    return TPE_OK;
}

int32_t tpe_last_screen_mode(const tpe_ctx* ctx) { return ctx ? ctx->screen_mode : -1; }

int tpe_last_prepare(tpe_ctx* ctx, float* ms) {
    if (!ctx) return TPE_ERR_ARG;
    if (ctx->prep_pending) {
        HIPCHK(ctx, hipEventSynchronize(ctx->ev_prep[1]));
        HIPCHK(ctx, hipEventElapsedTime(&ctx->prep_ms, ctx->ev_prep[0], ctx->ev_prep[1]));
        ctx->prep_pending = false;
    }
    if (ms) *ms = ctx->prep_ms;
    return TPE_OK;
}

int tpe_last_hot(const tpe_ctx* ctx, int64_t* listed, int32_t* fallback) {
    if (!ctx) return TPE_ERR_ARG;
    if (listed) *listed = ctx->hot_ran ? ctx->hot_listed : -1;
    if (fallback) *fallback = ctx->hot_fallback;
    return TPE_OK;
}

int tpe_last_drawn(const tpe_ctx* ctx, int64_t* quantized, int64_t* categorical) {
    if (!ctx) return TPE_ERR_ARG;
    if (quantized) *quantized = (int64_t)ctx->xdrawn_h[0];
    if (categorical) *categorical = (int64_t)ctx->xdrawn_h[1];
    return TPE_OK;
}

int64_t tpe_device_bytes(void) { return tpe_rt::device_bytes_held().load(std::memory_order_relaxed); }

int tpe_last_rescore_terms(const tpe_ctx* ctx, int64_t* terms) {
    if (!ctx) return TPE_ERR_ARG;
    if (terms) *terms = ctx->screen_rescore_terms;
    return TPE_OK;
}

TPE_DEV int tpe1_prepare(tpe_ctx* ctx, int64_t n_candidates, int32_t n_rounds) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (!ctx->P || ctx->P->n_labels <= 0) return ctx->fail(TPE_ERR_ARG, "no resident posterior");
    if (n_candidates < 0 || n_rounds < 1) return ctx->fail(TPE_ERR_ARG, "bad candidate/round count");
    // the rounds that use the index: tile rounds of >= kWinMinN candidates,
    // packed rounds of >= kWinMinN slots in total (launch_dense)
    if (ctx->precision != TPE_F64 || !ctx->screen || !ctx->expand || n_candidates * n_rounds < kWinMinN)
        return TPE_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    ctx->bx_t_next = n_candidates >= kTile ? kBxTTile : kBxT;   // (the map the rounds take)
    int rc = tpe_rt::bx_prepare(ctx);
    if (rc == TPE_OK && ctx->hot && n_candidates >= kWinMinN) rc = hot_tau_prepare(ctx, n_candidates);
    return rc;
}

TPE_DEV int tpe1_arm_prepare(tpe_ctx* ctx, int64_t n_candidates, int32_t n_rounds) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (n_candidates < 0 || (n_candidates > 0 && n_rounds < 1))
        return ctx->fail(TPE_ERR_ARG, "bad candidate/round count");
    ctx->arm_c = n_candidates;
    ctx->arm_r = n_candidates > 0 ? n_rounds : 0;
    return TPE_OK;
}

TPE_DEV int tpe1_set_option(tpe_ctx* ctx, int32_t option, int64_t value) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);   // (the header's rule: a pending deferred rebuild's report first)
    switch (option) {
        case TPE_OPT_SCREEN: ctx->screen = value != 0; break;
        case TPE_OPT_SPLITK: ctx->splitk = value != 0; break;
        case TPE_OPT_DEDUP: ctx->dedup = value != 0; break;
        case TPE_OPT_CHUNKS:
            if (value < 0 || value > 4096) return ctx->fail(TPE_ERR_ARG, "chunks must be in [0, 4096]");
            ctx->chunks_forced = (int32_t)value;
            break;
        case TPE_OPT_TIMING: ctx->timing = value != 0; break;
        case TPE_OPT_WINDOW: ctx->window = value != 0; break;
        case TPE_OPT_EXPAND: ctx->expand = value != 0; break;
        case TPE_OPT_EARLY: ctx->early = value != 0; break;
        case TPE_OPT_ZERO_WIN: ctx->zero_win = value != 0; break;
        case TPE_OPT_VALUE_ONLY: ctx->value_only = value != 0; break;
        case TPE_OPT_BX_T:
            if (value != 0 && (value < 32 || value > 128)) return ctx->fail(TPE_ERR_ARG, "index cut T must be 0 or in [32, 128]");
            ctx->bx_t_force = (int32_t)value;
            break;
        case TPE_OPT_PK_SLICED:
            if (value < 0 || value > kSlicedRescoreMax)
                return ctx->fail(TPE_ERR_ARG, "packed sliced re-score limit must be in [0, 65536]");
            ctx->pk_sliced = value;
            break;
        case TPE_OPT_DEFER_REPORT:
            if (!ctx->peers.empty() && value) return ctx->fail(TPE_ERR_ARG, "deferred reports: single-device contexts only");
            ctx->build.defer = value != 0;
            break;
        case TPE_OPT_BX_SPLIT:
            if (value < 0 || value > 8) return ctx->fail(TPE_ERR_ARG, "index window split must be in [0, 8]");
            ctx->bx_split = (int32_t)value;
            break;
        case TPE_OPT_MODE_MASK:
            if (value < 1 || value > 31) return ctx->fail(TPE_ERR_ARG, "family mask must be in [1, 31]");
            ctx->mode_mask = (int32_t)value;
            break;
        case TPE_OPT_AUX_FAMILIES: ctx->aux_families = value != 0; break;
        case TPE_OPT_RESCORE_CAP:
            if (value < 1) return ctx->fail(TPE_ERR_ARG, "re-score capacity must be positive");
            ctx->pk_cap = value;
            break;
        case TPE_OPT_HOT_DIV:
            if (value < 1 || value > (1 << 20)) return ctx->fail(TPE_ERR_ARG, "hot list divisor must be in [1, 2^20]");
            ctx->hot_cap_div = (double)value;
            break;
        case TPE_OPT_HOT:
            if (value < 0 || value > 2) return ctx->fail(TPE_ERR_ARG, "hot must be 0, 1 or 2");
            ctx->hot = (int32_t)value;
            break;
        case TPE_OPT_WIN_GROUPS:
            if (value < 0 || value > 64) return ctx->fail(TPE_ERR_ARG, "window groups must be in [0, 64]");
            ctx->win_groups = (int32_t)value;
            break;
        case TPE_OPT_WIN_T:
            if (value < 8 || value > 62) return ctx->fail(TPE_ERR_ARG, "window cut must be in [8, 62]");
            ctx->win_t = (int32_t)value;
            break;
        case TPE_OPT_WHOLE_N:
            if (value < 0) return ctx->fail(TPE_ERR_ARG, "whole candidate count must be >= 0");
            ctx->opt_whole_n = value;
            break;
        case TPE_OPT_WHOLE_ROUNDS:
            if (value < 0 || value > INT32_MAX) return ctx->fail(TPE_ERR_ARG, "whole round count");
            ctx->opt_whole_rounds = (int32_t)value;
            break;
        default: return ctx->fail(TPE_ERR_ARG, "unknown option " + std::to_string(option));
    }
    return TPE_OK;
}

int tpe_last_mode_stats(const tpe_ctx* ctx, float* ms, int64_t* evals) {
    if (!ctx) return TPE_ERR_ARG;
    for (int m = 0; m < kNumModes; ++m) {
        if (ms) ms[m] = ctx->mode_ms[m];
        if (evals) evals[m] = ctx->mode_evals[m];
    }
    return TPE_OK;
}

// ---- single-op entry points: a one-label posterior with both sides equal ----
// They run on the context's one-label slot; the resident posterior is
// untouched (restored on every return path).

namespace {
struct SingleSlot {
    tpe_ctx* ctx;
    explicit SingleSlot(tpe_ctx* c) : ctx(c) { ctx->P = &ctx->single; }
    ~SingleSlot() { ctx->P = &ctx->resident; }
};
}  // namespace

static int one_label_lpdf(tpe_ctx* ctx, int kind, const double* samples, int64_t n,
                          const double* w, const double* mu, const double* sg, int32_t k,
                          int32_t flags, double low, double high, double q, double* out) {
    if (!ctx) return TPE_ERR_ARG;
    SingleSlot slot(ctx);
    if (n == 0) return TPE_OK;  // empty samples -> empty result (tpe.py:115-116)
    if (!samples || !out || !w || !mu || !sg) return ctx->fail(TPE_ERR_ARG, "null pointer");
    tpe_label_desc d{};
    d.kind = kind;
    d.flags = flags;
    d.low = low;
    d.high = high;
    d.q = q;
    d.n_below = d.n_above = k;
    // the lpdf never checks low < high (only the samplers do)
    int rc = set_posterior_impl(ctx, &d, 1, w, mu, sg, k, false);
    if (rc) return rc;
    tpe_label_result r;
    return tpe_score(ctx, 0, samples, n, out, nullptr, &r);
}

int tpe_gmm1_lpdf(tpe_ctx* ctx, const double* samples, int64_t n, const double* weights,
                  const double* mus, const double* sigmas, int32_t k, int32_t flags, double low,
                  double high, double q, double* out) {
    TPE_SETTLE(ctx);
    return one_label_lpdf(ctx, TPE_GMM1, samples, n, weights, mus, sigmas, k, flags, low, high, q, out);
}

int tpe_lgmm1_lpdf(tpe_ctx* ctx, const double* samples, int64_t n, const double* weights,
                   const double* mus, const double* sigmas, int32_t k, int32_t flags, double low,
                   double high, double q, double* out) {
    TPE_SETTLE(ctx);
    return one_label_lpdf(ctx, TPE_LGMM1, samples, n, weights, mus, sigmas, k, flags, low, high, q, out);
}

int tpe_categorical_lpdf(tpe_ctx* ctx, const int64_t* samples, int64_t n, const double* p,
                         int32_t upper, double* out) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    SingleSlot slot(ctx);
    if (n == 0) return TPE_OK;
    if (!samples || !p || !out || upper <= 0) return ctx->fail(TPE_ERR_ARG, "bad arguments");
    tpe_label_desc d{};
    d.kind = TPE_CATEGORICAL;
    d.n_below = d.n_above = upper;
    int rc = set_posterior_impl(ctx, &d, 1, p, nullptr, nullptr, upper, false);
    if (rc) return rc;
    std::vector<double> c(n);
    for (int64_t i = 0; i < n; ++i) c[i] = (double)samples[i];
    tpe_label_result r;
    return tpe_score(ctx, 0, c.data(), n, out, nullptr, &r);
}

int tpe_broadcast_best(tpe_ctx* ctx, const double* below, const double* above, int64_t n,
                       int64_t* best) {
    if (!ctx || !best) return TPE_ERR_ARG;
    if (n <= 0) {
        *best = -1;
        return TPE_OK;
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, ctx->out_lb.reserve(n));
    HIPCHK(ctx, ctx->out_la.reserve(n));
    const int blocks = (int)std::min<int64_t>((n + kBlock - 1) / kBlock, 1024);
    HIPCHK(ctx, ctx->partials.reserve(blocks));
    HIPCHK(ctx, hipMemcpyAsync(ctx->out_lb.p, below, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->out_la.p, above, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_argmax, dim3(blocks), dim3(kBlock), 0, ctx->stream, ctx->out_lb.p,
                       ctx->out_la.p, n, ctx->partials.p);
    HIPCHK(ctx, hipGetLastError());
    std::vector<Partial> parts(blocks);
    HIPCHK(ctx, hipMemcpyAsync(parts.data(), ctx->partials.p, blocks * sizeof(Partial),
                               hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t bk = 0;
    int64_t bi = INT64_MAX;
    for (const Partial& p : parts)
        if (host_better(p.key, p.idx, bk, bi)) {
            bk = p.key;
            bi = p.idx;
        }
    *best = bi;
    return TPE_OK;
}

static int one_label_sample(tpe_ctx* ctx, int kind, const double* w, const double* mu,
                            const double* sg, int32_t k, int32_t flags, double low, double high,
                            double q, uint64_t seed, uint32_t stream, uint32_t round,
                            int64_t offset, int64_t n, double* out) {
    if (!ctx) return TPE_ERR_ARG;
    SingleSlot slot(ctx);
    if (n == 0) return TPE_OK;
    if (!out || !w) return ctx->fail(TPE_ERR_ARG, "null pointer");
    if (offset < 0 || offset + n > (int64_t)UINT32_MAX)
        return ctx->fail(TPE_ERR_ARG, "candidate indices must stay below 2^32");
    tpe_label_desc d{};
    d.kind = kind;
    d.flags = flags;
    d.low = low;
    d.high = high;
    d.q = q;
    d.n_below = d.n_above = k;
    int rc = set_posterior_impl(ctx, &d, 1, w, mu, sg, k, true);
    if (rc) return rc;
    ctx->P->h_labels[0].stream = (int32_t)stream;
    HIPCHK(ctx, hipMemcpy(ctx->P->labels.p, ctx->P->h_labels.data(), sizeof(DLabel), hipMemcpyHostToDevice));
    HIPCHK(ctx, ctx->cand.reserve(std::max<int64_t>(n, 1)));
    HIPCHK(ctx, ctx->rounds.reserve(1));
    HIPCHK(ctx, ctx->errflag.reserve(1));
    HIPCHK(ctx, hipMemcpyAsync(ctx->rounds.p, &round, sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->errflag.p, 0, sizeof(int32_t), ctx->stream));
    launch_sample_only(ctx, ctx->P->h_labels[0].mode, n, offset, seed, ctx->cand.p);
    HIPCHK(ctx, hipGetLastError());
    int32_t errh = 0;
    HIPCHK(ctx, hipMemcpyAsync(&errh, ctx->errflag.p, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(out, ctx->cand.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (errh & 1) return ctx->fail(TPE_ERR_SAMPLE, "truncated sampler: interval [low, high) not reached");
    return TPE_OK;
}

int tpe_gmm1_sample(tpe_ctx* ctx, const double* w, const double* mu, const double* sg, int32_t k,
                    int32_t flags, double low, double high, double q, uint64_t seed,
                    uint32_t stream, uint32_t round, int64_t offset, int64_t n, double* out) {
    TPE_SETTLE(ctx);
    return one_label_sample(ctx, TPE_GMM1, w, mu, sg, k, flags, low, high, q, seed, stream, round,
                            offset, n, out);
}

int tpe_lgmm1_sample(tpe_ctx* ctx, const double* w, const double* mu, const double* sg, int32_t k,
                     int32_t flags, double low, double high, double q, uint64_t seed,
                     uint32_t stream, uint32_t round, int64_t offset, int64_t n, double* out) {
    TPE_SETTLE(ctx);
    return one_label_sample(ctx, TPE_LGMM1, w, mu, sg, k, flags, low, high, q, seed, stream, round,
                            offset, n, out);
}

int tpe_categorical_sample(tpe_ctx* ctx, const double* p, int32_t upper, uint64_t seed,
                           uint32_t stream, uint32_t round, int64_t offset, int64_t n,
                           int64_t* out) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (n == 0) return TPE_OK;
    if (!out) return ctx->fail(TPE_ERR_ARG, "null pointer");
    std::vector<double> tmp(n);
    int rc = one_label_sample(ctx, TPE_CATEGORICAL, p, nullptr, nullptr, upper, 0, 0, 0, 0, seed,
                              stream, round, offset, n, tmp.data());
    if (rc) return rc;
    for (int64_t i = 0; i < n; ++i) out[i] = (int64_t)tmp[i];
    return TPE_OK;
}

}  // extern "C"
