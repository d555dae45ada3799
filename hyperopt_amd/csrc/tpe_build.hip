// tpe_build.hip -- the device posterior builder:
// the per-suggestion descriptor build that the reference redoes in Python on
// every call -- ap_filter_trials (hyperopt/tpe.py:624-648),
// linear_forgetting_weights (:385-398), adaptive_parzen_normal (:404-477),
// the categorical pseudocount posteriors (:581-617) -- for every label at
// once, followed by the fold into the engine's resident records (the same
// records tpe_set_posterior uploads).  Entry point: tpe_build_posterior.
//
// Pipeline (one HIP stream, no host round trip until the final DLabel read):
//   k_split      one workgroup: the n_below lowest losses (lexicographic
//                (loss, position) order -> a flag per trial)
//   k_partition  one workgroup per label: order-preserving split of the
//                label's observations into below / above (ballot + scan)
//   segmented radix sort (hipCUB) of every above list, stable
//   k_parzen     one workgroup per (label, side): sorted means with the prior
//                inserted, gap sigmas, clip, linear-forgetting weights,
//                numpy-ordered normalisation; categorical: weighted bincount
//                in observation order + pseudocounts
//   k_fold       one workgroup per label: p_accept, LSE shift, recentred
//                exp-scaled records, sampling records, DLabel fields
//
// Bit-exactness: every arithmetic step of the mixture build is an IEEE
// add/sub/mul/div/max in the reference's order (no FMA contraction), and sums
// follow numpy's pairwise summation tree, so (weights, mus, sigmas) equal the
// reference's for the same observations -- except where the reference itself
// is implementation-defined: np.argsort's (unstable quicksort) order of tied
// losses and tied observations.  Here ties are ordered by position (stable).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hyperopt_tpe.h"
#include "tpe_ctx.h"
#include "tpe_device.h"

using namespace tpe;
using namespace tpe_rt;

namespace {

constexpr int kSplitBlock = 1024;
constexpr int kPartBlock = 1024;
constexpr int kPartU = 4;   // k_partition: sub-chunks of kPartBlock per step
constexpr int kParzenBlock = 1024;
// k_parzen's and k_fold's loops take kFoldU components per thread per step,
// their loads issued together: one workgroup per label walks ~37k
// components at config 5, and one load round trip per element and loop made
// each ~0.2 ms (r5an).  Per component the arithmetic is unchanged; the
// loops' reductions are counts, min / max and flags (order-free).
constexpr int kFoldU = 4;
constexpr int kMaxLF = 64;          // below-list capacity per label (lf <= kMaxLF)
constexpr int kCatChunk = 8192;     // categorical bincount: observations staged in LDS
constexpr int kCatFewBins = 32;     // categorical bincount by ordered bin compaction up to here
constexpr int kCatFewChunk = 4096;  // its chunk: 64 groups of 64 (one wave scans the groups)

// ------------------------------------------------ numpy pairwise summation --
// np.sum of a contiguous float64 vector: chunks of 8192 (numpy's reduction
// buffer) added in order to 0.0; each chunk summed pairwise -- split n > 128
// at n2 = n/2 - (n/2) % 8, leaves of <= 128 with 8 accumulators
// (numpy/_core/src/umath/loops_utils.h.src).  On the device the leaves are
// summed in parallel and combined in the same tree order.

// The tree of one chunk (<= 8192 elements) has depth <= 7 and <= 65 leaves;
// every split point is a multiple of 8, so every leaf starts at a multiple
// of 8.  A partial (tail) chunk's tree is handled in parallel from register
// descents only: each 8-lane group descends from the root to the leaf holding
// its position 8q and sums it if the leaf starts there (the sum lands in LDS
// slot q), then the inner nodes are combined bottom-up, one level per
// barrier, each node adding its right child's slot into its left child's --
// the (left + right) order of numpy's recursion.
constexpr int64_t kNpChunk = 8192;
constexpr int kNpChunkLeaves = 64;   // a full chunk: 64 leaves of 128
constexpr int kPwDepth = 7;          // >= the depth of any tree of n < 8192
constexpr int kTailSlots = kNpChunk / 8;

__device__ __forceinline__ int32_t pw_split(int32_t n) {
    int32_t n2 = n / 2;
    return n2 - n2 % 8;
}

// the leaf (start, length) of the tree of n that holds position p
__device__ __forceinline__ void pw_leaf_at(int32_t n, int32_t p, int32_t& s0, int32_t& n0) {
    s0 = 0;
    n0 = n;
#pragma unroll
    for (int d = 0; d <= kPwDepth; ++d) {
        if (n0 <= 128) break;
        const int32_t n2 = pw_split(n0);
        if (p < s0 + n2) {
            n0 = n2;
        } else {
            s0 += n2;
            n0 -= n2;
        }
    }
}

// the node at depth d on path `path` (bit d-1 first; 0 = left); false if a
// leaf ends the path earlier
__device__ __forceinline__ bool pw_node_at(int32_t n, int d, int path, int32_t& s0, int32_t& n0) {
    s0 = 0;
    n0 = n;
    for (int k = d - 1; k >= 0; --k) {
        if (n0 <= 128) return false;
        const int32_t n2 = pw_split(n0);
        if ((path >> k) & 1) {
            s0 += n2;
            n0 -= n2;
        } else {
            n0 = n2;
        }
    }
    return true;
}

// np.sum(a[0:n]) by one workgroup: numpy reduces in buffer-sized chunks of
// 8192 elements, accumulated sequentially from 0.0, each chunk summed
// pairwise.  Leaves are summed in parallel (full chunks: 64 leaves of 128;
// the tail chunk's leaves found by register descents), the full chunks'
// balanced trees combined one chunk per thread, the tail's tree level by
// level, chunks added in order.  leaf_sum is this call's private global
// scratch (capacity >= n / 56 + 1).  Every thread returns the sum.
__device__ double block_np_sum(const double* __restrict__ a, int64_t n, double* __restrict__ leaf_sum) {
#pragma clang fp contract(off)
    __shared__ double chunk_sum[64];
    __shared__ double tail_slot[kTailSlots];
    __shared__ double res_sh;
    const int64_t n_chunks = (n + kNpChunk - 1) / kNpChunk;
    const int64_t full = n / kNpChunk;
    const int32_t tail = (int32_t)(n - full * kNpChunk);
    const int64_t n_full_leaves = full * kNpChunkLeaves;
    const int64_t total = n_full_leaves + (tail + 7) / 8;   // full leaves + tail positions
    __syncthreads();   // a[] was just written by the other threads of the block
    // leaves: 8 lanes per leaf, lane j accumulating pairwise_sum's r_j (the
    // stride-8 elements j, j + 8, ... in order -- all its loads in flight at
    // once), the ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) combine by
    // xor shuffles, then lane 0 adds the leaf's last n % 8 elements in order.
    // Tail positions that do not start a leaf have len 0 (uniform per group).
    for (int64_t t8 = threadIdx.x; t8 < total * 8; t8 += blockDim.x) {
        const int64_t t = t8 >> 3;
        const int j = (int)(t8 & 7);
        int64_t s, len;
        if (t < n_full_leaves) {
            s = t * 128;
            len = 128;
        } else {
            const int32_t p = (int32_t)(t - n_full_leaves) * 8;
            int32_t s0, n0;
            pw_leaf_at(tail, p, s0, n0);
            s = full * kNpChunk + p;
            len = s0 == p ? n0 : 0;
        }
        const double* x = a + s;
        const int64_t body = len - len % 8;
        double r = 0.0;
        if (len >= 8) {
            double v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = (8 * m + j < body) ? x[8 * m + j] : 0.0;
            r = v[0];
#pragma unroll
            for (int m = 1; m < 16; ++m)
                if (8 * m + j < body) r += v[m];
        }
        r += __shfl_xor(r, 1);
        r += __shfl_xor(r, 2);
        r += __shfl_xor(r, 4);
        if (j == 0 && (t < n_full_leaves || len > 0)) {
            double res;
            if (len < 8) {
                res = 0.0;
                for (int64_t i = 0; i < len; ++i) res += x[i];
            } else {
                res = r;
                for (int64_t i = body; i < len; ++i) res += x[i];
            }
            if (t < n_full_leaves) leaf_sum[t] = res;
            else tail_slot[t - n_full_leaves] = res;
        }
    }
    __syncthreads();
    // the tail's inner nodes, deepest level first: node (s0, n0) adds its
    // right child's slot into its left child's (= its own) slot
    if (tail > 128) {
        for (int d = kPwDepth - 1; d >= 0; --d) {
            for (int path = threadIdx.x; path < (1 << d); path += blockDim.x) {
                int32_t s0, n0;
                if (pw_node_at(tail, d, path, s0, n0) && n0 > 128)
                    tail_slot[s0 / 8] = tail_slot[s0 / 8] + tail_slot[(s0 + pw_split(n0)) / 8];
            }
            __syncthreads();
        }
    }
    // full chunk trees: one thread per chunk; sums beyond 64 chunks go
    // through the leaf buffer's own slots (each chunk's first leaf slot is
    // free once read)
    for (int64_t c = threadIdx.x; c < n_chunks; c += blockDim.x) {
        double v;
        if (c < full) {   // a full chunk's tree is perfectly balanced: pairs up, level by level
            double t[kNpChunkLeaves / 2];
            const double* ls = leaf_sum + c * kNpChunkLeaves;
#pragma unroll
            for (int j = 0; j < kNpChunkLeaves / 2; ++j) t[j] = ls[2 * j] + ls[2 * j + 1];
#pragma unroll
            for (int w = kNpChunkLeaves / 4; w >= 1; w /= 2)
#pragma unroll
                for (int j = 0; j < w; ++j) t[j] = t[2 * j] + t[2 * j + 1];
            v = t[0];
        } else {
            v = tail_slot[0];
        }
        if (c < 64) chunk_sum[c] = v;
        else leaf_sum[c * kNpChunkLeaves] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = 0.0;
        for (int64_t c = 0; c < n_chunks; ++c) r += c < 64 ? chunk_sum[c] : leaf_sum[c * kNpChunkLeaves];
        res_sh = r;
    }
    __syncthreads();
    return res_sh;
}

// ------------------------------------------------------ reference helpers --
// ascending total order of a loss (np.argsort puts NaN last; -0 == +0)
__device__ __forceinline__ uint64_t asc_key(double s) {
    if (s != s) return ~0ull;
    if (s == 0.0) s = 0.0;
    uint64_t b;
    __builtin_memcpy(&b, &s, 8);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// linear_forgetting_weights(n, lf)[i]  (tpe.py:385-398): a linspace(1/n, 1,
// n - lf) ramp (numpy: i * step + start, last element = stop exactly) and
// lf trailing ones.  The ramp constants are computed once per list.
struct LFRamp {
    int64_t num;      // ramp length n - lf (<= 0: all ones)
    double start, step;
};

__device__ __forceinline__ LFRamp lf_ramp(int64_t n, int32_t lf) {
#pragma clang fp contract(off)
    LFRamp r;
    r.num = n < lf ? 0 : n - lf;
    r.start = n > 0 ? 1.0 / (double)n : 0.0;
    r.step = r.num > 1 ? (1.0 - r.start) / (double)(r.num - 1) : 0.0;
    return r;
}

__device__ __forceinline__ double lf_weight(int64_t i, const LFRamp& r) {
#pragma clang fp contract(off)
    if (i >= r.num) return 1.0;
    if (r.num == 1) return r.start;
    if (i == r.num - 1) return 1.0;
    return (double)i * r.step + r.start;
}

__device__ __forceinline__ double np_maximum(double a, double b) { return (a != a || a > b) ? a : b; }
__device__ __forceinline__ double np_minimum(double a, double b) { return (a != a || a < b) ? a : b; }

// --------------------------------------------------------------- kernels --

// ap_filter_trials' split (tpe.py:636-645): flag the n_below lowest losses,
// ties by position.  Radix select in one workgroup: 8 passes of 8-bit digits
// over the order-preserving 64-bit keys locate the n_below-th smallest key
// K* (LDS histograms, wave-aggregated adds), then one pass flags every key
// < K* and the first (by position) of the keys == K* that complete n_below
// -- an ordered pass only when some keys == K* stay out.  That case is a tie
// of equal losses across the n_below boundary, where the reference's
// np.argsort (tpe.py:637, numpy's unstable sort) picks its own members:
// *split_tie is set so the caller can supply the reference's below set
// (tpe_build_posterior_resident_ordered).  R > 0: every thread holds its R
// keys (positions tid, tid + kSplitBlock, ...; T <= R kSplitBlock) in
// registers across the passes instead of reloading them (a history of 10^4
// trials: 32 -> ~10 us); R = 0 walks the losses in every pass.
//
// Slice mode (cand_key != nullptr; k_split_merge finishes): workgroup x
// takes the positions [x R kSplitBlock, (x + 1) R kSplitBlock) of the
// losses, zeroes their below flags and writes its m_sel smallest (key,
// position) pairs -- the keys < its K* and the first by position of those ==
// K* -- to cand[x m_sel ..] (unused slots: key ~0, position -1).  The
// n_below smallest pairs of all T -- the below set, ties by position -- are
// among the slices' n_below + 1 smallest, and so is the next one, whose key
// tells a tie across the boundary (one workgroup walking 50k losses 8 times
// took 115 us, r5an).
template <int R>
__global__ __launch_bounds__(kSplitBlock) void k_split(const double* __restrict__ losses_all, int64_t T_all,
                                                       int32_t n_below_all, uint8_t* __restrict__ below_all,
                                                       int32_t* __restrict__ split_tie, int32_t m_sel,
                                                       uint64_t* __restrict__ cand_key,
                                                       int64_t* __restrict__ cand_pos) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool slice = cand_key != nullptr;
    const int64_t base = slice ? (int64_t)blockIdx.x * R * kSplitBlock : 0;
    const double* losses = losses_all + base;
    uint8_t* below = below_all + base;
    const int64_t T = !slice ? T_all : (T_all - base < (int64_t)R * kSplitBlock ? T_all - base
                                                                                 : (int64_t)R * kSplitBlock);
    const int32_t n_below = !slice ? n_below_all : (int32_t)((int64_t)m_sel < T ? (int64_t)m_sel : T);
    if (slice)
        for (int32_t j = tid; j < m_sel; j += kSplitBlock) {
            cand_key[(size_t)blockIdx.x * m_sel + j] = ~0ull;
            cand_pos[(size_t)blockIdx.x * m_sel + j] = -1;
        }
    uint64_t kr[R > 0 ? R : 1];
    if constexpr (R > 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t i = (int64_t)r * kSplitBlock + tid;
            kr[r] = i < T ? asc_key(losses[i]) : 0ull;
        }
    }
    // f(position, key, valid) over this thread's positions; `valid` is
    // uniform-false only past T (register form: every lane runs every slot)
    auto each = [&](auto&& f) {
        if constexpr (R > 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t i = (int64_t)r * kSplitBlock + tid;
                f(i, kr[r], i < T);
            }
        } else {
            for (int64_t i = tid; i < T; i += kSplitBlock) f(i, asc_key(losses[i]), true);
        }
    };
    __shared__ uint32_t hist[256];
    __shared__ uint64_t prefix_sh;
    __shared__ int64_t need_sh;
    __shared__ int wcnt[kSplitBlock / 64];
    __shared__ uint32_t wsum[4];
    __shared__ int64_t base_sh;
    __shared__ uint32_t eq_sh;
    for (int64_t i = tid; i < T; i += kSplitBlock) below[i] = 0;
    if (n_below <= 0 || T <= 0) return;
    if (tid == 0) {
        prefix_sh = 0;
        need_sh = n_below;   // rank (1-based) of K* among the keys matching the prefix
    }
    uint64_t mask = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int b = tid; b < 256; b += kSplitBlock) hist[b] = 0;
        __syncthreads();
        const uint64_t prefix = prefix_sh;
        // the high digits of similar losses are mostly equal: the lanes that
        // share the first participating lane's digit add once per wave
        each([&](int64_t, uint64_t k, bool valid) {
            const bool part = valid && (k & mask) == prefix;
            const uint32_t d = (uint32_t)(k >> shift) & 255u;
            const uint64_t pm = __ballot(part);
            if (!pm) return;
            const int first = __builtin_ctzll(pm);
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, first);
            const uint64_t same = __ballot(part && d == d0);
            if (lane == first) atomicAdd(&hist[d0], (uint32_t)__popcll(same));
            else if (part && d != d0) atomicAdd(&hist[d], 1u);
        });
        __syncthreads();
        // the digit holding the need-th key: inclusive scan of the histogram
        // over the first four waves (shuffles, then the wave totals); the
        // bin whose range [excl, incl) of ranks holds need takes over
        const int64_t need = need_sh;
        uint32_t h = 0, incl = 0;
        if (tid < 256) {
            h = hist[tid];
            incl = h;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t t = __shfl_up(incl, off);
                if (lane >= off) incl += t;
            }
            if (lane == 63) wsum[wv] = incl;
        }
        __syncthreads();
        if (tid < 256) {
            for (int w = 0; w < wv; ++w) incl += wsum[w];
            const uint32_t excl = incl - h;
            if ((int64_t)excl < need && (int64_t)incl >= need) {
                need_sh = need - excl;
                prefix_sh = prefix | ((uint64_t)tid << shift);
                eq_sh = h;   // after the last digit: the number of keys == K*
            }
        }
        mask |= 255ull << shift;
        __syncthreads();
    }
    const uint64_t kstar = prefix_sh;
    const int64_t take_eq = need_sh;      // how many keys == K* join, in position order
    if (slice) {
        // the keys < K* (any slots), then the first take_eq keys == K* by
        // position after them
        __shared__ int32_t less_sh;
        if (tid == 0) {
            less_sh = 0;
            base_sh = 0;
        }
        __syncthreads();
        uint64_t* ck = cand_key + (size_t)blockIdx.x * m_sel;
        int64_t* cp = cand_pos + (size_t)blockIdx.x * m_sel;
        const int32_t n_less = n_below - (int32_t)take_eq;
        each([&](int64_t i, uint64_t k, bool valid) {
            if (valid && k < kstar) {
                const int32_t q = atomicAdd(&less_sh, 1);
                ck[q] = k;
                cp[q] = base + i;
            }
        });
        const uint64_t lt = (1ull << lane) - 1ull;
        for (int64_t c0 = 0; c0 < T; c0 += kSplitBlock) {
            const int64_t i = c0 + tid;
            const uint64_t k = i < T ? asc_key(losses[i]) : ~0ull;
            const bool eq = i < T && k == kstar;
            const uint64_t m = __ballot(eq);
            if (lane == 0) wcnt[wv] = __popcll(m);
            __syncthreads();
            int64_t r = base_sh + __popcll(m & lt);
            for (int w = 0; w < wv; ++w) r += wcnt[w];
            if (eq && r < take_eq) {
                ck[n_less + r] = k;
                cp[n_less + r] = base + i;
            }
            __syncthreads();
            if (tid == 0)
                for (int w = 0; w < kSplitBlock / 64; ++w) base_sh += wcnt[w];
            __syncthreads();
        }
        return;
    }
    if (take_eq == (int64_t)eq_sh) {      // every key == K* joins: no position order needed
        each([&](int64_t i, uint64_t k, bool valid) {
            if (valid && k <= kstar) below[i] = 1;
        });
        return;
    }
    if (tid == 0) {
        base_sh = 0;
        *split_tie = 1;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int64_t c0 = 0; c0 < T; c0 += kSplitBlock) {
        const int64_t i = c0 + tid;
        uint64_t k = ~0ull;
        if (i < T) k = asc_key(losses[i]);
        const bool eq = i < T && k == kstar;
        const uint64_t m = __ballot(eq);
        if (lane == 0) wcnt[wv] = __popcll(m);
        __syncthreads();
        int64_t r = base_sh + __popcll(m & lt);
        for (int w = 0; w < wv; ++w) r += wcnt[w];
        if (i < T && (k < kstar || (eq && r < take_eq))) below[i] = 1;
        __syncthreads();
        if (tid == 0)
            for (int w = 0; w < kSplitBlock / 64; ++w) base_sh += wcnt[w];
        __syncthreads();
    }
}

// The slices' candidates (k_split slice mode) -> the below set: each
// candidate's rank among all by (key, position), the n_below smallest
// flagged; a tie across the boundary when the next one has the key of the
// last taken.  One workgroup, up to kSplitMergeMax candidates.
constexpr int kSplitMergeMax = 2 * kSplitBlock;
__global__ __launch_bounds__(kSplitBlock) void k_split_merge(const uint64_t* __restrict__ cand_key,
                                                             const int64_t* __restrict__ cand_pos, int32_t n_cand,
                                                             int32_t n_below, uint8_t* __restrict__ below,
                                                             int32_t* __restrict__ split_tie) {
    __shared__ uint64_t ks[kSplitMergeMax];
    __shared__ int64_t ps[kSplitMergeMax];
    __shared__ uint64_t k_last, k_next;
    __shared__ int has_next;
    const int tid = threadIdx.x;
    for (int j = tid; j < n_cand; j += kSplitBlock) {
        ks[j] = cand_key[j];
        ps[j] = cand_pos[j] < 0 ? INT64_MAX : cand_pos[j];   // (unused slots last)
    }
    if (tid == 0) has_next = 0;
    __syncthreads();
    for (int j = tid; j < n_cand; j += kSplitBlock) {
        if (ps[j] == INT64_MAX) continue;
        const uint64_t k = ks[j];
        const int64_t p = ps[j];
        int32_t rank = 0;
        for (int q = 0; q < n_cand; ++q) rank += (ks[q] < k || (ks[q] == k && ps[q] < p)) ? 1 : 0;
        if (rank < n_below) below[p] = 1;
        if (rank == n_below - 1) k_last = k;
        if (rank == n_below) {
            k_next = k;
            has_next = 1;
        }
    }
    __syncthreads();
    if (tid == 0 && has_next && k_next == k_last) *split_tie = 1;
}

// ---------------------------------------------- device-resident history --
// Every label's observations live in a pool region [off, off + cap): in
// observation (tid) order (trial position, value) and, for continuous labels,
// also sorted by value with ties in observation order (key, observation
// index).  Appends sort only the new observations and merge them in.

// new observations of every label -> pool tail; st_idx = local index (sort values)
__global__ __launch_bounds__(kBlock) void k_hist_append(
    const int64_t* __restrict__ st_off, const int32_t* __restrict__ st_trial,
    const double* __restrict__ st_val, const int64_t* __restrict__ p_off,
    const int32_t* __restrict__ cnt_old, int32_t* __restrict__ p_trial, double* __restrict__ p_val,
    int32_t* __restrict__ st_idx) {
    const int l = blockIdx.y;
    const int64_t s0 = st_off[l], m = st_off[l + 1] - s0;
    const int64_t base = p_off[l] + cnt_old[l];
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < m; j += (int64_t)gridDim.x * kBlock) {
        p_trial[base + j] = st_trial[s0 + j];
        p_val[base + j] = st_val[s0 + j];
        st_idx[s0 + j] = (int32_t)j;
    }
}

// Large appends (a whole history at once) sort the staging batch with two
// chip-wide stable radix sorts instead of one block per label: by value, then
// by label.  Same key order and tie order as the segmented sort.
constexpr int64_t kGlobalSortMin = 4096;
__global__ __launch_bounds__(kBlock) void k_iota(int32_t* __restrict__ g, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        g[i] = (int32_t)i;
}

// label of each staging position (upper bound in the CSR offsets, minus one)
__global__ __launch_bounds__(kBlock) void k_label_of(
    const int64_t* __restrict__ st_off, int32_t L, const int32_t* __restrict__ g,
    uint32_t* __restrict__ lab, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int64_t p = g[i];
        int32_t lo = 0, hi = L + 1;
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (st_off[mid] <= p) lo = mid + 1; else hi = mid;
        }
        lab[i] = (uint32_t)(lo - 1);
    }
}

__global__ __launch_bounds__(kBlock) void k_sorted_gather(
    const int32_t* __restrict__ g, const double* __restrict__ st_val,
    const int32_t* __restrict__ st_idx, double* __restrict__ key_out,
    int32_t* __restrict__ idx_out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int32_t p = g[i];
        key_out[i] = st_val[p];
        idx_out[i] = st_idx[p];
    }
}

// copy every label's live prefix into a re-laid-out pool (growth)
__global__ __launch_bounds__(kBlock) void k_hist_regrow(
    const int64_t* __restrict__ off_old, const int64_t* __restrict__ off_new,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ t_old,
    const double* __restrict__ v_old, const double* __restrict__ k_old,
    const int32_t* __restrict__ i_old, int32_t* __restrict__ t_new, double* __restrict__ v_new,
    double* __restrict__ k_new, int32_t* __restrict__ i_new) {
    const int l = blockIdx.y;
    const int64_t a = off_old[l], b = off_new[l];
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < cnt[l]; i += (int64_t)gridDim.x * kBlock) {
        t_new[b + i] = t_old[a + i];
        v_new[b + i] = v_old[a + i];
        k_new[b + i] = k_old[a + i];
        i_new[b + i] = i_old[a + i];
    }
}

// stable merge of the sorted existing keys with the sorted new batch:
// existing element i -> i + #(new keys < key), new element j -> j +
// #(existing keys <= key): equal keys keep observation order
__global__ __launch_bounds__(kBlock) void k_hist_merge(
    const tpe_label_spec* __restrict__ specs, const int64_t* __restrict__ p_off,
    const int32_t* __restrict__ cnt_old, const int64_t* __restrict__ st_off,
    const double* __restrict__ s_key, const int32_t* __restrict__ s_idx,
    const double* __restrict__ n_key, const int32_t* __restrict__ n_idx,
    double* __restrict__ o_key, int32_t* __restrict__ o_idx) {
    const int l = blockIdx.y;
    if (specs[l].kind == TPE_CATEGORICAL) return;   // categorical: observation order only
    const int64_t off = p_off[l], c = cnt_old[l];
    const int64_t s0 = st_off[l], m = st_off[l + 1] - s0;
    const double* ok = s_key + off;
    const double* nk = n_key + s0;
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < c + m; e += (int64_t)gridDim.x * kBlock) {
        if (e < c) {
            const double k = ok[e];
            int64_t lo = 0, hi = m;                 // lower bound in the new batch
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (nk[mid] < k) lo = mid + 1; else hi = mid;
            }
            o_key[off + e + lo] = k;
            o_idx[off + e + lo] = s_idx[off + e];
        } else {
            const int64_t j = e - c;
            const double k = nk[j];
            int64_t lo = 0, hi = c;                 // upper bound in the existing keys
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (ok[mid] <= k) lo = mid + 1; else hi = mid;
            }
            o_key[off + j + lo] = k;
            o_idx[off + j + lo] = (int32_t)(c + n_idx[s0 + j]);
        }
    }
}

// ap_filter_trials' membership (tpe.py:639-646) from the resident history:
// phase A walks the observations in (tid) order -- the below list (<= lf, in
// order) and, per observation, its rank in the above list (-1 if it is not
// there); categorical labels keep their above list in observation order.
// Phase B walks a continuous label's value-sorted observations and keeps the
// above ones, in sorted order, with their above-list rank (the index the
// linear-forgetting weights are taken at).  Observations of trials without a
// loss (position < 0 or NaN loss) belong to neither set, as in the reference.
__global__ __launch_bounds__(kPartBlock) void k_partition(
    const tpe_label_spec* __restrict__ specs, const int64_t* __restrict__ p_off,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ p_trial,
    const double* __restrict__ p_val, const double* __restrict__ s_key,
    const int32_t* __restrict__ s_idx, const uint8_t* __restrict__ below,
    const double* __restrict__ losses, int64_t T, double* __restrict__ below_val,
    int32_t* __restrict__ arank, double* __restrict__ keys, int32_t* __restrict__ idx,
    int32_t* __restrict__ counts, int32_t* __restrict__ err, const int32_t* __restrict__ only) {
    const int l = only ? only[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t off = p_off[l], M = cnt[l];
    const bool cat = specs[l].kind == TPE_CATEGORICAL;
    __shared__ int base_b, base_a;
    if (tid == 0) base_b = base_a = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    // kPartU sub-chunks of kPartBlock observations per step: their loads
    // issued together, their ballots counted per wave, ONE barrier pair for
    // all of them (4 loads and 3 barriers per 1024 observations before: ~0.16
    // ms per 50k-observation label, r5an); positions and ranks unchanged
    constexpr int kW = kPartBlock / 64;
    __shared__ int wbu[kPartU][kW], wau[kPartU][kW];
    for (int64_t c0 = 0; c0 < M; c0 += (int64_t)kPartU * kPartBlock) {
        int32_t tr[kPartU];
        double vv[kPartU];
#pragma unroll
        for (int u = 0; u < kPartU; ++u) {
            const int64_t i = c0 + (int64_t)u * kPartBlock + tid;
            tr[u] = i < M ? p_trial[off + i] : -1;
            vv[u] = i < M ? p_val[off + i] : 0.0;
        }
        bool isb[kPartU], isa[kPartU];
#pragma unroll
        for (int u = 0; u < kPartU; ++u) {
            const int64_t i = c0 + (int64_t)u * kPartBlock + tid;
            const int32_t t = tr[u];
            isb[u] = isa[u] = false;
            if (i < M) {
                if (t >= 0 && t < T) {
                    const double ls = losses[t];
                    isb[u] = below[t] != 0;
                    isa[u] = !isb[u] && ls == ls;
                } else if (t >= T) {
                    atomicOr(err, 1);
                }
            }
        }
        uint64_t bb[kPartU], ba[kPartU];
#pragma unroll
        for (int u = 0; u < kPartU; ++u) {
            bb[u] = __ballot(isb[u]);
            ba[u] = __ballot(isa[u]);
            if (lane == 0) {
                wbu[u][wv] = __popcll(bb[u]);
                wau[u][wv] = __popcll(ba[u]);
            }
        }
        __syncthreads();
        int ob = base_b, oa = base_a;
#pragma unroll
        for (int u = 0; u < kPartU; ++u) {
            int pb = ob, pa = oa;   // this sub-chunk's wave offsets
            for (int w = 0; w < wv; ++w) {
                pb += wbu[u][w];
                pa += wau[u][w];
            }
            const int64_t i = c0 + (int64_t)u * kPartBlock + tid;
            if (isb[u]) {
                const int p = pb + __popcll(bb[u] & lt);
                if (p < kMaxLF) below_val[(size_t)l * kMaxLF + p] = vv[u];
                else atomicOr(err, 2);
            }
            if (i < M) {
                const int p = pa + __popcll(ba[u] & lt);
                if (cat) {
                    if (isa[u]) keys[off + p] = vv[u];
                } else {
                    arank[off + i] = isa[u] ? p : -1;
                }
            }
            for (int w = 0; w < kW; ++w) {   // (the sub-chunk's totals)
                ob += wbu[u][w];
                oa += wau[u][w];
            }
        }
        __syncthreads();
        if (tid == 0) {
            base_b = ob;
            base_a = oa;
        }
        __syncthreads();
    }
    const int nb = base_b, na = base_a;
    if (!cat) {   // phase B: sorted order
        __syncthreads();
        if (tid == 0) base_a = 0;
        __syncthreads();
        for (int64_t c0 = 0; c0 < M; c0 += (int64_t)kPartU * kPartBlock) {
            int32_t si_[kPartU];
            double kk[kPartU];
#pragma unroll
            for (int u = 0; u < kPartU; ++u) {
                const int64_t i = c0 + (int64_t)u * kPartBlock + tid;
                si_[u] = i < M ? s_idx[off + i] : 0;
                kk[u] = i < M ? s_key[off + i] : 0.0;
            }
            int32_t r[kPartU];
#pragma unroll
            for (int u = 0; u < kPartU; ++u) {
                const int64_t i = c0 + (int64_t)u * kPartBlock + tid;
                r[u] = i < M ? arank[off + si_[u]] : -1;
            }
            uint64_t ba[kPartU];
#pragma unroll
            for (int u = 0; u < kPartU; ++u) {
                ba[u] = __ballot(r[u] >= 0);
                if (lane == 0) wau[u][wv] = __popcll(ba[u]);
            }
            __syncthreads();
            int oa = base_a;
#pragma unroll
            for (int u = 0; u < kPartU; ++u) {
                int pa = oa;
                for (int w = 0; w < wv; ++w) pa += wau[u][w];
                if (r[u] >= 0) {
                    const int p = pa + __popcll(ba[u] & lt);
                    keys[off + p] = kk[u];
                    idx[off + p] = r[u];
                }
                for (int w = 0; w < kW; ++w) oa += wau[u][w];
            }
            __syncthreads();
            if (tid == 0) base_a = oa;
            __syncthreads();
        }
    }
    if (tid == 0) {
        counts[2 * l] = nb;
        counts[2 * l + 1] = na;
    }
}

// np.bincount(obs, weights=lf, minlength=upper) for upper <= kCatFewBins:
// every bin is a sequential sum in observation order, so the work is
// reordered around that chain instead of walking the list once per bin.
// Per chunk of kCatFewChunk observations:
//   1. per 64-observation group, a ballot per bin -> the group's bin counts;
//   2. one wave per bin scans its counts over the (<= 64) groups, and wave 0
//      scans the bin totals: every observation's slot in a bin-major list
//      whose bins keep observation order (a stable counting sort);
//   3. each observation's weight goes to its slot;
//   4. lane 0 of one wave per bin adds its bin's run in order, 16 LDS reads
//      in flight per batch -- the same additions, in the same order, as
//      np.bincount's loop.
// `out` (= w + o, zeroed) receives the counts; cbin is the caller's LDS.
__device__ void cat_bincount_few(const double* __restrict__ list, int64_t n, int32_t upper,
                                 const LFRamp& ramp, double* __restrict__ out,
                                 int32_t* __restrict__ cbin) {
#pragma clang fp contract(off)
    constexpr int kGroups = kCatFewChunk / 64;
    static_assert(kGroups <= 64, "one wave scans the groups");
    static_assert(kCatFewChunk <= kCatChunk, "cbin holds a chunk");
    __shared__ double cw[kCatFewChunk];
    __shared__ int32_t gcnt[kGroups][kCatFewBins];
    __shared__ int32_t btot[kCatFewBins], bbase[kCatFewBins];
    __shared__ double bsum[kCatFewBins];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    constexpr int kWaves = kParzenBlock / 64;
    if (tid < upper) bsum[tid] = 0.0;
    for (int64_t c0 = 0; c0 < n; c0 += kCatFewChunk) {
        const int m = (int)(n - c0 < kCatFewChunk ? n - c0 : kCatFewChunk);
        const int groups = (m + 63) / 64;
        // 1. bin ids (-1: not a bin) and per-group counts
        for (int g = wave; g < groups; g += kWaves) {
            const int i = g * 64 + lane;
            int32_t cb = -1;
            if (i < m) {
                const double v = list[c0 + i];   // (int64_t)v == b for some bin b, else -1
                cb = (v > -1.0 && v < (double)upper) ? (int32_t)(int64_t)v : -1;
                cbin[i] = cb;
            }
            for (int b = 0; b < upper; ++b) {
                const uint64_t mb = __ballot(cb == b);
                if (lane == b) gcnt[g][b] = __popcll(mb);
            }
        }
        __syncthreads();
        // 2. exclusive prefix of each bin's counts over the groups; bin totals
        for (int b = wave; b < upper; b += kWaves) {
            const int v = lane < groups ? gcnt[lane][b] : 0;
            int inc = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int u = __shfl_up(inc, d);
                if (lane >= d) inc += u;
            }
            if (lane < groups) gcnt[lane][b] = inc - v;
            if (lane == 63) btot[b] = inc;
        }
        __syncthreads();
        if (wave == 0) {
            const int v = lane < upper ? btot[lane] : 0;
            int inc = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int u = __shfl_up(inc, d);
                if (lane >= d) inc += u;
            }
            if (lane < upper) bbase[lane] = inc - v;
        }
        __syncthreads();
        // 3. weights to their slots (rank within the group's bin by mbcnt)
        for (int g = wave; g < groups; g += kWaves) {
            const int i = g * 64 + lane;
            const int32_t cb = i < m ? cbin[i] : -1;
            uint64_t own = 0;
            for (int b = 0; b < upper; ++b) {
                const uint64_t mb = __ballot(cb == b);
                if (cb == b) own = mb;
            }
            if (cb >= 0) {
                const int below = (int)__builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(own >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)own, 0u));
                cw[bbase[cb] + gcnt[g][cb] + below] = lf_weight(c0 + i, ramp);
            }
        }
        __syncthreads();
        // 4. each bin's run, in order, by one lane
        for (int b = wave; b < upper; b += kWaves) {
            if (lane == 0) {
                const double* run = cw + bbase[b];
                const int cnt = btot[b];
                double acc = bsum[b];
                int k = 0;
                for (; k + 16 <= cnt; k += 16) {
                    double v[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) v[j] = run[k + j];
#pragma unroll
                    for (int j = 0; j < 16; ++j) acc += v[j];
                }
                for (; k < cnt; ++k) acc += run[k];
                bsum[b] = acc;
            }
        }
        __syncthreads();
    }
    if (tid < upper) out[tid] = bsum[tid];
}

// adaptive_parzen_normal (tpe.py:404-477) / categorical pseudocounts
// (tpe.py:581-617) of one (label, side).  Output: (w, mu, sigma) at
// mix_off[2 l + side], component count in kcount[2 l + side].
__global__ __launch_bounds__(kParzenBlock) void k_parzen(
    const tpe_label_spec* __restrict__ specs, const double* __restrict__ cat_p,
    const int64_t* __restrict__ obs_off, const int32_t* __restrict__ counts,
    const double* __restrict__ below_val, const double* __restrict__ keys_unsorted,
    const double* __restrict__ keys_sorted, const int32_t* __restrict__ idx_sorted,
    const int64_t* __restrict__ mix_off, double prior_weight, int32_t lf, double* __restrict__ w,
    double* __restrict__ mu, double* __restrict__ sigma, int32_t* __restrict__ kcount,
    double* __restrict__ leaf_sum, const int64_t* __restrict__ order_off, const int32_t* __restrict__ order,
    int32_t* __restrict__ ties, int32_t* __restrict__ err, const int32_t* __restrict__ only) {
#pragma clang fp contract(off)
    const int l = only ? only[blockIdx.x] : (int)blockIdx.x, side = blockIdx.y, tid = threadIdx.x;
    const tpe_label_spec sp = specs[l];
    const int64_t n = counts[2 * l + side];
    const int64_t o = mix_off[2 * l + side];
    const int64_t off = obs_off[l];
    const double pw = prior_weight;
    __shared__ double bk[kMaxLF];
    __shared__ int32_t bi[kMaxLF];

    if (sp.kind == TPE_CATEGORICAL) {
        // weights = linear_forgetting_weights(len(obs)); counts = bincount(obs,
        // minlength=upper, weights) -- each bin a sequential sum in
        // observation order; pseudocounts; / np.sum(pseudocounts)
        // Up to kCatFewBins bins: ordered compaction by bin, then one lane
        // per bin adds its run (cat_bincount_few).  More bins: one wave per
        // bin; ballots over the list find the bin's observations in order,
        // and the wave adds their weights one by one through scalar registers
        // (v_readlane) -- the sequential order of np.bincount.  The list goes
        // through LDS as bin ids, kCatChunk observations at a time (coalesced
        // loads by the whole block; the waves then scan LDS).
        const double* list = side == 0 ? below_val + (size_t)l * kMaxLF : keys_unsorted + off;
        const int32_t upper = sp.upper;
        const LFRamp ramp = lf_ramp(n, lf);
        const int wave = tid >> 6, lane = tid & 63;
        __shared__ int32_t cbin[kCatChunk];
        for (int b = tid; b < upper; b += kParzenBlock) w[o + b] = 0.0;
        if (upper <= kCatFewBins) {
            cat_bincount_few(list, n, upper, ramp, w + o, cbin);
        } else {   // many bins: one wave per bin walks the list
            for (int64_t c0 = 0; c0 < n; c0 += kCatChunk) {
                const int64_t m = n - c0 < kCatChunk ? n - c0 : kCatChunk;
                for (int64_t i = tid; i < m; i += kParzenBlock) {
                    const double v = list[c0 + i];   // (int64_t)v == b for some bin b, else -1
                    cbin[i] = (v > -1.0 && v < (double)upper) ? (int32_t)(int64_t)v : -1;
                }
                __syncthreads();
                for (int b = wave; b < upper; b += kParzenBlock / 64) {
                    double cnt = w[o + b];
                    for (int64_t i0 = 0; i0 < m; i0 += 64) {
                        const int64_t i = i0 + lane;
                        const bool hit = i < m && cbin[i] == b;
                        uint64_t hm = __ballot(hit);
                        if (!hm) continue;
                        const double wl = hit ? lf_weight(c0 + i, ramp) : 0.0;
                        int64_t bits;
                        __builtin_memcpy(&bits, &wl, 8);
                        const int lo = (int)(uint32_t)bits, hi = (int)(uint32_t)(bits >> 32);
                        while (hm) {
                            const int j = __builtin_ctzll(hm);
                            hm &= hm - 1;
                            const uint64_t vb =
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(hi, j) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane(lo, j);
                            double v;
                            __builtin_memcpy(&v, &vb, 8);
                            cnt += v;
                        }
                    }
                    if (lane == 0) w[o + b] = cnt;
                }
                __syncthreads();
            }
        }
        __syncthreads();
        for (int b = tid; b < upper; b += kParzenBlock) {
            const double c = w[o + b];
            const double pseudo = sp.randint ? c + pw
                                             : c + (double)upper * (pw * cat_p[sp.p_off + b]);
            w[o + b] = pseudo;
            mu[o + b] = 0.0;
            sigma[o + b] = 0.0;
        }
        const double tot = block_np_sum(w + o, upper, leaf_sum + o);
        for (int b = tid; b < upper; b += kParzenBlock) w[o + b] = w[o + b] / tot;
        if (tid == 0) kcount[2 * l + side] = upper;
        return;
    }

    // sorted observations: below lists (<= lf) by a stable insertion sort in
    // LDS, above lists from the segmented radix sort (stable)
    const double* sk;
    const int32_t* si;
    if (side == 0) {
        // stable rank sort of the <= kMaxLF below values (ascending total
        // order: NaN last, as np.argsort; ties by position): a thread each
        if (tid < n) {
            const double* bv = below_val + (size_t)l * kMaxLF;
            const double v = bv[tid];
            const uint64_t kv = asc_key(v);
            int rank = 0;
            for (int64_t j = 0; j < n; ++j) {
                const uint64_t kj = asc_key(bv[j]);
                rank += (kj < kv || (kj == kv && j < tid)) ? 1 : 0;
            }
            bk[rank] = v;
            bi[rank] = (int32_t)tid;
        }
        __syncthreads();
        sk = bk;
        si = bi;
    } else {
        sk = keys_sorted + off;
        si = idx_sorted + off;
    }
    // a caller-supplied order of the above observations (the reference's
    // np.argsort(mus), tpe.py:433, computed on the host): same sorted values,
    // but tied observations -- and so their linear-forgetting weights -- in
    // numpy's order instead of by position
    bool supplied = false;
    if (side == 1 && order_off) {
        const int64_t b = order_off[l], e = order_off[l + 1];
        if (e > b) {
            if (e - b != n) {
                if (tid == 0) atomicOr(err, 8);
                return;
            }
            supplied = true;
            si = order + b;
        }
    }
    const double pmu = sp.prior_mu, psig = sp.prior_sigma;
    __shared__ int pos_sh;
    if (tid == 0) pos_sh = 0;
    __syncthreads();
    if (n == 1) {
        if (tid == 0) pos_sh = pmu < sk[0] ? 0 : 1;
    } else if (n >= 2) {
        // np.searchsorted(sorted, prior_mu), side='left' = the number of
        // sorted values < prior_mu: counted by every thread, summed per wave
        int cnt = 0;
        for (int64_t j0 = tid; j0 < n; j0 += (int64_t)kFoldU * kParzenBlock) {
            double v[kFoldU];
#pragma unroll
            for (int u = 0; u < kFoldU; ++u) {
                const int64_t j = j0 + (int64_t)u * kParzenBlock;
                v[u] = j < n ? sk[j] : pmu;   // (pmu: not counted)
            }
#pragma unroll
            for (int u = 0; u < kFoldU; ++u) cnt += v[u] < pmu ? 1 : 0;
        }
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
        if ((tid & 63) == 0 && cnt) atomicAdd(&pos_sh, cnt);
    }
    __syncthreads();
    const int64_t pos = pos_sh, K = n + 1;
    const bool use_lf = lf > 0 && lf < n;
    const LFRamp ramp = lf_ramp(n, lf);
    const double maxsigma = psig / 1.0;
    const double minsigma = psig / fmin(100.0, 1.0 + (double)K);
    // (kFoldU slots per thread per step, their loads issued together: the
    // values around each slot and its observation's rank; r5an)
    auto srtd = [&](int64_t q) { return q < pos ? sk[q] : (q == pos ? pmu : sk[q - 1]); };
    for (int64_t j0 = tid; j0 < K; j0 += (int64_t)kFoldU * kParzenBlock) {
        double vm[kFoldU], v0[kFoldU], vp[kFoldU];
        int32_t rr[kFoldU];
#pragma unroll
        for (int u = 0; u < kFoldU; ++u) {
            const int64_t j = j0 + (int64_t)u * kParzenBlock;
            const bool ok = j < K;
            vm[u] = ok && j >= 1 ? srtd(j - 1) : 0.0;
            v0[u] = ok ? srtd(j) : 0.0;
            vp[u] = ok && j + 1 < K ? srtd(j + 1) : 0.0;
            rr[u] = ok && j != pos ? si[j < pos ? j : j - 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < kFoldU; ++u) {
            const int64_t j = j0 + (int64_t)u * kParzenBlock;
            if (j >= K) continue;
            double s;
            if (n == 0) {
                s = psig;
            } else if (n == 1) {
                s = (j == pos) ? psig : psig * .5;
            } else if (j == 0) {
                s = vp[u] - v0[u];
            } else if (j == K - 1) {
                s = v0[u] - vm[u];
            } else {
                s = np_maximum(v0[u] - vm[u], vp[u] - v0[u]);
            }
            s = np_minimum(np_maximum(s, minsigma), maxsigma);   // np.clip
            if (j == pos) s = psig;
            double wt;
            if (j == pos) {
                wt = pw;
            } else {
                const int32_t r = rr[u];
                if (r < 0 || r >= n) {   // (a supplied order out of range)
                    atomicOr(err, 8);
                    wt = 0.0;
                } else {
                    wt = use_lf ? lf_weight(r, ramp) : 1.0;
                }
            }
            w[o + j] = wt;
            mu[o + j] = v0[u];
            sigma[o + j] = s;
        }
    }
    __syncthreads();
    // does the mixture depend on the order of tied observations?  Whenever
    // the weights differ (linear forgetting) and two observations share a
    // mu: the reference's np.argsort order then decides which weight sits in
    // which slot -- which weight meets a run end's sigma (the gap to the
    // neighbouring value) rather than the clipped minimum of its inner
    // slots, and the order of the normalising np.sum.
    if (use_lf && !supplied) {
        bool dep = false;
        for (int64_t j0 = 1 + tid; j0 < K; j0 += (int64_t)kFoldU * kParzenBlock) {
            double a[kFoldU], b[kFoldU];
#pragma unroll
            for (int u = 0; u < kFoldU; ++u) {
                const int64_t j = j0 + (int64_t)u * kParzenBlock;
                a[u] = j < K ? mu[o + j] : 0.0;
                b[u] = j < K ? mu[o + j - 1] : 1.0;
            }
#pragma unroll
            for (int u = 0; u < kFoldU; ++u) {
                const int64_t j = j0 + (int64_t)u * kParzenBlock;
                if (j < K && j != pos && j - 1 != pos && a[u] == b[u]) dep = true;
            }
        }
        if (__ballot(dep) && (tid & 63) == 0) atomicOr(ties + l, 1 << side);
    }
    const double tot = block_np_sum(w + o, K, leaf_sum + o);
    for (int64_t j0 = tid; j0 < K; j0 += (int64_t)kFoldU * kParzenBlock) {
        double v[kFoldU];
#pragma unroll
        for (int u = 0; u < kFoldU; ++u) {
            const int64_t j = j0 + (int64_t)u * kParzenBlock;
            if (j < K) v[u] = w[o + j];
        }
#pragma unroll
        for (int u = 0; u < kFoldU; ++u) {
            const int64_t j = j0 + (int64_t)u * kParzenBlock;
            if (j < K) w[o + j] = v[u] / tot;
        }
    }
    if (tid == 0) kcount[2 * l + side] = (int32_t)K;
}

__device__ __forceinline__ double dev_normal_cdf(double x, double m, double s) {
#pragma clang fp contract(off)
    const double bottom = fmax(sqrt(2.0) * s, kEps);   // tpe.py:102-107
    return 0.5 * (1.0 + erf((x - m) / bottom));
}

__device__ double block_max(double v) {
    __shared__ double wm[kParzenBlock / 64];
    __shared__ double res;
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = wm[0];
        for (int i = 1; i < kParzenBlock / 64; ++i) m = fmax(m, wm[i]);
        res = m;
    }
    __syncthreads();
    return res;
}

__device__ double block_min(double v) { return -block_max(-v); }

// k_fold's per-component transcendentals, spread over the chip (one
// workgroup per label would do them on one CU): the p_accept terms
// w (Phi(high) - Phi(low)) of bounded GMM1 / quantized mixtures, and the
// log-density constant -- w / sqrt(2 pi sigma^2) for GMM1 (k_fold divides by
// p_accept and takes the log, the reference's order), the whole
// log w - log(max(sigma, EPS) sqrt(2 pi)) for LGMM1 -- and the records'
// scale sqrt(1/2) / max(sigma, EPS).  Grid (slices, labels, sides).
constexpr int kTermBlock = 256;
__global__ __launch_bounds__(kTermBlock) void k_fold_terms(
    const DLabel* __restrict__ labels, const int32_t* __restrict__ kcount,
    const int64_t* __restrict__ mix_off, const double* __restrict__ w, const double* __restrict__ mu,
    const double* __restrict__ sigma, double* __restrict__ terms, double* __restrict__ cterm,
    double* __restrict__ ascale, const int32_t* __restrict__ only) {
#pragma clang fp contract(off)
    const int l = only ? only[blockIdx.y] : (int)blockIdx.y, side = blockIdx.z;
    const int mode = labels[l].mode;
    if (mode == CAT) return;
    const int64_t K = kcount[2 * l + side];
    const int64_t k = (int64_t)blockIdx.x * kTermBlock + threadIdx.x;
    if (k >= K) return;
    const int64_t o = mix_off[2 * l + side];
    const bool quant = mode == QUANT_GMM || mode == QUANT_LGMM;
    const bool is_lgmm = mode == DENSE_LGMM || mode == QUANT_LGMM;
    const double wk = w[o + k], mk = mu[o + k], sg = sigma[o + k];
    if ((labels[l].flags & 3) != 0 && (quant || !is_lgmm))   // tpe.py:139-142 / 279-282
        terms[o + k] = wk * (dev_normal_cdf(labels[l].high, mk, sg) -
                             dev_normal_cdf(labels[l].low, mk, sg));
    if (quant) return;
    ascale[o + k] = sqrt(0.5) / fmax(sg, kEps);   // the records' 1 / (sqrt 2 max(sigma, EPS))
    if (!is_lgmm) {   // log(w / sqrt(2 pi sigma^2) / p_accept), tpe.py:148-150
        const double Z = sqrt(2.0 * M_PI * (sg * sg));
        cterm[o + k] = wk / Z;
    } else {          // log w - log(max(sigma,EPS) sqrt(2 pi)), tpe.py:199-208
        const double s = fmax(sg, kEps);
        cterm[o + k] = log(wk) - log(s * sqrt(2.0 * M_PI));
    }
}

// The fold of tpe_set_posterior (tpe_engine.hip:fold_mixture) on the device:
// p_accept, the LSE shift M, the recentred exp-scaled fp64 records, fp32
// records, the below mixture's sampling records and the DLabel fields.
__global__ __launch_bounds__(kParzenBlock) void k_fold(
    DLabel* __restrict__ labels, const int32_t* __restrict__ kcount,
    const int64_t* __restrict__ mix_off, const double* __restrict__ w, const double* __restrict__ mu,
    const double* __restrict__ sigma, Comp<double>* __restrict__ c64, Comp<float>* __restrict__ c32,
    SampRec* __restrict__ samp, const double* __restrict__ terms, double* __restrict__ cterm,
    const double* __restrict__ ascale, double* __restrict__ leaf_sum, int32_t* __restrict__ err,
    const int32_t* __restrict__ only) {
#pragma clang fp contract(off)
    const int l = only ? only[blockIdx.x] : (int)blockIdx.x, tid = threadIdx.x;
    DLabel d = labels[l];
    const int64_t Kb = kcount[2 * l], Ka = kcount[2 * l + 1];
    const int64_t ob = mix_off[2 * l], oa = mix_off[2 * l + 1];
    const bool quant = d.mode == QUANT_GMM || d.mode == QUANT_LGMM;
    const bool is_lgmm = d.mode == DENSE_LGMM || d.mode == QUANT_LGMM;
    if (d.mode == CAT) {
        for (int side = 0; side < 2; ++side) {
            const int64_t o = side ? oa : ob, K = side ? Ka : Kb;
            for (int64_t k = tid; k < K; k += kParzenBlock) {
                const double p = w[o + k], lp = log(p);
                c64[o + k] = Comp<double>{0.0, 0.0, lp, p};
                c32[o + k] = Comp<float>{0.f, 0.f, (float)lp, (float)p};
            }
        }
    } else {
        double centre = 0.0;
        if (!quant) {  // recentre on the middle of both mixtures' means
            double lo = INFINITY, hi = -INFINITY;
            for (int64_t k = tid; k < Kb; k += kParzenBlock) {
                lo = fmin(lo, mu[ob + k]);
                hi = fmax(hi, mu[ob + k]);
            }
            for (int64_t k0 = tid; k0 < Ka; k0 += (int64_t)kFoldU * kParzenBlock) {
                double v[kFoldU];
#pragma unroll
                for (int u = 0; u < kFoldU; ++u) {
                    const int64_t k = k0 + (int64_t)u * kParzenBlock;
                    v[u] = k < Ka ? mu[oa + k] : mu[oa + k0];
                }
#pragma unroll
                for (int u = 0; u < kFoldU; ++u) {
                    lo = fmin(lo, v[u]);
                    hi = fmax(hi, v[u]);
                }
            }
            lo = block_min(lo);
            hi = block_max(hi);
            centre = (isfinite(lo) && isfinite(hi)) ? 0.5 * lo + 0.5 * hi : 0.0;
        }
        d.centre = centre;
        const bool bounded = (d.flags & 3) != 0;
        const double sK = sqrt(kExpScale), l2e = 1.4426950408889634;
#pragma unroll   // constant side: d's fields stay in registers
        for (int side = 0; side < 2; ++side) {
            const int64_t o = side ? oa : ob, K = side ? Ka : Kb;
            double p_accept = 1.0;   // (unused by dense LGMM1, tpe.py:265-307)
            if (bounded && (quant || !is_lgmm))   // terms from k_fold_terms
                p_accept = block_np_sum(terms + o, K, leaf_sum + o);
            if (quant) {
                (side ? d.logpacc_a : d.logpacc_b) = log(p_accept);
                for (int64_t k0 = tid; k0 < K; k0 += (int64_t)kFoldU * kParzenBlock) {
                    double sg[kFoldU], mk[kFoldU], wk[kFoldU];
#pragma unroll
                    for (int u = 0; u < kFoldU; ++u) {
                        const int64_t k = k0 + (int64_t)u * kParzenBlock;
                        if (k < K) {
                            sg[u] = sigma[o + k];
                            mk[u] = mu[o + k];
                            wk[u] = w[o + k];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < kFoldU; ++u) {
                        const int64_t k = k0 + (int64_t)u * kParzenBlock;
                        if (k >= K) continue;
                        const double a = 1.0 / fmax(sqrt(2.0) * sg[u], kEps);
                        c64[o + k] = Comp<double>{mk[u], a, 0.0, wk[u]};
                        c32[o + k] = Comp<float>{(float)mk[u], (float)a, 0.f, (float)wk[u]};
                    }
                }
                continue;
            }
            double M = -INFINITY;
            for (int64_t k0 = tid; k0 < K; k0 += (int64_t)kFoldU * kParzenBlock) {
                double ct[kFoldU];
#pragma unroll
                for (int u = 0; u < kFoldU; ++u) {
                    const int64_t k = k0 + (int64_t)u * kParzenBlock;
                    if (k < K) ct[u] = cterm[o + k];
                }
#pragma unroll
                for (int u = 0; u < kFoldU; ++u) {
                    const int64_t k = k0 + (int64_t)u * kParzenBlock;
                    if (k >= K) continue;
                    // GMM1: (w / Z) from k_fold_terms, then / p_accept and log
                    // (tpe.py:148-150); LGMM1: the whole constant (tpe.py:199-208)
                    const double c = !is_lgmm ? log(ct[u] / p_accept) : ct[u];
                    if (!is_lgmm) cterm[o + k] = c;
                    M = fmax(M, c);
                }
            }
            M = block_max(M);
            if (!isfinite(M)) M = 0.0;
            (side ? d.shift_a : d.shift_b) = M;
            double amax = 0.0;
            for (int64_t k0 = tid; k0 < K; k0 += (int64_t)kFoldU * kParzenBlock) {
                double av[kFoldU], cv[kFoldU], mv[kFoldU], wv[kFoldU];
#pragma unroll
                for (int u = 0; u < kFoldU; ++u) {
                    const int64_t k = k0 + (int64_t)u * kParzenBlock;
                    if (k < K) {
                        av[u] = ascale[o + k];
                        cv[u] = cterm[o + k];
                        mv[u] = mu[o + k];
                        wv[u] = w[o + k];
                    }
                }
#pragma unroll
                for (int u = 0; u < kFoldU; ++u) {
                    const int64_t k = k0 + (int64_t)u * kParzenBlock;
                    if (k >= K) continue;
                    const double a = av[u], c = cv[u];
                    c64[o + k] = Comp<double>{(mv[u] - centre) * (a * sK), a * sK, (c - M) * kExpScale, wv[u]};
                    const double a2 = a * sqrt(l2e);
                    const float a32 = (float)a2;
                    c32[o + k] = Comp<float>{(float)((mv[u] - centre) * a2), a32, (float)((c - M) * l2e),
                                             (float)wv[u]};
                    amax = fmax(amax, (double)a32);
                }
            }
            amax = block_max(amax);
            (side ? d.amax_a : d.amax_b) = (float)amax;
        }
    }
    // sampling records of the below mixture: the component, its raw weight,
    // then the shared fold (cumulative w m, truncation terms: samp_fold_block)
    if (tid == 0) {
        d.nb = (int32_t)Kb;
        d.na = (int32_t)Ka;
        d.ns = (int32_t)Kb;
        labels[l] = d;
    }
    for (int64_t k = tid; k < Kb; k += kParzenBlock) {
        SampRec r{};
        r.mu = d.mode == CAT ? 0.0 : mu[ob + k];
        r.sigma = d.mode == CAT ? 0.0 : sigma[ob + k];
        r.wd = w[ob + k];
        samp[d.samp_off + k] = r;
    }
    __syncthreads();
    if (!samp_fold_block(d, samp + d.samp_off, (int)Kb)) atomicOr(err, 4);
}

struct CopyArgs {
    uint32_t* dst[kCopyBatch];
    const uint32_t* src[kCopyBatch];
    int64_t words[kCopyBatch];
    int32_t n;
};
__global__ __launch_bounds__(kBlock) void k_copy_batch(CopyArgs a) {
    const int t = blockIdx.y;
    if (t >= a.n) return;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.words[t]; i += (int64_t)gridDim.x * kBlock)
        a.dst[t][i] = a.src[t][i];
}

// One scatter launch for a build's inputs: task y copies its bytes from the
// staging block (src >= 0: byte offset) or zero-fills them (src < 0).  Grid
// (<= 32, tasks).
constexpr int kUpBlock = 256;
__global__ __launch_bounds__(kUpBlock) void k_build_inputs(const UpTask* __restrict__ tasks,
                                                           const uint8_t* __restrict__ stage) {
    const UpTask t = tasks[blockIdx.y];
    const int64_t words = t.bytes >> 2;
    uint32_t* d = reinterpret_cast<uint32_t*>(t.dst);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(stage + (t.src >= 0 ? t.src : 0));
    for (int64_t i = (int64_t)blockIdx.x * kUpBlock + threadIdx.x; i < words; i += (int64_t)gridDim.x * kUpBlock)
        d[i] = t.src >= 0 ? sw[i] : 0u;
    if (blockIdx.x == 0 && threadIdx.x < (t.bytes & 3)) {
        const int64_t b = (words << 2) + threadIdx.x;
        t.dst[b] = t.src >= 0 ? stage[t.src + b] : (uint8_t)0;
    }
}

// A build's report in one block: the DLabels (dl_words 32-bit words), the
// error flag (16 bytes later) and the tie report (n_ties int32)
__global__ __launch_bounds__(kUpBlock) void k_build_report(const uint32_t* __restrict__ dl, int32_t dl_words,
                                                           const int32_t* __restrict__ err,
                                                           const int32_t* __restrict__ ties, int32_t n_ties,
                                                           uint32_t* __restrict__ out) {
    for (int32_t i = threadIdx.x; i < dl_words; i += kUpBlock) out[i] = dl[i];
    if (threadIdx.x == 0) out[dl_words] = (uint32_t)err[0];
    for (int32_t i = threadIdx.x; i < n_ties; i += kUpBlock) out[dl_words + 4 + i] = (uint32_t)ties[i];
}

}  // namespace

int tpe_rt::copy_batch(tpe_ctx* ctx, hipStream_t st, const CopySpec* specs, int n) {
    for (int i0 = 0; i0 < n; i0 += kCopyBatch) {
        CopyArgs a{};
        int64_t mx = 1;
        for (int t = 0; t < kCopyBatch && i0 + t < n; ++t) {
            const CopySpec& c = specs[i0 + t];
            if (c.bytes <= 0) continue;
            if ((c.bytes & 3) || ((uintptr_t)c.dst & 3) || ((uintptr_t)c.src & 3))
                return ctx->fail(TPE_ERR_ARG, "copy_batch: unaligned copy");
            a.dst[a.n] = (uint32_t*)c.dst;
            a.src[a.n] = (const uint32_t*)c.src;
            a.words[a.n] = c.bytes / 4;
            mx = std::max(mx, a.words[a.n]);
            ++a.n;
        }
        if (a.n == 0) continue;
        hipLaunchKernelGGL(k_copy_batch, dim3((unsigned)std::min<int64_t>((mx + kBlock - 1) / kBlock, 1024), a.n),
                           dim3(kBlock), 0, st, a);
        HIPCHK(ctx, hipGetLastError());
    }
    return TPE_OK;
}

// ============================================================ host side ====
namespace {

// k_split with the register form for histories of up to 16 kSplitBlock trials (32 spill)
int launch_split(tpe_ctx* ctx, hipStream_t st, const double* losses, int64_t T, int32_t n_below, uint8_t* below,
                 int32_t* split_tie) {
    const int64_t per = (T + kSplitBlock - 1) / kSplitBlock;
    const dim3 g(1), b(kSplitBlock);
    constexpr int64_t kSliceT = 16 * (int64_t)kSplitBlock;
    const int32_t m_sel = n_below + 1;
    const int64_t slices = (T + kSliceT - 1) / kSliceT;
    if (per <= 4) {
        hipLaunchKernelGGL(k_split<4>, g, b, 0, st, losses, T, n_below, below, split_tie, 0, nullptr, nullptr);
    } else if (per <= 8) {
        hipLaunchKernelGGL(k_split<8>, g, b, 0, st, losses, T, n_below, below, split_tie, 0, nullptr, nullptr);
    } else if (per <= 16) {
        hipLaunchKernelGGL(k_split<16>, g, b, 0, st, losses, T, n_below, below, split_tie, 0, nullptr, nullptr);
    } else if (n_below > 0 && slices * m_sel <= kSplitMergeMax) {
        // slices of 16 Ki losses, each in registers, merged by one workgroup
        auto& B = ctx->build;
        HIPCHK(ctx, B.split_key.reserve((size_t)slices * m_sel));
        HIPCHK(ctx, B.split_pos.reserve((size_t)slices * m_sel));
        hipLaunchKernelGGL(k_split<16>, dim3((unsigned)slices), b, 0, st, losses, T, n_below, below, split_tie,
                           m_sel, B.split_key.p, B.split_pos.p);
        hipLaunchKernelGGL(k_split_merge, g, b, 0, st, B.split_key.p, B.split_pos.p, (int32_t)(slices * m_sel),
                           n_below, below, split_tie);
    } else {
        hipLaunchKernelGGL(k_split<0>, g, b, 0, st, losses, T, n_below, below, split_tie, 0, nullptr, nullptr);
    }
    return TPE_OK;
}

int check_specs(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels, int64_t n_cat_p,
                const double* cat_p) {
    for (int32_t l = 0; l < n_labels; ++l) {
        const tpe_label_spec& s = specs[l];
        if (s.kind == TPE_CATEGORICAL) {
            if (s.upper <= 0) return ctx->fail(TPE_ERR_ARG, "categorical upper must be positive");
            if (!s.randint && (s.p_off < 0 || s.p_off + s.upper > n_cat_p || !cat_p))
                return ctx->fail(TPE_ERR_ARG, "categorical p out of range");
        } else if (s.kind == TPE_GMM1 || s.kind == TPE_LGMM1) {
            if ((s.flags & 3) == 1 || (s.flags & 3) == 2)
                return ctx->fail(TPE_ERR_TYPE, "low and high must both be given or both be None");
            if ((s.flags & 3) == 3 && !(s.low < s.high)) return ctx->fail(TPE_ERR_VALUE, "low >= high");
            if ((s.flags & TPE_HAS_Q) && !(s.q > 0) && !(s.q < 0))
                return ctx->fail(TPE_ERR_VALUE, "q must be non-zero");
            if (!(s.prior_sigma > 0)) return ctx->fail(TPE_ERR_VALUE, "prior sigma must be positive");
        } else {
            return ctx->fail(TPE_ERR_ARG, "label " + std::to_string(l) + ": unknown kind");
        }
        if ((s.flags & TPE_HAS_STREAM) && s.stream < 0)
            return ctx->fail(TPE_ERR_ARG, "label " + std::to_string(l) + ": negative stream");
    }
    return TPE_OK;
}

int history_reset(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels, const double* cat_p,
                  int64_t n_cat_p) {
    if (n_labels <= 0 || !specs) return ctx->fail(TPE_ERR_ARG, "tpe_history_reset: no labels");
    int rc = check_specs(ctx, specs, n_labels, n_cat_p, cat_p);
    if (rc) return rc;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    auto& B = ctx->build;
    B.specs_h.assign(specs, specs + n_labels);
    B.cap_h.assign(n_labels, 0);
    B.off_h.assign(n_labels, 0);
    B.cnt_h.assign(n_labels, 0);
    B.pool_cap = 0;
    HIPCHK(ctx, B.specs.reserve(n_labels));
    HIPCHK(ctx, B.cat_p.reserve(std::max<int64_t>(n_cat_p, 1)));
    HIPCHK(ctx, B.p_off.reserve(n_labels));
    HIPCHK(ctx, B.cnt.reserve(n_labels));
    HIPCHK(ctx, hipMemcpyAsync(B.specs.p, specs, n_labels * sizeof(tpe_label_spec),
                               hipMemcpyHostToDevice, ctx->stream));
    if (n_cat_p > 0 && cat_p)
        HIPCHK(ctx, hipMemcpyAsync(B.cat_p.p, cat_p, n_cat_p * sizeof(double), hipMemcpyHostToDevice,
                                   ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(B.cnt.p, 0, n_labels * sizeof(int32_t), ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(B.p_off.p, 0, n_labels * sizeof(int64_t), ctx->stream));
    B.hist_ready = true;
    ++B.hist_gen;
    return TPE_OK;
}

int history_append(tpe_ctx* ctx, const int64_t* n_new, const int32_t* obs_trial, const double* obs_val) {
    auto& B = ctx->build;
    ++B.hist_gen;   // (a failed append leaves the history unknown: no subset rebuild after it either)
    if (!B.hist_ready) return ctx->fail(TPE_ERR_ARG, "tpe_history_append before tpe_history_reset");
    const int32_t L = (int32_t)B.specs_h.size();
    std::vector<int64_t> st(L + 1, 0);
    for (int32_t l = 0; l < L; ++l) {
        if (n_new[l] < 0) return ctx->fail(TPE_ERR_ARG, "negative observation count");
        st[l + 1] = st[l] + n_new[l];
    }
    const int64_t total = st[L];
    if (total == 0) return TPE_OK;
    if (!obs_trial || !obs_val) return ctx->fail(TPE_ERR_ARG, "observations missing");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t sm = ctx->stream;
    // the previous append's copies out of the pinned staging buffers
    if (B.staged_pending) HIPCHK(ctx, hipEventSynchronize(B.ev_staged));
    B.staged_pending = false;
    if (!B.ev_staged) HIPCHK(ctx, hipEventCreateWithFlags(&B.ev_staged, hipEventDisableTiming));
    // growth: re-lay the pool out when a label outgrows its region
    bool grow = false;
    for (int32_t l = 0; l < L; ++l)
        if (B.cnt_h[l] + n_new[l] > B.cap_h[l]) grow = true;
    if (grow) {
        std::vector<int64_t> cap(L), off(L);
        int64_t pc = 0;
        for (int32_t l = 0; l < L; ++l) {
            const int64_t need = B.cnt_h[l] + n_new[l];
            cap[l] = need > B.cap_h[l] ? std::max<int64_t>(2 * need, 256) : B.cap_h[l];
            off[l] = pc;
            pc += cap[l];
        }
        if (pc >= INT32_MAX) return ctx->fail(TPE_ERR_ARG, "history too large");
        DevBuf<int32_t> t2, i2;
        DevBuf<double> v2, k2;
        DevBuf<int64_t> o2;
        HIPCHK(ctx, t2.reserve(pc));
        HIPCHK(ctx, i2.reserve(pc));
        HIPCHK(ctx, v2.reserve(pc));
        HIPCHK(ctx, k2.reserve(pc));
        HIPCHK(ctx, o2.reserve(L));
        HIPCHK(ctx, hipMemcpyAsync(o2.p, off.data(), L * sizeof(int64_t), hipMemcpyHostToDevice, sm));
        int32_t mx = 0;
        for (int32_t l = 0; l < L; ++l) mx = std::max(mx, B.cnt_h[l]);
        if (mx > 0 && B.pool_cap > 0)
            hipLaunchKernelGGL(k_hist_regrow, dim3((unsigned)std::min<int64_t>((mx + kBlock - 1) / kBlock, 1024), L),
                               dim3(kBlock), 0, sm, B.p_off.p, o2.p, B.cnt.p, B.p_trial.p, B.p_val.p,
                               B.s_key.p, B.s_idx.p, t2.p, v2.p, k2.p, i2.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipStreamSynchronize(sm));
        std::swap(B.p_trial, t2);
        std::swap(B.p_val, v2);
        std::swap(B.s_key, k2);
        std::swap(B.s_idx, i2);
        std::swap(B.p_off, o2);
        t2.release();
        v2.release();
        k2.release();
        i2.release();
        o2.release();
        HIPCHK(ctx, B.s_key2.reserve(pc));
        HIPCHK(ctx, B.s_idx2.reserve(pc));
        HIPCHK(ctx, B.arank.reserve(pc));
        HIPCHK(ctx, B.keys.reserve(pc));
        HIPCHK(ctx, B.idx.reserve(pc));
        B.cap_h = cap;
        B.off_h = off;
        B.pool_cap = pc;
    }
    HIPCHK(ctx, B.st_off.reserve(L + 1));
    HIPCHK(ctx, B.st_trial.reserve(total));
    HIPCHK(ctx, B.st_val.reserve(total));
    HIPCHK(ctx, B.st_idx.reserve(total));
    HIPCHK(ctx, B.st_idx_sorted.reserve(total));
    HIPCHK(ctx, B.st_key_sorted.reserve(total));
    HIPCHK(ctx, B.seg_begin.reserve(L));
    HIPCHK(ctx, B.seg_end.reserve(L));
    // the caller's arrays and this call's offsets into page-locked staging:
    // the copies below run on the stream while the host returns
    // one staging block (offsets, values, trials, segments, the new counts),
    // one H2D copy and one scatter launch (six copies before)
    auto al = [](int64_t v) { return (v + 15) / 16 * 16; };
    const int64_t o_off = 0, o_val = al((L + 1) * 8), o_trial = o_val + al(total * 8),
                  o_seg = o_trial + al(total * 4), o_cnt = o_seg + al(2 * (int64_t)L * 4),
                  o_end = o_cnt + al((int64_t)L * 4);
    HIPCHK(ctx, B.h_stage.resize(o_end));
    HIPCHK(ctx, B.d_stage.reserve(o_end));
    uint8_t* hs = B.h_stage.data();
    std::memcpy(hs + o_off, st.data(), (L + 1) * sizeof(int64_t));
    int32_t* seg = (int32_t*)(hs + o_seg);
    for (int32_t l = 0; l < L; ++l) {
        seg[l] = (int32_t)st[l];
        seg[L + l] = (int32_t)(B.specs_h[l].kind == TPE_CATEGORICAL ? st[l] : st[l + 1]);
    }
    std::memcpy(hs + o_trial, obs_trial, total * sizeof(int32_t));
    std::memcpy(hs + o_val, obs_val, total * sizeof(double));
    int32_t* cnt_new = (int32_t*)(hs + o_cnt);
    for (int32_t l = 0; l < L; ++l) cnt_new[l] = B.cnt_h[l] + (int32_t)n_new[l];
    HIPCHK(ctx, hipMemcpyAsync(B.d_stage.p, hs, o_end, hipMemcpyHostToDevice, sm));
    {
        const uint8_t* ds = B.d_stage.p;
        const CopySpec cs[5] = {{B.st_off.p, ds + o_off, (L + 1) * 8},
                                {B.st_trial.p, ds + o_trial, total * 4},
                                {B.st_val.p, ds + o_val, total * 8},
                                {B.seg_begin.p, ds + o_seg, (int64_t)L * 4},
                                {B.seg_end.p, ds + o_seg + (int64_t)L * 4, (int64_t)L * 4}};
        const int rc = tpe_rt::copy_batch(ctx, sm, cs, 5);
        if (rc) return rc;
    }
    int64_t mx_new = 0, mx_all = 0;
    for (int32_t l = 0; l < L; ++l) {
        mx_new = std::max(mx_new, n_new[l]);
        mx_all = std::max<int64_t>(mx_all, B.cnt_h[l] + n_new[l]);
    }
    hipLaunchKernelGGL(k_hist_append, dim3((unsigned)std::min<int64_t>((mx_new + kBlock - 1) / kBlock, 1024), L),
                       dim3(kBlock), 0, sm, B.st_off.p, B.st_trial.p, B.st_val.p, B.p_off.p, B.cnt.p,
                       B.p_trial.p, B.p_val.p, B.st_idx.p);
    HIPCHK(ctx, hipGetLastError());
    if (total >= kGlobalSortMin) {
        // two stable chip-wide sorts: by value, then by label
        HIPCHK(ctx, B.gs_a.reserve(total));
        HIPCHK(ctx, B.gs_b.reserve(total));
        HIPCHK(ctx, B.gs_lab.reserve(total));
        HIPCHK(ctx, B.gs_lab2.reserve(total));
        int lab_bits = 1;
        while ((1LL << lab_bits) < (int64_t)L) ++lab_bits;
        const unsigned gb = (unsigned)std::min<int64_t>((total + kBlock - 1) / kBlock, 2048);
        hipLaunchKernelGGL(k_iota, dim3(gb), dim3(kBlock), 0, sm, B.gs_a.p, total);
        HIPCHK(ctx, hipGetLastError());
        size_t b1 = 0, b2 = 0;
        HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, b1, B.st_val.p, B.st_key_sorted.p, B.gs_a.p,
                                                         B.gs_b.p, (int)total, 0, 64, sm));
        HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, b2, B.gs_lab.p, B.gs_lab2.p, B.gs_b.p,
                                                         B.gs_a.p, (int)total, 0, lab_bits, sm));
        HIPCHK(ctx, B.sort_tmp.reserve(std::max<size_t>(std::max(b1, b2), 1)));
        HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(B.sort_tmp.p, b1, B.st_val.p, B.st_key_sorted.p,
                                                         B.gs_a.p, B.gs_b.p, (int)total, 0, 64, sm));
        hipLaunchKernelGGL(k_label_of, dim3(gb), dim3(kBlock), 0, sm, B.st_off.p, L, B.gs_b.p, B.gs_lab.p, total);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipcub::DeviceRadixSort::SortPairs(B.sort_tmp.p, b2, B.gs_lab.p, B.gs_lab2.p, B.gs_b.p,
                                                         B.gs_a.p, (int)total, 0, lab_bits, sm));
        hipLaunchKernelGGL(k_sorted_gather, dim3(gb), dim3(kBlock), 0, sm, B.gs_a.p, B.st_val.p, B.st_idx.p,
                           B.st_key_sorted.p, B.st_idx_sorted.p, total);
        HIPCHK(ctx, hipGetLastError());
    } else {
        size_t bytes = 0;   // stable segmented radix sort of the new batch
        HIPCHK(ctx, hipcub::DeviceSegmentedRadixSort::SortPairs(
                        nullptr, bytes, B.st_val.p, B.st_key_sorted.p, B.st_idx.p, B.st_idx_sorted.p,
                        (int)total, L, B.seg_begin.p, B.seg_end.p, 0, 64, sm));
        HIPCHK(ctx, B.sort_tmp.reserve(std::max<size_t>(bytes, 1)));
        HIPCHK(ctx, hipcub::DeviceSegmentedRadixSort::SortPairs(
                        B.sort_tmp.p, bytes, B.st_val.p, B.st_key_sorted.p, B.st_idx.p, B.st_idx_sorted.p,
                        (int)total, L, B.seg_begin.p, B.seg_end.p, 0, 64, sm));
    }
    hipLaunchKernelGGL(k_hist_merge, dim3((unsigned)std::min<int64_t>((mx_all + kBlock - 1) / kBlock, 1024), L),
                       dim3(kBlock), 0, sm, B.specs.p, B.p_off.p, B.cnt.p, B.st_off.p, B.s_key.p,
                       B.s_idx.p, B.st_key_sorted.p, B.st_idx_sorted.p, B.s_key2.p, B.s_idx2.p);
    HIPCHK(ctx, hipGetLastError());
    std::swap(B.s_key, B.s_key2);
    std::swap(B.s_idx, B.s_idx2);
    for (int32_t l = 0; l < L; ++l) B.cnt_h[l] += (int32_t)n_new[l];
    {   // the new counts, from the staging block
        const CopySpec cs{B.cnt.p, B.d_stage.p + o_cnt, (int64_t)L * 4};
        const int rc = tpe_rt::copy_batch(ctx, sm, &cs, 1);
        if (rc) return rc;
    }
    // no wait here: the next append waits for these copies before it
    // rewrites the staging buffers (round 4 synchronised every append)
    HIPCHK(ctx, hipEventRecord(B.ev_staged, sm));
    B.staged_pending = true;
    return TPE_OK;
}

// below_h (optional): the below set per trial position, as the caller's
// np.argsort of the losses picks it (tpe.py:637); order_off / order
// (optional): per label, the order of its above observations (np.argsort,
// tpe.py:433; empty range = the device's position order); ties_out
// (optional, n_labels + 1): which mixtures depend on a tie order the caller
// did not supply (k_parzen, k_split).
// only_h / n_only (optional): rebuild just these labels of the resident
// posterior (with the supplied orders), keeping the others -- valid only
// right after a build of the same history with the same arguments, whose
// below set it reuses (so no below_h); the caller's labels are those whose
// mixtures depend on an order the previous build did not have.
constexpr int32_t kGammaCap = 25;   // ap_filter_trials(gamma_cap=DEFAULT_LF), tpe.py:35, 626

// 64-bit fingerprint of the losses' bit patterns (NaN payloads included):
// a label-subset rebuild reuses the device copy of the previous build's
// losses and below set, so it must be handed the same losses
uint64_t loss_fingerprint(const double* losses, int64_t n) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)n;
    for (int64_t t = 0; t < n; ++t) {
        uint64_t v;
        std::memcpy(&v, losses + t, sizeof(v));
        h = (h ^ v) * 0xff51afd7ed558ccdull;
        h ^= h >> 29;
    }
    return h;
}

// The end of a build, once its report is in (build_resident, or a deferred
// subset rebuild settled by the next call on the context): the error flags,
// the DLabels, the label groups, the posterior's flags and what the build
// was of.
int finish_build(tpe_ctx* ctx, BuildTail& t, int32_t* ties_out, int32_t* n_below_out) {
    auto& B = ctx->build;
    Posterior& P = ctx->resident;
    const int32_t n_labels = t.n_labels;
    const int64_t rep_dl = t.rep_dl;
    std::vector<DLabel>& dl = t.dl;
    const std::vector<int32_t>* grp = t.grp;
    const bool beside = t.beside, subset = t.subset;
    HIPCHK(ctx, hipStreamSynchronize(t.st));
    P.qc_ready = false;   // (set again below when the build succeeds)
    int32_t errh;
    std::memcpy(&errh, B.h_rep.data() + rep_dl, sizeof(int32_t));
    std::memcpy(dl.data(), B.h_rep.data(), rep_dl);
    B.last_ties.resize(n_labels + 1);
    std::memcpy(B.last_ties.data(), B.h_rep.data() + rep_dl + 16, (n_labels + 1) * sizeof(int32_t));
    B.last_n_below = t.n_below;
    if (ties_out) std::memcpy(ties_out, B.last_ties.data(), (n_labels + 1) * sizeof(int32_t));
    // (a deferred report: the round that settles it re-recorded ev0 / ev1)
    if (t.deferred) ctx->build_ms = -1.f;
    else HIPCHK(ctx, hipEventElapsedTime(&ctx->build_ms, ctx->ev0, ctx->ev1));
    if (errh & 1) return ctx->fail(TPE_ERR_ARG, "observation trial position out of range");
    if (errh & 2) return ctx->fail(TPE_ERR_ARG, "more below observations than the below set (duplicate trial in a label?)");
    if (errh & 4) return ctx->fail(TPE_ERR_VALUE, "below weights sum to zero");
    if (errh & 8) return ctx->fail(TPE_ERR_ARG, "supplied observation order does not fit the above set");

    std::vector<int32_t> cat;
    for (int m = 0; m < kNumModes; ++m) {
        P.group_off[m] = (int32_t)cat.size();
        cat.insert(cat.end(), grp[m].begin(), grp[m].end());
        P.h_group[m] = grp[m];
    }
    const bool groups_changed = cat != P.groups_h || !P.groups.p;
    if (groups_changed) {   // unchanged between rebuilds of one history
        HIPCHK(ctx, P.groups.reserve(std::max<size_t>(cat.size(), 1)));
        HIPCHK(ctx, hipMemcpy(P.groups.p, cat.data(), cat.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        P.groups_h = cat;
    }
    P.h_labels = dl;
    P.win_ready = false;
    P.zw_ready = false;
    P.qc_ready = t.qc_queued;
    // the index is kept when every dense label came out bit-identical (e.g.
    // a second build of the same history that only supplies the tie order
    // of quantized labels)
    if (!beside) P.bx_ready = tpe_rt::bx_keep_after(ctx, groups_changed);
    P.n_labels = n_labels;
    B.n_labels = n_labels;
    B.mix_h = t.mix;
    B.built_ok = true;
    B.built_gen = B.hist_gen;
    B.built_T = t.n_trials;
    B.built_valid = t.n_valid;
    B.built_gamma = t.gamma;
    B.built_pw = t.pw;
    B.built_lf = t.lf;
    if (!subset) B.built_loss_hash = t.loss_hash;
    if (n_below_out) *n_below_out = t.n_below;
    // the armed index, queued now: no caller round trip before it starts
    P.bx_prescan_ok = t.prescan && !P.bx_ready;
    if (t.arm_c > 0) return tpe1_prepare(ctx, t.arm_c, t.arm_r);
    return TPE_OK;
}

int build_resident(tpe_ctx* ctx, const double* losses, int64_t n_trials, int64_t n_valid,
                   double gamma, double prior_weight, int32_t lf, int32_t* n_below_out,
                   const uint8_t* below_h = nullptr, const int64_t* order_off_h = nullptr,
                   const int32_t* order_h = nullptr, int32_t* ties_out = nullptr,
                   const int32_t* only_h = nullptr, int32_t n_only = 0) {
    auto& B = ctx->build;
    const bool defer_report = B.defer;   // (consumed by this build, whatever happens)
    B.defer = false;
    if (!B.hist_ready) return ctx->fail(TPE_ERR_ARG, "no resident history (tpe_history_reset)");
    const bool subset = only_h != nullptr && n_only > 0;
    // an armed tpe_prepare (tpe_arm_prepare): consumed by a full build
    const int64_t arm_c = subset ? 0 : ctx->arm_c;
    const int32_t arm_r = subset ? 0 : ctx->arm_r;
    if (!subset) ctx->arm_c = ctx->arm_r = 0;
    if (subset) {
        if (below_h)
            return ctx->fail(TPE_ERR_ARG, "a label-subset rebuild keeps the previous build's below set");
        if (!B.built_ok || B.built_gen != B.hist_gen || B.built_T != n_trials || B.built_valid != n_valid ||
            B.built_gamma != gamma || B.built_pw != prior_weight || B.built_lf != lf ||
            B.n_labels != (int32_t)B.specs_h.size())
            return ctx->fail(TPE_ERR_ARG, "a label-subset rebuild must follow a build of the same history");
        if (n_trials > 0 && !losses) return ctx->fail(TPE_ERR_ARG, "tpe_build_posterior: bad trial arguments");
        if (loss_fingerprint(losses, n_trials) != B.built_loss_hash)
            return ctx->fail(TPE_ERR_ARG, "a label-subset rebuild must be given the previous build's losses");
        for (int32_t i = 0; i < n_only; ++i)
            if (only_h[i] < 0 || only_h[i] >= B.n_labels || (i && only_h[i] <= only_h[i - 1]))
                return ctx->fail(TPE_ERR_ARG, "subset labels must be increasing label indices");
    }
    B.built_ok = false;   // (set again once this build completes)
    ctx->resident.bx_prescan_ok = false;
    if (lf < 1 || lf >= kMaxLF) return ctx->fail(TPE_ERR_ARG, "linear forgetting must be in [1, 63]");
    if (n_trials < 0 || n_trials >= INT32_MAX || (n_trials > 0 && !losses) || n_valid < 0 ||
        n_valid > n_trials)
        return ctx->fail(TPE_ERR_ARG, "tpe_build_posterior: bad trial arguments");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int32_t n_labels = (int32_t)B.specs_h.size();
    Posterior& P = ctx->resident;
    ctx->P = &ctx->resident;
    // a subset rebuild of labels that are all non-dense (the quantized labels
    // given numpy's tie order) touches no dense label's DLabel, records or
    // sampling records -- what the expansion index reads: it runs on the aux
    // stream beside an index queued on the main one (tpe_prepare), and the
    // index is kept without the snapshot comparison.  (On the main stream it
    // waited for the whole index: ~0.35 ms of the config-3 fmin step.)
    bool beside = subset;
    for (int32_t i = 0; beside && i < n_only; ++i) {
        const tpe_label_spec& s = B.specs_h[only_h[i]];
        beside = s.kind == TPE_CATEGORICAL || (s.flags & TPE_HAS_Q) != 0;
    }
    hipStream_t st = beside ? ctx->aux : ctx->stream;

    // n_below = min(ceil(gamma sqrt(len(l_vals))), gamma_cap)   tpe.py:636 --
    // gamma_cap is ap_filter_trials' default DEFAULT_LF (tpe.py:626), which
    // build_posterior never overrides: independent of the linear forgetting
    const double nbd = std::ceil(gamma * std::sqrt((double)n_valid));
    const int32_t n_below = (int32_t)std::min<double>(nbd, (double)kGammaCap);
    if (below_h) {   // a supplied below set: n_below trials, each with a loss
        int64_t nb = 0;
        for (int64_t t = 0; t < n_trials; ++t)
            if (below_h[t]) {
                if (!(losses[t] == losses[t])) return ctx->fail(TPE_ERR_ARG, "below set holds a trial without a loss");
                ++nb;
            }
        if (nb != n_below) return ctx->fail(TPE_ERR_ARG, "below set size differs from n_below");
    }

    // static label fields, mixture / record regions
    std::vector<DLabel> dl(n_labels);
    std::vector<int64_t> mix(2 * (size_t)n_labels);
    std::vector<int32_t> grp[kNumModes];
    int64_t total = 0, samp_total = 0, max_cap = 1;
    for (int32_t l = 0; l < n_labels; ++l) {
        const tpe_label_spec& s = B.specs_h[l];
        DLabel& o = dl[l];
        std::memset(&o, 0, sizeof(o));
        const bool quant = (s.flags & TPE_HAS_Q) != 0;
        int64_t cap_b, cap_a;
        if (s.kind == TPE_CATEGORICAL) {
            o.mode = CAT;
            cap_b = cap_a = s.upper;
        } else {
            o.mode = s.kind == TPE_GMM1 ? (quant ? QUANT_GMM : DENSE_GMM) : (quant ? QUANT_LGMM : DENSE_LGMM);
            cap_b = lf + 1;
            cap_a = (int64_t)B.cnt_h[l] + 1;
        }
        o.flags = s.kind == TPE_CATEGORICAL ? 0 : (s.flags & (TPE_HAS_LOW | TPE_HAS_HIGH | TPE_HAS_Q));
        o.low = s.low;
        o.high = s.high;
        o.q = s.q;
        o.exp_low = std::exp(s.low);
        o.exp_high = std::exp(s.high);
        o.stream = (s.flags & TPE_HAS_STREAM) ? s.stream : l;
        o.comp_b = mix[2 * l] = total;
        total += cap_b;
        o.comp_a = mix[2 * l + 1] = total;
        total += cap_a;
        max_cap = std::max(max_cap, std::max(cap_b, cap_a));
        o.samp_off = samp_total;
        samp_total += cap_b;
        grp[o.mode].push_back(l);
    }
    const int64_t T = n_trials;
    HIPCHK(ctx, B.losses.reserve(std::max<int64_t>(T, 1)));
    HIPCHK(ctx, B.below.reserve(std::max<int64_t>(T, 1)));
    HIPCHK(ctx, B.below_val.reserve((size_t)n_labels * kMaxLF));
    HIPCHK(ctx, B.counts.reserve(2 * (size_t)n_labels));
    HIPCHK(ctx, B.kcount.reserve(2 * (size_t)n_labels));
    HIPCHK(ctx, B.keys.reserve(std::max<int64_t>(B.pool_cap, 1)));
    HIPCHK(ctx, B.idx.reserve(std::max<int64_t>(B.pool_cap, 1)));
    HIPCHK(ctx, B.arank.reserve(std::max<int64_t>(B.pool_cap, 1)));
    HIPCHK(ctx, B.w.reserve(total));
    HIPCHK(ctx, B.mu.reserve(total));
    HIPCHK(ctx, B.sigma.reserve(total));
    HIPCHK(ctx, B.mix_off.reserve(2 * (size_t)n_labels));
    HIPCHK(ctx, B.scratch.reserve(4 * (size_t)total));   // terms | leaf sums | constants | scales
    HIPCHK(ctx, P.labels.reserve(n_labels));
    HIPCHK(ctx, P.comps64.reserve(total));
    HIPCHK(ctx, P.comps32.reserve(total));
    HIPCHK(ctx, P.samp.reserve(samp_total));
    HIPCHK(ctx, ctx->build_err.reserve(1));
    HIPCHK(ctx, B.ties.reserve(n_labels + 1));
    // the build's inputs -- supplied orders, subset labels, losses, below
    // set, mixture offsets, DLabels, and the zeroed tie report and error
    // flag -- in ONE H2D copy from pinned staging and one scatter launch
    // (k_build_inputs) instead of up to 8 copies and memsets (~8 us of host
    // API time each, on the fmin step's critical path)
    const int64_t* order_off_d = nullptr;
    const int32_t* order_d = nullptr;
    std::vector<UpTask> up;
    std::vector<const void*> up_src;
    auto put = [&](const void* src, int64_t bytes, void* dst) {
        if (bytes <= 0) return;
        up.push_back(UpTask{0, (uint8_t*)dst, bytes, 0});
        up_src.push_back(src);
    };
    put(nullptr, (n_labels + 1) * (int64_t)sizeof(int32_t), B.ties.p);
    if (order_off_h && order_h && order_off_h[n_labels] > 0) {
        for (int32_t l = 0; l < n_labels; ++l)
            if (order_off_h[l + 1] < order_off_h[l] || order_off_h[l] < 0)
                return ctx->fail(TPE_ERR_ARG, "order offsets must not decrease");
        HIPCHK(ctx, B.order_off.reserve(n_labels + 1));
        HIPCHK(ctx, B.order.reserve(order_off_h[n_labels]));
        put(order_off_h, (n_labels + 1) * (int64_t)sizeof(int64_t), B.order_off.p);
        put(order_h, order_off_h[n_labels] * (int64_t)sizeof(int32_t), B.order.p);
        order_off_d = B.order_off.p;
        order_d = B.order.p;
    }
    const int32_t* only_d = nullptr;
    const int32_t nl_run = subset ? n_only : n_labels;
    if (subset) {
        // the other labels keep the previous build's records, DLabels and
        // mixtures; the losses, the below set and the offsets are the same
        HIPCHK(ctx, B.only.reserve(n_only));
        put(only_h, n_only * (int64_t)sizeof(int32_t), B.only.p);
        only_d = B.only.p;
    } else {
        put(losses, T * (int64_t)sizeof(double), B.losses.p);
        if (below_h) put(below_h, T, B.below.p);
        put(mix.data(), (int64_t)mix.size() * (int64_t)sizeof(int64_t), B.mix_off.p);
        put(dl.data(), n_labels * (int64_t)sizeof(DLabel), P.labels.p);
    }
    put(nullptr, sizeof(int32_t), ctx->build_err.p);
    {
        const int64_t head = ((int64_t)up.size() * (int64_t)sizeof(UpTask) + 255) / 256 * 256;
        int64_t o = head;
        for (UpTask& u : up) {
            u.src = up_src[&u - up.data()] ? o : -1;
            if (u.src >= 0) o += (u.bytes + 15) / 16 * 16;
        }
        if (B.up_pending) {   // (the previous build's copy out of the staging)
            HIPCHK(ctx, hipEventSynchronize(B.ev_up));
            B.up_pending = false;
        }
        HIPCHK(ctx, B.h_up.resize(o));
        HIPCHK(ctx, B.d_up.reserve(o));
        std::memcpy(B.h_up.data(), up.data(), up.size() * sizeof(UpTask));
        for (size_t i = 0; i < up.size(); ++i)
            if (up[i].src >= 0) std::memcpy(B.h_up.data() + up[i].src, up_src[i], up[i].bytes);
        HIPCHK(ctx, hipMemcpyAsync(B.d_up.p, B.h_up.data(), o, hipMemcpyHostToDevice, st));
        if (!B.ev_up) HIPCHK(ctx, hipEventCreateWithFlags(&B.ev_up, hipEventDisableTiming));
        HIPCHK(ctx, hipEventRecord(B.ev_up, st));
        B.up_pending = true;
        int64_t mx = 1;
        for (const UpTask& u : up) mx = std::max(mx, u.bytes);
        hipLaunchKernelGGL(k_build_inputs, dim3((unsigned)std::min<int64_t>((mx + 4 * kUpBlock - 1) / (4 * kUpBlock), 32),
                                                (unsigned)up.size()),
                           dim3(kUpBlock), 0, st, (const UpTask*)B.d_up.p, B.d_up.p);
        HIPCHK(ctx, hipGetLastError());
    }

    HIPCHK(ctx, hipEventRecord(ctx->ev0, st));
    if (T > 0 && !below_h && !subset) {
        const int rc = launch_split(ctx, st, B.losses.p, T, n_below, B.below.p, B.ties.p + n_labels);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(k_partition, dim3(nl_run), dim3(kPartBlock), 0, st, B.specs.p, B.p_off.p, B.cnt.p,
                       B.p_trial.p, B.p_val.p, B.s_key.p, B.s_idx.p, B.below.p, B.losses.p, T,
                       B.below_val.p, B.arank.p, B.keys.p, B.idx.p, B.counts.p, ctx->build_err.p, only_d);
    hipLaunchKernelGGL(k_parzen, dim3(nl_run, 2), dim3(kParzenBlock), 0, st, B.specs.p, B.cat_p.p,
                       B.p_off.p, B.counts.p, B.below_val.p, B.keys.p, B.keys.p, B.idx.p, B.mix_off.p,
                       prior_weight, lf, B.w.p, B.mu.p, B.sigma.p, B.kcount.p, B.scratch.p + total, order_off_d,
                       order_d, B.ties.p, ctx->build_err.p, only_d);
    hipLaunchKernelGGL(k_fold_terms, dim3((unsigned)((max_cap + kTermBlock - 1) / kTermBlock), nl_run, 2),
                       dim3(kTermBlock), 0, st, P.labels.p, B.kcount.p, B.mix_off.p, B.w.p, B.mu.p,
                       B.sigma.p, B.scratch.p, B.scratch.p + 2 * total, B.scratch.p + 3 * total, only_d);
    hipLaunchKernelGGL(k_fold, dim3(nl_run), dim3(kParzenBlock), 0, st, P.labels.p, B.kcount.p,
                       B.mix_off.p, B.w.p, B.mu.p, B.sigma.p, P.comps64.p, P.comps32.p, P.samp.p,
                       B.scratch.p, B.scratch.p + 2 * total, B.scratch.p + 3 * total, B.scratch.p + total,
                       ctx->build_err.p, only_d);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(ctx->ev1, st));
    // the report -- DLabels, error flag, tie report -- packed by one launch
    // into one block and read back with ONE copy (three before)
    const int64_t rep_dl = (int64_t)n_labels * (int64_t)sizeof(DLabel);
    const int64_t rep_bytes = rep_dl + 16 + (int64_t)(n_labels + 1) * (int64_t)sizeof(int32_t);
    HIPCHK(ctx, B.d_rep.reserve(rep_bytes));
    HIPCHK(ctx, B.h_rep.resize(rep_bytes));
    hipLaunchKernelGGL(k_build_report, dim3(1), dim3(kUpBlock), 0, st, (const uint32_t*)P.labels.p,
                       (int32_t)(rep_dl / 4), ctx->build_err.p, B.ties.p, n_labels + 1, (uint32_t*)B.d_rep.p);
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(B.h_rep.data(), B.d_rep.p, rep_bytes, hipMemcpyDeviceToHost, st));
    if (!beside) {   // does the expansion index of the previous posterior still hold?
        const int rc = tpe_rt::bx_keep_check(ctx);
        if (rc) return rc;
    }
    // the armed index's per-label scan rides on this sync when the label
    // groups (on the device since the previous build) are unchanged: the
    // index then starts without a round trip of its own
    bool prescan = false;
    if (!subset && arm_c > 0 && P.groups.p) {
        std::vector<int32_t> cat_now;
        for (int m = 0; m < kNumModes; ++m) cat_now.insert(cat_now.end(), grp[m].begin(), grp[m].end());
        bool same = cat_now == P.groups_h;
        for (int m = 0; same && m < kNumModes; ++m) same = grp[m] == P.h_group[m];
        if (same) {
            const int rc = tpe_rt::bx_prescan(ctx, st, &prescan);
            if (rc) return rc;
        }
    }
    // beside the index: the quantized labels' runs for the coming round
    // (k_qcompress) go on the aux stream too, under the same sync -- over the
    // previous build's label groups, which a subset rebuild of the same
    // history keeps (checked)
    bool qc_queued = false;
    if (beside && P.groups.p) {
        std::vector<int32_t> cat_now;
        for (int m = 0; m < kNumModes; ++m) cat_now.insert(cat_now.end(), grp[m].begin(), grp[m].end());
        if (cat_now == P.groups_h) {
            const int rc = tpe_rt::qc_launch(ctx, st);
            if (rc) return rc;
            qc_queued = true;
        }
    }
    BuildTail t;
    t.st = st;
    t.rep_dl = rep_dl;
    t.n_labels = n_labels;
    t.lf = lf;
    t.n_below = n_below;
    t.dl = std::move(dl);
    for (int m = 0; m < kNumModes; ++m) t.grp[m] = std::move(grp[m]);
    t.mix = std::move(mix);
    t.beside = beside;
    t.qc_queued = qc_queued;
    t.subset = subset;
    t.n_trials = n_trials;
    t.n_valid = n_valid;
    t.arm_c = arm_c;
    t.arm_r = arm_r;
    t.prescan = prescan;
    t.gamma = gamma;
    t.pw = prior_weight;
    if (!subset) t.loss_hash = loss_fingerprint(losses, n_trials);
    if (beside && subset && qc_queued && defer_report) {
        // deferred (TPE_OPT_DEFER_REPORT): the rebuild runs on the second
        // stream; the next round applies its report after queuing the dense
        // labels' kernels, which it does not touch (settle_build).  The
        // caller's tie report comes from tpe_build_report.
        t.deferred = true;
        B.pending.reset(new BuildTail(std::move(t)));
        if (ties_out) std::memset(ties_out, 0, (n_labels + 1) * sizeof(int32_t));
        if (n_below_out) *n_below_out = n_below;
        return TPE_OK;
    }
    return finish_build(ctx, t, ties_out, n_below_out);
}

}  // namespace

int tpe_rt::settle_build(tpe_ctx* ctx) {
    if (!ctx) return TPE_OK;
    auto& B = ctx->build;
    if (!B.pending) return TPE_OK;
    std::unique_ptr<BuildTail> t = std::move(B.pending);
    return finish_build(ctx, *t, nullptr, nullptr);
}

// ================================================================ C ABI ====
extern "C" {

TPE_DEV int tpe1_history_reset(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                      const double* cat_p, int64_t n_cat_p) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    return history_reset(ctx, specs, n_labels, cat_p, n_cat_p);
}

TPE_DEV int tpe1_history_append(tpe_ctx* ctx, const int64_t* n_new, const int32_t* obs_trial,
                       const double* obs_val) {
    if (!ctx || !n_new) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    return history_append(ctx, n_new, obs_trial, obs_val);
}

TPE_DEV int tpe1_build_posterior_resident(tpe_ctx* ctx, const double* losses, int64_t n_trials,
                                 int64_t n_valid, double gamma, double prior_weight, int32_t lf,
                                 int32_t* n_below_out) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    return build_resident(ctx, losses, n_trials, n_valid, gamma, prior_weight, lf, n_below_out);
}

TPE_DEV int tpe1_build_posterior_resident_ordered(tpe_ctx* ctx, const double* losses, int64_t n_trials,
                                                  int64_t n_valid, double gamma, double prior_weight,
                                                  int32_t lf, const uint8_t* below, const int64_t* order_off,
                                                  const int32_t* order, int32_t* n_below_out, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    return build_resident(ctx, losses, n_trials, n_valid, gamma, prior_weight, lf, n_below_out, below,
                          order_off, order, ties);
}

TPE_DEV int tpe1_rebuild_labels(tpe_ctx* ctx, const double* losses, int64_t n_trials, int64_t n_valid,
                                double gamma, double prior_weight, int32_t lf, const int64_t* order_off,
                                const int32_t* order, const int32_t* labels, int32_t n_only,
                                int32_t* n_below_out, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (!labels || n_only <= 0) return ctx->fail(TPE_ERR_ARG, "tpe_rebuild_labels: no labels");
    return build_resident(ctx, losses, n_trials, n_valid, gamma, prior_weight, lf, n_below_out, nullptr,
                          order_off, order, ties, labels, n_only);
}

TPE_DEV int tpe1_build_posterior(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                        const double* cat_p, int64_t n_cat_p, const double* losses,
                        int64_t n_trials, const int64_t* obs_off, const int32_t* obs_trial,
                        const double* obs_val, double gamma, double prior_weight, int32_t lf,
                        int32_t* n_below_out) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (n_labels <= 0 || !specs || !obs_off || n_trials < 0 || (n_trials > 0 && !losses))
        return ctx->fail(TPE_ERR_ARG, "tpe_build_posterior: bad arguments");
    if (obs_off[0] != 0 || obs_off[n_labels] < 0 || obs_off[n_labels] >= INT32_MAX)
        return ctx->fail(TPE_ERR_ARG, "observation offsets");
    std::vector<int64_t> n_new(n_labels);
    for (int32_t l = 0; l < n_labels; ++l) {
        n_new[l] = obs_off[l + 1] - obs_off[l];
        if (n_new[l] < 0) return ctx->fail(TPE_ERR_ARG, "observation offsets must not decrease");
    }
    int64_t n_valid = 0;
    for (int64_t t = 0; t < n_trials; ++t) n_valid += losses[t] == losses[t];
    int rc = history_reset(ctx, specs, n_labels, cat_p, n_cat_p);
    if (!rc) rc = history_append(ctx, n_new.data(), obs_trial, obs_val);
    if (!rc) rc = build_resident(ctx, losses, n_trials, n_valid, gamma, prior_weight, lf, n_below_out);
    if (rc) ctx->build.hist_ready = false;
    return rc;
}

TPE_DEV int tpe1_get_mixture(tpe_ctx* ctx, int32_t label, int32_t side, double* weights, double* mus,
                             double* sigmas, int32_t cap, int32_t* n) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    auto& B = ctx->build;
    if (label < 0 || label >= B.n_labels || side < 0 || side > 1 || ctx->resident.n_labels != B.n_labels)
        return ctx->fail(TPE_ERR_ARG, "tpe_get_mixture: no such built mixture");
    const DLabel& d = ctx->resident.h_labels[label];
    const int32_t K = side ? d.na : d.nb;
    if (n) *n = K;
    const int32_t m = std::min(K, std::max(cap, 0));
    const int64_t o = B.mix_h[2 * (size_t)label + side];
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (m > 0) {
        if (weights) HIPCHK(ctx, hipMemcpy(weights, B.w.p + o, m * sizeof(double), hipMemcpyDeviceToHost));
        if (mus) HIPCHK(ctx, hipMemcpy(mus, B.mu.p + o, m * sizeof(double), hipMemcpyDeviceToHost));
        if (sigmas) HIPCHK(ctx, hipMemcpy(sigmas, B.sigma.p + o, m * sizeof(double), hipMemcpyDeviceToHost));
    }
    return TPE_OK;
}

TPE_DEV int32_t tpe1_resident_labels(const tpe_ctx* ctx) { return ctx ? ctx->resident.n_labels : 0; }

TPE_DEV int tpe1_last_build_ms(const tpe_ctx* ctx, float* ms) {
    if (!ctx || !ms) return TPE_ERR_ARG;
    TPE_SETTLE(const_cast<tpe_ctx*>(ctx));
    *ms = ctx->build_ms;
    return TPE_OK;
}

TPE_DEV int tpe1_build_report(tpe_ctx* ctx, int32_t* n_below, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    TPE_SETTLE(ctx);
    if (n_below) *n_below = ctx->build.last_n_below;
    if (ties) {
        const auto& t = ctx->build.last_ties;
        if (t.empty()) return ctx->fail(TPE_ERR_ARG, "tpe_build_report: no build");
        std::memcpy(ties, t.data(), t.size() * sizeof(int32_t));
    }
    return TPE_OK;
}

}  // extern "C"
