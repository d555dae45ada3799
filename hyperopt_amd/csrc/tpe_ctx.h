// tpe_ctx.h -- the context shared by the suggestion engine (tpe_engine.hip)
// and the device posterior builder (tpe_build.hip): device buffers, the
// resident posterior, per-round scratch.  Host-side C++ only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "../../include/hyperopt_tpe.h"
#include "tpe_device.h"

struct tpe_ctx;

namespace tpe_rt {

struct RescoreChunkH {   // k_rescore work item: (round * labels + label position, chunk)
    int32_t cell, j;
};
// the re-score's plan, made on the device (k_rescore_plan): candidates to
// re-score, table entries, sliced or chunked, and whether the candidates
// exceed the buffers the host sized (the round then runs again)
struct RescorePlanH {
    int64_t total;
    int32_t ne, sliced, overflow, pad;
};

using tpe::Comp;
using tpe::DLabel;
using tpe::Partial;
using tpe::SampRec;

constexpr int kBlock = 256;
constexpr int kNumModes = 5;

// Per (round, quantized label) grid window decided on the host after k_qsample.
struct QInfo {
    int64_t jmin;
    int64_t G;        // table slots; 0 = evaluate every candidate directly
    int64_t tab_off;
    int64_t jlo, jhi;  // every grid index a candidate can take lies in [jlo, jhi] (empty: unknown)
    int64_t pad;
};

// device bytes held by every DevBuf of the process (tpe_device_bytes)
inline std::atomic<int64_t>& device_bytes_held() {
    static std::atomic<int64_t> n{0};
    return n;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    static void account(size_t elems, int sign) {
        device_bytes_held().fetch_add(sign * (int64_t)(elems * sizeof(T)), std::memory_order_relaxed);
    }
    // grows by at least 1/4 (a history that grows by one trial per call
    // would otherwise reallocate -- and hipFree synchronise the device --
    // on every build); the contents are not kept
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        release();
        const size_t want = std::max<size_t>(n, 1), grown = want + want / 4;
        hipError_t e = hipMalloc(&p, grown * sizeof(T));
        if (e == hipSuccess) {
            cap = grown;
            account(cap, 1);
            return e;
        }
        (void)hipGetLastError();   // (clear the failed allocation) exactly n, then
        e = hipMalloc(&p, want * sizeof(T));
        if (e == hipSuccess) {
            cap = want;
            account(cap, 1);
        }
        return e;
    }
    void release() {
        if (p) {
            (void)hipFree(p);
            account(cap, -1);
        }
        p = nullptr;
        cap = 0;
    }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap) {
        o.p = nullptr;
        o.cap = 0;
    }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            p = o.p;
            cap = o.cap;
            o.p = nullptr;
            o.cap = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }   // (every buffer a context holds goes with it)
};

// Page-locked host memory for the per-round read-backs: an async D2H copy
// into pageable memory runs as a staged copy the host waits for (~20 us
// each, several per round); into pinned memory it is one DMA on the stream.
template <typename T>
struct PinVec {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    hipError_t resize(size_t m) {
        if (m > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = n = 0;
            const size_t c = std::max<size_t>(m + m / 4, 16);
            const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), c * sizeof(T), hipHostMallocDefault);
            if (e != hipSuccess) {
                p = nullptr;
                return e;
            }
            cap = c;
        }
        n = m;
        return hipSuccess;
    }
    T* data() { return p; }
    const T* data() const { return p; }
    size_t size() const { return n; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    PinVec() = default;
    PinVec(const PinVec&) = delete;
    PinVec& operator=(const PinVec&) = delete;
    ~PinVec() {
        if (p) (void)hipHostFree(p);
    }
};

// the scalar read-backs of a call, in one pinned block
struct PinScalars {
    int32_t err = 0, hot_flag = 0, bx_diff = 1, pad = 0;
    unsigned long long screen_exec = 0, xdrawn[2] = {0, 0};
    RescorePlanH plan{};   // the packed map's re-score plan of the last round
};

struct Posterior {
    std::vector<DLabel> h_labels;
    std::vector<int32_t> h_group[kNumModes];   // label ids per mode
    int32_t n_labels = 0;
    DevBuf<DLabel> labels;
    DevBuf<Comp<double>> comps64;
    DevBuf<Comp<float>> comps32;
    DevBuf<SampRec> samp;
    DevBuf<int32_t> groups;              // concatenated h_group
    std::vector<int32_t> groups_h;       // host copy of what `groups` holds
    int32_t group_off[kNumModes] = {};
    // window index of the dense labels' above mixtures (windowed fp32 screen,
    // tpe_engine.hip k_win_*), built on first use after every posterior change
    bool win_ready = false;
    // exact-zero windows of the dense labels' above mixtures (packed
    // re-score, k_zero_windows): per component, prefix max of the largest x'
    // where its fp64 term can be nonzero, suffix min of the smallest
    bool zw_ready = false;
    DevBuf<double> zw_hi, zw_lo;
    DevBuf<int32_t> zw_wide, zw_n;       // per label at comp_a: its wide records; per label: their count
    // the quantized labels' above mixtures as runs of equal (mu, a)
    // (k_qcompress, for k_qtable): per label at comp_a, and their count
    bool qc_ready = false;
    DevBuf<Comp<double>> qcomp;
    DevBuf<int32_t> qc_n;
    int32_t win_t = 0;                   // the cut T the index was built for
    DevBuf<tpe::WinLabel> win;           // per label
    DevBuf<double> win_p, win_q;         // per component: prefix max of hi / suffix min of lo
    DevBuf<Comp<float>> win_wide;        // per label at comp_a: wide records, w = index bits
    DevBuf<int2> win_bins;               // per label: kWinBins windows [k_lo, k_hi)
    DevBuf<double> win_seg;              // per (label position, segment): max hi, min lo, wide count
    DevBuf<int32_t> win_hist;            // per label position: histogram of log2 interval widths
    DevBuf<uint8_t> win_flag;            // per component: 1 = wide
    DevBuf<double> win_skip;             // per label: kWinBins bounds of the mass a bin's window skips
    DevBuf<double> win_skip_part;        //   their partial sums per chunk of components
    // expansion screen index (tpe_expand.hip), built on first use after every
    // posterior change; bx_ok: every dense label has one (else the windowed
    // screen runs)
    bool bx_ready = false, bx_ok = false;
    // the index's per-label scan, queued by a full build under its report's
    // sync (bx_prescan) and consumed by the next bx_build: no round trip of its own
    bool bx_prescan_ok = false;
    PinVec<double> bx_scan_h;
    DevBuf<tpe::BxLabel> bx;             // per label
    std::vector<tpe::BxLabel> bx_h;
    PinVec<tpe::BxLabel> bx_up_h;        //   its upload's staging (pinned)
    DevBuf<double> bx_tab;               // per label: nbins rows of kBxRow doubles
    DevBuf<int32_t> bx_nc;               // per label at comp_a: unclipped above components
    DevBuf<tpe::BxTerm> bx_terms;        // per above record of a dense label: its bound terms (k_bx_terms)
    DevBuf<int32_t> bx_loff;             // per bin: the length of its list
    DevBuf<int32_t> bx_list;             // per bin: a slot of n_nc, the unclipped components reaching it
    DevBuf<double> bx_scan;              // per dense label position: range, a*, counts
    DevBuf<float2> bx_sb;                // hot-bin prefilter: per sub-bin (U, L) of the score
    DevBuf<float> bx_sbp;                //   and the below mixture's sampling mass of it
    DevBuf<double> bx_part;              // k_bx_table's split-window partial sums
    DevBuf<int2> bx_blocks;              // k_bx_table's 64-bin blocks (label position, first bin)
    PinVec<int2> bx_blocks_h;            //   staged (pinned: the copy is asynchronous)
    int64_t bx_sb_max = 0;               //   the most sub-bins of one label
    uint64_t bx_gen = 0;                 // bumped by every build of the tables (never 0 once built)
    // what the index was built from (the dense labels' DLabel, records and
    // sampling records, at the same offsets): a rebuild of the posterior that
    // leaves them bit-identical keeps the index (bx_keep_check)
    DevBuf<tpe::DLabel> bx_snap_l;
    DevBuf<tpe::Comp<double>> bx_snap_c;
    DevBuf<tpe::SampRec> bx_snap_s;
    DevBuf<int32_t> bx_snap_g;           // the dense label positions
    DevBuf<int32_t> bx_diff;             // compare result (0: identical)
    int32_t bx_snap_nl = 0;
    void release() {
        labels.release();
        comps64.release();
        comps32.release();
        samp.release();
        groups.release();
        groups_h.clear();
        win.release();
        win_p.release();
        win_q.release();
        win_wide.release();
        win_bins.release();
        win_seg.release();
        win_hist.release();
        win_flag.release();
        win_skip.release();
        win_skip_part.release();
        win_ready = false;
        zw_ready = false;
        qc_ready = false;
        qcomp.release();
        qc_n.release();
        zw_hi.release();
        zw_lo.release();
        zw_wide.release();
        zw_n.release();
        bx.release();
        bx_h.clear();
        bx_tab.release();
        bx_nc.release();
        bx_terms.release();
        bx_loff.release();
        bx_list.release();
        bx_scan.release();
        bx_sb.release();
        bx_sbp.release();
        bx_part.release();
        bx_blocks.release();
        bx_snap_l.release();
        bx_snap_c.release();
        bx_snap_s.release();
        bx_snap_g.release();
        bx_diff.release();
        bx_snap_nl = 0;
        bx_ready = bx_ok = false;
        n_labels = 0;
    }
};

// device-to-device copies in ONE launch, the specs passed by value (no
// table to upload): each was its own hipMemcpyAsync -- a blit kernel of ~5
// us on the device and ~7 us of host API time (tpe_build.hip)
struct CopySpec {
    void* dst;
    const void* src;
    int64_t bytes;   // a multiple of 4, both pointers 4-byte aligned
};
constexpr int kCopyBatch = 8;
int copy_batch(tpe_ctx* ctx, hipStream_t st, const CopySpec* specs, int n);

// one input of a build in its staging block (k_build_inputs)
struct UpTask {
    int64_t src;     // byte offset in the staging block; < 0: zero-fill
    uint8_t* dst;
    int64_t bytes;
    int64_t pad;
};

// What the end of a build applies on the host once its report is in
// (tpe_build.hip finish_build).  A subset rebuild beside the index with
// TPE_OPT_DEFER_REPORT leaves it pending: the next round settles it after
// queuing the dense labels' kernels (settle_build), every other entry point
// first thing.
struct BuildTail {
    hipStream_t st = nullptr;
    int64_t rep_dl = 0;
    int32_t n_labels = 0, lf = 0, n_below = 0;
    std::vector<DLabel> dl;
    std::vector<int32_t> grp[kNumModes];
    std::vector<int64_t> mix;
    bool beside = false, qc_queued = false, subset = false, deferred = false;
    int64_t n_trials = 0, n_valid = 0, arm_c = 0;
    int32_t arm_r = 0;
    bool prescan = false;                // the index's scan queued under this build's sync (bx_prescan)
    double gamma = 0.0, pw = 0.0;
    uint64_t loss_hash = 0;
};
int settle_build(tpe_ctx* ctx);

// The device posterior builder (tpe_build.hip): the resident history pool
// and the per-build scratch, grown on demand.
struct BuildBufs {
    // resident history (tpe_history_reset / tpe_history_append)
    std::vector<tpe_label_spec> specs_h;
    std::vector<int64_t> cap_h, off_h;   // per label pool capacity / offset
    std::vector<int32_t> cnt_h;          // per label observations held
    int64_t pool_cap = 0;
    bool hist_ready = false;
    DevBuf<tpe_label_spec> specs;
    DevBuf<double> cat_p;
    DevBuf<int64_t> p_off;         // pool offsets [L]
    DevBuf<int32_t> cnt;           // observations held [L]
    DevBuf<int32_t> p_trial;       // pool, observation order: trial position
    DevBuf<double> p_val;          //   and (transformed) value
    DevBuf<double> s_key, s_key2;  // pool, value order (continuous labels)
    DevBuf<int32_t> s_idx, s_idx2; //   observation index of each sorted key
    DevBuf<int32_t> arank;         // pool: rank in the above list, -1 if not above
    DevBuf<int64_t> st_off;        // staging of an append: CSR offsets [L + 1]
    DevBuf<int32_t> st_trial, st_idx, st_idx_sorted;
    DevBuf<double> st_val, st_key_sorted;
    DevBuf<int32_t> seg_begin, seg_end;
    DevBuf<uint8_t> sort_tmp;
    DevBuf<int32_t> gs_a, gs_b;    // large appends: staging positions through the two sorts
    DevBuf<uint32_t> gs_lab, gs_lab2; //   and the label of each position
    // an append's host side, page-locked: its H2D copies run on the stream
    // without the host waiting for them (the next append first waits for
    // ev_staged, the copies out of these buffers)
    PinVec<uint8_t> h_stage;       // offsets, values, trials, segments, new counts
    DevBuf<uint8_t> d_stage;
    hipEvent_t ev_staged = nullptr;
    bool staged_pending = false;
    // per build
    DevBuf<double> losses;
    DevBuf<uint8_t> below;         // per trial: in the below set
    DevBuf<double> keys;           // per label: above observations (sorted / in order)
    DevBuf<int32_t> idx;           //   and their above-list rank
    DevBuf<double> below_val;      // per label, <= lf below observations
    DevBuf<int32_t> counts;        // per label: below / above observation counts
    DevBuf<int32_t> kcount;        // per label: below / above component counts
    DevBuf<double> w, mu, sigma;   // the built mixtures (tpe_get_mixture)
    DevBuf<int64_t> mix_off;       // per label: below / above offsets into w/mu/sigma
    DevBuf<double> scratch;        // per-component terms | pairwise leaf sums
    DevBuf<int32_t> ties;          // per label: mixtures that depend on a tie order; [L]: split tie
    DevBuf<int64_t> order_off;     // supplied np.argsort orders of the above observations
    DevBuf<int32_t> order;
    int32_t n_labels = 0;          // labels of the last build (0: none resident)
    std::vector<int64_t> mix_h;    // host copy of mix_off
    // what the last build was of (a label-subset rebuild requires the same):
    // the history generation (bumped by every reset / append) and the arguments
    uint64_t hist_gen = 0, built_gen = 0;
    bool built_ok = false;
    int64_t built_T = -1, built_valid = -1;
    double built_gamma = 0.0, built_pw = 0.0;
    int32_t built_lf = 0;
    uint64_t built_loss_hash = 0;  // fingerprint of the losses (a subset rebuild reuses them)
    DevBuf<int32_t> only;          // the labels of a subset rebuild
    DevBuf<uint64_t> split_key;    // k_split's slices: their n_below + 1 smallest (key, position)
    DevBuf<int64_t> split_pos;
    bool defer = false;            // TPE_OPT_DEFER_REPORT: the next subset rebuild beside the index
    std::unique_ptr<BuildTail> pending;   //   its report, not yet applied
    std::vector<int32_t> last_ties;       // the last applied build's tie report (tpe_build_report)
    int32_t last_n_below = 0;
    // a build's inputs: one pinned staging block, one H2D copy, one scatter
    // launch (tpe_build.hip k_build_inputs); the next build waits for ev_up
    PinVec<uint8_t> h_up, h_rep;
    DevBuf<uint8_t> d_up, d_rep;   // (d_rep: the build's report, k_build_report)
    hipEvent_t ev_up = nullptr;
    bool up_pending = false;
    void release() {
        specs.release(); cat_p.release(); p_off.release(); cnt.release(); p_trial.release();
        p_val.release(); s_key.release(); s_key2.release(); s_idx.release(); s_idx2.release();
        arank.release(); st_off.release(); st_trial.release(); st_idx.release();
        st_idx_sorted.release(); st_val.release(); st_key_sorted.release(); seg_begin.release();
        seg_end.release(); sort_tmp.release(); gs_a.release(); gs_b.release(); gs_lab.release();
        gs_lab2.release(); losses.release(); below.release(); keys.release();
        idx.release(); below_val.release(); counts.release(); kcount.release(); w.release();
        mu.release(); sigma.release(); mix_off.release(); scratch.release(); ties.release();
        order_off.release(); order.release(); only.release(); split_key.release(); split_pos.release();
        d_up.release(); d_rep.release(); d_stage.release();
        if (ev_up) (void)hipEventDestroy(ev_up);
        ev_up = nullptr;
        up_pending = false;
        if (ev_staged) (void)hipEventDestroy(ev_staged);
        ev_staged = nullptr;
        staged_pending = false;
        built_ok = false;
        n_labels = 0;
        hist_ready = false;
        pool_cap = 0;
    }
};

// numpy's pairwise float64 summation (np.sum of a contiguous vector)
double np_pairwise_sum(const double* a, size_t n);

// Cross-shard exchange of the quantized labels' grid windows (per label the
// order-preserving min and max grid index, mm[0..nq) and mm[nq..2nq)): every
// shard of a multi-device round waits for all of them and continues with
// the window of the whole candidate set (tpe_multi.hip).
struct QExchange {
    virtual int exchange(tpe_ctx* ctx, std::vector<unsigned long long>& mm) = 0;
    virtual ~QExchange() {}
};

}  // namespace tpe_rt

struct tpe_ctx {
    using Partial = tpe::Partial;
    using QInfo = tpe_rt::QInfo;
    template <typename T>
    using DevBuf = tpe_rt::DevBuf<T>;
    using Posterior = tpe_rt::Posterior;
    static constexpr int kNumModes = tpe_rt::kNumModes;

    int device = 0;
    int precision = TPE_F64;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    hipEvent_t evm[kNumModes][2] = {};   // per-family kernel brackets
    bool mode_ran[kNumModes] = {};
    float mode_ms[kNumModes] = {};
    int64_t mode_evals[kNumModes] = {};
    std::string err;
    float score_ms = 0.f, round_ms = 0.f;
    int64_t evals = 0;
    bool dedup = true;                   // quantized grid-value tables
    bool timing = true;                  // HIP-event timing of rounds (TPE_OPT_TIMING)

    // The resident posterior (tpe_set_posterior) and a separate one-label
    // slot for the single-op entry points, so that GMM1_lpdf / GMM1 sampling
    // calls never clobber the posterior a suggestion loop has uploaded.
    Posterior resident, single;
    Posterior* P = &resident;

    // per-round scratch
    DevBuf<Partial> partials;
    DevBuf<tpe_label_result> results;
    DevBuf<uint32_t> rounds;
    DevBuf<int32_t> errflag;
    // the posterior builds' own error word (k_build_inputs zeroes it,
    // k_partition / k_parzen / k_fold set bits, k_build_report packs it):
    // a deferred rebuild still running on the second stream never shares a
    // word with the round's kernels on the main one
    DevBuf<int32_t> build_err;
    DevBuf<double> cand, out_lb, out_la;
    DevBuf<int32_t> one_group;
    DevBuf<int64_t> qj;
    DevBuf<unsigned long long> qmm;
    DevBuf<QInfo> qinfo;
    DevBuf<double2> qtab;
    DevBuf<unsigned long long> qkmax;    // per quantized label: the best score key over [jlo, jhi]
    DevBuf<int64_t> xfound;              // per (round, label) cell: the first candidate index found
                                         // holding its label's best drawable score (early exit)
    DevBuf<unsigned long long> xdrawn;   // candidates the early-exit kernels drew: quantized, categorical
    unsigned long long xdrawn_h[2] = {0, 0};
    bool cat_early = false;              // the last round's categorical labels ran k_cat_tiles
    DevBuf<double> xs, slice_part;       // split-K map: candidates, slice sums
    bool splitk = true;                  // split-K for small sampled rounds
    DevBuf<double> chunk_part;           // chunked packed map: x | below sum | above chunk sums
    int32_t chunks_forced = 0;           // TPE_OPT_CHUNKS: 1 = off, > 1 = fixed, 0 = auto
    // fp32 screen of the fp64 round (sampled tile-map rounds, TPE_F64): per
    // candidate an upper bound of its score, per (round, label) the largest
    // lower bound and the compacted candidates that can still win
    bool screen = true;                  // TPE_OPT_SCREEN
    DevBuf<float> scr_hi;
    DevBuf<double> scr_hid;              // expansion screen: fp64 upper bounds
    DevBuf<double2> bx_lohi;             //   packed map: fp64 (lower, upper) per candidate
    bool expand = true;                  // TPE_OPT_EXPAND: expansion screen when eligible
    // hot-bin prefilter of the expansion screen (TPE_OPT_HOT, tpe_device.h)
    int32_t hot = 1;                     // 0 off, 1 on, 2 test: force the fallback
    bool early = true;                   // early exit of quantized / categorical tile rounds
    bool zero_win = true;                // packed re-score skips the exactly-zero above terms
    bool zw_pending = false;             //   its windows launched this round (built iff its plan was not empty)
    double hot_cap_div = 16.0;           // hot lists hold n / hot_cap_div per cell (shrinks on overflow)
    DevBuf<double> hot_x;                // per cell: listed candidates' x (the fp64 draw kernel)
    DevBuf<uint32_t> rs_done;            // the round tail's last-workgroup counters (zeroed by its fills)
    bool dense_one = false;              // this round's dense rows hold their winner in slot 0 only (k_reduce)
    DevBuf<int32_t> hot_pc;              // per sub-bin word: the label's set bits before it (k_hot_prefix)
    DevBuf<uint32_t> hot_ucell;          // per (dense label, sampling component): its u-cells (k_hot_ucells)
    DevBuf<uint4> samp_img;              // per dense label: stage_samp's LDS image (k_samp_image)
    int32_t bx_split = 0;                // TPE_OPT_BX_SPLIT (0: auto)
    int64_t pk_sliced = 8192;            // TPE_OPT_PK_SLICED (0: never sliced)
    int32_t bx_t_force = 0;              // TPE_OPT_BX_T (0: auto)
    double bx_t_next = 64.0;             // the cut T of the next index built (set by its caller)
    DevBuf<int32_t> hot_i, hot_cnt;      //   their indices; per cell the count
    DevBuf<int32_t> hot_mi, hot_mcnt;    //   the marked candidates (k_hot_bx -> k_hot_draw); per segment the count
    DevBuf<unsigned long long> hot_t, hot_tau0;   // per cell largest L; per label tau0
    DevBuf<uint32_t> hot_bits;           // per sub-bin: U >= tau0 (words at sb_off / 32)
    DevBuf<int32_t> hot_flag;            // fallback flag
    DevBuf<int32_t> hot_items;           // k_screen_hot's work items: per cell the first, then the counter
    tpe_rt::PinVec<int32_t> hot_cnt_h;
    int64_t hot_listed = 0;              // last round: candidates the prefilter listed
    int32_t hot_fallback = 0;            // last round: 1 if it re-ran the plain screen
    bool hot_ran = false;
    int64_t hot_cells = 0;               //   cells of its lists (hot_cnt_h, read after the round's sync)
    bool hot_redo = false;               // the round runs again without the prefilter (its check failed)
    DevBuf<int64_t> rs_plan;             // the re-score's plan (k_rescore_plan: total, entries, sliced)
    bool value_only = false;             // TPE_OPT_VALUE_ONLY: packed rounds skip the lpdfs of certified winners
    int32_t mode_mask = 31;              // TPE_OPT_MODE_MASK: the label families sampled rounds launch
    int64_t pk_cap = 1 << 16;            // packed re-score: candidates its buffers hold (grows)
    bool pk_plan_pending = false;        // the packed plan awaits the round's sync
    bool pk_redo = false;                // the round runs again after a plan overflow
    tpe_label_result* dev_out = nullptr; // tpe_suggest_batch_device: the caller's device buffer
    float prep_ms = 0.f;                 // device ms of the last expansion-index build (bx_prepare)
    hipEvent_t ev_prep[2] = {};          //   its bracket, read when asked (tpe_last_prepare)
    bool prep_pending = false;
    uint64_t hot_tau0_gen = 0;           // hot_tau0 holds tau0 of this table generation
    int64_t hot_tau0_n = 0;              //   and this n
    int64_t arm_c = 0;                   // tpe_arm_prepare: the next full build queues the index for
    int32_t arm_r = 0;                   //   rounds of arm_c candidates x arm_r (0: disarmed)
    DevBuf<int32_t> scr_idx;
    DevBuf<unsigned long long> scr_lb;
    DevBuf<int32_t> scr_cnt;
    tpe_rt::PinVec<int32_t> scr_cnt_h;
    tpe_rt::PinVec<tpe_rt::PinScalars> pin;   // one entry: the scalar read-backs
    // a round's small read-backs (counts, flags, statistics, small result
    // sets): registered by defer_read, packed by ONE launch into one device
    // block and copied with ONE D2H before the round's sync (tpe_engine.hip)
    struct RepTask {
        const void* src;
        void* dst;
        int64_t bytes;
    };
    std::vector<RepTask> rep;
    tpe_rt::DevBuf<uint8_t> rep_d;
    tpe_rt::PinVec<uint8_t> rep_h;
    tpe_rt::PinVec<tpe_label_result> res_h;   // a round's results, staged before the caller's buffer
    static constexpr int kResPieces = 4;      //   read back in pieces when large (copy_out overlaps)
    hipEvent_t ev_res[kResPieces] = {};
    tpe_rt::PinVec<tpe::DLabel> dl_h;         // a build's label records, read back
    tpe_rt::PinVec<int32_t> ties_h;           //   and its tie report
    DevBuf<int64_t> scr_chunks;          // k_rescore chunk table ({cell, chunk} int32 pairs)
    DevBuf<int64_t> scr_list;            // packed map: per label, (round << 32 | candidate) to re-score
    DevBuf<Partial> scr_res;             //   their fp64 results
    DevBuf<int64_t> scr_rsel;            //   per (round, label): {first, count} int32 pairs
    DevBuf<int64_t> scr_off;             //   per label: offset of its entries in the compacted order
    DevBuf<int64_t> scr_range;           //   per label: its range of re-score table entries
    DevBuf<double> scr_planes;           //   re-score sums: below | x | above chunk c, per entry
    DevBuf<double> rs_x, rs_part;        // sliced re-score: candidates, slice sums
    DevBuf<int32_t> rs_win;              //   packed map: each entry's zero window
    DevBuf<int64_t> rs_g;                //   and their global indices
    std::vector<tpe_rt::RescoreChunkH> scr_chunks_h;
    int64_t screen_total = 0, screen_rescored = 0;   // last round
    int32_t screen_mode = 0;             // last round: tpe_last_screen_mode
    bool screen_pending = false;         // scr_cnt_h awaits the round's final sync
    // windowed screen (large tile-map rounds): candidates keyed by (round,
    // label, bin) and stably sorted with their (x' fp32, index) values
    bool window = true;                  // TPE_OPT_WINDOW
    int32_t win_t = tpe::kWinTDefault;   // TPE_OPT_WIN_T
    int32_t win_groups = 0;              // TPE_OPT_WIN_GROUPS (0: auto)
    DevBuf<uint32_t> win_keys[2], win_keys2[2];   // two slots: sort of group g + 1
    DevBuf<uint8_t> win_keys8[2], win_keys8b[2];  //   (coarse per-cell keys of large cells)
    DevBuf<uint64_t> win_vals[2], win_vals2[2];   //   while group g is screened
    DevBuf<uint8_t> win_tmp[2];
    hipStream_t aux = nullptr;           // key + sort of the next label group
    hipEvent_t ev_fork = nullptr, ev_sorted[2] = {}, ev_done[2] = {};
    hipEvent_t ev_cat[2] = {};           // the quantized + categorical labels' round on aux: fork, join
    bool aux_families = false;                 // TPE_OPT_AUX_FAMILIES
    std::vector<hipEvent_t> evw;         // per unit: k_screen_win brackets (timing)
    int32_t evw_used = 0;
    DevBuf<unsigned long long> win_evals;   // (candidate, component) terms the screen summed
    DevBuf<float2> win_lohi;             // packed map: per candidate (lower, upper) score bound
    int64_t screen_exec = 0;             // last round: terms summed by the screen
    int64_t screen_rescore_terms = 0;    // last round: fp64 terms of the re-scored candidates
    bool screen_exec_pending = false;
    unsigned long long screen_exec_h = 0;
    hipEvent_t evs[2] = {};              // brackets k_screen alone
    float screen_ms = 0.f;
    tpe_rt::BuildBufs build;             // device posterior builder scratch
    int64_t built_n_trials = 0;          // last tpe_build_posterior: history size
    int32_t built_n_below = 0;           //   and its below-set size
    float build_ms = 0.f;                // device time of the last build

    // multi-device contexts (tpe_ctx_create_multi): the primary context owns
    // one peer context per further device; a peer running one shard of a
    // round gets the whole problem's size and the window exchange
    std::vector<tpe_ctx*> peers;
    std::shared_ptr<void> workers;       // one persistent host thread per peer (tpe_multi.hip)
    std::shared_ptr<void> share;         // posterior export / import scratch (tpe_share.hip)
    int64_t hint_n = 0;                  // candidates per round over all shards (0: this call's)
    int32_t hint_rounds = 0;             // rounds over all shards (0: this call's)
    // the same, set by the caller for the life of the context (one process
    // per GPU, each holding one shard: TPE_OPT_WHOLE_N / _ROUNDS)
    int64_t opt_whole_n = 0;
    int32_t opt_whole_rounds = 0;
    tpe_rt::QExchange* qx = nullptr;
    int32_t shard_id = 0;                // this context's position in a sharded round
    // label shards of a multi-device context (tpe_multi.hip; set by
    // tpe_history_reset with at least one label per device): device d holds
    // the global labels lsh_ids[d] (increasing) of the resident history;
    // per global label its device and local index
    std::vector<std::vector<int32_t>> lsh_ids;
    std::vector<int32_t> lsh_dev, lsh_local;
    int32_t lsh_L = 0;
    bool lsh_enable = true;              // TPE_OPT_LABEL_SHARDS

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    int hip(hipError_t e, const char* what) {
        if (e == hipSuccess) return TPE_OK;
        err = std::string(what) + ": " + hipGetErrorString(e);
        return TPE_ERR_HIP;
    }
};

namespace tpe_rt {
// The windowed screen (tpe_window.hip).  win_prepare builds the window index
// of every dense label of the resident posterior (once per posterior);
// win_screen keys, sorts and screens rounds [z0, z0 + nz) of the dense
// group: per candidate its score's upper bound in `hi` at its SORTED
// position ((z nl + y) n + p), per (round, label) the largest lower bound in
// lbkey[z nl + y]; *sorted_vals maps the batch's sorted positions
// ((z - z0) nl + y) n + p back to candidate indices (low 32 bits).  Probe
// mode (cand_in != nullptr, one label, z0 = 0, nz = 1): the candidates are
// cand_in and s_out / e_out receive the fp32 score and its bound per index.
// Packed mode (cpack = C > 0, batched rounds with small C): one cell per
// label holding all nz rounds' candidates j = z C + i, and lohi[y nz C + j]
// receives (lower, upper) bound of each candidate's score (-inf, +inf:
// uncertified) for the per-round selection.
struct WinScreenArgs {
    const int32_t* grp;
    int32_t nl;
    int64_t n, cand_offset;
    uint64_t seed;
    int32_t z0, nz;
    const double* cand_in;
    float* hi;
    unsigned long long* lbkey;
    double *s_out, *e_out;
    int32_t cpack = 0;
    float2* lohi = nullptr;
    // a group of the round's labels: positions [y0, y0 + nl) of nl_all
    // (0: nl) -- the grp pointer is already offset by y0
    int32_t y0 = 0, nl_all = 0;
    int slot = 0;                        // sort buffers (two, for the pipeline)
};
int win_prepare(tpe_ctx* ctx);
// whole screen on ctx->stream (slot 0): reserve, key + sort, tiles
int win_screen(tpe_ctx* ctx, const WinScreenArgs& a, const uint64_t** sorted_vals);
// the pieces, for pipelining label groups over two streams: buffers for
// `nslots` slots of up to `total` candidates in `cells` cells (before any
// launch: growing a buffer frees it), key + sort into a.slot, the tiles
int win_reserve(tpe_ctx* ctx, size_t total, int64_t cells, int nslots);
int win_sort(tpe_ctx* ctx, const WinScreenArgs& a, hipStream_t st, const uint64_t** sorted);
int win_tiles(tpe_ctx* ctx, const WinScreenArgs& a, const uint64_t* sorted, hipStream_t st);
int64_t win_rounds_per_batch(int64_t n, int32_t nl);

// The expansion screen (tpe_expand.hip).  bx_prepare builds the bin tables
// and lists of every dense label of the resident posterior (once per
// posterior) and sets P->bx_ok when every dense label has one.
int bx_prepare(tpe_ctx* ctx);
uint64_t next_bx_gen();
int bx_build(tpe_ctx* ctx);
// Before a rebuild's final sync: queue the comparison of the rebuilt dense
// labels against the index's snapshot (result in ctx->pin[0].bx_diff after the
// sync); bx_keep_after: whether the index stays valid.
int bx_keep_check(tpe_ctx* ctx);
bool bx_keep_after(tpe_ctx* ctx, bool groups_changed);
// A full build with an armed index and unchanged label groups: queue the
// index's per-label scan and its read-back on `st` before the build's sync
// (bx_build then starts from it); *queued says whether it was
int bx_prescan(tpe_ctx* ctx, hipStream_t st, bool* queued);
// The quantized labels' above mixtures as runs (k_qcompress, tpe_engine.hip)
// queued on `st`; sets P->qc_ready.  The round queues it on its own stream
// when not ready; the subset rebuild beside the expansion index queues it on
// the aux stream, off the round's path.
int qc_launch(tpe_ctx* ctx, hipStream_t st);
}  // namespace tpe_rt

// per-device implementations of the entry points a multi-device context
// forwards or shards (tpe_multi.hip exports the public names)
// a deferred rebuild's report is applied before anything else reads or
// changes the context's posterior (every entry point that touches it;
// rounds settle it themselves after queuing the dense labels' kernels)
#define TPE_SETTLE(ctx)                                   \
    do {                                                  \
        const int settle_rc_ = tpe_rt::settle_build(ctx); \
        if (settle_rc_) return settle_rc_;                \
    } while (0)

#define TPE_DEV __attribute__((visibility("hidden")))
extern "C" {
TPE_DEV int tpe1_set_posterior(tpe_ctx* ctx, const tpe_label_desc* labels, int32_t n_labels,
                               const double* weights, const double* mus, const double* sigmas,
                               int64_t n_components);
TPE_DEV int tpe1_suggest(tpe_ctx* ctx, uint64_t seed, uint32_t round, int64_t n_candidates,
                         int64_t cand_offset, tpe_label_result* out);
TPE_DEV int tpe1_suggest_batch(tpe_ctx* ctx, uint64_t seed, const uint32_t* rounds,
                               int32_t n_rounds, int64_t n_candidates, int64_t cand_offset,
                               tpe_label_result* out);
TPE_DEV int tpe1_set_option(tpe_ctx* ctx, int32_t option, int64_t value);
TPE_DEV int tpe1_prepare(tpe_ctx* ctx, int64_t n_candidates, int32_t n_rounds);
TPE_DEV int tpe1_arm_prepare(tpe_ctx* ctx, int64_t n_candidates, int32_t n_rounds);
TPE_DEV int tpe1_history_reset(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                               const double* cat_p, int64_t n_cat_p);
TPE_DEV int tpe1_history_append(tpe_ctx* ctx, const int64_t* n_new, const int32_t* obs_trial,
                                const double* obs_val);
TPE_DEV int tpe1_build_posterior_resident(tpe_ctx* ctx, const double* losses, int64_t n_trials,
                                          int64_t n_valid, double gamma, double prior_weight,
                                          int32_t lf, int32_t* n_below_out);
TPE_DEV int tpe1_build_posterior_resident_ordered(tpe_ctx* ctx, const double* losses, int64_t n_trials,
                                                  int64_t n_valid, double gamma, double prior_weight,
                                                  int32_t lf, const uint8_t* below, const int64_t* order_off,
                                                  const int32_t* order, int32_t* n_below_out, int32_t* ties);
TPE_DEV int tpe1_rebuild_labels(tpe_ctx* ctx, const double* losses, int64_t n_trials, int64_t n_valid,
                                double gamma, double prior_weight, int32_t lf, const int64_t* order_off,
                                const int32_t* order, const int32_t* labels, int32_t n_only,
                                int32_t* n_below_out, int32_t* ties);
TPE_DEV int tpe1_build_posterior(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                                 const double* cat_p, int64_t n_cat_p, const double* losses,
                                 int64_t n_trials, const int64_t* obs_off, const int32_t* obs_trial,
                                 const double* obs_val, double gamma, double prior_weight,
                                 int32_t lf, int32_t* n_below_out);
TPE_DEV void tpe1_ctx_destroy(tpe_ctx* ctx);
TPE_DEV int tpe1_get_mixture(tpe_ctx* ctx, int32_t label, int32_t side, double* weights, double* mus,
                             double* sigmas, int32_t cap, int32_t* n);
TPE_DEV int32_t tpe1_resident_labels(const tpe_ctx* ctx);
TPE_DEV int tpe1_last_build_ms(const tpe_ctx* ctx, float* ms);
TPE_DEV int tpe1_build_report(tpe_ctx* ctx, int32_t* n_below, int32_t* ties);
TPE_DEV int tpe1_score(tpe_ctx* ctx, int32_t label, const double* cand, int64_t n, double* lpdf_below,
                       double* lpdf_above, tpe_label_result* out);
}

// entry points that read the primary context's posterior alone refuse a
// label-sharded multi-device context (its labels are spread over devices)
#define TPE_NOT_LSHARD(ctx)                                                                        \
    do {                                                                                         \
        if (!(ctx)->lsh_ids.empty())                                                             \
            return (ctx)->fail(TPE_ERR_ARG, "not available on a label-sharded multi-device context"); \
    } while (0)

#define HIPCHK(ctx, call)                                  \
    do {                                                   \
        int _rc = (ctx)->hip((call), #call);               \
        if (_rc != TPE_OK) return _rc;                     \
    } while (0)
