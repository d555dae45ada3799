// tpe_multi.hip -- multi-device contexts: one suggestion engine over several
// GPUs of one node behind the same C ABI (include/hyperopt_tpe.h).
//
// The reference plugs one synchronous `algo(new_ids, domain, trials, seed)`
// call per round into fmin (hyperopt/fmin.py:201-202), so the fan-out over
// GPUs lives inside the call: the primary context (first device) owns one
// peer context per further device, each with its own HIP stream, and
//   * posterior uploads / device builds / history appends / options are
//     forwarded to every device (the builds are deterministic, so every
//     device holds the bit-identical posterior);
//   * a suggestion round is split into contiguous shards -- the candidate
//     range [off, off + n) of every round when there are enough candidates,
//     else whole rounds (batched new_ids) -- one host thread per device runs
//     its shard on its stream, and the per-shard winners are merged with the
//     broadcast_best order (larger score, NaN greatest, lowest global index);
//   * decisions that change a summation order follow the whole problem
//     (tpe_ctx::hint_*), and the quantized labels' grid windows are
//     exchanged between the shards before their tables are built, so every
//     sharding returns the single-device winners bit for bit.
// Candidate indices are global (the Philox counter), so the shards draw
// exactly the single-device candidate set.
//
// Label shards (round 6; the resident-history path -- tpe_history_reset,
// append, the device builds, the index, the rounds -- with at least one
// label per device, TPE_OPT_LABEL_SHARDS on): labels are independent (one
// build_posterior_wrapper + broadcast_best per label, tpe.py:678-692,
// 769-778), so device d holds only its labels (longest processing time
// first: dense 1, quantized 1.5, categorical 0.5 -- parallel.label_shards'
// partition), keeps each label's Philox stream (TPE_HAS_STREAM = its space
// index), and uploads, appends, builds, indexes and runs whole rounds for
// those labels alone; the host scatters each device's winners (48 B per
// label) to their space positions.  The per-posterior work -- history
// append, build, tie orders, expansion index -- then divides over the
// devices with the candidates, where the candidate split repeats it on
// every device.  Spaces with fewer labels than devices, tpe_set_posterior
// and the one-shot tpe_build_posterior keep the candidate / round split.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <algorithm>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hyperopt_tpe.h"
#include "tpe_ctx.h"

namespace {

constexpr int64_t kMinShard = 1024;   // candidates per shard (one tile of the tile map)

int ndev(const tpe_ctx* c) { return 1 + (int)c->peers.size(); }

tpe_ctx* dev(tpe_ctx* c, int d) { return d == 0 ? c : c->peers[d - 1]; }

// One persistent host thread per peer device, created with the first
// fanned-out call and bound to its device once (a call used to spawn and
// join a thread per device): for_all hands every worker the same job and
// waits for the count of pending devices to drop to zero.
struct Workers {
    std::mutex mu;
    std::condition_variable cv_job, cv_done;
    const std::function<int(tpe_ctx*, int)>* job = nullptr;
    uint64_t gen = 0;
    int pending = 0;
    bool stop = false;
    std::vector<int> rc;
    std::vector<std::thread> th;

    ~Workers() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv_job.notify_all();
        for (auto& t : th) t.join();
    }
};

void worker_main(Workers* w, tpe_ctx* x, int d) {
    const bool bound = hipSetDevice(x->device) == hipSuccess;
    uint64_t seen = 0;
    for (;;) {
        std::unique_lock<std::mutex> lk(w->mu);
        w->cv_job.wait(lk, [&] { return w->stop || w->gen != seen; });
        if (w->stop) return;
        seen = w->gen;
        const auto* job = w->job;
        lk.unlock();
        int r;
        if (bound) {
            r = (*job)(x, d);
        } else {
            x->err = "hipSetDevice failed";
            r = TPE_ERR_HIP;
        }
        lk.lock();
        w->rc[d] = r;
        if (--w->pending == 0) w->cv_done.notify_all();
    }
}

Workers* workers_of(tpe_ctx* c) {
    if (!c->workers) {
        auto w = std::make_shared<Workers>();
        const int n = ndev(c);
        w->rc.assign(n, TPE_OK);
        for (int d = 1; d < n; ++d) w->th.emplace_back(worker_main, w.get(), dev(c, d), d);
        c->workers = std::static_pointer_cast<void>(w);
    }
    return static_cast<Workers*>(c->workers.get());
}

// Run fn(device context, d) on every device concurrently (the primary on
// the calling thread, the peers on their workers); the first failing
// device's code and message become the primary's.
int for_all(tpe_ctx* c, const std::function<int(tpe_ctx*, int)>& fn) {
    const int n = ndev(c);
    if (n == 1) return fn(c, 0);
    Workers* w = workers_of(c);
    {
        std::lock_guard<std::mutex> lk(w->mu);
        w->job = &fn;
        w->pending = n - 1;
        for (int d = 0; d < n; ++d) w->rc[d] = TPE_OK;
        ++w->gen;
    }
    w->cv_job.notify_all();
    const int rc0 = fn(c, 0);
    std::vector<int> rc;
    {
        std::unique_lock<std::mutex> lk(w->mu);
        w->cv_done.wait(lk, [&] { return w->pending == 0; });
        rc = w->rc;
    }
    rc[0] = rc0;
    for (int d = 0; d < n; ++d)
        if (rc[d] != TPE_OK) {
            if (d > 0) c->err = "device " + std::to_string(dev(c, d)->device) + ": " + dev(c, d)->err;
            return rc[d];
        }
    return TPE_OK;
}

// The window exchange of one sharded round: every shard posts its per-label
// min/max grid index and waits for the others; a shard that fails before
// posting aborts the exchange so nobody waits forever.
struct WindowExchange final : tpe_rt::QExchange {
    std::mutex mu;
    std::condition_variable cv;
    int expected, arrived = 0;
    bool aborted = false;
    std::vector<unsigned long long> mm;   // combined: min over [0, nq), max over [nq, 2 nq)
    std::vector<char> posted;             // per device: reached the exchange

    explicit WindowExchange(int n) : expected(n), posted(n, 0) {}

    int exchange(tpe_ctx* ctx, std::vector<unsigned long long>& local) override {
        std::unique_lock<std::mutex> lk(mu);
        if (ctx->shard_id >= 0 && ctx->shard_id < expected) posted[ctx->shard_id] = 1;
        const size_t nq = local.size() / 2;
        if (mm.empty()) {
            mm.assign(local.size(), 0ull);
            for (size_t i = 0; i < nq; ++i) mm[i] = ~0ull;
        }
        if (mm.size() != local.size()) {
            aborted = true;
            cv.notify_all();
            return ctx->fail(TPE_ERR_ARG, "multi-device round: shards disagree on the quantized labels");
        }
        for (size_t i = 0; i < nq; ++i) {
            mm[i] = local[i] < mm[i] ? local[i] : mm[i];
            mm[nq + i] = local[nq + i] > mm[nq + i] ? local[nq + i] : mm[nq + i];
        }
        if (++arrived == expected) cv.notify_all();
        cv.wait(lk, [&] { return arrived == expected || aborted || arrived + unposted == expected; });
        if (aborted) return ctx->fail(TPE_ERR_ARG, "multi-device round: another device failed");
        if (arrived != expected)
            return ctx->fail(TPE_ERR_ARG, "multi-device round: shards took different paths");
        local = mm;
        return TPE_OK;
    }

    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }

    // A shard that finished without posting (its round took a path without
    // quantized tables while another's did -- the shards' paths are meant to
    // be identical) must not leave the others waiting: fail them instead.
    void finished(int d) {
        std::lock_guard<std::mutex> lk(mu);
        if (!posted[d]) {
            ++unposted;
            cv.notify_all();
        }
    }
    int unposted = 0;
};

struct Shard {
    int64_t cand_lo = 0, n_cand = 0;   // candidate range of every round
    int32_t round_lo = 0, n_rounds = 0;
};

// Aggregate the last round's statistics of all devices into the primary:
// work summed, times the slowest device's.
void aggregate_stats(tpe_ctx* c) {
    const int n = ndev(c);
    int64_t evals = 0, scr_t = 0, scr_r = 0, scr_x = 0, scr_rt = 0;
    unsigned long long drawn[2] = {0, 0};
    float score_ms = 0.f, round_ms = 0.f, scr_ms = 0.f;
    float mode_ms[tpe_rt::kNumModes] = {};
    int64_t mode_ev[tpe_rt::kNumModes] = {};
    for (int d = 0; d < n; ++d) {
        const tpe_ctx* x = dev(c, d);
        evals += x->evals;
        scr_t += x->screen_total;
        scr_r += x->screen_rescored;
        scr_x += x->screen_exec;
        scr_rt += x->screen_rescore_terms;
        drawn[0] += x->xdrawn_h[0];
        drawn[1] += x->xdrawn_h[1];
        score_ms = std::max(score_ms, x->score_ms);
        round_ms = std::max(round_ms, x->round_ms);
        scr_ms = std::max(scr_ms, x->screen_ms);
        for (int m = 0; m < tpe_rt::kNumModes; ++m) {
            mode_ms[m] = std::max(mode_ms[m], x->mode_ms[m]);
            mode_ev[m] += x->mode_evals[m];
        }
    }
    c->evals = evals;
    c->screen_total = scr_t;
    c->screen_rescored = scr_r;
    c->screen_exec = scr_x;
    c->screen_rescore_terms = scr_rt;
    c->xdrawn_h[0] = drawn[0];
    c->xdrawn_h[1] = drawn[1];
    c->screen_mode = dev(c, 0)->screen_mode;
    c->score_ms = score_ms;
    c->round_ms = round_ms;
    c->screen_ms = scr_ms;
    for (int m = 0; m < tpe_rt::kNumModes; ++m) {
        c->mode_ms[m] = mode_ms[m];
        c->mode_evals[m] = mode_ev[m];
    }
}

// One sharded round (tpe_suggest / tpe_suggest_batch): shards by candidate
// range when every device gets at least kMinShard candidates of each round,
// else by whole rounds, else the primary runs it alone.
int sharded_round(tpe_ctx* c, uint64_t seed, const uint32_t* rounds, int32_t n_rounds,
                  int64_t n, int64_t cand_offset, tpe_label_result* out) {
    const int nd = ndev(c);
    const int32_t L = c->resident.n_labels;
    const bool by_cand = n >= (int64_t)nd * kMinShard;
    const bool by_round = !by_cand && n_rounds >= nd && n > 0;
    if (nd == 1 || L <= 0 || (!by_cand && !by_round))
        return tpe1_suggest_batch(c, seed, rounds, n_rounds, n, cand_offset, out);
    std::vector<Shard> sh(nd);
    for (int d = 0; d < nd; ++d) {
        if (by_cand) {
            const int64_t q = n / nd, r = n % nd;
            sh[d].n_cand = q + (d < r ? 1 : 0);
            sh[d].cand_lo = d * q + std::min<int64_t>(d, r);
            sh[d].round_lo = 0;
            sh[d].n_rounds = n_rounds;
        } else {
            const int32_t q = n_rounds / nd, r = n_rounds % nd;
            sh[d].n_rounds = q + (d < r ? 1 : 0);
            sh[d].round_lo = d * q + std::min<int32_t>(d, r);
            sh[d].cand_lo = 0;
            sh[d].n_cand = n;
        }
    }
    // per-shard outputs: candidate shards into their own blocks (merged
    // below), round shards straight into their rows of `out`
    std::vector<tpe_label_result> parts(by_cand ? (size_t)nd * n_rounds * L : 0);
    WindowExchange wx(nd);
    int rc = for_all(c, [&](tpe_ctx* x, int d) {
        x->hint_n = n;
        x->hint_rounds = n_rounds;
        x->qx = &wx;
        x->shard_id = d;
        tpe_label_result* o = by_cand ? parts.data() + (size_t)d * n_rounds * L
                                      : out + (size_t)sh[d].round_lo * L;
        // candidate shards merge by score: a value-only cell has none
        const bool vo = x->value_only;
        if (by_cand) x->value_only = false;
        int r = tpe1_suggest_batch(x, seed, rounds + sh[d].round_lo, sh[d].n_rounds, sh[d].n_cand,
                                   cand_offset + sh[d].cand_lo, o);
        x->value_only = vo;
        x->hint_n = 0;
        x->hint_rounds = 0;
        x->qx = nullptr;
        if (r) wx.abort();
        else wx.finished(d);
        return r;
    });
    if (rc) return rc;
    if (by_cand) {
        const int32_t rows = n_rounds * L;
        rc = tpe_merge_results(parts.data(), nd, rows, out);
        if (rc) return c->fail(rc, "merging the shards' winners failed");
    }
    aggregate_stats(c);
    return TPE_OK;
}

// -------------------------------------------------------- label shards ----
bool lsharded(const tpe_ctx* c) { return !c->lsh_ids.empty(); }

double label_cost(const tpe_label_spec& s) {
    if (s.kind == TPE_CATEGORICAL) return 0.5;
    return (s.flags & TPE_HAS_Q) ? 1.5 : 1.0;
}

// the partition: largest cost to the least-loaded device (ties: lower
// device, lower label), each device's labels in increasing order
void lsh_assign(tpe_ctx* c, const tpe_label_spec* specs, int32_t L) {
    const int nd = ndev(c);
    c->lsh_ids.assign(nd, {});
    std::vector<double> load(nd, 0.0);
    std::vector<int32_t> order(L);
    for (int32_t i = 0; i < L; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return label_cost(specs[a]) > label_cost(specs[b]); });
    for (int32_t i : order) {
        int d = 0;
        for (int k = 1; k < nd; ++k)
            if (load[k] < load[d]) d = k;
        c->lsh_ids[d].push_back(i);
        load[d] += label_cost(specs[i]);
    }
    c->lsh_dev.assign(L, 0);
    c->lsh_local.assign(L, 0);
    for (int d = 0; d < nd; ++d) {
        std::sort(c->lsh_ids[d].begin(), c->lsh_ids[d].end());
        for (size_t j = 0; j < c->lsh_ids[d].size(); ++j) {
            c->lsh_dev[c->lsh_ids[d][j]] = d;
            c->lsh_local[c->lsh_ids[d][j]] = (int32_t)j;
        }
    }
    c->lsh_L = L;
}

void lsh_clear(tpe_ctx* c) {
    c->lsh_ids.clear();
    c->lsh_dev.clear();
    c->lsh_local.clear();
    c->lsh_L = 0;
}

// a device's share of per-label orders (order_off[L + 1] / order over the
// global labels) in its local numbering
void lsh_orders(const std::vector<int32_t>& ids, const int64_t* order_off, const int32_t* order,
                std::vector<int64_t>& off, std::vector<int32_t>& ord) {
    off.assign(ids.size() + 1, 0);
    ord.clear();
    for (size_t j = 0; j < ids.size(); ++j) {
        const int64_t a = order_off[ids[j]], b = order_off[ids[j] + 1];
        ord.insert(ord.end(), order + a, order + b);
        off[j + 1] = (int64_t)ord.size();
    }
}

// a device's tie report (local labels + the split flag) into the global one
void lsh_ties_merge(const std::vector<int32_t>& ids, const std::vector<int32_t>& t, int32_t L, int32_t* ties) {
    for (size_t j = 0; j < ids.size(); ++j) ties[ids[j]] = t[j];
    ties[L] |= t[ids.size()];
}

// one round of every device's labels, scattered into out[round][label]
int lsh_round(tpe_ctx* c, uint64_t seed, const uint32_t* rounds, int32_t n_rounds, int64_t n, int64_t cand_offset,
              tpe_label_result* out) {
    const int nd = ndev(c);
    const int32_t L = c->lsh_L;
    std::vector<std::vector<tpe_label_result>> parts(nd);
    int rc = for_all(c, [&](tpe_ctx* x, int d) {
        const std::vector<int32_t>& ids = c->lsh_ids[d];
        parts[d].resize((size_t)n_rounds * ids.size());
        return tpe1_suggest_batch(x, seed, rounds, n_rounds, n, cand_offset, parts[d].data());
    });
    if (rc) return rc;
    for (int d = 0; d < nd; ++d) {
        const std::vector<int32_t>& ids = c->lsh_ids[d];
        const size_t Ld = ids.size();
        for (int32_t r = 0; r < n_rounds; ++r)
            for (size_t j = 0; j < Ld; ++j) {
                tpe_label_result v = parts[d][(size_t)r * Ld + j];
                v.label = ids[j];
                out[(size_t)r * L + ids[j]] = v;
            }
    }
    aggregate_stats(c);
    return TPE_OK;
}

}  // namespace

extern "C" {

int tpe_ctx_create_multi(const int* devices, int32_t n_devices, int precision, tpe_ctx** out) {
    if (!out || !devices || n_devices <= 0) return TPE_ERR_ARG;
    *out = nullptr;
    tpe_ctx* c = nullptr;
    int rc = tpe_ctx_create(devices[0], precision, &c);
    if (rc) return rc;
    for (int32_t d = 1; d < n_devices; ++d) {
        tpe_ctx* p = nullptr;
        rc = tpe_ctx_create(devices[d], precision, &p);
        if (rc) {
            tpe_ctx_destroy(c);
            return rc;
        }
        c->peers.push_back(p);
    }
    *out = c;
    return TPE_OK;
}

int32_t tpe_ctx_devices(const tpe_ctx* ctx, int32_t* devices, int32_t cap) {
    if (!ctx) return 0;
    const int n = 1 + (int)ctx->peers.size();
    for (int d = 0; d < n && d < cap; ++d)
        if (devices) devices[d] = d == 0 ? ctx->device : ctx->peers[d - 1]->device;
    return n;
}

void tpe_ctx_destroy(tpe_ctx* ctx) {
    if (!ctx) return;
    ctx->workers.reset();   // (joins the peer workers before their contexts go)
    for (tpe_ctx* p : ctx->peers) tpe1_ctx_destroy(p);
    ctx->peers.clear();
    tpe1_ctx_destroy(ctx);
}

int tpe_set_posterior(tpe_ctx* ctx, const tpe_label_desc* labels, int32_t n_labels,
                      const double* weights, const double* mus, const double* sigmas,
                      int64_t n_components) {
    if (!ctx) return TPE_ERR_ARG;
    lsh_clear(ctx);   // (uploaded posteriors: replicated, candidate / round split)
    return for_all(ctx, [&](tpe_ctx* x, int) {
        return tpe1_set_posterior(x, labels, n_labels, weights, mus, sigmas, n_components);
    });
}

int tpe_set_option(tpe_ctx* ctx, int32_t option, int64_t value) {
    if (!ctx) return TPE_ERR_ARG;
    if (option == TPE_OPT_LABEL_SHARDS) {   // (the multi-device context's own: from the next history reset)
        ctx->lsh_enable = value != 0;
        return TPE_OK;
    }
    return for_all(ctx, [&](tpe_ctx* x, int) { return tpe1_set_option(x, option, value); });
}

int tpe_prepare(tpe_ctx* ctx, int64_t n_candidates, int32_t n_rounds) {
    if (!ctx) return TPE_ERR_ARG;
    return for_all(ctx, [&](tpe_ctx* x, int) { return tpe1_prepare(x, n_candidates, n_rounds); });
}

int tpe_arm_prepare(tpe_ctx* ctx, int64_t n_candidates, int32_t n_rounds) {
    if (!ctx) return TPE_ERR_ARG;
    return for_all(ctx, [&](tpe_ctx* x, int) { return tpe1_arm_prepare(x, n_candidates, n_rounds); });
}

int tpe_history_reset(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                      const double* cat_p, int64_t n_cat_p) {
    if (!ctx) return TPE_ERR_ARG;
    const int nd = ndev(ctx);
    if (nd == 1 || !ctx->lsh_enable || !specs || n_labels < nd) {
        lsh_clear(ctx);
        return for_all(ctx, [&](tpe_ctx* x, int) {
            return tpe1_history_reset(x, specs, n_labels, cat_p, n_cat_p);
        });
    }
    lsh_assign(ctx, specs, n_labels);
    const int rc = for_all(ctx, [&](tpe_ctx* x, int d) {
        std::vector<tpe_label_spec> sub;
        for (int32_t g : ctx->lsh_ids[d]) {
            tpe_label_spec sp = specs[g];
            if (!(sp.flags & TPE_HAS_STREAM)) {   // (its stream: its space position)
                sp.flags |= TPE_HAS_STREAM;
                sp.stream = g;
            }
            sub.push_back(sp);
        }
        return tpe1_history_reset(x, sub.data(), (int32_t)sub.size(), cat_p, n_cat_p);
    });
    if (rc) lsh_clear(ctx);
    return rc;
}

int tpe_history_append(tpe_ctx* ctx, const int64_t* n_new, const int32_t* obs_trial,
                       const double* obs_val) {
    if (!ctx) return TPE_ERR_ARG;
    if (!lsharded(ctx))
        return for_all(ctx, [&](tpe_ctx* x, int) {
            return tpe1_history_append(x, n_new, obs_trial, obs_val);
        });
    if (!n_new) return ctx->fail(TPE_ERR_ARG, "tpe_history_append: no counts");
    const int32_t L = ctx->lsh_L;
    std::vector<int64_t> off(L + 1, 0);   // (the new observations: label after label)
    for (int32_t l = 0; l < L; ++l) {
        if (n_new[l] < 0) return ctx->fail(TPE_ERR_ARG, "tpe_history_append: negative count");
        off[l + 1] = off[l] + n_new[l];
    }
    return for_all(ctx, [&](tpe_ctx* x, int d) {
        const std::vector<int32_t>& ids = ctx->lsh_ids[d];
        std::vector<int64_t> nn(ids.size());
        std::vector<int32_t> tr;
        std::vector<double> va;
        for (size_t j = 0; j < ids.size(); ++j) {
            const int64_t a = off[ids[j]], b = off[ids[j] + 1];
            nn[j] = b - a;
            if (b > a) {
                tr.insert(tr.end(), obs_trial + a, obs_trial + b);
                va.insert(va.end(), obs_val + a, obs_val + b);
            }
        }
        return tpe1_history_append(x, nn.data(), tr.data(), va.data());
    });
}

int tpe_build_posterior_resident(tpe_ctx* ctx, const double* losses, int64_t n_trials,
                                 int64_t n_valid, double gamma, double prior_weight, int32_t lf,
                                 int32_t* n_below_out) {
    if (!ctx) return TPE_ERR_ARG;
    return for_all(ctx, [&](tpe_ctx* x, int d) {
        return tpe1_build_posterior_resident(x, losses, n_trials, n_valid, gamma, prior_weight, lf,
                                             d == 0 ? n_below_out : nullptr);
    });
}

int tpe_build_posterior_resident_ordered(tpe_ctx* ctx, const double* losses, int64_t n_trials,
                                         int64_t n_valid, double gamma, double prior_weight, int32_t lf,
                                         const uint8_t* below, const int64_t* order_off, const int32_t* order,
                                         int32_t* n_below_out, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    if (!lsharded(ctx))
        return for_all(ctx, [&](tpe_ctx* x, int d) {
            return tpe1_build_posterior_resident_ordered(x, losses, n_trials, n_valid, gamma, prior_weight, lf,
                                                         below, order_off, order, d == 0 ? n_below_out : nullptr,
                                                         d == 0 ? ties : nullptr);
        });
    const int nd = ndev(ctx);
    const int32_t L = ctx->lsh_L;
    std::vector<std::vector<int32_t>> td(nd);
    const int rc = for_all(ctx, [&](tpe_ctx* x, int d) {
        const std::vector<int32_t>& ids = ctx->lsh_ids[d];
        std::vector<int64_t> off;
        std::vector<int32_t> ord;
        const bool orders = order_off && order && order_off[L] > 0;
        if (orders) lsh_orders(ids, order_off, order, off, ord);
        td[d].assign(ids.size() + 1, 0);
        return tpe1_build_posterior_resident_ordered(x, losses, n_trials, n_valid, gamma, prior_weight, lf, below,
                                                     orders ? off.data() : nullptr, orders ? ord.data() : nullptr,
                                                     d == 0 ? n_below_out : nullptr, td[d].data());
    });
    if (rc) return rc;
    if (ties) {
        std::fill(ties, ties + L + 1, 0);
        for (int d = 0; d < nd; ++d) lsh_ties_merge(ctx->lsh_ids[d], td[d], L, ties);
    }
    return TPE_OK;
}

int tpe_rebuild_labels(tpe_ctx* ctx, const double* losses, int64_t n_trials, int64_t n_valid, double gamma,
                       double prior_weight, int32_t lf, const int64_t* order_off, const int32_t* order,
                       const int32_t* labels, int32_t n_only, int32_t* n_below_out, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    if (!lsharded(ctx))
        return for_all(ctx, [&](tpe_ctx* x, int d) {
            return tpe1_rebuild_labels(x, losses, n_trials, n_valid, gamma, prior_weight, lf, order_off, order,
                                       labels, n_only, d == 0 ? n_below_out : nullptr, d == 0 ? ties : nullptr);
        });
    if (!labels || n_only <= 0 || !order_off) return ctx->fail(TPE_ERR_ARG, "tpe_rebuild_labels: no labels");
    const int nd = ndev(ctx);
    const int32_t L = ctx->lsh_L;
    std::vector<std::vector<int32_t>> td(nd);
    std::vector<int32_t> nbd(nd, -1);
    const int rc = for_all(ctx, [&](tpe_ctx* x, int d) {
        const std::vector<int32_t>& ids = ctx->lsh_ids[d];
        td[d].assign(ids.size() + 1, 0);
        std::vector<int32_t> mine;   // (its labels of the subset, local numbers: increasing)
        for (int32_t i = 0; i < n_only; ++i) {
            const int32_t g = labels[i];
            if (g < 0 || g >= L) return x->fail(TPE_ERR_ARG, "tpe_rebuild_labels: label out of range");
            if (ctx->lsh_dev[g] == d) mine.push_back(ctx->lsh_local[g]);
        }
        if (mine.empty()) return TPE_OK;   // (its labels keep their build)
        std::vector<int64_t> off;
        std::vector<int32_t> ord;
        lsh_orders(ids, order_off, order, off, ord);
        return tpe1_rebuild_labels(x, losses, n_trials, n_valid, gamma, prior_weight, lf, off.data(), ord.data(),
                                   mine.data(), (int32_t)mine.size(), &nbd[d], td[d].data());
    });
    if (rc) return rc;
    if (n_below_out) {
        *n_below_out = 0;
        for (int d = 0; d < nd; ++d)
            if (nbd[d] >= 0) {
                *n_below_out = nbd[d];
                break;
            }
    }
    if (ties) {
        std::fill(ties, ties + L + 1, 0);
        for (int d = 0; d < nd; ++d) lsh_ties_merge(ctx->lsh_ids[d], td[d], L, ties);
    }
    return TPE_OK;
}

int tpe_build_report(tpe_ctx* ctx, int32_t* n_below, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    if (!lsharded(ctx)) return tpe1_build_report(ctx, n_below, ties);
    const int nd = ndev(ctx);
    const int32_t L = ctx->lsh_L;
    std::vector<std::vector<int32_t>> td(nd);
    int32_t nb0 = 0;
    const int rc = for_all(ctx, [&](tpe_ctx* x, int d) {
        td[d].assign(ctx->lsh_ids[d].size() + 1, 0);
        return tpe1_build_report(x, d == 0 ? &nb0 : nullptr, td[d].data());
    });
    if (rc) return rc;
    if (n_below) *n_below = nb0;
    if (ties) {
        std::fill(ties, ties + L + 1, 0);
        for (int d = 0; d < nd; ++d) lsh_ties_merge(ctx->lsh_ids[d], td[d], L, ties);
    }
    return TPE_OK;
}

int tpe_get_mixture(tpe_ctx* ctx, int32_t label, int32_t side, double* weights, double* mus, double* sigmas,
                    int32_t cap, int32_t* n) {
    if (!ctx) return TPE_ERR_ARG;
    if (!lsharded(ctx)) return tpe1_get_mixture(ctx, label, side, weights, mus, sigmas, cap, n);
    if (label < 0 || label >= ctx->lsh_L) return ctx->fail(TPE_ERR_ARG, "tpe_get_mixture: no such built mixture");
    tpe_ctx* x = dev(ctx, ctx->lsh_dev[label]);
    HIPCHK(ctx, hipSetDevice(x->device));
    const int rc = tpe1_get_mixture(x, ctx->lsh_local[label], side, weights, mus, sigmas, cap, n);
    if (rc) ctx->err = x->err;
    return rc;
}

int32_t tpe_label_device(const tpe_ctx* ctx, int32_t label) {
    if (!ctx || !lsharded(ctx) || label < 0 || label >= ctx->lsh_L) return -1;
    return ctx->lsh_dev[label];
}

int32_t tpe_resident_labels(const tpe_ctx* ctx) {
    if (!ctx) return 0;
    return lsharded(ctx) ? ctx->lsh_L : tpe1_resident_labels(ctx);
}

int tpe_last_build_ms(const tpe_ctx* ctx, float* ms) {
    if (!ctx || !ms) return TPE_ERR_ARG;
    if (!lsharded(ctx)) return tpe1_last_build_ms(ctx, ms);
    float m = 0.f;
    for (int d = 0; d < ndev(const_cast<tpe_ctx*>(ctx)); ++d) {
        float v = 0.f;
        const int rc = tpe1_last_build_ms(dev(const_cast<tpe_ctx*>(ctx), d), &v);
        if (rc) return rc;
        m = std::max(m, v);
    }
    *ms = m;
    return TPE_OK;
}

int tpe_score(tpe_ctx* ctx, int32_t label, const double* cand, int64_t n, double* lpdf_below, double* lpdf_above,
              tpe_label_result* out) {
    if (!ctx) return TPE_ERR_ARG;
    if (!lsharded(ctx)) return tpe1_score(ctx, label, cand, n, lpdf_below, lpdf_above, out);
    if (label < 0 || label >= ctx->lsh_L) return ctx->fail(TPE_ERR_ARG, "tpe_score: label out of range");
    tpe_ctx* x = dev(ctx, ctx->lsh_dev[label]);
    HIPCHK(ctx, hipSetDevice(x->device));
    const int rc = tpe1_score(x, ctx->lsh_local[label], cand, n, lpdf_below, lpdf_above, out);
    if (rc) ctx->err = x->err;
    if (!rc && out) out->label = label;
    return rc;
}

int tpe_build_posterior(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                        const double* cat_p, int64_t n_cat_p, const double* losses,
                        int64_t n_trials, const int64_t* obs_off, const int32_t* obs_trial,
                        const double* obs_val, double gamma, double prior_weight, int32_t lf,
                        int32_t* n_below_out) {
    if (!ctx) return TPE_ERR_ARG;
    lsh_clear(ctx);   // (the one-shot build: replicated, candidate / round split)
    return for_all(ctx, [&](tpe_ctx* x, int d) {
        return tpe1_build_posterior(x, specs, n_labels, cat_p, n_cat_p, losses, n_trials, obs_off,
                                    obs_trial, obs_val, gamma, prior_weight, lf,
                                    d == 0 ? n_below_out : nullptr);
    });
}

int tpe_suggest(tpe_ctx* ctx, uint64_t seed, uint32_t round, int64_t n_candidates,
                int64_t cand_offset, tpe_label_result* out) {
    if (!ctx || !out) return TPE_ERR_ARG;
    if (ctx->peers.empty()) return tpe1_suggest(ctx, seed, round, n_candidates, cand_offset, out);
    if (lsharded(ctx)) return lsh_round(ctx, seed, &round, 1, n_candidates, cand_offset, out);
    return sharded_round(ctx, seed, &round, 1, n_candidates, cand_offset, out);
}

int tpe_suggest_batch(tpe_ctx* ctx, uint64_t seed, const uint32_t* rounds, int32_t n_rounds,
                      int64_t n_candidates, int64_t cand_offset, tpe_label_result* out) {
    if (!ctx || !out || !rounds) return TPE_ERR_ARG;
    if (ctx->peers.empty())
        return tpe1_suggest_batch(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, out);
    if (n_rounds <= 0) return ctx->fail(TPE_ERR_ARG, "bad candidate/round count");
    if (lsharded(ctx)) return lsh_round(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, out);
    return sharded_round(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, out);
}

}  // extern "C"
