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
#include <hip/hip_runtime.h>

#include <condition_variable>
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
    return for_all(ctx, [&](tpe_ctx* x, int) {
        return tpe1_set_posterior(x, labels, n_labels, weights, mus, sigmas, n_components);
    });
}

int tpe_set_option(tpe_ctx* ctx, int32_t option, int64_t value) {
    if (!ctx) return TPE_ERR_ARG;
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
    return for_all(ctx, [&](tpe_ctx* x, int) {
        return tpe1_history_reset(x, specs, n_labels, cat_p, n_cat_p);
    });
}

int tpe_history_append(tpe_ctx* ctx, const int64_t* n_new, const int32_t* obs_trial,
                       const double* obs_val) {
    if (!ctx) return TPE_ERR_ARG;
    return for_all(ctx, [&](tpe_ctx* x, int) {
        return tpe1_history_append(x, n_new, obs_trial, obs_val);
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
    return for_all(ctx, [&](tpe_ctx* x, int d) {
        return tpe1_build_posterior_resident_ordered(x, losses, n_trials, n_valid, gamma, prior_weight, lf,
                                                     below, order_off, order, d == 0 ? n_below_out : nullptr,
                                                     d == 0 ? ties : nullptr);
    });
}

int tpe_rebuild_labels(tpe_ctx* ctx, const double* losses, int64_t n_trials, int64_t n_valid, double gamma,
                       double prior_weight, int32_t lf, const int64_t* order_off, const int32_t* order,
                       const int32_t* labels, int32_t n_only, int32_t* n_below_out, int32_t* ties) {
    if (!ctx) return TPE_ERR_ARG;
    return for_all(ctx, [&](tpe_ctx* x, int d) {
        return tpe1_rebuild_labels(x, losses, n_trials, n_valid, gamma, prior_weight, lf, order_off, order, labels,
                                   n_only, d == 0 ? n_below_out : nullptr, d == 0 ? ties : nullptr);
    });
}

int tpe_build_posterior(tpe_ctx* ctx, const tpe_label_spec* specs, int32_t n_labels,
                        const double* cat_p, int64_t n_cat_p, const double* losses,
                        int64_t n_trials, const int64_t* obs_off, const int32_t* obs_trial,
                        const double* obs_val, double gamma, double prior_weight, int32_t lf,
                        int32_t* n_below_out) {
    if (!ctx) return TPE_ERR_ARG;
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
    return sharded_round(ctx, seed, &round, 1, n_candidates, cand_offset, out);
}

int tpe_suggest_batch(tpe_ctx* ctx, uint64_t seed, const uint32_t* rounds, int32_t n_rounds,
                      int64_t n_candidates, int64_t cand_offset, tpe_label_result* out) {
    if (!ctx || !out || !rounds) return TPE_ERR_ARG;
    if (ctx->peers.empty())
        return tpe1_suggest_batch(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, out);
    if (n_rounds <= 0) return ctx->fail(TPE_ERR_ARG, "bad candidate/round count");
    return sharded_round(ctx, seed, rounds, n_rounds, n_candidates, cand_offset, out);
}

}  // extern "C"
