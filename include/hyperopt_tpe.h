/*
 * hyperopt_tpe.h -- C ABI of the MI355X (gfx950) TPE suggestion engine.
 *
 * Plain C, plain pointers and sizes; no torch or HIP types cross this
 * boundary.  Every entry point cites the reference function it replaces
 * (mvanveen/hyperopt, paths relative to the repository root).  The reference
 * is pure Python, so its "FFI" is the pyll operator registry: `scope.define`
 * (hyperopt/pyll/base.py:132-138) registers each numeric op by name and
 * `build_posterior` (hyperopt/tpe.py:651-739) wires them per hyperparameter.
 * The ops below are those registry entries, plus one fused entry point
 * (`tpe_suggest`) that runs the whole per-label chain on the GPU.
 *
 * All calls are synchronous with respect to the host: on return, outputs are
 * in the caller's buffers.  A context is not thread-safe; use one per thread.
 * Return value: TPE_OK (0) or a negative TPE_ERR_*; the message is available
 * from tpe_last_error(ctx) (or tpe_last_error(NULL) for tpe_ctx_create).
 */
#ifndef HYPEROPT_TPE_H
#define HYPEROPT_TPE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPE_ABI_VERSION 4

/* error codes; the Python layer maps them to the reference's exception types */
#define TPE_OK 0
#define TPE_ERR_VALUE (-1)   /* ValueError (e.g. 'low >= high', tpe.py:86-87)      */
#define TPE_ERR_TYPE (-2)    /* TypeError (e.g. non-vector params, tpe.py:117-122)  */
#define TPE_ERR_ARG (-3)     /* bad pointer / size / state                          */
#define TPE_ERR_HIP (-4)     /* HIP runtime failure                                 */
#define TPE_ERR_SAMPLE (-5)  /* truncated sampler could not reach the interval     */

/* arithmetic of the dense (unquantized) lpdf paths; quantized and sampling
 * paths always run in fp64 */
#define TPE_F64 0
#define TPE_F32 1

/* posterior families (the `<sampler>` names of tpe.py:712) */
#define TPE_GMM1 0         /* truncated Gaussian mixture            tpe.py:68-172  */
#define TPE_LGMM1 1        /* log-space Gaussian mixture            tpe.py:222-307 */
#define TPE_CATEGORICAL 2  /* categorical over 0..upper-1           tpe.py:56-63   */

/* presence flags for the optional `low`, `high`, `q` arguments (None in Python) */
#define TPE_HAS_LOW 1
#define TPE_HAS_HIGH 2
#define TPE_HAS_Q 4
/* tpe_label_spec only: `stream` names the label's Philox stream (default: its
 * position in the spec array) -- a process holding a subset of the labels
 * (label-sharded ranks) draws the candidates the whole space would */
#define TPE_HAS_STREAM 8

typedef struct tpe_ctx tpe_ctx;

/* One hyperparameter's pair of posteriors (the below/`l` and above/`g`
 * mixtures that build_posterior makes per label, tpe.py:684-692).
 * Mixture components live in flat arrays passed to tpe_set_posterior:
 *   GMM1/LGMM1: weights[off+k], mus[off+k], sigmas[off+k], k < n (as returned
 *               by adaptive_parzen_normal, tpe.py:404-477);
 *   CATEGORICAL: weights[off+k] = p[k] (pseudocount posterior,
 *               tpe.py:581-617); n == upper; mus/sigmas unused.
 * low/high/q are the GMM1/LGMM1 keyword arguments; for LGMM1 low/high are in
 * log space exactly as in the reference call LGMM1(..., low, high, q). */
typedef struct {
    int32_t kind;       /* TPE_GMM1 / TPE_LGMM1 / TPE_CATEGORICAL */
    int32_t flags;      /* TPE_HAS_LOW | TPE_HAS_HIGH | TPE_HAS_Q */
    double low;
    double high;
    double q;
    int64_t below_off;
    int64_t above_off;
    int32_t n_below;
    int32_t n_above;
} tpe_label_desc;       /* 56 bytes */

/* Observation transforms of the adaptive-Parzen samplers (tpe.py:493-576),
 * applied by the caller before tpe_build_posterior (so the transform is the
 * caller's own float64 log, bit-for-bit the reference's np.log):
 *   IDENTITY   uniform, quniform, normal, qnormal, randint, categorical
 *   LOG        loguniform, lognormal:          log(obs)
 *   LOG_FLOOR  qloguniform, qlognormal:        log(max(obs, floor)) */
#define TPE_OBS_IDENTITY 0
#define TPE_OBS_LOG 1
#define TPE_OBS_LOG_FLOOR 2

/* One hyperparameter as build_posterior sees it (tpe.py:678-692): the
 * sampler arguments of its posterior and the prior of its adaptive-Parzen
 * estimator. */
typedef struct {
    int32_t kind;        /* TPE_GMM1 / TPE_LGMM1 / TPE_CATEGORICAL             */
    int32_t flags;       /* TPE_HAS_LOW | TPE_HAS_HIGH | TPE_HAS_Q             */
    double low;          /* sampler arguments, as in tpe_label_desc            */
    double high;
    double q;
    double prior_mu;     /* ap_*_sampler prior (tpe.py:493-576)                */
    double prior_sigma;
    int32_t upper;       /* categorical: number of categories                  */
    int32_t randint;     /* categorical: 1 randint (counts + prior_weight,
                            tpe.py:581-589), 0 pchoice (counts + upper *
                            prior_weight * p, tpe.py:598-617)                  */
    int64_t p_off;       /* pchoice: offset of its p vector in cat_p           */
    int32_t stream;      /* with TPE_HAS_STREAM: the label's Philox stream     */
    int32_t reserved;    /* 0                                                  */
} tpe_label_spec;        /* 72 bytes */

/* Winner of one label's candidate set (broadcast_best, tpe.py:769-778). */
typedef struct {
    double value;       /* samples[best] (categorical: the integer index as double) */
    double score;       /* lpdf_below[best] - lpdf_above[best]                      */
    double lpdf_below;
    double lpdf_above;
    int64_t index;      /* GLOBAL candidate index of the winner (-1: no candidates) */
    int32_t label;
    int32_t status;     /* 0 ok; TPE_STATUS_VALUE_ONLY: index and value only        */
} tpe_label_result;     /* 48 bytes */

/* status of a TPE_OPT_VALUE_ONLY round's cell that the screen alone decided:
 * index and value are the winner's, score / lpdf_below / lpdf_above are NaN
 * (not computed).  Such records carry no order key, so tpe_merge_results and
 * tpe_merge_results_device refuse them (TPE_ERR_ARG). */
#define TPE_STATUS_VALUE_ONLY 1

int tpe_abi_version(void);

/* Hash of the sources the library was built from (16 hex digits); the
 * loader compares it with the sources in the tree and refuses a stale build. */
const char *tpe_source_hash(void);

/* device: HIP ordinal; precision: TPE_F64 or TPE_F32 */
int tpe_ctx_create(int device, int precision, tpe_ctx **out);

/* One context over several GPUs of the node (devices[0] first; a device may
 * repeat, e.g. to test sharding on one GPU).  Every entry point keeps its
 * meaning: posterior uploads, device builds, history appends and options
 * go to every device; tpe_suggest / tpe_suggest_batch split each round over
 * the devices -- contiguous global candidate ranges when every device gets
 * at least 1024 candidates of each round, else whole rounds -- one host
 * thread and HIP stream per device, and merge the per-device winners with
 * the broadcast_best order.  The results are bit-identical to a one-device
 * context's (the reference's single synchronous algo call per
 * round, hyperopt/fmin.py:201-202, keeps the fan-out inside the call).  The
 * single-op entry points, tpe_score and tpe_get_mixture use devices[0]. */
int tpe_ctx_create_multi(const int *devices, int32_t n_devices, int precision, tpe_ctx **out);

/* Devices of a context (writes at most cap ordinals); returns their count. */
int32_t tpe_ctx_devices(const tpe_ctx *ctx, int32_t *devices, int32_t cap);

/* Label shards of a multi-device context (TPE_OPT_LABEL_SHARDS): the
 * position in tpe_ctx_devices' list of the device holding `label` of the
 * resident history, or -1 when the context's labels are not sharded (one
 * device, replicated posteriors, no such label). */
int32_t tpe_label_device(const tpe_ctx *ctx, int32_t label);

void tpe_ctx_destroy(tpe_ctx *ctx);
const char *tpe_last_error(const tpe_ctx *ctx);

/* ---- reference operators, 1:1 (host buffers in and out) ------------------ */

/* GMM1_lpdf(samples, weights, mus, sigmas, low, high, q)   tpe.py:110-172 */
int tpe_gmm1_lpdf(tpe_ctx *ctx, const double *samples, int64_t n,
                  const double *weights, const double *mus, const double *sigmas,
                  int32_t k, int32_t flags, double low, double high, double q,
                  double *out);

/* LGMM1_lpdf(samples, weights, mus, sigmas, low, high, q)  tpe.py:265-307 */
int tpe_lgmm1_lpdf(tpe_ctx *ctx, const double *samples, int64_t n,
                   const double *weights, const double *mus, const double *sigmas,
                   int32_t k, int32_t flags, double low, double high, double q,
                   double *out);

/* categorical_lpdf(sample, p, upper)                        tpe.py:56-63 */
int tpe_categorical_lpdf(tpe_ctx *ctx, const int64_t *samples, int64_t n,
                         const double *p, int32_t upper, double *out);

/* np.argmax(below_llik - above_llik) of broadcast_best      tpe.py:769-778
 * (first NaN wins, NaN above +inf, lowest index wins ties) */
int tpe_broadcast_best(tpe_ctx *ctx, const double *below, const double *above,
                       int64_t n, int64_t *best);

/* GMM1(weights, mus, sigmas, low, high, q, rng, size)      tpe.py:68-99
 * Same distribution as the reference (component ~ weights, Gaussian draw,
 * accept iff low <= draw < high, round(x/q)*q); the random stream is
 * Philox4x32-10 keyed by `seed`, counter = (offset + i, attempt, stream,
 * round), so draw i is the same whatever the batching or GPU count. */
int tpe_gmm1_sample(tpe_ctx *ctx, const double *weights, const double *mus,
                    const double *sigmas, int32_t k, int32_t flags, double low,
                    double high, double q, uint64_t seed, uint32_t stream,
                    uint32_t round, int64_t offset, int64_t n, double *out);

/* LGMM1(weights, mus, sigmas, low, high, q, rng, size)     tpe.py:222-256 */
int tpe_lgmm1_sample(tpe_ctx *ctx, const double *weights, const double *mus,
                     const double *sigmas, int32_t k, int32_t flags, double low,
                     double high, double q, uint64_t seed, uint32_t stream,
                     uint32_t round, int64_t offset, int64_t n, double *out);

/* categorical(p, upper, rng, size)            hyperopt/pyll/stochastic.py:109-147 */
int tpe_categorical_sample(tpe_ctx *ctx, const double *p, int32_t upper,
                           uint64_t seed, uint32_t stream, uint32_t round,
                           int64_t offset, int64_t n, int64_t *out);

/* ---- resident posterior + fused suggestion round ------------------------- */

/* Upload the per-label posteriors (replaces the graph that
 * build_posterior/tpe_transform rebuild on every call, tpe.py:651-739,
 * 794-820).  Arrays are copied; the device copy stays resident until the
 * next call or tpe_ctx_destroy. */
int tpe_set_posterior(tpe_ctx *ctx, const tpe_label_desc *labels, int32_t n_labels,
                      const double *weights, const double *mus, const double *sigmas,
                      int64_t n_components);

/* Build the resident posterior ON THE DEVICE from the trial history
 * (replaces ap_filter_trials tpe.py:624-648, linear_forgetting_weights
 * :385-398, adaptive_parzen_normal :404-477 and the categorical pseudocount
 * posteriors :581-617 for every label, then the same upload as
 * tpe_set_posterior).
 *   losses[t], t < n_trials: loss of trial t, trials in tid order (the
 *       order suggest() sorts docs in, tpe.py:858); +inf for no loss;
 *   per label l, observations obs_off[l] .. obs_off[l+1]-1 in tid order:
 *       obs_trial = position t of the observation's trial in `losses`,
 *       obs_val   = the (already transformed, TPE_OBS_*) value;
 *   gamma, prior_weight: the tpe.suggest arguments; lf: the linear
 *       forgetting of the Parzen weights (adaptive_parzen_normal's LF,
 *       tpe.py:406; 25 = DEFAULT_LF in the reference, which never passes
 *       another -- tpe.suggest's linear_forgetting is unused, :828).
 * The below set is the n_below = min(ceil(gamma sqrt(n_trials)), 25) lowest
 * (gamma_cap = DEFAULT_LF, tpe.py:626,636, whatever lf is)
 * losses; equal losses and equal observations are ordered by position
 * (a stable sort; the reference's np.argsort order for ties is numpy's
 * unstable quicksort -- tpe_build_posterior_resident_ordered takes the
 * reference's order where it matters).  n_below_out (may be NULL) receives
 * n_below. */
int tpe_build_posterior(tpe_ctx *ctx, const tpe_label_spec *specs, int32_t n_labels,
                        const double *cat_p, int64_t n_cat_p,
                        const double *losses, int64_t n_trials,
                        const int64_t *obs_off, const int32_t *obs_trial,
                        const double *obs_val, double gamma, double prior_weight,
                        int32_t lf, int32_t *n_below_out);

/* Device-resident history (the columnar trial history of SURVEY §8f rank 1,
 * kept on the GPU): tpe_history_reset fixes the labels; tpe_history_append
 * adds only NEW observations (per label n_new[l] of them, concatenated
 * label-major: trial position in tid order and transformed value, as for
 * tpe_build_posterior) -- each label's observations are kept in observation
 * order and value-sorted (a stable merge of the sorted new batch), so a
 * rebuild sorts nothing; tpe_build_posterior_resident then rebuilds the
 * posterior from the current losses.  losses[t] = NaN marks a trial that is
 * not in the history (its observations join neither set, like a NaN-loss doc
 * in tpe.py:849-853); n_valid = the number of non-NaN losses (len(l_vals)).
 * tpe_build_posterior is reset + append(all) + build_resident. */
int tpe_history_reset(tpe_ctx *ctx, const tpe_label_spec *specs, int32_t n_labels,
                      const double *cat_p, int64_t n_cat_p);
int tpe_history_append(tpe_ctx *ctx, const int64_t *n_new, const int32_t *obs_trial,
                       const double *obs_val);
int tpe_build_posterior_resident(tpe_ctx *ctx, const double *losses, int64_t n_trials,
                                 int64_t n_valid, double gamma, double prior_weight,
                                 int32_t lf, int32_t *n_below_out);

/* tpe_build_posterior_resident with the reference's tie order (ap_filter_trials
 * tpe.py:637 `l_order = np.argsort(l_vals)` and adaptive_parzen_normal
 * tpe.py:433 `order = np.argsort(mus)`: numpy's unstable sort, whose order of
 * equal keys the device cannot reproduce, so the caller computes it with
 * numpy itself when it matters):
 *   below (NULL: the device split, ties by position): per trial position
 *       1 if the trial is in the below set -- exactly n_below trials, each
 *       with a loss;
 *   order_off[n_labels + 1], order (NULL: none supplied): label l's entries
 *       order[order_off[l] .. order_off[l+1]) are np.argsort of its above
 *       observations (in observation order) -- the above list's indices in
 *       value order; an empty range keeps the device's position order;
 *   ties (may be NULL; n_labels + 1 entries) receives what depends on a tie
 *       order the caller did not supply: ties[l] bit 1 (bit 0) when label l's
 *       above (below) mixture has equal mus while its linear-forgetting
 *       weights differ (the tie order decides which weight meets a run end's
 *       sigma, and the order of the normalising sum); ties[n_labels] = 1
 *       when equal losses straddle the n_below boundary of the split.
 * A caller that gets a non-zero flag computes the reference's order for it
 * and builds again (hyperopt_amd/posterior.py reference_orders). */
int tpe_build_posterior_resident_ordered(tpe_ctx *ctx, const double *losses, int64_t n_trials,
                                         int64_t n_valid, double gamma, double prior_weight,
                                         int32_t lf, const uint8_t *below, const int64_t *order_off,
                                         const int32_t *order, int32_t *n_below_out, int32_t *ties);

/* The ordered rebuild restricted to `labels` (n_only increasing label
 * indices): right after a build of the same resident history with the same
 * arguments (no append in between, or TPE_ERR_ARG), rebuild only those
 * labels with the supplied orders and keep the others' mixtures and records
 * -- the labels whose ties the previous build flagged, when equal losses did
 * not straddle the split (the below set is kept too).  Same outputs as
 * tpe_build_posterior_resident_ordered; the others' tie flags read 0. */
int tpe_rebuild_labels(tpe_ctx *ctx, const double *losses, int64_t n_trials, int64_t n_valid,
                       double gamma, double prior_weight, int32_t lf, const int64_t *order_off,
                       const int32_t *order, const int32_t *labels, int32_t n_only,
                       int32_t *n_below_out, int32_t *ties);

/* Read back one mixture of the resident posterior built by
 * tpe_build_posterior (side 0 below, 1 above): the (weights, mus, sigmas)
 * that adaptive_parzen_normal returns (categorical: p in weights).  *n
 * receives the component count; at most `cap` entries are written. */
int tpe_get_mixture(tpe_ctx *ctx, int32_t label, int32_t side, double *weights,
                    double *mus, double *sigmas, int32_t cap, int32_t *n);

/* Number of labels of the resident posterior (the row count tpe_suggest
 * writes per round). */
int32_t tpe_resident_labels(const tpe_ctx *ctx);

/* Device time (ms, HIP events) of the last tpe_build_posterior's kernels
 * (-1 for a rebuild whose report was deferred, TPE_OPT_DEFER_REPORT). */
int tpe_last_build_ms(const tpe_ctx *ctx, float *ms);

/* The last build's report, applied first if it was deferred
 * (TPE_OPT_DEFER_REPORT): n_below and the tie report tpe_rebuild_labels
 * returns (ties: n_labels + 1 entries, NULL to skip).  Replaces nothing in
 * the reference: the deferral is this library's (posterior.py
 * _build_reference_order reads it after the round). */
int tpe_build_report(tpe_ctx *ctx, int32_t *n_below, int32_t *ties);

/* One suggestion round over every resident label: sample n_candidates per
 * label from the below posterior (global candidate indices
 * cand_offset .. cand_offset+n_candidates-1), score them under both
 * posteriors and keep the best (the GMM1 -> *_lpdf x2 -> broadcast_best
 * chain of tpe.py:686-724, rec_eval'd per label at tpe.py:900).
 * out[label] receives the winner.  `round` separates independent rounds
 * (e.g. new_id) under one seed. */
int tpe_suggest(tpe_ctx *ctx, uint64_t seed, uint32_t round, int64_t n_candidates,
                int64_t cand_offset, tpe_label_result *out);

/* Batched independent rounds (several new_ids at once): round j uses
 * rounds[j]; out has n_rounds * n_labels entries, round-major. */
int tpe_suggest_batch(tpe_ctx *ctx, uint64_t seed, const uint32_t *rounds,
                      int32_t n_rounds, int64_t n_candidates, int64_t cand_offset,
                      tpe_label_result *out);

/* tpe_suggest_batch with the results left in DEVICE memory: d_out (on this
 * single-device context's GPU, n_rounds * n_labels entries) receives them
 * by a device-to-device copy, complete when the call returns -- the buffer a
 * process-per-GPU caller all-gathers over RCCL without a host round trip
 * (the reference's one algo call per round, fmin.py:201-202).
 * out (host, may be NULL) receives them too.  The call runs on the
 * context's own stream: the caller completes any work of its own streams on
 * d_out first. */
int tpe_suggest_batch_device(tpe_ctx *ctx, uint64_t seed, const uint32_t *rounds,
                             int32_t n_rounds, int64_t n_candidates, int64_t cand_offset,
                             tpe_label_result *d_out, tpe_label_result *out);

/* tpe_merge_results on device buffers of ctx's GPU (d_parts: n_parts blocks
 * of n results, e.g. an RCCL all-gather of the ranks' tpe_suggest_batch_device
 * outputs; d_out: n results), on the context's stream, complete on return.
 * d_parts must be complete when called (an H2D copy or collective on another
 * stream synchronised first: nothing orders it against this stream). */
int tpe_merge_results_device(tpe_ctx *ctx, const tpe_label_result *d_parts, int32_t n_parts,
                             int32_t n, tpe_label_result *d_out);

/* north_star's multi-GPU partition (the reference builds each
 * label's posterior once per suggest call, tpe.py:678-692, and the ranks here
 * split that work): a rank builds the posterior and expansion index of the
 * labels it owns (tpe_build_posterior_resident* over its label shard, each
 * spec carrying its TPE_HAS_STREAM space index), exports them as one device
 * blob, the ranks all-gather the blobs over RCCL, and each imports the
 * assembled posterior of every label to score its slice of the candidates
 * (cand_offset) -- the slices' winners merge with tpe_merge_results_device.
 *
 * tpe_export_posterior: the resident posterior, with its expansion index
 * (queued first when the context's screen would build one), into d_out on
 * this context's GPU.  *bytes receives the blob size; d_out NULL or cap
 * smaller than it is a size query (nothing written).  Complete on return.
 *
 * tpe_import_posterior: replace the resident posterior with the labels of
 * n_parts blobs in d_blobs (blob_bytes long; part p at part_off[p], a
 * multiple of 256, holding part_labels[p] labels).  label_ids lists, part
 * by part, the space index of each blob label: together a permutation of
 * 0..L-1, L = sum part_labels; imported label label_ids[i] is the resident
 * label of that index.  The records, sampling records and index come over
 * device to device (one copy kernel); rounds on the result are the rounds of
 * one context that built every label.  Complete on return.  The built
 * mixtures are not imported (tpe_get_mixture refuses until the next build). */
int tpe_export_posterior(tpe_ctx *ctx, void *d_out, int64_t cap, int64_t *bytes);
int tpe_import_posterior(tpe_ctx *ctx, const void *d_blobs, int64_t blob_bytes, const int64_t *part_off,
                         int32_t n_parts, const int32_t *part_labels, const int32_t *label_ids);

/* Score a caller-supplied candidate set for one resident label (the parity
 * entry point: identical candidates in, both lpdf vectors and the winner
 * out).  lpdf_below / lpdf_above may be NULL. */
int tpe_score(tpe_ctx *ctx, int32_t label, const double *cand, int64_t n,
              double *lpdf_below, double *lpdf_above, tpe_label_result *out);

/* Merge per-shard winners (e.g. gathered from every GPU over RCCL) with the
 * broadcast_best comparator: larger score, NaN greatest, then lowest global
 * index.  parts: n_parts blocks of n results each.  Host-only, no ctx. */
int tpe_merge_results(const tpe_label_result *parts, int32_t n_parts, int32_t n,
                      tpe_label_result *out);

/* Device time (ms, HIP events on the context stream) of the last fused round:
 * scoring kernels only, and the whole round including the reduction. */
int tpe_last_timing(const tpe_ctx *ctx, float *score_ms, float *round_ms);

/* Number of (candidate, component) lpdf evaluations the last round executed,
 * counted over both mixtures (categorical: 2 per candidate). */
int64_t tpe_last_evals(const tpe_ctx *ctx);

/* Per kernel family of the last round (index: 0 dense GMM1, 1 dense LGMM1,
 * 2 quantized GMM1, 3 quantized LGMM1, 4 categorical): device ms of that
 * family's launch and the evaluations it executed.  Arrays of 5.  Sampled
 * tile/packed rounds launch both dense families together: slot 0 then holds
 * the GMM1 + LGMM1 launch and its evaluations, slot 1 stays 0. */
int tpe_last_mode_stats(const tpe_ctx *ctx, float *ms, int64_t *evals);

/* Candidates the last round screened in fp32 (sampled tile-map rounds of
 * the dense GMM1/LGMM1 labels, TPE_F64 contexts) and how many of them it
 * re-scored in fp64 -- those whose rigorous fp32 error interval reaches the
 * largest lower bound of their round; the winner and its lpdfs are those
 * of the plain fp64 round (tpe_device.h screen_err).  screen_ms: device
 * time of the fp32 screening kernel alone (HIP events). */
int tpe_last_screen(const tpe_ctx *ctx, int64_t *screened, int64_t *rescored,
                    float *screen_ms);

/* (candidate, component) terms the last round's screen actually summed
 * (both mixtures).  The windowed screen (TPE_OPT_WINDOW) leaves out the
 * components whose terms stay below 2^-T (TPE_OPT_WIN_T) of the largest
 * coefficient over a whole tile; the plain screen sums them all (then this
 * is screened x (nb + na)).  Winners are unaffected. */
int tpe_last_screen_terms(const tpe_ctx *ctx, int64_t *terms);

/* (candidate, component) terms the last round's fp64 re-score evaluated:
 * every re-scored candidate over both mixtures of its label (the exact
 * GMM1_lpdf / LGMM1_lpdf of tpe.py:110-172,265-307 on that candidate).
 * With tpe_last_screen_terms this is the dense work the round executed. */
int tpe_last_rescore_terms(const tpe_ctx *ctx, int64_t *terms);

/* Candidates the last round actually drew for its quantized and categorical
 * labels (TPE_OPT_EARLY: the exact early exit stops a label's round once a
 * candidate holds the best score any draw can have; the rest are never
 * drawn).  The categorical evals in tpe_last_mode_stats count these. */
int tpe_last_drawn(const tpe_ctx *ctx, int64_t *quantized, int64_t *categorical);

/* Device memory the library holds right now, over every context of the
 * process (posteriors, resident histories, expansion indexes, round
 * buffers; the HIP runtime's own allocations not included), in bytes.
 * Buffers grow by 1/4 and are kept between calls, so after a run this is
 * its high-water mark. */
int64_t tpe_device_bytes(void);

/* Which screen the last round's dense tile-map labels went through: 0 none
 * (unscreened fp64, fp32 precision, or no dense tile round), 1 the plain
 * fp32 screen, 2 the windowed fp32 screen, 3 the expansion screen
 * (TPE_OPT_EXPAND); packed-map rounds report 3 when the expansion screen
 * ran, else 0. */
int32_t tpe_last_screen_mode(const tpe_ctx *ctx);

/* The hot-bin prefilter of the last round's expansion screen (TPE_OPT_HOT):
 * the candidates it listed for the expansion screen (-1: it did not run) --
 * the others were proven unable to win from their sub-bin's score interval
 * (tpe_device.h "hot-bin prefilter") -- and whether the round fell back to
 * screening every candidate (1: a round's best lower bound stayed below the
 * listing threshold).  Winners are unaffected either way. */
int tpe_last_hot(const tpe_ctx *ctx, int64_t *listed, int32_t *fallback);

/* Device milliseconds (HIP events; TPE_OPT_TIMING on) of the last build of
 * the expansion screen's index -- bin tables, lists and the prefilter's
 * sub-bin bounds -- which runs once per posterior, before its first large
 * sampled round or in tpe_prepare (0 if it has not run).  Waits for the
 * index if it is still running. */
int tpe_last_prepare(tpe_ctx *ctx, float *ms);

/* Diagnostic of the hot-bin prefilter (tests): for caller-supplied
 * candidates of one dense resident label, the interval [lower, upper] of
 * the fp64 score over each candidate's sub-bin (+inf / -inf outside the
 * bins): lower <= lpdf_below - lpdf_above <= upper of tpe_score; mass: the
 * sub-bin's sampling mass under the below mixture (0 outside). */
int tpe_hot_probe(tpe_ctx *ctx, int32_t label, const double *cand, int64_t n,
                  double *upper, double *lower, double *mass);

/* Diagnostic of the screen (tests): for caller-supplied candidates of one
 * dense resident label, the fp32 score lpdf_below - lpdf_above the screen
 * computes and its rigorous error bound (x 1.25, as used by the round):
 * |score32 - score64| <= err_bound for every finite bound.  With
 * TPE_OPT_WINDOW on and n >= 2048 the candidates go through the windowed
 * screen (sorted into tiles of neighbours, windows of components); with
 * TPE_OPT_EXPAND on, n >= 2048 and an eligible posterior, through the
 * expansion screen (score and bound in fp64). */
int tpe_screen_probe(tpe_ctx *ctx, int32_t label, const double *cand, int64_t n,
                     double *score32, double *err_bound);

/* Engine options (defaults in brackets):
 *   TPE_OPT_SCREEN  fp32 screen + fp64 re-score of sampled tile rounds [1]
 *   TPE_OPT_SPLITK  split-K map for small sampled rounds                [1]
 *   TPE_OPT_DEDUP   quantized labels scored once per grid value         [1]
 *   TPE_OPT_CHUNKS  chunks of the packed map's above mixtures (0 auto)  [0]
 *   TPE_OPT_WINDOW  windowed screen of large tile rounds: candidates sorted
 *                   into tiles of neighbours, each summed over the window of
 *                   components that can matter to it                   [1]
 *   TPE_OPT_WIN_T   the windowed screen's cut T: components left out of a
 *                   tile stay below 2^-T of the largest term (8..62)    [16]
 *   TPE_OPT_EXPAND  expansion screen of large tile rounds (taken before the
 *                   windowed one when every dense label qualifies): the
 *                   above mixture's equal-sigma components as a per-bin
 *                   Taylor polynomial in fp64, bounds ~1e-12, no sort   [1]
 *   TPE_OPT_HOT     hot-bin prefilter of the expansion screen: every
 *                   candidate is drawn and bounded by its sub-bin's score
 *                   interval; only those that can still win are scored
 *                   (2: tests -- a listing threshold no candidate reaches,
 *                   so every round takes the fallback)                  [1]
 *   TPE_OPT_EARLY   exact early exit of sampled tile rounds of quantized
 *                   (bounded) and categorical labels: candidates in index
 *                   order, stopped once one holds the best score any draw
 *                   can have (its first index is the np.argmax winner)  [1]
 *   TPE_OPT_HOT_DIV the hot-bin prefilter's lists hold n / HOT_DIV
 *                   candidates per (round, label) (at least 4096); a round
 *                   whose list overflows screens every candidate instead
 *                   and divides HOT_DIV by 4 for the next rounds        [16]
 *   TPE_OPT_ZERO_WIN  the packed map's fp64 re-score sums only the above
 *                   components whose terms can be nonzero at the wave's
 *                   candidates (the others are exactly +0.0: the same
 *                   bits)                                                 [1]
 *   TPE_OPT_VALUE_ONLY  packed-map rounds (batched small rounds) report
 *                   only the winner's index and value for a (round, label)
 *                   whose screen selected one candidate clearing every
 *                   other's upper bound by 1e-9 (relative): no fp64 lpdfs
 *                   are computed for it (score, lpdf_below, lpdf_above NaN);
 *                   the same index and value as the exact round.  For
 *                   callers that read the value only (tpe.suggest); not for
 *                   shards whose winners are merged by score            [0]
 *   TPE_OPT_RESCORE_CAP  candidates the packed map's re-score buffers hold
 *                   (grown when a round lists more: that round runs again;
 *                   tests set it small to take that path)               [65536]
 *   TPE_OPT_MODE_MASK  bit m set: rounds launch the labels of family m
 *                   (tpe_last_mode_stats' index: 1 | 2 dense, 4 | 8
 *                   quantized, 16 categorical); the other labels' result
 *                   entries are unspecified and their families' statistics
 *                   stay those of the round that last ran them.  Lets a
 *                   caller run the dense labels while the host still
 *                   computes the quantized labels' tie orders, then those
 *                   after their rebuild (posterior.py)                 [31]
 *   TPE_OPT_AUX_FAMILIES  sampled rounds run the quantized and categorical
 *                   labels on the context's second stream, beside the dense
 *                   labels' draw (joined before the reduction; results
 *                   unchanged; single-device contexts).  Their early exit's
 *                   draw counts (tpe_last_drawn, the families' evals) are
 *                   those of a scan in index order either way              [0]
 *   TPE_OPT_BX_SPLIT  workgroups per 64-bin block of the expansion index's
 *                   Taylor tables, each summing one part of the bins' window
 *                   (k_bx_table / k_bx_table_fin; 1..8, 0: enough for ~8192
 *                   workgroups)                                            [0]
 *   TPE_OPT_BX_T    the expansion index's window cut T (components left
 *                   out stay below 2^-T of the largest term; 32..128; 0:
 *                   64)                                                   [0]
 *   TPE_OPT_PK_SLICED  a packed-map round re-scores up to this many listed
 *                   candidates one wave per (64 candidates, summation slice)
 *                   instead of one thread per candidate walking its chunk
 *                   (same bits; 0: never; at most 65536)                [8192]
 *   TPE_OPT_DEFER_REPORT  1: the next tpe_rebuild_labels of quantized /
 *                   categorical labels only (run on the second stream
 *                   beside the expansion index) returns without waiting
 *                   for its report: its ties output is zeros, the next
 *                   round applies the report after queuing the dense
 *                   labels' kernels, any other call on the context first;
 *                   tpe_build_report then returns the real tie report
 *                   (single-device contexts; consumed by that rebuild)  [0]
 *   TPE_OPT_LABEL_SHARDS  multi-device contexts: the resident history's
 *                   labels partitioned over the devices (each device
 *                   appends, builds, indexes and runs whole rounds of its
 *                   labels; winners scattered to their space positions)
 *                   from the next tpe_history_reset with at least one label
 *                   per device; 0: every device holds every label and the
 *                   rounds split by candidates / rounds                  [1]
 *   TPE_OPT_WIN_GROUPS  label groups of a windowed round, each sorted on a
 *                   second stream while the previous one is screened
 *                   (0: one group; the chip is busy either way)          [0]
 *   TPE_OPT_TIMING  HIP-event timing of every round (tpe_last_timing,
 *                   tpe_last_mode_stats, tpe_last_screen's ms); off saves
 *                   ~20 event calls per round on latency-bound calls   [1]
 *   TPE_OPT_WHOLE_N, TPE_OPT_WHOLE_ROUNDS  the whole problem's candidates
 *                   per round / rounds when this context computes one shard
 *                   of it (one process per GPU); map choices that change a
 *                   summation order follow the whole problem, so the merged
 *                   shards equal one context's round bit for bit     [0: this call's]
 * None of them changes a winner; they exist for tests, experiments and
 * sharded runs (TPE_OPT_VALUE_ONLY drops the lpdfs a caller does not read). */
#define TPE_OPT_SCREEN 1
#define TPE_OPT_SPLITK 2
#define TPE_OPT_DEDUP 3
#define TPE_OPT_CHUNKS 4
#define TPE_OPT_WHOLE_N 5
#define TPE_OPT_WHOLE_ROUNDS 6
#define TPE_OPT_TIMING 7
#define TPE_OPT_WINDOW 8
#define TPE_OPT_WIN_T 9
#define TPE_OPT_WIN_GROUPS 10
#define TPE_OPT_EXPAND 11
#define TPE_OPT_HOT 12
#define TPE_OPT_EARLY 13
#define TPE_OPT_HOT_DIV 14
#define TPE_OPT_ZERO_WIN 15
#define TPE_OPT_VALUE_ONLY 16
#define TPE_OPT_RESCORE_CAP 17
#define TPE_OPT_MODE_MASK 18
#define TPE_OPT_AUX_FAMILIES 19
/* (20: TPE_OPT_HOT32, the fp32 draw kernel -- measured slower, removed in round 6) */
#define TPE_OPT_BX_SPLIT 21
#define TPE_OPT_BX_T 22
#define TPE_OPT_PK_SLICED 23
#define TPE_OPT_DEFER_REPORT 24
#define TPE_OPT_LABEL_SHARDS 25
int tpe_set_option(tpe_ctx *ctx, int32_t option, int64_t value);

/* Build now what the resident posterior's first round(s) of n_candidates
 * per label (n_rounds of them: tpe_suggest_batch) would build lazily: the
 * expansion screen's index (bin tables, lists, sub-bin bounds; fp64
 * contexts with the screen and TPE_OPT_EXPAND on, n_candidates x n_rounds
 * >= 8192; otherwise nothing) and, for rounds of >= 8192 candidates, the
 * hot-bin prefilter's threshold.  Lets a caller overlap the
 * index with host work (tpe.suggest computes numpy's tie orders meanwhile).
 * A later rebuild of the posterior that leaves every dense label
 * bit-identical keeps the index (compared on the device against a snapshot).
 * No reference counterpart: the reference has no index. */
int tpe_prepare(tpe_ctx *ctx, int64_t n_candidates, int32_t n_rounds);

/* Arm tpe_prepare(n_candidates, n_rounds) for the next device build of the
 * resident history (tpe_build_posterior_resident[_ordered], not a
 * label-subset rebuild): that build queues the index itself, right after its
 * own sync and before it returns -- tpe_prepare's work without the caller's
 * round trip between the two calls.  Every such build consumes the arm,
 * whether or not it queued anything (and a failed build queues nothing);
 * n_candidates = 0 disarms.  A tpe_prepare after it is a no-op.  No
 * reference counterpart (tpe.suggest's fresh posterior every step). */
int tpe_arm_prepare(tpe_ctx *ctx, int64_t n_candidates, int32_t n_rounds);

#ifdef __cplusplus
}
#endif

#endif /* HYPEROPT_TPE_H */
