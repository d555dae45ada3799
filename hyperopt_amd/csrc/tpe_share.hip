// tpe_share.hip -- the resident posterior and its expansion index as one
// device blob (tpe_export_posterior), and a posterior assembled from the
// blobs of several contexts (tpe_import_posterior): north_star's multi-GPU
// partition -- each rank builds the posterior and the index of
// the labels it owns once (a label-sharded fmin step), ONE all-gather shares
// those descriptors device to device, and every rank then scores its slice
// [r C/N, (r+1) C/N) of every label's candidates against the assembled
// posterior; the candidate shards' winners merge in broadcast_best's order
// (tpe.py:769-778).  Labels are independent in the reference (one
// build_posterior_wrapper + broadcast_best per label, tpe.py:678-692), so
// the assembled posterior is the one a single context holding every label
// would build: the same records, index and Philox streams, bit for bit.
//
// Blob layout (every section 256-byte aligned): ShareHeader, DLabel[L],
// BxLabel[L] (when the index exists), records fp64 / fp32 and sampling
// records over the label's offsets, then the index's bin tables, list counts,
// lists, unclipped-component ids and sub-bin bounds / masses.  The record and
// table offsets inside DLabel / BxLabel are the exporter's; the importer
// rebases them per part on the host (the headers and label records come to
// the host once) and moves every section with ONE copy kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hyperopt_tpe.h"
#include "tpe_ctx.h"
#include "tpe_device.h"

using namespace tpe;
using tpe_rt::kBlock;

namespace {

constexpr uint64_t kShareMagic = 0x31534f5045505455ull;   // "UTPEPOS1"
constexpr int kSections = 11;
enum { S_LAB, S_BX, S_C64, S_C32, S_SAMP, S_TAB, S_LOFF, S_LIST, S_NC, S_SB, S_SBP };

struct ShareHeader {
    uint64_t magic;
    int64_t n_labels, n_comps, n_samp, rows, lsum, bx_ok;
    int64_t off[kSections];   // section offsets from the blob start
    int64_t bytes[kSections];
    int64_t total;
    int64_t pad[2];
};
static_assert(sizeof(ShareHeader) % 16 == 0, "header");

int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }

// the blob's layout for the resident posterior (host metadata only)
ShareHeader share_layout(const tpe_rt::Posterior& P) {
    ShareHeader h{};
    h.magic = kShareMagic;
    h.n_labels = P.n_labels;
    for (const DLabel& d : P.h_labels) {
        h.n_comps = std::max<int64_t>({h.n_comps, d.comp_b + d.nb, d.comp_a + d.na});
        h.n_samp = std::max<int64_t>(h.n_samp, d.samp_off + d.ns);
    }
    // (no dense label: an index vacuously, as the full posterior's would hold)
    const bool dense = !P.h_group[DENSE_GMM].empty() || !P.h_group[DENSE_LGMM].empty();
    h.bx_ok = (P.bx_ready && (P.bx_ok || !dense)) ? 1 : 0;
    if (P.bx_ok && dense)
        for (int32_t l = 0; l < P.n_labels && l < (int32_t)P.bx_h.size(); ++l) {
            const BxLabel& b = P.bx_h[l];
            if (b.nbins <= 0) continue;
            h.rows = std::max<int64_t>(h.rows, b.tab_off + b.nbins);
            h.lsum = std::max<int64_t>(h.lsum, b.list_off + (int64_t)b.nbins * b.n_nc);
        }
    const int64_t sz[kSections] = {
        h.n_labels * (int64_t)sizeof(DLabel),
        h.bx_ok ? h.n_labels * (int64_t)sizeof(BxLabel) : 0,
        h.n_comps * (int64_t)sizeof(Comp<double>),
        h.n_comps * (int64_t)sizeof(Comp<float>),
        h.n_samp * (int64_t)sizeof(SampRec),
        h.rows * kBxRow * (int64_t)sizeof(double),
        h.rows * (int64_t)sizeof(int32_t),
        h.lsum * (int64_t)sizeof(int32_t),
        h.rows > 0 ? h.n_comps * (int64_t)sizeof(int32_t) : 0,
        h.rows * kBxSub * (int64_t)sizeof(float2),
        h.rows * kBxSub * (int64_t)sizeof(float)};
    int64_t o = align256(sizeof(ShareHeader));
    for (int s = 0; s < kSections; ++s) {
        h.off[s] = o;
        h.bytes[s] = sz[s];
        o = align256(o + sz[s]);
    }
    h.total = o;
    return h;
}

struct CopyTask {
    const uint32_t* src;
    uint32_t* dst;
    int64_t words;
};

// grid (blocks per task, tasks): task y copied by the workgroups of row y
__global__ __launch_bounds__(kBlock) void k_copy_tasks(const CopyTask* __restrict__ tasks) {
    const CopyTask t = tasks[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < t.words; i += (int64_t)gridDim.x * kBlock)
        t.dst[i] = t.src[i];
}

int run_copies(tpe_ctx* ctx, const std::vector<CopyTask>& tasks, tpe_rt::DevBuf<CopyTask>& dev,
               tpe_rt::PinVec<CopyTask>& pin) {
    std::vector<CopyTask> t;
    int64_t mx = 1;
    for (const CopyTask& c : tasks)
        if (c.words > 0) {
            t.push_back(c);
            mx = std::max(mx, c.words);
        }
    if (t.empty()) return TPE_OK;
    HIPCHK(ctx, pin.resize(t.size()));
    std::memcpy(pin.data(), t.data(), t.size() * sizeof(CopyTask));
    HIPCHK(ctx, dev.reserve(t.size()));
    HIPCHK(ctx, hipMemcpyAsync(dev.p, pin.data(), t.size() * sizeof(CopyTask), hipMemcpyHostToDevice, ctx->stream));
    const unsigned gx = (unsigned)std::min<int64_t>((mx + kBlock - 1) / kBlock, 64);
    hipLaunchKernelGGL(k_copy_tasks, dim3(gx, (unsigned)t.size()), dim3(kBlock), 0, ctx->stream, dev.p);
    return ctx->hip(hipGetLastError(), "posterior copy launch");
}

struct ShareScratch {
    tpe_rt::DevBuf<CopyTask> tasks;
    tpe_rt::PinVec<CopyTask> tasks_h;
    tpe_rt::PinVec<uint8_t> stage;
};

ShareScratch& scratch(tpe_ctx* ctx) {
    if (!ctx->share) ctx->share = std::make_shared<ShareScratch>();
    return *std::static_pointer_cast<ShareScratch>(ctx->share);
}

}  // namespace

extern "C" {

int tpe_export_posterior(tpe_ctx* ctx, void* d_out, int64_t cap, int64_t* bytes_out) {
    if (!ctx || !bytes_out) return TPE_ERR_ARG;
    TPE_NOT_LSHARD(ctx);
    TPE_SETTLE(ctx);
    if (!ctx->peers.empty()) return ctx->fail(TPE_ERR_ARG, "tpe_export_posterior: single-device contexts only");
    tpe_rt::Posterior& P = ctx->resident;
    if (P.n_labels <= 0) return ctx->fail(TPE_ERR_ARG, "tpe_export_posterior: no resident posterior");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    ctx->P = &ctx->resident;
    // the index of the coming large rounds: the exporter's own (queued now if not yet built)
    if (!P.bx_ready && ctx->screen && ctx->expand && ctx->precision == TPE_F64) {
        const int rc = tpe_rt::bx_prepare(ctx);
        if (rc) return rc;
    }
    const ShareHeader h = share_layout(P);
    *bytes_out = h.total;
    if (!d_out || cap < h.total) return TPE_OK;   // (a size query)
    uint8_t* o = (uint8_t*)d_out;
    ShareScratch& S = scratch(ctx);
    // the header and the label index records from the host (the device's
    // BxLabel array is absent when the space has no dense label)
    const size_t nbx = (size_t)h.bytes[S_BX];
    HIPCHK(ctx, S.stage.resize(sizeof(ShareHeader) + nbx));
    std::memcpy(S.stage.data(), &h, sizeof(ShareHeader));
    if (nbx) {
        // (the dense labels' records of a built index; zero elsewhere -- bx_h
        // is not rewritten by a build without dense labels)
        BxLabel* sb = reinterpret_cast<BxLabel*>(S.stage.data() + sizeof(ShareHeader));
        for (int32_t l = 0; l < P.n_labels; ++l) {
            const int m = P.h_labels[l].mode;
            sb[l] = (h.rows > 0 && (m == DENSE_GMM || m == DENSE_LGMM) && P.bx_h.size() == (size_t)P.n_labels)
                        ? P.bx_h[l] : BxLabel{};
        }
        HIPCHK(ctx, hipMemcpyAsync(o + h.off[S_BX], S.stage.data() + sizeof(ShareHeader), nbx, hipMemcpyHostToDevice,
                                   ctx->stream));
    }
    HIPCHK(ctx, hipMemcpyAsync(o, S.stage.data(), sizeof(ShareHeader), hipMemcpyHostToDevice, ctx->stream));
    // every section read from a buffer that holds it (checked: a layout
    // beyond a buffer is refused, never copied)
    std::vector<CopyTask> t;
    bool fits = true;
    auto task = [&](int s, const auto& buf) {
        if (h.bytes[s] <= 0) return;
        if (!buf.p || (size_t)h.bytes[s] > buf.cap * sizeof(*buf.p)) {
            fits = false;
            return;
        }
        t.push_back(CopyTask{(const uint32_t*)buf.p, (uint32_t*)(o + h.off[s]), h.bytes[s] / 4});
    };
    task(S_LAB, P.labels);
    task(S_C64, P.comps64);
    task(S_C32, P.comps32);
    task(S_SAMP, P.samp);
    if (h.bx_ok) {
        task(S_TAB, P.bx_tab);
        task(S_LOFF, P.bx_loff);
        task(S_LIST, P.bx_list);
        task(S_NC, P.bx_nc);
        task(S_SB, P.bx_sb);
        task(S_SBP, P.bx_sbp);
    }
    if (!fits) {
        (void)hipStreamSynchronize(ctx->stream);   // (the staged header copies)
        return ctx->fail(TPE_ERR_ARG, "tpe_export_posterior: a section exceeds its buffer");
    }
    int rc = run_copies(ctx, t, S.tasks, S.tasks_h);
    if (rc) return rc;
    // complete on return: the caller's collective reads the blob on another stream
    return ctx->hip(hipStreamSynchronize(ctx->stream), "posterior export");
}

int tpe_import_posterior(tpe_ctx* ctx, const void* d_blobs, int64_t blob_bytes, const int64_t* part_off,
                         int32_t n_parts, const int32_t* part_labels, const int32_t* label_ids) {
    if (!ctx || !d_blobs || !part_off || n_parts <= 0 || !part_labels || !label_ids) return TPE_ERR_ARG;
    TPE_NOT_LSHARD(ctx);
    TPE_SETTLE(ctx);
    if (!ctx->peers.empty()) return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: single-device contexts only");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const uint8_t* blobs = (const uint8_t*)d_blobs;
    int32_t L = 0;
    for (int32_t p = 0; p < n_parts; ++p) {
        if (part_labels[p] < 0) return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: negative label count");
        L += part_labels[p];
    }
    if (L <= 0) return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: no labels");
    std::vector<char> seen(L, 0);
    for (int32_t i = 0; i < L; ++i) {
        if (label_ids[i] < 0 || label_ids[i] >= L || seen[label_ids[i]])
            return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: label ids must be a permutation of 0..L-1");
        seen[label_ids[i]] = 1;
    }
    // each part's header and label / index records to the host (one copy
    // each, one wait): they fit in the first section block
    ShareScratch& S = scratch(ctx);
    const int64_t head = align256(sizeof(ShareHeader)) + align256((int64_t)L * sizeof(DLabel)) +
                         align256((int64_t)L * sizeof(BxLabel));
    std::vector<int64_t> avail(n_parts);
    for (int32_t p = 0; p < n_parts; ++p) {
        avail[p] = blob_bytes - part_off[p];
        if (part_off[p] < 0 || part_off[p] % 256 || avail[p] < (int64_t)sizeof(ShareHeader))
            return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: part " + std::to_string(p) + " offset");
    }
    HIPCHK(ctx, S.stage.resize((size_t)n_parts * head));
    for (int32_t p = 0; p < n_parts; ++p)
        HIPCHK(ctx, hipMemcpyAsync(S.stage.data() + (size_t)p * head, blobs + part_off[p],
                                   std::min(head, avail[p]), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<ShareHeader> hs(n_parts);
    for (int32_t p = 0; p < n_parts; ++p) {
        std::memcpy(&hs[p], S.stage.data() + (size_t)p * head, sizeof(ShareHeader));
        const ShareHeader& h = hs[p];
        if (h.magic != kShareMagic || h.n_labels != part_labels[p])
            return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: part " + std::to_string(p) +
                                              " is not a posterior blob of its label count");
        if (h.off[S_BX] + h.bytes[S_BX] > std::min(head, avail[p]) || h.total > avail[p])
            return ctx->fail(TPE_ERR_ARG, "tpe_import_posterior: part " + std::to_string(p) + " truncated");
    }
    // rebase: part p's records, sampling records, bin rows and list slots
    // follow the earlier parts'
    tpe_rt::Posterior& P = ctx->resident;
    ctx->P = &ctx->resident;
    ctx->build.n_labels = 0;   // (no built mixtures: tpe_get_mixture refuses)
    std::vector<DLabel> dl(L);
    std::vector<BxLabel> bxh(L, BxLabel{});
    bool bx_ok = true;
    int64_t nc = 0, ns = 0, rows = 0, lsum = 0;
    int32_t li0 = 0;
    std::vector<int64_t> cb(n_parts), sbase(n_parts), rb(n_parts), lb(n_parts);
    for (int32_t p = 0; p < n_parts; ++p) {
        const ShareHeader& h = hs[p];
        cb[p] = nc;
        sbase[p] = ns;
        rb[p] = rows;
        lb[p] = lsum;
        bx_ok = bx_ok && h.bx_ok;
        const uint8_t* base = S.stage.data() + (size_t)p * head;
        for (int32_t i = 0; i < part_labels[p]; ++i) {
            const int32_t g = label_ids[li0 + i];
            DLabel d;
            std::memcpy(&d, base + h.off[S_LAB] + (size_t)i * sizeof(DLabel), sizeof(DLabel));
            // each label must keep its space position as its Philox stream
            // (a part built without TPE_HAS_STREAM numbers its labels from 0:
            // its rounds would not be one context's rounds -- ADVICE r5)
            if (d.stream != g)
                return ctx->fail(TPE_ERR_ARG, "import: part " + std::to_string(p) + " label " + std::to_string(i) +
                                                  " has Philox stream " + std::to_string(d.stream) +
                                                  ", its space index is " + std::to_string(g));
            d.comp_b += nc;
            d.comp_a += nc;
            d.samp_off += ns;
            dl[g] = d;
            if (h.bx_ok && (d.mode == DENSE_GMM || d.mode == DENSE_LGMM)) {
                BxLabel b;
                std::memcpy(&b, base + h.off[S_BX] + (size_t)i * sizeof(BxLabel), sizeof(BxLabel));
                if (b.nbins > 0) {
                    b.tab_off += rows;
                    b.cnt_off += rows;
                    b.sb_off += rows * kBxSub;   // (rows: a multiple of 64 bins, so sb_off stays a multiple of 32)
                    b.list_off += lsum;
                }
                bxh[g] = b;
            }
        }
        nc += h.n_comps;
        ns += h.n_samp;
        rows += h.rows;
        lsum += h.lsum;
        li0 += part_labels[p];
    }
    std::vector<int32_t> grp[tpe_rt::kNumModes];
    for (int32_t l = 0; l < L; ++l) grp[dl[l].mode].push_back(l);
    std::vector<int32_t> cat;
    for (int m = 0; m < tpe_rt::kNumModes; ++m) {
        P.group_off[m] = (int32_t)cat.size();
        cat.insert(cat.end(), grp[m].begin(), grp[m].end());
        P.h_group[m] = grp[m];
    }
    HIPCHK(ctx, P.labels.reserve(L));
    HIPCHK(ctx, P.comps64.reserve(std::max<int64_t>(nc, 1)));
    HIPCHK(ctx, P.comps32.reserve(std::max<int64_t>(nc, 1)));
    HIPCHK(ctx, P.samp.reserve(std::max<int64_t>(ns, 1)));
    HIPCHK(ctx, P.groups.reserve(cat.size()));
    if (bx_ok) {
        HIPCHK(ctx, P.bx.reserve(L));
        HIPCHK(ctx, P.bx_tab.reserve((size_t)std::max<int64_t>(rows, 1) * kBxRow));
        HIPCHK(ctx, P.bx_loff.reserve((size_t)std::max<int64_t>(rows, 1)));
        HIPCHK(ctx, P.bx_list.reserve((size_t)std::max<int64_t>(lsum, 1)));
        HIPCHK(ctx, P.bx_nc.reserve(std::max<int64_t>(nc, 1)));
        HIPCHK(ctx, P.bx_sb.reserve((size_t)std::max<int64_t>(rows, 1) * kBxSub));
        HIPCHK(ctx, P.bx_sbp.reserve((size_t)std::max<int64_t>(rows, 1) * kBxSub));
    }
    // the label records and groups (pinned staging), then every section
    const size_t need = L * sizeof(DLabel) + L * sizeof(BxLabel) + cat.size() * sizeof(int32_t);
    HIPCHK(ctx, S.stage.resize(need));
    uint8_t* st = S.stage.data();
    std::memcpy(st, dl.data(), L * sizeof(DLabel));
    std::memcpy(st + L * sizeof(DLabel), bxh.data(), L * sizeof(BxLabel));
    std::memcpy(st + L * (sizeof(DLabel) + sizeof(BxLabel)), cat.data(), cat.size() * sizeof(int32_t));
    HIPCHK(ctx, hipMemcpyAsync(P.labels.p, st, L * sizeof(DLabel), hipMemcpyHostToDevice, ctx->stream));
    if (bx_ok)
        HIPCHK(ctx, hipMemcpyAsync(P.bx.p, st + L * sizeof(DLabel), L * sizeof(BxLabel), hipMemcpyHostToDevice,
                                   ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(P.groups.p, st + L * (sizeof(DLabel) + sizeof(BxLabel)),
                               cat.size() * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    std::vector<CopyTask> t;
    for (int32_t p = 0; p < n_parts; ++p) {
        const ShareHeader& h = hs[p];
        const uint8_t* b = blobs + part_off[p];
        auto add = [&](int s, void* dst) { t.push_back(CopyTask{(const uint32_t*)(b + h.off[s]), (uint32_t*)dst,
                                                                h.bytes[s] / 4}); };
        add(S_C64, P.comps64.p + cb[p]);
        add(S_C32, P.comps32.p + cb[p]);
        add(S_SAMP, P.samp.p + sbase[p]);
        if (bx_ok) {
            add(S_TAB, P.bx_tab.p + rb[p] * kBxRow);
            add(S_LOFF, P.bx_loff.p + rb[p]);
            add(S_LIST, P.bx_list.p + lb[p]);
            add(S_NC, P.bx_nc.p + cb[p]);
            add(S_SB, P.bx_sb.p + rb[p] * kBxSub);
            add(S_SBP, P.bx_sbp.p + rb[p] * kBxSub);
        }
    }
    int rc = run_copies(ctx, t, S.tasks, S.tasks_h);
    if (rc) return rc;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));   // (the pinned staging is reused by the next call)
    int32_t bins_max = 0;
    for (const BxLabel& b : bxh) bins_max = std::max(bins_max, b.nbins);
    P.groups_h = cat;
    P.h_labels = dl;
    P.n_labels = L;
    P.win_ready = false;
    P.zw_ready = false;
    P.qc_ready = false;
    P.bx_ok = bx_ok;
    P.bx_h = bx_ok ? bxh : std::vector<BxLabel>();
    P.bx_sb_max = bx_ok ? (int64_t)bins_max * kBxSub : 0;
    P.bx_snap_nl = 0;    // (no snapshot: a later build replaces the whole posterior)
    P.bx_prescan_ok = false;
    P.bx_ready = true;   // (ineligible parts: the windowed screen runs, as a build would decide)
    P.bx_gen = tpe_rt::next_bx_gen();
    return TPE_OK;
}

}  // extern "C"
