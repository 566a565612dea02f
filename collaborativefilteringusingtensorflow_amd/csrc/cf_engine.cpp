// cf_engine.cpp -- host side of the C ABI declared in include/cf_engine.h.
// Owns the device tables, the HBM-resident interaction graph, the device
// sampler position and the HIP stream; enqueues the gfx950 kernels of
// cf_kernels.hip / cf_eval.hip.  No exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/cf_engine.h"
#include "cf_kernels.h"
#include "cf_device.h"
#include <thread>

using namespace cfk;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define CF_HIP(expr)                                                                  \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess)                                                         \
            return fail(CF_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));  \
    } while (0)

#define CF_TRY(expr)            \
    do {                        \
        int _r = (expr);        \
        if (_r != CF_OK) return _r; \
    } while (0)

template <class T>
int dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) return CF_OK;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess)
        return fail(CF_ENOMEM, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B): " +
                                   hipGetErrorString(e));
    return CF_OK;
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

}  // namespace

// deterministic range flags kept per step (cf_engine::fx_bad)
constexpr int kFxSlots = 1024;

struct cf_engine {
    cf_config cfg{};
    hipStream_t stream = nullptr;
    bool own_stream = false;

    // graph (HBM)
    int64_t nnz = 0;
    int64_t* indptr = nullptr;
    int32_t* indices = nullptr;
    int4* pairs = nullptr;   // (u, i, row start, row length) per interaction
    int4* pf_recs[2] = {nullptr, nullptr};   // prefetched pair records per buffer set (StepArgs::pf_out)
    // speculative negative counts (StepArgs::spec_ph), per buffer set
    int2* spec_ph_[2] = {nullptr, nullptr};
    int* spec_n_[2] = {nullptr, nullptr};
    // cf_set_option "spec_neg": off by default since sorted batches (cfg2
    // 0.3541 -> 0.3511 ms/step off, three runs each, profiles/r05/ab/r05w_*:
    // psort's phantom zeroing costs 3 us, the fused draw no longer gains)
    int spec_neg = 0;
    // deterministic mode on the pos_sort path: fixed-point partials and the
    // users' int64 overflow accumulators (StepArgs::det_fx)
    long long* slotP64 = nullptr;
    unsigned long long* GU64 = nullptr;   // [hot_cap, d] compact rows of users past their slot cap
    int32_t* hotU = nullptr;              // [n_users] a hot user's compact row (psort)
    int* hot_n = nullptr;                 // rows handed out this batch
    int64_t hot_cap = 0;
    unsigned long long* GV64 = nullptr;
    int fx_cap = 0;
    int pf_cap = 0;
    int pair_prefetch = 0;   // measured slower at cfg2 (gradient launch +20 us, draw -2 us): off
    unsigned long long* pos_set = nullptr;  // Pos(u) membership set of (u << 32 | i) keys
    uint64_t pos_mask = 0;
    int neg_check = 0;       // cf_set_option("neg_check"): 1 = Pos(u) set, 0 = CSR row scan
    int64_t nnz_set = 0;     // interactions the set was built from
    int64_t* indptr_t = nullptr;
    int32_t* indices_t = nullptr;
    std::vector<int64_t> h_indptr;
    // sorted batches (round 5, cf_set_option "sorted_batches", default 1):
    // each batch's pairs in pair (CSR) order, so the draw reads its records
    // in ascending order, its users are nearly consecutive (their count
    // atomics share lines) and its row scans stay local.  The batch SET is
    // the epoch bijection's, unchanged.  Two slots: the current epoch's order
    // and the next one's, computed ahead on eo_stream (StepArgs::order)
    // 0 off, 1 on, 2 auto (kSortedAutoBatches batches per epoch and up): the
    // pair records sorted into batch-then-CSR order; 3 on, in the index form
    // (order[] into pairs[]: a quarter of the memory, one more dependent load)
    int sorted_batches = 2;
    bool sorted_auto_off = false;   // auto, and the orders did not fit in HBM (sorted_auto_fits)
    int64_t sorted_reserve_mb = 1024;
    // cf_set_option("epoch_sort"): 0 the counting scatter (cf_epoch.hip) where
    // it applies (<= kEpochMaxBins batches per epoch), 1 the hipCUB radix sort
    int epoch_sort = 0;
    // cf_set_option("user_runs"): sorted batches take user ranks / counts from
    // the batch's user runs (StepArgs::user_runs); 0 (default) = one returning
    // count atomic per pair -- the runs measured even at cfg2 (prep_body)
    int user_runs = 0;
    struct EpochOrder {
        int32_t* keys = nullptr;     // radix-sort path: [2 nnz]
        int32_t* vals = nullptr;     // index form: [nnz] (counting) or [2 nnz] (radix sort)
        void* tmp = nullptr;
        size_t tmp_bytes = 0;
        int64_t keys_cap = 0, vals_cap = 0;
        int64_t epoch = -1;
        int B = 0;
        const int32_t* order = nullptr;
        int4* recs = nullptr;        // records form (sorted_batches 1 / 2): the sorted pair records
        int64_t recs_cap = 0;        // elements, like keys_cap / vals_cap
        const int4* recs_sorted = nullptr;
        bool with_recs = false;
        hipEvent_t ready = nullptr;
        bool async = false;          // computed on eo_stream: the engine stream waits on `ready`
    } eo[2];
    hipStream_t eo_stream = nullptr;
    hipEvent_t eo_mark = nullptr;

    // tables
    float *U = nullptr, *V = nullptr, *b = nullptr;
    float *AU = nullptr, *AV = nullptr, *Ab = nullptr;
    float *GU = nullptr, *GV = nullptr, *Gb = nullptr;
    float *GV_own = nullptr, *Gb_own = nullptr;
    // amf_mode CF_AMF_APR: the batch's summed embedding-loss gradient of every
    // duplicated row (apr_embed_kernel), zero between steps; Δ = epsilon *
    // l2_normalize(row).  Rows seen once take Δ from their own pair.
    float *GadvU = nullptr, *GadvV = nullptr;
    // multi-rank (dense_item_apply): GadvV is the caller's buffer
    // (cf_bind_apr_item_grad), all-reduced between cf_step_local_apr_embed and
    // cf_step_local_grad so every item row's Δ comes from the global batch
    float* GadvV_bound = nullptr;
    int32_t* cntU_[2] = {nullptr, nullptr};  // per-row occurrence counts (0 between steps)
    int32_t* cntV_[2] = {nullptr, nullptr};
    // store-and-sum of duplicated rows: row r of a table owns the fixed slot
    // rows [r*cap, (r+1)*cap) (cf_set_option "slot_max" = item cap,
    // "slot_max_user" = user cap); rows above their cap use float atomics
    float* slotU = nullptr;   // [n_users * capU, d]
    float* slotV = nullptr;   // [n_items * capV, d]
    float* slotVb = nullptr;  // [n_items * capV] item-bias gradient beside each slot row (GBPR / PLR)
    int capU = 2, capV = 32;
    // user cap chosen at the first step from the batch's expected occurrences
    // per user (ensure_batch) until cf_set_option("slot_max_user") sets it
    bool capU_auto = true;
    // item records instead of item slot rows (cf_set_option "item_slots" 1):
    // 16 B per duplicated item occurrence + each pair's pre-update user row
    // (GBPR: its group blend row) stashed once (StepArgs::recV)
    int item_recs = 0;
    int4* recV = nullptr;     // [n_items * capV]
    int4* recVc = nullptr;    // deterministic mode: [B*(1+W)]
    float *stashU = nullptr, *stashB = nullptr;   // [stash_cap, d]
    int stash_cap = 0;
    // hot item rows (occurrences past capV) spread their float atomics over
    // GV and hot_rep - 1 extra copies (cf_set_option "hot_replicas")
    float* GVrep = nullptr;   // [hot_rep - 1][n_items, d]
    int hot_rep = 1;
    // positive-sorted gradient (cf_set_option "pos_sort"): positives counted
    // in cntP, pairs visited in positive-item order, one partial row per
    // (gradient block, positive item) in slotP (StepArgs::cntP)
    int pos_sort = 2;                 // 0 off, 1 on, 2 auto: on for B >= kPsortAutoB
    int capP = 8;                     // partial rows per item (slot_max_pos); later ones add with atomics
    int32_t* cntP_[2] = {nullptr, nullptr};
    int2* offPN = nullptr;            // [n_items + 1] exclusive scans of (positives, negatives) per item
    int32_t* srec = nullptr;          // [order_cap, psort_stride(n_neg)] sorted pair records
    int order_cap = 0;
    float* slotP = nullptr;           // [order_cap / kPsortPPB + 1 + n_items, d] (StepArgs::slotP)
    float* slotN = nullptr;           // [slotN_rows, d] compact negative slot rows (offN[j] + rank)
    int64_t slotN_rows = 0;           // order_cap * n_neg, doubled when speculative counts can apply
    void* psort_tmp = nullptr;
    size_t psort_tmp_bytes = 0;
    bool slots_ready = false;
    // cf_set_option("pipeline") for cf_train_steps: 0 = three launches per
    // step (prep, grad, apply); 1 = apply(s) + prep(s+1) fused (two launches);
    // 2 = grad(s) + prep(s+1) fused, apply(s) alone; 3 = as 2 on the pos_sort
    // path (grad_sort_kernel carries the draw), else as 1
    int pipeline = 1;

    // batch: two buffer sets, so that the sampler of step s+1 runs on the side
    // stream while step s's gradient and apply kernels run on the main stream
    int Bcap = 0;
    int32_t* occU_[2] = {nullptr, nullptr};
    int32_t* occV_[2] = {nullptr, nullptr};
    int32_t* rankU_[2] = {nullptr, nullptr};  // occurrence rank inside its row
    int32_t* rankV_[2] = {nullptr, nullptr};
    int set = 0;
    hipStream_t side = nullptr;
    hipEvent_t prep_done[2] = {nullptr, nullptr};
    hipEvent_t apply_done[2] = {nullptr, nullptr};
    double* loss_partial = nullptr;
    double* loss = nullptr;   // [0] running accumulator, [1] per-call scratch
    float* coefs = nullptr;   // [B, 2] CPLR tuple coefficients (cf_step_plr)
    int coefs_cap = 0;
    double* h_loss = nullptr; // pinned
    // deterministic fixed-point range flags (StepArgs::fx_bad), one word per
    // step since the last check_fx (step k of the call: word min(k, kFxSlots-1)),
    // so a failing call names its first bad step
    int* fx_bad = nullptr;
    int* h_fx_bad = nullptr;  // pinned [kFxSlots]
    int fx_step = 0;
    int32_t* h_stage = nullptr;
    size_t stage_cap = 0;
    int tuple_stride = 0;            // cf_step_plr: ids read from tuples [B, width]
    int32_t* d_bad = nullptr;        // device-batch range check (pack kernel)
    int32_t* h_bad = nullptr;        // pinned
    hipEvent_t stage_ev = nullptr;

    // device sampler position
    int64_t epoch = 0, batch = 0;
    int64_t full_row_user = -1;   // a user with every item as a positive (no negative exists)
    int sampler_B = 0;

    // user sharding + GBPR group exchange (cf_set_shard / cf_bind_exchange /
    // cf_xchg_*): this rank owns global users [shard_u0, shard_u1)
    int world = 1, rank = 0;
    int64_t shard_u0 = 0, shard_u1 = 0;
    std::vector<int64_t> h_bounds;
    int64_t* bounds = nullptr;       // [world + 1] device
    bool group_source_global = false;
    int32_t* xhist = nullptr;        // pack histogram [blocks][world]
    size_t xhist_cap = 0;
    int32_t* xcounts = nullptr;      // [world + 1] device
    int32_t* h_xcounts = nullptr;    // pinned mirror
    int32_t *x_send_ids = nullptr, *x_recv_ids = nullptr;             // bound (caller) buffers
    int32_t* x_own = nullptr;        // [recv cap] served row applies it (first server, no local occurrence)
    float *x_rows = nullptr, *x_grads = nullptr, *x_serve_rows = nullptr, *x_serve_grads = nullptr;
    int64_t x_send_cap = 0, x_recv_cap = 0;
    int x_stage = 0;                 // 0 idle, 1 begun, 2 served, 3 grads done
    int x_part = 0;                  // split step: gradient parts done (1: local-member pairs)
    bool x_items_done = false;       // split step: the items' apply ran (cf_xchg_finish_items)
    // the next exchange batch drawn ahead (cf_xchg_draw), taken by cf_xchg_adopt;
    // send_ids holds two halves of send_cap ids, one per buffer set
    bool x_pend = false;
    StepArgs x_pend_args{};
    int x_pend_set = 0, x_pend_B = 0, x_pend_sampler_B = 0;
    int64_t x_pend_epoch = 0, x_pend_batch = 0;

    // split local step (cf_step_local_grad / cf_step_local_apply): the step
    // between its two halves, and a batch already drawn + counted by the
    // previous apply launch (device sampler), with the sampler position it
    // was drawn from (restored if the draw is discarded)
    int lg_stage = 0;
    StepArgs lg_args{};
    int lg_set = 0, lg_B = 0;
    // the multi-rank item reduce in pieces (cf_set_option "item_pieces"):
    // cf_step_item_reduce(q, P) reduces item rows piece q; lg_pieces_left of
    // the current local step are still to come
    int item_pieces = 1;
    int lg_pieces_left = 0;
    bool lg_pieces_deferred = false;
    bool pend = false;
    StepArgs pend_args{};
    int pend_set = 0, pend_B = 0;
    int64_t pend_epoch = 0, pend_batch = 0;
    int pend_sampler_B = 0;
    StepArgs x_args{};
    int x_set = 0;
    int x_B = 0;

    // tables bound to caller device memory (cf_bind_table): the engine's own
    // buffer of table t while it is bound, else null
    float* own_tab[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    // item occurrences of the last local gradient launch: the rows of the
    // bound item gradient that cf_clear_item_grad re-zeroes
    const int32_t* last_occV = nullptr;
    int64_t last_nV = 0;
    int lg_done_set = -1;     // buffer set of the last cf_step_local_apply

    // deterministic mode (cf_set_option "deterministic"): sort-based ranks,
    // compact slots, no float atomics on duplicated rows (cf_det.hip)
    int det = 0;
    int64_t det_cap = 0;                 // occurrences the buffers below hold
    int32_t *det_keys = nullptr, *det_vals = nullptr, *det_off = nullptr;
    void* det_tmp = nullptr;
    size_t det_tmp_bytes = 0;
    float *slotUc = nullptr, *slotVc = nullptr, *slotVbc = nullptr;
    float *hotP = nullptr, *hotPb = nullptr;   // sums of the 64-slot tiles inside one row

    // model state
    int phase = 0;
    bool need_clip_U = false, need_clip_V = false;

    // eval workspace
    uint32_t* keys = nullptr;
    size_t keys_cap = 0;
    uint64_t* item_mask = nullptr;   // cf_score_topk's caller mask, one bit per item
    int64_t mask_words = 0;

    int topk_path = 0;  // cf_set_option("topk_path")
    int fused_variant = 0;  // cf_set_option("fused_variant")
    int dense_apply = 1;    // cf_set_option("dense_apply"): item-row apply outside pos_sort
    int grad_path = 0;  // cf_set_option("grad_path")
    int item_reduce = 1;  // cf_set_option("item_reduce"): dense mode counts item rows
    int bias_slots = 0;   // cf_set_option("bias_slots"): duplicated item-bias gradients in slots (1) or atomics (0)
    int prep_side = 0;  // cf_set_option("prep_stream"): 1 = side stream (overlap), 0 = main

    // profiling
    bool prof = false;
    uint32_t prof_mask = 0xFFFFFFFFu;  // cf_set_option("profile_mask"): kernel ids timed
    int prof_every = 1;                // cf_set_option("profile_every"): time every n-th launch
    int64_t prof_seen[CF_K_COUNT] = {};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[CF_K_COUNT];
    std::vector<hipEvent_t> ev_pool;
};

namespace {

int set_dev(cf_engine* e) {
    CF_HIP(hipSetDevice(e->cfg.device));
    return CF_OK;
}

struct ProfScope {
    cf_engine* e;
    int k;
    hipStream_t s;
    hipEvent_t a = nullptr, z = nullptr;
    static hipEvent_t get(cf_engine* e) {
        hipEvent_t x = nullptr;
        if (!e->ev_pool.empty()) {
            x = e->ev_pool.back();
            e->ev_pool.pop_back();
        } else if (hipEventCreate(&x) != hipSuccess) {
            x = nullptr;
        }
        return x;
    }
    ProfScope(cf_engine* e_, int k_, hipStream_t s_ = nullptr) : e(e_), k(k_), s(s_) {
        if (!e->prof || !((e->prof_mask >> k) & 1)) return;
        // sampled launches only; the once-per-epoch order is always timed, so
        // a count of its launches is exact (bench.py charges the rest)
        if (e->prof_seen[k]++ % e->prof_every != 0 && k != CF_K_EPOCH_ORDER) return;
        if (!s) s = e->stream;
        a = get(e);
        z = get(e);
        if (a) (void)hipEventRecord(a, s);
    }
    ~ProfScope() {
        if (!a || !z) return;
        (void)hipEventRecord(z, s);
        e->ev[k].emplace_back(a, z);
    }
};

bool has_bias(const cf_config& c) { return c.model == CF_GBPR || c.model == CF_PLR; }
int users_per_pair(const cf_config& c) { return c.model == CF_GBPR ? 1 + c.gsize : 1; }
int items_per_pair(const cf_config& c) { return 1 + c.n_neg; }
int group_count(const cf_config& c) { return c.model == CF_GBPR ? c.gsize : 0; }

// pos_sort applies: BPR / AMF / CML steps on the phased gradient kernel
// (must agree with fast_w() in cf_kernels.hip) and none of the modes it does
// not combine with
// auto pos_sort from this batch size up: below it the sort launches cost more
// than the fewer duplicate rows save (cfg2 A/B: -7 % at 2^19, -3.5 % at 2^18,
// even at 2^17)
constexpr int kPsortAutoB = 1 << 18;

// the engine's model / shape / slot form can take pos_sort (its buffers are
// allocated only then)
bool psort_possible(const cf_engine* e) {
    const cf_config& c = e->cfg;
    if (!e->pos_sort || e->item_recs || c.amf_mode == CF_AMF_APR) return false;   // apr: generic kernel
    if (c.dense_item_apply && e->item_reduce != 1) return false;   // the multi-rank item reduce: slot rows only
    if (c.model != CF_BPR && c.model != CF_AMF && c.model != CF_CML) return false;
    if ((int64_t)c.n_users * e->capU > INT32_MAX) return false;   // user slot rows ride in int32 records
    return c.n_factors <= 128 && (c.n_neg == 1 || c.n_neg == 5);
}

bool psort_active(const cf_engine* e, int B) {
    const cf_config& c = e->cfg;
    // deterministic mode keeps pos_sort (fixed-point sums, StepArgs::det_fx,
    // DESIGN 3.9) except on the multi-rank item reduce
    if (!psort_possible(e) || (e->pos_sort == 2 && B < kPsortAutoB) || (e->det && c.dense_item_apply) ||
        e->hot_rep > 1 ||
        e->neg_check == 2 || e->pipeline == 2)
        return false;
    if (e->grad_path == 1 || (e->grad_path == 0 && c.model == CF_CML && c.n_neg == 5)) return false;
    return true;
}

int ensure_slots(cf_engine* e) {
    if (e->slots_ready) return CF_OK;
    const cf_config& c = e->cfg;
    CF_HIP(hipStreamSynchronize(e->stream));
    dfree(e->slotU);
    dfree(e->slotV);
    dfree(e->slotVb);
    dfree(e->recV);
    dfree(e->GVrep);
    dfree(e->offPN);
    for (int k = 0; k < 2; ++k) dfree(e->cntP_[k]);
    if (e->psort_tmp) (void)hipFree(e->psort_tmp);
    e->psort_tmp = nullptr;
    if (psort_possible(e)) {
        CF_TRY(dalloc(&e->offPN, (size_t)c.n_items + 1));
        for (int k = 0; k < 2; ++k) {
            CF_TRY(dalloc(&e->cntP_[k], (size_t)c.n_items));
            CF_HIP(hipMemsetAsync(e->cntP_[k], 0, (size_t)c.n_items * 4, e->stream));
        }
        e->psort_tmp_bytes = psort_scratch(c.n_items);
        if (e->psort_tmp_bytes) {
            hipError_t he = hipMalloc(&e->psort_tmp, e->psort_tmp_bytes);
            if (he != hipSuccess) return fail(CF_ENOMEM, std::string("hipMalloc (psort scratch): ") + hipGetErrorString(he));
        }
    }
    CF_TRY(dalloc(&e->slotU, (size_t)c.n_users * e->capU * c.n_factors));
    if (!c.dense_item_apply || e->item_reduce == 1) {
        if (e->item_recs)
            CF_TRY(dalloc(&e->recV, (size_t)c.n_items * e->capV));
        else
            CF_TRY(dalloc(&e->slotV, (size_t)c.n_items * e->capV * c.n_factors));
        if (has_bias(c)) CF_TRY(dalloc(&e->slotVb, (size_t)c.n_items * e->capV));
    }
    if (!c.dense_item_apply) {
        if (e->hot_rep > 1) {
            const size_t n = (size_t)(e->hot_rep - 1) * c.n_items * c.n_factors;
            CF_TRY(dalloc(&e->GVrep, n));
            CF_HIP(hipMemsetAsync(e->GVrep, 0, n * sizeof(float), e->stream));
        }
    }
    e->slots_ready = true;
    return CF_OK;
}

// the deterministic step at batch size B takes the fixed-point pos_sort form
// (StepArgs::det_fx), which needs none of the sort-based form's buffers
bool det_fx_path(const cf_engine* e, int B) {
    return e->det && psort_possible(e) && !e->cfg.dense_item_apply && psort_active(e, B);
}

// B: the buffers' capacity (>= the step's batch); B_step: the step's batch,
// which decides the form
int ensure_det(cf_engine* e, int B, int B_step) {
    const cf_config& c = e->cfg;
    if (psort_possible(e) && !c.dense_item_apply) {   // the fixed-point pos_sort form (StepArgs::det_fx)
        if (B > e->fx_cap) {
            CF_HIP(hipStreamSynchronize(e->stream));
            CF_HIP(hipStreamSynchronize(e->side));
            dfree(e->slotP64);
            CF_TRY(dalloc(&e->slotP64, ((size_t)B / kPsortPPB + 1 + (size_t)c.n_items) * c.n_factors));
            // users past their slot cap: at most one per capU + 1 user
            // occurrences of the batch, each one compact int64 row (was one
            // row per user of the table: 512 MB at cfg2, round-3 ADVICE)
            dfree(e->GU64);
            const int64_t hc = (int64_t)B * users_per_pair(c) / (e->capU + 1) + 1;
            CF_TRY(dalloc(&e->GU64, (size_t)hc * c.n_factors));
            CF_HIP(hipMemsetAsync(e->GU64, 0, (size_t)hc * c.n_factors * 8, e->stream));
            e->hot_cap = hc;
            e->fx_cap = B;
        }
        if (!e->hotU) {
            CF_TRY(dalloc(&e->hotU, (size_t)c.n_users));
            CF_TRY(dalloc(&e->hot_n, 1));
            CF_HIP(hipMemsetAsync(e->hot_n, 0, sizeof(int), e->stream));
        }
        if (!e->GV64) {
            CF_TRY(dalloc(&e->GV64, (size_t)c.n_items * c.n_factors));
            CF_HIP(hipMemsetAsync(e->GV64, 0, (size_t)c.n_items * c.n_factors * 8, e->stream));
        }
        if (!e->fx_bad) {
            CF_TRY(dalloc(&e->fx_bad, (size_t)kFxSlots));
            CF_HIP(hipMemsetAsync(e->fx_bad, 0, kFxSlots * sizeof(int), e->stream));
            e->fx_step = 0;
        }
        if (det_fx_path(e, B_step)) return CF_OK;   // the sort-based buffers are not used
    }
    const int64_t nU = (int64_t)B * users_per_pair(c), nV = (int64_t)B * items_per_pair(c);
    const int64_t n = nU + nV;
    if (n <= e->det_cap && e->det_off) return CF_OK;
    CF_HIP(hipStreamSynchronize(e->stream));
    CF_HIP(hipStreamSynchronize(e->side));
    dfree(e->det_keys); dfree(e->det_vals); dfree(e->det_off); dfree(e->slotUc); dfree(e->slotVc);
    dfree(e->slotVbc);
    dfree(e->recVc);
    dfree(e->hotP);
    dfree(e->hotPb);
    if (e->det_tmp) (void)hipFree(e->det_tmp);
    e->det_tmp = nullptr;
    e->det_cap = 0;
    const int64_t rows = c.n_users + c.n_items;
    CF_TRY(dalloc(&e->det_keys, (size_t)(2 * n)));
    CF_TRY(dalloc(&e->det_vals, (size_t)(2 * n)));
    CF_TRY(dalloc(&e->det_off, (size_t)rows));
    CF_TRY(dalloc(&e->slotUc, (size_t)nU * c.n_factors));
    if (e->item_recs)
        CF_TRY(dalloc(&e->recVc, (size_t)nV));
    else
        CF_TRY(dalloc(&e->slotVc, (size_t)nV * c.n_factors));
    if (has_bias(c)) CF_TRY(dalloc(&e->slotVbc, (size_t)nV));
    CF_TRY(dalloc(&e->hotP, (size_t)(n / kDetTile + 1) * c.n_factors));
    CF_TRY(dalloc(&e->hotPb, (size_t)(n / kDetTile + 1)));
    e->det_tmp_bytes = det_ranks_scratch(n, rows);
    if (e->det_tmp_bytes) {
        hipError_t he = hipMalloc(&e->det_tmp, e->det_tmp_bytes);
        if (he != hipSuccess) return fail(CF_ENOMEM, std::string("hipMalloc (sort scratch): ") + hipGetErrorString(he));
    }
    e->det_cap = n;
    return CF_OK;
}

int ensure_stash(cf_engine* e, int B) {
    if (!e->item_recs || B <= e->stash_cap) return CF_OK;
    const cf_config& c = e->cfg;
    CF_HIP(hipStreamSynchronize(e->stream));
    CF_HIP(hipStreamSynchronize(e->side));
    dfree(e->stashU);
    dfree(e->stashB);
    CF_TRY(dalloc(&e->stashU, (size_t)B * c.n_factors));
    if (c.model == CF_GBPR) CF_TRY(dalloc(&e->stashB, (size_t)B * c.n_factors));
    e->stash_cap = B;
    return CF_OK;
}

int ensure_order(cf_engine* e, int B);

int ensure_batch(cf_engine* e, int B) {
    if (e->capU_auto && e->Bcap == 0) {
        // a user occurs Poisson(lam) times in a batch; its occurrences past
        // capU take float atomics and, in deterministic mode, a compact GU64
        // row handed out by ONE counter in psort (one address: ~88 grants per
        // us).  cfg2 at B = 2^19 (lam 0.52): capU 2 -> 16K hot users a step,
        // det psort 29 -> 101 us; capU 4 -> ~200 (det 0.480 -> 0.393 ms/step,
        // fast 0.3542 -> 0.3526, profiles/r05/ab/r05ad_*) for 512 MB more
        // slot rows.  Sparse batches (cfg4, B = 65,536) keep 2.
        const double lam = (double)B * users_per_pair(e->cfg) / (double)e->cfg.n_users;
        const int want = lam >= 0.25 ? 4 : 2;
        if (want != e->capU) {
            e->capU = want;
            e->slots_ready = false;
            e->fx_cap = 0;   // the compact GU64 rows scale with 1 / (capU + 1)
        }
    }
    CF_TRY(ensure_slots(e));
    CF_TRY(ensure_order(e, B));
    if (e->det) CF_TRY(ensure_det(e, std::max(B, e->Bcap), B));
    CF_TRY(ensure_stash(e, std::max(B, e->Bcap)));
    if (B <= e->Bcap) return CF_OK;
    CF_HIP(hipStreamSynchronize(e->stream));
    CF_HIP(hipStreamSynchronize(e->side));
    dfree(e->loss_partial);
    const size_t nU = (size_t)B * users_per_pair(e->cfg);
    const size_t nV = (size_t)B * items_per_pair(e->cfg);
    for (int k = 0; k < 2; ++k) {
        dfree(e->occU_[k]);
        dfree(e->occV_[k]);
        dfree(e->rankU_[k]);
        dfree(e->rankV_[k]);
        CF_TRY(dalloc(&e->occU_[k], nU));
        CF_TRY(dalloc(&e->occV_[k], nV));
        CF_TRY(dalloc(&e->rankU_[k], nU));
        CF_TRY(dalloc(&e->rankV_[k], nV));
    }
    CF_TRY(dalloc(&e->loss_partial, (size_t)grad_blocks_max(B)));
    e->Bcap = B;
    return CF_OK;
}

// speculative negative counts (StepArgs::spec_ph) can apply to a batch of B
// pairs: pos_sort's dense item apply (every item row visited, so a phantom
// holding rank 0 cannot hide an item from an owner rule) -- the same test as
// apply_args' dense_items
// Deterministic mode keeps them off: a phantom raises its item's count, so
// an item whose only real occurrence shares it with a phantom takes the
// summed path -- a fixed-point sum of one term, rounded to 2^-32 -- instead of
// the gradient launch's singleton Adagrad in fp32.  Both are valid steps, but
// the deterministic result must not depend on a performance option (round 5:
// BPR / AMF W = 1 spec on vs off differed in the last bits, deterministically).
bool spec_possible(const cf_engine* e, int64_t B) {
    return e->spec_neg && !e->det && e->cfg.n_items <= 2 * B * items_per_pair(e->cfg);
}

// compact negative slot rows for order_cap pairs: phantoms leave holes in the
// negatives' ranks, so the slots span up to twice the batch's negatives when
// speculative counts can apply -- otherwise B * W rows (round-4 ADVICE: the
// doubled array was ~128 MB never used at cfg2 shapes without spec_neg)
int64_t slotN_need(const cf_engine* e, int64_t cap) {
    return cap * e->cfg.n_neg * (spec_possible(e, cap) ? 2 : 1);
}

int ensure_order(cf_engine* e, int B) {
    if (!psort_possible(e)) return CF_OK;
    if (e->srec && B <= e->order_cap) {
        const int64_t need = slotN_need(e, e->order_cap);
        if (need <= e->slotN_rows) return CF_OK;
        // spec_neg switched on after the allocation: widen the slots only
        CF_HIP(hipStreamSynchronize(e->stream));
        CF_HIP(hipStreamSynchronize(e->side));
        dfree(e->slotN);
        e->slotN_rows = 0;
        CF_TRY(dalloc(&e->slotN, (size_t)need * e->cfg.n_factors));
        e->slotN_rows = need;
        return CF_OK;
    }
    CF_HIP(hipStreamSynchronize(e->stream));
    CF_HIP(hipStreamSynchronize(e->side));
    dfree(e->srec);
    dfree(e->slotN);
    e->slotN_rows = 0;
    dfree(e->slotP);
    for (int q = 0; q < 2; ++q) {
        dfree(e->spec_ph_[q]);
        dfree(e->spec_n_[q]);
    }
    CF_TRY(dalloc(&e->srec, (size_t)std::max(B, e->Bcap) * psort_stride(e->cfg.n_neg)));
    // one partial row per (gradient block, positive item): row block + item
    CF_TRY(dalloc(&e->slotP, ((size_t)std::max(B, e->Bcap) / kPsortPPB + 1 + (size_t)e->cfg.n_items) *
                                 e->cfg.n_factors));
    // compact negative slots offN[j] + rank (slotN_need)
    const int64_t nN = slotN_need(e, std::max(B, e->Bcap));
    CF_TRY(dalloc(&e->slotN, (size_t)nN * e->cfg.n_factors));
    e->slotN_rows = nN;
    // at most one phantom per negative (StepArgs::spec_ph)
    for (int q = 0; q < 2; ++q) {
        CF_TRY(dalloc(&e->spec_ph_[q], (size_t)std::max(B, e->Bcap) * e->cfg.n_neg));
        CF_TRY(dalloc(&e->spec_n_[q], 1));
        CF_HIP(hipMemsetAsync(e->spec_n_[q], 0, sizeof(int), e->stream));
    }
    // in-range ids from the start (a given-up fused scatter leaves old records)
    CF_HIP(hipMemsetAsync(e->srec, 0, (size_t)std::max(B, e->Bcap) * psort_stride(e->cfg.n_neg) * 4, e->stream));
    e->order_cap = std::max(B, e->Bcap);
    return CF_OK;
}

StepArgs base_step_args(cf_engine* e, int B, int k) {
    const cf_config& c = e->cfg;
    StepArgs a{};
    a.model = c.model;
    a.d = c.n_factors;
    a.W = c.n_neg;
    a.G = group_count(c);
    a.B = B;
    a.adversarial = (c.model == CF_AMF && e->phase == 1) ? 1 : 0;
    a.grad_path = e->grad_path;
    a.reg = c.reg;
    a.rho = c.rho;
    a.margin = c.margin;
    a.reg_cov = c.reg_cov;
    a.reg_adv = c.reg_adv;
    if (a.adversarial && c.amf_mode == CF_AMF_APR) {
        a.apr = 1;
        a.epsilon = c.epsilon;
        a.GadvU = e->GadvU;
        a.GadvV = c.dense_item_apply ? e->GadvV_bound : e->GadvV;
        a.apr_global = c.dense_item_apply ? 1 : 0;
    }
    a.use_rank_weight = c.use_rank_weight;
    a.n_items_f = (float)c.n_items;
    a.n_items = c.n_items;
    a.pairs = e->pairs;
    a.indptr = e->indptr;
    a.indices = e->indices;
    a.indptr_t = e->indptr_t;
    a.indices_t = e->indices_t;
    a.pos_set = e->neg_check ? e->pos_set : nullptr;
    a.pos_mask = e->pos_mask;
    a.lane_draw = e->neg_check == 2 ? 1 : 0;
    a.U = e->U; a.AU = e->AU; a.GU = e->GU;
    a.V = e->V; a.AV = e->AV; a.GV = e->GV;
    a.b = e->b; a.Ab = e->Ab; a.Gb = e->Gb;
    a.lr = c.lr;
    a.clip_norm = c.clip_norm;
    a.clip = c.model == CF_CML ? 1 : 0;
    a.occU = e->occU_[k];
    a.occV = e->occV_[k];
    a.cntU = e->cntU_[k];
    a.cntV = e->cntV_[k];
    a.rankU = e->rankU_[k];
    a.rankV = e->rankV_[k];
    a.slotU = e->slotU;
    a.slotV = e->slotV;
    a.slotVb = (has_bias(c) && (e->slotV || e->recV) && e->bias_slots) ? e->slotVb : nullptr;
    a.capU = e->capU;
    a.capV = e->capV;
    a.GVrep = e->GVrep;
    a.repV = e->GVrep ? e->hot_rep - 1 : 0;
    a.loss_partial = e->loss_partial;
    a.count_users = 1;
    a.count_items = (!c.dense_item_apply || e->item_reduce) ? 1 : 0;
    a.items_grad_only = (c.dense_item_apply && e->item_reduce) ? 1 : 0;
    if (c.dense_item_apply && e->item_reduce == 2) a.capV = 0;  // duplicates: float atomics
    const bool ps = psort_active(e, B) && e->cntP_[k] && e->srec && e->order_cap >= B;
    if (e->det && !ps) {   // compact slots at off[row] + rank, no caps, no atomics
        a.offU = e->det_off;
        a.offV = e->det_off + c.n_users;
        a.slotU = e->slotUc;
        a.slotV = e->slotVc;
        a.slotVb = has_bias(c) ? e->slotVbc : nullptr;
        a.capU = a.capV = 1 << 30;
        a.GVrep = nullptr;
        a.repV = 0;
        if (c.dense_item_apply) {   // the item reduce (item_reduce 1): stores, no atomics
            a.count_items = 1;
            a.items_grad_only = 1;
        }
    }
    if (e->item_recs && a.count_items && a.capV > 0) {
        a.recV = e->det ? e->recVc : e->recV;
        a.stashU = e->stashU;
        a.stashB = e->stashB;
    }
    if (ps) {
        a.cntP = e->cntP_[k];
        a.srec = e->srec;
        a.slotP = e->slotP;
        a.slotV = e->slotN;   // negatives: compact slots offN[j] + rank
        a.capP = e->capP;
        // speculative negative counts need the dense item apply of pos_sort
        // (every item row visited: a phantom holding rank 0 cannot hide an
        // item from an owner rule) -- the same test as apply_args
        if (a.count_items && spec_possible(e, B) && e->slotN_rows >= 2 * (int64_t)B * c.n_neg) {
            a.spec_ph = e->spec_ph_[k];
            a.spec_n = e->spec_n_[k];
        }
        if (e->det && e->slotP64 && e->fx_cap >= B && e->GU64 && e->GV64) {
            // deterministic: the fast path's launches, every sum in fixed point
            a.det_fx = 1;
            a.slotP64 = e->slotP64;
            a.GU64 = e->GU64;
            a.hotU = e->hotU;
            a.GV64 = e->GV64;
            a.fx_bad = e->fx_bad + std::min(e->fx_step++, kFxSlots - 1);
        }
    }
    a.shard_u0 = e->shard_u0;
    a.shard_u1 = e->shard_u1;
    a.plr_kind = c.plr_kind;
    a.alpha = c.alpha;
    a.beta = c.beta;
    a.gamma = c.gamma;
    a.train_bias = (c.model == CF_GBPR || (c.model == CF_PLR && c.plr_kind == CF_PLR_CPLR)) ? 1 : 0;
    a.coefs = e->coefs;
    a.xrows = e->x_rows;
    a.xgrads = e->x_grads;
    return a;
}

// sorted batches, auto: the epoch's order costs ~1 ms per 50M pairs (the
// inverse-bijection keys + a radix sort), once per epoch, on a low-priority
// stream beside the steps; same-box A/Bs with the orders on the clock
// (profiles/r05/ab/r05s_*): cfg2 B = 2^19 (95 batches per epoch) 0.3588 ->
// 0.3544 ms/step, B = 65,536 0.0740 -> 0.0724.  Below 16
// batches per epoch the order is mostly the synchronous first one
constexpr int64_t kSortedAutoBatches = 16;
bool sorted_batches_on(const cf_engine* e, int B) {
    if (e->sorted_batches == 0 || e->nnz > INT32_MAX || B < 1) return false;
    if (e->sorted_batches == 2 && e->sorted_auto_off) return false;
    return e->sorted_batches == 1 || e->sorted_batches == 3 || e->nnz / B >= kSortedAutoBatches;
}

// the epoch order's buffers for (nnz, B) and the option values: the counting
// scatter (cf_epoch.hip) writes the result once (records: int4[nnz], index
// form: int32[nnz]) and takes a small histogram scratch; the radix sort
// (more than kEpochMaxBins bins, or cf_set_option("epoch_sort", 1)) needs
// keys int32[2 nnz] and double-buffered values
struct EpochNeed {
    bool counting;
    int64_t keys, vals, recs;   // elements
    size_t tmp;                 // bytes
    double bytes() const { return 4.0 * (double)(keys + vals) + 16.0 * (double)recs + (double)tmp; }
};
EpochNeed epoch_need(const cf_engine* e, int B) {
    const int64_t nnz = e->nnz;
    const bool wr = e->sorted_batches != 3;   // the records form
    EpochNeed n{};
    n.counting = e->epoch_sort == 0 && epoch_count_ok(nnz, B);
    if (n.counting) {
        n.recs = wr ? nnz : 0;
        n.vals = wr ? 0 : nnz;
        n.tmp = epoch_count_scratch(nnz, B);
    } else {
        n.keys = 2 * nnz;
        n.recs = wr ? 2 * nnz : 0;
        n.vals = wr ? 0 : 2 * nnz;
        n.tmp = wr ? epoch_records_scratch(nnz, (int32_t)(nnz / B)) : epoch_order_scratch(nnz, (int32_t)(nnz / B));
    }
    return n;
}

// auto mode only: the two order slots take 2 x epoch_need (32 B per
// interaction in the default records form, 80 B on the radix-sort path).  An
// engine whose tables leave less than that (and a 1 GiB reserve) free keeps
// the unsorted batches -- the same batch sets, in permutation order --
// instead of failing its first step with CF_ENOMEM (the reserve:
// cf_set_option "sorted_auto_reserve_mb")
void free_epoch_orders(cf_engine* e) {
    (void)hipDeviceSynchronize();
    for (auto& o : e->eo) {
        dfree(o.keys);
        dfree(o.vals);
        dfree(o.recs);
        if (o.tmp) (void)hipFree(o.tmp);
        o.tmp = nullptr;
        o.tmp_bytes = 0;
        o.keys_cap = o.vals_cap = o.recs_cap = 0;
        o.epoch = -1;
        o.async = false;
        o.order = nullptr;
        o.recs_sorted = nullptr;
    }
}

bool sorted_auto_fits(cf_engine* e, int B) {
    const EpochNeed n = epoch_need(e, B);
    double more = 0.0;   // what the two slots still have to allocate
    for (const auto& o : e->eo) {
        if (o.keys_cap < n.keys) more += 4.0 * (double)n.keys;
        if (o.vals_cap < n.vals) more += 4.0 * (double)n.vals;
        if (o.recs_cap < n.recs) more += 16.0 * (double)n.recs;
        if (o.tmp_bytes < n.tmp) more += (double)n.tmp;
    }
    if (more == 0.0) return true;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return true;                            // unknown: the allocation decides
    }
    return (double)free_b >= more + (double)e->sorted_reserve_mb * (double)(1 << 20);
}

// grow one buffer of an order slot (the device is synchronised first: the
// old buffer may still be read by a draw or written by the other stream)
template <typename T>
int grow(T** p, int64_t* cap, int64_t need) {
    if (*cap >= need) return CF_OK;
    CF_HIP(hipDeviceSynchronize());
    dfree(*p);
    *cap = 0;
    CF_TRY(dalloc(p, (size_t)need));
    *cap = need;
    return CF_OK;
}

// the order of (epoch, B) in slot k, enqueued on stream st
int compute_epoch_order(cf_engine* e, int k, int64_t epoch, int B, hipStream_t st) {
    cf_engine::EpochOrder& o = e->eo[k];
    const int64_t nnz = e->nnz;
    const bool wr = e->sorted_batches != 3;   // the records form
    const EpochNeed n = epoch_need(e, B);
    CF_TRY(grow(&o.keys, &o.keys_cap, n.keys));
    CF_TRY(grow(&o.vals, &o.vals_cap, n.vals));
    CF_TRY(grow(&o.recs, &o.recs_cap, n.recs));
    if (n.tmp > o.tmp_bytes) {
        CF_HIP(hipDeviceSynchronize());
        if (o.tmp) (void)hipFree(o.tmp);
        o.tmp = nullptr;
        o.tmp_bytes = 0;
        hipError_t he = hipMalloc(&o.tmp, n.tmp);
        if (he != hipSuccess) return fail(CF_ENOMEM, std::string("hipMalloc (epoch order scratch): ") + hipGetErrorString(he));
        o.tmp_bytes = n.tmp;
    }
    const PermKey pk = make_perm_key((uint64_t)nnz, e->cfg.seed, (uint64_t)epoch);
    {
        ProfScope ps(e, CF_K_EPOCH_ORDER, st);
        if (n.counting) {
            CF_HIP(launch_epoch_count(pk, nnz, B, wr ? e->pairs : nullptr, wr ? o.recs : nullptr,
                                      wr ? nullptr : o.vals, o.tmp, o.tmp_bytes, st));
            o.recs_sorted = wr ? o.recs : nullptr;
            o.order = wr ? nullptr : o.vals;
        } else if (wr) {
            CF_HIP(launch_epoch_records(pk, nnz, B, e->pairs, o.keys, o.recs, o.tmp, o.tmp_bytes, &o.recs_sorted, st));
            o.order = nullptr;
        } else {
            CF_HIP(launch_epoch_order(pk, nnz, B, o.keys, o.vals, o.tmp, o.tmp_bytes, &o.order, st));
            o.recs_sorted = nullptr;
        }
        o.with_recs = wr;
    }
    o.epoch = epoch;
    o.B = B;
    o.async = st != e->stream;
    if (o.async) CF_HIP(hipEventRecord(o.ready, st));
    return CF_OK;
}

// the order of the sampler's epoch at batch size B, ready on the engine
// stream; the next epoch's is started on eo_stream
int epoch_order(cf_engine* e, int B, const int32_t** out, const int4** recs_out) {
    if (!e->eo_stream) {
        int lo = 0, hi = 0;
        CF_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        CF_HIP(hipStreamCreateWithPriority(&e->eo_stream, hipStreamNonBlocking, lo));   // lowest priority
        CF_HIP(hipEventCreateWithFlags(&e->eo_mark, hipEventDisableTiming));
        for (auto& o : e->eo) CF_HIP(hipEventCreateWithFlags(&o.ready, hipEventDisableTiming));
    }
    const int64_t ep = e->epoch;
    const bool wr = e->sorted_batches != 3;
    auto have = [&](const cf_engine::EpochOrder& o, int64_t epc) { return o.epoch == epc && o.B == B && o.with_recs == wr; };
    int k = have(e->eo[0], ep) ? 0 : have(e->eo[1], ep) ? 1 : -1;
    if (k < 0) {
        // not computed ahead (first epoch, a jump, another B): in order on the engine stream
        k = have(e->eo[0], ep + 1) ? 1 : 0;
        if (e->eo[k].async) CF_HIP(hipStreamWaitEvent(e->stream, e->eo[k].ready, 0));
        // a draw on the side stream (prep_stream 1) may still read the slot
        CF_HIP(hipEventRecord(e->eo_mark, e->side));
        CF_HIP(hipStreamWaitEvent(e->stream, e->eo_mark, 0));
        CF_TRY(compute_epoch_order(e, k, ep, B, e->stream));
        // the draw that reads it may be launched on the side stream
        // (prep_stream 1, cf_sample): that stream waits for the order too
        CF_HIP(hipEventRecord(e->eo_mark, e->stream));
        CF_HIP(hipStreamWaitEvent(e->side, e->eo_mark, 0));
    } else if (e->eo[k].async) {
        CF_HIP(hipStreamWaitEvent(e->stream, e->eo[k].ready, 0));
        CF_HIP(hipStreamWaitEvent(e->side, e->eo[k].ready, 0));
        e->eo[k].async = false;
    }
    *out = e->eo[k].order;
    *recs_out = e->eo[k].with_recs ? e->eo[k].recs_sorted : nullptr;
    cf_engine::EpochOrder& nx = e->eo[k ^ 1];
    if (!have(nx, ep + 1) && e->nnz / B >= 2) {
        // the next epoch's order, behind everything the engine stream holds
        // so far (the kernels that still read this slot's previous epoch)
        // (and the side stream's draws, prep_stream 1: a wait takes the
        // event's latest record, so one event serves both)
        CF_HIP(hipEventRecord(e->eo_mark, e->stream));
        CF_HIP(hipStreamWaitEvent(e->eo_stream, e->eo_mark, 0));
        CF_HIP(hipEventRecord(e->eo_mark, e->side));
        CF_HIP(hipStreamWaitEvent(e->eo_stream, e->eo_mark, 0));
        CF_TRY(compute_epoch_order(e, k ^ 1, ep + 1, B, e->eo_stream));
    }
    return CF_OK;
}

// position the device sampler for the next batch of B pairs
int sampler_args(cf_engine* e, int B, StepArgs* a) {
    if (!e->pairs) return fail(CF_ESTATE, "no interactions: call cf_set_interactions first");
    if ((int64_t)B > e->nnz) return fail(CF_EINVAL, "batch size exceeds the number of interactions");
    if (e->full_row_user >= 0)   // the reference's rejection loop would never end for this user
        return fail(CF_EINVAL, "user " + std::to_string(e->full_row_user) +
                                   " has every item as a positive; the device sampler cannot draw a negative");
    if (e->sampler_B != B) {
        if (e->sampler_B != 0 && e->batch != 0) {
            e->epoch += 1;
            e->batch = 0;
        }
        e->sampler_B = B;
    }
    const int64_t per_epoch = e->nnz / B;  // int(len(pairs)/batch_size), sampler_ranking.py:25
    if (e->batch >= per_epoch) {
        e->epoch += 1;
        e->batch = 0;
    }
    a->sample = 1;
    a->slot_base = (uint64_t)(e->batch * (int64_t)B);
    a->perm = make_perm_key((uint64_t)e->nnz, e->cfg.seed, (uint64_t)e->epoch);
    a->rng_key = mix64_host(e->cfg.seed ^ mix64_host((uint64_t)e->epoch * 0x9E3779B97F4A7C15ull +
                                                     0x2545F4914F6CDD1Dull));
    if (sorted_batches_on(e, B) && e->sorted_batches == 2 && !sorted_auto_fits(e, B)) e->sorted_auto_off = true;
    if (sorted_batches_on(e, B)) {
        const int32_t* ord = nullptr;
        const int4* recs = nullptr;
        const int rc = epoch_order(e, B, &ord, &recs);
        if (rc == CF_ENOMEM && e->sorted_batches == 2) {
            free_epoch_orders(e);   // auto: unsorted batches from here on
            e->sorted_auto_off = true;
        } else if (rc != CF_OK) {
            return rc;
        } else {
            a->order = ord;   // batch b's pairs at [bB, bB + B), CSR order
            a->order_recs = recs;
            a->user_runs = e->user_runs && group_count(e->cfg) == 0 ? 1 : 0;
        }
    }
    e->batch += 1;
    return CF_OK;
}

static bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable host memory: not an error for us
        return false;
    }
    return attr.type == hipMemoryTypeDevice;
}

// A batch in device memory: de-interleave and range-check on the device,
// then read the check back (one sync; the host path checks on the host).
static int stage_device_batch(cf_engine* e, const int32_t* pairs, const int32_t* negs,
                       const int32_t* groups, int B, int k, hipStream_t st) {
    const cf_config& c = e->cfg;
    const int W = c.n_neg, G = group_count(c);
    if (!is_device_ptr(negs) || (G > 0 && !is_device_ptr(groups)))
        return fail(CF_EINVAL, "a batch must be all host or all device memory");
    if (!e->d_bad) {
        CF_TRY(dalloc(&e->d_bad, 1));
        CF_HIP(hipHostMalloc((void**)&e->h_bad, sizeof(int32_t), hipHostMallocDefault));
    }
    PackArgs a{};
    a.u = pairs;
    a.us = e->tuple_stride ? e->tuple_stride : 2;
    a.j = negs;
    a.js = e->tuple_stride ? e->tuple_stride : W;
    a.g = groups;
    a.gs = G;
    a.B = B; a.W = W; a.G = G;
    a.n_users = c.n_users;
    a.n_items = c.n_items;
    a.sharded = e->world > 1 ? 1 : 0;
    a.shard_u0 = e->shard_u0;
    a.shard_u1 = e->shard_u1;
    a.total_users = e->world > 1 ? e->h_bounds[e->world] : c.n_users;
    a.occU = e->occU_[k];
    a.occV = e->occV_[k];
    a.bad = e->d_bad;
    CF_HIP(hipMemsetAsync(e->d_bad, 0x7F, sizeof(int32_t), st));
    CF_HIP(launch_pack_batch(a, st));
    CF_HIP(hipMemcpyAsync(e->h_bad, e->d_bad, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    CF_HIP(hipStreamSynchronize(st));
    if (*e->h_bad != kPackOk)
        return fail(CF_EINVAL, "device batch row " + std::to_string(*e->h_bad) + " has an id out of range");
    return CF_OK;
}

int stage_host_batch(cf_engine* e, const int32_t* pairs, const int32_t* negs,
                     const int32_t* groups, int B, int k, hipStream_t st) {
    const cf_config& c = e->cfg;
    const int W = c.n_neg, G = group_count(c);
    if (!pairs || !negs) return fail(CF_EINVAL, "pairs and negs are required");
    if (G > 0 && !groups) return fail(CF_EINVAL, "GBPR needs groups");
    if (is_device_ptr(pairs)) return stage_device_batch(e, pairs, negs, groups, B, k, st);
    if (is_device_ptr(negs) || (G > 0 && is_device_ptr(groups)))
        return fail(CF_EINVAL, "a batch must be all host or all device memory");
    const size_t us = e->tuple_stride ? (size_t)e->tuple_stride : 2;
    const size_t js = e->tuple_stride ? (size_t)e->tuple_stride : (size_t)W;
    const size_t nU = (size_t)B * (1 + G), nV = (size_t)B * (1 + W);
    const size_t need = nU + nV;
    if (need > e->stage_cap) {
        if (e->h_stage) {
            (void)hipEventSynchronize(e->stage_ev);
            (void)hipHostFree(e->h_stage);
            e->h_stage = nullptr;
        }
        CF_HIP(hipHostMalloc((void**)&e->h_stage, need * sizeof(int32_t), hipHostMallocDefault));
        e->stage_cap = need;
    } else {
        CF_HIP(hipEventSynchronize(e->stage_ev));
    }
    int32_t* su = e->h_stage;
    int32_t* sv = e->h_stage + nU;
    const int64_t nu = c.n_users, ni = c.n_items;
    for (int p = 0; p < B; ++p) {
        const int32_t u = pairs[us * p], i = pairs[us * p + 1];
        if (u < 0 || u >= nu || i < 0 || i >= ni)
            return fail(CF_EINVAL, "pair " + std::to_string(p) + " out of range");
        su[p] = u;
        sv[p] = i;
        for (int w = 0; w < W; ++w) {
            const int32_t j = negs[js * p + w];
            if (j < 0 || j >= ni) return fail(CF_EINVAL, "negative item out of range");
            sv[B + (size_t)p * W + w] = j;
        }
        for (int k = 0; k < G; ++k) {
            // group members are global user ids on a sharded engine; one
            // owned by another rank is coded -1 - id (cf_xchg_begin)
            const int32_t g = groups[(size_t)p * G + k];
            if (e->world > 1) {
                if (g < 0 || g >= e->h_bounds[e->world]) return fail(CF_EINVAL, "group user out of range");
                su[B + (size_t)p * G + k] =
                    (g >= e->shard_u0 && g < e->shard_u1) ? (int32_t)(g - e->shard_u0) : -1 - g;
                continue;
            }
            if (g < 0 || g >= nu) return fail(CF_EINVAL, "group user out of range");
            su[B + (size_t)p * G + k] = g;
        }
    }
    CF_HIP(hipMemcpyAsync(e->occU_[k], su, nU * sizeof(int32_t), hipMemcpyHostToDevice, st));
    CF_HIP(hipMemcpyAsync(e->occV_[k], sv, nV * sizeof(int32_t), hipMemcpyHostToDevice, st));
    CF_HIP(hipEventRecord(e->stage_ev, st));
    return CF_OK;
}

// Stage / position the batch of one step in buffer set k and launch its draw
// + count (prep) on stream ps.  Returns the step's arguments in *a.
// deterministic mode on the positive-sorted path must take the fixed-point
// form: its buffers not being ready is an engine bug, not a reason to run the
// float-atomic path while cf_step_path reports DETERMINISTIC
int check_det_args(cf_engine* e, const StepArgs& a) {
    if (e->det && a.cntP != nullptr && !a.det_fx)
        return fail(CF_ESTATE, "deterministic pos_sort step without its fixed-point buffers");
    if (e->det && a.cntP == nullptr && a.offU == nullptr && !e->cfg.dense_item_apply)
        return fail(CF_ESTATE, "deterministic step without its sort-based buffers");
    return CF_OK;
}

int begin_step(cf_engine* e, int B, const int32_t* pairs, const int32_t* negs,
               const int32_t* groups, int k, hipStream_t ps, StepArgs* a) {
    *a = base_step_args(e, B, k);
    CF_TRY(check_det_args(e, *a));
    if (pairs) {
        CF_TRY(stage_host_batch(e, pairs, negs, groups, B, k, ps));
        a->sample = 0;
    } else {
        CF_TRY(sampler_args(e, B, a));
    }
    ProfScope pr(e, CF_K_SAMPLE, ps);
    CF_HIP(launch_prep(*a, ps));
    return CF_OK;
}

// The rest of a step on the engine stream: slots, gradient (+ singleton
// Adagrad), duplicate apply (+ CML clip).  With `next`, the apply launch also
// draws and counts the next step's batch (launch_apply_prep).  Loss added to
// *loss_acc.
ApplyArgs apply_args(cf_engine* e, const StepArgs& a, int B, int k, double* loss_acc) {
    const cf_config& c = e->cfg;
    ApplyArgs p{};
    p.det_fx = a.det_fx;
    p.slotP64 = a.slotP64;
    p.GU64 = a.GU64;
    p.hotU = a.hotU;
    p.hot_n = a.det_fx ? e->hot_n : nullptr;
    p.GV64 = a.GV64;
    p.fx_bad = a.fx_bad;
    p.d = c.n_factors;
    p.lr = c.lr;
    p.clip_norm = c.clip_norm;
    p.clip = c.model == CF_CML ? 1 : 0;
    p.capU = a.capU;
    p.capV = a.capV;
    p.GVrep = a.GVrep;
    p.repV = a.repV;
    p.offU = a.offU;
    p.offV = a.offV;
    p.slotVb = a.slotVb;
    p.recV = a.recV;
    p.stashU = a.stashU;
    p.stashB = a.stashB;
    if (a.cntP != nullptr && a.count_items) {
        p.cntP = a.cntP;
        p.offPN = e->offPN;
        p.slotP = a.slotP;
        p.capP = a.capP;
        p.nPos = B;
        // visit every row of a table that is not much larger than the batch's
        // occurrences of it (cfg2 at 2^19: 100K items / 1.05M occurrences,
        // 1M users / 524K), else find the owners among the occurrences
        p.dense_items = c.n_items <= 2 * (int64_t)B * items_per_pair(c) ? 1 : 0;
        p.dense_users = c.n_users <= 2 * (int64_t)B * users_per_pair(c) ? 1 : 0;
    } else if (e->dense_apply && !e->det && !a.items_grad_only && a.count_items && c.model != CF_GBPR &&
             c.model != CF_PLR) {
        // slot rows / item records: one group per item row when the item table
        // is not much larger than the batch's item occurrences (cfg3 / cfg5:
        // 100K items, 393K occurrences); users keep the occurrence owners
        p.dense_items = c.n_items <= 2 * (int64_t)B * items_per_pair(c) ? 1 : 0;
        p.dense_users = 0;
    }
    p.n_users = c.n_users;
    p.item_r0 = 0;
    p.item_r1 = c.n_items;
    if (e->det && a.cntP == nullptr) {
        p.hotP = e->hotP;
        p.hotPb = e->hotPb;
    }
    p.n_items = c.n_items;
    p.count_users = a.count_users;
    p.count_items = a.count_items;
    p.items_grad_only = a.items_grad_only;
    if (a.items_grad_only && a.capV == 0) p.count_items = 0;  // item_reduce 2: nothing to reduce
    p.occU = e->occU_[k];
    p.rankU = e->rankU_[k];
    p.nU = (int64_t)B * users_per_pair(c);
    p.occV = e->occV_[k];
    p.rankV = e->rankV_[k];
    p.nV = (int64_t)B * items_per_pair(c);
    p.shard_u0 = e->shard_u0;
    p.slotU = a.slotU;
    p.slotV = a.slotV;
    p.cntU = e->cntU_[k];
    p.cntV = e->cntV_[k];
    p.U = e->U; p.AU = e->AU; p.GU = e->GU;
    p.V = e->V; p.AV = e->AV; p.GV = e->GV;
    p.b = a.train_bias ? e->b : nullptr;  // PRIGP keeps b fixed (prigp.py:145)
    p.Ab = e->Ab; p.Gb = e->Gb;
    p.loss_partial = e->loss_partial;
    p.n_partial = grad_blocks(a);
    p.loss_acc = loss_acc;
    return p;
}

// CML: the full-table clip pending after step 1 / a table upload
int pending_clips(cf_engine* e) {
    const cf_config& c = e->cfg;
    if (e->need_clip_U) {
        ProfScope ps(e, CF_K_CLIP);
        CF_HIP(launch_clip_full(e->U, c.n_users, c.n_factors, c.clip_norm, e->stream));
        e->need_clip_U = false;
    }
    if (!c.dense_item_apply && e->need_clip_V) {
        ProfScope ps(e, CF_K_CLIP);
        CF_HIP(launch_clip_full(e->V, c.n_items, c.n_factors, c.clip_norm, e->stream));
        e->need_clip_V = false;
    }
    return CF_OK;
}

// deterministic mode: replace the batch's atomic ranks by sort-based ones
// (and write off[row]) before its gradient launch
int det_ranks(cf_engine* e, const StepArgs& a) {
    if (!e->det || a.det_fx) return CF_OK;   // the fixed-point form needs no ranks
    const cf_config& c = e->cfg;
    const int64_t nU = (int64_t)a.B * users_per_pair(c), nV = (int64_t)a.B * items_per_pair(c);
    CF_HIP(launch_det_ranks(a.occU, nU, a.occV, nV, c.n_users, c.n_users + c.n_items, a.rankU, a.rankV,
                            e->det_off, e->det_keys, e->det_vals, e->det_tmp, e->det_tmp_bytes, e->stream));
    return CF_OK;
}

// deterministic mode, after the gradient launch: the sums of the sorted
// occurrence list's 64-slot tiles that lie inside one row, for the apply
int det_hot(cf_engine* e, const StepArgs& a) {
    if (!e->det || a.cntP != nullptr) return CF_OK;   // pos_sort sums no tiles
    const cf_config& c = e->cfg;
    HotArgs h{};
    h.d = c.n_factors;
    h.nU = (int64_t)a.B * users_per_pair(c);
    h.n = h.nU + (int64_t)a.B * items_per_pair(c);
    h.n_users = c.n_users;
    h.skeys = e->det_keys + h.n;   // the sort's output half
    h.slotU = a.slotU;
    h.slotV = a.recV ? nullptr : a.slotV;
    h.recV = a.recV;
    h.stashU = a.stashU;
    h.stashB = a.stashB;
    h.P = e->hotP;
    h.Pb = e->hotPb;
    CF_HIP(launch_det_hot(h, e->stream));
    return CF_OK;
}

// pos_sort: order the batch's pairs by positive item before its gradient launch
int psort(cf_engine* e, const StepArgs& a) {
    if (a.srec == nullptr) return CF_OK;
    ProfScope ps(e, CF_K_PSORT);
    PsortArgs q{};
    q.occU = a.occU; q.rankU = a.rankU;
    q.occV = a.occV; q.rankV = a.rankV;
    q.cntU = a.cntU; q.cntV = a.cntV; q.cntP = a.cntP;
    q.offPN = e->offPN;
    q.srec = e->srec;
    q.B = a.B; q.W = a.W; q.capU = a.capU;
    q.n_items = e->cfg.n_items;
    q.spec_ph = a.spec_ph;
    q.spec_n = a.spec_n;
    q.slotN = e->slotN;
    q.cntVw = a.cntV;
    q.d = e->cfg.n_factors;
    if (a.det_fx) {   // compact GU64 rows for the users past their slot cap
        q.hotU = e->hotU;
        q.hot_n = e->hot_n;
    }
    CF_HIP(launch_psort(q, e->psort_tmp, e->psort_tmp_bytes, e->stream));
    return CF_OK;
}

int finish_step(cf_engine* e, const StepArgs& a, int B, int k, double* loss_acc,
                const StepArgs* next) {
    CF_TRY(det_ranks(e, a));
    CF_TRY(psort(e, a));
    ApplyArgs p = apply_args(e, a, B, k, loss_acc);
    if (next && e->pipeline == 3 && a.srec != nullptr) {
        // pipeline 3 (pos_sort steps): the draw + count of step s+1 rides in
        // the positive-sorted gradient launch of step s, the apply runs alone;
        // psort of s+1 follows the apply, so offPN / srec / slotN stay single
        {
            ProfScope ps(e, CF_K_GRAD_PREP);
            CF_HIP(launch_grad(a, e->stream, next));
        }
        ProfScope ps(e, CF_K_APPLY);
        CF_HIP(launch_apply(p, e->stream));
        if (e->prep_side) CF_HIP(hipEventRecord(e->apply_done[k], e->stream));
        return pending_clips(e);
    }
    if (next && e->pipeline == 2) {
        p.n_partial = grad_blocks(a, true);   // the launch with draw blocks keeps 256-lane groups
        // the draw + count of step s+1 rides in the gradient launch of step s
        // (other buffer set), the duplicate apply runs alone
        {
            ProfScope ps(e, CF_K_GRAD_PREP);
            CF_HIP(launch_grad(a, e->stream, next));
        }
        CF_TRY(det_hot(e, a));
        ProfScope ps(e, CF_K_APPLY);
        CF_HIP(launch_apply(p, e->stream));
        if (e->prep_side) CF_HIP(hipEventRecord(e->apply_done[k], e->stream));
        return pending_clips(e);
    }
    {
        ProfScope ps(e, CF_K_STEP);
        CF_HIP(launch_grad(a, e->stream));
    }
    CF_TRY(det_hot(e, a));
    if (next) {
        ProfScope ps(e, CF_K_APPLY_PREP);
        CF_HIP(launch_apply_prep(p, *next, e->stream));
    } else {
        ProfScope ps(e, CF_K_APPLY);
        CF_HIP(launch_apply(p, e->stream));
    }
    if (e->prep_side) CF_HIP(hipEventRecord(e->apply_done[k], e->stream));
    return pending_clips(e);
}

// One step, host-fed (pairs != null) or from the device sampler.  With
// prep_stream=1 the draw / staging runs on the side stream, so that it can
// overlap the previous step's kernels.
int run_step(cf_engine* e, int B, const int32_t* pairs, const int32_t* negs,
             const int32_t* groups, double* loss_acc) {
    if (e->cfg.amf_mode == CF_AMF_APR && e->phase == 1 && e->cfg.dense_item_apply && !e->GadvV_bound)
        return fail(CF_ESTATE, "amf_mode apr with dense_item_apply: bind the apr item buffer first "
                               "(cf_bind_apr_item_grad)");
    CF_TRY(ensure_batch(e, B));
    const int k = e->set;
    e->set ^= 1;
    hipStream_t ps = e->prep_side ? e->side : e->stream;
    // set k was last used by step s-2: its apply must be done before reuse
    if (e->prep_side) CF_HIP(hipStreamWaitEvent(ps, e->apply_done[k], 0));
    StepArgs a;
    CF_TRY(begin_step(e, B, pairs, negs, groups, k, ps, &a));
    if (e->prep_side) {
        CF_HIP(hipEventRecord(e->prep_done[k], ps));
        CF_HIP(hipStreamWaitEvent(e->stream, e->prep_done[k], 0));
    }
    return finish_step(e, a, B, k, loss_acc, nullptr);
}

// n steps from the device sampler, pipelined on the engine stream: the apply
// launch of step s also draws and counts step s+1 (3 launches per step).
int run_steps_device(cf_engine* e, int B, int n, double* loss_acc) {
    if (n <= 0) return CF_OK;
    CF_TRY(ensure_batch(e, B));
    int k = e->set;
    if (e->prep_side) CF_HIP(hipStreamWaitEvent(e->stream, e->apply_done[k], 0));
    StepArgs a;
    CF_TRY(begin_step(e, B, nullptr, nullptr, nullptr, k, e->stream, &a));
    // the positive-sorted gradient launch of step s fetches step s+1's pair
    // records (StepArgs::pf_out); the draw of s+1 then reads them coalesced
    // (sorted batches read their records coalesced already: no prefetch)
    const bool pf = e->pair_prefetch && a.srec != nullptr && e->pipeline == 1 && !e->prep_side &&
                    a.pos_set == nullptr && a.order == nullptr &&
                    a.order_recs == nullptr;
    if (pf && e->pf_cap < B) {
        CF_HIP(hipStreamSynchronize(e->stream));
        for (int q = 0; q < 2; ++q) {
            dfree(e->pf_recs[q]);
            CF_TRY(dalloc(&e->pf_recs[q], (size_t)B));
        }
        e->pf_cap = B;
    }
    for (int s = 0; s < n; ++s) {
        StepArgs nx{};
        const bool more = s + 1 < n;
        if (more) {
            nx = base_step_args(e, B, k ^ 1);
            CF_TRY(check_det_args(e, nx));
            CF_TRY(sampler_args(e, B, &nx));
            if (pf) {
                a.pf_out = e->pf_recs[k ^ 1];
                a.pf_slot_base = nx.slot_base;
                a.pf_perm = nx.perm;
                a.pf_B = B;
                nx.pre_pairs = e->pf_recs[k ^ 1];
            }
        }
        CF_TRY(finish_step(e, a, B, k, loss_acc, more ? &nx : nullptr));
        a = nx;
        k ^= 1;
    }
    e->set = k;
    return CF_OK;
}

int run_items_dense(cf_engine* e) {
    const cf_config& c = e->cfg;
    DenseArgs d{};
    d.d = c.n_factors;
    d.lr = c.lr;
    d.clip_norm = c.clip_norm;
    d.clip = c.model == CF_CML ? 1 : 0;
    d.zero_g = 1;
    d.n_rows = c.n_items;
    d.X = e->V; d.A = e->AV; d.G = e->GV;
    d.b = e->b; d.Ab = e->Ab; d.Gb = e->Gb;
    {
        ProfScope ps(e, CF_K_APPLY_DENSE);
        CF_HIP(launch_apply_dense(d, e->stream));
    }
    if (e->need_clip_V) {
        ProfScope ps(e, CF_K_CLIP);
        CF_HIP(launch_clip_full(e->V, c.n_items, c.n_factors, c.clip_norm, e->stream));
        e->need_clip_V = false;
    }
    return CF_OK;
}

// deterministic mode: a fixed-point term or sum out of range (to_fx) during
// the calls since the last check fails the call -- the tables then hold NaN
// where a sum overflowed and are not a valid step (the fp32 path would show
// inf / NaN; the int64 sums would otherwise wrap silently)
int check_fx(cf_engine* e) {
    if (!e->fx_bad) return CF_OK;
    const int n = std::min(e->fx_step, kFxSlots);
    e->fx_step = 0;
    if (n == 0) return CF_OK;
    // every word: a step drawn ahead (or a split step) took its word when
    // its arguments were built and may write one at or above n
    CF_HIP(hipMemcpyAsync(e->h_fx_bad, e->fx_bad, (size_t)kFxSlots * sizeof(int), hipMemcpyDeviceToHost,
                          e->stream));
    CF_HIP(hipStreamSynchronize(e->stream));
    int first = -1;
    for (int q = 0; q < kFxSlots && first < 0; ++q)
        if (e->h_fx_bad[q] != 0) first = q;
    if (first < 0) return CF_OK;
    CF_HIP(hipMemsetAsync(e->fx_bad, 0, (size_t)kFxSlots * sizeof(int), e->stream));
    const std::string at = first == kFxSlots - 1 ? "at or after step " + std::to_string(first)
                                                  : "at step " + std::to_string(first);
    return fail(CF_ENUMERIC, "deterministic mode: a gradient term was not finite or outside the "
                             "fixed-point range (|g| >= 2^20, or a row sum >= 2^30) " + at +
                             " of the steps since the last check (0-based); that step and every later one "
                             "of the call are invalid");
}

int read_loss(cf_engine* e, int slot, double* out) {
    CF_HIP(hipMemcpyAsync(e->h_loss, e->loss + slot, sizeof(double), hipMemcpyDeviceToHost,
                          e->stream));
    CF_HIP(hipStreamSynchronize(e->stream));
    *out = *e->h_loss;
    CF_HIP(hipMemsetAsync(e->loss + slot, 0, sizeof(double), e->stream));
    return CF_OK;
}

// drop a batch the previous apply launch drew ahead: clear its occurrence
// counts and put the sampler back where that draw started
int discard_pending(cf_engine* e) {
    if (e->x_pend) {   // a drawn-ahead exchange batch: uncount it, rewind the sampler
        const cf_config& c = e->cfg;
        const StepArgs& a = e->x_pend_args;
        const int64_t nU = (int64_t)e->x_pend_B * users_per_pair(c), nV = (int64_t)e->x_pend_B * items_per_pair(c);
        if (a.count_users) CF_HIP(launch_uncount(a.occU, nU, a.cntU, e->stream));
        if (a.count_items) CF_HIP(launch_uncount(a.occV, nV, a.cntV, e->stream));
        if (a.count_items && a.cntP) CF_HIP(launch_uncount(a.occV, e->x_pend_B, a.cntP, e->stream));
        e->epoch = e->x_pend_epoch;
        e->batch = e->x_pend_batch;
        e->sampler_B = e->x_pend_sampler_B;
        e->set = e->x_pend_set;
        e->x_pend = false;
    }
    if (!e->pend) return CF_OK;
    const cf_config& c = e->cfg;
    const StepArgs& a = e->pend_args;
    const int64_t nU = (int64_t)e->pend_B * users_per_pair(c), nV = (int64_t)e->pend_B * items_per_pair(c);
    if (a.count_users) CF_HIP(launch_uncount(a.occU, nU, a.cntU, e->stream));
    if (a.count_items) CF_HIP(launch_uncount(a.occV, nV, a.cntV, e->stream));
    if (a.count_items && a.cntP) CF_HIP(launch_uncount(a.occV, e->pend_B, a.cntP, e->stream));
    if (a.spec_n) CF_HIP(launch_uncount_spec(a.spec_ph, a.spec_n, a.cntV, e->stream));
    e->epoch = e->pend_epoch;
    e->batch = e->pend_batch;
    e->sampler_B = e->pend_sampler_B;
    e->set = e->pend_set;
    e->pend = false;
    return CF_OK;
}

// a user-sharded GBPR engine steps only through the group exchange
int check_not_xchg(cf_engine* e) {
    if (e->cfg.model == CF_GBPR && e->group_source_global)
        return fail(CF_ESTATE, "user-sharded GBPR steps through cf_xchg_begin/serve/grad/finish");
    return CF_OK;
}

int check_engine(cf_engine* e) {
    if (!e) return fail(CF_EINVAL, "null engine");
    return set_dev(e);
}

float* table_ptr(cf_engine* e, int t, int64_t* n) {
    const cf_config& c = e->cfg;
    const int64_t ud = c.n_users * (int64_t)c.n_factors, id = c.n_items * (int64_t)c.n_factors;
    switch (t) {
        case CF_TABLE_USER: *n = ud; return e->U;
        case CF_TABLE_ITEM: *n = id; return e->V;
        case CF_TABLE_BIAS: *n = c.n_items; return e->b;
        case CF_TABLE_ACC_USER: *n = ud; return e->AU;
        case CF_TABLE_ACC_ITEM: *n = id; return e->AV;
        case CF_TABLE_ACC_BIAS: *n = c.n_items; return e->Ab;
        default: *n = 0; return nullptr;
    }
}

int check_device_ptr(const void* p, const char* what) {
    hipPointerAttribute_t attr;
    if (!p || hipPointerGetAttributes(&attr, p) != hipSuccess || attr.type != hipMemoryTypeDevice)
        return fail(CF_EINVAL, std::string(what) + " is not device memory");
    return CF_OK;
}

float** table_slot(cf_engine* e, int t) {
    switch (t) {
        case CF_TABLE_USER: return &e->U;
        case CF_TABLE_ITEM: return &e->V;
        case CF_TABLE_BIAS: return &e->b;
        case CF_TABLE_ACC_USER: return &e->AU;
        case CF_TABLE_ACC_ITEM: return &e->AV;
        case CF_TABLE_ACC_BIAS: return &e->Ab;
        default: return nullptr;
    }
}

// fused fp32-MFMA scoring + streaming top-k: no score matrix in HBM
int score_topk_fused(cf_engine* e, const int32_t* users, int n, int k, int exclude_train,
                     const uint64_t* item_mask, int32_t* idx_out, float* val_out) {
    const cf_config& c = e->cfg;
    int32_t* d_users = nullptr;
    int32_t* d_idx = nullptr;
    float* d_val = nullptr;
    int r = CF_OK;
    if ((r = dalloc(&d_users, (size_t)n)) || (r = dalloc(&d_idx, (size_t)n * k)) ||
        (val_out && (r = dalloc(&d_val, (size_t)n * k)))) {
        dfree(d_users); dfree(d_idx); dfree(d_val);
        return r;
    }
    FusedTopkArgs f{};
    f.model = c.model == CF_PLR ? CF_GBPR : c.model;  // U.V^T + b (prigp.py:137, cplr_u.py:146)
    f.d = c.n_factors;
    f.Dp = (c.n_factors + 7) & ~7;
    f.Dh = f.Dp / 2;
    f.n_users = n;
    f.n_items = c.n_items;
    f.k = k;
    f.users = d_users;
    f.U = e->U;
    f.V = e->V;
    f.b = e->b;
    f.exclude_train = exclude_train ? 1 : 0;
    f.indptr = e->indptr;
    f.indices = e->indices;
    f.idx_out = d_idx;
    f.val_out = d_val;
    f.variant = e->fused_variant;
    f.item_mask = item_mask;
    hipError_t he = hipMemcpyAsync(d_users, users, (size_t)n * 4, hipMemcpyHostToDevice, e->stream);
#ifdef CF_FUSED_STAMPS
    // diagnostic builds: per-wave cycles of each phase of the sweep, summed
    // over the waves and printed (tools/score_ab.py)
    const size_t n_st = (size_t)((n + 63) / 64) * 8 * 16;
    std::vector<unsigned long long> h_st(n_st, 0ull);
    if (he == hipSuccess) he = hipMalloc(&f.stamps, n_st * sizeof(unsigned long long));
    if (he == hipSuccess) he = hipMemsetAsync(f.stamps, 0, n_st * sizeof(unsigned long long), e->stream);
#endif
    if (he == hipSuccess) {
        ProfScope ps(e, CF_K_TOPK);
        he = launch_fused_topk(f, e->stream);
    }
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
#ifdef CF_FUSED_STAMPS
    if (he == hipSuccess) he = hipMemcpy(h_st.data(), f.stamps, n_st * sizeof(unsigned long long), hipMemcpyDefault);
    if (f.stamps) (void)hipFree(f.stamps);
    if (he == hipSuccess) {
        static const char* names[14] = {"stage", "bar1", "mfma", "cand_rest", "bar2", "tile_wait", "store",
                                        "compact", "bar3", "", "", "prefilter", "exact", ""};
        double tot[16] = {0};
        for (size_t q = 0; q < n_st; ++q) tot[q & 15] += (double)h_st[q];
        double all = 0.0;
        for (int q = 0; q < 14; ++q)
            if (q != 9 && q != 10) all += tot[q];
        std::fprintf(stderr, "fused stamps: total %.4e wave-cycles; exact-path wave-steps %.0f, compaction wave-steps %.0f\n",
                     all, tot[9], tot[10]);
        for (int q = 0; q < 14; ++q)
            if (q != 9 && q != 10 && q != 13)
                std::fprintf(stderr, "fused stamps: %-14s %.4e  %.3f\n", names[q], tot[q], tot[q] / all);
    }
#endif
    if (he == hipSuccess) he = hipMemcpy(idx_out, d_idx, (size_t)n * k * 4, hipMemcpyDefault);
    if (he == hipSuccess && val_out)
        he = hipMemcpy(val_out, d_val, (size_t)n * k * 4, hipMemcpyDefault);
    dfree(d_users); dfree(d_idx); dfree(d_val);
    if (he != hipSuccess) return fail(CF_EHIP, std::string("cf_score_topk (fused): ") + hipGetErrorString(he));
    return CF_OK;
}

}  // namespace

extern "C" {

const char* cf_version(void) { return "cf_engine 0.1 (gfx950)"; }

const char* cf_last_error(void) { return g_err.c_str(); }

int cf_device_count(int32_t* count_out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (count_out) *count_out = n;
    return CF_OK;
}

void cf_config_defaults(cf_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->model = CF_BPR;
    c->n_factors = 20;       // bprmf.py:15
    c->n_neg = 1;
    c->gsize = 1;
    c->lr = 0.1f;            // bprmf.py:16
    c->reg = 0.02f;          // bprmf.py:15
    c->rho = 0.5f;           // gbprmf.py:14
    c->margin = 1.5f;        // cml.py:16
    c->reg_cov = 1.0f;       // cml.py:16
    c->clip_norm = 1.0f;     // cml.py:16
    c->reg_adv = 1.0f;       // amf.py:15
    c->epsilon = 0.5f;       // amf.py:15
    c->acc_init = 0.1f;      // tf.train.AdagradOptimizer initial_accumulator_value
    c->use_rank_weight = 1;  // cml.py:16
    c->seed = 20261015ull;
    c->alpha = c->beta = c->gamma = 1.0f;  // prigp.py:22, cplr_u.py:21
}

int cf_create(const cf_config* cfg, cf_engine** out) {
    if (!cfg || !out) return fail(CF_EINVAL, "null argument");
    *out = nullptr;
    const cf_config& c = *cfg;
    if (c.model < CF_BPR || c.model > CF_PLR) return fail(CF_EINVAL, "unknown model");
    if (c.model == CF_PLR && !((c.plr_kind == CF_PLR_PRIGP && c.n_neg == 3) ||
                               (c.plr_kind == CF_PLR_CPLR && c.n_neg == 2)))
        return fail(CF_EINVAL, "PLR: PRIGP takes n_neg 3 (tuple width 5), CPLR n_neg 2 (width 4)");
    if (c.n_factors < 1 || c.n_factors > kMaxFactors) return fail(CF_EINVAL, "n_factors must be 1..256");
    if (c.n_users < 1 || c.n_users > INT32_MAX) return fail(CF_EINVAL, "n_users out of range");
    if (c.n_items < 2 || c.n_items > INT32_MAX) return fail(CF_EINVAL, "n_items out of range");
    if (c.n_users + c.n_items > INT32_MAX) return fail(CF_EINVAL, "n_users + n_items must fit int32 (row ids)");
    if (c.n_neg < 1 || c.n_neg > kMaxNeg) return fail(CF_EINVAL, "n_neg must be 1..64");
    if (c.model == CF_GBPR && (c.gsize < 1 || c.gsize > kMaxGroup))
        return fail(CF_EINVAL, "gsize must be 1..16");
    if (!(c.lr > 0.f) || !(c.acc_init > 0.f)) return fail(CF_EINVAL, "lr and acc_init must be > 0");
    if (c.model == CF_CML && !(c.clip_norm > 0.f)) return fail(CF_EINVAL, "clip_norm must be > 0");
    if (c.model == CF_CML && c.n_neg > 16) return fail(CF_EINVAL, "CML supports n_neg <= 16");
    if (c.amf_mode != CF_AMF_REFERENCE && c.amf_mode != CF_AMF_APR)
        return fail(CF_EINVAL, "amf_mode must be CF_AMF_REFERENCE (0) or CF_AMF_APR (1)");
    if (c.amf_mode == CF_AMF_APR && c.model != CF_AMF) return fail(CF_EINVAL, "amf_mode apr is an AMF mode");
    if (c.amf_mode == CF_AMF_APR && !(c.epsilon >= 0.f)) return fail(CF_EINVAL, "epsilon must be >= 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CF_EHIP, "no HIP device visible (the engine has no CPU fallback)");
    if (c.device < 0 || c.device >= ndev) return fail(CF_EINVAL, "device ordinal out of range");

    cf_engine* e = new (std::nothrow) cf_engine();
    if (!e) return fail(CF_ENOMEM, "host allocation failed");
    e->cfg = c;
    // item records by default for rows of >= 512 B: A/B on MI355X (ms/step,
    // rows -> records) cfg3 0.256 -> 0.230, cfg5 0.258 -> 0.227 (d 128, W 5);
    // cfg2 0.497 -> 0.519, cfg4 0.241 -> 0.254 (d 64: the apply's record ->
    // stash gather chain costs more than the smaller slot stores save)
    e->item_recs = (c.n_factors >= 128 && c.amf_mode != CF_AMF_APR) ? 1 : 0;   // apr: gradient rows only
    int r = CF_OK;
    auto bail = [&](int code) {
        cf_destroy(e);
        return code;
    };
    if ((r = set_dev(e)) != CF_OK) return bail(r);
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(CF_EHIP, "hipStreamCreate failed"));
    e->own_stream = true;
    if (hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(CF_EHIP, "hipStreamCreate failed"));
    if (hipEventCreateWithFlags(&e->stage_ev, hipEventDisableTiming) != hipSuccess)
        return bail(fail(CF_EHIP, "hipEventCreate failed"));
    for (int k = 0; k < 2; ++k)
        if (hipEventCreateWithFlags(&e->prep_done[k], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e->apply_done[k], hipEventDisableTiming) != hipSuccess)
            return bail(fail(CF_EHIP, "hipEventCreate failed"));
    (void)hipEventRecord(e->stage_ev, e->stream);
    const size_t ud = (size_t)c.n_users * c.n_factors, id = (size_t)c.n_items * c.n_factors;
    if ((r = dalloc(&e->U, ud)) || (r = dalloc(&e->AU, ud)) || (r = dalloc(&e->GU, ud)) ||
        (r = dalloc(&e->V, id)) || (r = dalloc(&e->AV, id)) || (r = dalloc(&e->GV_own, id)) ||
        (r = dalloc(&e->cntU_[0], (size_t)c.n_users)) || (r = dalloc(&e->cntV_[0], (size_t)c.n_items)) ||
        (r = dalloc(&e->cntU_[1], (size_t)c.n_users)) || (r = dalloc(&e->cntV_[1], (size_t)c.n_items)) ||
        (r = dalloc(&e->loss, 2)))
        return bail(r);
    if (has_bias(c)) {
        if ((r = dalloc(&e->b, (size_t)c.n_items)) || (r = dalloc(&e->Ab, (size_t)c.n_items)) ||
            (r = dalloc(&e->Gb_own, (size_t)c.n_items)))
            return bail(r);
    }
    e->GV = e->GV_own;
    e->Gb = e->Gb_own;
    e->shard_u1 = c.n_users;
    if (c.amf_mode == CF_AMF_APR) {
        if ((r = dalloc(&e->GadvU, ud))) return bail(r);
        if (hipMemsetAsync(e->GadvU, 0, ud * 4, e->stream) != hipSuccess)
            return bail(fail(CF_EHIP, "hipMemsetAsync failed"));
        if (!c.dense_item_apply) {   // multi-rank: the caller binds the item buffer
            if ((r = dalloc(&e->GadvV, id))) return bail(r);
            if (hipMemsetAsync(e->GadvV, 0, id * 4, e->stream) != hipSuccess)
                return bail(fail(CF_EHIP, "hipMemsetAsync failed"));
        }
    }
    if (hipHostMalloc((void**)&e->h_loss, sizeof(double), hipHostMallocDefault) != hipSuccess)
        return bail(fail(CF_ENOMEM, "pinned allocation failed"));
    if (hipHostMalloc((void**)&e->h_fx_bad, kFxSlots * sizeof(int), hipHostMallocDefault) != hipSuccess)
        return bail(fail(CF_ENOMEM, "pinned allocation failed"));
    *e->h_fx_bad = 0;
    hipStream_t s = e->stream;
    if (hipMemsetAsync(e->GU, 0, ud * 4, s) != hipSuccess ||
        hipMemsetAsync(e->GV, 0, id * 4, s) != hipSuccess ||
        hipMemsetAsync(e->U, 0, ud * 4, s) != hipSuccess ||
        hipMemsetAsync(e->V, 0, id * 4, s) != hipSuccess ||
        hipMemsetAsync(e->cntU_[0], 0, (size_t)c.n_users * 4, s) != hipSuccess ||
        hipMemsetAsync(e->cntV_[0], 0, (size_t)c.n_items * 4, s) != hipSuccess ||
        hipMemsetAsync(e->cntU_[1], 0, (size_t)c.n_users * 4, s) != hipSuccess ||
        hipMemsetAsync(e->cntV_[1], 0, (size_t)c.n_items * 4, s) != hipSuccess ||
        hipMemsetAsync(e->loss, 0, 2 * sizeof(double), s) != hipSuccess)
        return bail(fail(CF_EHIP, "hipMemsetAsync failed"));
    if (launch_fill(e->AU, (int64_t)ud, c.acc_init, s) != hipSuccess ||
        launch_fill(e->AV, (int64_t)id, c.acc_init, s) != hipSuccess)
        return bail(fail(CF_EHIP, "fill kernel failed"));
    if (has_bias(c)) {
        if (hipMemsetAsync(e->b, 0, (size_t)c.n_items * 4, s) != hipSuccess ||
            hipMemsetAsync(e->Gb, 0, (size_t)c.n_items * 4, s) != hipSuccess ||
            launch_fill(e->Ab, c.n_items, c.acc_init, s) != hipSuccess)
            return bail(fail(CF_EHIP, "bias init failed"));
    }
    e->need_clip_U = e->need_clip_V = (c.model == CF_CML);
    if (hipStreamSynchronize(s) != hipSuccess) return bail(fail(CF_EHIP, "stream sync failed"));
    *out = e;
    return CF_OK;
}

int cf_destroy(cf_engine* e) {
    if (!e) return CF_OK;
    (void)hipSetDevice(e->cfg.device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->side) (void)hipStreamSynchronize(e->side);
    for (auto& v : e->ev)
        for (auto& pr : v) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (auto x : e->ev_pool) (void)hipEventDestroy(x);
    for (int t = 0; t < 6; ++t)   // bound tables belong to the caller
        if (e->own_tab[t]) *table_slot(e, t) = e->own_tab[t];
    dfree(e->indptr); dfree(e->indices); dfree(e->pairs); dfree(e->indptr_t); dfree(e->indices_t);
    dfree(e->pf_recs[0]); dfree(e->pf_recs[1]); dfree(e->slotP64); dfree(e->GU64); dfree(e->GV64); dfree(e->fx_bad);
    dfree(e->hotU); dfree(e->hot_n);
    for (auto& o : e->eo) {
        dfree(o.keys);
        dfree(o.vals);
        dfree(o.recs);
        if (o.tmp) (void)hipFree(o.tmp);
        if (o.ready) (void)hipEventDestroy(o.ready);
    }
    if (e->eo_mark) (void)hipEventDestroy(e->eo_mark);
    if (e->eo_stream) (void)hipStreamDestroy(e->eo_stream);
    dfree(e->pos_set);
    dfree(e->U); dfree(e->V); dfree(e->b); dfree(e->AU); dfree(e->AV); dfree(e->Ab);
    dfree(e->GU); dfree(e->GV_own); dfree(e->Gb_own); dfree(e->GadvU); dfree(e->GadvV);
    for (int k = 0; k < 2; ++k) {
        dfree(e->cntU_[k]); dfree(e->cntV_[k]); dfree(e->occU_[k]); dfree(e->occV_[k]);
        dfree(e->rankU_[k]); dfree(e->rankV_[k]);
        if (e->prep_done[k]) (void)hipEventDestroy(e->prep_done[k]);
        if (e->apply_done[k]) (void)hipEventDestroy(e->apply_done[k]);
    }
    dfree(e->loss_partial); dfree(e->loss); dfree(e->keys); dfree(e->item_mask);
    dfree(e->slotU); dfree(e->slotV); dfree(e->slotVb); dfree(e->GVrep); dfree(e->x_own); dfree(e->coefs);
    dfree(e->bounds); dfree(e->xhist); dfree(e->xcounts);
    dfree(e->det_keys); dfree(e->det_vals); dfree(e->det_off); dfree(e->slotUc); dfree(e->slotVc);
    dfree(e->slotVbc); dfree(e->recV); dfree(e->recVc); dfree(e->stashU); dfree(e->stashB);
    dfree(e->hotP); dfree(e->hotPb);
    dfree(e->slotP); dfree(e->offPN); dfree(e->srec); dfree(e->slotN); dfree(e->cntP_[0]); dfree(e->cntP_[1]);
    if (e->psort_tmp) (void)hipFree(e->psort_tmp);
    if (e->det_tmp) (void)hipFree(e->det_tmp);
    if (e->h_xcounts) (void)hipHostFree(e->h_xcounts);
    if (e->h_loss) (void)hipHostFree(e->h_loss);
    if (e->h_fx_bad) (void)hipHostFree(e->h_fx_bad);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->h_bad) (void)hipHostFree(e->h_bad);
    dfree(e->d_bad);
    if (e->stage_ev) (void)hipEventDestroy(e->stage_ev);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    if (e->side) (void)hipStreamDestroy(e->side);
    delete e;
    return CF_OK;
}

int cf_set_stream(cf_engine* e, void* s) {
    CF_TRY(check_engine(e));
    CF_HIP(hipStreamSynchronize(e->stream));
    if (s) {
        if (e->own_stream) (void)hipStreamDestroy(e->stream);
        e->stream = (hipStream_t)s;
        e->own_stream = false;
    } else if (!e->own_stream) {
        CF_HIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
        e->own_stream = true;
    }
    return CF_OK;
}

int cf_synchronize(cf_engine* e) {
    CF_TRY(check_engine(e));
    CF_HIP(hipStreamSynchronize(e->side));
    CF_HIP(hipStreamSynchronize(e->stream));
    if (e->eo_stream) CF_HIP(hipStreamSynchronize(e->eo_stream));
    return CF_OK;
}

// the Pos(u) set of the current interactions (neg_check = 1), built on demand
int build_pos_set(cf_engine* e) {
    dfree(e->pos_set);
    const int64_t nnz = e->nnz_set;
    uint64_t cap = 1024;   // load factor <= 1/2
    while (cap < 2 * (uint64_t)nnz) cap <<= 1;
    CF_TRY(dalloc(&e->pos_set, (size_t)cap));
    e->pos_mask = cap - 1;
    CF_HIP(launch_build_pos_set(e->pairs, nnz, e->pos_set, e->pos_mask, e->stream));
    return CF_OK;
}

int cf_set_interactions(cf_engine* e, const int64_t* indptr, const int32_t* indices, int64_t nnz) {
    CF_TRY(check_engine(e));
    CF_TRY(discard_pending(e));
    const cf_config& c = e->cfg;
    if (!indptr || (nnz > 0 && !indices)) return fail(CF_EINVAL, "null CSR");
    if (nnz < 1) return fail(CF_EINVAL, "no interactions");
    if (nnz > INT32_MAX) return fail(CF_EINVAL, "nnz must be < 2^31 (int32 row offsets in the pair records)");
    if (indptr[0] != 0 || indptr[c.n_users] != nnz) return fail(CF_EINVAL, "indptr does not span nnz");
    int64_t full_row = -1;
    for (int64_t u = 0; u < c.n_users; ++u) {
        const int64_t rb = indptr[u], re = indptr[u + 1];
        if (re < rb) return fail(CF_EINVAL, "indptr not monotone");
        // only the device sampler needs a negative for every user; host-fed
        // and tuple models skip such users like sampler_uitj_ranking.py:28
        if (re - rb >= c.n_items && full_row < 0) full_row = u;
        for (int64_t k = rb; k < re; ++k) {
            const int32_t it = indices[k];
            if (it < 0 || it >= c.n_items) return fail(CF_EINVAL, "item id out of range");
            if (k > rb && indices[k - 1] >= it) return fail(CF_EINVAL, "CSR rows must be sorted, unique");
        }
    }
    // the sorted batches' cached epoch orders index the old pairs (and may
    // exceed the new nnz): let an order in flight finish, then drop them
    if (e->eo_stream) CF_HIP(hipStreamSynchronize(e->eo_stream));
    for (auto& o : e->eo) o.epoch = -1;
    e->sorted_auto_off = false;   // sorted_auto_fits decides again for the new nnz
    dfree(e->indptr); dfree(e->indices); dfree(e->pairs); dfree(e->indptr_t); dfree(e->indices_t);
    dfree(e->pos_set);
    CF_TRY(dalloc(&e->indptr, (size_t)c.n_users + 1));
    CF_TRY(dalloc(&e->indices, (size_t)nnz + 4));   // + 4: the draw's 16-B row loads never leave it
    CF_HIP(hipMemsetAsync(e->indices + nnz, 0xFF, 16, e->stream));
    CF_TRY(dalloc(&e->pairs, (size_t)nnz));
    CF_HIP(hipMemcpyAsync(e->indptr, indptr, ((size_t)c.n_users + 1) * 8, hipMemcpyHostToDevice, e->stream));
    CF_HIP(hipMemcpyAsync(e->indices, indices, (size_t)nnz * 4, hipMemcpyHostToDevice, e->stream));
    CF_HIP(launch_build_pairs(e->indptr, e->indices, c.n_users, e->pairs, e->stream));
    e->nnz_set = nnz;
    if (e->neg_check) CF_TRY(build_pos_set(e));
    if (c.model == CF_GBPR && !e->group_source_global) {
        // item -> users transpose (item_posUserList, sampler_gbpr.py:15)
        std::vector<int64_t> tp((size_t)c.n_items + 1, 0);
        for (int64_t k = 0; k < nnz; ++k) tp[(size_t)indices[k] + 1]++;
        for (int64_t i = 0; i < c.n_items; ++i) tp[i + 1] += tp[i];
        std::vector<int32_t> tu((size_t)nnz);
        std::vector<int64_t> fill(tp.begin(), tp.end() - 1);
        for (int64_t u = 0; u < c.n_users; ++u)
            for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k) tu[fill[indices[k]]++] = (int32_t)u;
        CF_TRY(dalloc(&e->indptr_t, (size_t)c.n_items + 1));
        CF_TRY(dalloc(&e->indices_t, (size_t)nnz));
        CF_HIP(hipMemcpyAsync(e->indptr_t, tp.data(), tp.size() * 8, hipMemcpyHostToDevice, e->stream));
        CF_HIP(hipMemcpyAsync(e->indices_t, tu.data(), tu.size() * 4, hipMemcpyHostToDevice, e->stream));
        CF_HIP(hipStreamSynchronize(e->stream));  // host vectors go out of scope
    }
    CF_HIP(hipStreamSynchronize(e->stream));
    e->h_indptr.assign(indptr, indptr + c.n_users + 1);
    e->full_row_user = full_row;
    e->nnz = nnz;
    e->epoch = 0;
    e->batch = 0;
    e->sampler_B = 0;
    return CF_OK;
}

int cf_init_params(cf_engine* e, float mean, float stddev, int32_t truncated, uint64_t seed) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    const int64_t ud = c.n_users * (int64_t)c.n_factors, id = c.n_items * (int64_t)c.n_factors;
    CF_HIP(launch_init_normal(e->U, ud, mean, stddev, truncated, mix64_host(seed ^ 0x55u), e->stream));
    CF_HIP(launch_init_normal(e->V, id, mean, stddev, truncated, mix64_host(seed ^ 0xAAu), e->stream));
    CF_HIP(launch_fill(e->AU, ud, c.acc_init, e->stream));
    CF_HIP(launch_fill(e->AV, id, c.acc_init, e->stream));
    if (has_bias(c)) {
        CF_HIP(launch_init_normal(e->b, c.n_items, mean, stddev, truncated, mix64_host(seed ^ 0xBBu), e->stream));
        CF_HIP(launch_fill(e->Ab, c.n_items, c.acc_init, e->stream));
    }
    e->need_clip_U = e->need_clip_V = (c.model == CF_CML);
    CF_HIP(hipStreamSynchronize(e->stream));
    return CF_OK;
}

int cf_set_table(cf_engine* e, int32_t t, const float* src, int64_t n) {
    CF_TRY(check_engine(e));
    int64_t want = 0;
    float* p = table_ptr(e, t, &want);
    if (!p) return fail(CF_EINVAL, "table not present in this model");
    if (n != want || !src) return fail(CF_EINVAL, "table size mismatch: want " + std::to_string(want));
    CF_HIP(hipMemcpyAsync(p, src, (size_t)n * 4, hipMemcpyDefault, e->stream));
    CF_HIP(hipStreamSynchronize(e->stream));
    if (e->cfg.model == CF_CML) {
        if (t == CF_TABLE_USER) e->need_clip_U = true;
        if (t == CF_TABLE_ITEM) e->need_clip_V = true;
    }
    return CF_OK;
}

int cf_get_table(cf_engine* e, int32_t t, float* dst, int64_t n) {
    CF_TRY(check_engine(e));
    CF_HIP(hipStreamSynchronize(e->side));
    int64_t want = 0;
    float* p = table_ptr(e, t, &want);
    if (!p) return fail(CF_EINVAL, "table not present in this model");
    if (n != want || !dst) return fail(CF_EINVAL, "table size mismatch: want " + std::to_string(want));
    CF_HIP(hipStreamSynchronize(e->stream));
    CF_HIP(hipMemcpy(dst, p, (size_t)n * 4, hipMemcpyDefault));
    return CF_OK;
}

// every table in one call, in enum cf_table order (U, V, b, AU, AV, Ab);
// NULL = keep / skip.  All sizes are implied by the config; b and Ab exist
// only for the bias models (GBPR, CPLR / PRIGP), passing them to another
// model is CF_EINVAL.  Nothing is copied unless every argument is valid.
static int params_check(cf_engine* e, const void* const* t) {
    for (int k = 0; k < 6; ++k) {
        if (!t[k]) continue;
        int64_t n = 0;
        if (!table_ptr(e, k, &n)) return fail(CF_EINVAL, "table " + std::to_string(k) + " not present in this model");
    }
    return CF_OK;
}

int cf_set_params(cf_engine* e, const float* U, const float* V, const float* b, const float* AU,
                  const float* AV, const float* Ab) {
    CF_TRY(check_engine(e));
    const void* t[6] = {U, V, b, AU, AV, Ab};
    CF_TRY(params_check(e, t));
    for (int k = 0; k < 6; ++k) {
        if (!t[k]) continue;
        int64_t n = 0;
        table_ptr(e, k, &n);
        CF_TRY(cf_set_table(e, k, (const float*)t[k], n));
    }
    return CF_OK;
}

int cf_get_params(cf_engine* e, float* U, float* V, float* b, float* AU, float* AV, float* Ab) {
    CF_TRY(check_engine(e));
    float* t[6] = {U, V, b, AU, AV, Ab};
    const void* tc[6] = {U, V, b, AU, AV, Ab};
    CF_TRY(params_check(e, tc));
    for (int k = 0; k < 6; ++k) {
        if (!t[k]) continue;
        int64_t n = 0;
        table_ptr(e, k, &n);
        CF_TRY(cf_get_table(e, k, t[k], n));
    }
    return CF_OK;
}

int cf_step(cf_engine* e, const int32_t* pairs, const int32_t* negs, const int32_t* groups,
            int32_t B, double* loss_out) {
    CF_TRY(check_engine(e));
    if (e->cfg.model == CF_PLR) return fail(CF_EINVAL, "tuple models step through cf_step_plr");
    CF_TRY(discard_pending(e));
    CF_TRY(check_not_xchg(e));
    if (B < 1) return fail(CF_EINVAL, "B must be >= 1");
    if (!pairs) return fail(CF_EINVAL, "host batch required (use cf_train_steps for the device sampler)");
    if (e->cfg.dense_item_apply && e->GV != e->GV_own)
        return fail(CF_ESTATE, "item gradient is bound to an external buffer: use cf_step_local/cf_step_items");
    double* acc = loss_out ? e->loss + 1 : e->loss;
    CF_TRY(run_step(e, B, pairs, negs, groups, acc));
    if (e->cfg.dense_item_apply) CF_TRY(run_items_dense(e));
    if (loss_out) CF_TRY(read_loss(e, 1, loss_out));
    if (e->det) CF_TRY(check_fx(e));
    return CF_OK;
}

int cf_step_plr(cf_engine* e, const int32_t* tuples, int32_t width, const float* coefs, int32_t B,
                double* loss_out) {
    CF_TRY(check_engine(e));
    CF_TRY(discard_pending(e));
    const cf_config& c = e->cfg;
    if (c.model != CF_PLR) return fail(CF_EINVAL, "cf_step_plr needs model CF_PLR");
    if (B < 1 || !tuples) return fail(CF_EINVAL, "bad arguments");
    if (width != c.n_neg + 2) return fail(CF_EINVAL, "tuple width must be n_neg + 2");
    if (c.plr_kind == CF_PLR_CPLR && !coefs) return fail(CF_EINVAL, "CPLR needs coefs [B, 2]");
    if (c.plr_kind == CF_PLR_CPLR) {
        CF_HIP(hipStreamSynchronize(e->stream));  // the previous step may still read the buffer
        if (B > e->coefs_cap) {
            dfree(e->coefs);
            CF_TRY(dalloc(&e->coefs, (size_t)B * 2));
            e->coefs_cap = B;
        }
        CF_HIP(hipMemcpy(e->coefs, coefs, (size_t)B * 2 * sizeof(float), hipMemcpyDefault));
    }
    double* acc = loss_out ? e->loss + 1 : e->loss;
    // ids straight from the tuples: u, i at columns 0, 1; the rest as negatives
    e->tuple_stride = width;
    const int r = run_step(e, B, tuples, tuples + 2, nullptr, acc);
    e->tuple_stride = 0;
    CF_TRY(r);
    if (loss_out) CF_TRY(read_loss(e, 1, loss_out));
    return CF_OK;
}

int cf_train_steps(cf_engine* e, int32_t B, int32_t n_steps, double* loss_sum_out) {
    CF_TRY(check_engine(e));
    if (e->cfg.model == CF_PLR) return fail(CF_EINVAL, "tuple models are host-fed (cf_step_plr)");
    CF_TRY(discard_pending(e));
    CF_TRY(check_not_xchg(e));
    if (B < 1 || n_steps < 0) return fail(CF_EINVAL, "bad B / n_steps");
    if (e->cfg.dense_item_apply && e->GV != e->GV_own)
        return fail(CF_ESTATE, "item gradient is bound to an external buffer: use cf_step_local/cf_step_items");
    double* acc = loss_sum_out ? e->loss + 1 : e->loss;
    if (e->cfg.dense_item_apply) {
        for (int s = 0; s < n_steps; ++s) {
            CF_TRY(run_step(e, B, nullptr, nullptr, nullptr, acc));
            CF_TRY(run_items_dense(e));
        }
    } else if (e->pipeline) {
        CF_TRY(run_steps_device(e, B, n_steps, acc));
    } else {
        for (int s = 0; s < n_steps; ++s) CF_TRY(run_step(e, B, nullptr, nullptr, nullptr, acc));
    }
    if (loss_sum_out) CF_TRY(read_loss(e, 1, loss_sum_out));
    if (e->det) CF_TRY(check_fx(e));
    return CF_OK;
}

// One training epoch of the device sampler, as one iteration of the
// reference's loop: n_batches = int(len(pairs) / batch_size) steps
// (bprmf.py:138-148), their mean pre-update batch loss as TraLoss
// (aveloss = np.mean(losses), bprmf.py:150).  The steps end at an epoch
// boundary: from a boundary (or after steps at another B) that is a whole
// epoch; from inside an epoch, the batches it has left.
int cf_train_epoch(cf_engine* e, int32_t B, double* mean_loss_out) {
    CF_TRY(check_engine(e));
    if (B < 1) return fail(CF_EINVAL, "B must be >= 1");
    if (!e->pairs) return fail(CF_ESTATE, "no interactions: call cf_set_interactions first");
    if ((int64_t)B > e->nnz) return fail(CF_EINVAL, "batch size exceeds the number of interactions");
    CF_TRY(discard_pending(e));   // the sampler position a caller sees
    const int64_t per_epoch = e->nnz / B;
    int64_t left = per_epoch;
    // sampler_args keeps the position when the batch size is this one, or
    // not yet set (cf_set_sampler_state on a fresh engine)
    if ((e->sampler_B == B || e->sampler_B == 0) && e->batch > 0 && e->batch < per_epoch)
        left = per_epoch - e->batch;
    if (left > INT32_MAX) return fail(CF_EINVAL, "epoch too long for one call");
    double sum = 0.0;
    CF_TRY(cf_train_steps(e, B, (int32_t)left, mean_loss_out ? &sum : nullptr));
    if (mean_loss_out) *mean_loss_out = sum / (double)left;
    return CF_OK;
}

int cf_sample(cf_engine* e, int32_t B, int32_t* pairs, int32_t* negs, int32_t* groups) {
    CF_TRY(check_engine(e));
    CF_TRY(discard_pending(e));
    const cf_config& c = e->cfg;
    if (B < 1 || !pairs || !negs) return fail(CF_EINVAL, "bad arguments");
    const int W = c.n_neg, G = group_count(c);
    if (G > 0 && !groups) return fail(CF_EINVAL, "GBPR needs a groups buffer");
    CF_TRY(ensure_batch(e, B));
    const int k = e->set;
    e->set ^= 1;
    StepArgs a = base_step_args(e, B, k);
    if (a.det_fx && e->fx_step > 0) e->fx_step -= 1;   // a draw, not a step: no range-flag word
    CF_TRY(sampler_args(e, B, &a));
    a.count_users = 0;
    a.count_items = 0;
    hipStream_t ps = e->prep_side ? e->side : e->stream;
    if (e->prep_side) CF_HIP(hipStreamWaitEvent(ps, e->apply_done[k], 0));
    CF_HIP(launch_prep(a, ps));
    const size_t nU = (size_t)B * (1 + G), nV = (size_t)B * (1 + W);
    std::vector<int32_t> hu(nU), hv(nV);
    CF_HIP(hipStreamSynchronize(ps));
    CF_HIP(hipMemcpy(hu.data(), e->occU_[k], nU * 4, hipMemcpyDeviceToHost));
    CF_HIP(hipMemcpy(hv.data(), e->occV_[k], nV * 4, hipMemcpyDeviceToHost));
    for (int p = 0; p < B; ++p) {
        pairs[2 * p] = hu[p];
        pairs[2 * p + 1] = hv[p];
        for (int w = 0; w < W; ++w) negs[(size_t)p * W + w] = hv[B + (size_t)p * W + w];
        for (int k = 0; k < G; ++k) {
            const int32_t g = hu[B + (size_t)p * G + k];
            // sharded engine: group members as GLOBAL user ids
            groups[(size_t)p * G + k] = e->world > 1 ? (g >= 0 ? (int32_t)(g + e->shard_u0) : -1 - g) : g;
        }
    }
    return CF_OK;
}

int cf_get_sampler_state(cf_engine* e, int64_t* epoch, int64_t* batch) {
    if (!e) return fail(CF_EINVAL, "null engine");
    if (e->x_pend) {  // an exchange batch drawn ahead is not consumed yet
        if (epoch) *epoch = e->x_pend_epoch;
        if (batch) *batch = e->x_pend_batch;
        return CF_OK;
    }
    if (e->pend) {  // a batch drawn ahead is not consumed yet
        if (epoch) *epoch = e->pend_epoch;
        if (batch) *batch = e->pend_batch;
        return CF_OK;
    }
    if (epoch) *epoch = e->epoch;
    if (batch) *batch = e->batch;
    return CF_OK;
}

int cf_set_sampler_state(cf_engine* e, int64_t epoch, int64_t batch) {
    if (e && e->pend) CF_TRY(discard_pending(e));
    if (!e) return fail(CF_EINVAL, "null engine");
    if (epoch < 0 || batch < 0) return fail(CF_EINVAL, "negative sampler state");
    e->epoch = epoch;
    e->batch = batch;
    return CF_OK;
}

int cf_begin_phase(cf_engine* e, int32_t phase) {
    CF_TRY(check_engine(e));
    CF_TRY(discard_pending(e));
    const cf_config& c = e->cfg;
    if (c.model != CF_AMF) return fail(CF_EINVAL, "phases exist only for AMF");
    if (phase != 0 && phase != 1) return fail(CF_EINVAL, "phase must be 0 or 1");
    if (phase == e->phase) return CF_OK;
    // each phase's train op owns its own AdagradOptimizer (amf.py:208-209):
    // its accumulators are still at acc_init when the phase starts
    CF_HIP(launch_fill(e->AU, c.n_users * (int64_t)c.n_factors, c.acc_init, e->stream));
    CF_HIP(launch_fill(e->AV, c.n_items * (int64_t)c.n_factors, c.acc_init, e->stream));
    e->phase = phase;
    return CF_OK;
}

int cf_bind_item_grad(cf_engine* e, void* ptr, int64_t n) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (!c.dense_item_apply) return fail(CF_ESTATE, "cf_bind_item_grad needs dense_item_apply=1");
    const int64_t id = c.n_items * (int64_t)c.n_factors;
    const int64_t want = id + (has_bias(c) ? c.n_items : 0);
    if (n != want) return fail(CF_EINVAL, "item-grad buffer must hold " + std::to_string(want) + " floats");
    if (!ptr) {
        e->GV = e->GV_own;
        e->Gb = e->Gb_own;
        return CF_OK;
    }
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, ptr) != hipSuccess || attr.type != hipMemoryTypeDevice)
        return fail(CF_EINVAL, "item-grad buffer is not device memory");
    e->GV = (float*)ptr;
    e->Gb = has_bias(c) ? (float*)ptr + id : e->Gb_own;
    CF_HIP(hipMemsetAsync(ptr, 0, (size_t)n * 4, e->stream));
    return CF_OK;
}

int cf_bind_apr_item_grad(cf_engine* e, void* ptr, int64_t n) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (c.amf_mode != CF_AMF_APR || !c.dense_item_apply)
        return fail(CF_ESTATE, "cf_bind_apr_item_grad needs amf_mode apr and dense_item_apply=1");
    if (e->lg_stage != 0) return fail(CF_ESTATE, "a split step is in progress");
    const int64_t id = c.n_items * (int64_t)c.n_factors;
    if (n != id) return fail(CF_EINVAL, "apr item buffer must hold " + std::to_string(id) + " floats");
    if (!ptr) {
        e->GadvV_bound = nullptr;
        return CF_OK;
    }
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, ptr) != hipSuccess || attr.type != hipMemoryTypeDevice)
        return fail(CF_EINVAL, "apr item buffer is not device memory");
    CF_HIP(hipMemsetAsync(ptr, 0, (size_t)n * 4, e->stream));
    e->GadvV_bound = (float*)ptr;
    return CF_OK;
}

// the split step's batch: drawn + counted by the previous apply launch, or
// drawn / packed now
static int local_batch(cf_engine* e, int32_t B, const int32_t* pairs, const int32_t* negs,
                       const int32_t* groups, StepArgs* a, int* k) {
    if (e->pend && (pairs || e->pend_B != B)) CF_TRY(discard_pending(e));
    CF_TRY(ensure_batch(e, B));
    if (e->pend) {
        *a = e->pend_args;
        *k = e->pend_set;
        e->pend = false;
    } else {
        *k = e->set;
        e->set ^= 1;
        CF_TRY(begin_step(e, B, pairs, negs, groups, *k, e->stream, a));
    }
    return CF_OK;
}

int cf_step_local_apr_embed(cf_engine* e, int32_t B, const int32_t* pairs, const int32_t* negs) {
    CF_TRY(check_engine(e));
    if (!e->cfg.dense_item_apply) return fail(CF_ESTATE, "the split step needs dense_item_apply=1");
    if (B < 1) return fail(CF_EINVAL, "B must be >= 1");
    if (e->lg_stage != 0) return fail(CF_ESTATE, "cf_step_local_apply of the previous step is missing");
    if (e->cfg.amf_mode != CF_AMF_APR || e->phase != 1)
        return fail(CF_ESTATE, "cf_step_local_apr_embed: amf_mode apr in the adversarial phase only");
    if (!e->GadvV_bound) return fail(CF_ESTATE, "bind the apr item buffer first (cf_bind_apr_item_grad)");
    StepArgs a;
    int k;
    CF_TRY(local_batch(e, B, pairs, negs, nullptr, &a, &k));
    {
        ProfScope ps(e, CF_K_STEP);
        CF_HIP(launch_apr_embed(a, e->stream));
    }
    e->lg_args = a;
    e->lg_set = k;
    e->lg_B = B;
    e->lg_stage = 3;   // the caller all-reduces the bound buffer, then cf_step_local_grad
    return CF_OK;
}

int cf_step_local_grad(cf_engine* e, int32_t B, const int32_t* pairs, const int32_t* negs,
                       const int32_t* groups) {
    CF_TRY(check_engine(e));
    if (!e->cfg.dense_item_apply) return fail(CF_ESTATE, "the split step needs dense_item_apply=1");
    CF_TRY(check_not_xchg(e));
    if (B < 1) return fail(CF_EINVAL, "B must be >= 1");
    StepArgs a;
    int k;
    if (e->lg_stage == 3) {   // after cf_step_local_apr_embed + the caller's all-reduce
        if (pairs || negs || groups || B != e->lg_B)
            return fail(CF_EINVAL, "after cf_step_local_apr_embed pass the same B and no batch");
        a = e->lg_args;
        k = e->lg_set;
        a.apr_embed_done = 1;
        e->lg_stage = 0;
    } else {
        if (e->lg_stage != 0) return fail(CF_ESTATE, "cf_step_local_apply of the previous step is missing");
        if (e->cfg.amf_mode == CF_AMF_APR && e->phase == 1)
            return fail(CF_ESTATE, "amf_mode apr: cf_step_local_apr_embed and the all-reduce of the bound "
                                   "buffer come first");
        CF_TRY(local_batch(e, B, pairs, negs, groups, &a, &k));
    }
    CF_TRY(det_ranks(e, a));
    CF_TRY(psort(e, a));
    {
        ProfScope ps(e, CF_K_STEP);
        CF_HIP(launch_grad(a, e->stream));
    }
    CF_TRY(det_hot(e, a));
    e->last_occV = a.occV;
    e->last_nV = (int64_t)B * items_per_pair(e->cfg);
    e->lg_pieces_left = 0;
    e->lg_pieces_deferred = false;
    if (a.items_grad_only && a.capV > 0) {
        // duplicated item rows: slot rows summed into the bound buffer now, so
        // it holds this rank's complete item gradient when the all-reduce starts
        ApplyArgs p = apply_args(e, a, B, k, nullptr);
        p.count_users = 0;
        if (e->item_pieces > 1 && p.dense_items) {
            // in pieces of item rows, each launched by cf_step_item_reduce just
            // before the caller's collective of that piece
            e->lg_pieces_left = e->item_pieces;
            e->lg_pieces_deferred = true;
        } else {
            ProfScope ps(e, CF_K_ITEM_REDUCE);
            CF_HIP(launch_apply(p, e->stream));
        }
    }
    e->lg_args = a;
    e->lg_set = k;
    e->lg_B = B;
    e->lg_stage = 1;
    return CF_OK;
}

// item rows [piece * chunk, (piece + 1) * chunk) of the local step's item
// reduce, chunk = n_items / n_pieces rounded up to 16 (kGroupsPerBlock)
static void piece_rows(int64_t n_items, int piece, int n_pieces, int64_t* r0, int64_t* r1) {
    int64_t chunk = (n_items + n_pieces - 1) / n_pieces;
    chunk = (chunk + kGroupsPerBlock - 1) / kGroupsPerBlock * kGroupsPerBlock;
    *r0 = std::min<int64_t>((int64_t)piece * chunk, n_items);
    *r1 = std::min<int64_t>(*r0 + chunk, n_items);
}

int cf_item_piece_rows(cf_engine* e, int32_t piece, int32_t n_pieces, int64_t* row0, int64_t* row1) {
    CF_TRY(check_engine(e));
    if (n_pieces < 1 || piece < 0 || piece >= n_pieces || !row0 || !row1) return fail(CF_EINVAL, "bad piece");
    piece_rows(e->cfg.n_items, piece, n_pieces, row0, row1);
    return CF_OK;
}

int cf_step_item_reduce(cf_engine* e, int32_t piece) {
    CF_TRY(check_engine(e));
    if (e->lg_stage != 1) return fail(CF_ESTATE, "cf_step_local_grad must come first");
    const int P = e->item_pieces;
    if (piece < 0 || piece >= P) return fail(CF_EINVAL, "piece must be 0 .. item_pieces-1");
    // the local step reduced its items whole (item_pieces 1, or not the
    // dense pos_sort apply): every piece is already complete
    if (!e->lg_pieces_deferred) return CF_OK;
    if (piece != P - e->lg_pieces_left) return fail(CF_ESTATE, "item-reduce pieces run in order 0 .. item_pieces-1");
    ApplyArgs p = apply_args(e, e->lg_args, e->lg_B, e->lg_set, nullptr);
    p.count_users = 0;
    piece_rows(e->cfg.n_items, piece, P, &p.item_r0, &p.item_r1);
    if (p.item_r1 > p.item_r0) {
        ProfScope ps(e, CF_K_ITEM_REDUCE);
        CF_HIP(launch_apply(p, e->stream));
    }
    e->lg_pieces_left -= 1;
    return CF_OK;
}

int cf_step_local_apply(cf_engine* e, int32_t next_B) {
    CF_TRY(check_engine(e));
    if (e->lg_stage != 1) return fail(CF_ESTATE, "cf_step_local_grad must come first");
    if (e->lg_pieces_left > 0)
        return fail(CF_ESTATE, "cf_step_item_reduce pieces of this step are still pending");
    if (next_B < 0) return fail(CF_EINVAL, "next_B must be >= 0");
    const int k = e->lg_set;
    ApplyArgs p = apply_args(e, e->lg_args, e->lg_B, k, e->loss);
    if (p.items_grad_only) p.count_items = 0;  // reduced in cf_step_local_grad
    e->lg_stage = 0;
    e->lg_done_set = k;
    if (next_B > 0 && next_B <= e->Bcap && e->prep_side == 0) {
        // draw + count the next batch in the same launch (other buffer set)
        StepArgs nx = base_step_args(e, next_B, k ^ 1);
        e->pend_epoch = e->epoch;
        e->pend_batch = e->batch;
        e->pend_sampler_B = e->sampler_B;
        CF_TRY(sampler_args(e, next_B, &nx));
        {
            ProfScope ps(e, CF_K_APPLY_PREP);
            CF_HIP(launch_apply_prep(p, nx, e->stream));
        }
        e->pend = true;
        e->pend_args = nx;
        e->pend_set = k ^ 1;
        e->pend_B = next_B;
        e->set = k;  // the set after the pending one
    } else {
        ProfScope ps(e, CF_K_APPLY);
        CF_HIP(launch_apply(p, e->stream));
    }
    return pending_clips(e);
}

int cf_step_local_draw(cf_engine* e, int32_t B) {
    CF_TRY(check_engine(e));
    if (!e->cfg.dense_item_apply) return fail(CF_ESTATE, "the split step needs dense_item_apply=1");
    CF_TRY(check_not_xchg(e));
    if (e->lg_stage != 0 || e->lg_done_set < 0)
        return fail(CF_ESTATE, "cf_step_local_draw follows cf_step_local_apply");
    if (e->pend) return fail(CF_ESTATE, "the next batch is already drawn");
    if (B < 1 || B > e->Bcap) return fail(CF_EINVAL, "B must be in [1, the largest batch stepped so far]");
    const int k = e->lg_done_set;
    StepArgs nx = base_step_args(e, B, k ^ 1);
    e->pend_epoch = e->epoch;
    e->pend_batch = e->batch;
    e->pend_sampler_B = e->sampler_B;
    CF_TRY(sampler_args(e, B, &nx));
    {
        ProfScope ps(e, CF_K_SAMPLE);
        CF_HIP(launch_prep(nx, e->stream));
    }
    e->pend = true;
    e->pend_args = nx;
    e->pend_set = k ^ 1;
    e->pend_B = B;
    e->set = k;
    return CF_OK;
}

int cf_step_local(cf_engine* e, int32_t B, const int32_t* pairs, const int32_t* negs,
                  const int32_t* groups) {
    CF_TRY(check_engine(e));
    if (e->cfg.amf_mode == CF_AMF_APR && e->phase == 1 && e->cfg.dense_item_apply) {
        // apr with no caller collective: this rank's sum is taken as the
        // global one (exact at world size 1)
        CF_TRY(cf_step_local_apr_embed(e, B, pairs, negs));
        CF_TRY(cf_step_local_grad(e, B, nullptr, nullptr, nullptr));
    } else {
        CF_TRY(cf_step_local_grad(e, B, pairs, negs, groups));
    }
    // the one-call form has no caller collective between item-reduce pieces
    // (item_pieces > 1 defers them): reduce every remaining piece here, so the
    // apply finds the item gradient complete
    while (e->lg_pieces_left > 0) CF_TRY(cf_step_item_reduce(e, e->item_pieces - e->lg_pieces_left));
    return cf_step_local_apply(e, 0);
}

int cf_step_items(cf_engine* e) {
    CF_TRY(check_engine(e));
    if (!e->cfg.dense_item_apply) return fail(CF_ESTATE, "cf_step_items needs dense_item_apply=1");
    e->last_nV = 0;   // the dense apply re-zeroes what it consumes
    return run_items_dense(e);
}

int cf_bind_table(cf_engine* e, int32_t t, void* ptr, int64_t n) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (t != CF_TABLE_ITEM && t != CF_TABLE_BIAS && t != CF_TABLE_ACC_ITEM && t != CF_TABLE_ACC_BIAS)
        return fail(CF_EINVAL, "only the item-side tables (item, bias and their accumulators) can be bound");
    int64_t want = 0;
    float** slot = table_slot(e, t);
    if (!table_ptr(e, t, &want)) return fail(CF_EINVAL, "table not present in this model");
    CF_TRY(discard_pending(e));
    CF_HIP(hipStreamSynchronize(e->stream));
    if (!ptr) {
        if (e->own_tab[t]) {
            CF_HIP(hipMemcpyAsync(e->own_tab[t], *slot, (size_t)want * 4, hipMemcpyDeviceToDevice, e->stream));
            CF_HIP(hipStreamSynchronize(e->stream));
            *slot = e->own_tab[t];
            e->own_tab[t] = nullptr;
        }
        return CF_OK;
    }
    if (n < want) return fail(CF_EINVAL, "bound table must hold at least " + std::to_string(want) + " floats");
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, ptr) != hipSuccess || attr.type != hipMemoryTypeDevice)
        return fail(CF_EINVAL, "bound table is not device memory");
    if ((float*)ptr == *slot) return CF_OK;
    CF_HIP(hipMemcpyAsync(ptr, *slot, (size_t)want * 4, hipMemcpyDeviceToDevice, e->stream));
    CF_HIP(hipStreamSynchronize(e->stream));
    if (!e->own_tab[t]) e->own_tab[t] = *slot;
    *slot = (float*)ptr;
    (void)c;
    return CF_OK;
}

int cf_bind_item_grad_split(cf_engine* e, void* gv, int64_t gv_n, void* gb, int64_t gb_n) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (!c.dense_item_apply) return fail(CF_ESTATE, "cf_bind_item_grad_split needs dense_item_apply=1");
    if (!gv) {
        e->GV = e->GV_own;
        e->Gb = e->Gb_own;
        return CF_OK;
    }
    const int64_t id = c.n_items * (int64_t)c.n_factors;
    if (gv_n < id) return fail(CF_EINVAL, "item-grad buffer must hold at least " + std::to_string(id) + " floats");
    CF_TRY(check_device_ptr(gv, "item-grad buffer"));
    if (has_bias(c)) {
        if (gb_n < c.n_items) return fail(CF_EINVAL, "bias-grad buffer must hold at least n_items floats");
        CF_TRY(check_device_ptr(gb, "bias-grad buffer"));
    }
    e->GV = (float*)gv;
    e->Gb = has_bias(c) ? (float*)gb : e->Gb_own;
    CF_HIP(hipMemsetAsync(gv, 0, (size_t)gv_n * 4, e->stream));
    if (has_bias(c)) CF_HIP(hipMemsetAsync(gb, 0, (size_t)gb_n * 4, e->stream));
    e->last_nV = 0;
    return CF_OK;
}

int cf_clear_item_grad(cf_engine* e) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (!c.dense_item_apply) return fail(CF_ESTATE, "cf_clear_item_grad needs dense_item_apply=1");
    if (e->last_nV <= 0) return CF_OK;
    float* gb = has_bias(c) ? e->Gb : nullptr;
    if (2 * e->last_nV < c.n_items) {
        CF_HIP(launch_zero_rows(e->last_occV, e->last_nV, e->GV, gb, c.n_factors, e->stream));
    } else {
        CF_HIP(hipMemsetAsync(e->GV, 0, (size_t)c.n_items * c.n_factors * 4, e->stream));
        if (gb) CF_HIP(hipMemsetAsync(gb, 0, (size_t)c.n_items * 4, e->stream));
    }
    e->last_nV = 0;
    return CF_OK;
}

int cf_step_items_range(cf_engine* e, int64_t row0, int64_t row1, const void* grad,
                        const void* grad_bias) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (!c.dense_item_apply) return fail(CF_ESTATE, "cf_step_items_range needs dense_item_apply=1");
    if (row0 < 0 || row1 < row0) return fail(CF_EINVAL, "bad row range");
    row0 = std::min<int64_t>(row0, c.n_items);
    row1 = std::min<int64_t>(row1, c.n_items);
    if (row1 > row0) {
        CF_TRY(check_device_ptr(grad, "grad"));
        if (has_bias(c)) CF_TRY(check_device_ptr(grad_bias, "grad_bias"));
        DenseArgs d{};
        d.d = c.n_factors;
        d.lr = c.lr;
        d.clip_norm = c.clip_norm;
        d.clip = c.model == CF_CML ? 1 : 0;
        d.zero_g = 0;
        d.n_rows = row1 - row0;
        d.X = e->V + row0 * c.n_factors;
        d.A = e->AV + row0 * c.n_factors;
        d.G = (float*)grad;
        if (has_bias(c)) {
            d.b = e->b + row0;
            d.Ab = e->Ab + row0;
            d.Gb = (float*)grad_bias;
        }
        {
            ProfScope ps(e, CF_K_APPLY_DENSE);
            CF_HIP(launch_apply_dense(d, e->stream));
        }
        if (e->need_clip_V) {   // CML: this rank's rows of the pending full clip
            ProfScope ps(e, CF_K_CLIP);
            CF_HIP(launch_clip_full(e->V + row0 * c.n_factors, row1 - row0, c.n_factors, c.clip_norm,
                                    e->stream));
        }
    }
    e->need_clip_V = false;
    return CF_OK;
}

// ---- user sharding + GBPR group exchange ------------------------------------
int cf_set_shard(cf_engine* e, int32_t world, int32_t rank, const int64_t* bounds) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (world < 1 || world > 64 || rank < 0 || rank >= world || !bounds)
        return fail(CF_EINVAL, "bad world / rank / bounds");
    if (bounds[0] != 0) return fail(CF_EINVAL, "bounds[0] must be 0");
    for (int r = 0; r < world; ++r)
        if (bounds[r + 1] < bounds[r]) return fail(CF_EINVAL, "bounds must be non-decreasing");
    if (bounds[world] > INT32_MAX) return fail(CF_EINVAL, "global user ids must fit int32");
    if (bounds[rank + 1] - bounds[rank] != c.n_users)
        return fail(CF_EINVAL, "this rank's user range must hold exactly n_users users");
    CF_HIP(hipStreamSynchronize(e->stream));
    e->world = world;
    e->rank = rank;
    e->shard_u0 = bounds[rank];
    e->shard_u1 = bounds[rank + 1];
    e->h_bounds.assign(bounds, bounds + world + 1);
    dfree(e->bounds);
    dfree(e->xcounts);
    CF_TRY(dalloc(&e->bounds, (size_t)world + 1));
    CF_TRY(dalloc(&e->xcounts, (size_t)world + 1));
    if (!e->h_xcounts)
        CF_HIP(hipHostMalloc((void**)&e->h_xcounts, 65 * sizeof(int32_t), hipHostMallocDefault));
    CF_HIP(hipMemcpy(e->bounds, bounds, ((size_t)world + 1) * 8, hipMemcpyHostToDevice));
    return CF_OK;
}

int cf_set_group_source(cf_engine* e, const int64_t* indptr_t, const int32_t* indices_t, int64_t nnz) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (c.model != CF_GBPR) return fail(CF_EINVAL, "group sources exist only for GBPR");
    if (e->h_bounds.empty()) return fail(CF_ESTATE, "call cf_set_shard first");
    if (!indptr_t || !indices_t || nnz < 1) return fail(CF_EINVAL, "null / empty item->user CSR");
    if (indptr_t[0] != 0 || indptr_t[c.n_items] != nnz) return fail(CF_EINVAL, "indptr_t does not span nnz");
    const int64_t nu = e->h_bounds[e->world];
    for (int64_t i = 0; i < c.n_items; ++i)
        if (indptr_t[i + 1] < indptr_t[i]) return fail(CF_EINVAL, "indptr_t not monotone");
    for (int64_t k = 0; k < nnz; ++k)
        if (indices_t[k] < 0 || indices_t[k] >= nu) return fail(CF_EINVAL, "user id out of range");
    CF_HIP(hipStreamSynchronize(e->stream));
    dfree(e->indptr_t);
    dfree(e->indices_t);
    CF_TRY(dalloc(&e->indptr_t, (size_t)c.n_items + 1));
    CF_TRY(dalloc(&e->indices_t, (size_t)nnz));
    CF_HIP(hipMemcpy(e->indptr_t, indptr_t, ((size_t)c.n_items + 1) * 8, hipMemcpyHostToDevice));
    CF_HIP(hipMemcpy(e->indices_t, indices_t, (size_t)nnz * 4, hipMemcpyHostToDevice));
    e->group_source_global = true;
    return CF_OK;
}

int cf_bind_exchange(cf_engine* e, void* send_ids, void* rows, void* grads, int64_t send_cap,
                     void* recv_ids, void* serve_rows, void* serve_grads, int64_t recv_cap) {
    CF_TRY(check_engine(e));
    if (e->x_stage != 0) return fail(CF_ESTATE, "an exchange step is in progress");
    if (send_cap < 0 || recv_cap < 0) return fail(CF_EINVAL, "negative capacity");
    if (send_cap > 0) {
        CF_TRY(check_device_ptr(send_ids, "send_ids"));
        CF_TRY(check_device_ptr(rows, "rows"));
        CF_TRY(check_device_ptr(grads, "grads"));
    }
    if (recv_cap > 0) {
        CF_TRY(check_device_ptr(recv_ids, "recv_ids"));
        CF_TRY(check_device_ptr(serve_rows, "serve_rows"));
        CF_TRY(check_device_ptr(serve_grads, "serve_grads"));
    }
    e->x_send_ids = (int32_t*)send_ids;
    e->x_rows = (float*)rows;
    e->x_grads = (float*)grads;
    e->x_send_cap = send_cap;
    e->x_recv_ids = (int32_t*)recv_ids;
    e->x_serve_rows = (float*)serve_rows;
    e->x_serve_grads = (float*)serve_grads;
    dfree(e->x_own);
    CF_TRY(dalloc(&e->x_own, (size_t)(recv_cap > 0 ? recv_cap : 1)));
    e->x_recv_cap = recv_cap;
    return CF_OK;
}

static int check_xchg(cf_engine* e, int stage) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (c.model != CF_GBPR || !c.dense_item_apply || e->h_bounds.empty())
        return fail(CF_ESTATE, "the group exchange needs GBPR, dense_item_apply=1 and cf_set_shard");
    if (!e->group_source_global) return fail(CF_ESTATE, "set the global item->user CSR first (cf_set_group_source)");
    if (e->x_stage != stage) return fail(CF_ESTATE, "exchange calls out of order (begin, serve, grad, finish)");
    if (e->det) return fail(CF_ESTATE, "deterministic mode does not cover the GBPR group exchange (float atomics of served rows)");
    return CF_OK;
}

// draw (or stage) one exchange batch into buffer set k and pack its remote
// group members by owner into half k of send_ids; counts stay on the device
static int xchg_stage(cf_engine* e, int32_t B, const int32_t* pairs, const int32_t* negs,
                      const int32_t* groups, int k, int half, StepArgs* a) {
    if (B < 1) return fail(CF_EINVAL, "bad arguments");
    if (e->GV == e->GV_own) return fail(CF_ESTATE, "bind the item-gradient buffer first (cf_bind_item_grad)");
    const cf_config& c = e->cfg;
    const int n = B * group_count(c);
    if (n > e->x_send_cap) return fail(CF_EINVAL, "exchange send capacity < B * gsize (cf_bind_exchange)");
    CF_TRY(ensure_batch(e, B));
    CF_TRY(begin_step(e, B, pairs, negs, groups, k, e->stream, a));
    const size_t nblk = (size_t)(n + kBlock - 1) / kBlock;
    if (nblk * (size_t)e->world > e->xhist_cap) {
        CF_HIP(hipStreamSynchronize(e->stream));
        dfree(e->xhist);
        CF_TRY(dalloc(&e->xhist, nblk * (size_t)e->world));
        e->xhist_cap = nblk * (size_t)e->world;
    }
    XchgArgs x{};
    x.n = n;
    x.world = e->world;
    x.bounds = e->bounds;
    x.occ = e->occU_[k] + B;
    x.hist = e->xhist;
    x.counts = e->xcounts;
    x.send_ids = e->x_send_ids + (int64_t)half * e->x_send_cap;
    CF_HIP(launch_xchg_pack(x, e->stream));
    return CF_OK;
}

int cf_xchg_begin(cf_engine* e, int32_t B, const int32_t* pairs, const int32_t* negs,
                  const int32_t* groups, int32_t* send_counts_out) {
    CF_TRY(check_xchg(e, 0));
    if (!send_counts_out) return fail(CF_EINVAL, "bad arguments");
    CF_TRY(discard_pending(e));
    const int k = e->set;
    e->set ^= 1;
    StepArgs a;
    CF_TRY(xchg_stage(e, B, pairs, negs, groups, k, 0, &a));   // send_ids half 0
    CF_HIP(hipMemcpyAsync(e->h_xcounts, e->xcounts, ((size_t)e->world + 1) * 4, hipMemcpyDeviceToHost,
                          e->stream));
    CF_HIP(hipStreamSynchronize(e->stream));
    for (int r = 0; r < e->world; ++r) send_counts_out[r] = e->h_xcounts[r];
    e->x_args = a;
    e->x_set = k;
    e->x_B = B;
    e->x_stage = 1;
    e->x_part = 0;
    e->x_items_done = false;
    return CF_OK;
}

int cf_xchg_draw(cf_engine* e, int32_t B, void* send_counts_dev, int32_t* half_out) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (c.model != CF_GBPR || !c.dense_item_apply || e->h_bounds.empty() || !e->group_source_global)
        return fail(CF_ESTATE, "the group exchange needs GBPR, dense_item_apply=1, cf_set_shard and cf_set_group_source");
    if (e->det) return fail(CF_ESTATE, "deterministic mode does not cover the GBPR group exchange");
    if (e->x_pend) return fail(CF_ESTATE, "an exchange batch is already drawn (cf_xchg_adopt takes it)");
    if (!half_out) return fail(CF_EINVAL, "null half_out");
    CF_TRY(check_device_ptr(send_counts_dev, "send_counts_dev"));
    const int k = e->set;
    const int64_t ep = e->epoch, bt = e->batch;
    const int sb = e->sampler_B;
    e->set ^= 1;
    StepArgs a;
    CF_TRY(xchg_stage(e, B, nullptr, nullptr, nullptr, k, k, &a));
    CF_HIP(hipMemcpyAsync((int32_t*)send_counts_dev + (int64_t)k * e->world, e->xcounts,
                          (size_t)e->world * 4, hipMemcpyDeviceToDevice, e->stream));
    e->x_pend = true;
    e->x_pend_args = a;
    e->x_pend_set = k;
    e->x_pend_B = B;
    e->x_pend_epoch = ep;
    e->x_pend_batch = bt;
    e->x_pend_sampler_B = sb;
    *half_out = k;
    return CF_OK;
}

int cf_xchg_adopt(cf_engine* e, int32_t B) {
    CF_TRY(check_xchg(e, 0));
    if (!e->x_pend) return fail(CF_EAGAIN, "no exchange batch drawn ahead (cf_xchg_draw)");
    if (e->x_pend_B != B) {   // drawn at another batch size: drop it (uncount, rewind the sampler)
        const int drawn = e->x_pend_B;
        CF_TRY(discard_pending(e));
        return fail(CF_EAGAIN, "the batch drawn ahead has B=" + std::to_string(drawn) + ", not " +
                                   std::to_string(B) + ": discarded, draw again");
    }
    e->x_args = e->x_pend_args;
    e->x_set = e->x_pend_set;
    e->x_B = e->x_pend_B;
    e->x_pend = false;
    e->x_stage = 1;
    e->x_part = 0;
    e->x_items_done = false;
    return CF_OK;
}

int cf_xchg_serve(cf_engine* e, int64_t n_recv) {
    CF_TRY(check_xchg(e, 1));
    if (n_recv < 0 || n_recv > e->x_recv_cap) return fail(CF_EINVAL, "n_recv exceeds the bound receive capacity");
    CF_HIP(launch_xchg_serve(e->x_recv_ids, n_recv, e->shard_u0, e->cntU_[e->x_set], e->x_own, e->U,
                             e->x_serve_rows,
                             e->cfg.n_factors, e->stream));
    e->x_stage = 2;
    return CF_OK;
}

int cf_xchg_grad(cf_engine* e) {
    CF_TRY(check_xchg(e, 2));
    if (e->x_part != 0) return fail(CF_ESTATE, "a split gradient (cf_xchg_grad_part) is in progress");
    const StepArgs& a = e->x_args;
    {
        ProfScope ps(e, CF_K_STEP);
        CF_HIP(launch_grad(a, e->stream));
    }
    e->last_occV = a.occV;
    e->last_nV = (int64_t)e->x_B * items_per_pair(e->cfg);
    e->x_stage = 3;
    return CF_OK;
}

// split step: pairs whose group members are all local (part 1, beside the
// member-row all-to-all), then the others (part 2, after it); each part
// writes its own half of the loss partials
int cf_xchg_grad_part(cf_engine* e, int32_t part) {
    if (part == 0) return cf_xchg_grad(e);
    CF_TRY(check_xchg(e, 2));
    if (part != 1 && part != 2) return fail(CF_EINVAL, "part must be 0, 1 or 2");
    if (part != e->x_part + 1) return fail(CF_ESTATE, "gradient parts run in order: 1 (local members), then 2");
    StepArgs a = e->x_args;
    a.member_pass = part;
    if (part == 2) a.loss_partial = e->loss_partial + grad_blocks(e->x_args);
    {
        ProfScope ps(e, part == 1 ? CF_K_STEP : CF_K_STEP_REMOTE);
        CF_HIP(launch_grad(a, e->stream));
    }
    e->x_part = part;
    if (part == 2) {
        e->last_occV = a.occV;
        e->last_nV = (int64_t)e->x_B * items_per_pair(e->cfg);
        e->x_stage = 3;
    }
    return CF_OK;
}

// loss partials of this exchange step's gradient launch(es)
static int xchg_partials(cf_engine* e) { return grad_blocks(e->x_args) * (e->x_part == 2 ? 2 : 1); }

// split step: the item rows' summed gradient into the bound buffer (the item
// exchange can start), before the served gradients arrive for the users
int cf_xchg_finish_items(cf_engine* e) {
    CF_TRY(check_xchg(e, 3));
    if (e->x_items_done) return fail(CF_ESTATE, "the items of this exchange step are already finished");
    ApplyArgs p = apply_args(e, e->x_args, e->x_B, e->x_set, nullptr);   // the users' apply folds the loss
    p.count_users = 0;
    p.n_partial = xchg_partials(e);
    if (p.count_items) {
        ProfScope ps(e, CF_K_APPLY);
        CF_HIP(launch_apply(p, e->stream));
    }
    e->x_items_done = true;
    return CF_OK;
}

int cf_xchg_finish(cf_engine* e, int64_t n_recv) {
    CF_TRY(check_xchg(e, 3));
    if (n_recv < 0 || n_recv > e->x_recv_cap) return fail(CF_EINVAL, "n_recv exceeds the bound receive capacity");
    CF_HIP(launch_xchg_accumulate(e->x_recv_ids, n_recv, e->shard_u0, e->x_serve_grads, e->GU,
                                  e->cfg.n_factors, e->stream));
    ApplyArgs p = apply_args(e, e->x_args, e->x_B, e->x_set, e->loss);
    p.served_ids = e->x_recv_ids;   // served rows with no local occurrence apply here
    p.served_own = e->x_own;
    p.nS = n_recv;
    p.n_partial = xchg_partials(e);
    if (e->x_items_done) p.count_items = 0;
    {
        ProfScope ps(e, CF_K_APPLY);
        CF_HIP(launch_apply(p, e->stream));
    }
    e->x_stage = 0;
    e->x_part = 0;
    e->x_items_done = false;
    return CF_OK;
}

int cf_take_loss(cf_engine* e, double* out) {
    CF_TRY(check_engine(e));
    if (!out) return fail(CF_EINVAL, "null output");
    return read_loss(e, 0, out);
}

int cf_score_topk(cf_engine* e, const int32_t* users, int32_t n, int32_t k, const uint8_t* mask_or_NULL,
                  int32_t* idx_out, float* val_out) {
    // NULL: the reference's filter (each user's train items); a mask: exactly
    // the items it flags, for every user
    return cf_score_topk_ex(e, users, n, k, mask_or_NULL ? 0 : 1, mask_or_NULL, idx_out, val_out);
}

int cf_score_topk_ex(cf_engine* e, const int32_t* users, int32_t n, int32_t k, int32_t exclude_train,
                     const uint8_t* item_mask, int32_t* idx_out, float* val_out) {
    CF_TRY(check_engine(e));
    const cf_config& c = e->cfg;
    if (n < 0 || !idx_out || (n > 0 && !users)) return fail(CF_EINVAL, "bad arguments");
    if (k < 1 || k > 4096) return fail(CF_EINVAL, "k must be 1..4096");
    if (exclude_train && !e->indptr) return fail(CF_ESTATE, "exclude_train needs cf_set_interactions");
    if (n == 0) return CF_OK;
    // the caller's item mask (uint8 [n_items], host or device) as one bit per
    // item, 64 items per word -- the fused kernel ORs one word into each
    // 64-item tile's exclusion mask, the materialised path zeroes the keys
    const uint64_t* d_mask = nullptr;
    if (item_mask) {
        const int64_t nw = (c.n_items + 63) / 64;
        std::vector<uint8_t> hm;
        if (is_device_ptr(item_mask)) {
            hm.resize((size_t)c.n_items);
            CF_HIP(hipMemcpy(hm.data(), item_mask, (size_t)c.n_items, hipMemcpyDeviceToHost));
            item_mask = hm.data();
        }
        std::vector<uint64_t> bits((size_t)nw, 0ull);
        for (int64_t j = 0; j < c.n_items; ++j)
            if (item_mask[j]) bits[(size_t)(j >> 6)] |= 1ull << (j & 63);
        if (e->mask_words < nw) {
            dfree(e->item_mask);
            CF_TRY(dalloc(&e->item_mask, (size_t)nw));
            e->mask_words = nw;
        }
        CF_HIP(hipMemcpyAsync(e->item_mask, bits.data(), (size_t)nw * 8, hipMemcpyHostToDevice, e->stream));
        CF_HIP(hipStreamSynchronize(e->stream));   // `bits` is pageable and local
        d_mask = e->item_mask;
    }
    std::vector<int32_t> host_users;
    if (is_device_ptr(users)) {  // device ids (torch): checked from a host copy
        host_users.resize((size_t)n);
        CF_HIP(hipMemcpy(host_users.data(), users, (size_t)n * 4, hipMemcpyDeviceToHost));
        users = host_users.data();
    }
    for (int r = 0; r < n; ++r)
        if (users[r] < 0 || users[r] >= c.n_users) return fail(CF_EINVAL, "user id out of range");
    CF_HIP(hipStreamSynchronize(e->side));
    const bool fused_ok = k <= kFusedMaxWideK && c.n_factors <= kFusedMaxD;
    if (e->topk_path == 2 && !fused_ok)
        return fail(CF_EINVAL, "fused top-k needs k <= 128 and n_factors <= 128");
    if (fused_ok && e->topk_path != 1)
        return score_topk_fused(e, users, n, k, exclude_train, d_mask, idx_out, val_out);
    const size_t row_bytes = (size_t)c.n_items * 4;
    const size_t budget = (size_t)512 << 20;
    int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, budget / row_bytes));
    if ((size_t)chunk * row_bytes > e->keys_cap) {
        dfree(e->keys);
        CF_TRY(dalloc(&e->keys, (size_t)chunk * c.n_items));
        e->keys_cap = (size_t)chunk * row_bytes;
    }
    int32_t* d_users = nullptr;
    int32_t* d_idx = nullptr;
    float* d_val = nullptr;
    int r = CF_OK;
    if ((r = dalloc(&d_users, (size_t)n)) || (r = dalloc(&d_idx, (size_t)n * k)) ||
        (r = dalloc(&d_val, (size_t)n * k))) {
        dfree(d_users); dfree(d_idx); dfree(d_val);
        return r;
    }
    hipError_t he = hipMemcpyAsync(d_users, users, (size_t)n * 4, hipMemcpyHostToDevice, e->stream);
    for (int u0 = 0; he == hipSuccess && u0 < n; u0 += chunk) {
        const int m = std::min(chunk, n - u0);
        ScoreArgs s{};
        s.model = c.model == CF_PLR ? CF_GBPR : c.model;
        s.d = c.n_factors;
        s.n_users = m;
        s.n_items = c.n_items;
        s.users = d_users + u0;
        s.U = e->U;
        s.V = e->V;
        s.b = e->b;
        s.keys = e->keys;
        s.exclude_train = exclude_train ? 1 : 0;
        s.indptr = e->indptr;
        s.indices = e->indices;
        s.item_mask = d_mask;
        {
            ProfScope ps(e, CF_K_SCORE);
            he = launch_score(s, e->stream);
        }
        if (he != hipSuccess) break;
        TopkArgs t{};
        t.k = k;
        t.n_items = c.n_items;
        t.keys = e->keys;
        t.idx_out = d_idx + (size_t)u0 * k;
        t.val_out = d_val + (size_t)u0 * k;
        {
            ProfScope ps(e, CF_K_TOPK);
            he = launch_topk(t, m, e->stream);
        }
    }
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he == hipSuccess) he = hipMemcpy(idx_out, d_idx, (size_t)n * k * 4, hipMemcpyDefault);
    if (he == hipSuccess && val_out)
        he = hipMemcpy(val_out, d_val, (size_t)n * k * 4, hipMemcpyDefault);
    dfree(d_users); dfree(d_idx); dfree(d_val);
    if (he != hipSuccess) return fail(CF_EHIP, std::string("cf_score_topk: ") + hipGetErrorString(he));
    return CF_OK;
}

int cf_set_option(cf_engine* e, const char* name, int64_t value) {
    if (!e || !name) return fail(CF_EINVAL, "null argument");
    CF_TRY(set_dev(e));   // some options (re)allocate device buffers
    const std::string n(name);
    if (n == "dense_apply") {
        if (value < 0 || value > 1) return fail(CF_EINVAL, "dense_apply must be 0 or 1");
        e->dense_apply = (int)value;
        return CF_OK;
    }
    if (n == "fused_variant") {
        if (value < 0 || value > 3) return fail(CF_EINVAL, "fused_variant must be 0, 1, 2 or 3");
        e->fused_variant = (int)value;
        return CF_OK;
    }
    if (n == "topk_path") {
        if (value < 0 || value > 2) return fail(CF_EINVAL, "topk_path must be 0, 1 or 2");
        e->topk_path = (int)value;
        return CF_OK;
    }
    if (n == "item_pieces") {   // the multi-rank item reduce in pieces (cf_step_item_reduce)
        if (value < 1 || value > 64) return fail(CF_EINVAL, "item_pieces must be 1 .. 64");
        if (e->lg_stage != 0) return fail(CF_ESTATE, "a split step is in progress");
        e->item_pieces = (int)value;
        return CF_OK;
    }
    if (n == "sorted_batches") {   // each batch's pairs in CSR order (StepArgs::order)
        if (value < 0 || value > 3) return fail(CF_EINVAL, "sorted_batches must be 0, 1, 2 or 3");
        CF_TRY(discard_pending(e));
        e->sorted_batches = (int)value;
        e->sorted_auto_off = false;
        return CF_OK;
    }
    if (n == "user_runs") {   // StepArgs::user_runs
        if (value < 0 || value > 1) return fail(CF_EINVAL, "user_runs must be 0 or 1");
        CF_TRY(discard_pending(e));
        e->user_runs = (int)value;
        return CF_OK;
    }
    if (n == "epoch_sort") {   // how the sorted batches' epoch order is formed (epoch_need)
        if (value < 0 || value > 1) return fail(CF_EINVAL, "epoch_sort must be 0 or 1");
        CF_TRY(discard_pending(e));
        if (e->eo_stream) CF_HIP(hipStreamSynchronize(e->eo_stream));
        e->epoch_sort = (int)value;
        for (auto& o : e->eo) o.epoch = -1;   // recomputed in the new form
        return CF_OK;
    }
    if (n == "sorted_auto_reserve_mb") {   // HBM auto mode leaves free beside the orders (sorted_auto_fits)
        if (value < 0) return fail(CF_EINVAL, "sorted_auto_reserve_mb must be >= 0");
        CF_TRY(discard_pending(e));
        e->sorted_reserve_mb = value;
        e->sorted_auto_off = false;
        return CF_OK;
    }
    if (n == "spec_neg") {   // speculative negative counts in the pos_sort draw (StepArgs::spec_ph)
        if (value < 0 || value > 1) return fail(CF_EINVAL, "spec_neg must be 0 or 1");
        CF_TRY(discard_pending(e));   // a drawn-ahead batch was counted under the old setting
        e->spec_neg = (int)value;
        return CF_OK;
    }
    if (n == "pair_prefetch") {
        if (value < 0 || value > 1) return fail(CF_EINVAL, "pair_prefetch must be 0 or 1");
        if (value == 1 && !pair_prefetch_built())
            return fail(CF_EINVAL, "pair_prefetch: this build has the prefetch compiled out (-DCF_PAIR_PREFETCH=1)");
        e->pair_prefetch = (int)value;
        return CF_OK;
    }
    if (n == "prep_stream") {
        if (value < 0 || value > 1) return fail(CF_EINVAL, "prep_stream must be 0 or 1");
        CF_HIP(hipStreamSynchronize(e->stream));
        CF_HIP(hipStreamSynchronize(e->side));
        e->prep_side = (int)value;
        return CF_OK;
    }
    if (n == "profile_every") {
        if (value < 1 || value > 1 << 20) return fail(CF_EINVAL, "profile_every must be >= 1");
        e->prof_every = (int)value;
        return CF_OK;
    }
    if (n == "profile_mask") {
        e->prof_mask = (uint32_t)value;
        return CF_OK;
    }
    if (n == "pipeline") {
        if (value < 0 || value > 3) return fail(CF_EINVAL, "pipeline must be 0, 1, 2 or 3");
        CF_TRY(discard_pending(e));
        e->pipeline = (int)value;
        return CF_OK;
    }
    if (n == "slot_max" || n == "slot_max_user") {
        if (value < 1 || value > 256) return fail(CF_EINVAL, n + " must be in [1, 256]");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        if (n == "slot_max") {
            e->capV = (int)value;
        } else {
            e->capU = (int)value;
            e->capU_auto = false;
        }
        e->slots_ready = false;   // re-sized at the next step
        if (n == "slot_max_user") e->fx_cap = 0;   // the compact GU64 rows scale with 1 / (capU + 1)
        return CF_OK;
    }
    if (n == "hot_replicas") {
        if (value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
            return fail(CF_EINVAL, "hot_replicas must be 1, 2, 4, 8 or 16");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        e->hot_rep = (int)value;
        e->slots_ready = false;
        return CF_OK;
    }
    if (n == "neg_check") {
#ifdef CF_LANE_DRAW
        if (value < 0 || value > 2) return fail(CF_EINVAL, "neg_check must be 0, 1 or 2");
#else
        if (value < 0 || value > 1)
            return fail(CF_EINVAL, "neg_check must be 0 or 1 (2, the one-lane-per-pair draw, needs a -DCF_LANE_DRAW build)");
#endif
        CF_TRY(discard_pending(e));
        e->neg_check = (int)value;
        if (value >= 1 && e->pairs && !e->pos_set) CF_TRY(build_pos_set(e));
        return CF_OK;
    }
    if (n == "item_reduce") {
        if (value < 0 || value > 2) return fail(CF_EINVAL, "item_reduce must be 0, 1 or 2");
        if (e->lg_stage != 0 || e->x_stage != 0) return fail(CF_ESTATE, "a split step is in progress");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        e->item_reduce = (int)value;
        e->slots_ready = false;
        return CF_OK;
    }
    if (n == "bias_slots") {
        if (value < 0 || value > 1) return fail(CF_EINVAL, "bias_slots must be 0 or 1");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        e->bias_slots = (int)value;
        return CF_OK;
    }
    if (n == "item_slots") {   // 0: gradient rows, 1: (pair, alpha, beta) records + user-row stash
        if (value < 0 || value > 1) return fail(CF_EINVAL, "item_slots must be 0 or 1");
        if (value == 1 && e->cfg.amf_mode == CF_AMF_APR)
            return fail(CF_EINVAL, "item_slots 1 (records alpha * X + beta * V) cannot carry apr's perturbed rows");
        if (e->lg_stage != 0 || e->x_stage != 0) return fail(CF_ESTATE, "a split step is in progress");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        CF_HIP(hipStreamSynchronize(e->side));
        if (e->item_recs == (int)value) return CF_OK;
        e->item_recs = (int)value;
        e->slots_ready = false;      // slot rows <-> records
        e->det_cap = 0;              // deterministic buffers likewise
        if (e->Bcap > 0) {
            CF_TRY(ensure_slots(e));
            if (e->det) CF_TRY(ensure_det(e, e->Bcap, e->Bcap));
            CF_TRY(ensure_stash(e, e->Bcap));
        }
        return CF_OK;
    }
    if (n == "deterministic") {
        if (value < 0 || value > 1) return fail(CF_EINVAL, "deterministic must be 0 or 1");
        if (value == 1 && e->cfg.amf_mode == CF_AMF_APR)
            return fail(CF_EINVAL, "deterministic mode does not cover amf_mode apr (its Δ sums are float atomics)");
        if (e->lg_stage != 0 || e->x_stage != 0) return fail(CF_ESTATE, "a split step is in progress");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        e->det = (int)value;
        if (e->det && e->Bcap > 0) CF_TRY(ensure_det(e, e->Bcap, e->Bcap));
        return CF_OK;
    }
    if (n == "grad_path") {
        if (value < 0 || value > 3) return fail(CF_EINVAL, "grad_path must be 0, 1, 2 or 3");
        CF_TRY(discard_pending(e));   // a drawn-ahead batch was counted for the old path (pos_sort)
        e->grad_path = (int)value;
        return CF_OK;
    }
    if (n == "pos_sort" || n == "slot_max_pos") {
        if (n == "pos_sort" && (value < 0 || value > 2)) return fail(CF_EINVAL, "pos_sort must be 0, 1 or 2");
        if (n == "slot_max_pos" && (value < 1 || value > 256))
            return fail(CF_EINVAL, "slot_max_pos must be in [1, 256]");
        if (e->lg_stage != 0 || e->x_stage != 0) return fail(CF_ESTATE, "a split step is in progress");
        CF_TRY(discard_pending(e));
        CF_HIP(hipStreamSynchronize(e->stream));
        CF_HIP(hipStreamSynchronize(e->side));
        if (n == "pos_sort") e->pos_sort = (int)value; else e->capP = (int)value;
        e->slots_ready = false;
        if (e->Bcap > 0) {
            CF_TRY(ensure_slots(e));
            CF_TRY(ensure_order(e, e->Bcap));
        }
        return CF_OK;
    }
    return fail(CF_EINVAL, "unknown option " + n);
}

int cf_step_path(cf_engine* e, int32_t B, int32_t* flags_out) {
    if (!e || !flags_out) return fail(CF_EINVAL, "null argument");
    if (B < 1) return fail(CF_EINVAL, "B must be >= 1");
    const cf_config& c = e->cfg;
    StepArgs a{};
    a.model = c.model;
    a.d = c.n_factors;
    a.W = c.n_neg;
    a.G = group_count(c);
    a.grad_path = e->grad_path;
    int f = 0;
    if (grad_fast_w(a) != 0) f |= CF_PATH_PHASED;
    if (psort_active(e, B)) f |= CF_PATH_POS_SORT;
    else if (grad_lds(a)) f |= CF_PATH_LDS;   // (pos_sort takes the sorted kernel)
    if (e->item_recs && (!c.dense_item_apply || e->item_reduce)) f |= CF_PATH_ITEM_RECORDS;
    if (e->det) f |= CF_PATH_DETERMINISTIC;
    if (c.dense_item_apply) f |= CF_PATH_DENSE_ITEMS;
    if (e->pairs && sorted_batches_on(e, B)) f |= CF_PATH_SORTED_BATCHES;
    f |= (e->pipeline & 3) << 8;
    *flags_out = f;
    return CF_OK;
}

int cf_profile_enable(cf_engine* e, int32_t on) {
    if (!e) return fail(CF_EINVAL, "null engine");
    e->prof = on != 0;
    return CF_OK;
}

int cf_profile_read(cf_engine* e, int32_t kid, double* total_ms, int64_t* launches) {
    CF_TRY(check_engine(e));
    if (kid < 0 || kid >= CF_K_COUNT) return fail(CF_EINVAL, "bad kernel id");
    CF_HIP(hipStreamSynchronize(e->stream));
    double t = 0.0;
    for (auto& pr : e->ev[kid]) {
        float ms = 0.f;
        CF_HIP(hipEventSynchronize(pr.second));   // events of the epoch-order stream too
        CF_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = (int64_t)e->ev[kid].size();
    return CF_OK;
}

int cf_profile_reset(cf_engine* e) {
    CF_TRY(check_engine(e));
    CF_HIP(hipStreamSynchronize(e->stream));
    for (auto& n : e->prof_seen) n = 0;
    for (auto& v : e->ev) {
        for (auto& pr : v) {
            e->ev_pool.push_back(pr.first);
            e->ev_pool.push_back(pr.second);
        }
        v.clear();
    }
    return CF_OK;
}

}  // extern "C"

// errors of the other host translation units (cf_ingest.cpp)
namespace cfi {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace cfi
