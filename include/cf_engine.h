/*
 * cf_engine.h -- C ABI of the MI355X-native pairwise-ranking (BPR-style)
 * training engine.  Plain C, no torch / HIP types in any signature, so it is
 * callable from ctypes (stdlib), cffi, or any FFI.
 *
 * The reference (BinFuPKU/CollaborativeFilteringUsingTensorflow) has no native
 * layer: its hot path is duck-typed Python over TensorFlow-1 graphs.  Each
 * entry point below replaces one piece of that Python/TF surface; the
 * replaced reference code is cited per function (paths relative to the
 * reference repo root).  INTEGRATION.md shows the ctypes binding.
 *
 * Conventions
 *  - Every function returns 0 (CF_OK) on success or a negative cf_status;
 *    cf_last_error() returns a thread-local message for the last failure.
 *    No C++ exception crosses this boundary.
 *  - Caller buffers are borrowed for the call and copied; the engine owns
 *    all device memory.  Batches (cf_step, cf_step_local*, cf_xchg_begin,
 *    cf_step_plr), tables (cf_set_table / cf_get_table) and cf_score_topk's
 *    users / outputs may be host memory or HIP device memory (e.g.
 *    torch.Tensor.data_ptr()), told apart by a pointer-attribute query
 *    (SURVEY 8(b)); a device batch is unpacked and range-checked on the
 *    device.  A batch is all host or all device.  Device inputs must be
 *    complete (their producer stream synchronised) before the call.
 *  - A handle is not thread-safe: one handle per thread.  All device work is
 *    enqueued on the engine's HIP stream; functions that write host outputs
 *    synchronise that stream before returning.
 *  - Ids are 0-based int32 (users, items), CSR row pointers are int64.
 */
#ifndef CF_ENGINE_H
#define CF_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CF_ABI_VERSION 1

/* opaque handle: device tables, accumulators, CSR, sampler state, stream */
typedef struct cf_engine cf_engine;

/* model kinds -- the four ranking models on the hot path */
enum cf_model {
    CF_BPR = 0,   /* src/models/pl/models/bprmf.py   */
    CF_GBPR = 1,  /* src/models/pl/models/gbprmf.py  */
    CF_CML = 2,   /* src/models/pl/models/cml.py     */
    CF_AMF = 3,   /* src/models/others/models/amf.py */
    CF_PLR = 4    /* tuple ranking: PRIGP (prigp.py:99-130) / CPLR (cplr_u.py:106-137) */
};

enum cf_plr_kind {
    CF_PLR_PRIGP = 0,  /* (u,i,j,t,k): -log s(ui-uj) - alpha log s(ut-uk); U,V trained, b fixed */
    CF_PLR_CPLR = 1    /* (u,i,t,j)+(c_ui,c_ut): alpha/beta/gamma weighted, coefficient-scaled;
                          U,V,b trained */
};

enum cf_status {
    CF_OK = 0,
    CF_EINVAL = -1,   /* bad argument / shape                         */
    CF_EHIP = -2,     /* HIP runtime error (message has the HIP text)  */
    CF_ESTATE = -3,   /* call out of order (e.g. no interactions set)  */
    CF_ENOMEM = -4,   /* device or host allocation failed              */
    CF_EAGAIN = -5,   /* cf_xchg_adopt: no batch of that size drawn ahead
                         (none drawn, dropped, or drawn at another B and
                         now discarded): draw one (cf_xchg_draw) and retry */
    CF_ENUMERIC = -6  /* deterministic mode: a gradient term was not finite
                         or left the fixed-point range (|g| >= 2^20, a row
                         sum >= 2^30); the step is invalid (the fp32 path
                         would carry the inf / NaN into the tables)       */
};

/* parameter tables addressable by cf_set_table / cf_get_table */
enum cf_table {
    CF_TABLE_USER = 0,      /* U   [n_users, d]  user_embed                 */
    CF_TABLE_ITEM = 1,      /* V   [n_items, d]  item_embed                 */
    CF_TABLE_BIAS = 2,      /* b   [n_items]     item_bias (GBPR only)      */
    CF_TABLE_ACC_USER = 3,  /* Adagrad accumulator of U                     */
    CF_TABLE_ACC_ITEM = 4,  /* Adagrad accumulator of V                     */
    CF_TABLE_ACC_BIAS = 5   /* Adagrad accumulator of b (GBPR only)         */
};

/* kernels timed by the built-in HIP-event profiler */
enum cf_kernel_id {
    CF_K_SAMPLE = 0,     /* batch draw / load + per-row occurrence counts     */
    CF_K_STEP = 1,       /* gather + loss + gradients + singleton-row Adagrad  */
    CF_K_APPLY = 2,      /* Adagrad of duplicated rows from summed gradients  */
    CF_K_APPLY_DENSE = 3,/* dense item Adagrad (after cross-rank all-reduce)  */
    CF_K_CLIP = 4,       /* CML full-table clip_by_norm                       */
    CF_K_SCORE = 5,      /* user x item scoring tile kernel                   */
    CF_K_TOPK = 6,       /* masked per-user top-k                             */
    CF_K_SLOT = 7,       /* (retired: fixed per-row slot ranges need no pass)  */
    CF_K_APPLY_PREP = 8, /* apply of step s fused with the draw of step s+1    */
    CF_K_GRAD_PREP = 9,  /* gradient of step s + draw of step s+1 (pipeline 2) */
    CF_K_APPLY_SLOT = 10,/* (retired pipeline 2)                               */
    CF_K_ITEM_REDUCE = 11,/* multi-rank: duplicated item rows' summed gradient
                            into the bound buffer, before the all-reduce    */
    CF_K_PSORT = 12,     /* pos_sort: scan of the positive counts + scatter of
                            the pairs into positive-item order               */
    CF_K_STEP_REMOTE = 13,/* split exchange step: the gradient of the pairs with
                            a remote group member (cf_xchg_grad_part 2)      */
    CF_K_EPOCH_ORDER = 14,/* sorted batches: an epoch's pair order (inverse
                            bijection keys + radix sort by batch), once per epoch */
    CF_K_COUNT = 15
};

/*
 * Engine configuration.  Replaces the model constructors' keyword arguments:
 *   BPRMF(n_users, n_items, topN, split_method, eval_metrics, reg, n_factors,
 *         batch_size, max_iter, lr, init_mean, init_stddev, device)
 *         -- src/models/pl/models/bprmf.py:13-18
 *   GBPRMF(..., rho, gsize, ...)      -- src/models/pl/models/gbprmf.py:14-19
 *   CML(..., reg_cov, margin, use_rank_weight, clip_norm, ...)
 *                                     -- src/models/pl/models/cml.py:14-20
 *   AMF(..., epsilon, reg_adv, adv_method, reg, ...)
 *                                     -- src/models/others/models/amf.py:13-19
 * and the samplers' n_neg / gsize      -- src/samplers/sampler_ranking.py:8,
 *                                         src/samplers/sampler_gbpr.py:8
 */
typedef struct cf_config {
    int32_t model;            /* enum cf_model                                  */
    int32_t n_factors;        /* d, 1..256                                      */
    int64_t n_users;          /* rows of U held by THIS engine (a user shard)   */
    int64_t n_items;          /* rows of V (replicated on every rank)           */
    int32_t n_neg;            /* W negatives per (u,i) pair, 1..64 (CML 1..16)  */
    int32_t gsize;            /* G group users per pair (GBPR), 1..16           */
    float lr;                 /* Adagrad learning rate (constant; see DESIGN)   */
    float reg;                /* L2 coefficient (BPR/GBPR/AMF)                  */
    float rho;                /* GBPR group blend                               */
    float margin;             /* CML hinge margin                               */
    float reg_cov;            /* CML L2 coefficient ("covariance" loss)         */
    float clip_norm;          /* CML row-norm bound                             */
    float reg_adv;            /* AMF adversarial-loss weight                    */
    float epsilon;            /* AMF perturbation radius (inert in ref mode)    */
    float acc_init;           /* Adagrad initial accumulator, 0.1 in TF1        */
    int32_t use_rank_weight;  /* CML rank weight on/off                         */
    int32_t device;           /* HIP device ordinal                             */
    int32_t dense_item_apply; /* 1: item Adagrad over all rows (multi-rank)     */
    int32_t plr_kind;         /* enum cf_plr_kind (CF_PLR)                      */
    uint64_t seed;            /* device sampler / init seed                     */
    float alpha, beta, gamma; /* PLR term weights (prigp.py:128, cplr_u.py:136) */
    int32_t amf_mode;         /* AMF adversarial phase: CF_AMF_REFERENCE (0, the
                                 default) is what amf.py:139-162 computes -- Δ = 0,
                                 because the tf.assign ops of __update_adv__
                                 (amf.py:117-137) never run; CF_AMF_APR (1) runs
                                 them as written for adv_method "grad":
                                 Δ_X = epsilon * l2_normalize(dL_embed/dX, axis 1)
                                 from the step's pre-update rows (stop-gradient),
                                 perturbing U_u, V_i, V_j in ui and V_j in uj
                                 (amf.py:96-116).  Not deterministic, slot rows
                                 (item_slots 0); across ranks see
                                 cf_step_local_apr_embed; DESIGN 3.13           */
} cf_config;

enum cf_amf_mode { CF_AMF_REFERENCE = 0, CF_AMF_APR = 1 };

/* ---- lifecycle ---------------------------------------------------------- */
const char* cf_version(void);
const char* cf_last_error(void);
int cf_device_count(int32_t* count_out);
void cf_config_defaults(cf_config* cfg);              /* TF1 defaults, BPR */
int cf_create(const cf_config* cfg, cf_engine** out);
int cf_destroy(cf_engine* eng);
/* Use an external HIP stream (hipStream_t as void*); NULL = engine stream. */
int cf_set_stream(cf_engine* eng, void* hip_stream);
int cf_synchronize(cf_engine* eng);

/* ---- data ---------------------------------------------------------------- */
/*
 * Train interactions as host CSR (rows sorted ascending).  Replaces
 *   useritem_pairs = np.array(trasR.nonzero()).T   sampler_ranking.py:13
 *   user_posItemset = {u: set(row)}                sampler_ranking.py:14
 *   item_posUserList (transpose rows)              sampler_gbpr.py:15
 * The engine keeps the CSR, the nnz-ordered (u,i) pair list and, for GBPR,
 * the item->user transpose in HBM.
 */
int cf_set_interactions(cf_engine* eng, const int64_t* host_indptr,
                        const int32_t* host_indices, int64_t nnz);

/*
 * Initialise U, V (, b) with N(mean, stddev) -- truncated at 2 sigma when
 * truncated != 0 (tf.truncated_normal_initializer, bprmf.py:29-34) or plain
 * (tf.random_normal_initializer, cml.py:32-37) -- and every accumulator to
 * acc_init (tf.global_variables_initializer, bprmf.py:136).
 */
int cf_init_params(cf_engine* eng, float mean, float stddev,
                   int32_t truncated, uint64_t seed);
/* Host <-> device copy of one table (enum cf_table); n_elems must match. */
int cf_set_table(cf_engine* eng, int32_t table, const float* host_src,
                 int64_t n_elems);
int cf_get_table(cf_engine* eng, int32_t table, float* host_dst,
                 int64_t n_elems);
/*
 * Every parameter table in one call, enum cf_table order:
 * U [n_users,d], V [n_items,d], b [n_items], AU, AV, Ab (the model's
 * variables and their Adagrad slots: bprmf.py:24-34 + the optimizer's
 * accumulators; checkpoint / restore).  NULL = keep (set) or skip (get); b
 * and Ab exist only for the bias models (GBPR, PLR) -- non-NULL for another
 * model is CF_EINVAL, and nothing is copied unless every argument is valid.
 * Host or device memory, as cf_set_table / cf_get_table.
 */
int cf_set_params(cf_engine* eng, const float* U, const float* V, const float* b,
                  const float* AU, const float* AV, const float* Ab);
int cf_get_params(cf_engine* eng, float* U, float* V, float* b, float* AU,
                  float* AV, float* Ab);

/* ---- training ------------------------------------------------------------ */
/*
 * One optimizer step on a host-fed batch: the body of
 *   sess.run(train_op, {useritem: pairs, negItems: negs[, group: groups]})
 *     bprmf.py:143-148 / gbprmf.py:162-166 / cml.py:185-190 / amf.py:219-227
 * pairs [B,2] (u,i), negs [B,W], groups [B,G] (GBPR only, else NULL), all
 * host int32.  Computes the pre-update loss, sums duplicate-row gradients
 * (TF1 _deduplicate_indexed_slices) and applies SparseApplyAdagrad once per
 * touched row; CML then clips rows to clip_norm (cml.py:119-129).
 * loss_out (may be NULL) receives the pre-update batch loss and forces a
 * stream sync; with NULL the call is asynchronous.
 */
int cf_step(cf_engine* eng, const int32_t* host_pairs,
            const int32_t* host_negs, const int32_t* host_groups, int32_t B,
            double* loss_out);

/*
 * n_steps steps fed by the on-device sampler: per epoch a bijective shuffle
 * of the nnz pairs, floor(nnz/B) batches of B consecutive shuffled pairs,
 * W uniform negatives per pair rejected while j in Pos(u), and (GBPR) G
 * group users drawn uniformly with replacement from Pos^-1(i).  Replaces the
 * sampler threads (sampler_ranking.py:22-37, sampler_uij_ranking.py:22-38,
 * sampler_gbpr.py:23-43) feeding the train loop.  loss_sum_out (may be NULL:
 * asynchronous) receives the sum of the n_steps pre-update batch losses.
 */
int cf_train_steps(cf_engine* eng, int32_t B, int32_t n_steps,
                   double* loss_sum_out);

/*
 * One iteration of the reference's train loop on the device sampler:
 * n_batches = int(len(tra_tuple) / batch_size) steps (bprmf.py:138-148),
 * ending at an epoch boundary -- a whole epoch from a boundary (or after
 * steps at another B), the batches the sampler's epoch has left otherwise --
 * and mean_loss_out (may be NULL: asynchronous) = the mean of their
 * pre-update batch losses, the reference's TraLoss (aveloss = np.mean(losses),
 * bprmf.py:150; gbprmf.py:168, cml.py:192, amf.py:229).
 */
int cf_train_epoch(cf_engine* eng, int32_t B, double* mean_loss_out);

/*
 * Draw the next batch of the device sampler without training (advances the
 * same stream cf_train_steps consumes).  Replaces Sampler.next_batch()
 * (sampler_ranking.py:39-40).  groups may be NULL unless GBPR.
 */
int cf_sample(cf_engine* eng, int32_t B, int32_t* host_pairs,
              int32_t* host_negs, int32_t* host_groups);

/* Device-sampler position: epoch and batch index inside the epoch. */
int cf_get_sampler_state(cf_engine* eng, int64_t* epoch_out,
                         int64_t* batch_out);
int cf_set_sampler_state(cf_engine* eng, int64_t epoch, int64_t batch);

/*
 * AMF phase switch (amf.py:243-244): phase 1 = adversarial (BPR loss plus
 * reg_adv * softplus(-clip(x,-80,1e8))); the switch also resets every
 * accumulator to acc_init because the second train op owns a fresh
 * AdagradOptimizer (amf.py:157-162, built at amf.py:209).  phase 0 = BPR.
 */
int cf_begin_phase(cf_engine* eng, int32_t phase);

/* ---- split step for multi-rank data parallelism --------------------------- */
/*
 * Bind an external device buffer of n_items*d (+ n_items for GBPR) fp32
 * that receives this rank's dense item gradient (e.g. torch tensor memory
 * all-reduced by RCCL).  Requires dense_item_apply=1.
 */
int cf_bind_item_grad(cf_engine* eng, void* device_ptr, int64_t n_elems);
/* Phase 1: sample (or host-feed when host_pairs != NULL), forward,
 * scatter the gradient; apply the user update (users are rank-local).  The
 * item gradient is left in the bound buffer. */
int cf_step_local(cf_engine* eng, int32_t B, const int32_t* host_pairs,
                  const int32_t* host_negs, const int32_t* host_groups);
/* Phase 1 in two halves, so that the item all-reduce can start as soon as the
 * item gradient is complete and overlap the rest:
 *   cf_step_local_grad   sample / host-feed, count, slots, gradient
 *   (start the all-reduce of the item-gradient buffer)
 *   cf_step_local_apply  user Adagrad; next_B > 0 also draws + counts the
 *                        next device-sampled batch of next_B pairs in the
 *                        same launch (used by the next cf_step_local_grad
 *                        with that B and no host batch; any other call drops
 *                        it and rewinds the sampler).
 * cf_step_local = cf_step_local_grad + cf_step_local_apply(0). */
int cf_step_local_grad(cf_engine* eng, int32_t B, const int32_t* host_pairs,
                       const int32_t* host_negs, const int32_t* host_groups);
int cf_step_local_apply(cf_engine* eng, int32_t next_B);
/* The item reduce of cf_step_local_grad in pieces (round 4):
 * with cf_set_option("item_pieces", P > 1) on the pos_sort path,
 * cf_step_local_grad leaves the duplicated item rows unsummed and the caller
 * runs cf_step_item_reduce(eng, q) for q = 0 .. P-1, in order, each followed
 * by the all-reduce of that piece's rows [row0, row1) of the bound buffer
 * (cf_item_piece_rows), so piece q's collective runs while piece q+1 is
 * reduced.  cf_step_local_apply fails with CF_ESTATE while pieces are left.
 * Replaces the reduce inside cf_step_local_grad (the same launch, cut by item
 * rows; TF1 sums every duplicate before the update, gbprmf.py:101-106,
 * bprmf.py:83-88). */
int cf_step_item_reduce(cf_engine* eng, int32_t piece);
int cf_item_piece_rows(cf_engine* eng, int32_t piece, int32_t n_pieces, int64_t* row0, int64_t* row1);
/* AMF apr across ranks (amf_mode CF_AMF_APR with dense_item_apply=1; DESIGN
 * 3.13): an item row's Δ = epsilon * l2_normalize of its embedding-loss
 * gradient over the GLOBAL batch (amf.py:130-137 on the concatenated batch),
 * so its sum crosses ranks before the gradient launch -- SURVEY 8(e)'s second
 * all-reduce.  Bind an n_items*d fp32 device buffer once; in the adversarial
 * phase each step is
 *   cf_step_local_apr_embed(eng, B, pairs|NULL, negs|NULL)  this rank's sums
 *   (all-reduce the bound buffer)
 *   cf_step_local_grad(eng, B, NULL, NULL, NULL)  the step on the summed Δ;
 *                                 it clears the buffer after reading it
 * and then the usual item exchange.  cf_step_local_grad without the embed
 * fails with CF_ESTATE in that phase; cf_step_local (one call, no caller
 * collective) runs both halves, exact at world size 1. */
int cf_bind_apr_item_grad(cf_engine* eng, void* device_ptr, int64_t n_elems);
int cf_step_local_apr_embed(cf_engine* eng, int32_t B, const int32_t* host_pairs, const int32_t* host_negs);
/* Phase 2, after the buffer holds the cross-rank sum: dense item Adagrad
 * (and CML clip of updated rows); zeroes the buffer. */
int cf_step_items(cf_engine* eng);
/* Draw + count the next device-sampled batch of B pairs after
 * cf_step_local_apply(eng, 0) (the next cf_step_local_grad with that B takes
 * it), so that the draw can run beside a collective of its own. */
int cf_step_local_draw(cf_engine* eng, int32_t B);
/*
 * Item-range ownership (reduce-scatter -> owner Adagrad -> all-gather), the
 * alternative to the all-reduce + replicated item Adagrad above; same
 * arithmetic (TF1 sums over the whole global batch before the update,
 * gbprmf.py:101-106, bprmf.py:83-88):
 *   cf_bind_item_grad_split  dense item gradient (>= n_items*d floats) and,
 *                            GBPR, bias gradient (>= n_items) in caller
 *                            buffers, e.g. padded to world * chunk rows so a
 *                            reduce-scatter splits them evenly
 *   cf_step_local_grad / _apply (/ _draw) as above
 *   (reduce-scatter of the gradient buffers: rank r receives rows
 *    [r*chunk, (r+1)*chunk))
 *   cf_clear_item_grad       re-zero the rows of the bound gradient buffers
 *                            the last local gradient touched (stream-ordered
 *                            after the collective that read them)
 *   cf_step_items_range      Adagrad (+ CML clip) of item rows [row0, row1)
 *                            from gradient rows in `grad` ((row1-row0)*d) and
 *                            `grad_bias` (GBPR); all-zero rows are untouched
 *   (all-gather of the owned rows of V (and b) into every rank's table:
 *    bind the table storage with cf_bind_table so the collective writes it)
 * Only the owner keeps the accumulator rows of its range current.
 */
int cf_bind_item_grad_split(cf_engine* eng, void* grad_items, int64_t n_grad_items,
                            void* grad_bias, int64_t n_grad_bias);
int cf_clear_item_grad(cf_engine* eng);
int cf_step_items_range(cf_engine* eng, int64_t row0, int64_t row1, const void* grad,
                        const void* grad_bias);
/* Use caller device memory (>= the table's size in floats, e.g. padded for an
 * all-gather) as the storage of CF_TABLE_ITEM, CF_TABLE_BIAS,
 * CF_TABLE_ACC_ITEM or CF_TABLE_ACC_BIAS; the current contents are copied
 * in.  NULL returns the table to engine-owned memory (contents copied
 * back).  The caller keeps the buffer alive while it is bound. */
int cf_bind_table(cf_engine* eng, int32_t table, void* device_ptr, int64_t n_elems);
/* ---- user sharding + GBPR group exchange ------------------------
 * A user-sharded GBPR engine draws each pair's group members from the item's
 * users over ALL ranks (item_posUserList, sampler_gbpr.py:15,41); a member
 * owned by another rank is fetched from its owner and its gradient row sent
 * back, so each step equals one step on the concatenated global batch.
 * Protocol per step (the caller runs the three all-to-alls, e.g. RCCL through
 * torch.distributed.all_to_all_single, on the engine stream):
 *   cf_xchg_begin    sample (or take the host batch; groups = GLOBAL user ids),
 *                    count, pack the remote members' ids by owner into
 *                    send_ids; send_counts_out[r] = ids for rank r (syncs)
 *     or, with no host round trip (device sampler):
 *   cf_xchg_draw     (one step AHEAD) draw + count + pack the next batch into
 *                    buffer set h = *half_out: its ids go to send_ids half h,
 *                    its per-owner counts to send_counts_dev[h*world ..]
 *                    (device int32 [2, world]); the caller all-to-alls the
 *                    counts and copies them to the host asynchronously
 *   cf_xchg_adopt    take the drawn batch as this step's (stage begun); B
 *                    must be the size it was drawn at, else it is discarded
 *                    (counts cleared, sampler rewound) and CF_EAGAIN returned
 *   all-to-all       send_ids -> recv_ids (ids this rank serves)
 *   cf_xchg_serve    copy the served rows (pre-update) into serve_rows
 *   all-to-all       serve_rows -> rows (in send_ids order)
 *   cf_xchg_grad     slots + gradient; remote members' gradient rows -> grads
 *   all-to-all       grads -> serve_grads
 *   cf_xchg_finish   add the served rows' gradients, user Adagrad
 * then the item exchange (all-reduce + cf_step_items, or the item-range
 * reduce-scatter path) as for cf_step_local.  A served row's count word is
 * flagged, so all its contributions are summed before the update (TF1 dedup
 * semantics).  Requires GBPR, dense_item_apply=1.  send_ids holds
 * 2 * send_cap ids: cf_xchg_begin packs into half 0, cf_xchg_draw into the
 * half it returns.
 * A drawn-ahead batch is dropped (sampler rewound) by any other stepping or
 * sampling call.
 * Split form (overlaps the exchanges with compute; same results):
 *   cf_xchg_serve, then the rows all-to-all issued ASYNCHRONOUSLY, and
 *   cf_xchg_grad_part(1)  the pairs whose group members are all local (no
 *                         received row needed) while the rows are in flight
 *   wait for the rows; cf_xchg_grad_part(2)  the other pairs
 *   the grads all-to-all issued asynchronously, and
 *   cf_xchg_finish_items  the item rows' summed gradient into the bound item
 *                         buffer: the item exchange may start now
 *   wait for the grads; cf_xchg_finish  as above, users only.
 * cf_xchg_grad_part(0) = cf_xchg_grad.  Replaces nothing in the reference
 * (no multi-GPU there); keeps gbprmf.py:101-106's sum-before-update. */
int cf_set_shard(cf_engine* eng, int32_t world, int32_t rank, const int64_t* user_bounds /*[world+1]*/);
/* global item -> user CSR (sampler_gbpr.py:15), user ids global */
int cf_set_group_source(cf_engine* eng, const int64_t* indptr_t, const int32_t* indices_t, int64_t nnz);
int cf_bind_exchange(cf_engine* eng, void* send_ids, void* rows, void* grads, int64_t send_cap,
                     void* recv_ids, void* serve_rows, void* serve_grads, int64_t recv_cap);
int cf_xchg_begin(cf_engine* eng, int32_t B, const int32_t* host_pairs, const int32_t* host_negs,
                  const int32_t* host_groups, int32_t* send_counts_out);
int cf_xchg_draw(cf_engine* eng, int32_t B, void* send_counts_dev, int32_t* half_out);
int cf_xchg_adopt(cf_engine* eng, int32_t B);
int cf_xchg_serve(cf_engine* eng, int64_t n_recv);
int cf_xchg_grad(cf_engine* eng);
int cf_xchg_grad_part(cf_engine* eng, int32_t part);
int cf_xchg_finish_items(cf_engine* eng);
int cf_xchg_finish(cf_engine* eng, int64_t n_recv);

/* Which kernels a step of B pairs takes with the current options (bench
 * keys its committed PMC counters by it; tests assert the path under test):
 * a bitmask of cf_path_flag, plus the pipeline option in bits 8-9. */
enum cf_path_flag {
    CF_PATH_PHASED = 1,         /* phased gradient kernel (grad_fast_kernel), else generic */
    CF_PATH_POS_SORT = 2,       /* positive-sorted gradient (psort + partial rows)         */
    CF_PATH_ITEM_RECORDS = 4,   /* item records + user-row stash instead of slot rows      */
    CF_PATH_DETERMINISTIC = 8,  /* sort-based ranks, compact slots, no float atomics       */
    CF_PATH_DENSE_ITEMS = 16,   /* multi-rank item path (dense item gradient)              */
    CF_PATH_LDS = 32,           /* gradient kernel with LDS-staged negatives (grad_lds_kernel) */
    CF_PATH_SORTED_BATCHES = 64 /* device-sampled batches in CSR order (option "sorted_batches";
                                   auto turns off for good once the orders did not fit in HBM) */
};
int cf_step_path(cf_engine* eng, int32_t B, int32_t* flags_out);

/* Pre-update loss accumulated since the last call (syncs), then reset. */
int cf_take_loss(cf_engine* eng, double* loss_sum_out);

/* ---- tuple ranking step (CF_PLR) ------------------------------------------------
 * One host-fed optimizer step on B tuples [B, width] (int32):
 *   PRIGP width 5: (u, i, j, t, k)  (sampler_prigp.py:51; prigp.py:99-130)
 *   CPLR  width 4: (u, i, t, j)     (sampler_uitj_ranking.py:35; cplr_u.py:106-137)
 * with coefs [B, 2] = (coefMat[u,i], coefMat[u,t]) for CPLR (NULL for PRIGP).
 * Scores s_x = <U_u, V_x> + b_x; loss = sum of weighted -log sigmoid terms
 * + reg (l2(U_u) + l2(V_items) + l2(b_items)); TF1 dedup-sum Adagrad. */
int cf_step_plr(cf_engine* eng, const int32_t* host_tuples, int32_t width, const float* host_coefs,
                int32_t B, double* loss_out);

/* ---- evaluation ----------------------------------------------------------- */
/*
 * For each of n users: scores over all items (U.V^T [+ b for GBPR],
 * -|u-v|^2 for CML: bprmf.py:77-81, gbprmf.py:95-99, cml.py:111-117,
 * amf.py:144-148), drop the excluded items and return the top k item ids
 * sorted by score descending, ties to the lower id (TopKV2) -- the
 * reference's __recommend (bprmf.py:90-103; its top_k over max|train|+topN
 * then the python filter loop equals filtering before the selection).
 * mask_or_NULL: NULL = exclude each user's train items (the
 * reference's filter); else uint8 [n_items], exactly the items with
 * mask[j] != 0 are excluded for every user (an all-zero mask: the raw top-k).
 * idx_out [n,k] int32 (-1 pads when fewer than k items remain), val_out
 * [n,k] float (may be NULL).  k <= 128 and d <= 128 stream through the fused
 * MFMA + top-k kernel (no score matrix in HBM); larger k materialise scores
 * per user chunk.
 */
int cf_score_topk(cf_engine* eng, const int32_t* host_users, int32_t n,
                  int32_t k, const uint8_t* mask_or_NULL, int32_t* host_idx_out,
                  float* host_val_out);
/* The same with both exclusions: exclude_train != 0 drops each user's train
 * items, item_mask (NULL = none) the flagged items on top. */
int cf_score_topk_ex(cf_engine* eng, const int32_t* host_users, int32_t n,
                     int32_t k, int32_t exclude_train, const uint8_t* item_mask,
                     int32_t* host_idx_out, float* host_val_out);

/*
 * Engine options (name, value):
 *   "topk_path"  0 = auto (fused MFMA+top-k when k <= 128 and d <= 128, else
 *                materialised scores + radix select), 1 = materialised,
 *                2 = fused (CF_EINVAL when k/d exceed its limits)
 *   "fused_variant" the fused scoring + top-k kernel: 0 = sequential (MFMAs,
 *                then the candidate test; default), 1 = software-pipelined
 *                (tile t's candidate test beside tile t+1's MFMAs; measured
 *                slower, kept for A/B; CML always takes 0), 2 = specialised
 *                waves (measured slower), 3 = 128 users per block at one
 *                block per CU (half the V-tile staging per FLOP; k <= 28).
 *                Same output.
 *   "grad_path"  0 = auto (BPR / AMF / CML at W = 5, 64 < d <= 128, d % 4 == 0
 *                without pos_sort: the kernel with LDS-staged negative rows;
 *                else the phased gradient kernel for W in {1,5}, d <= 128,
 *                GBPR group size 1, except CML at W = 5; generic kernel
 *                otherwise), 1 = generic kernel always, 2 = phased kernel
 *                whenever eligible, 3 = the LDS-staged kernel whenever
 *                eligible.  All give the same arithmetic.
 *   "prep_stream" 0 = everything in order on the engine stream (default);
 *                1 = sample/count on a side stream, overlapping the previous
 *                step's gradient.  Same results.
 *   "slot_max"   occurrence k < slot_max of a duplicated item row stores its
 *                gradient row in a plain slot row (row r owns the fixed range
 *                [r*slot_max, (r+1)*slot_max)); later occurrences of a hot row
 *                add into a float accumulator with atomics; the apply sums
 *                both (default 32).  Same arithmetic up to fp32 summation
 *                order.
 *   "slot_max_user" the same for user rows (default: chosen at the first
 *                step, 4 when a batch holds >= 0.25 occurrences per user on
 *                average, else 2).
 *   "hot_replicas" the atomic part of a hot item row is spread over this many
 *                accumulator copies by occurrence rank (1, 2, 4, 8, 16;
 *                default 1: at cfg2 the copies' extra apply reads cost more
 *                than the spread atomics save).
 *   "pipeline"   how cf_train_steps overlaps consecutive steps (same results):
 *                1 = the duplicate apply of step s with the draw + count of
 *                step s+1, two launches per step (default); 2 = the draw +
 *                count of step s+1 inside step s's gradient launch, the apply
 *                alone (measured 4.7 us/step slower at cfg2); 3 = as 2 for
 *                positive-sorted steps (the draw rides in grad_sort_kernel,
 *                psort of s+1 follows the apply), else as 1; 0 = one step
 *                at a time, three launches.
 *   "sorted_batches" the device sampler's batches read in pair (CSR) order:
 *                the same batch sets as the epoch bijection, each batch's
 *                pairs ascending, so the draw's records, user count atomics
 *                and row scans stay local.  Each epoch's pair records are
 *                radix-sorted by batch (keys from the inverse bijection, the
 *                16-B records as values) ahead, on a low-priority stream, and
 *                the draw reads them sequentially.  0 off, 1 on, 2 auto
 *                (default: on when an epoch has >= 16 batches), 3 on in the
 *                index form (sorted pair indices into the records: a quarter
 *                of the memory, one more dependent load in the draw)
 *   "neg_check"  how the device draw rejects a negative candidate in Pos(u):
 *                1 = probe an open-addressed set of the (u, i) pairs (16 B
 *                per interaction, built when selected; ~1 sector per
 *                candidate), 0 = scan the user's sorted CSR row (default:
 *                8 candidates per scan; A/B at cfg2 within noise), 2 = the
 *                set probed by one lane per pair (measured slower, DESIGN).
 *                The same batches every way: each negative takes its first
 *                attempt outside Pos(u) in the same draw sequence.
 *   "bias_slots" GBPR / CPLR item bias of a duplicated row: 1 = stored in a
 *                bias slot beside the row's gradient slot and summed by the
 *                apply, 0 = one float atomic per occurrence (default: at
 *                cfg4 the atomics cost the gradient launch nothing measurable,
 *                165.1 vs 164.9 us, and the slot sums cost the apply 4 us).
 *   "item_slots" what a duplicated item occurrence stores for the apply:
 *                0 = its gradient row (4d B), 1 = a 16-B record (pair, alpha,
 *                beta, which) -- every item gradient is alpha * X + beta *
 *                V_row with X the pair's pre-update user row (or GBPR's group
 *                blend), which the pair stashes once -- so the apply sums
 *                alpha * X from the stash plus (sum of beta) * V_row.  Same
 *                results up to fp32 summation order.  Default: 1 when
 *                n_factors >= 128 (measured 10-12 % faster steps at cfg3 /
 *                cfg5), else 0 (4-5 % slower at cfg2 / cfg4, d = 64).
 *   "deterministic" 1 = bitwise-reproducible steps: occurrence ranks from a
 *                stable sort of the batch's row ids, every occurrence of a
 *                duplicated row stored in its own compact slot and summed in
 *                batch order, no float atomics anywhere (the GBPR group
 *                exchange is excluded); 0 = the fast path (default), whose
 *                rank order -- and so the last bits of duplicate sums --
 *                follows the order the count atomics land.  Where pos_sort
 *                is active (round 3) the mode keeps the fast path's launches
 *                and takes every sum of gradient rows in 64-bit fixed point
 *                (2^-32 units; int64 partial rows and int64 atomics), which
 *                is exact in any order, so no sort runs.
 *   "item_pieces" P = 1 (default) .. 64: the multi-rank item reduce in P
 *                pieces of item rows (cf_step_item_reduce).
 *   "spec_neg"   1 = where pos_sort is active with its dense item
 *                apply (n_items <= 2 B (1 + W)), the draw issues each
 *                negative's count atomic for its FIRST candidate before the
 *                row scan that accepts or rejects it (its latency overlaps
 *                the scan); a rejected first candidate leaves a phantom
 *                occurrence whose slot row psort zeroes.  Same batches, same
 *                sums up to fp32 order; 0 (default since round 5's sorted
 *                batches: 3 us faster at cfg2) = count after the scan.
 *   "pair_prefetch" 1 = the pos_sort gradient launch also fetches the next
 *                step's shuffled pair records for its draw (cf_train_steps);
 *                measured slower at cfg2 (its registers cost the gradient
 *                launch a wave per SIMD), so 0 (default), and the default
 *                build compiles it out: 1 then fails with CF_EINVAL (build
 *                with -DCF_PAIR_PREFETCH=1).
 *   "pos_sort"   1 = the gradient launch visits the batch's pairs in
 *                positive-item order (a counting sort by the draw's positive
 *                counts, two short launches before it), so the pairs of one
 *                gradient block that share a positive item sum that item's
 *                gradient in LDS and store one partial row per block instead
 *                of one slot row (or float atomics) per occurrence; the apply
 *                adds the partials to the negatives' slot rows.  BPR / AMF /
 *                CML on the phased kernel (W in {1, 5}, d <= 128), not with
 *                item_slots 1, hot_replicas > 1, pipeline 2 or
 *                a dense item apply other than item_reduce 1 (the option is
 *                ignored there; with item_reduce 1 the multi-rank item reduce
 *                sums the partials into the bound gradient).  Same
 *                results up to fp32 summation order.  0 = off; 2 = auto
 *                (default): on for batches of >= 2^18 pairs (cfg2: 7 %
 *                faster steps at 2^19, 3.5 % at 2^18, even at 2^17).
 *   "slot_max_pos" positive partial rows per item row under pos_sort (default
 *                8; later partials of a hot item add with float atomics --
 *                int64 atomics in deterministic mode).
 *   "item_reduce" dense_item_apply engines (the multi-rank step): 1 =
 *                item occurrences are counted like user ones, a row seen
 *                once stores its gradient row into the bound buffer, a
 *                duplicated row stores slot rows summed by a short reduce
 *                launch in cf_step_local_grad (default; plain stores instead
 *                of one float atomic per element and occurrence); 2 = rows
 *                seen once store, every occurrence of a duplicated row adds
 *                with float atomics (no reduce launch); 0 = every item
 *                occurrence adds into the buffer with float atomics.
 *                Same sums either way (fp32 summation order differs).
 *   "profile_mask" bit k set = cf_profile_enable times kernel id k (default
 *                all): timing only the kernel of interest keeps the event
 *                pairs of the others out of a timed loop.
 *   "profile_every" time only every n-th launch of each kernel id (default
 *                1): an event pair per step costs the loop a few us, so a
 *                timed loop samples its launches.
 */
int cf_set_option(cf_engine* eng, const char* name, int64_t value);

/* ---- measurement ----------------------------------------------------------- */
/* HIP-event timing of every launch of each cf_kernel_id on the engine stream. */
int cf_profile_enable(cf_engine* eng, int32_t on);
int cf_profile_read(cf_engine* eng, int32_t kernel_id,
                    double* total_ms_out, int64_t* launches_out);
int cf_profile_reset(cf_engine* eng);

/* ---- rating-file ingest ----------------------------------
 * Native IOUtil.loadSparseR (src/utils/IOUtil.py:8-16) + Util.split_row /
 * matBinarize (src/utils/Util.py:5-16), same rules: ',' else ';' else
 * whitespace fields; 2 fields = 1, 3 fields = float(rating), others ignored;
 * Python index wrap for negative ids; the last write of an entry wins; zeros
 * are not stored.  cf_ratings_csr with binarize != 0 keeps entries with
 * value > threshold as 1.0 (matBinarize); pass NULL indices/values first to
 * size the output (nnz_out).  Host-only: needs no HIP device. */
typedef struct cf_ratings cf_ratings;
int cf_ratings_load(const char* path, int64_t n_users, int64_t n_items, int32_t n_threads,
                    cf_ratings** out, int64_t* nnz_out);
int cf_ratings_csr(const cf_ratings* r, int32_t binarize, double threshold, int64_t* indptr,
                   int32_t* indices, double* values, int64_t* nnz_out);
int cf_ratings_free(cf_ratings* r);

/* ---- bit-exact host sampler ------------------------------
 * The reference samplers' batch stream for np.random.seed(seed) set right
 * before the sampler is built (sampler_ranking.py:22-37 kind 0,
 * sampler_uij_ranking.py:22-38 kind 1, sampler_gbpr.py:23-43 kind 2):
 * numpy's legacy MT19937 RandomState shuffle / randint / choice restated
 * (csrc/cf_mt_sampler.cpp).  Host batches, fed with cf_step. */
typedef struct cf_mt_sampler cf_mt_sampler;
int cf_mt_sampler_create(const int64_t* indptr, const int32_t* indices, int64_t n_users,
                         int64_t n_items, int32_t kind, int32_t n_neg, int32_t gsize,
                         int32_t batch_size, uint32_t seed, cf_mt_sampler** out);
int cf_mt_sampler_next(cf_mt_sampler* s, int32_t* pairs /*[B,2]*/, int32_t* negs /*[B,W]*/,
                       int32_t* groups /*[B,G] | NULL*/);
int cf_mt_sampler_state(const cf_mt_sampler* s, int64_t* epoch_out, int64_t* batch_out);
int cf_mt_sampler_free(cf_mt_sampler* s);

/* ---- tuple samplers of the PRIGP / CPLR drop-ins (host) ------------------------
 * kind 0: PRIGP (u,i,j,t,k) tuples [B,5] (sampler_prigp.py:24-52); kind 1:
 * CPLR (u,i,t,j) tuples [B,4] + coefs [B,2] (sampler_uitj_ranking.py:22-38).
 * Train CSR (sorted rows) + coefficient CSR (sorted rows, float64 values).
 * The same draws, in the same order, on the same legacy MT19937 stream as
 * the Python restatements in _tuple.py for RandomState(seed). */
typedef struct cf_tuple_sampler cf_tuple_sampler;
int cf_tuple_sampler_create(int32_t kind, const int64_t* indptr, const int32_t* indices,
                            int64_t n_users, int64_t n_items, const int64_t* coef_indptr,
                            const int32_t* coef_indices, const double* coef_values,
                            int32_t batch_size, uint32_t seed, cf_tuple_sampler** out);
int cf_tuple_sampler_next(cf_tuple_sampler* s, int32_t* tuples, float* coefs /* CPLR | NULL */);
int cf_tuple_sampler_free(cf_tuple_sampler* s);

/* ---- attention-weighted MF ensemble ----------------------
 * src/models/pl/models/ensemble.py: K members U[K,n_users,d], V[K,n_items,d],
 * H[K,d] (all truncated-normal), trained on sampler_uij_ranking (u,i,j)
 * batches with dense Adagrad (ensemble.py:146) and lr decayed 0.98/epoch by
 * the caller (cf_ens_set_lr, ensemble.py:218).  The loss is the reference
 * graph's, including its [B] x [B,1] broadcast (ensemble.py:84-91): all B x B
 * (p, q) pairs of z = sum_k w_k(i_p) s_k(i_q) - w_k(j_p) s_k(j_q),
 * w_k = softmax_k(<U_k[u] o V_k[x], h_k>) -- plus reg * (l2 of the looked-up
 * rows + l2(H)).  Tables for get/set: 0 U, 1 V, 2 H, 3-5 their Adagrad
 * accumulators; sizes in floats.  Recommend = ensemble.py:128-140 scores
 * + the top-k / exclude rules of cf_score_topk. */
typedef struct cf_ensemble cf_ensemble;
int cf_ens_create(int64_t n_users, int64_t n_items, int32_t K, int32_t d, float reg, float lr,
                  float acc_init, int32_t device, cf_ensemble** out);
int cf_ens_destroy(cf_ensemble* e);
int cf_ens_init_params(cf_ensemble* e, float mean, float stddev, int32_t truncated, uint64_t seed);
int cf_ens_set_lr(cf_ensemble* e, float lr);
int cf_ens_set_table(cf_ensemble* e, int32_t table, const float* host_src, int64_t n);
int cf_ens_get_table(cf_ensemble* e, int32_t table, float* host_dst, int64_t n);
int cf_ens_set_interactions(cf_ensemble* e, const int64_t* indptr, const int32_t* indices, int64_t nnz);
/* one optimizer step on B host triplets [B,3] int32; loss_out (may be NULL,
 * else syncs) = the pre-update loss of the batch */
int cf_ens_step(cf_ensemble* e, const int32_t* host_uij, int32_t B, double* loss_out);
/* W-negative variants: pairs [B,2] + negs [B,W] (W <= 8)
 * from sampler_ranking.  Loss per pair and negative, no [B, B] broadcast:
 * lam * sum_w -log sigmoid(r_i - r_jw), r_x = sum_k w_k(x) s_k(x)
 * (ensemble_.py:75-118, lam = 1, singles = 0); singles = 1 adds every
 * member's own BPR terms sum_k sum_w -log sigmoid(s_k(i) - s_k(j_w)) with
 * lam = ensemble_lambda (ensemble__.py:102-145).  Same reg and dense Adagrad. */
int cf_ens_step_w(cf_ensemble* e, const int32_t* host_pairs, const int32_t* host_negs, int32_t W,
                  int32_t B, float lam, int32_t singles, double* loss_out);
/* sum of the step losses since the last call (syncs), then reset */
int cf_ens_take_loss(cf_ensemble* e, double* sum_out);
int cf_ens_score_topk(cf_ensemble* e, const int32_t* host_users, int32_t n, int32_t k,
                      int32_t exclude_train, int32_t* host_idx_out, float* host_val_out);

/* ---- synthetic implicit-feedback graphs (bench configs) --------- */
/*
 * Users [u_begin, u_end) of a graph with per-user degree 1 + Poisson(mean-1)
 * and items drawn without replacement from Zipf(zipf_s) popularity over a
 * seeded random item permutation.  Deterministic per (seed, user): any user
 * shard reproduces the same rows.  Step 1 fills indptr_out [u_end-u_begin+1]
 * (indptr_out[0] = 0); step 2 fills indices_out [indptr_out[last]] sorted per
 * row.  n_threads <= 0 uses all hardware threads.
 */
int cf_synth_degrees(int64_t n_users, double mean_degree, uint64_t seed,
                     int64_t u_begin, int64_t u_end, int64_t* host_indptr_out);
int cf_synth_items(int64_t n_items, double zipf_s, uint64_t seed,
                   int64_t u_begin, int64_t u_end, const int64_t* host_indptr,
                   int32_t* host_indices_out, int32_t n_threads);
/* The item -> user transpose of the whole graph (users of each item in
 * increasing id order) -- the GBPR group source of a user-sharded engine
 * (item_posUserList, sampler_gbpr.py:15) -- without materialising the
 * user -> item CSR: indptr_t_out [n_items+1], indices_t_out [nnz] with nnz
 * the last entry of cf_synth_degrees over all users. */
int cf_synth_item_users(int64_t n_users, int64_t n_items, double mean_degree, double zipf_s,
                        uint64_t seed, int64_t* host_indptr_t_out, int32_t* host_indices_t_out,
                        int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif /* CF_ENGINE_H */
