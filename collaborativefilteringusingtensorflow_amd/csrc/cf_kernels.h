// cf_kernels.h -- argument blocks shared by the host engine (cf_engine.cpp)
// and the gfx950 kernels (cf_kernels.hip, cf_eval.hip).  Plain structs passed
// by value as kernel arguments; no torch types anywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cfk {

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kBlock = 256;        // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kGL = 16;            // lanes per pair / per row ("group")
constexpr int kGroupsPerBlock = kBlock / kGL;   // 16
#ifndef CF_PAIRS_PER_GROUP
#define CF_PAIRS_PER_GROUP 2
#endif
constexpr int kPairsPerGroup = CF_PAIRS_PER_GROUP;  // pairs one group carries through grad
constexpr int kPairsPerBlock = kGroupsPerBlock * kPairsPerGroup;  // 32
constexpr int kMaxNeg = 64;
constexpr int kMaxGroup = 16;
constexpr int kMaxFactors = 256;

enum Model { BPR = 0, GBPR = 1, CML = 2, AMF = 3, PLR = 4 };

// Keyed bijection on [0, n) used as the per-epoch shuffle of the nnz pairs
// (replaces np.random.shuffle(useritem_pairs), sampler_ranking.py:24).
struct PermKey {
    uint64_t n;       // domain size (nnz)
    uint64_t mask;    // 2^bits - 1, 2^bits >= n
    uint32_t shift;   // xorshift amount
    uint32_t pad;
    uint64_t k[3];    // round keys
    uint64_t m[3];    // odd round multipliers
};

struct StepArgs {
    // model hyper-parameters
    int model;
    int d;
    int W;           // negatives per pair
    int G;           // group users per pair (GBPR)
    int B;           // pairs in this step
    int adversarial; // AMF phase flag
    int grad_path;   // 0 auto, 1 generic grad_kernel, 2 phased grad_fast_kernel when eligible
    float reg, rho, margin, reg_cov, reg_adv;
    // AMF apr (cf_config.amf_mode 1, adversarial phase): Δ_X = epsilon *
    // l2_normalize(dL_embed/dX); GadvU / GadvV hold the batch's summed
    // embedding-loss gradient of duplicated rows (zero between steps)
    int apr;
    float epsilon;
    float* GadvU;
    float* GadvV;
    int apr_global;       // multi-rank: GadvV holds every item row's sum over all ranks
    int apr_embed_done;   // cf_step_local_apr_embed ran (and the caller all-reduced GadvV)
    int use_rank_weight;
    float n_items_f;
    int64_t n_items;
    float lr, clip_norm;
    int clip;            // CML: clip every updated row
    // sampler
    int sample;          // 1: draw batch on device; 0: batch already in occ*
    int count_users;     // count user-row occurrences (sparse user apply)
    int count_items;     // count item-row occurrences (sparse item apply)
    int items_grad_only; // multi-rank item reduce: item rows get their summed
                         // gradient in GV (no Adagrad here; cf_step_items after the all-reduce)
    uint64_t slot_base;  // position of this batch inside the epoch shuffle
    uint64_t rng_key;    // per-epoch draw key
    PermKey perm;
    // graph
    const int4* __restrict__ pairs;         // [nnz] (u, i, row start, row length), CSR order
    const int64_t* __restrict__ indptr;     // [n_users+1]
    const int32_t* __restrict__ indices;    // [nnz] sorted per user
    const int64_t* __restrict__ indptr_t;   // [n_items+1] (GBPR)
    const int32_t* __restrict__ indices_t;  // [nnz] users of each item
    // Pos(u) membership for the negative draw: open-addressed set of
    // (u << 32 | i) keys, linear probing (null: scan the user's CSR row)
    const unsigned long long* __restrict__ pos_set;
    uint64_t pos_mask;                      // capacity - 1 (power of two)
    // pair-record prefetch (round 3, cf_set_option "pair_prefetch"): the
    // positive-sorted gradient launch of step s also fetches step s+1's
    // shuffled pair records -- pairs[permute(pf_slot_base + p, pf_perm)] for
    // p < pf_B, one per 16-lane group -- into pf_out[p], so that step s+1's
    // draw (pre_pairs = that buffer) reads them coalesced and starts at the
    // row scan.  Same records, same batches.  null = off
    int4* __restrict__ pf_out;
    uint64_t pf_slot_base;
    PermKey pf_perm;
    int pf_B;
    const int4* __restrict__ pre_pairs;     // the draw's record of pair p at [p] (null: pairs[permute(..)])
    // sorted batches (round 5, cf_set_option "sorted_batches"): the epoch's
    // pair indices batch by batch, each batch in pair (CSR) order -- the draw
    // takes pairs[order[slot]] instead of pairs[permute(slot)]: the same
    // batch set, its records read in ascending order, its users nearly
    // consecutive; null = off
    const int32_t* __restrict__ order;
    // the records form (sorted_batches 1 / 2): the records themselves in
    // that order, read sequentially by the draw; null = off (the index form,
    // sorted_batches 3, sets only `order`)
    const int4* __restrict__ order_recs;
    // sorted batches of a model without group users (cf_set_option
    // "user_runs"): a user's occurrences are one run of consecutive pairs, so
    // the draw takes user ranks and counts from the runs (prep_body) instead
    // of one returning count atomic per pair
    int user_runs;
    // deterministic mode on the positive-sorted path (round 3):
    // every sum of gradient rows is taken in 64-bit fixed point (kFxOne
    // units), which is associative, so the result does not depend on the
    // order the atomic ranks gave the occurrences: positive partials are
    // int64 rows (slotP64), duplicated users past their slot cap add with
    // int64 atomics (GU64), the per-pair losses add as integers (kFxLoss)
    int det_fx;
    long long* __restrict__ slotP64;        // [B / kPsortPPB + 1 + n_items, d] (as slotP)
    // users past their slot cap: compact int64 rows (round 5; was [n_users, d],
    // 512 MB at cfg2): psort gives each such user a row hotU[u] in the batch
    unsigned long long* __restrict__ GU64;  // [hot rows, d], zero between steps
    const int32_t* __restrict__ hotU;       // [n_users] compact row of a user past its cap (this batch)
    unsigned long long* __restrict__ GV64;  // [n_items, d]: positive partials past capP, zero between steps
    int* __restrict__ fx_bad;               // set when a term / sum leaves the fixed-point range (to_fx)
    // speculative negative counts (round 4; pos_sort with the dense item
    // apply): the draw issues the returning count atomic of each negative's
    // FIRST candidate before the row scan that accepts or rejects it, so the
    // atomic's latency overlaps the scan instead of following it.  A rejected
    // first candidate (probability |Pos(u)| / n_items) leaves a phantom
    // occurrence (item, rank) in spec_ph: psort zeroes its compact slot row
    // (or resets the count of an item the phantom alone touched), the
    // gradient launch re-zeroes spec_n for the next draw into this buffer
    // set, and a discarded draw uncounts the phantoms.  null = off
    int2* __restrict__ spec_ph;             // [B * W]
    int* __restrict__ spec_n;
    int lane_draw;                          // 1: one lane per pair (neg_check 2, with the set)
    // tables (updated in place for rows seen once in the batch)
    float* __restrict__ U; float* __restrict__ AU; float* __restrict__ GU;
    float* __restrict__ V; float* __restrict__ AV; float* __restrict__ GV;
    float* __restrict__ b; float* __restrict__ Ab; float* __restrict__ Gb;
    // batch occurrence lists and per-row counts
    int32_t* __restrict__ occU;   // [B*(1+G)] u | groups
    int32_t* __restrict__ occV;   // [B*(1+W)] i | negatives
    int32_t* __restrict__ cntU;   // [n_users] occurrences in this batch (0 between steps)
    int32_t* __restrict__ cntV;   // [n_items]
    // duplicated rows (store-and-sum): occurrence rank inside its row (prep's
    // returning count atomic); row r owns the slot rows [r*cap, (r+1)*cap)
    int32_t* __restrict__ rankU;  // [B*(1+G)]
    int32_t* __restrict__ rankV;  // [B*(1+W)]
    float* __restrict__ slotU;    // [n_users * capU, d]
    float* __restrict__ slotV;    // [n_items * capV, d]
    int capU, capV;               // occurrences at rank >= cap use float atomics into G
    float* __restrict__ GVrep;    // [repV][n_items, d] extra item accumulators (hot rows)
    int repV;                     // replica mask: item occurrence k >= capV adds to copy k & repV
    // deterministic mode (cf_set_option "deterministic"): ranks come from a
    // stable sort of the batch's row ids, every occurrence of a duplicated row
    // owns the compact slot off[row] + rank (no caps, no float atomics), the
    // GBPR / PLR item-bias gradient too (slotVb); null = the fast path
    const int32_t* __restrict__ offU;   // [n_users] first sorted position of each touched row
    const int32_t* __restrict__ offV;   // [n_items]
    float* __restrict__ slotVb;         // [B*(1+W)] bias gradient per item occurrence
    // item records (cf_set_option "item_slots" 1): a duplicated item
    // occurrence in its slot range stores (pair, alpha, beta, which) -- its
    // gradient is alpha * X + beta * V_row, X = stashU[pair] (which 0) or
    // stashB[pair] (GBPR's group blend, which 1) -- instead of a slot row;
    // null = slot rows
    int4* __restrict__ recV;            // [n_items * capV] (deterministic mode: [B*(1+W)])
    float* __restrict__ stashU;         // [B, d] each pair's pre-update user row
    float* __restrict__ stashB;         // [B, d] GBPR blend rows
    double* __restrict__ loss_partial;  // [grad grid]
    // positive-sorted gradient (cf_set_option "pos_sort"; BPR / AMF / CML on
    // the phased kernel): the draw counts a pair's positive item in cntP
    // (rankV[p] = its rank among the batch's positives of that item) and its
    // negatives in cntV; psort orders the pairs by positive item (order), so
    // the pairs of one gradient block that share a positive item sum its
    // gradient in LDS and store ONE partial row per (block, item): partial k =
    // b - offP[i] / kPsortPPB of block b goes to slotP[b + i] when k < capP --
    // unique, since the runs are contiguous in item order, and item i's
    // partials are the contiguous rows [offP[i] / kPsortPPB + i, + min(blocks
    // its run spans, capP)) in block order -- else it adds with float atomics
    // into GV (deterministic mode: int64 atomics into GV64), so the apply's
    // chain for a Zipf-head item stays capP + 1 rows.  null cntP = off
    int32_t* __restrict__ cntP;         // [n_items] positives per item (0 between steps)
    // [B, psort_stride(W)] the pair at each positive-sorted position as one
    // contiguous record (u, i, j_0 .. j_{W-1}, then the ranks of u, j_0, ..
    // as 16-bit halves, clamped to 0xFFFF -- a rank only matters below the
    // slot caps, <= 256), so the gradient launch reads its ids coalesced
    const int32_t* __restrict__ srec;
    float* __restrict__ slotP;          // [B / kPsortPPB + 1 + n_items, d]
    int capP;
    // ... and the negatives in compact slots: with pos_sort, slotV is the
    // [B * W, d] array where negative occurrence k of item j stores its
    // gradient row at offN[j] + k (offN = exclusive scan of the negatives'
    // counts cntV), so an item's negative rows are contiguous.  psort writes
    // both scans interleaved, offPN[r] = (offP[r], offN[r]), r <= n_items
    // (offPN[n_items] = the totals): an item's counts are the differences of
    // two adjacent entries, one 16-B read
    // user sharding (GBPR group exchange): this rank owns global users
    // [shard_u0, shard_u1); a group member owned elsewhere is coded -1 - id in
    // occU until the exchange recodes it -1 - (its row in xrows / xgrads)
    int64_t shard_u0, shard_u1;
    const float* __restrict__ xrows;  // [sent, d] rows of other ranks' group users
    float* __restrict__ xgrads;       // [sent, d] their gradient rows
    // split exchange step (cf_xchg_grad_part): 1 = only the pairs whose group
    // members are all this rank's users (runs while the member rows are in
    // flight), 2 = only the others; 0 = every pair
    int member_pass;
    // tuple ranking (PLR): occV holds the tuple's items, W = width - 2
    int plr_kind;                     // 0 PRIGP, 1 CPLR
    float alpha, beta, gamma;
    int train_bias;                   // CPLR trains b (cplr_u.py:152); PRIGP does not (prigp.py:145)
    const float* __restrict__ coefs;  // [B, 2] CPLR (coefMat[u,i], coefMat[u,t])
};

// a row of this rank's user table that other ranks' batches touch: its count
// word carries this flag, so it takes the summed (float-atomic) path
constexpr int32_t kRemoteFlag = 1 << 24;
// positive-sorted positions per gradient block (the phased kernel at one pair
// per 16-lane group): partial k of an item covers the positions of block
// offP[i] / kPsortPPB + k
constexpr int kPsortPPB = kGroupsPerBlock;
// fixed-point units of the deterministic pos_sort path: gradients 2^-32
// (|sum| < 2^31), per-pair losses 2^-24 (a step's integer total < 2^53)
constexpr float kFxOne = 4294967296.f;
constexpr double kFxInv = 1.0 / 4294967296.0;
constexpr double kFxLoss = 16777216.0;
// the guarded range (to_fx): terms |x| < 2^20, sums |x| < 2^30 (in units: 2^62)
constexpr float kFxTermMax = 1048576.f;
constexpr long long kFxSumMax = 1ll << 62;

// A pos_sort record carries every occurrence's resolved destination --
// psort_scatter reads the batch's final counts and offsets, so the gradient
// launch issues its accumulator loads together with the rows (no dependent
// count phase).  Ints per record, int4-aligned (W = 1 -> 8, W = 5 -> 16):
//   [u, i, j_0 .. j_{W-1}, su, pi, sj_0 .. sj_{W-1}, 0 padding]
// su / sj: >= 0 the slot row (users u * capU + rank, negatives the compact
// slot offN[j] + rank), kSlotApply = the row's only occurrence in the batch
// (Adagrad in place), kSlotAtomic = float atomics into the dense gradient;
// pi = offP[i], bit 31 set when the positive is its item's only occurrence
__host__ __device__ constexpr int psort_stride(int W) { return (4 + 2 * W + 3) & ~3; }
constexpr int32_t kSlotApply = -1;
constexpr int32_t kSlotAtomic = -2;

struct XchgArgs {
    int n;                        // group occurrences (B * G)
    int world;
    const int64_t* __restrict__ bounds;   // [world + 1] global user id ranges
    int32_t* __restrict__ occ;            // [n] group occurrences (occU + B)
    int32_t* __restrict__ hist;           // [blocks][world] remote occurrences per block
    int32_t* __restrict__ counts;         // [world + 1] per owner, [world] = total
    int32_t* __restrict__ send_ids;       // [n] global ids packed by owner
};

struct ApplyArgs {
    int det_fx;                               // fixed-point sums (StepArgs::det_fx)
    const long long* __restrict__ slotP64;
    unsigned long long* __restrict__ GU64;   // StepArgs::GU64 (compact rows via hotU)
    const int32_t* __restrict__ hotU;
    int* __restrict__ hot_n;                 // the compact rows handed out by psort; block 0 re-zeroes it
    unsigned long long* __restrict__ GV64;
    int* __restrict__ fx_bad;                 // StepArgs::fx_bad
    int d;
    float lr;
    float clip_norm;
    int clip;            // CML: clip updated rows
    int capU, capV;      // fixed slot range per row
    float* __restrict__ GVrep;  // hot item rows: extra accumulators (StepArgs)
    int repV;
    int64_t n_items;
    int count_users, count_items;
    int items_grad_only; // item owners store the summed gradient row into GV
    // work items: the batch's occurrences (+ the served rows of the group
    // exchange); the owner of a duplicated row applies it
    const int32_t* __restrict__ occU;
    const int32_t* __restrict__ rankU;
    int64_t nU;
    const int32_t* __restrict__ occV;
    const int32_t* __restrict__ rankV;
    int64_t nV;
    const int32_t* __restrict__ served_ids;   // global user ids
    const int32_t* __restrict__ served_own;   // 1: this served row applies it
    int64_t nS;
    int64_t shard_u0;
    const float* __restrict__ slotU;
    const float* __restrict__ slotV;
    const int32_t* __restrict__ offU;    // deterministic mode (StepArgs)
    const int32_t* __restrict__ offV;
    const float* __restrict__ slotVb;
    const int4* __restrict__ recV;       // item records (StepArgs)
    const float* __restrict__ stashU;
    const float* __restrict__ stashB;
    // deterministic mode: sums of the 64-slot tiles that lie inside one row
    // (det_hot_kernel); a row with >= 2 x 64 slots adds them in tile order
    // between its head and tail slots
    const float* __restrict__ hotP;      // [tiles, d]
    const float* __restrict__ hotPb;     // [tiles] records: the tile's beta sum
    // positive-sorted gradient (StepArgs): positives are occV[0, nPos);
    // negatives' compact slot rows at slotV[offN[r] + k]
    int32_t* __restrict__ cntP;
    const int2* __restrict__ offPN;      // [n_items + 1] (offP, offN), see StepArgs
    const float* __restrict__ slotP;     // see StepArgs
    int capP;
    int64_t nPos;
    // pos_sort apply: visit every item row (dense_items) / every user row
    // (dense_users) instead of finding the owners among the occurrences --
    // when the table is not much larger than the batch's occurrences of it
    int dense_items, dense_users;
    // dense item rows [item_r0, item_r1) only (the multi-rank item reduce in
    // pieces, cf_step_item_reduce; default the whole table)
    int64_t item_r0, item_r1;
    int64_t n_users;
    int32_t* __restrict__ cntU;
    int32_t* __restrict__ cntV;
    float* __restrict__ U; float* __restrict__ AU; float* __restrict__ GU;
    float* __restrict__ V; float* __restrict__ AV; float* __restrict__ GV;
    float* __restrict__ b; float* __restrict__ Ab; float* __restrict__ Gb;  // nullable
    // loss reduction (block 0)
    const double* __restrict__ loss_partial;
    int n_partial;
    double* __restrict__ loss_acc;
};

// deterministic mode: the slot sums of every 64-position tile of the sorted
// occurrence list (users [0, nU), then items) that lies inside one row
constexpr int kDetTile = 64;
struct HotArgs {
    int d;
    int64_t n, nU, n_users;
    const int32_t* __restrict__ skeys;   // sorted row keys (items offset by n_users)
    const float* __restrict__ slotU;     // compact user slot rows
    const float* __restrict__ slotV;     // compact item slot rows (null with records)
    const int4* __restrict__ recV;       // compact item records (null with slot rows)
    const float* __restrict__ stashU;
    const float* __restrict__ stashB;
    float* __restrict__ P;               // [n / kDetTile, d]
    float* __restrict__ Pb;              // [n / kDetTile]
};
hipError_t launch_det_hot(const HotArgs& h, hipStream_t s);

struct DenseArgs {
    int d;
    float lr;
    float clip_norm;
    int clip;
    int zero_g;          // re-zero the consumed gradient rows (the all-reduced
                         // buffer is reused; a reduce-scatter slice is not)
    int64_t n_rows;
    float* __restrict__ X; float* __restrict__ A; float* __restrict__ G;
    float* __restrict__ b; float* __restrict__ Ab; float* __restrict__ Gb;  // nullable
};

struct ScoreArgs {
    int model;
    int d;
    int n_users;            // users in this chunk
    int64_t n_items;
    const int32_t* __restrict__ users;   // [n_users] global ids
    const float* __restrict__ U;
    const float* __restrict__ V;
    const float* __restrict__ b;         // nullable
    uint32_t* __restrict__ keys;         // [n_users, n_items] order-preserving keys
    int exclude_train;
    const int64_t* __restrict__ indptr;
    const int32_t* __restrict__ indices;
    const uint64_t* __restrict__ item_mask;   // [ceil(n_items / 64)] excluded items (bit j % 64 of word j / 64), nullable
};

// fused scoring GEMM (fp32 MFMA) + streaming per-user top-k, d <= 128, k <= 128
constexpr int kFusedUsers = 64;
constexpr int kFusedItems = 64;
constexpr int kFusedMaxD = 128;
constexpr int kFusedCap = 92;    // candidate slots per user (LDS for two blocks per CU)
constexpr int kFusedMaxK = kFusedCap - kFusedItems;   // a compacted list + one tile's 64 fit
// 28 < k <= 128 (round 5: GBPR's topN = 100, testgbprmf.py:23-32): 192 slots
// per user, ~130 KB of LDS, one block per CU
constexpr int kFusedCapWide = 192;
constexpr int kFusedMaxWideK = kFusedCapWide - kFusedItems;

struct FusedTopkArgs {
    int model;
    int d, Dp, Dh;            // Dp = d rounded up to 8, Dh = Dp / 2
    int n_users;              // users in this launch
    int64_t n_items;
    int k;
    const int32_t* __restrict__ users;
    const float* __restrict__ U;
    const float* __restrict__ V;
    const float* __restrict__ b;         // GBPR bias (nullable)
    int exclude_train;
    const int64_t* __restrict__ indptr;
    const int32_t* __restrict__ indices;
    int32_t* __restrict__ idx_out;       // [n_users, k]
    float* __restrict__ val_out;         // [n_users, k] (nullable)
    int variant;                         // 0: the sequential kernel, 1: software-pipelined (A/B)
    const uint64_t* __restrict__ item_mask;   // as ScoreArgs::item_mask, nullable
    unsigned long long* stamps;          // -DCF_FUSED_STAMPS diagnostic builds only: [blocks][waves][8]
};

struct TopkArgs {
    int k;
    int64_t n_items;
    const uint32_t* __restrict__ keys;
    int32_t* __restrict__ idx_out;   // [n_users, k]
    float* __restrict__ val_out;     // [n_users, k]
};

// ---- host launchers (cf_kernels.hip / cf_eval.hip) -------------------------
hipError_t launch_prep(const StepArgs& a, hipStream_t s);   // sample/load + count
// gather, loss, grads, singleton apply; with `next`, the same launch also
// draws and counts the next step's batch (other buffer set)
hipError_t launch_grad(const StepArgs& a, hipStream_t s, const StepArgs* next = nullptr);
// AMF apr: the embedding-loss pass alone (cf_step_local_apr_embed)
hipError_t launch_apr_embed(const StepArgs& a, hipStream_t s);
// the phased gradient kernel's compile-time W (1 or 5) a step takes, 0 = generic
int grad_fast_w(const StepArgs& a);
// the step takes grad_lds_kernel (LDS-staged negatives)
bool grad_lds(const StepArgs& a);
// blocks (= loss partials) of the grad launch for this step shape
int grad_blocks(const StepArgs& a, bool with_draw = false);
int grad_blocks_max(int B);  // upper bound over every grad variant
hipError_t launch_apply(const ApplyArgs& a, hipStream_t s);
// apply of step s and prep of step s+1 in one launch (device-sampler pipeline)
hipError_t launch_apply_prep(const ApplyArgs& p, const StepArgs& next, hipStream_t s);

hipError_t launch_apply_dense(const DenseArgs& a, hipStream_t s);
// zero the rows of G (and Gb, nullable) that a batch's occurrences touched
hipError_t launch_zero_rows(const int32_t* occ, int64_t n, float* G, float* Gb, int d, hipStream_t s);
hipError_t launch_clip_full(float* X, int64_t n_rows, int d, float clip_norm, hipStream_t s);
hipError_t launch_init_normal(float* X, int64_t n, float mean, float stddev, int truncated,
                              uint64_t seed, hipStream_t s);
hipError_t launch_fill(float* X, int64_t n, float v, hipStream_t s);
// zero the counts of a batch's occurrences (a drawn-ahead batch is dropped)
hipError_t launch_uncount(const int32_t* occ, int64_t n, int32_t* cnt, hipStream_t s);

// A caller batch already in device memory (torch tensors): user / item /
// negative / group ids read with row strides (cf_step: pairs [B,2], negs
// [B,W], groups [B,G]; cf_step_plr: tuples [B,width]) into the occurrence
// arrays, range-checked on the device; *bad = the first offending row
// (initialised to kPackOk by the caller).  Out-of-range ids are stored as 0.
constexpr int32_t kPackOk = 0x7F7F7F7F;
struct PackArgs {
    const int32_t* u; int us;        // u = u[p*us], i = u[p*us + 1]
    const int32_t* j; int js;        // negative w = j[p*js + w]
    const int32_t* g; int gs;        // group k = g[p*gs + k]
    int B, W, G;
    int64_t n_users, n_items;
    int sharded;                     // group ids are global: own -> local, else -1 - id
    int64_t shard_u0, shard_u1, total_users;
    int32_t* occU; int32_t* occV; int32_t* bad;
};
hipError_t launch_pack_batch(const PackArgs& a, hipStream_t s);
// deterministic ranks (cf_det.hip): a stable radix sort of the batch's row ids
// (users, then items offset by n_users) gives every occurrence its rank among
// the earlier occurrences of its row, and off[row] = the row's first sorted
// position; tmp / keys / vals sized by det_ranks_scratch
size_t det_ranks_scratch(int64_t n_occ, int64_t n_rows);
hipError_t launch_det_ranks(const int32_t* occU, int64_t nU, const int32_t* occV, int64_t nV,
                            int64_t n_users, int64_t n_rows, int32_t* rankU, int32_t* rankV,
                            int32_t* off, int32_t* keys, int32_t* vals, void* tmp, size_t tmp_bytes,
                            hipStream_t s);
// positive-sorted gradient: offPN = exclusive scans of (cntP, cntV) (two
// launches of tile sums + tile scans), then the pair records at
// srec[offP[i_p] + rankV[p]] for the B pairs; tmp sized by psort_scratch
size_t psort_scratch(int64_t n_items);
struct PsortArgs {
    const int32_t* occU; const int32_t* rankU;
    const int32_t* occV; const int32_t* rankV;
    const int32_t* cntU;                 // the batch's final counts
    // deterministic mode: a user's occurrence of rank capU (the user is past
    // its slot cap) takes the next compact GU64 row, hotU[u] (null = off)
    int32_t* hotU;
    int* hot_n;
    const int32_t* cntV; const int32_t* cntP;
    int2* offPN;                         // written: [n_items + 1] exclusive scans of (cntP, cntV)
    int32_t* srec;                       // [B, psort_stride(W)]
    int B, W, capU;
    int64_t n_items;
    // speculative negative counts (StepArgs::spec_ph): the phantoms' compact
    // slot rows of slotN are zeroed, a phantom-only item's count reset
    const int2* spec_ph;
    const int* spec_n;
    float* slotN;
    int32_t* cntVw;
    int d;
};
hipError_t launch_psort(const PsortArgs& a, void* tmp, size_t tmp_bytes, hipStream_t s);
// sorted batches: keys / vals hold 2 * nnz int32 each; *order_out = the
// epoch's pair indices sorted by (batch, pair) -- batch b at [b B, (b+1) B)
size_t epoch_order_scratch(int64_t nnz, int32_t n_batches);
hipError_t launch_epoch_order(const PermKey& p, int64_t nnz, int B, int32_t* keys, int32_t* vals, void* tmp,
                              size_t tmp_bytes, const int32_t** order_out, hipStream_t s);
// the records form (sorted_batches 1 / 2): the records instead (recs: 2 * nnz
// int4), *recs_out = the epoch's pair records in that order
// (both hipCUB radix sorts: the fallback above kEpochMaxBins bins and
// cf_set_option("epoch_sort", 1); the default is launch_epoch_count)
size_t epoch_records_scratch(int64_t nnz, int32_t n_batches);
hipError_t launch_epoch_records(const PermKey& p, int64_t nnz, int B, const int4* pairs, int32_t* keys, int4* recs,
                                void* tmp, size_t tmp_bytes, const int4** recs_out, hipStream_t s);
// the same orders as one hand-written counting sort by batch id
// (cf_epoch.hip), for nnz <= 2^31 and at most kEpochMaxBins = nnz / B + 1
// bins: out_recs[nnz] (records form, pairs != null) or out_idx[nnz] (index
// form), bitwise the stable radix sort's result
constexpr int kEpochMaxBins = 1024;
bool epoch_count_ok(int64_t nnz, int B);
size_t epoch_count_scratch(int64_t nnz, int B);
hipError_t launch_epoch_count(const PermKey& p, int64_t nnz, int B, const int4* pairs, int4* out_recs,
                              int32_t* out_idx, void* tmp, size_t tmp_bytes, hipStream_t s);
// a discarded draw's phantoms (StepArgs::spec_ph): uncount them, re-zero spec_n
hipError_t launch_uncount_spec(const int2* ph, int* n, int32_t* cnt, hipStream_t s);
// grad_sort_kernel carries the pair-record prefetch (StepArgs::pf_out)
bool pair_prefetch_built();
hipError_t launch_build_pos_set(const int4* pairs, int64_t nnz, unsigned long long* set,
                                uint64_t mask, hipStream_t s);
hipError_t launch_build_pairs(const int64_t* indptr, const int32_t* indices, int64_t n_users,
                              int4* pairs, hipStream_t s);
hipError_t launch_score(const ScoreArgs& a, hipStream_t s);
hipError_t launch_topk(const TopkArgs& a, int n_users, hipStream_t s);
hipError_t launch_fused_topk(const FusedTopkArgs& a, hipStream_t s);
// group exchange: pack the remote group members of a batch by owner
hipError_t launch_xchg_pack(const XchgArgs& a, hipStream_t s);
// owner side: flag + gather the requested rows; scatter-add their gradients
hipError_t launch_xchg_serve(const int32_t* ids, int64_t n, int64_t u0, int32_t* cntU, int32_t* own,
                             const float* U, float* rows, int d, hipStream_t s);
hipError_t launch_xchg_accumulate(const int32_t* ids, int64_t n, int64_t u0, const float* grads,
                                  float* GU, int d, hipStream_t s);

// host-side mirror of the device bijection (for key generation)
PermKey make_perm_key(uint64_t n, uint64_t seed, uint64_t epoch);
uint64_t mix64_host(uint64_t z);

}  // namespace cfk
