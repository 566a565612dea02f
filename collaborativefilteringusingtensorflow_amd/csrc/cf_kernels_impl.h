// cf_kernels_impl.h -- the gfx950 device code of the engine, shared by the
// translation units that instantiate it: cf_kernels.hip (draw, apply, dense,
// exchange, the exported launchers) and cf_grad_<model>.hip (one gradient
// launcher per model, compiled in parallel).  Templates and inline helpers
// only; every non-template kernel and exported function lives in one .hip.
#pragma once
// cf_kernels.hip -- the training hot path for gfx950 (MI355X / CDNA4).
//
// One optimizer step of BPRMF / GBPRMF / CML / AMF is four launches; the
// unit of parallelism is a 16-lane group per (u,i) pair / per row, four per
// wave, so a wave keeps four pairs' gathers in flight.
//
//  prep_kernel   draw the batch on device -- epoch bijection over the nnz
//                pairs, W negatives whose membership in Pos(u) the 16 lanes
//                test cooperatively against the user's sorted CSR row
//                (one coalesced pass, group-OR of hit masks, redraw only the
//                rejected ones), G group users from the item's CSC column --
//                or take a host-fed batch; then count every touched row's
//                occurrences (returning atomicAdd: the old value is the
//                occurrence's rank inside its row).
//  grad_kernel   gather U[u], V[i], V[j] (+U[g], b) rows, group-reduce the
//                dots / distances, evaluate the loss and dL/dx, form every
//                per-occurrence gradient row.  A row that occurs ONCE in the
//                batch is updated right here with SparseApplyAdagrad
//                (acc += g^2; w -= lr*g/sqrt(acc); CML: clip) -- its
//                pre-update value is already in registers.  A duplicated
//                row's gradient is a plain store into its slot row: row r
//                owns the fixed slot range [r*cap, (r+1)*cap) and occurrence
//                k of r (prep's returning count atomic) writes slot r*cap + k.
//                Hot rows (> cap occurrences) scatter-add into a dense fp32
//                accumulator with float atomics.  So duplicates SUM before
//                the update: TF1's _deduplicate_indexed_slices.
//  apply_kernel  one lane per occurrence: the first occurrence (rank 0) of a
//                duplicated row sums the row's slot rows in rank order (or
//                takes its atomic sum), applies Adagrad and resets the count.
//                Fixed slot ranges: no duplicate list, no scan, no extra launch.
//
// Float atomics run at the memory side at ~1.3 TB/s chip-wide, plain stores
// at ~6 TB/s: the store-and-sum form moves the duplicate gradients ~4x faster.
// Reference semantics: src/models/pl/models/bprmf.py:52-88,
// gbprmf.py:58-106, cml.py:55-129, src/models/others/models/amf.py:66-162;
// samplers src/samplers/sampler_ranking.py:22-37, sampler_gbpr.py:23-43.
#include <algorithm>

#include "cf_kernels.h"
#include "cf_device.h"

namespace cfk {

// ---------------------------------------------------------------------------
// 16-lane group helpers.  A row of d floats is held as EPL slots per lane.
// Rows that fill every slot (d == 16*EPL: d = 16, 32, 64, 128, 256) use the
// vector layout: lane gl holds VW = min(EPL, 4) contiguous floats of each
// 64*VW-byte stripe, so one dwordx{VW} instruction moves a whole stripe of
// four rows (one per group of the wave) -- a 256-B row (d = 64) is one
// 16-B-per-lane access.  Other d use the scalar layout: element s*16 + gl,
// masked by e < d.  Arithmetic is layout-blind (slot-wise, with group
// reductions); memory stays row-major either way.
// ---------------------------------------------------------------------------
// The vector layout measured no faster on the gather (46.0 vs 44.9 us, cfg2
// grad without atomics) and its float atomics touch four 64-B segments per
// row-stripe instead of one (grad 105 vs 50 us), so the scalar layout is the
// default; -DCF_VEC_ROWS=1 builds the vector layout for experiments.
#ifndef CF_VEC_ROWS
#define CF_VEC_ROWS 0
#endif
// Round 5: rows of d > 64 (EPL >= 8: cfg3 / cfg5's d = 128) take the vector
// layout by default -- the apply's 512-B slot and table rows move as two
// float4 per lane: cfg5 apply + draw 96.2 -> 88.8 us, 0.2013 -> 0.1940
// ms/step; the d = 64 kernels keep the scalar one (cfg2 gradient 164.5 ->
// 194.5 us with it, cfg4 apply 77.4 -> 86.0; profiles/r05/ab/r05h_*).  The
// mapping is per kernel (memory rows are always natural order), so kernels
// with different layouts exchange rows freely
#ifndef CF_VEC_ROWS_WIDE
#define CF_VEC_ROWS_WIDE 1
#endif
template <int EPL>
__host__ __device__ constexpr bool vec_rows() { return CF_VEC_ROWS || (CF_VEC_ROWS_WIDE && EPL >= 8); }
template <int EPL>
struct Lay {
    static constexpr int VW = vec_rows<EPL>() ? (EPL >= 4 ? 4 : EPL) : 1;
    static constexpr int NQ = EPL / VW;  // stripes per row
};

// element index of slot s in lane gl (full rows: vector layout)
template <int EPL>
__device__ __forceinline__ int elem_of(int s, int gl, bool full) {
    constexpr int VW = Lay<EPL>::VW;
    return full ? (s / VW) * (kGL * VW) + gl * VW + (s % VW) : s * kGL + gl;
}

template <int EPL>
__device__ __forceinline__ void row_ld(const float* __restrict__ row, int d, int gl, float fill,
                                       float (&x)[EPL]) {
    constexpr int VW = Lay<EPL>::VW;
    if (vec_rows<EPL>() && d == kGL * EPL) {
#pragma unroll
        for (int q = 0; q < Lay<EPL>::NQ; ++q) {
            const float* p = row + q * (kGL * VW) + gl * VW;
            if constexpr (VW == 4) {
                const float4 v = *reinterpret_cast<const float4*>(p);
                x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
            } else if constexpr (VW == 2) {
                const float2 v = *reinterpret_cast<const float2*>(p);
                x[2 * q] = v.x; x[2 * q + 1] = v.y;
            } else {
                x[q] = p[0];
            }
        }
    } else {
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const int e = s * kGL + gl;
            x[s] = (e < d) ? row[e] : fill;
        }
    }
}

template <int EPL>
__device__ __forceinline__ void row_st(float* __restrict__ row, int d, int gl, const float (&x)[EPL]) {
    constexpr int VW = Lay<EPL>::VW;
    if (vec_rows<EPL>() && d == kGL * EPL) {
#pragma unroll
        for (int q = 0; q < Lay<EPL>::NQ; ++q) {
            float* p = row + q * (kGL * VW) + gl * VW;
            if constexpr (VW == 4) {
                *reinterpret_cast<float4*>(p) = make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
            } else if constexpr (VW == 2) {
                *reinterpret_cast<float2*>(p) = make_float2(x[2 * q], x[2 * q + 1]);
            } else {
                p[0] = x[q];
            }
        }
    } else {
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const int e = s * kGL + gl;
            if (e < d) row[e] = x[s];
        }
    }
}

template <int EPL>
__device__ __forceinline__ void row_zero(float* __restrict__ row, int d, int gl) {
    float z[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) z[s] = 0.f;
    row_st<EPL>(row, d, gl, z);
}
// the sum over a 16-lane group, identical in every lane of it.  A group is
// one DPP row, so (round 4) the butterfly runs on DPP: quad_perm [1,0,3,2]
// and [2,3,0,1] sum each quad, row_half_mirror adds the other quad of the
// half-row (every lane of a quad holds the same value by then, so any
// partner in it gives the same sum) and row_mirror the other half-row --
// four VALU ops with a DPP operand instead of four ds_bpermute round trips
// through the LDS crossbar.  Called group-uniformly (no lane of the row is
// inactive).  CF_DPP_GSUM 0: the xor butterfly on __shfl_xor.
#ifndef CF_DPP_GSUM
#define CF_DPP_GSUM 1
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float gsum(float v) {
#if CF_DPP_GSUM
    v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);   // row_half_mirror
    v += dpp_f<0x140>(v);   // row_mirror
#else
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 1, 64);
#endif
    return v;
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// OR over a 16-lane group (one DPP row), the same steps as gsum
__device__ __forceinline__ uint32_t gor(uint32_t v) {
#if CF_DPP_GSUM
    v |= dpp_u<0xB1>(v);
    v |= dpp_u<0x4E>(v);
    v |= dpp_u<0x141>(v);
    v |= dpp_u<0x140>(v);
#else
    v |= (uint32_t)__shfl_xor((int)v, 8, 64);
    v |= (uint32_t)__shfl_xor((int)v, 4, 64);
    v |= (uint32_t)__shfl_xor((int)v, 2, 64);
    v |= (uint32_t)__shfl_xor((int)v, 1, 64);
#endif
    return v;
}

template <int EPL>
__device__ __forceinline__ void gload(const float* __restrict__ X, int64_t r, int d, int gl,
                                      float (&x)[EPL]) {
    row_ld<EPL>(X + r * (int64_t)d, d, gl, 0.f, x);
}

template <int EPL>
__device__ __forceinline__ void gatomic(float* __restrict__ G, int64_t r, int d, int gl,
                                        const float (&g)[EPL]) {
    float* row = G + r * (int64_t)d;
    const bool full = vec_rows<EPL>() && d == kGL * EPL;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = elem_of<EPL>(s, gl, full);
        if (e < d) unsafeAtomicAdd(row + e, g[s]);
    }
}

// deterministic mode on the positive-sorted path (StepArgs::det_fx): row sums
// in 64-bit fixed point -- integer adds are associative, so a sum does not
// depend on the order the occurrences arrive in (the atomic ranks, which
// pairs share a gradient block).  to_fx rounds once per term.  The range is
// guarded (StepArgs::fx_bad): a term that is not finite or has |x| >= 2^20,
// or a sum with |x| >= 2^30, raises the engine's flag -- the call then
// fails with CF_ENUMERIC instead of leaving a wrapped integer in the table --
// and a sum past the range converts back to NaN, as the fp32 path would
// carry an inf / NaN gradient into the table.  Terms below 2^20 cannot wrap
// the 2^63 range of a sum of fewer than 2^11 of them; a longer sum of
// terms that large belongs to a run whose terms crossed 2^20 already.
__device__ __forceinline__ long long to_fx(float x, int* __restrict__ bad) {
    if (!(fabsf(x) < kFxTermMax)) *bad = 1;
    return __float2ll_rn(x * kFxOne);
}
__device__ __forceinline__ float from_fx(long long v, int* __restrict__ bad) {
    if (v >= kFxSumMax || v <= -kFxSumMax) {
        *bad = 1;
        return __builtin_nanf("");
    }
    return (float)((double)v * kFxInv);
}

template <int EPL>
__device__ __forceinline__ void fx_ld_add(const long long* __restrict__ row, int d, int gl, long long (&t)[EPL]) {
    const bool full = vec_rows<EPL>() && d == kGL * EPL;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = elem_of<EPL>(s, gl, full);
        if (e < d) t[s] += row[e];
    }
}

template <int EPL>
__device__ __forceinline__ void fx_st(long long* __restrict__ row, int d, int gl, const long long (&t)[EPL]) {
    const bool full = vec_rows<EPL>() && d == kGL * EPL;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = elem_of<EPL>(s, gl, full);
        if (e < d) row[e] = t[s];
    }
}

template <int EPL>
__device__ __forceinline__ void fx_atomic(unsigned long long* __restrict__ row, int d, int gl, const float (&g)[EPL],
                                          int* __restrict__ bad) {
    const bool full = vec_rows<EPL>() && d == kGL * EPL;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = elem_of<EPL>(s, gl, full);
        if (e < d) atomicAdd(row + e, (unsigned long long)to_fx(g[s], bad));
    }
}

template <int EPL>
__device__ __forceinline__ float gdot(const float (&x)[EPL], const float (&y)[EPL]) {
    float t = 0.f;
#pragma unroll
    for (int s = 0; s < EPL; ++s) t = fmaf(x[s], y[s], t);
    return gsum(t);
}

// SparseApplyAdagrad on one row whose pre-update value x0 is in registers
// (+ tf.clip_by_norm for CML): acc += g^2; x = x0 - lr*g/sqrt(acc)
template <int EPL>
__device__ __forceinline__ void gapply(float* __restrict__ X, float* __restrict__ A, int64_t r,
                                       int d, int gl, const float (&x0)[EPL],
                                       const float (&g)[EPL], float lr, bool clip, float c) {
    float* xr = X + r * (int64_t)d;
    float* ar = A + r * (int64_t)d;
    float acc[EPL], x[EPL];
    row_ld<EPL>(ar, d, gl, 1.f, acc);
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        acc[s] = fmaf(g[s], g[s], acc[s]);
        x[s] = x0[s] - adagrad_delta(lr, g[s], acc[s]);
    }
    if (clip) {
        const float n = sqrtf(gdot<EPL>(x, x));
        const float den = fmaxf(n, c);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * c) / den;
    }
    row_st<EPL>(xr, d, gl, x);
    row_st<EPL>(ar, d, gl, acc);
}

template <int EPL>
__device__ __forceinline__ void gstore(float* __restrict__ S, int64_t r, int d, int gl,
                                       const float (&g)[EPL]) {
    row_st<EPL>(S + r * (int64_t)d, d, gl, g);
}

// slot row of one occurrence of a duplicated row: row r owns the fixed slots
// [r*cap, (r+1)*cap) and occurrence `rank` < cap stores there.  Occurrences
// at rank >= cap of a hot row, every occurrence of a row flagged by the group
// exchange and those of an uncounted table go to float atomics: -1 - k means
// accumulator copy k (0 = G itself; items spread a hot row over repV + 1
// copies by rank, so its atomics do not all queue on one address)
__device__ __forceinline__ int64_t slot_of(int count, int64_t r, int rank, int cap, int rep,
                                           const int32_t* __restrict__ off) {
    if (off != nullptr) return count >= 2 ? (int64_t)off[r] + rank : -1;  // deterministic: compact
    if (count >= 2 && !(count & kRemoteFlag) && rank < cap) return r * (int64_t)cap + rank;
    return -1 - (rank & rep);
}

// the accumulator an atomic-path occurrence adds to (see slot_of)
__device__ __forceinline__ float* acc_of(float* G, int64_t slot, const StepArgs& a) {
    return slot == -1 ? G : a.GVrep + (-2 - slot) * a.n_items * (int64_t)a.d;
}

// row r of X: singleton -> apply now; duplicated -> its slot row (summed by
// apply_kernel in rank order) or, for hot rows, float atomics into G
template <int EPL>
__device__ __forceinline__ void gfinish(float* __restrict__ X, float* __restrict__ A,
                                        float* __restrict__ G, float* __restrict__ S,
                                        int32_t* __restrict__ cnt,
                                        int64_t r, int count, int64_t slot, int d, int gl,
                                        const float (&x0)[EPL], const float (&g)[EPL],
                                        const StepArgs& a) {
    if (count == 1) {
        if (a.items_grad_only && X == a.V)
            gstore<EPL>(G, r, d, gl, g);  // sole writer of the zeroed dense row
        else
            gapply<EPL>(X, A, r, d, gl, x0, g, a.lr, a.clip != 0, a.clip_norm);
        if (gl == 0) cnt[r] = 0;
    } else if (slot >= 0) {
        gstore<EPL>(S, slot, d, gl, g);
    } else {
        gatomic<EPL>(acc_of(G, slot, a), r, d, gl, g);
        // item_reduce 2 (no reduce launch): the atomic path resets the count
        // itself; a count read as 0 by a later occurrence still means atomics
        if (a.items_grad_only && a.capV == 0 && X == a.V && gl == 0) cnt[r] = 0;
    }
}

// A duplicated item row's gradient from one pair is alpha * X + beta * V_row,
// X the pair's pre-update user row (stashU) or, for GBPR's positive, its
// group blend rho/G sum U_g + (1-rho) U_u (stashB): with item records
// (cf_set_option "item_slots" 1) the slot gets the 16-B record
// (pair, alpha, beta, which) instead of the 4d-B gradient row, and the apply
// sums alpha * X from the stash + (sum of beta) * V_row.  Rows seen once and
// hot rows past their slot range take gfinish with g in registers.
template <int EPL>
__device__ __forceinline__ void ifinish(const StepArgs& a, int64_t r, int count, int64_t slot, int p,
                                        float alpha, float beta, int which, int gl,
                                        const float (&x0)[EPL], const float (&g)[EPL]) {
    if (a.recV != nullptr && count >= 2 && slot >= 0) {
        if (gl == 0) a.recV[slot] = make_int4(p, __float_as_int(alpha), __float_as_int(beta), which);
        return;
    }
    gfinish<EPL>(a.V, a.AV, a.GV, a.slotV, a.cntV, r, count, slot, a.d, gl, x0, g, a);
}

__device__ __forceinline__ void bias_finish(const StepArgs& a, int64_t r, int count, float g,
                                            int64_t slot) {
    // GBPR / CPLR item bias: one scalar per row, summed like the row itself
    if (count == 1) {
        if (!a.items_grad_only) {
            const float acc = fmaf(g, g, a.Ab[r]);
            a.Ab[r] = acc;
            a.b[r] -= adagrad_delta(a.lr, g, acc);
        } else {
            a.Gb[r] = g;   // multi-rank item reduce: the sole writer of a zeroed entry
        }
    } else if (slot >= 0 && a.slotVb != nullptr) {
        a.slotVb[slot] = g;   // beside the row's slot row; the apply sums them in rank order
    } else {
        unsafeAtomicAdd(a.Gb + r, g);   // a hot row past its slot range
    }
}

// bias_finish with the row's bias and accumulator already in registers (the
// phased kernel loads them with the rows): no load at the end of the pair
__device__ __forceinline__ void bias_finish_pre(const StepArgs& a, int64_t r, int count, float g,
                                                int64_t slot, float b0, float ab0) {
    if (count == 1 && !a.items_grad_only) {
        const float acc = fmaf(g, g, ab0);
        a.Ab[r] = acc;
        a.b[r] = b0 - adagrad_delta(a.lr, g, acc);
    } else {
        bias_finish(a, r, count, g, slot);
    }
}

__device__ __forceinline__ float neg_log_sigmoid(float x) {
    // literal -log(sigmoid(x)) as in bprmf.py:70 / gbprmf.py:88
    return -logf(rcp_1p(expf(-x)));
}

__device__ __forceinline__ float softplus(float x) {
    // tf.nn.softplus: log(1 + exp(x)), evaluated stably
    return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
}

__device__ __forceinline__ int32_t draw_item(uint64_t key, uint64_t ctr, int64_t n_items) {
    return (int32_t)uniform_below(mix64(key + ctr), (uint64_t)n_items);
}

// ---------------------------------------------------------------------------
// prep: sample (or load) the batch and count row occurrences
// ---------------------------------------------------------------------------
// The draw runs 8 lanes per pair (32 pairs per block): one wave generation
// covers a 65,536-pair batch at full occupancy, and a user's row (~51 ids at
// cfg2) is tested in one batch of up to 8 independent 32-B loads.
#ifndef CF_PREP_GL
#define CF_PREP_GL 8       // lanes per pair in the draw (a power of two, 2..16)
#endif
#ifndef CF_PREP_CHUNKS
#define CF_PREP_CHUNKS 8   // row chunks in flight per candidate test
#endif
constexpr int kPrepGL = CF_PREP_GL;
constexpr int kPrepPairsPerBlock = kBlock / kPrepGL;
constexpr int kPrepChunks = CF_PREP_CHUNKS;
// W = 1 (cfg2): 4 lanes per pair (round 4).  Four candidates per row scan
// still leave a rejection of all of them at |Pos(u)|^4 / n_items^4, and a
// wave draws 16 pairs instead of 8 -- half the draw's waves, whose integer
// hashing (permute, draw_item) is paid per wave-instruction whatever the
// lanes.  Each lane keeps 64 / 4 = 16 row chunks in flight (one scan covers
// 64 ids, as the 8-lane group's 8 x 8).  W = 5 keeps 8 lanes: all five
// negatives' first attempts in one scan.
#ifndef CF_PREP_GL_W1
#define CF_PREP_GL_W1 4
#endif
#ifndef CF_PREP_CHUNKS_W1
#define CF_PREP_CHUNKS_W1 (64 / CF_PREP_GL_W1)
#endif
__host__ __device__ constexpr int prep_chunks(int pgl) { return pgl == kPrepGL ? kPrepChunks : CF_PREP_CHUNKS_W1; }
// row scan in 16-B loads (4 ids per lane per chunk): measured SLOWER at cfg2
// (same box, r03: draw alone 183 vs 119 us, 0.489 vs 0.399 ms/step;
// profiles/r03/ab_draw_vec_sortw.txt) -- the masked 4 x 8 compare per chunk
// and the misaligned 128-B spans cost more than the fewer load instructions
// save; 4-B loads stay the default
#ifndef CF_PREP_VEC
#define CF_PREP_VEC 0
#endif
#ifndef CF_PREP_VCHUNKS
#define CF_PREP_VCHUNKS 4 // 128-B row chunks in flight per group (512 ids)
#endif
constexpr int kPrepVChunks = CF_PREP_VCHUNKS;

// OR over the PGL lanes of a draw group.  A group of 4 or 8 lanes lies in
// one DPP row: quad_perm steps OR each quad, row_half_mirror the other quad
// of an 8-lane group (round 4; CF_DPP_DRAW 0: __shfl_xor)
#ifndef CF_DPP_DRAW
#define CF_DPP_DRAW 1
#endif
template <int PGL = kPrepGL>
__device__ __forceinline__ uint32_t gor8(uint32_t v) {
    if constexpr (CF_DPP_DRAW && (PGL == 4 || PGL == 8)) {
        v |= dpp_u<0xB1>(v);   // quad_perm [1,0,3,2]
        v |= dpp_u<0x4E>(v);   // quad_perm [2,3,0,1]
        if constexpr (PGL == 8) v |= dpp_u<0x141>(v);   // row_half_mirror
        return v;
    }
#pragma unroll
    for (int o = PGL / 2; o >= 1; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}
// lane k of the caller's PGL-lane group, broadcast (k compile-time after
// unrolling); a 4-lane group is a quad: quad_perm [k,k,k,k]
template <int PGL>
__device__ __forceinline__ int32_t gbcast(int32_t v, int k) {
    if constexpr (CF_DPP_DRAW && PGL == 4) {
        switch (k) {
            case 0: return (int32_t)dpp_u<0x00>((uint32_t)v);
            case 1: return (int32_t)dpp_u<0x55>((uint32_t)v);
            case 2: return (int32_t)dpp_u<0xAA>((uint32_t)v);
            default: return (int32_t)dpp_u<0xFF>((uint32_t)v);
        }
    }
    return __shfl(v, k, PGL);
}

constexpr unsigned long long kPosEmpty = ~0ull;

__device__ __forceinline__ uint64_t pos_slot(unsigned long long key, uint64_t mask) {
    return mix64(key) & mask;
}

// j in Pos(u)?  Expected ~1.5 probes at load factor <= 1/2, mostly in one
// 64-B sector (linear probing)
__device__ __forceinline__ bool is_positive(const StepArgs& a, int u, int32_t j) {
    const unsigned long long key = ((unsigned long long)(uint32_t)u << 32) | (uint32_t)j;
    uint64_t s = pos_slot(key, a.pos_mask);
    while (true) {
        const unsigned long long t = a.pos_set[s];
        if (t == key) return true;
        if (t == kPosEmpty) return false;
        s = (s + 1) & a.pos_mask;
    }
}

// Which of the group's candidates cand[0, ncand) lie in the user's sorted
// CSR row [rb, re) (bit c of the group-OR'ed result).  CF_PREP_VEC: lane gl
// reads 16 B (4 ids) of every 128-B chunk from the 16-B-aligned start at or
// before rb, kPrepVChunks chunks in flight -- a 51-id row is two load
// instructions instead of seven 4-B ones (the indices allocation is padded
// by 4 ids, so an int4 never leaves it); ids outside [rb, re) never match.
template <int PGL = kPrepGL>
__device__ __forceinline__ uint32_t row_hits(const int32_t* __restrict__ ind, int64_t rb, int64_t re, int gl,
                                             const int32_t (&cand)[PGL], int ncand) {
    constexpr int kPrepGL = PGL;                   // the group's lanes
    constexpr int kPrepChunks = prep_chunks(PGL);  // chunks in flight per lane
    uint32_t hit = 0;
#if CF_PREP_VEC
    constexpr int CW = 4 * kPrepGL;   // ids per chunk
    const int64_t a0 = rb & ~(int64_t)3;
    const int nch = (int)((re - a0 + CW - 1) / CW);
    for (int c0 = 0; c0 < nch; c0 += kPrepVChunks) {
        int4 el[kPrepVChunks];
#pragma unroll
        for (int q = 0; q < kPrepVChunks; ++q) {
            const int64_t t = a0 + (int64_t)(c0 + q) * CW + 4 * gl;
            el[q] = (t < re) ? *reinterpret_cast<const int4*>(ind + t) : make_int4(-1, -1, -1, -1);
        }
#pragma unroll
        for (int q = 0; q < kPrepVChunks; ++q) {
            const int64_t t = a0 + (int64_t)(c0 + q) * CW + 4 * gl;
            const int32_t e4[4] = {el[q].x, el[q].y, el[q].z, el[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool in = t + e >= rb && t + e < re;
#pragma unroll
                for (int c = 0; c < kPrepGL; ++c)
                    hit |= (in && c < ncand && e4[e] == cand[c]) ? (1u << c) : 0u;
            }
        }
    }
#else
    const int nchunk = (int)((re - rb + kPrepGL - 1) / kPrepGL);
    for (int c0 = 0; c0 < nchunk; c0 += kPrepChunks) {
        int32_t el[kPrepChunks];
#pragma unroll
        for (int q = 0; q < kPrepChunks; ++q) {
            const int64_t t = rb + (int64_t)(c0 + q) * kPrepGL + gl;
            el[q] = (t < re) ? ind[t] : -1;
        }
#pragma unroll
        for (int q = 0; q < kPrepChunks; ++q)
#pragma unroll
            for (int c = 0; c < kPrepGL; ++c)
                hit |= (c < ncand && el[q] == cand[c]) ? (1u << c) : 0u;
    }
#endif
    return hit;
}

template <int MODEL, int PGL = kPrepGL>
__device__ __forceinline__ void prep_body(const StepArgs& a, int block) {
    const int gl = threadIdx.x & (PGL - 1);
    const int p = block * (kBlock / PGL) + (threadIdx.x / PGL);
    if (p >= a.B) return;  // whole group leaves; no block barrier below
    const int W = a.W;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const int B = a.B;
    int u, i;
    uint64_t key = 0;
    int64_t rb = 0, re = 0;
    if (a.sample) {
        const uint64_t slot = a.slot_base + (uint64_t)p;
        // shuffled pair order (sampler_ranking.py:24); one 16-B record per pair
        // carries the user's CSR extent, so the row scan does not wait on a
        // dependent indptr load.  pre_pairs: the record the previous step's
        // gradient launch fetched (StepArgs::pf_out), read coalesced
#ifdef CF_EXP_DRAW_NOREC   // attribution only (wrong batches): no record load
        const int4 pr = make_int4((int)(slot % 1000000), (int)(slot % 100000), (int)((slot * 50) % 40000000), 50);
#else
        const int4 pr = a.pre_pairs != nullptr ? a.pre_pairs[p]
                      : a.order_recs != nullptr ? a.order_recs[slot]
                      : a.order != nullptr   ? a.pairs[a.order[slot]]
                                             : a.pairs[permute(slot, a.perm)];
#endif
        u = pr.x;
        i = pr.y;
        key = mix64(a.rng_key ^ (slot * 0xD1B54A32D192ED03ull));
        rb = (int64_t)(uint32_t)pr.z;
        re = rb + pr.w;
    } else {
        u = a.occU[p];
        i = a.occV[p];
    }
    // sorted batches without group users (StepArgs::user_runs, cf_set_option
    // "user_runs", default 0): the batch is in CSR order, so each user's
    // occurrences are one run of consecutive pairs.  rank = the pair's place
    // in its run, count = the run's length, added by the run's first pair with
    // a non-returning atomic; the wave's first and last runs may continue in
    // the neighbouring waves and add their in-wave length with one returning
    // atomic, the base of their ranks -- two returning atomics per wave
    // instead of one per pair (the neighbours' users come from the adjacent
    // groups by shuffle).  Measured EVEN at cfg2 (apply + draw 139.3 vs 140.2
    // us same box, profiles/r06/r06e): the returning user atomics are not what
    // bounds the draw.  Storing the interior runs' counts with plain stores
    // instead made the fused apply + draw launch 58 us SLOWER (198 vs 140 us;
    // the draw alone only +3 us, pipeline 0), and loading the wave's edge
    // records to settle those runs too +23 us.  Kept as an option for that record.
    const bool runs = a.user_runs != 0 && a.sample && a.count_users;   // wave-uniform
    int run_rank = 0, run_len = 0, run_lead = 0, run_base = 0;
    bool run_atomic = false;
    if (runs) {
        constexpr int GPW = kWave / PGL;
        const int lane = threadIdx.x & 63, lead = lane & ~(PGL - 1), g = lane / PGL;
        const int uprev = __shfl_up(u, PGL, kWave), unext = __shfl_down(u, PGL, kWave);
        const bool head = g == 0 || uprev != u;
        const bool tail = g == GPW - 1 || p + 1 >= B || unext != u;
        const uint64_t H = __ballot(gl == 0 && head), T = __ballot(gl == 0 && tail);
        const uint64_t hm = H & ((2ull << lead) - 1ull);    // heads at or before this pair (group 0's at least)
        const uint64_t tm = T & ~((1ull << lead) - 1ull);   // tails at or after it (the last active group's at least)
        run_lead = 63 - __clzll((long long)hm);
        const int last = __ffsll((unsigned long long)tm) - 1;
        run_rank = (lead - run_lead) / PGL;
        run_len = (last - run_lead) / PGL + 1;
        run_atomic = run_lead == 0 || last == (GPW - 1) * PGL;
    }
    // the user's and the positive's returning count atomics need only the
    // record: issued first, they are in flight during the row scan (their
    // ranks are stored at the end).  pos_sort: the positive's rank among the
    // batch's positives of i (the negatives count in cntV), psort's key
    int rk_u = 0, rk_i = 0;
#ifdef CF_EXP_DRAW_NOATOM   // attribution only (wrong ranks): no count atomics
    if (false) {
#else
    if (gl == 0) {
#endif
        if (runs) {
            if (run_rank == 0) {   // the run's first pair in this wave
                if (run_atomic) run_base = atomicAdd(&a.cntU[u], run_len);
                else (void)atomicAdd(&a.cntU[u], run_len);   // (a plain store: 58 us slower, above)
            }
        } else if (a.count_users) {
            rk_u = atomicAdd(&a.cntU[u], 1);
        }
        if (a.count_items) rk_i = atomicAdd(a.cntP != nullptr ? &a.cntP[i] : &a.cntV[i], 1);
    }
    const bool spec = a.sample && a.spec_n != nullptr && a.count_items && a.pos_set == nullptr;
    for (int w0 = 0; w0 < W; w0 += PGL) {
        const int nw = (W - w0 < PGL) ? (W - w0) : PGL;
        const int w = w0 + gl;
        int32_t j = -1;
        if (a.sample && a.pos_set != nullptr) {
            // negItems = randint(0, n_items), redrawn while j in Pos(u)
            // (sampler_ranking.py:30-36): negative w takes the first attempt
            // k = 0, 1, .. of draw(key, (w << 32) + k) outside Pos(u) -- the
            // same sequence as the row scan below, one set probe per attempt
            if (gl < nw) {
                uint64_t ctr = (uint64_t)w << 32;
                j = draw_item(key, ctr++, a.n_items);
                while (is_positive(a, u, j)) j = draw_item(key, ctr++, a.n_items);
                a.occV[B + p * W + w] = j;
            }
        } else if (a.sample) {
            // negItems = randint(0, n_items), redrawn while j in Pos(u)
            // (sampler_ranking.py:30-36).  Negative w takes the first
            // candidate of the sequence draw(key, (w << 32) + k), k = 0, 1, ..
            // that is not a positive.  The first C = 8 / nw candidates of every
            // negative are tested in ONE row scan (lane l holds attempt l / nw
            // of negative l % nw), so a rejection rarely costs another pass.
            const int C = PGL / nw;
            const int nl = C * nw;
            int32_t jl = -1;
            if (gl < nl) jl = draw_item(key, ((uint64_t)(w0 + gl % nw) << 32) + (uint64_t)(gl / nw), a.n_items);
            // speculative count of attempt 0 (lane w - w0 < nw holds it), in
            // flight during the scan (StepArgs::spec_ph)
            int rk_s = 0;
#ifndef CF_EXP_DRAW_NOATOM
            if (spec && gl < nw) rk_s = atomicAdd(&a.cntV[jl], 1);
#endif
            uint32_t hit = 0;
            {
                int32_t cand[PGL];
#pragma unroll
                for (int k = 0; k < PGL; ++k) cand[k] = gbcast<PGL>(jl, k);
#ifndef CF_EXP_DRAW_NOSCAN   // attribution only (wrong batches): no row scan
                hit = gor8<PGL>(row_hits<PGL>(a.indices, rb, re, gl, cand, nl));
#endif
            }
            // lane w < nw: the first accepted attempt of negative w
            // (the winning lane found from the group-uniform hit mask first:
            // one shuffle instead of one per attempt)
            int win = -1;
            for (int c = 0; c < C; ++c) {
                const int src = c * nw + (gl % nw);
                if (win < 0 && !((hit >> src) & 1u)) win = src;
            }
            const int32_t cv = __shfl(jl, win < 0 ? 0 : win, PGL);
            const bool done = win >= 0;
            if (done && gl < nw) j = cv;
            // rare: every tested attempt of some negative was a positive ->
            // continue its sequence at attempt C, one candidate per lane
            uint32_t pending = gor8<PGL>((gl < nw && !done) ? (1u << gl) : 0u);
            uint64_t ctr = ((uint64_t)w << 32) + (uint64_t)C;
            if ((pending >> gl) & 1u) j = draw_item(key, ctr++, a.n_items);
            while (pending != 0u) {  // group-uniform
                int32_t cand[PGL];
#pragma unroll
                for (int k = 0; k < PGL; ++k) cand[k] = gbcast<PGL>(j, k);
                uint32_t h2 = gor8<PGL>(row_hits<PGL>(a.indices, rb, re, gl, cand, nw)) & pending;
                if ((h2 >> gl) & 1u) j = draw_item(key, ctr++, a.n_items);
                pending = h2;
            }
            if (gl < nw) {
                a.occV[B + p * W + w] = j;
                if (spec) {
                    if (j != jl) {   // attempt 0 was a positive: a phantom, then the real count
                        a.spec_ph[atomicAdd(a.spec_n, 1)] = make_int2(jl, rk_s);
                        rk_s = atomicAdd(&a.cntV[j], 1);
                    }
                    a.rankV[B + p * W + w] = rk_s;
                }
            }
            if (spec) continue;   // counted above
        } else if (gl < nw) {
            j = a.occV[B + p * W + w];
        }
        if (a.count_items && gl < nw) a.rankV[B + p * W + w] = atomicAdd(&a.cntV[j], 1);
    }
    if (MODEL == GBPR) {
        for (int k = gl; k < G; k += PGL) {
            int32_t g;
            if (a.sample) {
                // group = np.random.choice(item_posUserList[i], gsize): uniform,
                // with replacement, may contain u (sampler_gbpr.py:41)
                const int64_t cb = a.indptr_t[i], ce = a.indptr_t[i + 1];
                const uint64_t h = mix64(key + ((uint64_t)(kMaxNeg + k) << 32));
                g = a.indices_t[cb + (int64_t)uniform_below(h, (uint64_t)(ce - cb))];
                // user-sharded engine: the item's users are global ids; one
                // owned by another rank is coded -1 - id (fetched by the group exchange)
                g = (g >= a.shard_u0 && g < a.shard_u1) ? g - a.shard_u0 : -1 - g;
                a.occU[B + p * G + k] = g;
            } else {
                g = a.occU[B + p * G + k];
            }
            if (a.count_users && g >= 0) a.rankU[B + p * G + k] = atomicAdd(&a.cntU[g], 1);
        }
    }
    if (runs) rk_u = __shfl(run_base, run_lead, kWave) + run_rank;   // every lane: the run's base
    if (gl == 0) {
        if (a.sample) {
            a.occU[p] = u;
            a.occV[p] = i;
        }
        if (a.count_users) a.rankU[p] = rk_u;
        if (a.count_items) a.rankV[p] = rk_i;
    }
}

// ---------------------------------------------------------------------------
// prep, one lane per pair (neg_check = 2): with the Pos(u) set a pair needs no
// cooperative row scan, so a wave draws 64 pairs at once -- 8x the pairs of
// the 8-lane groups per wave generation -- and every negative's probes are in
// flight together.  Same draw sequence as prep_body (negative w takes the
// first attempt k = 0, 1, .. of draw(key, (w << 32) + k) outside Pos(u)), so
// the same batches.  Measured SLOWER than the 8-lane groups at every bench
// config (cfg2 draw 135 vs 118 us, apply + draw 266 vs 232 us; cfg4 apply +
// draw 100 vs 67 us): 64 scattered probes and returning count atomics per
// wave instruction serialise in the address path, and 8-lane groups keep
// more waves -- more independent chains -- in flight.  Kept as an option.
// ---------------------------------------------------------------------------
// Built only with -DCF_LANE_DRAW (its registers would otherwise count against
// every launch that carries a draw branch)
#ifndef CF_LANE_DRAW
#define CF_LANE_DRAW 0
#endif
__host__ __device__ __forceinline__ bool lane_prep(const StepArgs& a) {
    return CF_LANE_DRAW && a.lane_draw != 0 && (!a.sample || a.pos_set != nullptr);
}

template <int MODEL, int WT>
__device__ __forceinline__ void prep_lane_body(const StepArgs& a, int block) {
    const int p = block * kBlock + (int)threadIdx.x;
    if (p >= a.B) return;  // no block barrier below
    constexpr int NJ = WT > 0 ? WT : 1;
    const int W = WT > 0 ? WT : a.W;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const int B = a.B;
    int u, i;
    uint64_t key = 0;
    if (a.sample) {
        const uint64_t slot = a.slot_base + (uint64_t)p;
        const int4 pr = a.order_recs != nullptr ? a.order_recs[slot]
                      : a.order != nullptr ? a.pairs[a.order[slot]]
                                           : a.pairs[permute(slot, a.perm)];   // sampler_ranking.py:24
        u = pr.x;
        i = pr.y;
        key = mix64(a.rng_key ^ (slot * 0xD1B54A32D192ED03ull));
    } else {
        u = a.occU[p];
        i = a.occV[p];
    }
    int64_t cb = 0, ce = 0;   // GBPR: the item's user column, fetched beside the probes
    if (MODEL == GBPR && a.sample) {
        cb = a.indptr_t[i];
        ce = a.indptr_t[i + 1];
    }
    for (int w0 = 0; w0 < W; w0 += NJ) {
        int32_t j[NJ];
        if (a.sample) {
            // negItems = randint(0, n_items), redrawn while j in Pos(u)
            // (sampler_ranking.py:30-36), every negative's probe chain at once
            uint64_t ctr[NJ], s[NJ];
            unsigned long long kk[NJ];
            uint32_t pend = 0;
#pragma unroll
            for (int q = 0; q < NJ; ++q) {
                ctr[q] = (uint64_t)(w0 + q) << 32;
                j[q] = draw_item(key, ctr[q]++, a.n_items);
                kk[q] = ((unsigned long long)(uint32_t)u << 32) | (uint32_t)j[q];
                s[q] = pos_slot(kk[q], a.pos_mask);
                pend |= (w0 + q < W) ? (1u << q) : 0u;
            }
            while (pend) {
                unsigned long long t[NJ];
#pragma unroll
                for (int q = 0; q < NJ; ++q) t[q] = ((pend >> q) & 1u) ? a.pos_set[s[q]] : kPosEmpty;
#pragma unroll
                for (int q = 0; q < NJ; ++q) {
                    if (!((pend >> q) & 1u)) continue;
                    if (t[q] == kk[q]) {            // a positive: the next attempt
                        j[q] = draw_item(key, ctr[q]++, a.n_items);
                        kk[q] = ((unsigned long long)(uint32_t)u << 32) | (uint32_t)j[q];
                        s[q] = pos_slot(kk[q], a.pos_mask);
                    } else if (t[q] == kPosEmpty) { // not in Pos(u): accepted
                        pend &= ~(1u << q);
                    } else {                        // another key: probe on
                        s[q] = (s[q] + 1) & a.pos_mask;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NJ; ++q)
                if (w0 + q < W) a.occV[B + (int64_t)p * W + w0 + q] = j[q];
        } else {
#pragma unroll
            for (int q = 0; q < NJ; ++q)
                if (w0 + q < W) j[q] = a.occV[B + (int64_t)p * W + w0 + q];
        }
        if (a.count_items) {
#pragma unroll
            for (int q = 0; q < NJ; ++q)
                if (w0 + q < W) a.rankV[B + (int64_t)p * W + w0 + q] = atomicAdd(&a.cntV[j[q]], 1);
        }
    }
    if (MODEL == GBPR) {
        for (int k = 0; k < G; ++k) {
            int32_t g;
            if (a.sample) {
                // group = np.random.choice(item_posUserList[i], gsize) (sampler_gbpr.py:41)
                const uint64_t h = mix64(key + ((uint64_t)(kMaxNeg + k) << 32));
                g = a.indices_t[cb + (int64_t)uniform_below(h, (uint64_t)(ce - cb))];
                g = (g >= a.shard_u0 && g < a.shard_u1) ? g - a.shard_u0 : -1 - g;
                a.occU[B + (int64_t)p * G + k] = g;
            } else {
                g = a.occU[B + (int64_t)p * G + k];
            }
            if (a.count_users && g >= 0) a.rankU[B + (int64_t)p * G + k] = atomicAdd(&a.cntU[g], 1);
        }
    }
    if (a.sample) {
        a.occU[p] = u;
        a.occV[p] = i;
    }
    if (a.count_users) a.rankU[p] = atomicAdd(&a.cntU[u], 1);
    if (a.count_items) a.rankV[p] = atomicAdd(&a.cntV[i], 1);
}

// ---------------------------------------------------------------------------
// the device draw with NP pairs per 8-lane group (CF_PREP_PAIRS): the draw is
// latency-bound (pair record -> row scan -> returning count atomics), so a
// group carries NP pairs' chains at once -- both pairs' records, then both
// row scans' chunks, then both pairs' atomics in flight together.  Same
// candidates, acceptance rule and counts as prep_body (the same batches).
// Device sampler with the CSR row scan and W <= the group width only;
// everything else takes prep_body.  Measured SLOWER at cfg2 (same box, r03:
// draw alone 130 vs 120 us, apply + draw 199 vs 190 us, step 0.408 vs 0.3995
// ms; profiles/r03/ab_draw_pairs.txt): the draw is not short of chains in
// flight per wave -- its returning count atomics and the row-scan requests
// bound it -- so one pair per group stays the default; -DCF_PREP_PAIRS=2
// builds the variant.
// ---------------------------------------------------------------------------
#ifndef CF_PREP_PAIRS
#define CF_PREP_PAIRS 1
#endif
constexpr int kPrepPairs = CF_PREP_PAIRS;

__host__ __device__ __forceinline__ bool multi_prep(const StepArgs& a) {
    return kPrepPairs > 1 && a.sample && a.pos_set == nullptr && a.W <= kPrepGL && !lane_prep(a);
}

template <int MODEL>
__device__ __forceinline__ void prep_body_np(const StepArgs& a, int block) {
    constexpr int PGL = kPrepGL, NP = kPrepPairs;
    const int gl = threadIdx.x & (PGL - 1);
    const int grp = threadIdx.x / PGL;
    const int W = a.W, B = a.B;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const int nw = W, C = PGL / nw, nl = C * nw;
    int p[NP], u[NP], i[NP], nchunk[NP];
    bool ok[NP];
    uint64_t key[NP];
    int64_t rb[NP], re[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        p[k] = (block * NP + k) * kPrepPairsPerBlock + grp;
        ok[k] = p[k] < B;   // group-uniform
    }
    if (!ok[0]) return;    // (p[k] grows with k) whole group leaves; no block barrier below
    // pair records (one 16-B load each, all in flight)
    int4 pr[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const uint64_t slot = a.slot_base + (uint64_t)p[k];
        key[k] = mix64(a.rng_key ^ (slot * 0xD1B54A32D192ED03ull));
        if (ok[k]) pr[k] = a.order_recs != nullptr ? a.order_recs[slot]
                         : a.order != nullptr ? a.pairs[a.order[slot]]
                                              : a.pairs[permute(slot, a.perm)];   // sampler_ranking.py:24
    }
    int maxchunk = 0;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        u[k] = ok[k] ? pr[k].x : 0;
        i[k] = ok[k] ? pr[k].y : 0;
        rb[k] = ok[k] ? (int64_t)(uint32_t)pr[k].z : 0;
        re[k] = ok[k] ? rb[k] + pr[k].w : 0;
        nchunk[k] = (int)((re[k] - rb[k] + PGL - 1) / PGL);
        maxchunk = nchunk[k] > maxchunk ? nchunk[k] : maxchunk;
    }
    // negItems = randint(0, n_items), redrawn while j in Pos(u)
    // (sampler_ranking.py:30-36): lane l holds attempt l / nw of negative
    // l % nw; every pair's first C attempts are tested in one row scan
    int32_t jl[NP];
    uint32_t hit[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        jl[k] = (gl < nl) ? draw_item(key[k], ((uint64_t)(gl % nw) << 32) + (uint64_t)(gl / nw), a.n_items) : -1;
        hit[k] = 0u;
    }
    {
        int32_t cand[NP][PGL];
#pragma unroll
        for (int k = 0; k < NP; ++k)
#pragma unroll
            for (int c = 0; c < PGL; ++c) cand[k][c] = gbcast<PGL>(jl[k], c);
        for (int c0 = 0; c0 < maxchunk; c0 += kPrepChunks) {
            int32_t el[NP][kPrepChunks];
#pragma unroll
            for (int k = 0; k < NP; ++k)
#pragma unroll
                for (int q = 0; q < kPrepChunks; ++q) {
                    const int64_t t = rb[k] + (int64_t)(c0 + q) * PGL + gl;
                    el[k][q] = (t < re[k]) ? a.indices[t] : -1;
                }
#pragma unroll
            for (int k = 0; k < NP; ++k)
#pragma unroll
                for (int q = 0; q < kPrepChunks; ++q)
#pragma unroll
                    for (int c = 0; c < PGL; ++c)
                        hit[k] |= (c < nl && el[k][q] == cand[k][c]) ? (1u << c) : 0u;
        }
    }
    int32_t j[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        hit[k] = gor8(hit[k]);
        // lane w < nw: the first accepted attempt of negative w
        bool done = false;
        j[k] = -1;
        for (int c = 0; c < C; ++c) {
            const int src = c * nw + (gl % nw);
            const int32_t cv = __shfl(jl[k], src, PGL);
            if (!done && gl < nw && !((hit[k] >> src) & 1u)) {
                j[k] = cv;
                done = true;
            }
        }
        // rare: every tested attempt of some negative was a positive ->
        // continue its sequence at attempt C, one candidate per lane
        uint32_t pending = gor8((ok[k] && gl < nw && !done) ? (1u << gl) : 0u);
        uint64_t ctr = ((uint64_t)gl << 32) + (uint64_t)C;
        if ((pending >> gl) & 1u) j[k] = draw_item(key[k], ctr++, a.n_items);
        while (pending != 0u) {  // group-uniform
            int32_t cand[PGL];
#pragma unroll
            for (int c = 0; c < PGL; ++c) cand[c] = gbcast<PGL>(j[k], c);
            uint32_t h2 = 0;
            for (int c0 = 0; c0 < nchunk[k]; c0 += kPrepChunks) {
                int32_t el[kPrepChunks];
#pragma unroll
                for (int q = 0; q < kPrepChunks; ++q) {
                    const int64_t t = rb[k] + (int64_t)(c0 + q) * PGL + gl;
                    el[q] = (t < re[k]) ? a.indices[t] : -1;
                }
#pragma unroll
                for (int q = 0; q < kPrepChunks; ++q)
#pragma unroll
                    for (int c = 0; c < PGL; ++c)
                        h2 |= (c < nw && el[q] == cand[c]) ? (1u << c) : 0u;
            }
            h2 = gor8(h2) & pending;
            if ((h2 >> gl) & 1u) j[k] = draw_item(key[k], ctr++, a.n_items);
            pending = h2;
        }
    }
    // occurrences and their ranks (returning count atomics), every pair's at once
    int32_t rj[NP], ru[NP], ri[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        if (ok[k] && gl < nw) {
            a.occV[B + p[k] * W + gl] = j[k];
            if (a.count_items) rj[k] = atomicAdd(&a.cntV[j[k]], 1);
        }
        if (ok[k] && gl == 0) {
            a.occU[p[k]] = u[k];
            a.occV[p[k]] = i[k];
            if (a.count_users) ru[k] = atomicAdd(&a.cntU[u[k]], 1);
            // pos_sort: the positive's rank among the batch's positives of i
            if (a.count_items) ri[k] = atomicAdd(a.cntP != nullptr ? &a.cntP[i[k]] : &a.cntV[i[k]], 1);
        }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        if (ok[k] && gl < nw && a.count_items) a.rankV[B + p[k] * W + gl] = rj[k];
        if (ok[k] && gl == 0) {
            if (a.count_users) a.rankU[p[k]] = ru[k];
            if (a.count_items) a.rankV[p[k]] = ri[k];
        }
    }
    if (MODEL == GBPR) {
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            if (!ok[k]) continue;
            for (int q = gl; q < G; q += PGL) {
                // group = np.random.choice(item_posUserList[i], gsize) (sampler_gbpr.py:41)
                const int64_t cb = a.indptr_t[i[k]], ce = a.indptr_t[i[k] + 1];
                const uint64_t h = mix64(key[k] + ((uint64_t)(kMaxNeg + q) << 32));
                int32_t g = a.indices_t[cb + (int64_t)uniform_below(h, (uint64_t)(ce - cb))];
                g = (g >= a.shard_u0 && g < a.shard_u1) ? g - a.shard_u0 : -1 - g;
                a.occU[B + p[k] * G + q] = g;
                if (a.count_users && g >= 0) a.rankU[B + p[k] * G + q] = atomicAdd(&a.cntU[g], 1);
            }
        }
    }
}

// the draw + count of one block of a step's batch: one lane per pair when no
// row scan is needed (lane_prep), several pairs per 8-lane group on the
// device sampler's row scan (multi_prep), else prep_body
template <int MODEL>
__device__ __forceinline__ void prep_any(const StepArgs& a, int block) {
#if CF_LANE_DRAW
    if (lane_prep(a)) {
        if (a.W == 1) prep_lane_body<MODEL, 1>(a, block);
        else if (a.W == 5) prep_lane_body<MODEL, 5>(a, block);
        else prep_lane_body<MODEL, 0>(a, block);
        return;
    }
#endif
    if (multi_prep(a)) {
        prep_body_np<MODEL>(a, block);
        return;
    }
    if (a.W == 1)
        prep_body<MODEL, CF_PREP_GL_W1>(a, block);
    else
        prep_body<MODEL>(a, block);
}

__host__ __device__ __forceinline__ int prep_pairs_per_block(const StepArgs& a) {
    return lane_prep(a) ? kBlock : multi_prep(a) ? kPrepPairs * kPrepPairsPerBlock
                                 : a.W == 1 ? kBlock / CF_PREP_GL_W1 : kPrepPairsPerBlock;
}

template <int MODEL>
__global__ __launch_bounds__(kBlock) void prep_kernel(StepArgs a) {
    prep_any<MODEL>(a, blockIdx.x);
}

// ---------------------------------------------------------------------------
// grad: gather, loss, gradient rows, singleton apply / duplicate scatter
// ---------------------------------------------------------------------------
// Negative-item rows of one pair.  With a compile-time W (WT > 0) every index,
// count and row is fetched up front -- the whole pair's gather is in flight
// at once; WT == 0 is the generic runtime-W path that loads per negative.
template <int EPL, int WT>
struct NegRows {
    static constexpr int N = WT > 0 ? WT : 1;
    int j[N];
    int c[N];
    int64_t sl[N];  // slot row (or -1)
    float v[N][EPL];
    __device__ __forceinline__ void prefetch(const StepArgs& a, int p, int gl) {
        if constexpr (WT > 0) {
            int rk[N];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                j[w] = a.occV[a.B + p * WT + w];
                rk[w] = a.count_items ? a.rankV[a.B + p * WT + w] : 0;
            }
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                c[w] = a.count_items ? a.cntV[j[w]] : 0;
                sl[w] = slot_of(c[w], j[w], rk[w], a.capV, a.repV, a.offV);
                gload<EPL>(a.V, j[w], a.d, gl, v[w]);
            }
        }
    }
    // slot holding negative w (loads it first on the generic path)
    __device__ __forceinline__ int get(const StepArgs& a, int p, int w, int gl) {
        if constexpr (WT > 0) {
            return w;
        } else {
            j[0] = a.occV[a.B + p * a.W + w];
            const int rk = a.count_items ? a.rankV[a.B + p * a.W + w] : 0;
            c[0] = a.count_items ? a.cntV[j[0]] : 0;
            sl[0] = slot_of(c[0], j[0], rk, a.capV, a.repV, a.offV);
            gload<EPL>(a.V, j[0], a.d, gl, v[0]);
            return 0;
        }
    }
};

// AMF apr (cf_config.amf_mode 1): Δ of row r = epsilon * l2_normalize(the
// batch's summed embedding-loss gradient of r), tf.nn.l2_normalize(x, 1) =
// x * rsqrt(max(sum x^2, 1e-12)) (amf.py:131-137).  A row seen once takes the
// gradient of its own pair, g1, from registers; a duplicated row the sum that
// apr_embed_kernel left in Gadv.  dx may alias g1.
template <int EPL>
__device__ __forceinline__ void apr_delta(const float* __restrict__ Gadv, int64_t r, int count, int d, int gl,
                                          float eps, const float (&g1)[EPL], float (&dx)[EPL]) {
    if (count >= 2) {
        gload<EPL>(Gadv, r, d, gl, dx);
    } else {
#pragma unroll
        for (int s = 0; s < EPL; ++s) dx[s] = g1[s];
    }
    const float sc = eps * rsqrtf(fmaxf(gdot<EPL>(dx, dx), 1e-12f));
#pragma unroll
    for (int s = 0; s < EPL; ++s) dx[s] *= sc;
}

// One AMF apr pair of the adversarial phase (amf.py:92-116, 139-162 with the
// assigns of __update_adv__ run): loss softplus(-x) + reg_adv *
// softplus(-clip(x', -80, 1e8)) + reg * L2, x = <u,i> - <u,j>,
// x' = <u+Δu, i+Δi> - <u, j+Δj> (the user is not perturbed in uj,
// amf.py:110); Δ is a constant (stop_gradient, amf.py:131-132).  Pass 1 forms
// the pair's own embedding-loss gradients of u and i (the rows seen once take
// Δ from them), pass 2 the loss and the gradient rows.
template <int EPL, int WT>
__device__ __forceinline__ void apr_pair(const StepArgs& a, int p, int gl, int u, int i, int cu, int ci,
                                         int64_t su, int64_t si, const float (&uu)[EPL], const float (&vi)[EPL],
                                         NegRows<EPL, WT>& J, float& loss_g, float& sq) {
    const int d = a.d;
    const int W = WT > 0 ? WT : a.W;
    const float ui = gdot<EPL>(uu, vi);
    float g1[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) g1[s] = 0.f;
    float sc = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const int sl = J.get(a, p, w, gl);
        const float c = -rcp_1p(expf(ui - gdot<EPL>(uu, J.v[sl])));
        sc += c;
#pragma unroll
        for (int s = 0; s < EPL; ++s) g1[s] = fmaf(c, vi[s] - J.v[sl][s], g1[s]);
    }
    float up[EPL], ip[EPL];
    apr_delta<EPL>(a.GadvU, u, cu, d, gl, a.epsilon, g1, up);
#pragma unroll
    for (int s = 0; s < EPL; ++s) g1[s] = sc * uu[s];
    // multi-rank (apr_global): every item row's Δ from the all-reduced sum
    apr_delta<EPL>(a.GadvV, i, a.apr_global ? 2 : ci, d, gl, a.epsilon, g1, ip);
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        up[s] += uu[s];
        ip[s] += vi[s];
    }
    const float uiP = gdot<EPL>(up, ip);
    float gu[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) gu[s] = a.reg * uu[s];
    float scP = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const int sl = J.get(a, p, w, gl);
        const float x = ui - gdot<EPL>(uu, J.v[sl]);
        const float c = -rcp_1p(expf(x));
        loss_g += softplus(-x);
        float jp[EPL];
#pragma unroll
        for (int s = 0; s < EPL; ++s) jp[s] = -c * uu[s];
        apr_delta<EPL>(a.GadvV, J.j[sl], a.apr_global ? 2 : J.c[sl], d, gl, a.epsilon, jp, jp);
#pragma unroll
        for (int s = 0; s < EPL; ++s) jp[s] += J.v[sl][s];
        const float xP = uiP - gdot<EPL>(uu, jp);
        loss_g += a.reg_adv * softplus(-fmaxf(fminf(xP, 1e8f), -80.f));
        const float cP = (xP >= -80.f && xP <= 1e8f) ? a.reg_adv * -rcp_1p(expf(xP)) : 0.f;
        scP += cP;
        float gj[EPL];
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            gu[s] = fmaf(c, vi[s] - J.v[sl][s], gu[s]);
            gu[s] = fmaf(cP, ip[s] - jp[s], gu[s]);
            gj[s] = -(c + cP) * uu[s] + a.reg * J.v[sl][s];
            sq = fmaf(J.v[sl][s], J.v[sl][s], sq);
        }
        ifinish<EPL>(a, J.j[sl], J.c[sl], J.sl[sl], p, -(c + cP), a.reg, 0, gl, J.v[sl], gj);
    }
    float gi[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        gi[s] = fmaf(sc, uu[s], fmaf(scP, up[s], a.reg * vi[s]));
        sq = fmaf(uu[s], uu[s], sq);
        sq = fmaf(vi[s], vi[s], sq);
    }
    gfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, gu, a);
    ifinish<EPL>(a, i, ci, si, p, sc, a.reg, 0, gl, vi, gi);
}

template <int MODEL, int EPL, int WT>
__device__ __forceinline__ void grad_body(const StepArgs& a, int block) {
    __shared__ double s_loss[kGroupsPerBlock];
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    const int d = a.d;
    const int W = WT > 0 ? WT : a.W;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const int B = a.B;
    float loss_g = 0.f;  // group-uniform: embedding loss (+ GBPR bias L2)
    float sq = 0.f;      // lane-partial sum of squares for the L2 term

    for (int k = 0; k < kPairsPerGroup; ++k) {
        const int p = (block * kPairsPerGroup + k) * kGroupsPerBlock + grp;
        if (p >= B) break;  // group-uniform
        if (MODEL == GBPR && a.member_pass != 0) {   // split exchange step (group-uniform)
            bool local = true;
            for (int k2 = 0; k2 < G; ++k2) local &= a.occU[B + p * G + k2] >= 0;
            if (local != (a.member_pass == 1)) continue;
        }
        const int u = a.occU[p];
        const int i = a.occV[p];
        const int ru = a.count_users ? a.rankU[p] : 0;
        const int ri = a.count_items ? a.rankV[p] : 0;
        NegRows<EPL, WT> J;
        J.prefetch(a, p, gl);
        const int cu = a.count_users ? a.cntU[u] : 0;
        const int ci = a.count_items ? a.cntV[i] : 0;
        const int64_t su = slot_of(cu, u, ru, a.capU, 0, a.offU);
        const int64_t si = slot_of(ci, i, ri, a.capV, a.repV, a.offV);
        float uu[EPL], vi[EPL];
        gload<EPL>(a.U, u, d, gl, uu);
        gload<EPL>(a.V, i, d, gl, vi);
        if (a.recV != nullptr) gstore<EPL>(a.stashU, p, d, gl, uu);   // item records' X

        if (MODEL == BPR || MODEL == AMF) {
            // x = <u,i> - <u,j>;  c = dL/dx = sigmoid(x) - 1   (A.1, A.4)
            const float ui = gdot<EPL>(uu, vi);
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int sl = J.get(a, p, w, gl);
                const float x = ui - gdot<EPL>(uu, J.v[sl]);
                float c = -rcp_1p(expf(x));
                if (MODEL == AMF) {
                    loss_g += softplus(-x);
                    if (a.adversarial) {
                        // + reg_adv * softplus(-clip_by_value(x, -80, 1e8)), Δ == 0
                        const float xc = fmaxf(fminf(x, 1e8f), -80.f);
                        loss_g += a.reg_adv * softplus(-xc);
                        if (x >= -80.f && x <= 1e8f) c *= (1.f + a.reg_adv);
                    }
                } else {
                    loss_g += neg_log_sigmoid(x);
                }
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(c, vi[s] - J.v[sl][s], gu[s]);
                    gj[s] = -c * uu[s] + a.reg * J.v[sl][s];
                    sq = fmaf(J.v[sl][s], J.v[sl][s], sq);
                }
                ifinish<EPL>(a, J.j[sl], J.c[sl], J.sl[sl], p, -c, a.reg, 0, gl, J.v[sl], gj);
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += a.reg * uu[s];
                gi[s] = sc * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, gu, a);
            ifinish<EPL>(a, i, ci, si, p, sc, a.reg, 0, gl, vi, gi);
        } else if (MODEL == GBPR) {
            // ui = rho*mean_k<g_k,i> + (1-rho)<u,i> + b_i ; uj = <u,j> + b_j   (A.2)
            const float bi = a.b[i];
            const float ui_u = gdot<EPL>(uu, vi);
            float sg[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) sg[s] = 0.f;
            for (int k2 = 0; k2 < G; ++k2) {
                float gk[EPL];
                const int g = a.occU[B + p * G + k2];
                gload<EPL>(g >= 0 ? a.U : a.xrows, g >= 0 ? g : -1 - g, d, gl, gk);
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    sg[s] += gk[s];
                    sq = fmaf(gk[s], gk[s], sq);
                }
            }
            const float Gf = (float)G;
            const float ui = a.rho * (gdot<EPL>(sg, vi) / Gf) + (1.f - a.rho) * ui_u + bi;
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int sl = J.get(a, p, w, gl);
                const int j = J.j[sl];
                const float bj = a.b[j];
                const float x = ui - (gdot<EPL>(uu, J.v[sl]) + bj);
                const float c = -rcp_1p(expf(x));
                loss_g += neg_log_sigmoid(x) + 0.5f * a.reg * bj * bj;
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(-c, J.v[sl][s], gu[s]);
                    gj[s] = -c * uu[s];  // no L2 on V[j] (gbprmf.py:59-64)
                }
                if (gl == 0) bias_finish(a, j, J.c[sl], -c + a.reg * bj, J.sl[sl]);
                ifinish<EPL>(a, j, J.c[sl], J.sl[sl], p, -c, 0.f, 0, gl, J.v[sl], gj);
            }
            const float rg = a.rho / Gf;
            float gi[EPL], bl[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += (1.f - a.rho) * sc * vi[s] + a.reg * uu[s];
                bl[s] = rg * sg[s] + (1.f - a.rho) * uu[s];
                gi[s] = sc * bl[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            if (a.recV != nullptr) gstore<EPL>(a.stashB, p, d, gl, bl);
            gfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, gu, a);
            for (int k2 = 0; k2 < G; ++k2) {
                const int g = a.occU[B + p * G + k2];
                float gk[EPL], gg[EPL];
                gload<EPL>(g >= 0 ? a.U : a.xrows, g >= 0 ? g : -1 - g, d, gl, gk);
#pragma unroll
                for (int s = 0; s < EPL; ++s) gg[s] = rg * sc * vi[s] + a.reg * gk[s];
                if (g < 0) {  // another rank's user: its gradient row goes back to the owner
                    gstore<EPL>(a.xgrads, -1 - g, d, gl, gg);
                    continue;
                }
                const int cg = a.cntU[g];
                const int64_t sg_ = slot_of(cg, g, a.rankU[B + p * G + k2], a.capU, 0, a.offU);
                gfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, g, cg, sg_, d, gl, gk, gg, a);
            }
            if (gl == 0) bias_finish(a, i, ci, sc, si);
            ifinish<EPL>(a, i, ci, si, p, sc, a.reg, 1, gl, vi, gi);
        } else if (MODEL == PLR) {
            // tuple ranking: s_x = <u, v_x> + b_x over the tuple's items
            // (x0 = i, x1.. = J); weighted -log sigmoid(coef (s_a - s_b)) terms
            //   PRIGP (u,i,j,t,k): (i,j; 1; 1), (t,k; 1; alpha)       prigp.py:99-130
            //   CPLR (u,i,t,j) + (c0,c1): (i,t; (c0+1)/(c1+1); alpha),
            //        (t,j; c1+1; beta), (i,j; c0+1; gamma)           cplr_u.py:106-137
            constexpr int NX = WT + 1;
            float sx[NX], bx[NX], ds[NX];
            sx[0] = gdot<EPL>(uu, vi);
            bx[0] = a.b[i];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                sx[w + 1] = gdot<EPL>(uu, J.v[w]);
                bx[w + 1] = a.b[J.j[w]];
            }
#pragma unroll
            for (int x = 0; x < NX; ++x) {
                sx[x] += bx[x];
                ds[x] = 0.f;
                loss_g += 0.5f * a.reg * bx[x] * bx[x];
            }
            auto term = [&](int xa, int xb, float coef, float wt) {
                const float z = coef * (sx[xa] - sx[xb]);
                loss_g += wt * neg_log_sigmoid(z);
                const float g = wt * coef * (-rcp_1p(expf(z)));
                ds[xa] += g;
                ds[xb] -= g;
            };
            if (a.plr_kind == 0) {
                term(0, 1, 1.f, 1.f);
                if (NX > 3) term(2, 3 < NX ? 3 : 2, 1.f, a.alpha);
            } else {
                const float uij = a.coefs[2 * p] + 1.f, utj = a.coefs[2 * p + 1] + 1.f;
                term(0, 1, uij / utj, a.alpha);
                term(1, 2 < NX ? 2 : 1, utj, a.beta);
                term(0, 2 < NX ? 2 : 1, uij, a.gamma);
            }
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = a.reg * uu[s] + ds[0] * vi[s];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(ds[w + 1], J.v[w][s], gu[s]);
                    gj[s] = ds[w + 1] * uu[s] + a.reg * J.v[w][s];
                    sq = fmaf(J.v[w][s], J.v[w][s], sq);
                }
                if (a.train_bias && gl == 0) bias_finish(a, J.j[w], J.c[w], ds[w + 1] + a.reg * bx[w + 1], J.sl[w]);
                ifinish<EPL>(a, J.j[w], J.c[w], J.sl[w], p, ds[w + 1], a.reg, 0, gl, J.v[w], gj);
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gi[s] = ds[0] * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, gu, a);
            if (a.train_bias && gl == 0) bias_finish(a, i, ci, ds[0] + a.reg * bx[0], si);
            ifinish<EPL>(a, i, ci, si, p, ds[0], a.reg, 0, gl, vi, gi);
        } else {  // CML (A.3); W <= 16 so lane w keeps dn_w
            float du[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) du[s] = uu[s] - vi[s];
            const float dp = gdot<EPL>(du, du);
            float dn_lane = 0.f;
            float m = INFINITY;
            int imp = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int sl = J.get(a, p, w, gl);
                float t[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) t[s] = uu[s] - J.v[sl][s];
                const float dn = gdot<EPL>(t, t);
                if (gl == w) dn_lane = dn;
                m = fminf(m, dn);
                imp += (dp - dn + a.margin > 0.f) ? 1 : 0;
            }
            const unsigned long long tie = __ballot(gl < W && dn_lane == m);
            const float cnt = (float)__popcll((tie >> (threadIdx.x & 48)) & 0xFFFFull);
            const float z = dp - m + a.margin;
            const float lw =
                a.use_rank_weight ? logf((float)imp / (float)W * a.n_items_f + 1.f) : 1.f;
            loss_g += fmaxf(z, 0.f) * lw;
            const float aa = (z > 0.f) ? lw : 0.f;
            const bool l2 = a.reg_cov > 0.f;
            float gu[EPL], gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] = 2.f * aa * du[s];
                gi[s] = -2.f * aa * du[s];
            }
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const float dnw = __shfl(dn_lane, w, kGL);
                const float share = (dnw == m) ? 1.f / cnt : 0.f;
                const int sl = J.get(a, p, w, gl);  // generic path reloads the row
                float gj[EPL];
                const float coef = 2.f * aa * share;
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    const float dv = uu[s] - J.v[sl][s];
                    gu[s] = fmaf(-coef, dv, gu[s]);
                    gj[s] = coef * dv;
                    if (l2) {
                        gj[s] += a.reg_cov * J.v[sl][s];
                        sq = fmaf(J.v[sl][s], J.v[sl][s], sq);
                    }
                }
                // a touched row with a zero gradient is still clipped (cml.py:128-129)
                ifinish<EPL>(a, J.j[sl], J.c[sl], J.sl[sl], p, coef, (l2 ? a.reg_cov : 0.f) - coef, 0, gl,
                             J.v[sl], gj);
            }
            if (l2) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] += a.reg_cov * uu[s];
                    gi[s] += a.reg_cov * vi[s];
                    sq = fmaf(uu[s], uu[s], sq);
                    sq = fmaf(vi[s], vi[s], sq);
                }
            }
            gfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, gu, a);
            ifinish<EPL>(a, i, ci, si, p, -2.f * aa, 2.f * aa + (l2 ? a.reg_cov : 0.f), 0, gl, vi, gi);
        }
    }

    // ---- per-block pre-update loss partial (fixed summation order) --------------
    const float coef = (MODEL == CML) ? (a.reg_cov > 0.f ? a.reg_cov : 0.f) : a.reg;
    const float sq_g = gsum(sq);
    if (gl == 0) s_loss[grp] = (double)loss_g + 0.5 * (double)coef * (double)sq_g;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < kGroupsPerBlock; ++k) t += s_loss[k];
        a.loss_partial[block] = t;
    }
}

// Horizontal fusion on the device-sampler pipeline: the grid carries the ng
// gradient blocks of step s and the np draw + count blocks of step s+1
// (independent work: the other buffer set), spread evenly over the block ids
// so that the latency-bound draw fills the gaps of the gather.  np == 0 is the
// plain gradient launch.
__device__ __forceinline__ bool minor_block(int b, int nmajor, int nminor, int& idx) {
#ifdef CF_GRAD_PREP_TAIL  // experiment: the draw blocks after every gradient block
    if (b >= nmajor) {
        idx = b - nmajor;
        return true;
    }
    idx = b;
    return false;
#endif
    const int64_t tot = (int64_t)nmajor + nminor;
    const int lo = (int)(((int64_t)b * nminor) / tot);
    const int hi = (int)(((int64_t)(b + 1) * nminor) / tot);
    idx = (hi > lo) ? lo : b - lo;
    return hi > lo;
}

// The same with the minor blocks front-loaded (experiment, CF_APPLY_DRAW_SKEW):
// the number of minor blocks before block b is F(b) = nminor - floor(nminor
// (tot - b)^2 / tot^2), whose slope falls from 2 nminor / tot to 0, so the
// latency-bound draw starts first and the bandwidth-bound apply blocks form
// the tail.  Needs nminor <= nmajor (slope <= 1: at most one minor block per
// block id); otherwise the even spread.
// BACK: the mirror image, F(b) = floor(nminor b^2 / tot^2): the draw blocks
// thin at the start and dense at the end (the apply's bandwidth first).
template <bool BACK = false>
__device__ __forceinline__ bool minor_block_front(int b, int nmajor, int nminor, int& idx) {
    if (nminor > nmajor) return minor_block(b, nmajor, nminor, idx);
    const int64_t tot = (int64_t)nmajor + nminor;
    auto F = [&](int64_t x) {
        // x^2 nminor <= tot^3 < 2^63 for tot < 2^21
        if (BACK) return (x * x * (int64_t)nminor) / (tot * tot);
        const int64_t r = tot - x;
        return (int64_t)nminor - (r * r * (int64_t)nminor) / (tot * tot);
    };
    const int64_t lo = F(b), hi = F((int64_t)b + 1);
    idx = (int)((hi > lo) ? lo : (int64_t)b - lo);
    return hi > lo;
}

// DRAW: the launch also carries the draw blocks of the next step (pipeline
// 2); without it the draw's registers do not count against the gradient
template <int MODEL, int EPL, int WT, bool DRAW>
__global__ __launch_bounds__(kBlock) void grad_kernel(StepArgs a, StepArgs nx, int ng, int np) {
    int idx = blockIdx.x;
    if (DRAW && minor_block(blockIdx.x, ng, np, idx))
        prep_any<MODEL == GBPR ? GBPR : BPR>(nx, idx);
    else
        grad_body<MODEL, EPL, WT>(a, idx);
}

// ---------------------------------------------------------------------------
// grad, phased fast path (compile-time W, G <= 1, d <= 128).
//
// CDNA retires loads, stores and atomics through ONE in-order vmcnt counter:
// a load issued after a float atomic cannot be waited for before the atomic
// drains (~3k cycles under load).  So a group first issues EVERY load of its
// P pairs -- indices, then rows and occurrence counts, then the Adagrad
// accumulator rows of the rows that occur once -- and only then computes and
// issues the updates / atomics.  Same arithmetic as grad_kernel.
// ---------------------------------------------------------------------------
template <int EPL>
__device__ __forceinline__ void gload_acc(const float* __restrict__ A, int64_t r, int d, int gl,
                                          bool want, float (&acc)[EPL]) {
#pragma unroll
    for (int s = 0; s < EPL; ++s) acc[s] = 1.f;
#ifdef CF_EXP_NO_ACC
    want = false;
#endif
#ifdef CF_EXP_ACC_ALWAYS  // issue the accumulator rows with the table rows (no dependent phase)
    want = true;
#endif
    if (want) row_ld<EPL>(A + r * (int64_t)d, d, gl, 1.f, acc);
}

// SparseApplyAdagrad with the accumulator row already in registers
template <int EPL>
__device__ __forceinline__ void gapply_pre(float* __restrict__ X, float* __restrict__ A, int64_t r,
                                           int d, int gl, const float (&x0)[EPL],
                                           const float (&acc0)[EPL], const float (&g)[EPL],
                                           float lr, bool clip, float c) {
    float acc[EPL], x[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        acc[s] = fmaf(g[s], g[s], acc0[s]);
        x[s] = x0[s] - adagrad_delta(lr, g[s], acc[s]);
    }
    if (clip) {
        const float n = sqrtf(gdot<EPL>(x, x));
        const float den = fmaxf(n, c);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * c) / den;
    }
    row_st<EPL>(X + r * (int64_t)d, d, gl, x);
    row_st<EPL>(A + r * (int64_t)d, d, gl, acc);
}

template <int EPL>
__device__ __forceinline__ void gfinish_pre(float* __restrict__ X, float* __restrict__ A,
                                            float* __restrict__ G, float* __restrict__ S,
                                            int32_t* __restrict__ cnt,
                                            int64_t r, int count, int64_t slot, int d, int gl,
                                            const float (&x0)[EPL], const float (&acc0)[EPL],
                                            const float (&g)[EPL], const StepArgs& a) {
    // CF_EXP_* are bench-only attribution builds (wrong results by design)
    if (count == 1) {
        if (a.items_grad_only && X == a.V) {
            gstore<EPL>(G, r, d, gl, g);  // sole writer of the zeroed dense row
        } else {
#ifndef CF_EXP_NO_SINGLE
            gapply_pre<EPL>(X, A, r, d, gl, x0, acc0, g, a.lr, a.clip != 0, a.clip_norm);
#endif
        }
        if (gl == 0) cnt[r] = 0;
    } else if (slot >= 0) {
        gstore<EPL>(S, slot, d, gl, g);
    } else {
#ifndef CF_EXP_NO_ATOMIC
        if (a.GU64 != nullptr && X == a.U)   // deterministic pos_sort: a user past its slot cap
            fx_atomic<EPL>(a.GU64 + (int64_t)a.hotU[r] * d, d, gl, g, a.fx_bad);
        else
            gatomic<EPL>(acc_of(G, slot, a), r, d, gl, g);
#endif
        if (a.items_grad_only && a.capV == 0 && X == a.V && gl == 0) cnt[r] = 0;  // see gfinish
    }
}

// gfinish_pre with ifinish's item records (see there)
template <int EPL>
__device__ __forceinline__ void ifinish_pre(const StepArgs& a, int64_t r, int count, int64_t slot, int p,
                                            float alpha, float beta, int which, int gl,
                                            const float (&x0)[EPL], const float (&acc0)[EPL],
                                            const float (&g)[EPL]) {
    if (a.recV != nullptr && count >= 2 && slot >= 0) {
        if (gl == 0) a.recV[slot] = make_int4(p, __float_as_int(alpha), __float_as_int(beta), which);
        return;
    }
    gfinish_pre<EPL>(a.V, a.AV, a.GV, a.slotV, a.cntV, r, count, slot, a.d, gl, x0, acc0, g, a);
}

template <int MODEL, int EPL, int WT>
struct PairRows {
    static constexpr int NG = (MODEL == GBPR) ? 1 : 0;
    static constexpr int NGA = NG > 0 ? NG : 1;
    int p, u, i, cu, ci, ru, ri;
    int oi;   // pos_sort: offP[i], the item's first positive-sorted position
    int j[WT], cj[WT], rj[WT];
    int g[NGA], cg[NGA], rg[NGA];
    int64_t su, si, sj[WT], sg[NGA];  // slot rows (or -1)
    float uu[EPL], vi[EPL], au[EPL], ai[EPL];
    float vj[WT][EPL], aj[WT][EPL];
    float ug[NGA][EPL], ag[NGA][EPL];
    float bi, bj[WT];
    float abi, abj[WT];   // GBPR: bias accumulators of rows seen once

    // pos_sort: the pair at positive-sorted position pos, from its contiguous
    // record (coalesced across the wave's groups): ids and every occurrence's
    // resolved destination (psort_scatter), so no count loads follow
    __device__ __forceinline__ void load_idx_sorted(const StepArgs& a, int pos) {
        constexpr int RS = psort_stride(WT);
        const int4* r = reinterpret_cast<const int4*>(a.srec + (int64_t)pos * RS);
        int32_t v[RS];
#pragma unroll
        for (int k = 0; k < RS / 4; ++k) {
            const int4 q = r[k];
            v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
        }
        u = v[0];
        i = v[1];
        p = pos;   // (the pair index itself is not needed on this path)
        ri = 0;
        ru = 0;
        const int32_t su_code = v[2 + WT], pi = v[3 + WT];
        cu = su_code == kSlotApply ? 1 : 2;
        su = su_code >= 0 ? su_code : -1;
        ci = pi < 0 ? 1 : 2;
        oi = pi & 0x7FFFFFFF;
        si = -1;
#pragma unroll
        for (int w = 0; w < WT; ++w) {
            j[w] = v[2 + w];
            rj[w] = 0;
            const int32_t sc = v[4 + WT + w];
            cj[w] = sc == kSlotApply ? 1 : 2;
            sj[w] = sc >= 0 ? sc : -1;
        }
    }
    __device__ __forceinline__ void load_idx(const StepArgs& a, int pair) {
        p = pair;
        u = a.occU[p];
        i = a.occV[p];
        ru = a.count_users ? a.rankU[p] : 0;
        ri = a.count_items ? a.rankV[p] : 0;
#pragma unroll
        for (int w = 0; w < WT; ++w) {
            j[w] = a.occV[a.B + p * WT + w];
            rj[w] = a.count_items ? a.rankV[a.B + p * WT + w] : 0;
        }
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            g[k] = a.occU[a.B + p + k];
            rg[k] = a.count_users ? a.rankU[a.B + p + k] : 0;
        }
    }
    template <bool SORT = false>
    __device__ __forceinline__ void load_rows(const StepArgs& a, int gl) {
        if constexpr (SORT) {
            // destinations came with the record: the accumulator rows of the
            // rows seen once are issued with the table rows (one load phase)
            gload<EPL>(a.U, u, a.d, gl, uu);
            gload<EPL>(a.V, i, a.d, gl, vi);
#pragma unroll
            for (int w = 0; w < WT; ++w) gload<EPL>(a.V, j[w], a.d, gl, vj[w]);
            const bool item_acc = !a.items_grad_only;
            gload_acc<EPL>(a.AU, u, a.d, gl, cu == 1, au);
            gload_acc<EPL>(a.AV, i, a.d, gl, item_acc && ci == 1, ai);
#pragma unroll
            for (int w = 0; w < WT; ++w) gload_acc<EPL>(a.AV, j[w], a.d, gl, item_acc && cj[w] == 1, aj[w]);
            return;
        }
        cu = a.count_users ? a.cntU[u] : 0;
        ci = a.count_items ? a.cntV[i] : 0;
#pragma unroll
        for (int w = 0; w < WT; ++w) cj[w] = a.count_items ? a.cntV[j[w]] : 0;
#pragma unroll
        for (int k = 0; k < NG; ++k) cg[k] = (a.count_users && g[k] >= 0) ? a.cntU[g[k]] : 0;
        gload<EPL>(a.U, u, a.d, gl, uu);
        gload<EPL>(a.V, i, a.d, gl, vi);
#pragma unroll
        for (int w = 0; w < WT; ++w) gload<EPL>(a.V, j[w], a.d, gl, vj[w]);
#pragma unroll
        for (int k = 0; k < NG; ++k)
            gload<EPL>(g[k] >= 0 ? a.U : a.xrows, g[k] >= 0 ? g[k] : -1 - g[k], a.d, gl, ug[k]);
        if (MODEL == GBPR) {
            bi = a.b[i];
#pragma unroll
            for (int w = 0; w < WT; ++w) bj[w] = a.b[j[w]];
        }
    }
    template <bool SORT = false>
    __device__ __forceinline__ void load_acc(const StepArgs& a, int gl) {
        if constexpr (SORT) return;   // loaded with the rows (load_rows)
        su = slot_of(cu, u, ru, a.capU, 0, a.offU);
        si = slot_of(ci, i, ri, a.capV, a.repV, a.offV);
#pragma unroll
        for (int w = 0; w < WT; ++w) sj[w] = slot_of(cj[w], j[w], rj[w], a.capV, a.repV, a.offV);
#pragma unroll
        for (int k = 0; k < NG; ++k) sg[k] = slot_of(cg[k], g[k], rg[k], a.capU, 0, a.offU);
        gload_acc<EPL>(a.AU, u, a.d, gl, cu == 1, au);
        const bool item_acc = !a.items_grad_only;
        gload_acc<EPL>(a.AV, i, a.d, gl, item_acc && ci == 1, ai);
#pragma unroll
        for (int w = 0; w < WT; ++w) gload_acc<EPL>(a.AV, j[w], a.d, gl, item_acc && cj[w] == 1, aj[w]);
#pragma unroll
        for (int k = 0; k < NG; ++k) gload_acc<EPL>(a.AU, g[k], a.d, gl, cg[k] == 1, ag[k]);
        if (MODEL == GBPR) {
            abi = (item_acc && ci == 1) ? a.Ab[i] : 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) abj[w] = (item_acc && cj[w] == 1) ? a.Ab[j[w]] : 0.f;
        }
    }

    // SORT: the positive item's gradient row goes to the group's LDS row
    // srow (summed over the block's run of pairs sharing the item by
    // psort_head) instead of being finished here
    template <bool SORT = false>
    __device__ __forceinline__ void update(const StepArgs& a, int gl, float& loss_g, float& sq,
                                           float* srow = nullptr) {
        const int d = a.d;
        if (a.recV != nullptr) {   // item records' X: only pairs that leave one
            bool need = MODEL != GBPR && ci >= 2 && si >= 0;
#pragma unroll
            for (int w = 0; w < WT; ++w) need |= cj[w] >= 2 && sj[w] >= 0;
            if (need) gstore<EPL>(a.stashU, p, d, gl, uu);
        }
        if (MODEL == BPR || MODEL == AMF) {
            const float ui = gdot<EPL>(uu, vi);
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                const float x = ui - gdot<EPL>(uu, vj[w]);
                float c = -rcp_1p(expf(x));
                if (MODEL == AMF) {
                    loss_g += softplus(-x);
                    if (a.adversarial) {
                        const float xc = fmaxf(fminf(x, 1e8f), -80.f);
                        loss_g += a.reg_adv * softplus(-xc);
                        if (x >= -80.f && x <= 1e8f) c *= (1.f + a.reg_adv);
                    }
                } else {
                    loss_g += neg_log_sigmoid(x);
                }
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(c, vi[s] - vj[w][s], gu[s]);
                    gj[s] = -c * uu[s] + a.reg * vj[w][s];
                    sq = fmaf(vj[w][s], vj[w][s], sq);
                }
                ifinish_pre<EPL>(a, j[w], cj[w], sj[w], p, -c, a.reg, 0, gl, vj[w], aj[w], gj);
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += a.reg * uu[s];
                gi[s] = sc * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, au, gu, a);
            if constexpr (SORT) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) srow[s * kGL + gl] = gi[s];
            } else {
                ifinish_pre<EPL>(a, i, ci, si, p, sc, a.reg, 0, gl, vi, ai, gi);
            }
        } else if (MODEL == GBPR) {  // G == 1
            const float ui_u = gdot<EPL>(uu, vi);
#pragma unroll
            for (int s = 0; s < EPL; ++s) sq = fmaf(ug[0][s], ug[0][s], sq);
            const float ui = a.rho * gdot<EPL>(ug[0], vi) + (1.f - a.rho) * ui_u + bi;
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                const float x = ui - (gdot<EPL>(uu, vj[w]) + bj[w]);
                const float c = -rcp_1p(expf(x));
                loss_g += neg_log_sigmoid(x) + 0.5f * a.reg * bj[w] * bj[w];
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(-c, vj[w][s], gu[s]);
                    gj[s] = -c * uu[s];
                }
                if (gl == 0) bias_finish_pre(a, j[w], cj[w], -c + a.reg * bj[w], sj[w], bj[w], abj[w]);
                ifinish_pre<EPL>(a, j[w], cj[w], sj[w], p, -c, 0.f, 0, gl, vj[w], aj[w], gj);
            }
            const float rg = a.rho;  // rho / G with G == 1
            float gi[EPL], gg[EPL], bl[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += (1.f - a.rho) * sc * vi[s] + a.reg * uu[s];
                bl[s] = rg * ug[0][s] + (1.f - a.rho) * uu[s];
                gi[s] = sc * bl[s] + a.reg * vi[s];
                gg[s] = rg * sc * vi[s] + a.reg * ug[0][s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, au, gu, a);
            if (g[0] >= 0)
                gfinish_pre<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, g[0], cg[0], sg[0], d, gl, ug[0], ag[0], gg, a);
            else  // another rank's user: its gradient row goes back to the owner
                gstore<EPL>(a.xgrads, -1 - g[0], d, gl, gg);
            if (gl == 0) bias_finish_pre(a, i, ci, sc, si, bi, abi);
            if (a.recV != nullptr && ci >= 2 && si >= 0) gstore<EPL>(a.stashB, p, d, gl, bl);
            ifinish_pre<EPL>(a, i, ci, si, p, sc, a.reg, 1, gl, vi, ai, gi);
        } else {  // CML
            float du[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) du[s] = uu[s] - vi[s];
            const float dp = gdot<EPL>(du, du);
            float dn[WT];
            float m = INFINITY;
            int imp = 0;
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                float t[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) t[s] = uu[s] - vj[w][s];
                dn[w] = gdot<EPL>(t, t);
                m = fminf(m, dn[w]);
                imp += (dp - dn[w] + a.margin > 0.f) ? 1 : 0;
            }
            float cnt = 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) cnt += (dn[w] == m) ? 1.f : 0.f;
            const float z = dp - m + a.margin;
            const float lw =
                a.use_rank_weight ? logf((float)imp / (float)WT * a.n_items_f + 1.f) : 1.f;
            loss_g += fmaxf(z, 0.f) * lw;
            const float aa = (z > 0.f) ? lw : 0.f;
            const bool l2 = a.reg_cov > 0.f;
            float gu[EPL], gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] = 2.f * aa * du[s];
                gi[s] = -2.f * aa * du[s];
            }
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                const float share = (dn[w] == m) ? 1.f / cnt : 0.f;
                const float coef = 2.f * aa * share;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    const float dv = uu[s] - vj[w][s];
                    gu[s] = fmaf(-coef, dv, gu[s]);
                    gj[s] = coef * dv;
                    if (l2) {
                        gj[s] += a.reg_cov * vj[w][s];
                        sq = fmaf(vj[w][s], vj[w][s], sq);
                    }
                }
                ifinish_pre<EPL>(a, j[w], cj[w], sj[w], p, coef, (l2 ? a.reg_cov : 0.f) - coef, 0, gl,
                                 vj[w], aj[w], gj);
            }
            if (l2) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] += a.reg_cov * uu[s];
                    gi[s] += a.reg_cov * vi[s];
                    sq = fmaf(uu[s], uu[s], sq);
                    sq = fmaf(vi[s], vi[s], sq);
                }
            }
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, uu, au, gu, a);
            if constexpr (SORT) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) srow[s * kGL + gl] = gi[s];
            } else {
                ifinish_pre<EPL>(a, i, ci, si, p, -2.f * aa, 2.f * aa + (l2 ? a.reg_cov : 0.f), 0, gl, vi, ai, gi);
            }
        }
    }
};

// pos_sort: the first group of a run of the block's pairs that share the
// positive item i sums the run's gradient rows (LDS, in position order) and
// finishes the item once for the whole run: Adagrad now if the run is the
// item's only occurrence in the batch, else the block's partial row ->
// slotP[block + i] (StepArgs: item i's partials are contiguous, block order)
// or, past capP, float atomics
template <int MODEL, int EPL, int WT, int GPB, bool FX>
__device__ __forceinline__ void psort_head(const StepArgs& a, const PairRows<MODEL, EPL, WT>& r, int block,
                                           int grp, int gl, const float (*s_gi)[kGL * EPL],
                                           const int* s_item) {
    const int k = block - r.oi / kPsortPPB;   // the item's k-th partial
    if (FX && r.ci != 1) {   // deterministic: the block's partial as an exact fixed-point sum
        long long t[EPL];
#pragma unroll
        for (int s = 0; s < EPL; ++s) t[s] = to_fx(s_gi[grp][s * kGL + gl], a.fx_bad);
        for (int q = grp + 1; q < GPB && s_item[q] == r.i; ++q) {
#pragma unroll
            for (int s = 0; s < EPL; ++s) t[s] += to_fx(s_gi[q][s * kGL + gl], a.fx_bad);
        }
        if (k < a.capP) {
            fx_st<EPL>(a.slotP64 + ((int64_t)block + r.i) * a.d, a.d, gl, t);
        } else {   // past capP: int64 atomics, exact in any order
            unsigned long long* row = a.GV64 + (int64_t)r.i * a.d;
            const bool full = vec_rows<EPL>() && a.d == kGL * EPL;
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                const int e = elem_of<EPL>(s, gl, full);
                if (e < a.d) atomicAdd(row + e, (unsigned long long)t[s]);
            }
        }
        return;
    }
    float g[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) g[s] = s_gi[grp][s * kGL + gl];
    for (int q = grp + 1; q < GPB && s_item[q] == r.i; ++q) {
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] += s_gi[q][s * kGL + gl];
    }
    if (r.ci == 1) {
        if (a.items_grad_only)   // multi-rank item reduce: the sole writer of the zeroed dense row
            gstore<EPL>(a.GV, r.i, a.d, gl, g);
        else
            gapply_pre<EPL>(a.V, a.AV, r.i, a.d, gl, r.vi, r.ai, g, a.lr, a.clip != 0, a.clip_norm);
        if (gl == 0) a.cntP[r.i] = 0;
    } else {
        if (k < a.capP)
            gstore<EPL>(a.slotP, (int64_t)block + r.i, a.d, gl, g);
        else
            gatomic<EPL>(a.GV, r.i, a.d, gl, g);
    }
}

template <int MODEL, int EPL, int WT, int P, int GPB = kGroupsPerBlock, bool SORT = false, bool FX = false>
__device__ __forceinline__ void grad_fast_body(const StepArgs& a, int block) {
    // pos_sort: P positive-sorted tiles of GPB positions per block (pair k of
    // group grp is position (block P + k) GPB + grp), each tile with its own
    // LDS run sums, so P tiles' rows are in flight before the first computes
    static_assert(!SORT || (MODEL != GBPR && GPB == kPsortPPB), "pos_sort: tiles of kPsortPPB positions");
    __shared__ double s_loss[GPB];
    __shared__ float s_gi[SORT ? P * GPB : 1][SORT ? kGL * EPL : 1];
    __shared__ int s_item[SORT ? P * GPB : 1];
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    float loss_g = 0.f;
    float sq = 0.f;
    PairRows<MODEL, EPL, WT> pr[P];
    int pp[P];
    bool ok[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        pp[k] = (block * P + k) * GPB + grp;
        ok[k] = pp[k] < a.B;
    }
    // pair-record prefetch for the next step (StepArgs::pf_out): issued
    // first, stored last, so its latency hides under this block's pairs
    int4 pfr = make_int4(0, 0, 0, 0);
    int64_t pfp = -1;
#ifndef CF_PAIR_PREFETCH
// 1: the prefetch compiled in.  Its registers take grad_sort_kernel<BPR, 4, 1>
// from 75 to 81 VGPRs, 6 -> 5 waves / SIMD: the cfg2 gradient launch ran
// 197.3 us with it, 179.9 us without (same box, round 4,
// profiles/r04/ab_occupancy/ab_r04_ab1.txt); the engine refuses the option unless built in
#define CF_PAIR_PREFETCH 0
#endif
    if constexpr (SORT && CF_PAIR_PREFETCH) {
        if (a.pf_out != nullptr && gl == 0) {
            const int64_t q = (int64_t)block * GPB + grp;
            if (q < a.pf_B) {
                pfp = q;
                pfr = a.pairs[permute(a.pf_slot_base + (uint64_t)q, a.pf_perm)];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) {
            if constexpr (SORT)
                pr[k].load_idx_sorted(a, pp[k]);   // pp = positive-sorted position
            else
                pr[k].load_idx(a, pp[k]);
        }
    if constexpr (MODEL == GBPR) {   // split exchange step: this pass's pairs only (group-uniform)
        if (a.member_pass != 0) {
#pragma unroll
            for (int k = 0; k < P; ++k) {
                bool local = true;
#pragma unroll
                for (int m = 0; m < PairRows<MODEL, EPL, WT>::NG; ++m) local &= pr[k].g[m] >= 0;
                if (local != (a.member_pass == 1)) ok[k] = false;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].template load_rows<SORT>(a, gl);
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].template load_acc<SORT>(a, gl);
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].template update<SORT>(a, gl, loss_g, sq, SORT ? &s_gi[k * GPB + grp][0] : nullptr);
    if constexpr (SORT) {
        // psort consumed this buffer set's phantoms: re-zero the count for
        // the set's next draw (StepArgs::spec_ph)
        if (block == 0 && threadIdx.x == 0 && a.spec_n != nullptr) *a.spec_n = 0;
#pragma unroll
        for (int k = 0; k < P; ++k)
            if (gl == 0) s_item[k * GPB + grp] = ok[k] ? pr[k].i : -1;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < P; ++k)
            if (ok[k] && (grp == 0 || s_item[k * GPB + grp - 1] != pr[k].i))
                psort_head<MODEL, EPL, WT, GPB, FX>(a, pr[k], block * P + k, grp, gl, s_gi + k * GPB,
                                                    s_item + k * GPB);
    }

    const float coef = (MODEL == CML) ? (a.reg_cov > 0.f ? a.reg_cov : 0.f) : a.reg;
    const float sq_g = gsum(sq);
    if (gl == 0) {
        const double lp = (double)loss_g + 0.5 * (double)coef * (double)sq_g;
        // deterministic: integer units, so the block and fold sums are exact
        s_loss[grp] = FX ? rint(lp * kFxLoss) : lp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < GPB; ++k) t += s_loss[k];
        a.loss_partial[block] = t;
    }
    if constexpr (SORT && CF_PAIR_PREFETCH) {
        if (pfp >= 0) a.pf_out[pfp] = pfr;
    }
}

// FULL (round 5): as grad_sort_kernel's, for the phased kernel without draw
// blocks -- cfg2 at SURVEY's B = 65,536 (pos_sort off) runs this one
template <int MODEL, int EPL, int WT, int P, bool DRAW, bool SORT = false, bool FULL = false>
#ifdef CF_GRAD_WAVES_PER_EU
#define CF_GRAD_ATTR __attribute__((amdgpu_waves_per_eu(CF_GRAD_WAVES_PER_EU, 8)))
#else
#define CF_GRAD_ATTR
#endif
__global__ __launch_bounds__(kBlock) CF_GRAD_ATTR void grad_fast_kernel(StepArgs a, StepArgs nx, int ng, int np) {
    if constexpr (FULL) __builtin_assume(a.d == kGL * EPL);
    int idx = blockIdx.x;
    if (DRAW && minor_block(blockIdx.x, ng, np, idx))
        prep_any<MODEL == GBPR ? GBPR : BPR>(nx, idx);
    else
        grad_fast_body<MODEL, EPL, WT, P, kGroupsPerBlock, SORT>(a, idx);
}

// the positive-sorted gradient launch (pos_sort) as its own kernel, so its
// register budget can be set apart from the other phased instantiations:
// CF_SORT_MIN_WAVES = minimum waves per SIMD (8 = at most 64 VGPRs).  8 was
// measured SLOWER at cfg2 (gradient launch 236 vs 179 us: the 74-VGPR body
// spills), so the budget is left to the compiler (6 waves/SIMD)
#ifndef CF_SORT_MIN_WAVES
#define CF_SORT_MIN_WAVES 1
#endif
#ifndef CF_ASSUME_FULL_ROWS
#define CF_ASSUME_FULL_ROWS 1
#endif
#ifndef CF_ASSUME_FULL_FAST
#define CF_ASSUME_FULL_FAST 1   // grad_fast_kernel's FULL instantiation at d = 64 (round 5)
#endif
// the same for apply_ps_kernel: measured even at cfg2/4/5 (round 4) -- the
// apply hoists more loads (79 -> 92 VGPRs, one wave per SIMD less), off
#ifndef CF_ASSUME_FULL_APPLY
#define CF_ASSUME_FULL_APPLY 0
#endif
// CF_SORT_TILES positive-sorted tiles per block (grad_fast_body)
#ifndef CF_SORT_TILES
#define CF_SORT_TILES 1
#endif
#ifndef CF_SORT_XCD
#define CF_SORT_XCD 1   // round 5: XCD-contiguous sorted tiles (cfg2 gradient 170 -> 163 us, profiles/r05/ab)
#endif
// DRAW (round 5, pipeline 3): the launch also carries the draw + count blocks
// of step s+1 (other buffer set), interleaved with the gradient blocks -- the
// draw is latency-bound, the gradient launch waits on memory 59 % of its
// wave cycles -- and the apply of step s then runs alone
template <int MODEL, int EPL, int WT, bool FX = false, bool FULL = false, bool DRAW = false>
__global__ __launch_bounds__(kBlock, CF_SORT_MIN_WAVES) void grad_sort_kernel(StepArgs a, StepArgs nx, int ng,
                                                                             int np) {
    // FULL: the launcher takes this instantiation only for full rows (d ==
    // 16 EPL), so every per-element `e < d` guard folds away -- each guarded
    // load / store was an exec-mask save, a branch and a restore: 1,907 ->
    // 1,285 instructions at cfg2 (round 4)
    if constexpr (FULL) __builtin_assume(a.d == kGL * EPL);
    int idx = blockIdx.x;
    if constexpr (DRAW) {
        if (minor_block(blockIdx.x, ng, np, idx)) {
            prep_any<BPR>(nx, idx);
            return;
        }
    }
#if CF_SORT_XCD
    // XCD-contiguous tiles: workgroups are dealt round-robin over the 8 XCDs
    // (b and b + 8 share one), so XCD x takes the contiguous run of sorted
    // tiles [x * full + min(x, rem), ...) -- a Zipf-head positive item whose
    // run spans many tiles is then gathered through one XCD's L2
    if constexpr (!DRAW) {
        const int nb = (int)gridDim.x, full = nb >> 3, rem = nb & 7, x = idx & 7;
        idx = x * full + (x < rem ? x : rem) + (idx >> 3);
    }
#endif
    grad_fast_body<MODEL, EPL, WT, CF_SORT_TILES, kGroupsPerBlock, true, FX>(a, idx);
}

// the same gradient blocks at one wave per workgroup (no draw blocks): a
// finer dispatch granule, so the last round of workgroups leaves less of the
// chip idle (a step's gradient launch is only ~2.7 rounds of 256-lane blocks)
template <int MODEL, int EPL, int WT, int P>
__global__ __launch_bounds__(kWave) void grad_fast_wave_kernel(StepArgs a) {
    grad_fast_body<MODEL, EPL, WT, P, kWave / kGL>(a, blockIdx.x);
}

// ---------------------------------------------------------------------------
// grad with LDS-staged negatives (d = 128, W = 5; BPR / AMF / CML; no
// pos_sort, no fused draw): cfg3 / cfg5's instantiation.
//
// The phased kernel keeps a pair's seven rows plus the accumulators of its
// singleton rows in registers: 218 VGPRs at d = 128 (2 waves / SIMD; CML 256
// + AGPRs, 1 wave).  Here the five negative rows of a wave's four pairs go
// from memory straight into LDS with global_load_lds_dwordx4 -- no VGPR
// destination, one wave-instruction moves two 512-B rows -- 40 KB per block,
// so four blocks (16 waves) fit a CU's 160 KB, and registers hold only u, i
// and the accumulator rows.  A negative's row is read from LDS where its term
// is formed (BPR / AMF once; CML for the distance, then for the gradient).
// Each wave reads only the rows it staged itself: no barrier.
// Element mapping: slot s of lane gl is element ((s ^ par) << 4) | gl, par =
// the group's parity, so the two groups of a ds_read_b32 half-wave (lanes
// 0-31, 32-63) hit different banks (staged rows are 128 dwords apart).
// Same arithmetic as grad_fast_kernel up to fp32 summation order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int elem_par(int s, int gl, int par) { return ((s ^ par) << 4) | gl; }

// full rows only (d == 16 * EPL): no element masks, straight-line code
template <int EPL>
__device__ __forceinline__ void prow_ld(const float* __restrict__ row, int gl, int par, float (&x)[EPL]) {
#pragma unroll
    for (int s = 0; s < EPL; ++s) x[s] = row[elem_par(s, gl, par)];
}

template <int EPL>
__device__ __forceinline__ void prow_st(float* __restrict__ row, int gl, int par, const float (&x)[EPL]) {
#pragma unroll
    for (int s = 0; s < EPL; ++s) row[elem_par(s, gl, par)] = x[s];
}

template <int EPL>
__device__ __forceinline__ void prow_atomic(float* __restrict__ row, int gl, int par, const float (&g)[EPL]) {
#pragma unroll
    for (int s = 0; s < EPL; ++s) unsafeAtomicAdd(row + elem_par(s, gl, par), g[s]);
}

// gapply_pre / gfinish_pre / ifinish_pre in the parity mapping
template <int EPL>
__device__ __forceinline__ void papply(float* __restrict__ X, float* __restrict__ A, int64_t r, int d, int gl,
                                       int par, const float (&x0)[EPL], const float (&acc0)[EPL],
                                       const float (&g)[EPL], float lr, bool clip, float c) {
    float acc[EPL], x[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        acc[s] = fmaf(g[s], g[s], acc0[s]);
        x[s] = x0[s] - adagrad_delta(lr, g[s], acc[s]);
    }
    if (clip) {
        const float n = sqrtf(gdot<EPL>(x, x));
        const float den = fmaxf(n, c);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * c) / den;
    }
    prow_st<EPL>(X + r * (int64_t)d, gl, par, x);
    prow_st<EPL>(A + r * (int64_t)d, gl, par, acc);
}

template <int EPL>
__device__ __forceinline__ void pfinish(float* __restrict__ X, float* __restrict__ A, float* __restrict__ G,
                                        float* __restrict__ S, int32_t* __restrict__ cnt, int64_t r, int count,
                                        int64_t slot, int d, int gl, int par, const float (&x0)[EPL],
                                        const float (&acc0)[EPL], const float (&g)[EPL], const StepArgs& a) {
    if (count == 1) {
        if (a.items_grad_only && X == a.V)
            prow_st<EPL>(G + r * (int64_t)d, gl, par, g);   // sole writer of the zeroed dense row
        else
            papply<EPL>(X, A, r, d, gl, par, x0, acc0, g, a.lr, a.clip != 0, a.clip_norm);
        if (gl == 0) cnt[r] = 0;
    } else if (slot >= 0) {
        prow_st<EPL>(S + slot * (int64_t)d, gl, par, g);
    } else {
        prow_atomic<EPL>(acc_of(G, slot, a) + r * (int64_t)d, gl, par, g);
        if (a.items_grad_only && a.capV == 0 && X == a.V && gl == 0) cnt[r] = 0;  // see gfinish
    }
}

template <int EPL>
__device__ __forceinline__ void pifinish(const StepArgs& a, int64_t r, int count, int64_t slot, int p,
                                         float alpha, float beta, int which, int gl, int par,
                                         const float (&x0)[EPL], const float (&acc0)[EPL],
                                         const float (&g)[EPL]) {
    if (a.recV != nullptr && count >= 2 && slot >= 0) {
        if (gl == 0) a.recV[slot] = make_int4(p, __float_as_int(alpha), __float_as_int(beta), which);
        return;
    }
    pfinish<EPL>(a.V, a.AV, a.GV, a.slotV, a.cntV, r, count, slot, a.d, gl, par, x0, acc0, g, a);
}

template <int EPL>
__device__ __forceinline__ void pacc_ld(const float* __restrict__ A, int64_t r, int d, int gl, int par, bool want,
                                        float (&acc)[EPL]) {
#pragma unroll
    for (int s = 0; s < EPL; ++s) acc[s] = 1.f;
    if (want) prow_ld<EPL>(A + r * (int64_t)d, gl, par, acc);
}

// minimum waves per SIMD the LDS-staged kernel is built for (1 = the
// compiler's register budget; LDS alone allows 4)
#ifndef CF_LDS_WAVES
#define CF_LDS_WAVES 1
#endif
#ifndef CF_LDS_WAVES_GBPR
#define CF_LDS_WAVES_GBPR 1   // 4 (with CF_LDS_STAGE_ACC: 128 VGPRs, 12-B spill) measured slower (r04j)
#endif
#define CF_LDS_ATTR __attribute__((amdgpu_waves_per_eu(MODEL == GBPR ? CF_LDS_WAVES_GBPR : CF_LDS_WAVES, 8)))
// one negative's LDS reads are not hoisted above the previous negative's
// terms (the scheduler would otherwise keep all five rows live)
#ifndef CF_LDS_FENCE
#define CF_LDS_FENCE 1
#endif
#if CF_LDS_FENCE
#define CF_LDS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define CF_LDS_SCHED_FENCE() ((void)0)
#endif
// EPL = 8 (d = 128): BPR / AMF / CML, 40 KB of staged rows per block, a
// negative's accumulator loaded where it is finished (rows seen once are rare
// at 100K items).  EPL = 4 (d = 64): GBPR at G = 1 (cfg4), 20 KB per block;
// at 1M items nearly every negative is its row's only occurrence, so the
// negatives' accumulators are loaded with the rows (GBPR's ACC_EARLY).
template <int MODEL, int EPL, int WT>
__global__ __launch_bounds__(kBlock) CF_LDS_ATTR void grad_lds_kernel(StepArgs a) {
    constexpr int ROW = kGL * EPL;            // floats per staged row (full rows only)
    constexpr int RPI = kWave * 4 / ROW;      // rows per LDS-DMA wave-instruction (16 B per lane)
    constexpr int LPR = kWave / RPI;          // lanes per row
    constexpr int RPW = (kWave / kGL) * WT;   // staged rows per wave
    constexpr bool ACC_EARLY = MODEL == GBPR;
    static_assert(RPW % RPI == 0, "whole rows per LDS-DMA wave-instruction");
    static_assert(MODEL == BPR || MODEL == AMF || MODEL == CML || MODEL == GBPR, "no tuples here");
    // 40 KB (d = 128) / 20 KB (d = 64) per block; the loss partials reuse it
    __shared__ float s_v[kGroupsPerBlock * WT * ROW];
    // GBPR (ACC_EARLY): the negatives' accumulator rows staged the same way
    // (round 4) instead of held in 20 VGPRs -- 40 KB per block, four blocks per
    // CU, and the registers for four waves per SIMD
#ifndef CF_LDS_STAGE_ACC
#define CF_LDS_STAGE_ACC 0   // 1 measured slower at cfg4 (131.6 vs 126.2 us with 4 waves, 12-B spill; r04j)
#endif
    constexpr bool STAGE_ACC = ACC_EARLY && CF_LDS_STAGE_ACC;
    __shared__ float s_a[STAGE_ACC ? kGroupsPerBlock * WT * ROW : 1];
    const int lane = threadIdx.x & (kWave - 1);
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    const int par = grp & 1;
    const int d = a.d;
    const int p = blockIdx.x * kGroupsPerBlock + grp;
    bool ok = p < a.B;

    // ids (every lane of the group loads the same words)
    int u = 0, i = 0, ru = 0, ri = 0, g = 0, rg = 0;
    int j[WT], rj[WT];
#pragma unroll
    for (int w = 0; w < WT; ++w) {
        j[w] = -1;
        rj[w] = 0;
    }
    if (ok) {
        u = a.occU[p];
        i = a.occV[p];
        ru = a.count_users ? a.rankU[p] : 0;
        ri = a.count_items ? a.rankV[p] : 0;
#pragma unroll
        for (int w = 0; w < WT; ++w) {
            j[w] = a.occV[a.B + p * WT + w];
            rj[w] = a.count_items ? a.rankV[a.B + p * WT + w] : 0;
        }
        if (MODEL == GBPR) {   // G = 1: the group member (-1 - k: row k of xrows, another rank's user)
            g = a.occU[a.B + p];
            rg = a.count_users ? a.rankU[a.B + p] : 0;
            // split exchange step: only this pass's pairs (group-uniform)
            if (a.member_pass != 0 && (g >= 0) != (a.member_pass == 1)) ok = false;
        }
    }
    if (!ok) {
#pragma unroll
        for (int w = 0; w < WT; ++w) j[w] = -1;   // nothing staged for this group
    }
    // stage the negatives: wave-instruction k moves the wave's rows
    // RPI*k .. RPI*k + RPI - 1 (LPR lanes each, 16 B per lane); row r is
    // negative r % WT of the wave's pair r / WT, whose id lane (r / WT) * 16 +
    // r % WT holds
    {
        int jsel = -1;
#pragma unroll
        for (int w = 0; w < WT; ++w)
            if (gl == w) jsel = j[w];
        float* wbase = s_v + (threadIdx.x >> 6) * RPW * ROW;
        float* abase = s_a + (STAGE_ACC ? (threadIdx.x >> 6) * RPW * ROW : 0);
        const int c4 = (lane % LPR) * 4;
        const bool stage_acc = STAGE_ACC && !a.items_grad_only;
#pragma unroll
        for (int k = 0; k < RPW / RPI; ++k) {
            const int r = RPI * k + lane / LPR;
            const int q = r / WT;
            const int jj = __shfl(jsel, q * kGL + (r - q * WT), kWave);
            if (jj >= 0)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(a.V + (int64_t)jj * d + c4),
                    (__attribute__((address_space(3))) void*)(wbase + RPI * k * ROW), 16, 0, 0);
            // every negative's accumulator row (at 1M items nearly all are
            // their row's only occurrence; no count is needed to issue it)
            if (stage_acc && jj >= 0)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(a.AV + (int64_t)jj * d + c4),
                    (__attribute__((address_space(3))) void*)(abase + RPI * k * ROW), 16, 0, 0);
        }
    }
    // counts and the u / i rows, then slots and the accumulator rows of the
    // rows this batch touches once
    int cu = 0, ci = 0, cg = 0, cj[WT];
    float uu[EPL], vi[EPL], ug[MODEL == GBPR ? EPL : 1];
    float bi = 0.f, bj[WT];   // GBPR item biases
#pragma unroll
    for (int w = 0; w < WT; ++w) {
        cj[w] = 0;
        bj[w] = 0.f;
    }
    if (ok) {
        cu = a.count_users ? a.cntU[u] : 0;
        ci = a.count_items ? a.cntV[i] : 0;
#pragma unroll
        for (int w = 0; w < WT; ++w) cj[w] = a.count_items ? a.cntV[j[w]] : 0;
        prow_ld<EPL>(a.U + (int64_t)u * d, gl, par, uu);
        prow_ld<EPL>(a.V + (int64_t)i * d, gl, par, vi);
        if constexpr (MODEL == GBPR) {
            cg = (a.count_users && g >= 0) ? a.cntU[g] : 0;
            prow_ld<EPL>(g >= 0 ? a.U + (int64_t)g * d : a.xrows + (int64_t)(-1 - g) * d, gl, par, ug);
            bi = a.b[i];
#pragma unroll
            for (int w = 0; w < WT; ++w) bj[w] = a.b[j[w]];
        }
    }
    // slot rows as int32 (n_users * capU and n_items * capV < 2^31 wherever
    // this kernel runs: 10M x 2, 1M x 32 at cfg4): 8 VGPRs fewer than int64
    int32_t su = -1, si = -1, sg = -1, sj[WT];
    float au[EPL], ai[EPL], ag[MODEL == GBPR ? EPL : 1], aje[ACC_EARLY && !STAGE_ACC ? WT : 1][EPL];
    float abi = 0.f, abj[WT];   // GBPR: bias accumulators of rows seen once
    const bool item_acc = !a.items_grad_only;
#pragma unroll
    for (int w = 0; w < WT; ++w) abj[w] = 0.f;
    if (ok) {
        su = slot_of(cu, u, ru, a.capU, 0, a.offU);
        si = slot_of(ci, i, ri, a.capV, a.repV, a.offV);
#pragma unroll
        for (int w = 0; w < WT; ++w) sj[w] = slot_of(cj[w], j[w], rj[w], a.capV, a.repV, a.offV);
        pacc_ld<EPL>(a.AU, u, d, gl, par, cu == 1, au);
        pacc_ld<EPL>(a.AV, i, d, gl, par, item_acc && ci == 1, ai);
        if constexpr (MODEL == GBPR) {
            sg = slot_of(cg, g, rg, a.capU, 0, a.offU);
            pacc_ld<EPL>(a.AU, g, d, gl, par, g >= 0 && cg == 1, ag);
            abi = (item_acc && ci == 1) ? a.Ab[i] : 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) abj[w] = (item_acc && cj[w] == 1) ? a.Ab[j[w]] : 0.f;
        }
        if constexpr (ACC_EARLY && !STAGE_ACC) {
#pragma unroll
            for (int w = 0; w < WT; ++w) pacc_ld<EPL>(a.AV, j[w], d, gl, par, item_acc && cj[w] == 1, aje[w]);
        }
    }
    // the staged rows have landed (an LDS-DMA retires on vmcnt).  The
    // builtin, not inline asm: the compiler's wait tracking sees it and stops
    // guarding every later LDS read with a vmcnt wait for the DMA
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)

    float loss_g = 0.f, sq = 0.f;
    if (ok) {
        const float* sv = s_v + grp * WT * ROW;
        if (a.recV != nullptr) {   // item records' X: only pairs that leave one
            bool need = MODEL != GBPR && ci >= 2 && si >= 0;
#pragma unroll
            for (int w = 0; w < WT; ++w) need |= cj[w] >= 2 && sj[w] >= 0;
            if (need) prow_st<EPL>(a.stashU + (int64_t)p * d, gl, par, uu);
        }
        if (MODEL == BPR || MODEL == AMF) {
            // terms first (no stores), then u and i, then the negatives'
            // gradient rows from the staged rows again: no store of one
            // negative sits between the next one's loads and their use
            const float ui = gdot<EPL>(uu, vi);
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
            float cw[WT];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                float vj[EPL];
                prow_ld<EPL>(sv + w * ROW, gl, par, vj);
                const float x = ui - gdot<EPL>(uu, vj);
                float c = -rcp_1p(expf(x));
                if (MODEL == AMF) {
                    loss_g += softplus(-x);
                    if (a.adversarial) {
                        const float xc = fmaxf(fminf(x, 1e8f), -80.f);
                        loss_g += a.reg_adv * softplus(-xc);
                        if (x >= -80.f && x <= 1e8f) c *= (1.f + a.reg_adv);
                    }
                } else {
                    loss_g += neg_log_sigmoid(x);
                }
                sc += c;
                cw[w] = c;
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(c, vi[s] - vj[s], gu[s]);
                    sq = fmaf(vj[s], vj[s], sq);
                }
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += a.reg * uu[s];
                gi[s] = sc * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            pfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, par, uu, au, gu, a);
            pifinish<EPL>(a, i, ci, si, p, sc, a.reg, 0, gl, par, vi, ai, gi);
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                CF_LDS_SCHED_FENCE();
                float vj[EPL], aj[EPL], gj[EPL];
                pacc_ld<EPL>(a.AV, j[w], d, gl, par, item_acc && cj[w] == 1, aj);
                prow_ld<EPL>(sv + w * ROW, gl, par, vj);
#pragma unroll
                for (int s = 0; s < EPL; ++s) gj[s] = -cw[w] * uu[s] + a.reg * vj[s];
                pifinish<EPL>(a, j[w], cj[w], sj[w], p, -cw[w], a.reg, 0, gl, par, vj, aj, gj);
            }
        } else if (MODEL == CML) {
            float du[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) du[s] = uu[s] - vi[s];
            const float dp = gdot<EPL>(du, du);
            float dn[WT];
            float m = INFINITY;
            int imp = 0;
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                CF_LDS_SCHED_FENCE();
                float t[EPL];
                prow_ld<EPL>(sv + w * ROW, gl, par, t);
#pragma unroll
                for (int s = 0; s < EPL; ++s) t[s] = uu[s] - t[s];
                dn[w] = gdot<EPL>(t, t);
                m = fminf(m, dn[w]);
                imp += (dp - dn[w] + a.margin > 0.f) ? 1 : 0;
            }
            float cnt = 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) cnt += (dn[w] == m) ? 1.f : 0.f;
            const float z = dp - m + a.margin;
            const float lw = a.use_rank_weight ? logf((float)imp / (float)WT * a.n_items_f + 1.f) : 1.f;
            loss_g += fmaxf(z, 0.f) * lw;
            const float aa = (z > 0.f) ? lw : 0.f;
            const bool l2 = a.reg_cov > 0.f;
            float gu[EPL], gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] = 2.f * aa * du[s];
                gi[s] = -2.f * aa * du[s];
            }
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                const float share = (dn[w] == m) ? 1.f / cnt : 0.f;
                const float coef = 2.f * aa * share;
                CF_LDS_SCHED_FENCE();
                float vj[EPL], gj[EPL], aj[EPL];
                pacc_ld<EPL>(a.AV, j[w], d, gl, par, item_acc && cj[w] == 1, aj);
                prow_ld<EPL>(sv + w * ROW, gl, par, vj);
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    const float dv = uu[s] - vj[s];
                    gu[s] = fmaf(-coef, dv, gu[s]);
                    gj[s] = coef * dv;
                    if (l2) {
                        gj[s] += a.reg_cov * vj[s];
                        sq = fmaf(vj[s], vj[s], sq);
                    }
                }
                // a touched row with a zero gradient is still clipped (cml.py:128-129)
                pifinish<EPL>(a, j[w], cj[w], sj[w], p, coef, (l2 ? a.reg_cov : 0.f) - coef, 0, gl, par, vj,
                              aj, gj);
            }
            if (l2) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] += a.reg_cov * uu[s];
                    gi[s] += a.reg_cov * vi[s];
                    sq = fmaf(uu[s], uu[s], sq);
                    sq = fmaf(vi[s], vi[s], sq);
                }
            }
            pfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, par, uu, au, gu, a);
            pifinish<EPL>(a, i, ci, si, p, -2.f * aa, 2.f * aa + (l2 ? a.reg_cov : 0.f), 0, gl, par, vi, ai, gi);
        } else if constexpr (MODEL == GBPR) {   // G == 1 (gbprmf.py:58-106)
#pragma unroll
            for (int s = 0; s < EPL; ++s) sq = fmaf(ug[s], ug[s], sq);
            const float ui = a.rho * gdot<EPL>(ug, vi) + (1.f - a.rho) * gdot<EPL>(uu, vi) + bi;
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
            float cw[WT];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                float vj[EPL];
                prow_ld<EPL>(sv + w * ROW, gl, par, vj);
                const float x = ui - (gdot<EPL>(uu, vj) + bj[w]);
                const float c = -rcp_1p(expf(x));
                loss_g += neg_log_sigmoid(x) + 0.5f * a.reg * bj[w] * bj[w];
                sc += c;
                cw[w] = c;
#pragma unroll
                for (int s = 0; s < EPL; ++s) gu[s] = fmaf(-c, vj[s], gu[s]);
            }
            const float rg_ = a.rho;   // rho / G with G == 1
            float gi[EPL], gg[EPL], bl[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += (1.f - a.rho) * sc * vi[s] + a.reg * uu[s];
                bl[s] = rg_ * ug[s] + (1.f - a.rho) * uu[s];
                gi[s] = sc * bl[s] + a.reg * vi[s];
                gg[s] = rg_ * sc * vi[s] + a.reg * ug[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            pfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, u, cu, su, d, gl, par, uu, au, gu, a);
            if (g >= 0)
                pfinish<EPL>(a.U, a.AU, a.GU, a.slotU, a.cntU, g, cg, sg, d, gl, par, ug, ag, gg, a);
            else   // another rank's user: its gradient row goes back to the owner
                prow_st<EPL>(a.xgrads + (int64_t)(-1 - g) * d, gl, par, gg);
            if (gl == 0) bias_finish_pre(a, i, ci, sc, si, bi, abi);
            if (a.recV != nullptr && ci >= 2 && si >= 0) prow_st<EPL>(a.stashB + (int64_t)p * d, gl, par, bl);
            pifinish<EPL>(a, i, ci, si, p, sc, a.reg, 1, gl, par, vi, ai, gi);
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                CF_LDS_SCHED_FENCE();
                float vj[EPL], gj[EPL];
                prow_ld<EPL>(sv + w * ROW, gl, par, vj);
#pragma unroll
                for (int s = 0; s < EPL; ++s) gj[s] = -cw[w] * uu[s];   // no L2 on V[j] (gbprmf.py:59-64)
                if (gl == 0) bias_finish_pre(a, j[w], cj[w], -cw[w] + a.reg * bj[w], sj[w], bj[w], abj[w]);
                if constexpr (STAGE_ACC) {
                    float aj[EPL];
#pragma unroll
                    for (int s = 0; s < EPL; ++s) aj[s] = 1.f;
                    if (item_acc && cj[w] == 1) prow_ld<EPL>(s_a + grp * WT * ROW + w * ROW, gl, par, aj);
                    pifinish<EPL>(a, j[w], cj[w], sj[w], p, -cw[w], 0.f, 0, gl, par, vj, aj, gj);
                } else {
                    pifinish<EPL>(a, j[w], cj[w], sj[w], p, -cw[w], 0.f, 0, gl, par, vj, aje[ACC_EARLY ? w : 0], gj);
                }
            }
        }
    }

    // each group's loss partial goes into its own wave's staged rows, which
    // that wave no longer reads
    const float coef = (MODEL == CML) ? (a.reg_cov > 0.f ? a.reg_cov : 0.f) : a.reg;
    const float sq_g = gsum(sq);
    double* s_loss = reinterpret_cast<double*>(s_v);
    constexpr int kWaveD = RPW * ROW / 2;   // doubles per wave region
    if (gl == 0)
        s_loss[(grp >> 2) * kWaveD + (grp & 3)] = (double)loss_g + 0.5 * (double)coef * (double)sq_g;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < kGroupsPerBlock; ++k) t += s_loss[(k >> 2) * kWaveD + (k & 3)];
        a.loss_partial[blockIdx.x] = t;
    }
}

// ---------------------------------------------------------------------------
// apply the summed gradient of every duplicated row: the TF1 IndexedSlices
// dedup-sum + SparseApplyAdagrad (bprmf.py:74-75 and siblings).
// One lane per work item -- the batch's user occurrences, item occurrences
// and (group exchange) served rows.  The owner of a duplicated row is its
// rank-0 occurrence (or, for a served row with no local occurrence, its first
// server).  Owners are ballot-compacted and handed to the wave's four 16-lane
// groups: the row's slot rows r*cap + [0, count) summed in rank order, or the
// atomic sum in G for a hot row (G re-zeroed); Adagrad; the count reset.
// Block 0 also folds the grad kernel's loss partials.
// ---------------------------------------------------------------------------
// a duplicated row's slots [lo, hi) (base s0) added to g in rank order:
// gradient rows, or item records (alpha X from the stash into g, beta into bsum)
template <int EPL, int NF>
__device__ __forceinline__ void slot_sum(const ApplyArgs& a, bool isU, int64_t s0, int lo, int hi, int gl,
                                         float (&g)[EPL], float& bsum) {
    if (!isU && a.recV != nullptr) {
        for (int t0 = lo; t0 < hi; t0 += NF) {
            int4 rc[NF];
            float h[NF][EPL];
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < hi) rc[q] = a.recV[s0 + t0 + q];
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < hi) gload<EPL>(rc[q].w ? a.stashB : a.stashU, rc[q].x, a.d, gl, h[q]);
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < hi) {
                    const float al = __int_as_float(rc[q].y);
#pragma unroll
                    for (int s = 0; s < EPL; ++s) g[s] = fmaf(al, h[q][s], g[s]);
                    bsum += __int_as_float(rc[q].z);
                }
        }
    } else {
        const float* S = isU ? a.slotU : a.slotV;
        for (int t0 = lo; t0 < hi; t0 += NF) {
            float h[NF][EPL];
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < hi) gload<EPL>(S, s0 + t0 + q, a.d, gl, h[q]);
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < hi) {
#pragma unroll
                    for (int s = 0; s < EPL; ++s) g[s] += h[q][s];
                }
        }
    }
}

// HOT: the deterministic-mode launch that adds whole-tile sums (its own
// instantiation: the tile path's registers would slow every fast-path apply)
template <int EPL, bool HOT = false, bool FX = false>
__device__ __forceinline__ void apply_row(const ApplyArgs& a, int64_t r, bool isU, int c, int gl) {
    int32_t* cnt = isU ? a.cntU : a.cntV;
    float* X = isU ? a.U : a.V;
    float* A = isU ? a.AU : a.AV;
    float* G = isU ? a.GU : a.GV;
    const int cap = isU ? a.capU : a.capV;
    // multi-rank item reduce: the row's summed gradient goes to GV for the
    // all-reduce; the table and accumulator are left to cf_step_items
    const bool reduce_only = !isU && a.items_grad_only;
    float x[EPL], acc[EPL], g[EPL];
    if (!reduce_only) {
        gload<EPL>(X, r, a.d, gl, x);
        gload_acc<EPL>(A, r, a.d, gl, true, acc);
    }
    // c = the row's count word: occurrences, plus kRemoteFlag for a row the
    // group exchange served (all its contributions went to G)
    const int flagged = c & kRemoteFlag;
    const int local = c & (kRemoteFlag - 1);
    const int32_t* off = isU ? a.offU : a.offV;   // deterministic mode: compact slots
    const int ns = flagged ? 0 : (off != nullptr || local < cap) ? local : cap;
#pragma unroll
    for (int s = 0; s < EPL; ++s) g[s] = 0.f;
#ifndef CF_APPLY_NF
#define CF_APPLY_NF 4
#endif
    constexpr int NF = CF_APPLY_NF;  // slot rows in flight, summed in rank order (8: occupancy 5, slower)
    // slots [0, ns) in rank order -- or, in deterministic mode for a row of
    // >= 2 whole 64-slot tiles, the head before its first whole tile, the
    // tiles' sums (det_hot_kernel) in tile order, then the tail
    const int64_t s0 = off != nullptr ? (int64_t)off[r] : r * (int64_t)cap;
    float bsum = 0.f;
    if (HOT && off != nullptr && ns >= 2 * kDetTile) {
        const int64_t gs = (isU ? 0 : a.nU) + off[r], ge = gs + ns;
        const int64_t qa = (gs + kDetTile - 1) / kDetTile, qb = ge / kDetTile;
        slot_sum<EPL, NF>(a, isU, s0, 0, (int)(qa * kDetTile - gs), gl, g, bsum);
        for (int64_t q0 = qa; q0 < qb; q0 += NF) {
            float h[NF][EPL];
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (q0 + q < qb) gload<EPL>(a.hotP, q0 + q, a.d, gl, h[q]);
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (q0 + q < qb) {
#pragma unroll
                    for (int s = 0; s < EPL; ++s) g[s] += h[q][s];
                    if (!isU && a.recV != nullptr) bsum += a.hotPb[q0 + q];
                }
        }
        slot_sum<EPL, NF>(a, isU, s0, (int)(qb * kDetTile - gs), ns, gl, g, bsum);
    } else if (FX && isU) {
        // deterministic pos_sort (users): the slot rows and the int64 atomic
        // overflow (GU64) summed exactly in fixed point, in any order
        long long t[EPL];
#pragma unroll
        for (int s = 0; s < EPL; ++s) t[s] = 0;
        for (int t0 = 0; t0 < ns; t0 += NF) {
            float h[NF][EPL];
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < ns) gload<EPL>(a.slotU, s0 + t0 + q, a.d, gl, h[q]);
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < ns) {
#pragma unroll
                    for (int s = 0; s < EPL; ++s) t[s] += to_fx(h[q][s], a.fx_bad);
                }
        }
        if (local > cap) {
            unsigned long long* row = a.GU64 + (int64_t)a.hotU[r] * a.d;
            fx_ld_add<EPL>(reinterpret_cast<const long long*>(row), a.d, gl, t);
            long long z[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) z[s] = 0;
            fx_st<EPL>(reinterpret_cast<long long*>(row), a.d, gl, z);
        }
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] = from_fx(t[s], a.fx_bad);
    } else {
        slot_sum<EPL, NF>(a, isU, s0, 0, ns, gl, g, bsum);
    }
    if (!isU && a.recV != nullptr) {
        if (reduce_only) gload<EPL>(X, r, a.d, gl, x);
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] = fmaf(bsum, x[s], g[s]);
    }
    if (off == nullptr && (flagged || local > cap) && !(FX && isU)) {  // the atomic sums: G, and for items the copies in use
        const int nrep = isU ? 0 : a.repV;   // copies 1..repV (unused ones are zero)
        float h[EPL];
        gload<EPL>(G, r, a.d, gl, h);
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] += h[s];
        if (!reduce_only) row_zero<EPL>(G + r * a.d, a.d, gl);
        for (int k = 0; k < nrep; ++k) {
            float* Gk = a.GVrep + (int64_t)k * a.n_items * a.d;
            gload<EPL>(Gk, r, a.d, gl, h);
#pragma unroll
            for (int s = 0; s < EPL; ++s) g[s] += h[s];
            row_zero<EPL>(Gk + r * a.d, a.d, gl);
        }
    }
    // item bias (GBPR / CPLR): its slots in rank order (lane 0) + what hot-row
    // atomics left in Gb
    float gbias = 0.f;
    const bool bias_row = !isU && a.slotVb != nullptr && a.Gb != nullptr;
    if (bias_row) {   // the group's 16 lanes load the slots, a fixed-order butterfly sums them
        const int64_t s0 = off != nullptr ? (int64_t)off[r] : r * (int64_t)cap;
        float t = 0.f;
        for (int q = gl; q < ns; q += kGL) t += a.slotVb[s0 + q];
        gbias = gsum(t) + a.Gb[r];
    }
    if (reduce_only) {
        row_st<EPL>(G + r * (int64_t)a.d, a.d, gl, g);
        if (gl == 0) {
            cnt[r] = 0;
            if (bias_row) a.Gb[r] = gbias;
        }
        return;
    }
    gapply_pre<EPL>(X, A, r, a.d, gl, x, acc, g, a.lr, a.clip != 0, a.clip_norm);
    if (gl == 0) {
        cnt[r] = 0;
        if (!isU && a.b != nullptr) {
            const float gb = bias_row ? gbias : a.Gb[r];
            const float ab = fmaf(gb, gb, a.Ab[r]);
            a.Ab[r] = ab;
            a.b[r] -= adagrad_delta(a.lr, gb, ab);
            a.Gb[r] = 0.f;
        }
    }
}

// pos_sort: a duplicated item row's gradient = its negatives' slot rows
// (rank order) + its positive partials (block order) + the float-atomic sum
// of what overflowed either range; Adagrad; both counts reset
template <int EPL>
__device__ __forceinline__ void rows_sum(const float* __restrict__ S, int64_t s0, int n, int d, int gl,
                                         float (&g)[EPL]) {
    constexpr int NF = CF_APPLY_NF;
    for (int t0 = 0; t0 < n; t0 += NF) {
        float h[NF][EPL];
#pragma unroll
        for (int q = 0; q < NF; ++q)
            if (t0 + q < n) gload<EPL>(S, s0 + t0 + q, d, gl, h[q]);
#pragma unroll
        for (int q = 0; q < NF; ++q)
            if (t0 + q < n) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) g[s] += h[q][s];
            }
    }
}

#ifndef CF_APPLY_NF_PS
#define CF_APPLY_NF_PS 8   // rows in flight per group in the pos_sort item apply
#endif
template <int EPL, bool FX = false>
__device__ __forceinline__ void apply_item_ps(const ApplyArgs& a, int64_t r, int gl, int cn, int cp, int o,
                                              int on) {
    // multi-rank item reduce: the summed row goes to GV for the exchange
    const bool reduce_only = a.items_grad_only;
    float x[EPL], acc[EPL], g[EPL];
    if (!reduce_only) {
        gload<EPL>(a.V, r, a.d, gl, x);
        gload_acc<EPL>(a.AV, r, a.d, gl, true, acc);
    }
    const int np = cp > 0 ? (o + cp - 1) / kPsortPPB - o / kPsortPPB + 1 : 0;
    const int nn = cn;   // every negative occurrence has its compact slot
    const int npp = np < a.capP ? np : a.capP;
    const float* P0 = a.slotP + ((int64_t)(o / kPsortPPB) + r) * a.d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) g[s] = 0.f;
    // the negatives' compact slot rows [on, on + nn) in rank order (contiguous),
    // then the positives' partial rows in block order: all independent loads,
    // NF of them in flight
    const int nt = nn + npp;
    constexpr int NF = CF_APPLY_NF_PS;
    if constexpr (FX) {
        // deterministic: the negatives' rows and the int64 partials summed
        // exactly in fixed point (the order the atomic ranks gave them is moot)
        long long t[EPL];
#pragma unroll
        for (int s = 0; s < EPL; ++s) t[s] = 0;
        for (int t0 = 0; t0 < nn; t0 += NF) {
            float h[NF][EPL];
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < nn) row_ld<EPL>(a.slotV + ((int64_t)on + t0 + q) * a.d, a.d, gl, 0.f, h[q]);
#pragma unroll
            for (int q = 0; q < NF; ++q)
                if (t0 + q < nn) {
#pragma unroll
                    for (int s = 0; s < EPL; ++s) t[s] += to_fx(h[q][s], a.fx_bad);
                }
        }
        // the partials, NF / 2 int64 rows in flight (a Zipf-head item has
        // hundreds: one at a time they were a serial chain of load latencies)
        const long long* P64 = a.slotP64 + ((int64_t)(o / kPsortPPB) + r) * a.d;
        constexpr int NF2 = NF / 2 > 0 ? NF / 2 : 1;
        const bool full = vec_rows<EPL>() && a.d == kGL * EPL;
        for (int t0 = 0; t0 < npp; t0 += NF2) {
            long long h[NF2][EPL];
#pragma unroll
            for (int q = 0; q < NF2; ++q)
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    const int e = elem_of<EPL>(s, gl, full);
                    h[q][s] = (t0 + q < npp && e < a.d) ? P64[(int64_t)(t0 + q) * a.d + e] : 0ll;
                }
#pragma unroll
            for (int q = 0; q < NF2; ++q)
#pragma unroll
                for (int s = 0; s < EPL; ++s) t[s] += h[q][s];
        }
        if (np > a.capP) {   // the int64 atomic overflow (GV64), re-zeroed
            long long* row = reinterpret_cast<long long*>(a.GV64 + r * a.d);
            fx_ld_add<EPL>(row, a.d, gl, t);
            long long z[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) z[s] = 0;
            fx_st<EPL>(row, a.d, gl, z);
        }
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] = from_fx(t[s], a.fx_bad);
    }
    for (int t0 = 0; t0 < (FX ? 0 : nt); t0 += NF) {
        float h[NF][EPL];
#pragma unroll
        for (int q = 0; q < NF; ++q) {
            const int t = t0 + q;
            if (t < nt) {
                const float* row = t < nn ? a.slotV + ((int64_t)on + t) * a.d
                                          : P0 + (int64_t)(t - nn) * a.d;
                row_ld<EPL>(row, a.d, gl, 0.f, h[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < NF; ++q)
            if (t0 + q < nt) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) g[s] += h[q][s];
            }
    }
    if (!FX && np > a.capP) {   // partials past the positives' slot range: float atomics into GV
        float h[EPL];
        gload<EPL>(a.GV, r, a.d, gl, h);
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] += h[s];
        if (!reduce_only) row_zero<EPL>(a.GV + r * a.d, a.d, gl);
    }
    if (reduce_only)
        row_st<EPL>(a.GV + r * (int64_t)a.d, a.d, gl, g);
    else
        gapply_pre<EPL>(a.V, a.AV, r, a.d, gl, x, acc, g, a.lr, a.clip != 0, a.clip_norm);
    if (gl == 0) {
        a.cntV[r] = 0;
        a.cntP[r] = 0;
    }
}

// block 0 of an apply launch folds the gradient launch's loss partials in a
// fixed order (eight partials in flight per lane, not a chain of loads)
template <int BS>
__device__ __forceinline__ void fold_loss(const ApplyArgs& a) {
    constexpr int NWV = BS / kWave;
    __shared__ double s_red[NWV];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    double t = 0.0;
    for (int k0 = threadIdx.x; k0 < a.n_partial; k0 += 8 * BS) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int k = k0 + q * BS;
            v[q] = k < a.n_partial ? a.loss_partial[k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) t += v[q];
    }
    t = wave_sum_d(t);
    if (lane == 0) s_red[wv] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tt = 0.0;
        for (int w = 0; w < NWV; ++w) tt += s_red[w];
        a.loss_acc[0] += a.det_fx ? tt / kFxLoss : tt;   // det_fx: an exact integer sum
    }
}

// ---------------------------------------------------------------------------
// pos_sort apply (apply_ps_kernel).  A duplicated item's gradient is its
// negatives' compact slot rows (rank order) + its positive partials (block
// order) + the float-atomic sum of what overflowed either range -- TF1's
// dedup-sum (bprmf.py:83-88) -- then Adagrad and both counts reset.
//  * dense items: one 16-lane group per item row (at the bench batch 99 % of
//    the items are duplicated): its counts and offsets, then every row it
//    sums, in one round of independent loads -- no owner detection chain;
//  * wave blocks: 64 candidates per wave -- every user row (dense users:
//    one coalesced count load per wave), or the batch's user / item
//    occurrences (an owner is a rank-0 occurrence with count >= 2; for items
//    the rank-0 positive when the item has positives in the batch, from the
//    immutable offP, else the rank-0 negative) -- ballot-compacted and taken
//    by the wave's four groups four at a time (no LDS, no barrier).
// ---------------------------------------------------------------------------
template <int EPL, bool FX>
__device__ __forceinline__ void apply_ps_item_block(const ApplyArgs& a, int block) {
    const int grp = threadIdx.x >> 4, gl = threadIdx.x & (kGL - 1);
    const int64_t r = a.item_r0 + (int64_t)block * kGroupsPerBlock + grp;
    if (r >= a.item_r1) return;
    const int2 o0 = a.offPN[r], o1 = a.offPN[r + 1];
    const int cp = o1.x - o0.x, cn = o1.y - o0.y;
    if (cn + cp < 2) return;   // untouched, or seen once (applied by the gradient launch)
    apply_item_ps<EPL, FX>(a, r, gl, cn, cp, o0.x, o0.y);
}

template <int EPL, bool FX>
__device__ __forceinline__ void apply_ps_wave(const ApplyArgs& a, int64_t wave) {
    const int lane = lane_id(), gw = lane >> 4, gl = lane & (kGL - 1);
    const int64_t nUw = !a.count_users ? 0 : a.dense_users ? a.n_users : a.nU;
    const int64_t nVw = (a.count_items && !a.dense_items) ? a.nV : 0;
    const int64_t q = wave * kWave + lane;
    int row = -1, isU = 0, c = 0;
    if (q < nUw) {
        if (a.dense_users) {
            c = a.cntU[q];
            if (c >= 2) row = (int)q;
        } else {
            const int rk = a.rankU[q], r = a.occU[q];
            if (rk == 0 && r >= 0) {
                c = a.cntU[r];
                if (c >= 2) row = r;
            }
        }
        isU = 1;
    } else if (q < nUw + nVw) {
        const int64_t k = q - nUw;
        const int rk = a.rankV[k], r = a.occV[k];
        if (rk == 0) {
            // the rank-0 positive owns an item with positives in the batch
            // (offP[r+1] - offP[r] > 0, immutable during the launch), else the
            // rank-0 negative
            const int2 o0 = a.offPN[r], o1 = a.offPN[r + 1];
            if ((k < a.nPos) == (o1.x > o0.x)) {
                c = (o1.x - o0.x) + (o1.y - o0.y);
                if (c >= 2) row = r;
            }
        }
    }
    unsigned long long m = __ballot(row >= 0);
    while (m != 0ull) {   // wave-uniform: four owners per round, one per group
        unsigned long long mm = m;
        for (int k = 0; k < gw; ++k) mm &= mm - 1ull;
        const int src = mm != 0ull ? __ffsll((long long)mm) - 1 : 0;
        const bool have = mm != 0ull;
        for (int k = 0; k < 4; ++k) m &= m - 1ull;
        const int rr = __shfl(row, src, kWave);
        const int ru = __shfl(isU, src, kWave);
        const int cc = __shfl(c, src, kWave);
        if (!have) continue;   // group-uniform
        if (ru) {
            apply_row<EPL, false, FX>(a, rr, true, cc, gl);
        } else {
            const int2 o0 = a.offPN[rr], o1 = a.offPN[rr + 1];
            apply_item_ps<EPL, FX>(a, rr, gl, o1.y - o0.y, o1.x - o0.x, o0.x, o0.y);
        }
    }
}

// the same dense item blocks outside pos_sort (slot rows or item records in
// per-row slot ranges, round 3): one 16-lane group per item row reads the
// row's count -- 16 consecutive rows' counts per block, one coalesced read --
// and applies a duplicated row (apply_row); no owner detection among the
// batch's item occurrences
template <int EPL>
__device__ __forceinline__ void apply_rows_item_block(const ApplyArgs& a, int block) {
    const int grp = threadIdx.x >> 4, gl = threadIdx.x & (kGL - 1);
    const int64_t r = a.item_r0 + (int64_t)block * kGroupsPerBlock + grp;
    if (r >= a.item_r1) return;
    const int c = a.cntV[r];
    if (c < 2) return;   // untouched, or seen once (applied by the gradient launch)
    apply_row<EPL>(a, r, false, c, gl);
}

// grid: [0, nbI) dense item blocks, [nbI, nbI + nbW) wave blocks, then (with
// DRAW) the draw + count blocks of the next step (other buffer set).  PS:
// pos_sort's item rows (offPN), else apply_rows_item_block
// The draw blocks are interleaved with the apply blocks (minor_block,
// round 4): the apply is bandwidth-bound (~4.9 TB/s), the draw latency-bound
// (~1 TB/s), and with the draw after every apply block the two overlapped
// for only ~16 us of a 187 us launch at cfg2 (apply 84 us and draw 119 us
// as separate launches).  -DCF_APPLY_DRAW_TAIL=1: the old order.
#ifndef CF_APPLY_DRAW_TAIL
#define CF_APPLY_DRAW_TAIL 0
#endif
#ifndef CF_APPLY_DRAW_SKEW
// 1: the draw blocks front-loaded (minor_block_front): cfg2 apply + draw 141
// -> 163 us, B = 65,536 0.0699 -> 0.0783 ms/step (same box, r06k), slower;
// 2: back-loaded, 155 vs 140 us (r06k2), slower too; 0: evenly interleaved
#define CF_APPLY_DRAW_SKEW 0
#endif
// minimum waves per SIMD the pos_sort apply is built for: 7 (72 VGPRs, 12-B
// spill) measured even-to-slower at cfg2 (round 4, profiles/r04/ab/ab_r04w_occupancy.txt)
#ifndef CF_APPLY_MIN_WAVES
#define CF_APPLY_MIN_WAVES 1
#endif
template <int EPL, bool DRAW, bool PS = true, bool FX = false, bool FULL = false>
__global__ __launch_bounds__(kBlock, CF_APPLY_MIN_WAVES) void apply_ps_kernel(ApplyArgs p, StepArgs nx, int nbI, int nbW) {
    // FULL: full rows (d == 16 EPL), the `e < d` guards fold away (grad_sort_kernel)
    if constexpr (FULL) __builtin_assume(p.d == kGL * EPL);
    int b = blockIdx.x;
    if (blockIdx.x == 0 && p.loss_acc != nullptr) fold_loss<kBlock>(p);
    // the compact GU64 rows of this batch are handed out again by the next psort
    if (FX && blockIdx.x == 0 && threadIdx.x == 0 && p.hot_n != nullptr) *p.hot_n = 0;
    if constexpr (DRAW && !CF_APPLY_DRAW_TAIL) {
        int idx;
        const int nmin = (int)gridDim.x - nbI - nbW;
        if (CF_APPLY_DRAW_SKEW == 1   ? minor_block_front<false>(blockIdx.x, nbI + nbW, nmin, idx)
            : CF_APPLY_DRAW_SKEW == 2 ? minor_block_front<true>(blockIdx.x, nbI + nbW, nmin, idx)
                                      : minor_block(blockIdx.x, nbI + nbW, nmin, idx)) {
            prep_any<BPR>(nx, idx);
            return;
        }
        b = idx;
    }
    if (b < nbI) {
        if constexpr (PS)
            apply_ps_item_block<EPL, FX>(p, b);
        else
            apply_rows_item_block<EPL>(p, b);
    } else if (b < nbI + nbW) {
        apply_ps_wave<EPL, FX>(p, (int64_t)(b - nbI) * kWavesPerBlock + (threadIdx.x >> 6));
    } else if constexpr (DRAW) {
        prep_any<BPR>(nx, b - nbI - nbW);
    }
}

// Deterministic mode: one block per 64-position tile of the sorted occurrence
// list.  A tile whose first and last positions hold the same row lies inside
// that row: its 16 groups sum four slots each (rows, or item records over the
// stash), group 0 adds the 16 partials in group order -- a fixed tree, so the
// row's sum stays bitwise reproducible -- and stores the tile's sum.
template <int EPL>
__global__ __launch_bounds__(kBlock) void det_hot_kernel(HotArgs h) {
    __shared__ float s_p[kGroupsPerBlock][kGL * EPL];
    __shared__ float s_b[kGroupsPerBlock];
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    const int64_t ntiles = h.n / kDetTile;
    for (int64_t q = blockIdx.x; q < ntiles; q += gridDim.x) {
        const int64_t p0 = q * kDetTile;
        const int32_t k0 = h.skeys[p0];
        if (k0 != h.skeys[p0 + kDetTile - 1]) continue;   // block-uniform
        const bool isU = k0 < h.n_users;
        float g[EPL], t[4][EPL];
        float bs = 0.f;
#pragma unroll
        for (int s = 0; s < EPL; ++s) g[s] = 0.f;
        constexpr int PER = kDetTile / kGroupsPerBlock;   // 4
        const int64_t pos = p0 + grp * PER;
        if (isU) {
#pragma unroll
            for (int k = 0; k < PER; ++k) gload<EPL>(h.slotU, pos + k, h.d, gl, t[k]);
#pragma unroll
            for (int k = 0; k < PER; ++k)
#pragma unroll
                for (int s = 0; s < EPL; ++s) g[s] += t[k][s];
        } else if (h.recV != nullptr) {
            int4 rc[PER];
#pragma unroll
            for (int k = 0; k < PER; ++k) rc[k] = h.recV[pos + k - h.nU];
#pragma unroll
            for (int k = 0; k < PER; ++k) gload<EPL>(rc[k].w ? h.stashB : h.stashU, rc[k].x, h.d, gl, t[k]);
#pragma unroll
            for (int k = 0; k < PER; ++k) {
                const float al = __int_as_float(rc[k].y);
#pragma unroll
                for (int s = 0; s < EPL; ++s) g[s] = fmaf(al, t[k][s], g[s]);
                bs += __int_as_float(rc[k].z);
            }
        } else {
#pragma unroll
            for (int k = 0; k < PER; ++k) gload<EPL>(h.slotV, pos + k - h.nU, h.d, gl, t[k]);
#pragma unroll
            for (int k = 0; k < PER; ++k)
#pragma unroll
                for (int s = 0; s < EPL; ++s) g[s] += t[k][s];
        }
#pragma unroll
        for (int s = 0; s < EPL; ++s) s_p[grp][gl * EPL + s] = g[s];
        if (gl == 0) s_b[grp] = bs;
        __syncthreads();
        if (grp == 0) {
#pragma unroll
            for (int s = 0; s < EPL; ++s) g[s] = s_p[0][gl * EPL + s];
            bs = s_b[0];
            for (int k = 1; k < kGroupsPerBlock; ++k) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) g[s] += s_p[k][gl * EPL + s];
                bs += s_b[k];
            }
            gstore<EPL>(h.P, q, h.d, gl, g);
            if (gl == 0) h.Pb[q] = bs;
        }
        __syncthreads();   // s_p reused by the next tile
    }
}


#ifndef CF_APPLY_DETECT_WAVES
#define CF_APPLY_DETECT_WAVES 1   // 4 measured slower: ~46 owners per block, ~3 per group in series
#endif
// waves of an apply block that find owners (kApplyChunk work items each)
constexpr int kApplyDetectWaves = CF_APPLY_DETECT_WAVES;
#ifndef CF_APPLY_CHUNK
// work items per detecting wave (<= 64).  A/B at cfg2: 64 best; 32 and 16
// double / quadruple the apply blocks and delay the fused draw (34 -> 42 / 50
// us); one-wave apply blocks (CF_APPLY_WAVE_BLOCKS) serialise ~3 owners per
// group (standalone apply 24 -> 45 us)
#define CF_APPLY_CHUNK 64
#endif
constexpr int kApplyChunk = CF_APPLY_CHUNK;

// BS = workgroup size (256, or 64 for one-wave apply blocks)
template <int EPL, int BS = kBlock, bool HOT = false>
__device__ __forceinline__ void apply_body(const ApplyArgs& a, int block, int nblocks) {
    constexpr int NWV = BS / kWave, NGR = BS / kGL;
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const int gl = lane & (kGL - 1);
    if (block == 0 && a.loss_acc != nullptr) fold_loss<BS>(a);
    // a block takes kApplyDetectWaves x 64 work items at a time: those waves
    // find their owners (~18 % of the occurrences at cfg2), then the block's
    // 16 groups apply them round-robin
    constexpr int NW = kApplyDetectWaves < NWV ? kApplyDetectWaves : NWV;
    __shared__ unsigned long long s_mask[NW];
    __shared__ int64_t s_row[NW * kWave];
    __shared__ int s_isU[NW * kWave];
    __shared__ int s_cnt[NW * kWave];   // the owner's count, read once in the check
    const int64_t nU = a.count_users ? a.nU : 0, nV = a.count_items ? a.nV : 0;
    const int64_t total = nU + nV + a.nS;
    const int group = threadIdx.x >> 4;
    constexpr int64_t chunk = (int64_t)NW * kApplyChunk;
    for (int64_t base = (int64_t)block * chunk; base < total; base += (int64_t)nblocks * chunk) {
        if (wv < NW) {
            const int64_t q = lane < kApplyChunk ? base + wv * kApplyChunk + lane : total;
            int64_t row = -1;
            int isU = 0, c = 0;
            if (q < nU) {
                if (a.rankU[q] == 0) {
                    const int32_t r = a.occU[q];
                    c = r >= 0 ? a.cntU[r] : 0;
                    if (c >= 2) {
                        row = r;
                        isU = 1;
                    }
                }
            } else if (q < nU + nV) {
                const int64_t k = q - nU;
                if (a.rankV[k] == 0) {
                    const int32_t r = a.occV[k];
                    c = a.cntV[r];
                    if (c >= 2) row = r;
                }
            } else if (q < total) {
                const int64_t k = q - nU - nV;
                if (a.served_own[k]) {
                    row = (int64_t)a.served_ids[k] - a.shard_u0;
                    isU = 1;
                    c = a.cntU[row];
                }
            }
            const unsigned long long m = __ballot(row >= 0);
            s_row[wv * kWave + lane] = row;
            s_isU[wv * kWave + lane] = isU;
            s_cnt[wv * kWave + lane] = c;
            if (lane == 0) s_mask[wv] = m;
        }
        __syncthreads();
        // owners in (wave, lane) order; group g applies owners g, g + 16, ...
        // -- the four groups of a wave take four different owners at once
        for (int t = group;; t += NGR) {
            int rem = t, src = -1;
            for (int w = 0; w < NW; ++w) {
                unsigned long long m = s_mask[w];
                const int c = __popcll(m);
                if (rem < c) {
                    for (int q = 0; q < rem; ++q) m &= m - 1ull;
                    src = w * kWave + __ffsll((long long)m) - 1;
                    break;
                }
                rem -= c;
            }
            if (src < 0) break;  // group-uniform
            apply_row<EPL, HOT>(a, s_row[src], s_isU[src] != 0, s_cnt[src], gl);
        }
        __syncthreads();  // s_* reused by the next chunk
    }
}

template <int EPL, bool HOT>
__global__ __launch_bounds__(kBlock) void apply_kernel(ApplyArgs a) {
    apply_body<EPL, kBlock, HOT>(a, blockIdx.x, gridDim.x);
}

// one-wave apply blocks: the detecting wave's own four groups apply its owners
template <int EPL>
__global__ __launch_bounds__(kWave) void apply_wave_kernel(ApplyArgs a) {
    apply_body<EPL, kWave>(a, blockIdx.x, gridDim.x);
}

// horizontal fusion on the device-sampler path: apply of step s (blocks
// [0, napply)) beside the draw + count of step s+1 (the rest) -- independent
// work (other buffer set), one launch instead of two
template <int EPL, int MODEL, bool HOT>
#ifndef CF_APPLY_PREP_ORDER
#define CF_APPLY_PREP_ORDER 0  // 0: apply blocks first, 1: draw blocks first, 2: interleaved
#endif
__global__ __launch_bounds__(kBlock) void apply_prep_kernel(ApplyArgs p, StepArgs a, int napply) {
#if CF_APPLY_PREP_ORDER != 0
    const int nprep = (int)gridDim.x - napply;
#endif
#if CF_APPLY_PREP_ORDER == 2
    int idx;
    if (minor_block(blockIdx.x, napply, nprep, idx))
        prep_any<MODEL>(a, idx);
    else
        apply_body<EPL, kBlock, HOT>(p, idx, napply);
#elif CF_APPLY_PREP_ORDER == 1
    if ((int)blockIdx.x < nprep)
        prep_any<MODEL>(a, blockIdx.x);
    else
        apply_body<EPL, kBlock, HOT>(p, blockIdx.x - nprep, napply);
#else
    if ((int)blockIdx.x < napply)
        apply_body<EPL, kBlock, HOT>(p, blockIdx.x, napply);
    else
        prep_any<MODEL>(a, blockIdx.x - napply);
#endif
}

// ---------------------------------------------------------------------------
// dense item apply (multi-rank: after the all-reduce every replica applies the
// identical update; a row whose summed gradient is all-zero is an exact no-op
// of SparseApplyAdagrad, so it is skipped)
// ---------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(kBlock) void apply_dense_kernel(DenseArgs a) {
    const int gl = threadIdx.x & (kGL - 1);
    const int64_t g0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
    const int64_t ng = ((int64_t)gridDim.x * kBlock) >> 4;
    for (int64_t r = g0; r < a.n_rows; r += ng) {
        float g[EPL];
        gload<EPL>(a.G, r, a.d, gl, g);
        uint32_t nz = 0;
#pragma unroll
        for (int s = 0; s < EPL; ++s) nz |= (g[s] != 0.f) ? 1u : 0u;
        if (gor(nz) == 0u) continue;  // group-uniform
        float x[EPL];
        gload<EPL>(a.X, r, a.d, gl, x);
        if (a.zero_g) row_zero<EPL>(a.G + r * (int64_t)a.d, a.d, gl);
        gapply<EPL>(a.X, a.A, r, a.d, gl, x, g, a.lr, a.clip != 0, a.clip_norm);
    }
    if (a.b != nullptr) {
        const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        const int64_t nt = (int64_t)gridDim.x * kBlock;
        for (int64_t r = t0; r < a.n_rows; r += nt) {
            const float g = a.Gb[r];
            if (g != 0.f) {
                const float acc = fmaf(g, g, a.Ab[r]);
                a.Ab[r] = acc;
                a.b[r] -= adagrad_delta(a.lr, g, acc);
                if (a.zero_g) a.Gb[r] = 0.f;
            }
        }
    }
}

// the rows of the dense item gradient a batch touched, re-zeroed after the
// collective that consumed them (cheaper than a memset when the batch touches
// fewer rows than the table has)
template <int EPL>
__global__ __launch_bounds__(kBlock) void zero_rows_kernel(const int32_t* __restrict__ occ, int64_t n,
                                                           float* __restrict__ G, float* __restrict__ Gb,
                                                           int d) {
    const int gl = threadIdx.x & (kGL - 1);
    const int64_t g0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
    const int64_t ng = ((int64_t)gridDim.x * kBlock) >> 4;
    for (int64_t q = g0; q < n; q += ng) {
        const int32_t r = occ[q];
        row_zero<EPL>(G + (int64_t)r * d, d, gl);
        if (Gb != nullptr && gl == 0) Gb[r] = 0.f;
    }
}

template <int EPL>
__global__ __launch_bounds__(kBlock) void clip_full_kernel(float* __restrict__ X, int64_t n_rows,
                                                           int d, float c) {
    const int gl = threadIdx.x & (kGL - 1);
    const int64_t g0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
    const int64_t ng = ((int64_t)gridDim.x * kBlock) >> 4;
    for (int64_t r = g0; r < n_rows; r += ng) {
        float x[EPL];
        gload<EPL>(X, r, d, gl, x);
        const float n = sqrtf(gdot<EPL>(x, x));
        const float den = fmaxf(n, c);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * c) / den;
        row_st<EPL>(X + r * (int64_t)d, d, gl, x);
    }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static int epl_for(int d) {
    const int e = (d + kGL - 1) / kGL;
    return e <= 1 ? 1 : e <= 2 ? 2 : e <= 4 ? 4 : e <= 8 ? 8 : 16;
}

#ifndef CF_FAST_PAIRS_W1
#define CF_FAST_PAIRS_W1 1  // cfg2 grad: P=1 44.2 us, P=2 49.8, P=3 55.6, P=4 61.9 (occupancy wins)
#endif
#ifndef CF_FAST_PAIRS_W5
#define CF_FAST_PAIRS_W5 1
#endif
// GBPR at d <= 64 (EPL <= 4): two pairs per 16-lane group keep more rows of
// the 10M-user / 1M-item tables in flight (cfg4 grad 164.9 -> 157.6 us); at
// d = 128 the second pair's registers cost occupancy (cfg5 AMF 148 -> 253 us)
#ifndef CF_FAST_PAIRS_GBPR_W5
#define CF_FAST_PAIRS_GBPR_W5 2
#endif

#ifndef CF_GRAD_LDS
#define CF_GRAD_LDS 1   // 0: auto never takes grad_lds_kernel (grad_path 3 still does)
#endif

#ifndef CF_GRAD_LDS_GBPR
#define CF_GRAD_LDS_GBPR 1   // 0: auto keeps GBPR (cfg4) on the phased kernel (grad_path 3 still takes it)
#endif
// the LDS-staged W = 5 kernel (grad_lds_kernel): grad_path 3, or auto where
// it applies -- BPR / AMF / CML at d = 128, GBPR (G = 1) at d = 64; one pair
// per 16-lane group, 16 per block
static bool lds_path(const StepArgs& a) {
    if (a.apr) return false;   // AMF apr: the generic kernel (apr_pair)
    const bool want = a.grad_path == 3 || (a.grad_path == 0 && CF_GRAD_LDS);
    if (!want || a.W != 5 || a.srec != nullptr) return false;
    if (a.model == BPR || a.model == AMF || a.model == CML) return a.d == 128;
    if (a.model == GBPR) return a.d == 64 && a.G == 1 && (a.grad_path == 3 || CF_GRAD_LDS_GBPR);
    return false;
}

// which grad kernel a step takes (see launch_grad_m): 1 = W=1 fast, 5 = W=5
// fast (or the LDS-staged kernel), 0 = generic
static int fast_w(const StepArgs& a) {
    if (a.apr) return 0;   // AMF apr: the generic kernel (apr_pair)
    if (lds_path(a)) return 5;
    // CML at W = 5 keeps five distance rows and the clip live per pair: the
    // generic kernel measured faster than the phased one there (cfg3: 160 vs
    // 184 us), so auto (grad_path 0) leaves it on the generic kernel unless
    // the LDS-staged kernel applies; 2 forces the phased kernel
    const bool ok = a.grad_path != 1 && epl_for(a.d) <= 8 && (a.model != GBPR || a.G == 1) &&
                    !(a.grad_path == 0 && a.model == CML && a.W == 5);
    return ok && (a.W == 1 || a.W == 5) ? a.W : 0;
}

#ifndef CF_GRAD_WAVE_BLOCKS
// 1: fast path without draw blocks in one-wave workgroups (measured no faster
// at cfg2: 43.9 vs 44.2 us), 0: 256-lane workgroups
#define CF_GRAD_WAVE_BLOCKS 0
#endif

static int prep_blocks(const StepArgs* nx) {
    if (!nx || nx->B <= 0) return 0;
    const int ppb = prep_pairs_per_block(*nx);
    return (nx->B + ppb - 1) / ppb;
}

template <int MODEL, int WT, bool DRAW>
static hipError_t launch_grad_w_d(const StepArgs& a, const StepArgs& n, int ng, int np, hipStream_t s) {
    const dim3 grid(ng + np), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((grad_kernel<MODEL, 1, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 2: hipLaunchKernelGGL((grad_kernel<MODEL, 2, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 4: hipLaunchKernelGGL((grad_kernel<MODEL, 4, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 8: hipLaunchKernelGGL((grad_kernel<MODEL, 8, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        default: hipLaunchKernelGGL((grad_kernel<MODEL, 16, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
    }
    return hipGetLastError();
}

template <int MODEL, int WT>
static hipError_t launch_grad_w(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    const int ng = (a.B + kPairsPerBlock - 1) / kPairsPerBlock, np = prep_blocks(nx);
    const StepArgs n = nx ? *nx : a;
    return np > 0 ? launch_grad_w_d<MODEL, WT, true>(a, n, ng, np, s)
                  : launch_grad_w_d<MODEL, WT, false>(a, n, ng, 0, s);
}

// grad_sort_kernel by row width; FX: the deterministic fixed-point form;
// DRAW: with the next step's draw blocks (pipeline 3)
template <int MODEL, int WT, bool FX, bool DRAW>
static hipError_t launch_sort_e(const StepArgs& a, const StepArgs& n, int ng, int np, dim3 grid, bool full,
                                hipStream_t s) {
    const dim3 block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((grad_sort_kernel<MODEL, 1, WT, FX, false, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 2: hipLaunchKernelGGL((grad_sort_kernel<MODEL, 2, WT, FX, false, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 4:
            if (full) hipLaunchKernelGGL((grad_sort_kernel<MODEL, 4, WT, FX, true, DRAW>), grid, block, 0, s, a, n, ng, np);
            else hipLaunchKernelGGL((grad_sort_kernel<MODEL, 4, WT, FX, false, DRAW>), grid, block, 0, s, a, n, ng, np);
            break;
        default:
            if (full && !FX) hipLaunchKernelGGL((grad_sort_kernel<MODEL, 8, WT, FX, true, DRAW>), grid, block, 0, s, a, n, ng, np);
            else hipLaunchKernelGGL((grad_sort_kernel<MODEL, 8, WT, FX, false, DRAW>), grid, block, 0, s, a, n, ng, np);
            break;
    }
    return hipGetLastError();
}

template <int MODEL, int WT, int P>
static hipError_t launch_grad_fast(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    if (CF_GRAD_WAVE_BLOCKS && prep_blocks(nx) == 0) {
        // the grid must match grad_blocks(): P * 4 pairs per one-wave block
        constexpr int gpb = kWave / kGL;
        const dim3 grid((a.B + P * gpb - 1) / (P * gpb)), block(kWave);
        switch (epl_for(a.d)) {
            case 1: hipLaunchKernelGGL((grad_fast_wave_kernel<MODEL, 1, WT, P>), grid, block, 0, s, a); break;
            case 2: hipLaunchKernelGGL((grad_fast_wave_kernel<MODEL, 2, WT, P>), grid, block, 0, s, a); break;
            case 4: hipLaunchKernelGGL((grad_fast_wave_kernel<MODEL, 4, WT, P>), grid, block, 0, s, a); break;
            default: hipLaunchKernelGGL((grad_fast_wave_kernel<MODEL, 8, WT, P>), grid, block, 0, s, a); break;
        }
        return hipGetLastError();
    }
    // the grid must match grad_blocks(): P * kGroupsPerBlock pairs per block
    const int ng = (a.B + P * kGroupsPerBlock - 1) / (P * kGroupsPerBlock), np = prep_blocks(nx);
    const StepArgs n = nx ? *nx : a;
    const dim3 grid(ng + np), block(kBlock);
    if constexpr (MODEL != GBPR && P == 1) {
        if (a.srec != nullptr) {   // pos_sort; with nx (pipeline 3) the next draw rides along
            const int sg = (a.B + CF_SORT_TILES * kPsortPPB - 1) / (CF_SORT_TILES * kPsortPPB);
            const dim3 sgrid(sg + np);
            const bool full = CF_ASSUME_FULL_ROWS && a.d == kGL * epl_for(a.d);
            if (np > 0)
                return a.det_fx ? launch_sort_e<MODEL, WT, true, true>(a, n, sg, np, sgrid, full, s)
                                : launch_sort_e<MODEL, WT, false, true>(a, n, sg, np, sgrid, full, s);
            return a.det_fx ? launch_sort_e<MODEL, WT, true, false>(a, n, sg, 0, sgrid, full, s)
                            : launch_sort_e<MODEL, WT, false, false>(a, n, sg, 0, sgrid, full, s);
        }
    }
    if (a.srec != nullptr) return hipErrorInvalidValue;
    if (np > 0) {
        switch (epl_for(a.d)) {
            case 1: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 1, WT, P, true>), grid, block, 0, s, a, n, ng, np); break;
            case 2: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 2, WT, P, true>), grid, block, 0, s, a, n, ng, np); break;
            case 4: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 4, WT, P, true>), grid, block, 0, s, a, n, ng, np); break;
            default: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 8, WT, P, true>), grid, block, 0, s, a, n, ng, np); break;
        }
    } else {
        const bool full = CF_ASSUME_FULL_FAST && a.d == kGL * epl_for(a.d);
        switch (epl_for(a.d)) {
            case 1: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 1, WT, P, false>), grid, block, 0, s, a, n, ng, 0); break;
            case 2: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 2, WT, P, false>), grid, block, 0, s, a, n, ng, 0); break;
            case 4:
                if (full) hipLaunchKernelGGL((grad_fast_kernel<MODEL, 4, WT, P, false, false, true>), grid, block, 0, s, a, n, ng, 0);
                else hipLaunchKernelGGL((grad_fast_kernel<MODEL, 4, WT, P, false>), grid, block, 0, s, a, n, ng, 0);
                break;
            default: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 8, WT, P, false>), grid, block, 0, s, a, n, ng, 0); break;
        }
    }
    return hipGetLastError();
}

// W = 1 (BPRMF driver) and W = 5 (AMF / CML / GBPR drivers) with G <= 1 and
// d <= 128 take the phased fast path; anything else the generic kernel
// tuple ranking: prefetched tuples of width 4 (CPLR, W = 2) or 5 (PRIGP, W = 3)
static hipError_t launch_grad_plr(const StepArgs& a, hipStream_t s) {
    if (a.W == 2) return launch_grad_w<PLR, 2>(a, nullptr, s);
    if (a.W == 3) return launch_grad_w<PLR, 3>(a, nullptr, s);
    return hipErrorInvalidValue;
}

template <int MODEL>
static hipError_t launch_grad_m(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    const int e = epl_for(a.d);
    if constexpr (MODEL == BPR || MODEL == AMF || MODEL == CML || MODEL == GBPR) {
        // a fused draw (pipeline 2) takes the phased kernel (grad_blocks with
        // the draw counts its grid)
        if (lds_path(a) && prep_blocks(nx) == 0) {
            const dim3 grid((a.B + kGroupsPerBlock - 1) / kGroupsPerBlock), block(kBlock);
            if constexpr (MODEL == GBPR)
                hipLaunchKernelGGL((grad_lds_kernel<GBPR, 4, 5>), grid, block, 0, s, a);
            else
                hipLaunchKernelGGL((grad_lds_kernel<MODEL, 8, 5>), grid, block, 0, s, a);
            return hipGetLastError();
        }
    }
    const int fw = fast_w(a);
    if (fw == 1) return launch_grad_fast<MODEL, 1, CF_FAST_PAIRS_W1>(a, nx, s);
    if (fw == 5 && MODEL == GBPR && e <= 4) return launch_grad_fast<MODEL, 5, CF_FAST_PAIRS_GBPR_W5>(a, nx, s);
    if (fw == 5) return launch_grad_fast<MODEL, 5, CF_FAST_PAIRS_W5>(a, nx, s);
    if (a.W == 1) return launch_grad_w<MODEL, 1>(a, nx, s);
    if (a.W == 5 && e <= 8) return launch_grad_w<MODEL, 5>(a, nx, s);
    return launch_grad_w<MODEL, 0>(a, nx, s);
}

// one gradient launcher per model, each in its own translation unit
hipError_t launch_grad_bpr(const StepArgs& a, const StepArgs* nx, hipStream_t s);
hipError_t launch_grad_amf(const StepArgs& a, const StepArgs* nx, hipStream_t s);
hipError_t launch_grad_cml(const StepArgs& a, const StepArgs* nx, hipStream_t s);
hipError_t launch_grad_gbpr(const StepArgs& a, const StepArgs* nx, hipStream_t s);
hipError_t launch_grad_plr_t(const StepArgs& a, hipStream_t s);

}  // namespace cfk
