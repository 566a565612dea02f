// cf_kernels.hip -- the training hot path for gfx950 (MI355X / CDNA4).
//
// One optimizer step of BPRMF / GBPRMF / CML / AMF is three launches; the
// unit of parallelism is a 16-lane group per (u,i) pair / per row, four per
// wave, so a wave keeps four pairs' gathers in flight.
//
//  prep_kernel   draw the batch on device -- epoch bijection over the nnz
//                pairs, W negatives whose membership in Pos(u) the 16 lanes
//                test cooperatively against the user's sorted CSR row
//                (one coalesced pass, group-OR of hit masks, redraw only the
//                rejected ones), G group users from the item's CSC column --
//                or take a host-fed batch; then count every touched row's
//                occurrences in the batch (one no-return atomicAdd each).
//  grad_kernel   gather U[u], V[i], V[j] (+U[g], b) rows, group-reduce the
//                dots / distances, evaluate the loss and dL/dx, form every
//                per-occurrence gradient row.  A row that occurs ONCE in the
//                batch is updated right here with SparseApplyAdagrad
//                (acc += g^2; w -= lr*g/sqrt(acc); CML: clip) -- its
//                pre-update value is already in registers.  A row that
//                occurs several times scatter-adds into a dense fp32
//                accumulator (float atomics, 64-B segments), so duplicates
//                SUM before the update: TF1's _deduplicate_indexed_slices
//                (SURVEY 0.4).
//  apply_kernel  scans the count arrays (int4 per lane) and applies the
//                summed gradient of every duplicated row (count > 1), then
//                zeroes its accumulator row and count.
//
// Reference semantics: src/models/pl/models/bprmf.py:52-88,
// gbprmf.py:58-106, cml.py:55-129, src/models/others/models/amf.py:66-162;
// samplers src/samplers/sampler_ranking.py:22-37, sampler_gbpr.py:23-43.
#include "cf_kernels.h"
#include "cf_device.h"

namespace cfk {

// ---------------------------------------------------------------------------
// 16-lane group helpers: element e of a row lives in lane (e % 16), slot
// e / 16, so one load instruction reads 64 contiguous bytes of four rows.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float gsum(float v) {
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 1, 64);
    return v;
}

__device__ __forceinline__ uint32_t gor(uint32_t v) {
    v |= (uint32_t)__shfl_xor((int)v, 8, 64);
    v |= (uint32_t)__shfl_xor((int)v, 4, 64);
    v |= (uint32_t)__shfl_xor((int)v, 2, 64);
    v |= (uint32_t)__shfl_xor((int)v, 1, 64);
    return v;
}

template <int EPL>
__device__ __forceinline__ void gload(const float* __restrict__ X, int64_t r, int d, int gl,
                                      float (&x)[EPL]) {
    const float* row = X + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        x[s] = (e < d) ? row[e] : 0.f;
    }
}

template <int EPL>
__device__ __forceinline__ void gatomic(float* __restrict__ G, int64_t r, int d, int gl,
                                        const float (&g)[EPL]) {
    float* row = G + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        if (e < d) unsafeAtomicAdd(row + e, g[s]);
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
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        acc[s] = (e < d) ? ar[e] : 1.f;
    }
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        acc[s] = fmaf(g[s], g[s], acc[s]);
        x[s] = x0[s] - (lr * g[s]) / sqrtf(acc[s]);
    }
    if (clip) {
        const float n = sqrtf(gdot<EPL>(x, x));
        const float den = fmaxf(n, c);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * c) / den;
    }
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        if (e < d) {
            xr[e] = x[s];
            ar[e] = acc[s];
        }
    }
}

// row r of X: singleton -> apply now; duplicated -> accumulate
template <int EPL>
__device__ __forceinline__ void gfinish(float* __restrict__ X, float* __restrict__ A,
                                        float* __restrict__ G, int32_t* __restrict__ cnt,
                                        int64_t r, int count, int d, int gl,
                                        const float (&x0)[EPL], const float (&g)[EPL],
                                        const StepArgs& a) {
    if (count == 1) {
        gapply<EPL>(X, A, r, d, gl, x0, g, a.lr, a.clip != 0, a.clip_norm);
        if (gl == 0) cnt[r] = 0;
    } else {
        gatomic<EPL>(G, r, d, gl, g);
    }
}

__device__ __forceinline__ void bias_finish(const StepArgs& a, int64_t r, int count, float g) {
    // GBPR item bias: one scalar row
    if (count == 1) {
        const float acc = fmaf(g, g, a.Ab[r]);
        a.Ab[r] = acc;
        a.b[r] -= (a.lr * g) / sqrtf(acc);
    } else {
        unsafeAtomicAdd(a.Gb + r, g);
    }
}

__device__ __forceinline__ float neg_log_sigmoid(float x) {
    // literal -log(sigmoid(x)) as in bprmf.py:70 / gbprmf.py:88
    return -logf(1.f / (1.f + expf(-x)));
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
template <int MODEL>
__global__ __launch_bounds__(kBlock) void prep_kernel(StepArgs a) {
    const int gl = threadIdx.x & (kGL - 1);
    const int p = blockIdx.x * kGroupsPerBlock + (threadIdx.x >> 4);
    if (p >= a.B) return;  // whole group leaves; no block barrier below
    const int W = a.W;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const int B = a.B;
    int u, i;
    uint64_t key = 0;
    int64_t rb = 0, re = 0;
    if (a.sample) {
        const uint64_t slot = a.slot_base + (uint64_t)p;
        const uint64_t idx = permute(slot, a.perm);   // shuffled pair order (sampler_ranking.py:24)
        const int2 pr = a.pairs[idx];
        u = pr.x;
        i = pr.y;
        key = mix64(a.rng_key ^ (slot * 0xD1B54A32D192ED03ull));
        rb = a.indptr[u];
        re = a.indptr[u + 1];
    } else {
        u = a.occU[p];
        i = a.occV[p];
    }
    const int nchunk = (int)((re - rb + kGL - 1) / kGL);
    for (int w0 = 0; w0 < W; w0 += kGL) {
        const int nw = (W - w0 < kGL) ? (W - w0) : kGL;
        const int w = w0 + gl;
        int32_t j = -1;
        if (a.sample) {
            // negItems = randint(0, n_items), redrawn while j in Pos(u)
            // (sampler_ranking.py:30-36); lane w owns candidate w
            uint64_t ctr = (uint64_t)w << 32;
            if (gl < nw) j = draw_item(key, ctr++, a.n_items);
            uint32_t pending = (nw >= 32) ? 0xFFFFFFFFu : ((1u << nw) - 1u);
            for (;;) {
                uint32_t hit = 0;
                for (int c = 0; c < nchunk; ++c) {
                    const int64_t t = rb + (int64_t)c * kGL + gl;
                    const int32_t el = (t < re) ? a.indices[t] : -1;
                    for (int k = 0; k < nw; ++k) {
                        const int32_t cand = __shfl(j, k, kGL);
                        hit |= (el == cand) ? (1u << k) : 0u;
                    }
                }
                hit = gor(hit) & pending;
                if (hit == 0u) break;  // group-uniform
                if ((hit >> gl) & 1u) j = draw_item(key, ctr++, a.n_items);
                pending = hit;
            }
            if (gl < nw) a.occV[B + p * W + w] = j;
        } else if (gl < nw) {
            j = a.occV[B + p * W + w];
        }
        if (a.count_items && gl < nw) atomicAdd(&a.cntV[j], 1);
    }
    if (MODEL == GBPR && gl < G) {
        int32_t g;
        if (a.sample) {
            // group = np.random.choice(item_posUserList[i], gsize): uniform,
            // with replacement, may contain u (sampler_gbpr.py:41)
            const int64_t cb = a.indptr_t[i], ce = a.indptr_t[i + 1];
            const uint64_t h = mix64(key + ((uint64_t)(kMaxNeg + gl) << 32));
            g = a.indices_t[cb + (int64_t)uniform_below(h, (uint64_t)(ce - cb))];
            a.occU[B + p * G + gl] = g;
        } else {
            g = a.occU[B + p * G + gl];
        }
        if (a.count_users) atomicAdd(&a.cntU[g], 1);
    }
    if (gl == 0) {
        if (a.sample) {
            a.occU[p] = u;
            a.occV[p] = i;
        }
        if (a.count_users) atomicAdd(&a.cntU[u], 1);
        if (a.count_items) atomicAdd(&a.cntV[i], 1);
    }
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
    float v[N][EPL];
    __device__ __forceinline__ void prefetch(const StepArgs& a, int p, int gl) {
        if constexpr (WT > 0) {
#pragma unroll
            for (int w = 0; w < WT; ++w) j[w] = a.occV[a.B + p * WT + w];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                c[w] = a.count_items ? a.cntV[j[w]] : 0;
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
            c[0] = a.count_items ? a.cntV[j[0]] : 0;
            gload<EPL>(a.V, j[0], a.d, gl, v[0]);
            return 0;
        }
    }
};

template <int MODEL, int EPL, int WT>
__global__ __launch_bounds__(kBlock) void grad_kernel(StepArgs a) {
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
        const int p = (blockIdx.x * kPairsPerGroup + k) * kGroupsPerBlock + grp;
        if (p >= B) break;  // group-uniform
        const int u = a.occU[p];
        const int i = a.occV[p];
        NegRows<EPL, WT> J;
        J.prefetch(a, p, gl);
        const int cu = a.count_users ? a.cntU[u] : 0;
        const int ci = a.count_items ? a.cntV[i] : 0;
        float uu[EPL], vi[EPL];
        gload<EPL>(a.U, u, d, gl, uu);
        gload<EPL>(a.V, i, d, gl, vi);

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
                float c = -1.f / (1.f + expf(x));
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
                gfinish<EPL>(a.V, a.AV, a.GV, a.cntV, J.j[sl], J.c[sl], d, gl, J.v[sl], gj, a);
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += a.reg * uu[s];
                gi[s] = sc * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish<EPL>(a.U, a.AU, a.GU, a.cntU, u, cu, d, gl, uu, gu, a);
            gfinish<EPL>(a.V, a.AV, a.GV, a.cntV, i, ci, d, gl, vi, gi, a);
        } else if (MODEL == GBPR) {
            // ui = rho*mean_k<g_k,i> + (1-rho)<u,i> + b_i ; uj = <u,j> + b_j   (A.2)
            const float bi = a.b[i];
            const float ui_u = gdot<EPL>(uu, vi);
            float sg[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) sg[s] = 0.f;
            for (int k2 = 0; k2 < G; ++k2) {
                float gk[EPL];
                gload<EPL>(a.U, a.occU[B + p * G + k2], d, gl, gk);
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
                const float c = -1.f / (1.f + expf(x));
                loss_g += neg_log_sigmoid(x) + 0.5f * a.reg * bj * bj;
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(-c, J.v[sl][s], gu[s]);
                    gj[s] = -c * uu[s];  // no L2 on V[j] (gbprmf.py:59-64)
                }
                if (gl == 0) bias_finish(a, j, J.c[sl], -c + a.reg * bj);
                gfinish<EPL>(a.V, a.AV, a.GV, a.cntV, j, J.c[sl], d, gl, J.v[sl], gj, a);
            }
            const float rg = a.rho / Gf;
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += (1.f - a.rho) * sc * vi[s] + a.reg * uu[s];
                gi[s] = sc * (rg * sg[s] + (1.f - a.rho) * uu[s]) + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish<EPL>(a.U, a.AU, a.GU, a.cntU, u, cu, d, gl, uu, gu, a);
            for (int k2 = 0; k2 < G; ++k2) {
                const int g = a.occU[B + p * G + k2];
                const int cg = a.cntU[g];
                float gk[EPL], gg[EPL];
                gload<EPL>(a.U, g, d, gl, gk);
#pragma unroll
                for (int s = 0; s < EPL; ++s) gg[s] = rg * sc * vi[s] + a.reg * gk[s];
                gfinish<EPL>(a.U, a.AU, a.GU, a.cntU, g, cg, d, gl, gk, gg, a);
            }
            if (gl == 0) bias_finish(a, i, ci, sc);
            gfinish<EPL>(a.V, a.AV, a.GV, a.cntV, i, ci, d, gl, vi, gi, a);
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
                gfinish<EPL>(a.V, a.AV, a.GV, a.cntV, J.j[sl], J.c[sl], d, gl, J.v[sl], gj, a);
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
            gfinish<EPL>(a.U, a.AU, a.GU, a.cntU, u, cu, d, gl, uu, gu, a);
            gfinish<EPL>(a.V, a.AV, a.GV, a.cntV, i, ci, d, gl, vi, gi, a);
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
        a.loss_partial[blockIdx.x] = t;
    }
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
    if (want) {
        const float* row = A + r * (int64_t)d;
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const int e = s * kGL + gl;
            if (e < d) acc[s] = row[e];
        }
    }
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
        x[s] = x0[s] - (lr * g[s]) / sqrtf(acc[s]);
    }
    if (clip) {
        const float n = sqrtf(gdot<EPL>(x, x));
        const float den = fmaxf(n, c);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * c) / den;
    }
    float* xr = X + r * (int64_t)d;
    float* ar = A + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        if (e < d) {
            xr[e] = x[s];
            ar[e] = acc[s];
        }
    }
}

template <int EPL>
__device__ __forceinline__ void gfinish_pre(float* __restrict__ X, float* __restrict__ A,
                                            float* __restrict__ G, int32_t* __restrict__ cnt,
                                            int64_t r, int count, int d, int gl,
                                            const float (&x0)[EPL], const float (&acc0)[EPL],
                                            const float (&g)[EPL], const StepArgs& a) {
    if (count == 1) {
        gapply_pre<EPL>(X, A, r, d, gl, x0, acc0, g, a.lr, a.clip != 0, a.clip_norm);
        if (gl == 0) cnt[r] = 0;
    } else {
        gatomic<EPL>(G, r, d, gl, g);
    }
}

template <int MODEL, int EPL, int WT>
struct PairRows {
    static constexpr int NG = (MODEL == GBPR) ? 1 : 0;
    static constexpr int NGA = NG > 0 ? NG : 1;
    int u, i, cu, ci;
    int j[WT], cj[WT];
    int g[NGA], cg[NGA];
    float uu[EPL], vi[EPL], au[EPL], ai[EPL];
    float vj[WT][EPL], aj[WT][EPL];
    float ug[NGA][EPL], ag[NGA][EPL];
    float bi, bj[WT];

    __device__ __forceinline__ void load_idx(const StepArgs& a, int p) {
        u = a.occU[p];
        i = a.occV[p];
#pragma unroll
        for (int w = 0; w < WT; ++w) j[w] = a.occV[a.B + p * WT + w];
#pragma unroll
        for (int k = 0; k < NG; ++k) g[k] = a.occU[a.B + p + k];
    }
    __device__ __forceinline__ void load_rows(const StepArgs& a, int gl) {
        cu = a.count_users ? a.cntU[u] : 0;
        ci = a.count_items ? a.cntV[i] : 0;
#pragma unroll
        for (int w = 0; w < WT; ++w) cj[w] = a.count_items ? a.cntV[j[w]] : 0;
#pragma unroll
        for (int k = 0; k < NG; ++k) cg[k] = a.count_users ? a.cntU[g[k]] : 0;
        gload<EPL>(a.U, u, a.d, gl, uu);
        gload<EPL>(a.V, i, a.d, gl, vi);
#pragma unroll
        for (int w = 0; w < WT; ++w) gload<EPL>(a.V, j[w], a.d, gl, vj[w]);
#pragma unroll
        for (int k = 0; k < NG; ++k) gload<EPL>(a.U, g[k], a.d, gl, ug[k]);
        if (MODEL == GBPR) {
            bi = a.b[i];
#pragma unroll
            for (int w = 0; w < WT; ++w) bj[w] = a.b[j[w]];
        }
    }
    __device__ __forceinline__ void load_acc(const StepArgs& a, int gl) {
        gload_acc<EPL>(a.AU, u, a.d, gl, cu == 1, au);
        gload_acc<EPL>(a.AV, i, a.d, gl, ci == 1, ai);
#pragma unroll
        for (int w = 0; w < WT; ++w) gload_acc<EPL>(a.AV, j[w], a.d, gl, cj[w] == 1, aj[w]);
#pragma unroll
        for (int k = 0; k < NG; ++k) gload_acc<EPL>(a.AU, g[k], a.d, gl, cg[k] == 1, ag[k]);
    }

    __device__ __forceinline__ void update(const StepArgs& a, int gl, float& loss_g, float& sq) {
        const int d = a.d;
        if (MODEL == BPR || MODEL == AMF) {
            const float ui = gdot<EPL>(uu, vi);
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                const float x = ui - gdot<EPL>(uu, vj[w]);
                float c = -1.f / (1.f + expf(x));
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
                gfinish_pre<EPL>(a.V, a.AV, a.GV, a.cntV, j[w], cj[w], d, gl, vj[w], aj[w], gj, a);
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += a.reg * uu[s];
                gi[s] = sc * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.cntU, u, cu, d, gl, uu, au, gu, a);
            gfinish_pre<EPL>(a.V, a.AV, a.GV, a.cntV, i, ci, d, gl, vi, ai, gi, a);
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
                const float c = -1.f / (1.f + expf(x));
                loss_g += neg_log_sigmoid(x) + 0.5f * a.reg * bj[w] * bj[w];
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(-c, vj[w][s], gu[s]);
                    gj[s] = -c * uu[s];
                }
                if (gl == 0) bias_finish(a, j[w], cj[w], -c + a.reg * bj[w]);
                gfinish_pre<EPL>(a.V, a.AV, a.GV, a.cntV, j[w], cj[w], d, gl, vj[w], aj[w], gj, a);
            }
            const float rg = a.rho;  // rho / G with G == 1
            float gi[EPL], gg[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += (1.f - a.rho) * sc * vi[s] + a.reg * uu[s];
                gi[s] = sc * (rg * ug[0][s] + (1.f - a.rho) * uu[s]) + a.reg * vi[s];
                gg[s] = rg * sc * vi[s] + a.reg * ug[0][s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.cntU, u, cu, d, gl, uu, au, gu, a);
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.cntU, g[0], cg[0], d, gl, ug[0], ag[0], gg, a);
            if (gl == 0) bias_finish(a, i, ci, sc);
            gfinish_pre<EPL>(a.V, a.AV, a.GV, a.cntV, i, ci, d, gl, vi, ai, gi, a);
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
                gfinish_pre<EPL>(a.V, a.AV, a.GV, a.cntV, j[w], cj[w], d, gl, vj[w], aj[w], gj, a);
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
            gfinish_pre<EPL>(a.U, a.AU, a.GU, a.cntU, u, cu, d, gl, uu, au, gu, a);
            gfinish_pre<EPL>(a.V, a.AV, a.GV, a.cntV, i, ci, d, gl, vi, ai, gi, a);
        }
    }
};

template <int MODEL, int EPL, int WT, int P>
__global__ __launch_bounds__(kBlock) void grad_fast_kernel(StepArgs a) {
    __shared__ double s_loss[kGroupsPerBlock];
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    float loss_g = 0.f;
    float sq = 0.f;
    PairRows<MODEL, EPL, WT> pr[P];
    int pp[P];
    bool ok[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        pp[k] = (blockIdx.x * P + k) * kGroupsPerBlock + grp;
        ok[k] = pp[k] < a.B;
    }
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].load_idx(a, pp[k]);
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].load_rows(a, gl);
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].load_acc(a, gl);
#pragma unroll
    for (int k = 0; k < P; ++k)
        if (ok[k]) pr[k].update(a, gl, loss_g, sq);

    const float coef = (MODEL == CML) ? (a.reg_cov > 0.f ? a.reg_cov : 0.f) : a.reg;
    const float sq_g = gsum(sq);
    if (gl == 0) s_loss[grp] = (double)loss_g + 0.5 * (double)coef * (double)sq_g;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < kGroupsPerBlock; ++k) t += s_loss[k];
        a.loss_partial[blockIdx.x] = t;
    }
}

// ---------------------------------------------------------------------------
// apply the summed gradient of every duplicated row (count > 1)
// ---------------------------------------------------------------------------
template <int EPL>
__global__ __launch_bounds__(kBlock) void apply_kernel(ApplyArgs a) {
    __shared__ double s_red[kWavesPerBlock];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const int gw = lane >> 4;       // group inside the wave
    const int gl = lane & (kGL - 1);
    if (blockIdx.x == 0 && a.loss_acc != nullptr) {
        double t = 0.0;
        for (int k = threadIdx.x; k < a.n_partial; k += kBlock) t += a.loss_partial[k];
        t = wave_sum_d(t);
        if (lane == 0) s_red[wv] = t;
        __syncthreads();
        if (threadIdx.x == 0) a.loss_acc[0] += (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    }
    const bool isU = (int)blockIdx.x < a.blocksU;
    const int64_t blk = isU ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - a.blocksU;
    const int64_t n = isU ? a.n_users : a.n_items;
    int32_t* cnt = isU ? a.cntU : a.cntV;
    float* X = isU ? a.U : a.V;
    float* A = isU ? a.AU : a.AV;
    float* G = isU ? a.GU : a.GV;
    const bool bias = !isU && a.b != nullptr;

    const int rpt = isU ? 4 : 1;                   // rows per thread
    const int64_t base_row = blk * (isU ? kApplyRowsPerBlockU : kApplyRowsPerBlockV);
    const int64_t r0 = base_row + (int64_t)threadIdx.x * rpt;
    int c4[4] = {0, 0, 0, 0};
    if (rpt == 4 && r0 + 3 < n) {
        const int4 v = *reinterpret_cast<const int4*>(cnt + r0);
        c4[0] = v.x; c4[1] = v.y; c4[2] = v.z; c4[3] = v.w;
    } else {
        for (int q = 0; q < rpt; ++q) c4[q] = (r0 + q < n) ? cnt[r0 + q] : 0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q >= rpt) break;  // block-uniform
        const bool win = c4[q] > 1;
        const int64_t r_l = r0 + q;
        if (bias && win) {
            const float g = a.Gb[r_l];
            const float acc = fmaf(g, g, a.Ab[r_l]);
            a.Ab[r_l] = acc;
            a.b[r_l] -= (a.lr * g) / sqrtf(acc);
            a.Gb[r_l] = 0.f;
        }
        const unsigned long long m = __ballot(win);
        const int nwin = __popcll(m);
        for (int base = 0; base < nwin; base += 4) {  // wave-uniform
            const int my = base + gw;
            unsigned long long mm = m;
            for (int t = 0; t < my && mm; ++t) mm &= mm - 1ull;
            const int pos = (my < nwin) ? __ffsll((long long)mm) - 1 : 0;
            const int64_t r = base_row + __shfl((int)threadIdx.x * rpt + q, pos, 64);
            if (my < nwin) {  // group-uniform
                float g[EPL], x[EPL];
                gload<EPL>(G, r, a.d, gl, g);
                gload<EPL>(X, r, a.d, gl, x);
                float* gr = G + r * a.d;
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    const int e = s * kGL + gl;
                    if (e < a.d) gr[e] = 0.f;
                }
                gapply<EPL>(X, A, r, a.d, gl, x, g, a.lr, a.clip != 0, a.clip_norm);
            }
        }
        if (win) cnt[r_l] = 0;
    }
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
        float* gr = a.G + r * (int64_t)a.d;
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const int e = s * kGL + gl;
            if (e < a.d) gr[e] = 0.f;
        }
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
                a.b[r] -= (a.lr * g) / sqrtf(acc);
                a.Gb[r] = 0.f;
            }
        }
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
        float* xr = X + r * (int64_t)d;
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const int e = s * kGL + gl;
            if (e < d) xr[e] = (x[s] * c) / den;
        }
    }
}

__global__ void init_normal_kernel(float* __restrict__ X, int64_t n, float mean, float stddev,
                                   int truncated, uint64_t seed) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = t0; k < n; k += nt) {
        uint64_t ctr = 0;
        float z;
        do {
            const uint64_t h = mix64(seed ^ mix64((uint64_t)k * 0x9E3779B97F4A7C15ull + ctr++));
            const float u1 = ((uint32_t)(h >> 40) + 0.5f) * (1.f / 16777216.f);  // (0,1)
            const float u2 = ((uint32_t)(h & 0xFFFFFF)) * (1.f / 16777216.f);
            z = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
        } while (truncated && fabsf(z) > 2.f);
        X[k] = mean + stddev * z;
    }
}

__global__ void fill_kernel(float* __restrict__ X, int64_t n, float v) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = t0; k < n; k += nt) X[k] = v;
}

__global__ void build_pairs_kernel(const int64_t* __restrict__ indptr,
                                   const int32_t* __restrict__ indices, int64_t n_users,
                                   int2* __restrict__ pairs) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t u = t0; u < n_users; u += nt)
        for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k)
            pairs[k] = make_int2((int)u, indices[k]);
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static int epl_for(int d) {
    const int e = (d + kGL - 1) / kGL;
    return e <= 1 ? 1 : e <= 2 ? 2 : e <= 4 ? 4 : e <= 8 ? 8 : 16;
}

#ifndef CF_FAST_PAIRS_W1
#define CF_FAST_PAIRS_W1 2
#endif
#ifndef CF_FAST_PAIRS_W5
#define CF_FAST_PAIRS_W5 1
#endif

// which grad kernel a step takes (see launch_grad_m): 1 = W=1 fast, 5 = W=5
// fast, 0 = generic
static int fast_w(const StepArgs& a) {
    const bool ok = a.grad_path != 1 && epl_for(a.d) <= 8 && (a.model != GBPR || a.G == 1);
    return ok && (a.W == 1 || a.W == 5) ? a.W : 0;
}

int grad_blocks(const StepArgs& a) {
    const int fw = fast_w(a);
    const int B = a.B;
    const int ppb = fw == 1 ? CF_FAST_PAIRS_W1 * kGroupsPerBlock
                  : fw == 5 ? CF_FAST_PAIRS_W5 * kGroupsPerBlock : kPairsPerBlock;
    return (B + ppb - 1) / ppb;
}

int grad_blocks_max(int B) { return (B + kGroupsPerBlock - 1) / kGroupsPerBlock; }

hipError_t launch_prep(const StepArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    const int blocks = (a.B + kGroupsPerBlock - 1) / kGroupsPerBlock;
    switch (a.model) {
        case GBPR: hipLaunchKernelGGL(prep_kernel<GBPR>, dim3(blocks), dim3(kBlock), 0, s, a); break;
        default: hipLaunchKernelGGL(prep_kernel<BPR>, dim3(blocks), dim3(kBlock), 0, s, a); break;
    }
    return hipGetLastError();
}

template <int MODEL, int WT>
static hipError_t launch_grad_w(const StepArgs& a, hipStream_t s) {
    const dim3 grid((a.B + kPairsPerBlock - 1) / kPairsPerBlock), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((grad_kernel<MODEL, 1, WT>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((grad_kernel<MODEL, 2, WT>), grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL((grad_kernel<MODEL, 4, WT>), grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL((grad_kernel<MODEL, 8, WT>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((grad_kernel<MODEL, 16, WT>), grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

template <int MODEL, int WT, int P>
static hipError_t launch_grad_fast(const StepArgs& a, hipStream_t s) {
    // the grid must match grad_blocks(): P * kGroupsPerBlock pairs per block
    const int blocks = (a.B + P * kGroupsPerBlock - 1) / (P * kGroupsPerBlock);
    const dim3 grid(blocks), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 1, WT, P>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 2, WT, P>), grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 4, WT, P>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((grad_fast_kernel<MODEL, 8, WT, P>), grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

// W = 1 (BPRMF driver) and W = 5 (AMF / CML / GBPR drivers) with G <= 1 and
// d <= 128 take the phased fast path; anything else the generic kernel
template <int MODEL>
static hipError_t launch_grad_m(const StepArgs& a, hipStream_t s) {
    const int e = epl_for(a.d);
    const int fw = fast_w(a);
    if (fw == 1) return launch_grad_fast<MODEL, 1, CF_FAST_PAIRS_W1>(a, s);
    if (fw == 5) return launch_grad_fast<MODEL, 5, CF_FAST_PAIRS_W5>(a, s);
    if (a.W == 1) return launch_grad_w<MODEL, 1>(a, s);
    if (a.W == 5 && e <= 8) return launch_grad_w<MODEL, 5>(a, s);
    return launch_grad_w<MODEL, 0>(a, s);
}

hipError_t launch_grad(const StepArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    switch (a.model) {
        case BPR: return launch_grad_m<BPR>(a, s);
        case GBPR: return launch_grad_m<GBPR>(a, s);
        case CML: return launch_grad_m<CML>(a, s);
        default: return launch_grad_m<AMF>(a, s);
    }
}

hipError_t launch_apply(const ApplyArgs& a, hipStream_t s) {
    const int bV = a.apply_items ? (int)((a.n_items + kApplyRowsPerBlockV - 1) / kApplyRowsPerBlockV) : 0;
    int blocks = a.blocksU + bV;
    if (blocks == 0) blocks = 1;  // block 0 still reduces the loss
    const dim3 grid(blocks), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL(apply_kernel<1>, grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL(apply_kernel<2>, grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL(apply_kernel<4>, grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL(apply_kernel<8>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(apply_kernel<16>, grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

static int row_grid(int64_t n_rows) {
    int64_t b = (n_rows + kGroupsPerBlock - 1) / kGroupsPerBlock;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_apply_dense(const DenseArgs& a, hipStream_t s) {
    const dim3 grid(row_grid(a.n_rows)), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL(apply_dense_kernel<1>, grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL(apply_dense_kernel<2>, grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL(apply_dense_kernel<4>, grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL(apply_dense_kernel<8>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(apply_dense_kernel<16>, grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_clip_full(float* X, int64_t n_rows, int d, float c, hipStream_t s) {
    const dim3 grid(row_grid(n_rows)), block(kBlock);
    switch (epl_for(d)) {
        case 1: hipLaunchKernelGGL(clip_full_kernel<1>, grid, block, 0, s, X, n_rows, d, c); break;
        case 2: hipLaunchKernelGGL(clip_full_kernel<2>, grid, block, 0, s, X, n_rows, d, c); break;
        case 4: hipLaunchKernelGGL(clip_full_kernel<4>, grid, block, 0, s, X, n_rows, d, c); break;
        case 8: hipLaunchKernelGGL(clip_full_kernel<8>, grid, block, 0, s, X, n_rows, d, c); break;
        default: hipLaunchKernelGGL(clip_full_kernel<16>, grid, block, 0, s, X, n_rows, d, c); break;
    }
    return hipGetLastError();
}

static int grid_for(int64_t n) {
    int64_t b = (n + kBlock - 1) / kBlock;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_init_normal(float* X, int64_t n, float mean, float stddev, int truncated,
                              uint64_t seed, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(init_normal_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, X, n, mean,
                       stddev, truncated, seed);
    return hipGetLastError();
}

hipError_t launch_fill(float* X, int64_t n, float v, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, X, n, v);
    return hipGetLastError();
}

hipError_t launch_build_pairs(const int64_t* indptr, const int32_t* indices, int64_t n_users,
                              int2* pairs, hipStream_t s) {
    if (n_users <= 0) return hipSuccess;
    hipLaunchKernelGGL(build_pairs_kernel, dim3(grid_for(n_users)), dim3(kBlock), 0, s, indptr,
                       indices, n_users, pairs);
    return hipGetLastError();
}

uint64_t mix64_host(uint64_t z) { return mix64(z); }

PermKey make_perm_key(uint64_t n, uint64_t seed, uint64_t epoch) {
    PermKey p{};
    p.n = n;
    uint32_t bits = 1;
    while (bits < 63 && (1ull << bits) < n) ++bits;
    p.mask = (1ull << bits) - 1ull;
    p.shift = bits / 2 > 0 ? bits / 2 : 1;
    uint64_t h = mix64(seed ^ mix64(epoch + 0x5851F42D4C957F2Dull));
    for (int r = 0; r < 3; ++r) {
        h = mix64(h + (uint64_t)r);
        p.k[r] = h & p.mask;
        p.m[r] = (mix64(h ^ 0xA0761D6478BD642Full) | 1ull);
    }
    return p;
}

}  // namespace cfk
