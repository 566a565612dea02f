// cf_kernels.hip -- the training hot path for gfx950 (MI355X / CDNA4).
//
// One optimizer step of BPRMF / GBPRMF / CML / AMF is two launches:
//
//  step_kernel   phase A (lane = pair): draw the batch on device -- epoch
//                bijection over the nnz pairs, W negatives with rejection
//                against the user's sorted CSR row, G group users from the
//                item's CSC column -- or read a host-fed batch; claim each
//                touched row's "winner" occurrence with one atomicExch on a
//                per-row stamp (the first occurrence of a row in the batch
//                applies its Adagrad update).
//                phase B (lane = embedding dimension): gather U[u], V[i],
//                V[j] (+U[g], b) rows, wave-reduce the dots / distances,
//                evaluate the loss and dL/dx, and scatter-add every
//                per-occurrence gradient row into dense fp32 accumulators
//                (one 256-B float-atomic wave instruction per d=64 row).
//                Duplicate rows therefore SUM before the update -- the TF1
//                _deduplicate_indexed_slices semantics.
//  apply_kernel  one wave per winner row: acc += g^2; w -= lr*g/sqrt(acc)
//                (SparseApplyAdagrad), zero the accumulator row, and for
//                CML clip the updated row to clip_norm (cml.py:119-129).
//
// Reference semantics: src/models/pl/models/bprmf.py:52-88,
// gbprmf.py:58-106, cml.py:55-129, src/models/others/models/amf.py:66-162;
// samplers src/samplers/sampler_ranking.py:22-37, sampler_gbpr.py:23-43.
#include "cf_kernels.h"
#include "cf_device.h"

namespace cfk {

template <int EPL>
__device__ __forceinline__ void load_row(const float* __restrict__ X, int64_t r, int d, int lane,
                                         float (&x)[EPL]) {
    const float* row = X + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kWave + lane;
        x[s] = (e < d) ? row[e] : 0.f;
    }
}

template <int EPL>
__device__ __forceinline__ void atomic_row(float* __restrict__ G, int64_t r, int d, int lane,
                                           const float (&g)[EPL]) {
    float* row = G + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kWave + lane;
        if (e < d) unsafeAtomicAdd(row + e, g[s]);
    }
}

template <int EPL>
__device__ __forceinline__ float dot_part(const float (&x)[EPL], const float (&y)[EPL]) {
    float t = 0.f;
#pragma unroll
    for (int s = 0; s < EPL; ++s) t = fmaf(x[s], y[s], t);
    return t;
}

__device__ __forceinline__ float neg_log_sigmoid(float x) {
    // literal -log(sigmoid(x)) as in bprmf.py:70 / gbprmf.py:88
    return -logf(1.f / (1.f + expf(-x)));
}

__device__ __forceinline__ float softplus(float x) {
    // tf.nn.softplus: log(1 + exp(x)), evaluated stably
    return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
}

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// ---------------------------------------------------------------------------
// fused step
// ---------------------------------------------------------------------------
template <int MODEL, int EPL>
__global__ __launch_bounds__(kBlock) void step_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    __shared__ double s_loss[kWavesPerBlock];

    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const int W = a.W;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const int stride = 2 + W + G;  // ints per pair record in LDS
    int* sw = smem + wv * kPairsPerWave * stride;
    const int p0 = (blockIdx.x * kWavesPerBlock + wv) * kPairsPerWave;

    // ---- phase A: lane = pair ------------------------------------------------
    if (lane < kPairsPerWave) {
        const int p = p0 + lane;
        int* rec = sw + lane * stride;
        if (p < a.B) {
            int u, i;
            if (a.sample) {
                const uint64_t slot = a.slot_base + (uint64_t)p;
                const uint64_t idx = permute(slot, a.perm);
                const int2 pr = a.pairs[idx];
                u = pr.x;
                i = pr.y;
                const uint64_t key = mix64(a.rng_key ^ (slot * 0xD1B54A32D192ED03ull));
                const int64_t rb = a.indptr[u], re = a.indptr[u + 1];
                for (int w = 0; w < W; ++w) {
                    // negItems = randint(0, n_items), redrawn while j in Pos(u)
                    // (sampler_ranking.py:30-36)
                    uint64_t ctr = (uint64_t)w << 32;
                    int32_t j;
                    do {
                        j = (int32_t)uniform_below(mix64(key + ctr), (uint64_t)a.n_items);
                        ++ctr;
                    } while (sorted_contains(a.indices, rb, re, j));
                    rec[2 + w] = j;
                    a.occV[a.B + p * W + w] = j;
                }
                if (MODEL == GBPR) {
                    // group = np.random.choice(item_posUserList[i], gsize)
                    // -- uniform, with replacement, may contain u (sampler_gbpr.py:41)
                    const int64_t cb = a.indptr_t[i], ce = a.indptr_t[i + 1];
                    for (int k = 0; k < G; ++k) {
                        const uint64_t h = mix64(key + ((uint64_t)(kMaxNeg + k) << 32));
                        const int32_t g =
                            a.indices_t[cb + (int64_t)uniform_below(h, (uint64_t)(ce - cb))];
                        rec[2 + W + k] = g;
                        a.occU[a.B + p * G + k] = g;
                    }
                }
                a.occU[p] = u;
                a.occV[p] = i;
            } else {
                u = a.occU[p];
                i = a.occV[p];
                for (int w = 0; w < W; ++w) rec[2 + w] = a.occV[a.B + p * W + w];
                for (int k = 0; k < G; ++k) rec[2 + W + k] = a.occU[a.B + p * G + k];
            }
            rec[0] = u;
            rec[1] = i;
            if (a.mark_users) {
                a.flagU[p] = atomicExch(&a.markU[u], a.stamp) != a.stamp;
                for (int k = 0; k < G; ++k)
                    a.flagU[a.B + p * G + k] =
                        atomicExch(&a.markU[rec[2 + W + k]], a.stamp) != a.stamp;
            }
            if (a.mark_items) {
                a.flagV[p] = atomicExch(&a.markV[i], a.stamp) != a.stamp;
                for (int w = 0; w < W; ++w)
                    a.flagV[a.B + p * W + w] = atomicExch(&a.markV[rec[2 + w]], a.stamp) != a.stamp;
            }
        }
    }
    __syncthreads();
    if (!a.grads) return;

    // ---- phase B: lane = embedding dimension ------------------------------------
    const int d = a.d;
    float loss_w = 0.f;   // wave-uniform: embedding loss (+ GBPR bias L2)
    float sq = 0.f;       // lane-partial sum of squares for the L2 term
    for (int pp = 0; pp < kPairsPerWave; ++pp) {
        const int p = p0 + pp;
        if (p >= a.B) break;
        const int* rec = sw + pp * stride;
        const int u = rfl(rec[0]);
        const int i = rfl(rec[1]);
        float uu[EPL], vi[EPL];
        load_row<EPL>(a.U, u, d, lane, uu);
        load_row<EPL>(a.V, i, d, lane, vi);

        if (MODEL == BPR || MODEL == AMF) {
            // x = <u,i> - <u,j>;  c = dL/dx = sigmoid(x) - 1   (A.1, A.4)
            const float ui = wave_sum(dot_part<EPL>(uu, vi));
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
            for (int w = 0; w < W; ++w) {
                const int j = rfl(rec[2 + w]);
                float vj[EPL];
                load_row<EPL>(a.V, j, d, lane, vj);
                const float uj = wave_sum(dot_part<EPL>(uu, vj));
                const float x = ui - uj;
                float c = -1.f / (1.f + expf(x));
                if (MODEL == AMF) {
                    loss_w += softplus(-x);
                    if (a.adversarial) {
                        // + reg_adv * softplus(-clip_by_value(x, -80, 1e8)), Δ == 0
                        const float xc = fmaxf(fminf(x, 1e8f), -80.f);
                        loss_w += a.reg_adv * softplus(-xc);
                        if (x >= -80.f && x <= 1e8f) c *= (1.f + a.reg_adv);
                    }
                } else {
                    loss_w += neg_log_sigmoid(x);
                }
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(c, vi[s] - vj[s], gu[s]);
                    gj[s] = -c * uu[s] + a.reg * vj[s];
                    sq = fmaf(vj[s], vj[s], sq);
                }
                atomic_row<EPL>(a.GV, j, d, lane, gj);
            }
            float gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] += a.reg * uu[s];
                gi[s] = sc * uu[s] + a.reg * vi[s];
                sq = fmaf(uu[s], uu[s], sq);
                sq = fmaf(vi[s], vi[s], sq);
            }
            atomic_row<EPL>(a.GU, u, d, lane, gu);
            atomic_row<EPL>(a.GV, i, d, lane, gi);
        } else if (MODEL == GBPR) {
            // ui = rho*mean_k<g_k,i> + (1-rho)<u,i> + b_i ; uj = <u,j> + b_j   (A.2)
            const float bi = a.b[i];
            const float ui_u = wave_sum(dot_part<EPL>(uu, vi));
            float sg[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) sg[s] = 0.f;
            for (int k = 0; k < G; ++k) {
                float gk[EPL];
                load_row<EPL>(a.U, rfl(rec[2 + W + k]), d, lane, gk);
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    sg[s] += gk[s];
                    sq = fmaf(gk[s], gk[s], sq);
                }
            }
            const float Gf = (float)G;
            const float ui_g = wave_sum(dot_part<EPL>(sg, vi)) / Gf;
            const float ui = a.rho * ui_g + (1.f - a.rho) * ui_u + bi;
            float gu[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
            float sc = 0.f;
            for (int w = 0; w < W; ++w) {
                const int j = rfl(rec[2 + w]);
                const float bj = a.b[j];
                float vj[EPL];
                load_row<EPL>(a.V, j, d, lane, vj);
                const float uj = wave_sum(dot_part<EPL>(uu, vj)) + bj;
                const float x = ui - uj;
                const float c = -1.f / (1.f + expf(x));
                loss_w += neg_log_sigmoid(x) + 0.5f * a.reg * bj * bj;
                sc += c;
                float gj[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) {
                    gu[s] = fmaf(-c, vj[s], gu[s]);
                    gj[s] = -c * uu[s];  // no L2 on V[j] (gbprmf.py:59-64)
                }
                atomic_row<EPL>(a.GV, j, d, lane, gj);
                if (lane == 0) unsafeAtomicAdd(a.Gb + j, -c + a.reg * bj);
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
            atomic_row<EPL>(a.GU, u, d, lane, gu);
            for (int k = 0; k < G; ++k) {
                const int g = rfl(rec[2 + W + k]);
                float gk[EPL], gg[EPL];
                load_row<EPL>(a.U, g, d, lane, gk);
#pragma unroll
                for (int s = 0; s < EPL; ++s) gg[s] = rg * sc * vi[s] + a.reg * gk[s];
                atomic_row<EPL>(a.GU, g, d, lane, gg);
            }
            atomic_row<EPL>(a.GV, i, d, lane, gi);
            if (lane == 0) unsafeAtomicAdd(a.Gb + i, sc);
        } else {  // CML (A.3)
            float du[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) du[s] = uu[s] - vi[s];
            const float dp = wave_sum(dot_part<EPL>(du, du));
            float dn_lane = 0.f;  // lane w keeps dn_w
            float m = INFINITY;
            int imp = 0;
            for (int w = 0; w < W; ++w) {
                float vj[EPL];
                load_row<EPL>(a.V, rfl(rec[2 + w]), d, lane, vj);
                float t[EPL];
#pragma unroll
                for (int s = 0; s < EPL; ++s) t[s] = uu[s] - vj[s];
                const float dn = wave_sum(dot_part<EPL>(t, t));
                if (lane == w) dn_lane = dn;
                m = fminf(m, dn);
                imp += (dp - dn + a.margin > 0.f) ? 1 : 0;
            }
            const unsigned long long tie = __ballot(lane < W && dn_lane == m);
            const float cnt = (float)__popcll(tie);
            const float z = dp - m + a.margin;
            const float lw =
                a.use_rank_weight ? logf((float)imp / (float)W * a.n_items_f + 1.f) : 1.f;
            loss_w += fmaxf(z, 0.f) * lw;
            const float aa = (z > 0.f) ? lw : 0.f;
            const bool l2 = a.reg_cov > 0.f;
            float gu[EPL], gi[EPL];
#pragma unroll
            for (int s = 0; s < EPL; ++s) {
                gu[s] = 2.f * aa * du[s];
                gi[s] = -2.f * aa * du[s];
            }
            for (int w = 0; w < W; ++w) {
                const float dnw = __shfl(dn_lane, w, 64);
                const float share = (dnw == m) ? 1.f / cnt : 0.f;
                if (share == 0.f && !l2) continue;  // wave-uniform
                const int j = rfl(rec[2 + w]);
                float vj[EPL], gj[EPL];
                load_row<EPL>(a.V, j, d, lane, vj);
                const float coef = 2.f * aa * share;
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
                atomic_row<EPL>(a.GV, j, d, lane, gj);
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
            atomic_row<EPL>(a.GU, u, d, lane, gu);
            atomic_row<EPL>(a.GV, i, d, lane, gi);
        }
    }

    // ---- per-block pre-update loss partial (deterministic order) -----------------
    float coef = (MODEL == CML) ? (a.reg_cov > 0.f ? a.reg_cov : 0.f) : a.reg;
    const float sq_w = wave_sum(sq);
    if (lane == 0) s_loss[wv] = (double)loss_w + 0.5 * (double)coef * (double)sq_w;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < kWavesPerBlock; ++k) t += s_loss[k];
        a.loss_partial[blockIdx.x] = t;
    }
}

// ---------------------------------------------------------------------------
// Adagrad apply over the winner rows of the batch
// ---------------------------------------------------------------------------
template <int EPL, bool CLIP>
__device__ __forceinline__ void apply_row(float* __restrict__ X, float* __restrict__ A,
                                          float* __restrict__ G, int64_t r, int d, int lane,
                                          float lr, float clip_norm) {
    float* xr = X + r * (int64_t)d;
    float* ar = A + r * (int64_t)d;
    float* gr = G + r * (int64_t)d;
    float x[EPL], acc[EPL], g[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kWave + lane;
        const bool ok = e < d;
        g[s] = ok ? gr[e] : 0.f;
        acc[s] = ok ? ar[e] : 1.f;
        x[s] = ok ? xr[e] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        acc[s] = fmaf(g[s], g[s], acc[s]);     // accum += grad^2
        x[s] -= (lr * g[s]) / sqrtf(acc[s]);   // var -= lr*grad*rsqrt(accum)
    }
    if (CLIP) {
        // tf.clip_by_norm(t, c, axes=[1]) = t*c / max(|t|, c)
        const float n = sqrtf(wave_sum(dot_part<EPL>(x, x)));
        const float den = fmaxf(n, clip_norm);
#pragma unroll
        for (int s = 0; s < EPL; ++s) x[s] = (x[s] * clip_norm) / den;
    }
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kWave + lane;
        if (e < d) {
            xr[e] = x[s];
            ar[e] = acc[s];
            gr[e] = 0.f;
        }
    }
}

template <int EPL, bool CLIP>
__global__ __launch_bounds__(kBlock) void apply_kernel(ApplyArgs a) {
    __shared__ double s_red[kWavesPerBlock];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    if (blockIdx.x == 0 && a.loss_acc != nullptr) {
        double t = 0.0;
        for (int k = threadIdx.x; k < a.n_partial; k += kBlock) t += a.loss_partial[k];
        t = wave_sum_d(t);
        if (lane == 0) s_red[wv] = t;
        __syncthreads();
        if (threadIdx.x == 0) a.loss_acc[0] += (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    }
    const bool isU = (int)blockIdx.x < a.blocksU;
    const int blk = isU ? (int)blockIdx.x : (int)blockIdx.x - a.blocksU;
    const int n = isU ? a.nU : a.nV;
    const int32_t* occ = isU ? a.occU : a.occV;
    const uint8_t* flag = isU ? a.flagU : a.flagV;
    float* X = isU ? a.U : a.V;
    float* A = isU ? a.AU : a.AV;
    float* G = isU ? a.GU : a.GV;

    const int o = (blk * kWavesPerBlock + wv) * kWave + lane;
    const bool win = o < n && flag[o] != 0;
    const int r_l = win ? occ[o] : 0;
    if (!isU && a.b != nullptr && win) {
        const float g = a.Gb[r_l];
        const float acc = fmaf(g, g, a.Ab[r_l]);
        a.Ab[r_l] = acc;
        a.b[r_l] -= (a.lr * g) / sqrtf(acc);
        a.Gb[r_l] = 0.f;
    }
    unsigned long long mask = __ballot(win);
    while (mask) {
        const int l = __ffsll((long long)mask) - 1;
        mask &= mask - 1ull;
        const int r = rfl(__shfl(r_l, l, 64));
        apply_row<EPL, CLIP>(X, A, G, r, a.d, lane, a.lr, a.clip_norm);
    }
}

// dense item apply (multi-rank: after the all-reduce every replica applies the
// identical update; rows with an all-zero gradient are exact no-ops in TF too)
template <int EPL, bool CLIP>
__global__ __launch_bounds__(kBlock) void apply_dense_kernel(DenseArgs a) {
    const int lane = lane_id();
    const int64_t wave0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t r = wave0; r < a.n_rows; r += nwaves) {
        float g[EPL];
        load_row<EPL>(a.G, r, a.d, lane, g);
        bool nz = false;
#pragma unroll
        for (int s = 0; s < EPL; ++s) nz |= (g[s] != 0.f);
        if (__ballot(nz) == 0ull) continue;
        apply_row<EPL, CLIP>(a.X, a.A, a.G, r, a.d, lane, a.lr, a.clip_norm);
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
    const int lane = lane_id();
    const int64_t wave0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
    for (int64_t r = wave0; r < n_rows; r += nwaves) {
        float x[EPL];
        load_row<EPL>(X, r, d, lane, x);
        const float n = sqrtf(wave_sum(dot_part<EPL>(x, x)));
        const float den = fmaxf(n, c);
        float* xr = X + r * (int64_t)d;
#pragma unroll
        for (int s = 0; s < EPL; ++s) {
            const int e = s * kWave + lane;
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
static int epl_for(int d) { return d <= 64 ? 1 : (d <= 128 ? 2 : 4); }

template <int MODEL>
static hipError_t launch_step_m(const StepArgs& a, hipStream_t s) {
    const int blocks = (a.B + kPairsPerBlock - 1) / kPairsPerBlock;
    const int G = (MODEL == GBPR) ? a.G : 0;
    const size_t lds = (size_t)kPairsPerBlock * (2 + a.W + G) * sizeof(int);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((step_kernel<MODEL, 1>), dim3(blocks), dim3(kBlock), lds, s, a); break;
        case 2: hipLaunchKernelGGL((step_kernel<MODEL, 2>), dim3(blocks), dim3(kBlock), lds, s, a); break;
        default: hipLaunchKernelGGL((step_kernel<MODEL, 4>), dim3(blocks), dim3(kBlock), lds, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_step(const StepArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    switch (a.model) {
        case BPR: return launch_step_m<BPR>(a, s);
        case GBPR: return launch_step_m<GBPR>(a, s);
        case CML: return launch_step_m<CML>(a, s);
        default: return launch_step_m<AMF>(a, s);
    }
}

hipError_t launch_apply(const ApplyArgs& a, hipStream_t s) {
    const int per_block = kWavesPerBlock * kWave;
    const int bV = a.apply_items ? (a.nV + per_block - 1) / per_block : 0;
    const int blocks = a.blocksU + bV;
    if (blocks == 0) return hipSuccess;
    const int e = epl_for(a.d);
#define CF_APPLY(EPL, CL) \
    hipLaunchKernelGGL((apply_kernel<EPL, CL>), dim3(blocks), dim3(kBlock), 0, s, a)
    if (a.clip) {
        if (e == 1) CF_APPLY(1, true); else if (e == 2) CF_APPLY(2, true); else CF_APPLY(4, true);
    } else {
        if (e == 1) CF_APPLY(1, false); else if (e == 2) CF_APPLY(2, false); else CF_APPLY(4, false);
    }
#undef CF_APPLY
    return hipGetLastError();
}

hipError_t launch_apply_dense(const DenseArgs& a, hipStream_t s) {
    const int64_t waves = a.n_rows;
    int blocks = (int)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    const int e = epl_for(a.d);
#define CF_DENSE(EPL, CL) \
    hipLaunchKernelGGL((apply_dense_kernel<EPL, CL>), dim3(blocks), dim3(kBlock), 0, s, a)
    if (a.clip) {
        if (e == 1) CF_DENSE(1, true); else if (e == 2) CF_DENSE(2, true); else CF_DENSE(4, true);
    } else {
        if (e == 1) CF_DENSE(1, false); else if (e == 2) CF_DENSE(2, false); else CF_DENSE(4, false);
    }
#undef CF_DENSE
    return hipGetLastError();
}

hipError_t launch_clip_full(float* X, int64_t n_rows, int d, float c, hipStream_t s) {
    int blocks = (int)((n_rows + kWavesPerBlock - 1) / kWavesPerBlock);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    const int e = epl_for(d);
    if (e == 1) hipLaunchKernelGGL((clip_full_kernel<1>), dim3(blocks), dim3(kBlock), 0, s, X, n_rows, d, c);
    else if (e == 2) hipLaunchKernelGGL((clip_full_kernel<2>), dim3(blocks), dim3(kBlock), 0, s, X, n_rows, d, c);
    else hipLaunchKernelGGL((clip_full_kernel<4>), dim3(blocks), dim3(kBlock), 0, s, X, n_rows, d, c);
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
    p.mask = (bits >= 64) ? ~0ull : ((1ull << bits) - 1ull);
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
