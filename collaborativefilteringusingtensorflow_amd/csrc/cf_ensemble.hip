// cf_ensemble.hip -- the Ensemble model (src/models/pl/models/ensemble.py),
// the consumer of sampler_uij_ranking, on gfx950.
//
// K attention-weighted MF members: U[K, n_users, d], V[K, n_items, d],
// H[K, d].  For a (u, i, j) batch of B triplets (ensemble.py:71-109):
//   s_k(x) = <U_k[u], V_k[x]>,  e_k(x) = <U_k[u] o V_k[x], h_k>,
//   w_k(x) = exp(e_k(x)) / sum_k' exp(e_k'(x))          (x = i or j)
// and -- because ensemble.py:87-90 multiplies a [B] vector by a [B, 1] one --
// the loss runs over ALL B x B (p, q) combinations of the batch:
//   z[p, q] = sum_k w_k(i_p) s_k(i_q) - w_k(j_p) s_k(j_q)
//   L = sum_{p,q} -log sigmoid(z[p, q]) + reg (sum_k l2(U_k[u]) + l2(V_k[i,j]) + l2(H))
// TF1 takes the gradient of the strided slice user_embeds[k] densely, so the
// optimizer is dense ApplyAdagrad over the whole tables: exactly the summed
// gradient on the touched rows (an untouched row's update is a no-op).
//
// One step = four launches:
//   ens_pair_kernel    one 16-lane group per triplet: gather the 3K rows,
//                      s / e / w per member, L2 partials;
//   ens_cross_kernel   64 x 64 (p, q) tiles: z, the loss, c = dL/dz, row sums
//                      (dL/dw) and column sums (dL/ds) -> float atomics;
//   ens_grad_kernel    per triplet: softmax backward, the gradient rows of
//                      U_k[u], V_k[i], V_k[j] (float atomics into dense
//                      accumulators) and of H (LDS-reduced per block);
//   apply_dense_kernel dense Adagrad of U, V, H (cf_kernels.hip), skipping
//                      rows whose summed gradient is zero.
// The recommend step (ensemble.py:115-140) scores sum_k s_k w_k for every
// (user, item) and reuses the top-k selection of cf_eval.hip.
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cf_engine.h"
#include "cf_device.h"
#include "cf_kernels.h"

namespace cfi {
int set_error(int code, const std::string& msg);  // cf_engine.cpp
}

namespace cfk {

constexpr int kEnsMaxK = 8;
constexpr int kEnsTile = 64;

struct EnsArgs {
    int K, d, B;
    int64_t n_users, n_items;
    float reg;
    const int32_t* __restrict__ uij;     // [B, 3]
    const float* __restrict__ U;         // [K, n_users, d]
    const float* __restrict__ V;         // [K, n_items, d]
    const float* __restrict__ H;         // [K, d]
    float* __restrict__ GU;
    float* __restrict__ GV;
    float* __restrict__ GH;
    float* __restrict__ si;              // [K, B] s_k(i_p)
    float* __restrict__ sj;
    float* __restrict__ wi;              // [K, B] w_k(i_p)
    float* __restrict__ wj;
    float* __restrict__ gsi;             // [K, B] dL/ds_k(i_q)  (zeroed)
    float* __restrict__ gsj;
    float* __restrict__ gwi;             // [K, B] dL/dw_k(i_p)  (zeroed)
    float* __restrict__ gwj;
    double* __restrict__ loss_partial;   // [pair blocks + cross blocks]
    double* __restrict__ loss_acc;       // running sum until cf_ens_take_loss
    int n_pair_blocks;
};

__device__ __forceinline__ float g16sum(float v) {
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 1, 64);
    return v;
}

__global__ __launch_bounds__(kBlock) void ens_pair_kernel(EnsArgs a) {
    __shared__ double s_l[kGroupsPerBlock];
    const int gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int p = blockIdx.x * kGroupsPerBlock + grp;
    float sq = 0.f;
    if (p < a.B) {
        const int64_t u = a.uij[3 * p], i = a.uij[3 * p + 1], j = a.uij[3 * p + 2];
        float ai[kEnsMaxK], aj[kEnsMaxK], Ai = 0.f, Aj = 0.f;
        for (int k = 0; k < a.K; ++k) {
            const float* uk = a.U + ((int64_t)k * a.n_users + u) * a.d;
            const float* ik = a.V + ((int64_t)k * a.n_items + i) * a.d;
            const float* jk = a.V + ((int64_t)k * a.n_items + j) * a.d;
            const float* hk = a.H + (int64_t)k * a.d;
            float s_i = 0.f, s_j = 0.f, e_i = 0.f, e_j = 0.f;
            for (int e = gl; e < a.d; e += 16) {
                const float x = uk[e], y = ik[e], z = jk[e], h = hk[e];
                s_i = fmaf(x, y, s_i);
                s_j = fmaf(x, z, s_j);
                e_i = fmaf(x * y, h, e_i);
                e_j = fmaf(x * z, h, e_j);
                sq = fmaf(x, x, sq);
                sq = fmaf(y, y, sq);
                sq = fmaf(z, z, sq);
            }
            s_i = g16sum(s_i);
            s_j = g16sum(s_j);
            ai[k] = expf(g16sum(e_i));   // tf.exp(ui . h_k), ensemble.py:83
            aj[k] = expf(g16sum(e_j));
            Ai += ai[k];
            Aj += aj[k];
            if (gl == 0) {
                a.si[(int64_t)k * a.B + p] = s_i;
                a.sj[(int64_t)k * a.B + p] = s_j;
            }
        }
        if (gl == 0)
            for (int k = 0; k < a.K; ++k) {
                a.wi[(int64_t)k * a.B + p] = ai[k] / Ai;
                a.wj[(int64_t)k * a.B + p] = aj[k] / Aj;
            }
    }
    const float t = g16sum(sq);
    if (gl == 0) s_l[grp] = 0.5 * (double)a.reg * (double)t;
    __syncthreads();
    if (threadIdx.x == 0) {
        double acc = 0.0;
        for (int g = 0; g < kGroupsPerBlock; ++g) acc += s_l[g];
        if (blockIdx.x == 0)   // reg * l2(H), once
            for (int e = 0; e < a.K * a.d; ++e) acc += 0.5 * (double)a.reg * (double)a.H[e] * a.H[e];
        a.loss_partial[blockIdx.x] = acc;
        atomicAdd(a.loss_acc, acc);
    }
}

// (p, q) tile: thread (tp = tid / 16, tq = tid % 16) owns p in tp*4 + [0,4),
// q in tq + 16*[0,4)
__global__ __launch_bounds__(kBlock) void ens_cross_kernel(EnsArgs a) {
    __shared__ float s_wi[kEnsMaxK][kEnsTile], s_wj[kEnsMaxK][kEnsTile];
    __shared__ float s_si[kEnsMaxK][kEnsTile], s_sj[kEnsMaxK][kEnsTile];
    __shared__ float s_col[2 * kEnsMaxK][kEnsTile];
    __shared__ double s_l[kWavesPerBlock];
    const int p0 = blockIdx.y * kEnsTile, q0 = blockIdx.x * kEnsTile;
    const int K = a.K;
    for (int t = threadIdx.x; t < K * kEnsTile; t += kBlock) {
        const int k = t / kEnsTile, r = t % kEnsTile;
        const int p = p0 + r, q = q0 + r;
        s_wi[k][r] = p < a.B ? a.wi[(int64_t)k * a.B + p] : 0.f;
        s_wj[k][r] = p < a.B ? a.wj[(int64_t)k * a.B + p] : 0.f;
        s_si[k][r] = q < a.B ? a.si[(int64_t)k * a.B + q] : 0.f;
        s_sj[k][r] = q < a.B ? a.sj[(int64_t)k * a.B + q] : 0.f;
        s_col[k][r] = 0.f;
        s_col[K + k][r] = 0.f;
    }
    __syncthreads();
    const int tp = threadIdx.x >> 4, tq = threadIdx.x & 15;
    double lsum = 0.0;
    for (int m = 0; m < 4; ++m) {
        const int pr = tp * 4 + m;
        const bool pv = p0 + pr < a.B;
        float rwi[kEnsMaxK], rwj[kEnsMaxK];
        for (int k = 0; k < K; ++k) rwi[k] = rwj[k] = 0.f;
        for (int n = 0; n < 4; ++n) {
            const int qc = tq + 16 * n;
            if (!pv || q0 + qc >= a.B) continue;
            float z = 0.f;
            for (int k = 0; k < K; ++k)
                z += s_wi[k][pr] * s_si[k][qc] - s_wj[k][pr] * s_sj[k][qc];
            lsum += (double)(-logf(1.f / (1.f + expf(-z))));   // -log(sigmoid), ensemble.py:107
            const float c = -1.f / (1.f + expf(z));             // d/dz
            for (int k = 0; k < K; ++k) {
                rwi[k] = fmaf(c, s_si[k][qc], rwi[k]);
                rwj[k] = fmaf(-c, s_sj[k][qc], rwj[k]);
                atomicAdd(&s_col[k][qc], c * s_wi[k][pr]);
                atomicAdd(&s_col[K + k][qc], -c * s_wj[k][pr]);
            }
        }
        for (int k = 0; k < K; ++k) {   // sum over the 16 lanes sharing this p
            const float x = g16sum(rwi[k]), y = g16sum(rwj[k]);
            if (tq == 0 && pv) {
                atomicAdd(a.gwi + (int64_t)k * a.B + p0 + pr, x);
                atomicAdd(a.gwj + (int64_t)k * a.B + p0 + pr, y);
            }
        }
    }
    lsum = wave_sum_d(lsum);
    if (lane_id() == 0) s_l[threadIdx.x >> 6] = lsum;
    __syncthreads();
    for (int t = threadIdx.x; t < K * kEnsTile; t += kBlock) {
        const int k = t / kEnsTile, r = t % kEnsTile;
        if (q0 + r < a.B) {
            atomicAdd(a.gsi + (int64_t)k * a.B + q0 + r, s_col[k][r]);
            atomicAdd(a.gsj + (int64_t)k * a.B + q0 + r, s_col[K + k][r]);
        }
    }
    if (threadIdx.x == 0) {
        const double t = (s_l[0] + s_l[1]) + (s_l[2] + s_l[3]);
        a.loss_partial[a.n_pair_blocks + blockIdx.y * gridDim.x + blockIdx.x] = t;
        atomicAdd(a.loss_acc, t);
    }
}

__global__ __launch_bounds__(kBlock) void ens_grad_kernel(EnsArgs a) {
    extern __shared__ float s_gh[];   // [K, d]
    for (int t = threadIdx.x; t < a.K * a.d; t += kBlock)
        s_gh[t] = (blockIdx.x == 0) ? a.reg * a.H[t] : 0.f;   // + reg * H, once
    __syncthreads();
    const int gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int p = blockIdx.x * kGroupsPerBlock + grp;
    if (p < a.B) {
        const int64_t u = a.uij[3 * p], i = a.uij[3 * p + 1], j = a.uij[3 * p + 2];
        // softmax backward: de_k = w_k (dw_k - sum_k' w_k' dw_k')
        float dotI = 0.f, dotJ = 0.f;
        for (int k = 0; k < a.K; ++k) {
            dotI += a.wi[(int64_t)k * a.B + p] * a.gwi[(int64_t)k * a.B + p];
            dotJ += a.wj[(int64_t)k * a.B + p] * a.gwj[(int64_t)k * a.B + p];
        }
        for (int k = 0; k < a.K; ++k) {
            const int64_t kp = (int64_t)k * a.B + p;
            const float dei = a.wi[kp] * (a.gwi[kp] - dotI);
            const float dej = a.wj[kp] * (a.gwj[kp] - dotJ);
            const float dsi = a.gsi[kp], dsj = a.gsj[kp];
            const int64_t ru = (int64_t)k * a.n_users + u;
            const int64_t ri = (int64_t)k * a.n_items + i, rj = (int64_t)k * a.n_items + j;
            const float* uk = a.U + ru * a.d;
            const float* ik = a.V + ri * a.d;
            const float* jk = a.V + rj * a.d;
            const float* hk = a.H + (int64_t)k * a.d;
            for (int e = gl; e < a.d; e += 16) {
                const float x = uk[e], y = ik[e], z = jk[e], h = hk[e];
                const float vi = fmaf(dei, h, dsi);   // dL/d(u o i)
                const float vj = fmaf(dej, h, dsj);   // dL/d(u o j)
                unsafeAtomicAdd(a.GU + ru * a.d + e, fmaf(vi, y, fmaf(vj, z, a.reg * x)));
                unsafeAtomicAdd(a.GV + ri * a.d + e, fmaf(vi, x, a.reg * y));
                unsafeAtomicAdd(a.GV + rj * a.d + e, fmaf(vj, x, a.reg * z));
                atomicAdd(&s_gh[k * a.d + e], dei * (x * y) + dej * (x * z));
            }
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < a.K * a.d; t += kBlock) unsafeAtomicAdd(a.GH + t, s_gh[t]);
}

// (user, item) ensemble scores -> order-preserving keys (topk_kernel input);
// one thread per item, a block per 256 items of one user
__global__ __launch_bounds__(kBlock) void ens_score_kernel(int K, int d, int64_t n_users,
                                                           int64_t n_items, const int32_t* users,
                                                           const float* __restrict__ U,
                                                           const float* __restrict__ V,
                                                           const float* __restrict__ H,
                                                           uint32_t* __restrict__ keys,
                                                           int exclude_train,
                                                           const int64_t* __restrict__ indptr,
                                                           const int32_t* __restrict__ indices) {
    extern __shared__ float s_uh[];   // [K][2][d]: U_k[u], U_k[u] o h_k
    const int c = blockIdx.y;
    const int64_t u = users[c];
    for (int t = threadIdx.x; t < K * d; t += kBlock) {
        const int k = t / d, e = t % d;
        const float x = U[((int64_t)k * n_users + u) * d + e];
        s_uh[(2 * k) * d + e] = x;
        s_uh[(2 * k + 1) * d + e] = x * H[t];
    }
    __syncthreads();
    const int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (it >= n_items) return;
    float num = 0.f, den = 0.f;
    for (int k = 0; k < K; ++k) {
        const float* vk = V + ((int64_t)k * n_items + it) * d;
        float s = 0.f, e = 0.f;
        for (int q = 0; q < d; ++q) {
            const float y = vk[q];
            s = fmaf(s_uh[(2 * k) * d + q], y, s);
            e = fmaf(s_uh[(2 * k + 1) * d + q], y, e);
        }
        const float w = expf(e);   // ensemble.py:134-139: sum_k s_k exp(e_k) / sum_k exp(e_k)
        num = fmaf(s, w, num);
        den += w;
    }
    uint32_t key = float_key(num / den);
    if (exclude_train && sorted_contains(indices, indptr[u], indptr[u + 1], (int32_t)it)) key = 0u;
    keys[(int64_t)c * n_items + it] = key;
}

// ---------------------------------------------------------------------------
// W-negative variants (ensemble_.py:75-118, ensemble__.py:102-145): per pair
// p, items x in {i, j_0..j_{W-1}}: r_x = sum_k w_k(x) s_k(x); loss
// lam * sum_w -log sigmoid(r_i - r_jw) (+ the members' own BPR terms
// sum_k sum_w -log sigmoid(s_k(i) - s_k(j_w)) when `singles`).  One 16-lane
// group per pair; the K x (1+W) scores and weights live in LDS.
// ---------------------------------------------------------------------------
constexpr int kEnsMaxW = 8;

struct EnsWArgs {
    int K, d, B, W, singles;
    int64_t n_users, n_items;
    float reg, lam;
    const int32_t* __restrict__ pairs;   // [B, 2]
    const int32_t* __restrict__ negs;    // [B, W]
    const float* __restrict__ U;
    const float* __restrict__ V;
    const float* __restrict__ H;
    float* __restrict__ GU;
    float* __restrict__ GV;
    float* __restrict__ GH;
    double* __restrict__ loss_partial;   // [blocks]
    double* __restrict__ loss_acc;
};

__global__ __launch_bounds__(kBlock) void ens_w_kernel(EnsWArgs a) {
    constexpr int X1 = kEnsMaxW + 1;
    __shared__ float s_s[kGroupsPerBlock][kEnsMaxK][X1];   // s_k(x), then dL/ds_k(x)
    __shared__ float s_w[kGroupsPerBlock][kEnsMaxK][X1];   // w_k(x), then dL/de_k(x)
    __shared__ double s_l[kGroupsPerBlock];
    extern __shared__ float s_gh[];                        // [K, d]
    for (int t = threadIdx.x; t < a.K * a.d; t += kBlock)
        s_gh[t] = (blockIdx.x == 0) ? a.reg * a.H[t] : 0.f;   // + reg * H, once
    __syncthreads();
    const int gl = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int p = blockIdx.x * kGroupsPerBlock + grp;
    const int K = a.K, W = a.W, NX = 1 + a.W;
    float sq = 0.f, lossf = 0.f;
    if (p < a.B) {
        const int64_t u = a.pairs[2 * p];
        auto item = [&](int x) -> int64_t { return x == 0 ? a.pairs[2 * p + 1] : a.negs[(int64_t)p * W + x - 1]; };
        // scores s_k(x) and attention logits, per member
        for (int k = 0; k < K; ++k) {
            const float* uk = a.U + ((int64_t)k * a.n_users + u) * a.d;
            const float* hk = a.H + (int64_t)k * a.d;
            for (int x = 0; x < NX; ++x) {
                const float* vk = a.V + ((int64_t)k * a.n_items + item(x)) * a.d;
                float sv = 0.f, ev = 0.f;
                for (int e = gl; e < a.d; e += 16) {
                    const float uu = uk[e], vv = vk[e];
                    sv = fmaf(uu, vv, sv);
                    ev = fmaf(uu * vv, hk[e], ev);
                    sq = fmaf(vv, vv, sq);
                    if (x == 0) sq = fmaf(uu, uu, sq);
                }
                sv = g16sum(sv);
                ev = g16sum(ev);
                if (gl == 0) {
                    s_s[grp][k][x] = sv;
                    s_w[grp][k][x] = expf(ev);   // exp(<u o v, h_k>), ensemble_.py:89-91
                }
            }
        }
        if (gl == 0) {
            float r[X1], den[X1];
            for (int x = 0; x < NX; ++x) {
                den[x] = 0.f;
                for (int k = 0; k < K; ++k) den[x] += s_w[grp][k][x];
                r[x] = 0.f;
                for (int k = 0; k < K; ++k) {
                    s_w[grp][k][x] /= den[x];
                    r[x] = fmaf(s_s[grp][k][x], s_w[grp][k][x], r[x]);
                }
            }
            // dL/dr_x for the ensemble term
            float gr[X1];
            gr[0] = 0.f;
            for (int w = 1; w < NX; ++w) {
                const float z = r[0] - r[w];
                lossf += a.lam * (-logf(1.f / (1.f + expf(-z))));
                const float c = a.lam * (-1.f / (1.f + expf(z)));
                gr[0] += c;
                gr[w] = -c;
            }
            // singles: the members' own BPR terms (ensemble__.py:118-133)
            float ds0[kEnsMaxK];
            for (int k = 0; k < K; ++k) ds0[k] = 0.f;
            for (int k = 0; k < K; ++k) {
                const float si = s_s[grp][k][0];
                for (int x = 0; x < NX; ++x) {
                    const float wv = s_w[grp][k][x], sv = s_s[grp][k][x];
                    float ds = gr[x] * wv;
                    const float de = gr[x] * wv * (sv - r[x]);   // softmax backward
                    if (a.singles && x > 0) {
                        const float z = si - sv;
                        lossf += -logf(1.f / (1.f + expf(-z)));
                        const float c = -1.f / (1.f + expf(z));
                        ds0[k] += c;
                        ds -= c;
                    }
                    s_s[grp][k][x] = ds;   // now dL/ds_k(x) (the positive's singles part added below)
                    s_w[grp][k][x] = de;   // now dL/de_k(x)
                }
            }
            for (int k = 0; k < K; ++k) s_s[grp][k][0] += ds0[k];
        }
        __builtin_amdgcn_wave_barrier();
        // gradient rows: d(u o v_x) = ds + de * h_k
        for (int k = 0; k < K; ++k) {
            const int64_t ru = (int64_t)k * a.n_users + u;
            const float* uk = a.U + ru * a.d;
            const float* hk = a.H + (int64_t)k * a.d;
            for (int e = gl; e < a.d; e += 16) {
                const float uu = uk[e], h = hk[e];
                float gu = a.reg * uu;
                float gh = 0.f;
                for (int x = 0; x < NX; ++x) {
                    const int64_t rx = (int64_t)k * a.n_items + item(x);
                    const float vv = a.V[rx * a.d + e];
                    const float ds = s_s[grp][k][x], de = s_w[grp][k][x];
                    const float gx = fmaf(de, h, ds);
                    gu = fmaf(gx, vv, gu);
                    unsafeAtomicAdd(a.GV + rx * a.d + e, fmaf(gx, uu, a.reg * vv));
                    gh = fmaf(de, uu * vv, gh);
                }
                unsafeAtomicAdd(a.GU + ru * a.d + e, gu);
                atomicAdd(&s_gh[k * a.d + e], gh);
            }
        }
    }
    const float t = g16sum(sq);
    if (gl == 0) s_l[grp] = (double)lossf + 0.5 * (double)a.reg * (double)t;
    __syncthreads();
    for (int t2 = threadIdx.x; t2 < a.K * a.d; t2 += kBlock) unsafeAtomicAdd(a.GH + t2, s_gh[t2]);
    if (threadIdx.x == 0) {
        double acc = 0.0;
        for (int g = 0; g < kGroupsPerBlock; ++g) acc += s_l[g];
        if (blockIdx.x == 0)
            for (int e = 0; e < a.K * a.d; ++e) acc += 0.5 * (double)a.reg * (double)a.H[e] * a.H[e];
        a.loss_partial[blockIdx.x] = acc;
        atomicAdd(a.loss_acc, acc);
    }
}

}  // namespace cfk

using namespace cfk;

struct cf_ensemble {
    int64_t n_users = 0, n_items = 0;
    int K = 0, d = 0;
    float reg = 0.f, lr = 0.1f, acc_init = 0.1f;
    int device = 0;
    hipStream_t stream = nullptr;
    float *U = nullptr, *V = nullptr, *H = nullptr;
    float *AU = nullptr, *AV = nullptr, *AH = nullptr;
    float *GU = nullptr, *GV = nullptr, *GH = nullptr;
    int64_t* indptr = nullptr;
    int32_t* indices = nullptr;
    int Bcap = 0;
    int32_t* uij = nullptr;
    float* scratch = nullptr;   // si sj wi wj gsi gsj gwi gwj: 8 x [K, B]
    double* loss_partial = nullptr;
    double* loss_acc = nullptr;
    int loss_cap = 0;
    std::vector<double> h_loss;
};

namespace {

template <class T>
int ealloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) return CF_OK;
    if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess)
        return cfi::set_error(CF_ENOMEM, "hipMalloc(" + std::to_string(n * sizeof(T)) + " B) failed");
    return CF_OK;
}

template <class T>
void efree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

#define ENS_HIP(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) return cfi::set_error(CF_EHIP, std::string(#expr) + ": " +        \
                                                                 hipGetErrorString(_e));       \
    } while (0)
#define ENS_TRY(expr)           \
    do {                        \
        int _r = (expr);        \
        if (_r != CF_OK) return _r; \
    } while (0)

float* ens_table(cf_ensemble* e, int t, int64_t* n) {
    const int64_t nu = (int64_t)e->K * e->n_users * e->d, ni = (int64_t)e->K * e->n_items * e->d;
    const int64_t nh = (int64_t)e->K * e->d;
    switch (t) {
        case 0: *n = nu; return e->U;
        case 1: *n = ni; return e->V;
        case 2: *n = nh; return e->H;
        case 3: *n = nu; return e->AU;
        case 4: *n = ni; return e->AV;
        case 5: *n = nh; return e->AH;
        default: *n = 0; return nullptr;
    }
}

int dense_apply(cf_ensemble* e, float* X, float* A, float* G, int64_t rows) {
    DenseArgs d{};
    d.d = e->d;
    d.lr = e->lr;
    d.clip = 0;
    d.zero_g = 1;
    d.n_rows = rows;
    d.X = X; d.A = A; d.G = G;
    ENS_HIP(launch_apply_dense(d, e->stream));
    return CF_OK;
}

}  // namespace

extern "C" {

int cf_ens_create(int64_t n_users, int64_t n_items, int32_t K, int32_t d, float reg, float lr,
                  float acc_init, int32_t device, cf_ensemble** out) {
    if (!out || n_users < 1 || n_items < 2 || K < 1 || K > kEnsMaxK || d < 1 || d > kMaxFactors ||
        !(lr > 0.f) || !(acc_init > 0.f))
        return cfi::set_error(CF_EINVAL, "bad ensemble configuration (K 1..8, d 1..256)");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return cfi::set_error(CF_EHIP, "no HIP device visible (the engine has no CPU fallback)");
    if (device < 0 || device >= ndev) return cfi::set_error(CF_EINVAL, "device ordinal out of range");
    ENS_HIP(hipSetDevice(device));
    cf_ensemble* e = new cf_ensemble();
    e->n_users = n_users; e->n_items = n_items; e->K = K; e->d = d;
    e->reg = reg; e->lr = lr; e->acc_init = acc_init; e->device = device;
    auto bail = [&](int r) { cf_ens_destroy(e); return r; };
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(cfi::set_error(CF_EHIP, "hipStreamCreate failed"));
    const size_t nu = (size_t)K * n_users * d, ni = (size_t)K * n_items * d, nh = (size_t)K * d;
    int r;
    if ((r = ealloc(&e->U, nu)) || (r = ealloc(&e->AU, nu)) || (r = ealloc(&e->GU, nu)) ||
        (r = ealloc(&e->V, ni)) || (r = ealloc(&e->AV, ni)) || (r = ealloc(&e->GV, ni)) ||
        (r = ealloc(&e->H, nh)) || (r = ealloc(&e->AH, nh)) || (r = ealloc(&e->GH, nh)) ||
        (r = ealloc(&e->loss_acc, 1)))
        return bail(r);
    if (hipMemsetAsync(e->GU, 0, nu * 4, e->stream) != hipSuccess ||
        hipMemsetAsync(e->loss_acc, 0, 8, e->stream) != hipSuccess ||
        hipMemsetAsync(e->GV, 0, ni * 4, e->stream) != hipSuccess ||
        hipMemsetAsync(e->GH, 0, nh * 4, e->stream) != hipSuccess ||
        launch_fill(e->AU, (int64_t)nu, acc_init, e->stream) != hipSuccess ||
        launch_fill(e->AV, (int64_t)ni, acc_init, e->stream) != hipSuccess ||
        launch_fill(e->AH, (int64_t)nh, acc_init, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        return bail(cfi::set_error(CF_EHIP, "ensemble init failed"));
    *out = e;
    return CF_OK;
}

int cf_ens_destroy(cf_ensemble* e) {
    if (!e) return CF_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    efree(e->U); efree(e->V); efree(e->H); efree(e->AU); efree(e->AV); efree(e->AH);
    efree(e->GU); efree(e->GV); efree(e->GH); efree(e->indptr); efree(e->indices);
    efree(e->uij); efree(e->scratch); efree(e->loss_partial); efree(e->loss_acc);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return CF_OK;
}

int cf_ens_init_params(cf_ensemble* e, float mean, float stddev, int32_t truncated, uint64_t seed) {
    if (!e) return cfi::set_error(CF_EINVAL, "null ensemble");
    ENS_HIP(hipSetDevice(e->device));
    const int64_t nu = (int64_t)e->K * e->n_users * e->d, ni = (int64_t)e->K * e->n_items * e->d;
    ENS_HIP(launch_init_normal(e->U, nu, mean, stddev, truncated, mix64(seed ^ 0x11u), e->stream));
    ENS_HIP(launch_init_normal(e->V, ni, mean, stddev, truncated, mix64(seed ^ 0x22u), e->stream));
    ENS_HIP(launch_init_normal(e->H, (int64_t)e->K * e->d, mean, stddev, truncated, mix64(seed ^ 0x33u),
                               e->stream));
    ENS_HIP(hipStreamSynchronize(e->stream));
    return CF_OK;
}

int cf_ens_set_lr(cf_ensemble* e, float lr) {
    if (!e || !(lr > 0.f)) return cfi::set_error(CF_EINVAL, "lr must be > 0");
    e->lr = lr;   // ensemble.py:218 decays it by 0.98 per epoch
    return CF_OK;
}

int cf_ens_set_table(cf_ensemble* e, int32_t t, const float* src, int64_t n) {
    if (!e || !src) return cfi::set_error(CF_EINVAL, "null argument");
    int64_t want = 0;
    float* p = ens_table(e, t, &want);
    if (!p || n != want) return cfi::set_error(CF_EINVAL, "ensemble table size mismatch: want " + std::to_string(want));
    ENS_HIP(hipSetDevice(e->device));
    ENS_HIP(hipStreamSynchronize(e->stream));
    ENS_HIP(hipMemcpy(p, src, (size_t)n * 4, hipMemcpyHostToDevice));
    return CF_OK;
}

int cf_ens_get_table(cf_ensemble* e, int32_t t, float* dst, int64_t n) {
    if (!e || !dst) return cfi::set_error(CF_EINVAL, "null argument");
    int64_t want = 0;
    float* p = ens_table(e, t, &want);
    if (!p || n != want) return cfi::set_error(CF_EINVAL, "ensemble table size mismatch: want " + std::to_string(want));
    ENS_HIP(hipSetDevice(e->device));
    ENS_HIP(hipStreamSynchronize(e->stream));
    ENS_HIP(hipMemcpy(dst, p, (size_t)n * 4, hipMemcpyDeviceToHost));
    return CF_OK;
}

int cf_ens_set_interactions(cf_ensemble* e, const int64_t* indptr, const int32_t* indices, int64_t nnz) {
    if (!e || !indptr || (nnz > 0 && !indices)) return cfi::set_error(CF_EINVAL, "null CSR");
    if (indptr[0] != 0 || indptr[e->n_users] != nnz) return cfi::set_error(CF_EINVAL, "indptr does not span nnz");
    for (int64_t u = 0; u < e->n_users; ++u)
        for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k)
            if (indices[k] < 0 || indices[k] >= e->n_items || (k > indptr[u] && indices[k - 1] >= indices[k]))
                return cfi::set_error(CF_EINVAL, "CSR rows must hold sorted, unique, in-range items");
    ENS_HIP(hipSetDevice(e->device));
    ENS_HIP(hipStreamSynchronize(e->stream));
    efree(e->indptr);
    efree(e->indices);
    ENS_TRY(ealloc(&e->indptr, (size_t)e->n_users + 1));
    ENS_TRY(ealloc(&e->indices, (size_t)(nnz > 0 ? nnz : 1)));
    ENS_HIP(hipMemcpy(e->indptr, indptr, ((size_t)e->n_users + 1) * 8, hipMemcpyHostToDevice));
    if (nnz > 0) ENS_HIP(hipMemcpy(e->indices, indices, (size_t)nnz * 4, hipMemcpyHostToDevice));
    return CF_OK;
}

int cf_ens_step(cf_ensemble* e, const int32_t* uij, int32_t B, double* loss_out) {
    if (!e || !uij || B < 1) return cfi::set_error(CF_EINVAL, "bad arguments");
    // the reference loss is B x B (ensemble.py:84-91): 64 x 64 tiles over it
    if (B > (1 << 16)) return cfi::set_error(CF_EINVAL, "B must be <= 65536 (the loss is B x B)");
    for (int p = 0; p < B; ++p)
        if (uij[3 * p] < 0 || uij[3 * p] >= e->n_users || uij[3 * p + 1] < 0 ||
            uij[3 * p + 1] >= e->n_items || uij[3 * p + 2] < 0 || uij[3 * p + 2] >= e->n_items)
            return cfi::set_error(CF_EINVAL, "triplet " + std::to_string(p) + " out of range");
    ENS_HIP(hipSetDevice(e->device));
    const int K = e->K;
    const int npb = (B + kGroupsPerBlock - 1) / kGroupsPerBlock;
    const int nt = (B + kEnsTile - 1) / kEnsTile;
    if (B > e->Bcap) {
        ENS_HIP(hipStreamSynchronize(e->stream));
        efree(e->uij);
        efree(e->scratch);
        ENS_TRY(ealloc(&e->uij, (size_t)B * 3));
        ENS_TRY(ealloc(&e->scratch, (size_t)8 * K * B));
        e->Bcap = B;
    }
    const int nl = npb + nt * nt;
    if (nl > e->loss_cap) {
        ENS_HIP(hipStreamSynchronize(e->stream));
        efree(e->loss_partial);
        ENS_TRY(ealloc(&e->loss_partial, (size_t)nl));
        e->loss_cap = nl;
        e->h_loss.resize((size_t)nl);
    }
    ENS_HIP(hipMemcpyAsync(e->uij, uij, (size_t)B * 12, hipMemcpyHostToDevice, e->stream));
    EnsArgs a{};
    a.K = K; a.d = e->d; a.B = B;
    a.n_users = e->n_users; a.n_items = e->n_items; a.reg = e->reg;
    a.uij = e->uij; a.U = e->U; a.V = e->V; a.H = e->H;
    a.GU = e->GU; a.GV = e->GV; a.GH = e->GH;
    const size_t kb = (size_t)K * B;
    a.si = e->scratch; a.sj = a.si + kb; a.wi = a.sj + kb; a.wj = a.wi + kb;
    a.gsi = a.wj + kb; a.gsj = a.gsi + kb; a.gwi = a.gsj + kb; a.gwj = a.gwi + kb;
    a.loss_partial = e->loss_partial;
    a.loss_acc = e->loss_acc;
    a.n_pair_blocks = npb;
    ENS_HIP(hipMemsetAsync(a.gsi, 0, 4 * kb * 4, e->stream));
    hipLaunchKernelGGL(ens_pair_kernel, dim3(npb), dim3(kBlock), 0, e->stream, a);
    hipLaunchKernelGGL(ens_cross_kernel, dim3(nt, nt), dim3(kBlock), 0, e->stream, a);
    hipLaunchKernelGGL(ens_grad_kernel, dim3(npb), dim3(kBlock), (size_t)K * e->d * 4, e->stream, a);
    ENS_HIP(hipGetLastError());
    ENS_TRY(dense_apply(e, e->U, e->AU, e->GU, (int64_t)K * e->n_users));
    ENS_TRY(dense_apply(e, e->V, e->AV, e->GV, (int64_t)K * e->n_items));
    ENS_TRY(dense_apply(e, e->H, e->AH, e->GH, K));
    if (loss_out) {
        ENS_HIP(hipMemcpyAsync(e->h_loss.data(), e->loss_partial, (size_t)nl * 8, hipMemcpyDeviceToHost,
                               e->stream));
        ENS_HIP(hipStreamSynchronize(e->stream));
        double t = 0.0;
        for (int q = 0; q < nl; ++q) t += e->h_loss[(size_t)q];
        *loss_out = t;
    }
    return CF_OK;
}

int cf_ens_step_w(cf_ensemble* e, const int32_t* pairs, const int32_t* negs, int32_t W, int32_t B,
                  float lam, int32_t singles, double* loss_out) {
    if (!e || !pairs || !negs || B < 1) return cfi::set_error(CF_EINVAL, "bad arguments");
    if (W < 1 || W > kEnsMaxW) return cfi::set_error(CF_EINVAL, "W must be 1..8");
    for (int p = 0; p < B; ++p) {
        bool ok = pairs[2 * p] >= 0 && pairs[2 * p] < e->n_users && pairs[2 * p + 1] >= 0 &&
                  pairs[2 * p + 1] < e->n_items;
        for (int w = 0; w < W; ++w) ok = ok && negs[(size_t)p * W + w] >= 0 && negs[(size_t)p * W + w] < e->n_items;
        if (!ok) return cfi::set_error(CF_EINVAL, "pair " + std::to_string(p) + " out of range");
    }
    ENS_HIP(hipSetDevice(e->device));
    const int K = e->K;
    const int nb = (B + kGroupsPerBlock - 1) / kGroupsPerBlock;
    const size_t need = (size_t)B * (2 + W);
    if (need > (size_t)e->Bcap * 3) {   // reuse the uij buffer for [pairs | negs]
        ENS_HIP(hipStreamSynchronize(e->stream));
        efree(e->uij);
        efree(e->scratch);
        ENS_TRY(ealloc(&e->uij, need));
        ENS_TRY(ealloc(&e->scratch, (size_t)8 * K * ((need + 2) / 3)));
        e->Bcap = (int)((need + 2) / 3);
    }
    if (nb > e->loss_cap) {
        ENS_HIP(hipStreamSynchronize(e->stream));
        efree(e->loss_partial);
        ENS_TRY(ealloc(&e->loss_partial, (size_t)nb));
        e->loss_cap = nb;
        e->h_loss.resize((size_t)nb);
    }
    ENS_HIP(hipMemcpyAsync(e->uij, pairs, (size_t)B * 8, hipMemcpyHostToDevice, e->stream));
    ENS_HIP(hipMemcpyAsync(e->uij + 2 * (size_t)B, negs, (size_t)B * W * 4, hipMemcpyHostToDevice, e->stream));
    EnsWArgs a{};
    a.K = K; a.d = e->d; a.B = B; a.W = W; a.singles = singles ? 1 : 0;
    a.n_users = e->n_users; a.n_items = e->n_items;
    a.reg = e->reg; a.lam = lam;
    a.pairs = e->uij; a.negs = e->uij + 2 * (size_t)B;
    a.U = e->U; a.V = e->V; a.H = e->H;
    a.GU = e->GU; a.GV = e->GV; a.GH = e->GH;
    a.loss_partial = e->loss_partial;
    a.loss_acc = e->loss_acc;
    hipLaunchKernelGGL(ens_w_kernel, dim3(nb), dim3(kBlock), (size_t)K * e->d * 4, e->stream, a);
    ENS_HIP(hipGetLastError());
    ENS_TRY(dense_apply(e, e->U, e->AU, e->GU, (int64_t)K * e->n_users));
    ENS_TRY(dense_apply(e, e->V, e->AV, e->GV, (int64_t)K * e->n_items));
    ENS_TRY(dense_apply(e, e->H, e->AH, e->GH, K));
    if (loss_out) {
        ENS_HIP(hipMemcpyAsync(e->h_loss.data(), e->loss_partial, (size_t)nb * 8, hipMemcpyDeviceToHost,
                               e->stream));
        ENS_HIP(hipStreamSynchronize(e->stream));
        double t = 0.0;
        for (int q = 0; q < nb; ++q) t += e->h_loss[(size_t)q];
        *loss_out = t;
    }
    return CF_OK;
}

int cf_ens_take_loss(cf_ensemble* e, double* sum_out) {
    if (!e || !sum_out) return cfi::set_error(CF_EINVAL, "null argument");
    ENS_HIP(hipSetDevice(e->device));
    ENS_HIP(hipMemcpyAsync(sum_out, e->loss_acc, 8, hipMemcpyDeviceToHost, e->stream));
    ENS_HIP(hipMemsetAsync(e->loss_acc, 0, 8, e->stream));
    ENS_HIP(hipStreamSynchronize(e->stream));
    return CF_OK;
}

int cf_ens_score_topk(cf_ensemble* e, const int32_t* users, int32_t n, int32_t k, int32_t exclude_train,
                      int32_t* idx_out, float* val_out) {
    if (!e || n < 0 || !idx_out || (n > 0 && !users)) return cfi::set_error(CF_EINVAL, "bad arguments");
    if (k < 1 || k > 4096) return cfi::set_error(CF_EINVAL, "k must be 1..4096");
    if (exclude_train && !e->indptr) return cfi::set_error(CF_ESTATE, "exclude_train needs cf_ens_set_interactions");
    if (n == 0) return CF_OK;
    for (int r = 0; r < n; ++r)
        if (users[r] < 0 || users[r] >= e->n_users) return cfi::set_error(CF_EINVAL, "user id out of range");
    ENS_HIP(hipSetDevice(e->device));
    const size_t row_bytes = (size_t)e->n_items * 4;
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, ((size_t)256 << 20) / row_bytes));
    uint32_t* keys = nullptr;
    int32_t *d_users = nullptr, *d_idx = nullptr;
    float* d_val = nullptr;
    int r;
    if ((r = ealloc(&keys, (size_t)chunk * e->n_items)) || (r = ealloc(&d_users, (size_t)n)) ||
        (r = ealloc(&d_idx, (size_t)n * k)) || (r = ealloc(&d_val, (size_t)n * k))) {
        efree(keys); efree(d_users); efree(d_idx); efree(d_val);
        return r;
    }
    hipError_t he = hipMemcpyAsync(d_users, users, (size_t)n * 4, hipMemcpyHostToDevice, e->stream);
    for (int u0 = 0; he == hipSuccess && u0 < n; u0 += chunk) {
        const int m = std::min(chunk, n - u0);
        const dim3 grid((unsigned)((e->n_items + kBlock - 1) / kBlock), (unsigned)m);
        hipLaunchKernelGGL(ens_score_kernel, grid, dim3(kBlock), (size_t)2 * e->K * e->d * 4, e->stream,
                           e->K, e->d, e->n_users, e->n_items, d_users + u0, e->U, e->V, e->H, keys,
                           exclude_train, e->indptr, e->indices);
        he = hipGetLastError();
        if (he != hipSuccess) break;
        TopkArgs t{};
        t.k = k;
        t.n_items = e->n_items;
        t.keys = keys;
        t.idx_out = d_idx + (size_t)u0 * k;
        t.val_out = d_val + (size_t)u0 * k;
        he = launch_topk(t, m, e->stream);
    }
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he == hipSuccess) he = hipMemcpy(idx_out, d_idx, (size_t)n * k * 4, hipMemcpyDeviceToHost);
    if (he == hipSuccess && val_out) he = hipMemcpy(val_out, d_val, (size_t)n * k * 4, hipMemcpyDeviceToHost);
    efree(keys); efree(d_users); efree(d_idx); efree(d_val);
    if (he != hipSuccess) return cfi::set_error(CF_EHIP, std::string("cf_ens_score_topk: ") + hipGetErrorString(he));
    return CF_OK;
}

}  // extern "C"
