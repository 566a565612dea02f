/*
 * cf_oracle.c -- CPU ORACLE in plain C.  TEST INFRASTRUCTURE, NOT PRODUCT.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this (oracle/build/libcf_oracle.so).  It restates the same TF1 semantics
 * as oracle/cf_oracle.py (which tests cross-check it against), single-
 * threaded, plus an OpenMP trainer (oracle_train_mt) for the all-cores CPU
 * baseline of SURVEY 8(d):
 *   BPRMF  src/models/pl/models/bprmf.py:52-88
 *   GBPRMF src/models/pl/models/gbprmf.py:58-106
 *   CML    src/models/pl/models/cml.py:55-129   (full-table clip every step)
 *   AMF    src/models/others/models/amf.py:66-162 (reference mode, Δ = 0)
 * with duplicate-row gradients summed before one SparseApplyAdagrad per
 * touched row (acc += g^2; w -= lr*g/sqrt(acc)).  Dense fp32 gradient
 * accumulators + touched-row lists implement the dedup.
 *
 * It also restates the sampler (epoch bijection over the nnz pairs, W
 * negatives redrawn while in Pos(u)) so that the CPU baseline times the same
 * end-to-end work unit as the GPU path: sample + forward + backward + dedup
 * + Adagrad.  Parity status: see oracle/cf_oracle.py ("parity unpinned" for
 * the TF arithmetic itself).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int model; /* 0 BPR, 1 GBPR, 2 CML, 3 AMF */
    int d, W, G;
    int64_t n_users, n_items;
    float lr, reg, rho, margin, reg_cov, clip_norm, reg_adv;
    int use_rank_weight, adversarial;
} oracle_cfg;

typedef struct {
    float *U, *V, *b, *AU, *AV, *Ab;
    float *GU, *GV, *Gb;          /* zeroed dense accumulators (caller-owned) */
    uint8_t *tU, *tV;             /* touched flags, zeroed */
    int32_t *listU, *listV;       /* touched lists, capacity >= occurrences */
} oracle_state;

static float sigm(float x) { return 1.f / (1.f + expf(-x)); }
static float softplusf(float x) { return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x)); }

static void touch(uint8_t* t, int32_t* list, int* n, int32_t r) {
    if (!t[r]) { t[r] = 1; list[(*n)++] = r; }
}

static void adagrad_rows(float* X, float* A, float* G, uint8_t* t, const int32_t* list, int n,
                         int d, float lr) {
    for (int k = 0; k < n; ++k) {
        const int64_t r = list[k];
        float* x = X + r * d; float* a = A + r * d; float* g = G + r * d;
        for (int e = 0; e < d; ++e) {
            a[e] += g[e] * g[e];
            x[e] -= (lr * g[e]) / sqrtf(a[e]);
            g[e] = 0.f;
        }
        t[r] = 0;
    }
}

static void clip_all(float* X, int64_t n, int d, float c) {
    for (int64_t r = 0; r < n; ++r) {
        float* x = X + r * d;
        double s = 0.0;
        for (int e = 0; e < d; ++e) s += (double)x[e] * x[e];
        const float nrm = sqrtf((float)s);
        const float den = nrm > c ? nrm : c;
        for (int e = 0; e < d; ++e) x[e] = (x[e] * c) / den;
    }
}

static float dotf(const float* a, const float* b, int d) {
    float s = 0.f;
    for (int e = 0; e < d; ++e) s += a[e] * b[e];
    return s;
}

/* one step on a host batch; returns the pre-update loss */
double oracle_step(const oracle_cfg* c, oracle_state* s, const int32_t* pairs,
                   const int32_t* negs, const int32_t* groups, int B) {
    const int d = c->d, W = c->W, G = c->model == 1 ? c->G : 0;
    double loss = 0.0, sq = 0.0;
    int nU = 0, nV = 0;
    float* gu = (float*)calloc((size_t)d, sizeof(float));
    float* sg = (float*)calloc((size_t)d, sizeof(float));
    float* dn = (float*)calloc((size_t)W, sizeof(float));
    for (int p = 0; p < B; ++p) {
        const int32_t u = pairs[2 * p], i = pairs[2 * p + 1];
        const float* uu = s->U + (int64_t)u * d;
        const float* vi = s->V + (int64_t)i * d;
        float* GUu = s->GU + (int64_t)u * d;
        float* GVi = s->GV + (int64_t)i * d;
        touch(s->tU, s->listU, &nU, u);
        touch(s->tV, s->listV, &nV, i);
        memset(gu, 0, (size_t)d * sizeof(float));
        if (c->model == 0 || c->model == 3) {
            const float ui = dotf(uu, vi, d);
            float sc = 0.f;
            for (int w = 0; w < W; ++w) {
                const int32_t j = negs[(int64_t)p * W + w];
                const float* vj = s->V + (int64_t)j * d;
                float* GVj = s->GV + (int64_t)j * d;
                touch(s->tV, s->listV, &nV, j);
                const float x = ui - dotf(uu, vj, d);
                float cc = sigm(x) - 1.f;
                if (c->model == 3) {
                    loss += softplusf(-x);
                    if (c->adversarial) {
                        const float xc = fmaxf(fminf(x, 1e8f), -80.f);
                        loss += c->reg_adv * softplusf(-xc);
                        if (x >= -80.f && x <= 1e8f) cc *= (1.f + c->reg_adv);
                    }
                } else {
                    loss += -log(sigm(x));
                }
                sc += cc;
                for (int e = 0; e < d; ++e) {
                    gu[e] += cc * (vi[e] - vj[e]);
                    GVj[e] += -cc * uu[e] + c->reg * vj[e];
                    sq += (double)vj[e] * vj[e];
                }
            }
            for (int e = 0; e < d; ++e) {
                GUu[e] += gu[e] + c->reg * uu[e];
                GVi[e] += sc * uu[e] + c->reg * vi[e];
                sq += (double)uu[e] * uu[e] + (double)vi[e] * vi[e];
            }
        } else if (c->model == 1) {
            const float ui_u = dotf(uu, vi, d);
            memset(sg, 0, (size_t)d * sizeof(float));
            for (int k = 0; k < G; ++k) {
                const int32_t g = groups[(int64_t)p * G + k];
                const float* ug = s->U + (int64_t)g * d;
                touch(s->tU, s->listU, &nU, g);
                for (int e = 0; e < d; ++e) { sg[e] += ug[e]; sq += (double)ug[e] * ug[e]; }
            }
            const float ui = c->rho * (dotf(sg, vi, d) / (float)G) + (1.f - c->rho) * ui_u + s->b[i];
            float sc = 0.f;
            for (int w = 0; w < W; ++w) {
                const int32_t j = negs[(int64_t)p * W + w];
                const float* vj = s->V + (int64_t)j * d;
                float* GVj = s->GV + (int64_t)j * d;
                touch(s->tV, s->listV, &nV, j);
                const float bj = s->b[j];
                const float x = ui - (dotf(uu, vj, d) + bj);
                const float cc = sigm(x) - 1.f;
                loss += -log(sigm(x)) + 0.5 * c->reg * bj * bj;
                sc += cc;
                for (int e = 0; e < d; ++e) { gu[e] -= cc * vj[e]; GVj[e] += -cc * uu[e]; }
                s->Gb[j] += -cc + c->reg * bj;
            }
            const float rg = c->rho / (float)G;
            for (int e = 0; e < d; ++e) {
                GUu[e] += gu[e] + (1.f - c->rho) * sc * vi[e] + c->reg * uu[e];
                GVi[e] += sc * (rg * sg[e] + (1.f - c->rho) * uu[e]) + c->reg * vi[e];
                sq += (double)uu[e] * uu[e] + (double)vi[e] * vi[e];
            }
            for (int k = 0; k < G; ++k) {
                const int32_t g = groups[(int64_t)p * G + k];
                const float* ug = s->U + (int64_t)g * d;
                float* GUg = s->GU + (int64_t)g * d;
                for (int e = 0; e < d; ++e) GUg[e] += rg * sc * vi[e] + c->reg * ug[e];
            }
            s->Gb[i] += sc;
        } else { /* CML */
            float dp = 0.f, m = INFINITY;
            int imp = 0;
            for (int e = 0; e < d; ++e) dp += (uu[e] - vi[e]) * (uu[e] - vi[e]);
            for (int w = 0; w < W; ++w) {
                const float* vj = s->V + (int64_t)negs[(int64_t)p * W + w] * d;
                float t = 0.f;
                for (int e = 0; e < d; ++e) t += (uu[e] - vj[e]) * (uu[e] - vj[e]);
                dn[w] = t;
                if (t < m) m = t;
                imp += (dp - t + c->margin > 0.f);
            }
            int cnt = 0;
            for (int w = 0; w < W; ++w) cnt += (dn[w] == m);
            const float z = dp - m + c->margin;
            const float lw = c->use_rank_weight ? logf((float)imp / (float)W * (float)c->n_items + 1.f) : 1.f;
            loss += (z > 0.f ? z : 0.f) * lw;
            const float aa = z > 0.f ? lw : 0.f;
            const int l2 = c->reg_cov > 0.f;
            for (int e = 0; e < d; ++e) {
                gu[e] = 2.f * aa * (uu[e] - vi[e]);
                GVi[e] += -2.f * aa * (uu[e] - vi[e]) + (l2 ? c->reg_cov * vi[e] : 0.f);
                if (l2) sq += (double)uu[e] * uu[e] + (double)vi[e] * vi[e];
            }
            for (int w = 0; w < W; ++w) {
                const int32_t j = negs[(int64_t)p * W + w];
                const float* vj = s->V + (int64_t)j * d;
                float* GVj = s->GV + (int64_t)j * d;
                touch(s->tV, s->listV, &nV, j);
                const float coef = (dn[w] == m) ? 2.f * aa / (float)cnt : 0.f;
                for (int e = 0; e < d; ++e) {
                    const float dv = uu[e] - vj[e];
                    gu[e] -= coef * dv;
                    GVj[e] += coef * dv + (l2 ? c->reg_cov * vj[e] : 0.f);
                    if (l2) sq += (double)vj[e] * vj[e];
                }
            }
            for (int e = 0; e < d; ++e) GUu[e] += gu[e] + (l2 ? c->reg_cov * uu[e] : 0.f);
        }
    }
    const float coefL2 = c->model == 2 ? (c->reg_cov > 0.f ? c->reg_cov : 0.f) : c->reg;
    loss += 0.5 * coefL2 * sq;
    if (c->model == 1) {
        for (int k = 0; k < nV; ++k) {
            const int32_t r = s->listV[k];
            const float g = s->Gb[r];
            s->Ab[r] += g * g;
            s->b[r] -= (c->lr * g) / sqrtf(s->Ab[r]);
            s->Gb[r] = 0.f;
        }
    }
    adagrad_rows(s->U, s->AU, s->GU, s->tU, s->listU, nU, d, c->lr);
    adagrad_rows(s->V, s->AV, s->GV, s->tV, s->listV, nV, d, c->lr);
    if (c->model == 2) {
        clip_all(s->U, c->n_users, d, c->clip_norm);
        clip_all(s->V, c->n_items, d, c->clip_norm);
    }
    free(gu); free(sg); free(dn);
    return loss;
}

/* ---- sampler restatement (for the CPU baseline) ------------------------------ */
static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int contains(const int32_t* a, int64_t lo, int64_t hi, int32_t key) {
    const int64_t end = hi;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo < end && a[lo] == key;
}

/*
 * n_steps of sample + step (BPR/AMF/CML, W negatives) on a CSR graph:
 * batch b of epoch e takes pairs perm_e(b*B .. b*B+B-1), perm_e = a keyed
 * bijection (xor/multiply/xorshift rounds, cycle-walked).  pairs_coo is the
 * nnz-ordered (u,i) list.  Returns the summed pre-update loss.
 */
/* batch b of epoch e: pairs perm_e(b*B .. b*B+B-1) and W rejected-in-Pos(u)
 * negatives per pair, for pairs [p0, p1) of the batch */
typedef struct {
    uint64_t k[3], mul[3], mask;
    int shift;
} oracle_perm;

static void perm_init(oracle_perm* pm, int64_t nnz, uint64_t seed, int64_t epoch) {
    int bits = 1;
    while (bits < 63 && (1ull << bits) < (uint64_t)nnz) ++bits;
    pm->mask = (1ull << bits) - 1ull;
    pm->shift = bits / 2 > 0 ? bits / 2 : 1;
    uint64_t h = mix64(seed ^ mix64((uint64_t)epoch + 0x5851F42D4C957F2Dull));
    for (int r = 0; r < 3; ++r) {
        h = mix64(h + (uint64_t)r);
        pm->k[r] = h & pm->mask;
        pm->mul[r] = mix64(h ^ 0xA0761D6478BD642Full) | 1ull;
    }
}

static void draw_pairs(const oracle_cfg* c, const oracle_perm* pm, const int64_t* indptr,
                       const int32_t* indices, const int32_t* pairs_coo, int64_t nnz, int B,
                       int64_t batch, int64_t epoch, uint64_t seed, int p0, int p1,
                       int32_t* batch_pairs, int32_t* batch_negs) {
    for (int p = p0; p < p1; ++p) {
        uint64_t x = (uint64_t)(batch * B + p);
        do {
            for (int r = 0; r < 3; ++r) {
                x = (x ^ pm->k[r]) & pm->mask;
                x = (x * pm->mul[r]) & pm->mask;
                x ^= x >> pm->shift;
            }
        } while (x >= (uint64_t)nnz);
        const int32_t u = pairs_coo[2 * x], i = pairs_coo[2 * x + 1];
        batch_pairs[2 * p] = u;
        batch_pairs[2 * p + 1] = i;
        const uint64_t key = mix64(seed ^ ((uint64_t)(batch * B + p) * 0xD1B54A32D192ED03ull) ^ (uint64_t)epoch);
        for (int w = 0; w < c->W; ++w) {
            uint64_t ctr = (uint64_t)w << 32;
            int32_t j;
            do {
                j = (int32_t)(((unsigned __int128)mix64(key + ctr) * (uint64_t)c->n_items) >> 64);
                ++ctr;
            } while (contains(indices, indptr[u], indptr[u + 1], j));
            batch_negs[(int64_t)p * c->W + w] = j;
        }
    }
}

/*
 * n_steps of sample + step (BPR/AMF/CML, W negatives) on a CSR graph:
 * batch b of epoch e takes pairs perm_e(b*B .. b*B+B-1), perm_e = a keyed
 * bijection (xor/multiply/xorshift rounds, cycle-walked).  pairs_coo is the
 * nnz-ordered (u,i) list.  Returns the summed pre-update loss.
 */
double oracle_train(const oracle_cfg* c, oracle_state* s, const int64_t* indptr,
                    const int32_t* indices, const int32_t* pairs_coo, int64_t nnz, int B,
                    int n_steps, uint64_t seed, int32_t* batch_pairs, int32_t* batch_negs) {
    double total = 0.0;
    const int64_t per_epoch = nnz / B;
    int64_t epoch = 0, batch = 0;
    oracle_perm pm;
    perm_init(&pm, nnz, seed, 0);
    for (int st = 0; st < n_steps; ++st) {
        if (batch >= per_epoch) { ++epoch; batch = 0; perm_init(&pm, nnz, seed, epoch); }
        draw_pairs(c, &pm, indptr, indices, pairs_coo, nnz, B, batch, epoch, seed, 0, B,
                   batch_pairs, batch_negs);
        total += oracle_step(c, s, batch_pairs, batch_negs, NULL, B);
        ++batch;
    }
    return total;
}

/*
 * The same work unit on n_threads cores (BPR / AMF): the draw and the
 * per-pair forward/backward run over pair ranges; each occurrence's gradient
 * row goes to its own slot; then thread t sums the slots of the rows it owns
 * (row % n_threads == t) in occurrence order and applies Adagrad to them --
 * the dedup-sum of the single-thread step, partitioned by row.  Returns the
 * summed pre-update loss (-1 for a model it does not cover).
 */
double oracle_train_mt(const oracle_cfg* c, oracle_state* s, const int64_t* indptr,
                       const int32_t* indices, const int32_t* pairs_coo, int64_t nnz, int B,
                       int n_steps, uint64_t seed, int32_t* batch_pairs, int32_t* batch_negs,
                       int n_threads) {
    if (c->model != 0 && c->model != 3) return -1.0;
    const int d = c->d, W = c->W, S = 2 + W;
    const int T = n_threads > 0 ? n_threads : 1;
    float* og = (float*)malloc((size_t)B * S * d * sizeof(float));
    int32_t* lists = (int32_t*)malloc((size_t)T * B * S * sizeof(int32_t));
    double* part = (double*)calloc((size_t)T * 8, sizeof(double));
    if (!og || !lists || !part) { free(og); free(lists); free(part); return -2.0; }
    double total = 0.0;
    const int64_t per_epoch = nnz / B;
    int64_t epoch = 0, batch = 0;
    oracle_perm pm;
    perm_init(&pm, nnz, seed, 0);
    for (int st = 0; st < n_steps; ++st) {
        if (batch >= per_epoch) { ++epoch; batch = 0; perm_init(&pm, nnz, seed, epoch); }
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num(), nt = omp_get_num_threads();
            const int p0 = (int)((int64_t)B * t / nt), p1 = (int)((int64_t)B * (t + 1) / nt);
            draw_pairs(c, &pm, indptr, indices, pairs_coo, nnz, B, batch, epoch, seed, p0, p1,
                       batch_pairs, batch_negs);
            double loss = 0.0, sq = 0.0;
            for (int p = p0; p < p1; ++p) {
                const int32_t u = batch_pairs[2 * p], i = batch_pairs[2 * p + 1];
                const float* uu = s->U + (int64_t)u * d;
                const float* vi = s->V + (int64_t)i * d;
                float* gu = og + ((size_t)p * S) * d;
                float* gi = gu + d;
                const float ui = dotf(uu, vi, d);
                float sc = 0.f;
                for (int e = 0; e < d; ++e) gu[e] = 0.f;
                for (int w = 0; w < W; ++w) {
                    const int32_t j = batch_negs[(int64_t)p * W + w];
                    const float* vj = s->V + (int64_t)j * d;
                    float* gj = gu + (size_t)(2 + w) * d;
                    const float x = ui - dotf(uu, vj, d);
                    float cc = sigm(x) - 1.f;
                    if (c->model == 3) {
                        loss += softplusf(-x);
                        if (c->adversarial) {
                            const float xc = fmaxf(fminf(x, 1e8f), -80.f);
                            loss += c->reg_adv * softplusf(-xc);
                            if (x >= -80.f && x <= 1e8f) cc *= (1.f + c->reg_adv);
                        }
                    } else {
                        loss += -log(sigm(x));
                    }
                    sc += cc;
                    for (int e = 0; e < d; ++e) {
                        gu[e] += cc * (vi[e] - vj[e]);
                        gj[e] = -cc * uu[e] + c->reg * vj[e];
                        sq += (double)vj[e] * vj[e];
                    }
                }
                for (int e = 0; e < d; ++e) {
                    gu[e] += c->reg * uu[e];
                    gi[e] = sc * uu[e] + c->reg * vi[e];
                    sq += (double)uu[e] * uu[e] + (double)vi[e] * vi[e];
                }
            }
            part[8 * t] = loss + 0.5 * c->reg * sq;
#pragma omp barrier
            /* every table row belongs to thread row % nt: sum its slots, apply */
            int32_t* lu = lists + (size_t)t * B * S;
            int nu = 0, nv = 0;
            int32_t* lv = lu + B;
            for (int p = 0; p < B; ++p) {
                const int32_t u = batch_pairs[2 * p];
                if (u % nt == t) {
                    float* G = s->GU + (int64_t)u * d;
                    const float* g = og + ((size_t)p * S) * d;
                    if (!s->tU[u]) { s->tU[u] = 1; lu[nu++] = u; }
                    for (int e = 0; e < d; ++e) G[e] += g[e];
                }
                for (int k = 1; k < S; ++k) {
                    const int32_t r = k == 1 ? batch_pairs[2 * p + 1] : batch_negs[(int64_t)p * W + k - 2];
                    if (r % nt != t) continue;
                    float* G = s->GV + (int64_t)r * d;
                    const float* g = og + ((size_t)p * S + k) * d;
                    if (!s->tV[r]) { s->tV[r] = 1; lv[nv++] = r; }
                    for (int e = 0; e < d; ++e) G[e] += g[e];
                }
            }
            adagrad_rows(s->U, s->AU, s->GU, s->tU, lu, nu, d, c->lr);
            adagrad_rows(s->V, s->AV, s->GV, s->tV, lv, nv, d, c->lr);
        }
        for (int t = 0; t < T; ++t) total += part[8 * t];
        ++batch;
    }
    free(og); free(lists); free(part);
    return total;
}
