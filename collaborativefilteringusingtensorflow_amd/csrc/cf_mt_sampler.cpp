// cf_mt_sampler.cpp -- bit-exact host mode of the reference samplers
// (SURVEY 8(f) row 4).
//
// Reproduces, for a seed given to np.random.seed(seed) right before the
// reference sampler is built, the exact batch stream of
//   src/samplers/sampler_ranking.py:22-37      (kind 0)
//   src/samplers/sampler_uij_ranking.py:22-38  (kind 1, W = 1)
//   src/samplers/sampler_gbpr.py:23-43         (kind 2)
// on its producer side, by restating the algorithms of numpy's legacy
// RandomState (numpy/random/mtrand.pyx + src/mt19937, src/distributions):
//   * seed(s), s < 2^32: MT19937 init_genrand(s);
//   * shuffle(x) of the [nnz, 2] pair array: for i = n-1 .. 1, j =
//     random_interval(i) (masked rejection on next_uint32), swap rows i, j;
//   * randint(0, n[, size]) (int64, legacy => masked): rng = n - 1,
//     mask = smallest 2^k - 1 >= rng, redraw next_uint32 & mask while > rng;
//   * choice(list, G) with replacement, no p: randint(0, len, size=G), then
//     index the list.
// Stream order per batch: negatives randint (B, W); GBPR: the discarded
// group randint (B, G); then per pair, per negative, the rejection redraws,
// then (GBPR) the group choice.  Epochs re-shuffle the already shuffled pair
// array (np.random.shuffle in place, sampler_ranking.py:24) and yield
// floor(nnz / B) batches.  The consumer-side last-batch race of the
// reference's queue is not reproduced: this is the stream the
// producer computed.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cf_engine.h"

namespace cfi {
int set_error(int code, const std::string& msg);  // cf_engine.cpp
}

namespace {

struct MT19937 {
    uint32_t mt[624];
    int mti = 625;
    void seed(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        mti = 624;
    }
    uint32_t next32() {
        static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
        if (mti >= 624) {
            int k = 0;
            for (; k < 624 - 397; ++k) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
                mt[k] = mt[k + 397] ^ (y >> 1) ^ mag01[y & 1u];
            }
            for (; k < 623; ++k) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
                mt[k] = mt[k + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
            }
            const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
            mti = 0;
        }
        uint32_t y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    uint64_t next64() {
        const uint64_t hi = next32();
        return (hi << 32) | next32();
    }
};

inline uint64_t smear_mask(uint64_t m) {
    m |= m >> 1;
    m |= m >> 2;
    m |= m >> 4;
    m |= m >> 8;
    m |= m >> 16;
    m |= m >> 32;
    return m;
}

// random_interval(max): uniform in [0, max] by masked rejection
uint64_t random_interval(MT19937& g, uint64_t max) {
    if (max == 0) return 0;
    const uint64_t mask = smear_mask(max);
    uint64_t v;
    if (max <= 0xffffffffull) {
        while ((v = (g.next32() & mask)) > max) {
        }
    } else {
        while ((v = (g.next64() & mask)) > max) {
        }
    }
    return v;
}

// legacy randint(low, high) for one int64 element: masked bounded draw of
// rng = high - 1 - low (32-bit generator when rng fits 32 bits)
int64_t randint(MT19937& g, int64_t low, int64_t high) {
    const uint64_t rng = (uint64_t)(high - 1 - low);
    if (rng == 0) return low;
    if (rng <= 0xffffffffull) {
        if (rng == 0xffffffffull) return low + (int64_t)g.next32();
        const uint32_t mask = (uint32_t)smear_mask(rng);
        uint32_t v;
        while ((v = (g.next32() & mask)) > (uint32_t)rng) {
        }
        return low + (int64_t)v;
    }
    if (rng == 0xffffffffffffffffull) return low + (int64_t)g.next64();
    const uint64_t mask = smear_mask(rng);
    uint64_t v;
    while ((v = (g.next64() & mask)) > rng) {
    }
    return low + (int64_t)v;
}

}  // namespace

struct cf_mt_sampler {
    int kind = 0;
    int64_t n_users = 0, n_items = 0;
    int W = 1, G = 0, B = 1;
    std::vector<int64_t> indptr;
    std::vector<int32_t> indices;     // sorted rows: membership by binary search
    std::vector<int64_t> indptr_t;    // item -> users (sorted), GBPR
    std::vector<int32_t> indices_t;
    std::vector<int32_t> pairs;       // [nnz, 2], shuffled in place each epoch
    int64_t nnz = 0, per_epoch = 0, batch = 0, epoch = -1;
    MT19937 g;

    bool positive(int64_t u, int64_t j) const {
        const int32_t* b = indices.data() + indptr[(size_t)u];
        const int32_t* e = indices.data() + indptr[(size_t)u + 1];
        return std::binary_search(b, e, (int32_t)j);
    }
    void shuffle() {
        for (int64_t i = nnz - 1; i >= 1; --i) {
            const int64_t j = (int64_t)random_interval(g, (uint64_t)i);
            if (i == j) continue;
            std::swap(pairs[(size_t)(2 * i)], pairs[(size_t)(2 * j)]);
            std::swap(pairs[(size_t)(2 * i + 1)], pairs[(size_t)(2 * j + 1)]);
        }
    }
};

extern "C" {

int cf_mt_sampler_create(const int64_t* indptr, const int32_t* indices, int64_t n_users,
                         int64_t n_items, int32_t kind, int32_t n_neg, int32_t gsize,
                         int32_t batch_size, uint32_t seed, cf_mt_sampler** out) {
    if (!out || !indptr || n_users < 1 || n_items < 1 || kind < 0 || kind > 2 || batch_size < 1)
        return cfi::set_error(CF_EINVAL, "bad arguments");
    if (kind == 1) n_neg = 1;
    if (n_neg < 1 || (kind == 2 && gsize < 1)) return cfi::set_error(CF_EINVAL, "bad n_neg / gsize");
    const int64_t nnz = indptr[n_users];
    if (nnz < 1 || !indices) return cfi::set_error(CF_EINVAL, "no interactions");
    if (batch_size > nnz) return cfi::set_error(CF_EINVAL, "batch size exceeds the number of interactions");
    for (int64_t u = 0; u < n_users; ++u) {
        if (indptr[u + 1] < indptr[u]) return cfi::set_error(CF_EINVAL, "indptr not monotone");
        if (indptr[u + 1] - indptr[u] >= n_items)
            return cfi::set_error(CF_EINVAL, "a user has every item as a positive");
        for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k) {
            if (indices[k] < 0 || indices[k] >= n_items) return cfi::set_error(CF_EINVAL, "item id out of range");
            if (k > indptr[u] && indices[k - 1] >= indices[k])
                return cfi::set_error(CF_EINVAL, "CSR rows must be sorted, unique");
        }
    }
    cf_mt_sampler* s = new cf_mt_sampler();
    s->kind = kind;
    s->n_users = n_users;
    s->n_items = n_items;
    s->W = n_neg;
    s->G = kind == 2 ? gsize : 0;
    s->B = batch_size;
    s->nnz = nnz;
    s->per_epoch = nnz / batch_size;  // int(len(pairs) / batch_size), sampler_ranking.py:25
    s->indptr.assign(indptr, indptr + n_users + 1);
    s->indices.assign(indices, indices + nnz);
    // useritem_pairs = np.array(trasR.nonzero()).T: row-major, columns sorted
    s->pairs.resize((size_t)(2 * nnz));
    for (int64_t u = 0; u < n_users; ++u)
        for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k) {
            s->pairs[(size_t)(2 * k)] = (int32_t)u;
            s->pairs[(size_t)(2 * k + 1)] = indices[k];
        }
    if (kind == 2) {  // item_posUserList = trasR.transpose().rows (users ascending)
        s->indptr_t.assign((size_t)n_items + 1, 0);
        for (int64_t k = 0; k < nnz; ++k) s->indptr_t[(size_t)indices[k] + 1]++;
        for (int64_t i = 0; i < n_items; ++i) s->indptr_t[i + 1] += s->indptr_t[i];
        s->indices_t.resize((size_t)nnz);
        std::vector<int64_t> fill(s->indptr_t.begin(), s->indptr_t.end() - 1);
        for (int64_t u = 0; u < n_users; ++u)
            for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k)
                s->indices_t[(size_t)fill[(size_t)indices[k]]++] = (int32_t)u;
    }
    s->g.seed(seed);
    s->batch = s->per_epoch;  // the first next() shuffles
    *out = s;
    return CF_OK;
}

int cf_mt_sampler_next(cf_mt_sampler* s, int32_t* pairs, int32_t* negs, int32_t* groups) {
    if (!s || !pairs || !negs || (s->kind == 2 && !groups)) return cfi::set_error(CF_EINVAL, "bad arguments");
    if (s->batch >= s->per_epoch) {
        s->shuffle();  // np.random.shuffle(self.useritem_pairs), sampler_ranking.py:24
        s->batch = 0;
        s->epoch += 1;
    }
    const int B = s->B, W = s->W, G = s->G;
    const int32_t* src = s->pairs.data() + (size_t)(2 * s->batch * (int64_t)B);
    std::memcpy(pairs, src, (size_t)B * 2 * sizeof(int32_t));
    // negItems_batch = np.random.randint(0, n_items, size=(B, W))
    for (int64_t k = 0; k < (int64_t)B * W; ++k) negs[k] = (int32_t)randint(s->g, 0, s->n_items);
    // sampler_gbpr.py:34 draws a (B, G) block of users it later overwrites
    for (int64_t k = 0; k < (int64_t)B * G; ++k) (void)randint(s->g, 0, s->n_users);
    for (int p = 0; p < B; ++p) {
        const int64_t u = pairs[2 * p], i = pairs[2 * p + 1];
        for (int w = 0; w < W; ++w)
            while (s->positive(u, negs[(size_t)p * W + w]))
                negs[(size_t)p * W + w] = (int32_t)randint(s->g, 0, s->n_items);
        if (G > 0) {  // np.random.choice(item_posUserList[i], gsize)
            const int64_t cb = s->indptr_t[(size_t)i], ce = s->indptr_t[(size_t)i + 1];
            for (int k = 0; k < G; ++k)
                groups[(size_t)p * G + k] = s->indices_t[(size_t)(cb + randint(s->g, 0, ce - cb))];
        }
    }
    s->batch += 1;
    return CF_OK;
}

int cf_mt_sampler_state(const cf_mt_sampler* s, int64_t* epoch_out, int64_t* batch_out) {
    if (!s) return cfi::set_error(CF_EINVAL, "null sampler");
    if (epoch_out) *epoch_out = s->batch >= s->per_epoch ? s->epoch + 1 : s->epoch;
    if (batch_out) *batch_out = s->batch >= s->per_epoch ? 0 : s->batch;
    return CF_OK;
}

int cf_mt_sampler_free(cf_mt_sampler* s) {
    delete s;
    return CF_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Tuple samplers of the PRIGP / CPLR drop-ins (_tuple.py PRIGPSampler /
// UITJSampler, which restate src/samplers/sampler_prigp.py:24-52 and
// sampler_uitj_ranking.py:22-38 on a seeded RandomState): the same draws in
// the same order on the same legacy MT19937 stream, so a native sampler and
// its Python restatement yield identical batches for one seed.  The Python
// loops bound the tuple models' drivers at ~0.2M tuples/s; these run the
// identical stream natively.
// ---------------------------------------------------------------------------
namespace {

// legacy RandomState.random_sample(): 53-bit double from two 32-bit draws
double legacy_double(MT19937& g) {
    const int32_t a = (int32_t)(g.next32() >> 5), b = (int32_t)(g.next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

}  // namespace

struct cf_tuple_sampler {
    int kind = 0;  // 0 PRIGP (u,i,j,t,k), 1 CPLR (u,i,t,j) + coefs
    int64_t n_users = 0, n_items = 0;
    int B = 1;
    std::vector<int64_t> indptr, cindptr, utptr;
    std::vector<int32_t> indices, cindices, ut;    // train rows, coefficient rows, coef-only items
    std::vector<double> cvalues;
    std::vector<int32_t> nvals;                     // distinct coefficient values per user
    std::vector<uint8_t> valid;                     // CPLR: user can be drawn
    std::vector<int32_t> pairs;
    int64_t nnz = 0, per_epoch = 0, batch = 0;
    MT19937 g;
    bool has_gauss = false;
    double gauss = 0.0;

    static bool in(const std::vector<int32_t>& v, int64_t b, int64_t e, int32_t x) {
        return std::binary_search(v.begin() + b, v.begin() + e, x);
    }
    double randn() {  // legacy_gauss: polar Box-Muller, second value cached
        if (has_gauss) {
            has_gauss = false;
            return gauss;
        }
        double x1, x2, r2;
        do {
            x1 = 2.0 * legacy_double(g) - 1.0;
            x2 = 2.0 * legacy_double(g) - 1.0;
            r2 = x1 * x1 + x2 * x2;
        } while (r2 >= 1.0 || r2 == 0.0);
        const double f = std::sqrt(-2.0 * std::log(r2) / r2);
        gauss = f * x1;
        has_gauss = true;
        return f * x2;
    }
    double coef(int64_t u, int32_t x) const {
        const auto b = cindices.begin() + cindptr[(size_t)u], e = cindices.begin() + cindptr[(size_t)u + 1];
        const auto it = std::lower_bound(b, e, x);
        return (it != e && *it == x) ? cvalues[(size_t)(it - cindices.begin())] : 0.0;
    }
};

extern "C" {

int cf_tuple_sampler_create(int32_t kind, const int64_t* indptr, const int32_t* indices,
                            int64_t n_users, int64_t n_items, const int64_t* coef_indptr,
                            const int32_t* coef_indices, const double* coef_values,
                            int32_t batch_size, uint32_t seed, cf_tuple_sampler** out) {
    if (!out || !indptr || !coef_indptr || n_users < 1 || n_items < 2 || kind < 0 || kind > 1 ||
        batch_size < 1)
        return cfi::set_error(CF_EINVAL, "bad arguments");
    const int64_t nnz = indptr[n_users], cnnz = coef_indptr[n_users];
    if (nnz < 1 || !indices || (cnnz > 0 && (!coef_indices || !coef_values)))
        return cfi::set_error(CF_EINVAL, "no interactions / coefficients");
    for (int pass = 0; pass < 2; ++pass) {
        const int64_t* ip = pass ? coef_indptr : indptr;
        const int32_t* ix = pass ? coef_indices : indices;
        for (int64_t u = 0; u < n_users; ++u) {
            if (ip[u + 1] < ip[u]) return cfi::set_error(CF_EINVAL, "indptr not monotone");
            for (int64_t k = ip[u]; k < ip[u + 1]; ++k)
                if (ix[k] < 0 || ix[k] >= n_items || (k > ip[u] && ix[k - 1] >= ix[k]))
                    return cfi::set_error(CF_EINVAL, "CSR rows must hold sorted, unique, in-range ids");
        }
    }
    cf_tuple_sampler* s = new cf_tuple_sampler();
    s->kind = kind;
    s->n_users = n_users;
    s->n_items = n_items;
    s->B = batch_size;
    s->nnz = nnz;
    s->indptr.assign(indptr, indptr + n_users + 1);
    s->indices.assign(indices, indices + nnz);
    s->cindptr.assign(coef_indptr, coef_indptr + n_users + 1);
    s->cindices.assign(coef_indices, coef_indices + cnnz);
    s->cvalues.assign(coef_values, coef_values + cnnz);
    s->nvals.assign((size_t)n_users, 0);
    for (int64_t u = 0; u < n_users; ++u) {  // len(set(values of row u))
        std::vector<double> v(coef_values + coef_indptr[u], coef_values + coef_indptr[u + 1]);
        std::sort(v.begin(), v.end());
        s->nvals[(size_t)u] = (int32_t)(std::unique(v.begin(), v.end()) - v.begin());
    }
    if (kind == 0) {
        if (batch_size > nnz) {
            delete s;
            return cfi::set_error(CF_EINVAL, "batch size exceeds the number of interactions");
        }
        s->per_epoch = nnz / batch_size;
        s->pairs.resize((size_t)(2 * nnz));   // np.array(R.nonzero()).T
        for (int64_t u = 0; u < n_users; ++u)
            for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k) {
                s->pairs[(size_t)(2 * k)] = (int32_t)u;
                s->pairs[(size_t)(2 * k + 1)] = indices[k];
            }
        s->batch = s->per_epoch;  // the first next() shuffles
    } else {
        // ut[u] = sorted(coef items of u that are not train items of u)
        s->utptr.assign((size_t)n_users + 1, 0);
        s->valid.assign((size_t)n_users, 0);
        bool any = false;
        for (int64_t u = 0; u < n_users; ++u) {
            for (int64_t k = coef_indptr[u]; k < coef_indptr[u + 1]; ++k)
                if (!cf_tuple_sampler::in(s->indices, indptr[u], indptr[u + 1], coef_indices[k]))
                    s->ut.push_back(coef_indices[k]);
            s->utptr[(size_t)u + 1] = (int64_t)s->ut.size();
            const int64_t nui = indptr[u + 1] - indptr[u], nut = s->utptr[u + 1] - s->utptr[u];
            s->valid[(size_t)u] = nui > 0 && nut > 0 && nui + nut < n_items;
            any = any || s->valid[(size_t)u];
        }
        if (!any) {
            delete s;
            return cfi::set_error(CF_EINVAL, "no user has both train and coefficient-only items");
        }
    }
    s->g.seed(seed);
    *out = s;
    return CF_OK;
}

int cf_tuple_sampler_next(cf_tuple_sampler* s, int32_t* tuples, float* coefs) {
    if (!s || !tuples || (s->kind == 1 && !coefs)) return cfi::set_error(CF_EINVAL, "bad arguments");
    const int B = s->B;
    MT19937& g = s->g;
    const int64_t ni = s->n_items;
    if (s->kind == 0) {  // PRIGPSampler.next_batch
        if (s->batch >= s->per_epoch) {
            for (int64_t i = s->nnz - 1; i >= 1; --i) {  // rng.shuffle(self.pairs)
                const int64_t j = (int64_t)random_interval(g, (uint64_t)i);
                if (i == j) continue;
                std::swap(s->pairs[(size_t)(2 * i)], s->pairs[(size_t)(2 * j)]);
                std::swap(s->pairs[(size_t)(2 * i + 1)], s->pairs[(size_t)(2 * j + 1)]);
            }
            s->batch = 0;
        }
        const int32_t* src = s->pairs.data() + (size_t)(2 * s->batch * (int64_t)B);
        for (int p = 0; p < B; ++p) {
            tuples[5 * p] = src[2 * p];
            tuples[5 * p + 1] = src[2 * p + 1];
        }
        for (int p = 0; p < B; ++p) tuples[5 * p + 2] = (int32_t)randint(g, 0, ni);  // randint(0, n, B)
        s->batch += 1;
        for (int p = 0; p < B; ++p) {
            const int64_t u = tuples[5 * p];
            const int32_t i = tuples[5 * p + 1];
            int32_t j = tuples[5 * p + 2];
            while (cf_tuple_sampler::in(s->indices, s->indptr[u], s->indptr[u + 1], j))
                j = (int32_t)randint(g, 0, ni);
            int32_t t = i, k = j;
            const int64_t cb = s->cindptr[(size_t)u], ce = s->cindptr[(size_t)u + 1];
            const int nv = s->nvals[(size_t)u];
            if (nv > 0) {
                const int64_t len = ce - cb;
                t = s->cindices[(size_t)(cb + randint(g, 0, len))];
                k = (int32_t)randint(g, 0, ni);
                while (cf_tuple_sampler::in(s->cindices, cb, ce, k)) k = (int32_t)randint(g, 0, ni);
                if (nv > 1 && s->randn() < (double)len / (double)ni) {
                    k = s->cindices[(size_t)(cb + randint(g, 0, len))];
                    while (s->coef(u, t) == s->coef(u, k)) k = s->cindices[(size_t)(cb + randint(g, 0, len))];
                    if (s->coef(u, t) < s->coef(u, k)) std::swap(t, k);
                }
            }
            tuples[5 * p + 2] = j;
            tuples[5 * p + 3] = t;
            tuples[5 * p + 4] = k;
        }
        return CF_OK;
    }
    for (int p = 0; p < B; ++p) {  // UITJSampler.next_batch
        int64_t u = randint(g, 0, s->n_users);
        while (!s->valid[(size_t)u]) u = randint(g, 0, s->n_users);
        const int64_t ib = s->indptr[(size_t)u], ie = s->indptr[(size_t)u + 1];
        const int64_t tb = s->utptr[(size_t)u], te = s->utptr[(size_t)u + 1];
        const int32_t i = s->indices[(size_t)(ib + randint(g, 0, ie - ib))];
        const int32_t t = s->ut[(size_t)(tb + randint(g, 0, te - tb))];
        int32_t j = (int32_t)randint(g, 0, ni);
        while (cf_tuple_sampler::in(s->indices, ib, ie, j) || cf_tuple_sampler::in(s->ut, tb, te, j))
            j = (int32_t)randint(g, 0, ni);
        tuples[4 * p] = (int32_t)u;
        tuples[4 * p + 1] = i;
        tuples[4 * p + 2] = t;
        tuples[4 * p + 3] = j;
        coefs[2 * p] = (float)s->coef(u, i);
        coefs[2 * p + 1] = (float)s->coef(u, t);
    }
    return CF_OK;
}

int cf_tuple_sampler_free(cf_tuple_sampler* s) {
    delete s;
    return CF_OK;
}

}  // extern "C"
