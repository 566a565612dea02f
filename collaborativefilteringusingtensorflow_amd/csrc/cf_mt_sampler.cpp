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
