// cf_synth.cpp -- synthetic implicit-feedback graphs for the benchmark
// configurations of SURVEY 8(d): per-user degree 1 + Poisson(mean-1), items
// drawn without replacement from a Zipf(s) popularity over a seeded random
// item permutation.  Every user's row depends only on (seed, user id), so a
// rank that owns users [u_begin, u_end) regenerates exactly its shard.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cf_engine.h"

namespace {

inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline double u01(uint64_t h) { return ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

int64_t poisson(double lam, uint64_t key) {
    // inversion; lam is small (tens), exp(-lam) stays representable below ~700
    if (lam <= 0.0) return 0;
    double u = u01(mix64(key));
    double p = std::exp(-lam), F = p;
    int64_t k = 0;
    while (u > F && k < 100000) {
        ++k;
        p *= lam / (double)k;
        F += p;
        if (p == 0.0) break;
    }
    return k;
}

}  // namespace

extern "C" {

int cf_synth_degrees(int64_t n_users, double mean_degree, uint64_t seed, int64_t u_begin,
                     int64_t u_end, int64_t* indptr_out) {
    if (!indptr_out || u_begin < 0 || u_end < u_begin || u_end > n_users || mean_degree < 1.0)
        return CF_EINVAL;
    indptr_out[0] = 0;
    const uint64_t key = mix64(seed ^ 0xD6E8FEB86659FD93ull);
    for (int64_t u = u_begin; u < u_end; ++u) {
        const int64_t deg = 1 + poisson(mean_degree - 1.0, key ^ mix64((uint64_t)u));
        indptr_out[u - u_begin + 1] = indptr_out[u - u_begin] + deg;
    }
    return CF_OK;
}

}  // extern "C"

namespace {

// the item side of the generator: Zipf CDF over popularity ranks and the
// seeded rank -> item permutation; row(u) is user u's sorted item list
struct ItemGen {
    int64_t n_items;
    std::vector<double> cdf;
    std::vector<int32_t> perm;
    uint64_t ikey;

    ItemGen(int64_t n, double zipf_s, uint64_t seed) : n_items(n), cdf((size_t)n), perm((size_t)n) {
        double acc = 0.0;
        for (int64_t r = 0; r < n; ++r) {
            acc += std::pow((double)(r + 1), -zipf_s);
            cdf[(size_t)r] = acc;
        }
        for (auto& v : cdf) v /= acc;
        cdf.back() = 1.0;
        for (int64_t i = 0; i < n; ++i) perm[(size_t)i] = (int32_t)i;
        const uint64_t pkey = mix64(seed ^ 0x9FB21C651E98DF25ull);
        for (int64_t i = n - 1; i > 0; --i) {
            const uint64_t j = (uint64_t)(u01(mix64(pkey + (uint64_t)i)) * (double)(i + 1));
            std::swap(perm[(size_t)i], perm[(size_t)std::min<uint64_t>(j, (uint64_t)i)]);
        }
        ikey = mix64(seed ^ 0x2D358DCCAA6C78A5ull);
    }

    // deg distinct items drawn from the popularity, sorted; false if impossible
    bool row(int64_t u, int64_t deg, std::vector<int32_t>& out) const {
        out.clear();
        if (deg >= n_items) return false;
        const uint64_t ukey = ikey ^ mix64((uint64_t)u * 0xC2B2AE3D27D4EB4Full);
        uint64_t ctr = 0;
        while ((int64_t)out.size() < deg) {
            const double x = u01(mix64(ukey + ctr++));
            const int64_t r = std::lower_bound(cdf.begin(), cdf.end(), x) - cdf.begin();
            const int32_t it = perm[(size_t)std::min<int64_t>(r, n_items - 1)];
            if (std::find(out.begin(), out.end(), it) == out.end()) out.push_back(it);
            if (ctr > (uint64_t)deg * 4096 + 1000000) return false;
        }
        std::sort(out.begin(), out.end());
        return true;
    }
};

int threads_for(int32_t n_threads, int64_t work) {
    int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    return (int)std::min<int64_t>(nt, std::max<int64_t>(1, work));
}

int64_t degree_of(int64_t u, double mean_degree, uint64_t seed) {
    const uint64_t key = mix64(seed ^ 0xD6E8FEB86659FD93ull);
    return 1 + poisson(mean_degree - 1.0, key ^ mix64((uint64_t)u));
}

}  // namespace

extern "C" {

int cf_synth_items(int64_t n_items, double zipf_s, uint64_t seed, int64_t u_begin, int64_t u_end,
                   const int64_t* indptr, int32_t* indices_out, int32_t n_threads) {
    if (!indptr || !indices_out || n_items < 2 || u_end < u_begin) return CF_EINVAL;
    const int64_t nu = u_end - u_begin;
    const ItemGen gen(n_items, zipf_s, seed);
    const int nt = threads_for(n_threads, nu);
    std::vector<int> status((size_t)nt, CF_OK);
    auto work = [&](int t) {
        const int64_t lo = u_begin + nu * t / nt, hi = u_begin + nu * (t + 1) / nt;
        std::vector<int32_t> row;
        for (int64_t u = lo; u < hi; ++u) {
            const int64_t b = indptr[u - u_begin], e = indptr[u - u_begin + 1];
            if (!gen.row(u, e - b, row)) { status[(size_t)t] = CF_EINVAL; return; }
            std::memcpy(indices_out + b, row.data(), (size_t)(e - b) * sizeof(int32_t));
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (int s : status)
        if (s != CF_OK) return s;
    return CF_OK;
}

int cf_synth_item_users(int64_t n_users, int64_t n_items, double mean_degree, double zipf_s,
                        uint64_t seed, int64_t* indptr_t_out, int32_t* indices_t_out,
                        int32_t n_threads) {
    if (!indptr_t_out || !indices_t_out || n_users < 1 || n_items < 2 || mean_degree < 1.0)
        return CF_EINVAL;
    const ItemGen gen(n_items, zipf_s, seed);
    const int nt = threads_for(n_threads, n_users);
    // pass 1: per-thread item degrees over contiguous user ranges
    std::vector<std::vector<int64_t>> cnt((size_t)nt);
    std::vector<int> status((size_t)nt, CF_OK);
    auto count = [&](int t) {
        std::vector<int64_t>& c = cnt[(size_t)t];
        c.assign((size_t)n_items, 0);
        const int64_t lo = n_users * t / nt, hi = n_users * (t + 1) / nt;
        std::vector<int32_t> row;
        for (int64_t u = lo; u < hi; ++u) {
            if (!gen.row(u, degree_of(u, mean_degree, seed), row)) { status[(size_t)t] = CF_EINVAL; return; }
            for (int32_t it : row) c[(size_t)it]++;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(count, t);
        count(0);
        for (auto& x : th) x.join();
    }
    for (int s : status)
        if (s != CF_OK) return s;
    // item-major offsets; thread t writes after threads < t, so every item's
    // users come out in increasing id order (the transpose of the CSR)
    int64_t run = 0;
    for (int64_t i = 0; i < n_items; ++i) {
        indptr_t_out[i] = run;
        for (int t = 0; t < nt; ++t) {
            const int64_t c = cnt[(size_t)t][(size_t)i];
            cnt[(size_t)t][(size_t)i] = run;
            run += c;
        }
    }
    indptr_t_out[n_items] = run;
    auto fill = [&](int t) {
        std::vector<int64_t>& off = cnt[(size_t)t];
        const int64_t lo = n_users * t / nt, hi = n_users * (t + 1) / nt;
        std::vector<int32_t> row;
        for (int64_t u = lo; u < hi; ++u) {
            gen.row(u, degree_of(u, mean_degree, seed), row);
            for (int32_t it : row) indices_t_out[off[(size_t)it]++] = (int32_t)u;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fill, t);
    fill(0);
    for (auto& x : th) x.join();
    return CF_OK;
}

}  // extern "C"
