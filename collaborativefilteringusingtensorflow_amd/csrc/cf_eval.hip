// cf_eval.hip -- recommend step for gfx950: user x item scores, exclusion of
// the user's train items, per-user top-k sorted by score descending with ties
// to the lower item id (TF TopKV2).  Reference: __predict__ + __recommend,
// src/models/pl/models/bprmf.py:77-103 (and gbprmf.py:95-121,
// cml.py:111-144, amf.py:144-177).  Filtering the train items BEFORE the
// selection is equivalent to the reference's over-fetch of
// max|train(u)|+topN followed by the python filter loop.
#include "cf_kernels.h"
#include "cf_device.h"

namespace cfk {

constexpr int kTile = 64;   // 64 users x 64 items per block
constexpr int kTk = 16;     // k-slab staged in LDS

template <int MODEL>
__global__ __launch_bounds__(kBlock) void score_kernel(ScoreArgs a) {
    __shared__ float Us[kTk][kTile + 1];
    __shared__ float Vs[kTk][kTile + 1];
    const int tu = threadIdx.x >> 4;   // 0..15 -> user rows tu*4 + m
    const int ti = threadIdx.x & 15;   // 0..15 -> item cols ti + 16*n
    const int u0 = blockIdx.y * kTile;
    const int64_t i0 = (int64_t)blockIdx.x * kTile;
    const int d = a.d;
    float acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = 0.f;

    for (int k0 = 0; k0 < d; k0 += kTk) {
        for (int t = threadIdx.x; t < kTile * kTk; t += kBlock) {
            const int r = t / kTk, kk = t % kTk;
            const int kd = k0 + kk;
            const int uu = u0 + r;
            Us[kk][r] = (uu < a.n_users && kd < d) ? a.U[(int64_t)a.users[uu] * d + kd] : 0.f;
            const int64_t ii = i0 + r;
            Vs[kk][r] = (ii < a.n_items && kd < d) ? a.V[ii * d + kd] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kTk; ++kk) {
            float av[4], bv[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) av[m] = Us[kk][tu * 4 + m];
#pragma unroll
            for (int n = 0; n < 4; ++n) bv[n] = Vs[kk][ti + 16 * n];
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    if (MODEL == CML) {
                        const float t = av[m] - bv[n];
                        acc[m][n] = fmaf(t, t, acc[m][n]);
                    } else {
                        acc[m][n] = fmaf(av[m], bv[n], acc[m][n]);
                    }
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int uu = u0 + tu * 4 + m;
        if (uu >= a.n_users) continue;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int64_t ii = i0 + ti + 16 * n;
            if (ii >= a.n_items) continue;
            float s = acc[m][n];
            if (MODEL == CML) s = -s;
            if (MODEL == GBPR) s += a.b[ii];
            a.keys[(int64_t)uu * a.n_items + ii] = float_key(s);
        }
    }
}

__global__ __launch_bounds__(kBlock) void mask_train_kernel(ScoreArgs a) {
    const int c = blockIdx.x;
    if (c >= a.n_users) return;
    const int u = a.users[c];
    const int64_t rb = a.indptr[u], re = a.indptr[u + 1];
    uint32_t* row = a.keys + (int64_t)c * a.n_items;
    for (int64_t t = rb + threadIdx.x; t < re; t += kBlock) row[a.indices[t]] = 0u;
}

// block-wide exclusive scan of a 0/1 flag (256 threads); returns prefix,
// writes the block total to *total
__device__ __forceinline__ int block_excl_scan(int flag, int* s_wave, int* total) {
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const unsigned long long bal = __ballot(flag);
    const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s_wave[wv] = __popcll(bal);
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kWavesPerBlock; ++k) {
        const int v = s_wave[k];
        if (k < wv) base += v;
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return base + in_wave;
}

constexpr int kMaxTopk = 4096;

__global__ __launch_bounds__(kBlock) void topk_kernel(TopkArgs a) {
    __shared__ unsigned int hist[256];
    __shared__ unsigned long long cand[kMaxTopk];
    __shared__ int s_wave[kWavesPerBlock];
    __shared__ unsigned int s_sel[3];  // digit, remaining, zero count
    const int c = blockIdx.x;
    const uint32_t* kr = a.keys + (int64_t)c * a.n_items;
    const int64_t n = a.n_items;
    const int tid = threadIdx.x;

    // count excluded (key 0) entries
    if (tid == 0) s_sel[2] = 0;
    __syncthreads();
    {
        unsigned int z = 0;
        for (int64_t t = tid; t < n; t += kBlock) z += (kr[t] == 0u);
        if (z) atomicAdd(&s_sel[2], z);
    }
    __syncthreads();
    const int64_t valid = n - (int64_t)s_sel[2];
    const int k_eff = (int)((int64_t)a.k < valid ? (int64_t)a.k : valid);

    uint32_t prefix = 0, pmask = 0;
    unsigned int remaining = (unsigned)k_eff;
    if (k_eff > 0) {
        for (int shift = 24; shift >= 0; shift -= 8) {
            for (int t = tid; t < 256; t += kBlock) hist[t] = 0;
            __syncthreads();
            for (int64_t t = tid; t < n; t += kBlock) {
                const uint32_t x = kr[t];
                if (x != 0u && (x & pmask) == prefix) atomicAdd(&hist[(x >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (tid == 0) {
                unsigned int cum = 0;
                int dsel = 0;
                for (int dgt = 255; dgt >= 0; --dgt) {
                    const unsigned int h = hist[dgt];
                    if (cum + h >= remaining) { dsel = dgt; break; }
                    cum += h;
                }
                s_sel[0] = (unsigned)dsel;
                s_sel[1] = remaining - cum;
            }
            __syncthreads();
            prefix |= s_sel[0] << shift;
            pmask |= 255u << shift;
            remaining = s_sel[1];
            __syncthreads();
        }
    }
    const uint32_t T = prefix;          // k-th largest valid key
    const int need_eq = (int)remaining; // how many keys == T to take (lowest ids first)

    int kpad = 1;
    while (kpad < k_eff) kpad <<= 1;
    for (int t = tid; t < kpad; t += kBlock) cand[t] = 0ull;
    __syncthreads();

    int out_base = 0, eq_base = 0;
    if (k_eff > 0) {
        for (int64_t t0 = 0; t0 < n; t0 += kBlock) {
            const int64_t t = t0 + tid;
            const uint32_t x = (t < n) ? kr[t] : 0u;
            const int is_eq = (x == T && x != 0u) ? 1 : 0;
            int eq_tot;
            const int eq_rank = eq_base + block_excl_scan(is_eq, s_wave, &eq_tot);
            const int sel = (x > T) || (is_eq && eq_rank < need_eq);
            int sel_tot;
            const int pos = out_base + block_excl_scan(sel, s_wave, &sel_tot);
            if (sel && pos < kMaxTopk)
                cand[pos] = ((unsigned long long)x << 32) | (0xFFFFFFFFull - (unsigned long long)t);
            out_base += sel_tot;
            eq_base += eq_tot;
            if (out_base >= k_eff) break;   // uniform
        }
    }
    __syncthreads();

    // bitonic sort, descending on (key, -id)
    for (int size = 2; size <= kpad; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < kpad; t += kBlock) {
                const int partner = t ^ stride;
                if (partner > t) {
                    const bool desc = ((t & size) == 0);
                    const unsigned long long x = cand[t], y = cand[partner];
                    if (desc ? (x < y) : (x > y)) {
                        cand[t] = y;
                        cand[partner] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int r = tid; r < a.k; r += kBlock) {
        int id = -1;
        float v = __int_as_float(0x7fc00000);
        if (r < k_eff) {
            const unsigned long long e = cand[r];
            id = (int)(0xFFFFFFFFull - (e & 0xFFFFFFFFull));
            v = key_float((uint32_t)(e >> 32));
        }
        a.idx_out[(int64_t)c * a.k + r] = id;
        if (a.val_out) a.val_out[(int64_t)c * a.k + r] = v;
    }
}

hipError_t launch_score(const ScoreArgs& a, hipStream_t s) {
    if (a.n_users <= 0) return hipSuccess;
    dim3 grid((unsigned)((a.n_items + kTile - 1) / kTile), (unsigned)((a.n_users + kTile - 1) / kTile));
    switch (a.model) {
        case GBPR: hipLaunchKernelGGL(score_kernel<GBPR>, grid, dim3(kBlock), 0, s, a); break;
        case CML: hipLaunchKernelGGL(score_kernel<CML>, grid, dim3(kBlock), 0, s, a); break;
        default: hipLaunchKernelGGL(score_kernel<BPR>, grid, dim3(kBlock), 0, s, a); break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !a.exclude_train) return e;
    hipLaunchKernelGGL(mask_train_kernel, dim3(a.n_users), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_topk(const TopkArgs& a, int n_users, hipStream_t s) {
    if (n_users <= 0) return hipSuccess;
    hipLaunchKernelGGL(topk_kernel, dim3(n_users), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace cfk
