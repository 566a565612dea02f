// cf_device.h -- gfx950 device helpers: counter-based RNG, the keyed epoch
// bijection, 64-lane wave reductions, order-preserving float keys.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cf_kernels.h"

namespace cfk {

// SplitMix64 finaliser: a strong 64-bit mixer, used as a counter-based RNG
// (every draw is hash(key, counter) -- no RNG state to carry between steps).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// floor(h * n / 2^64): uniform in [0, n) with bias <= n / 2^64.
__device__ __forceinline__ uint64_t uniform_below(uint64_t h, uint64_t n) {
    return __umul64hi(h, n);
}

// One bijective pass on [0, 2^bits): xor key, multiply by odd, xorshift.
__host__ __device__ __forceinline__ uint64_t perm_rounds(uint64_t x, const PermKey& p) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        x = (x ^ p.k[r]) & p.mask;
        x = (x * p.m[r]) & p.mask;
        x ^= x >> p.shift;
    }
    return x;
}

// Cycle-walking restriction of the 2^bits bijection to [0, n): a bijection.
__host__ __device__ __forceinline__ uint64_t permute(uint64_t x, const PermKey& p) {
    do {
        x = perm_rounds(x, p);
    } while (x >= p.n);
    return x;
}

// Inverse of perm_rounds; mi[r] = the inverse of p.m[r] modulo 2^64
// (perm_mul_inverse), which is also its inverse modulo 2^bits.  A round's
// xorshift x ^= x >> s is undone by y ^ (y >> s) ^ (y >> 2s) ^ ..
struct PermInv {
    uint64_t mi[3];
};
__host__ __device__ __forceinline__ uint64_t perm_mul_inverse(uint64_t m) {
    uint64_t inv = m;   // m * m == 1 mod 8 for odd m: 3 correct bits, doubled per step
#pragma unroll
    for (int i = 0; i < 6; ++i) inv *= 2ull - m * inv;
    return inv;
}
__host__ __device__ __forceinline__ uint64_t perm_rounds_inv(uint64_t x, const PermKey& p, const PermInv& v) {
#pragma unroll
    for (int r = 2; r >= 0; --r) {
        uint64_t z = x;
        for (uint32_t t = p.shift; t < 64; t += p.shift) z ^= x >> t;
        x = (z * v.mi[r]) & p.mask;
        x = (x ^ p.k[r]) & p.mask;
    }
    return x;
}
// the slot a pair index comes from: permute(perm_inverse(q)) == q
__host__ __device__ __forceinline__ uint64_t perm_inverse(uint64_t q, const PermKey& p, const PermInv& v) {
    do {
        q = perm_rounds_inv(q, p, v);
    } while (q >= p.n);
    return q;
}

// butterfly sum: every lane ends with the bitwise-identical total
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// inclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// SparseApplyAdagrad's step as TF1 computes it, grad * lr * rsqrt(accum)
// (training_ops.cc ApplyAdagrad), with the hardware reciprocal square root
// (1 ulp) instead of an IEEE divide + sqrt sequence
__device__ __forceinline__ float adagrad_delta(float lr, float g, float acc) {
    return g * lr * __builtin_amdgcn_rsqf(acc);
}

// 1 / (1 + e) with the hardware reciprocal (1 ulp): the logistic pieces of
// the BPR loss and its derivative; e = inf gives 0 as the IEEE divide does
__device__ __forceinline__ float rcp_1p(float e) { return __builtin_amdgcn_rcpf(1.f + e); }

// Order-preserving map float -> uint32 (larger float => larger key).  Key 0
// is reserved for "excluded" (train items under exclude_train).
__device__ __forceinline__ uint32_t float_key(float f) {
    uint32_t u = __float_as_uint(f);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return u < 1u ? 1u : u;
}
__device__ __forceinline__ float key_float(uint32_t u) {
    u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    return __uint_as_float(u);
}

// lower_bound membership test in a sorted int32 run [lo, hi)
__device__ __forceinline__ bool sorted_contains(const int32_t* __restrict__ a, int64_t lo,
                                                int64_t hi, int32_t key) {
    const int64_t end = hi;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        int32_t v = a[mid];
        if (v < key) lo = mid + 1; else hi = mid;
    }
    return lo < end && a[lo] == key;
}

}  // namespace cfk
