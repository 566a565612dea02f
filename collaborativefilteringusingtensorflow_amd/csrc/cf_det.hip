// cf_det.hip -- deterministic occurrence ranks (cf_set_option "deterministic").
//
// The fast path ranks the occurrences of a row by the order their returning
// count atomics land, so the order in which a duplicated row's gradients are
// summed -- and with it the last bits of the fp32 sum -- changes run to run.
// TF1's CPU UnsortedSegmentSum behind AdagradOptimizer (bprmf.py:83-88) is
// deterministic; this restores that property: a stable LSD radix sort of the
// batch's row ids (users, then items offset by n_users) puts every row's
// occurrences in batch order, rank = sorted position - the row's first sorted
// position (off[row]), and the gradient kernels store occurrence k of row r
// in the compact slot off[r] + k, which the apply sums in k order.
#include <hipcub/hipcub.hpp>

#include "cf_kernels.h"

namespace cfk {

namespace {

__global__ void det_keys_kernel(const int32_t* __restrict__ occU, int64_t nU,
                                const int32_t* __restrict__ occV, int64_t nV, int64_t n_users,
                                int32_t* __restrict__ keys, int32_t* __restrict__ vals) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = t0; q < nU + nV; q += nt) {
        keys[q] = q < nU ? occU[q] : (int32_t)(n_users + occV[q - nU]);
        vals[q] = (int32_t)q;
    }
}

// every user key sorts before every item key (items are offset by n_users),
// so the items' sorted positions start at nU: a row's slot base is its first
// sorted position inside its own table's part ([0, nU) users, [0, nV) items)
__device__ __forceinline__ int64_t part_base(int32_t key, int64_t n_users, int64_t nU) {
    return key >= n_users ? nU : 0;
}

// the first position of every row present in the batch, within its table's part
__global__ void det_heads_kernel(const int32_t* __restrict__ skeys, int64_t n, int64_t n_users,
                                 int64_t nU, int32_t* __restrict__ off) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = t0; p < n; p += nt) {
        const int32_t k = skeys[p];
        if (p == 0 || k != skeys[p - 1]) off[k] = (int32_t)(p - part_base(k, n_users, nU));
    }
}

__global__ void det_rank_kernel(const int32_t* __restrict__ skeys, const int32_t* __restrict__ svals,
                                int64_t n, int64_t n_users, int64_t nU, const int32_t* __restrict__ off,
                                int32_t* __restrict__ rankU, int32_t* __restrict__ rankV) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = t0; p < n; p += nt) {
        const int32_t k = skeys[p];
        const int32_t q = svals[p];
        const int32_t rk = (int32_t)(p - part_base(k, n_users, nU) - off[k]);
        if (q < nU) rankU[q] = rk;
        else rankV[q - nU] = rk;
    }
}

int key_bits(int64_t n_rows) {
    int b = 1;
    while (b < 31 && (1ll << b) < n_rows) ++b;
    return b;
}

int grid_of(int64_t n) {
    int64_t b = (n + 255) / 256;
    return (int)(b < 1 ? 1 : b > 4096 ? 4096 : b);
}

// positive-sorted gradient: pair p goes to position offP[i_p] + its rank
// among the batch's positives of i_p (counting sort by positive item), as
// one record of psort_stride(W) ints:
//   [u, i, j_0 .. j_{W-1}, (ru | rj0 << 16), (rj1 | rj2 << 16), .., 0 padding]
// -- the ranks of u and of the negatives as 16-bit halves (clamped to
// 0xFFFF), ru in the low half of the first rank word (load_idx_sorted)
__device__ __forceinline__ int32_t rank16(int32_t r) { return r < 0xFFFF ? r : 0xFFFF; }

template <int W>
__global__ void psort_scatter_kernel(const int32_t* __restrict__ occU, const int32_t* __restrict__ rankU,
                                     const int32_t* __restrict__ occV, const int32_t* __restrict__ rankV,
                                     int B, const int32_t* __restrict__ offP, int32_t* __restrict__ srec) {
    constexpr int RS = psort_stride(W);
    const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
    const int nt = gridDim.x * blockDim.x;
    for (int p = t0; p < B; p += nt) {
        const int32_t i = occV[p];
        int32_t v[RS], rk[W + 2];
        v[0] = occU[p];
        v[1] = i;
        rk[0] = rank16(rankU[p]);
        rk[W + 1] = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int64_t q = (int64_t)B + (int64_t)p * W + w;
            v[2 + w] = occV[q];
            rk[1 + w] = rank16(rankV[q]);
        }
#pragma unroll
        for (int k = 0; k < (W + 2) / 2; ++k) v[2 + W + k] = rk[2 * k] | (rk[2 * k + 1] << 16);
#pragma unroll
        for (int k = 2 + W + (W + 2) / 2; k < RS; ++k) v[k] = 0;
        int4* r = reinterpret_cast<int4*>(srec + (int64_t)(offP[i] + rankV[p]) * RS);
#pragma unroll
        for (int k = 0; k < RS / 4; ++k) r[k] = make_int4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
}

}  // namespace

size_t psort_scratch(int64_t n_items) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                           (int)n_items);
    return bytes;
}

hipError_t launch_psort(const int32_t* occU, const int32_t* rankU, const int32_t* occV, const int32_t* rankV,
                        int B, int W, const int32_t* cntP, int32_t* offP, int32_t* srec, int64_t n_items,
                        void* tmp, size_t tmp_bytes, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    size_t bytes = tmp_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, bytes, cntP, offP, (int)n_items, s);
    if (e != hipSuccess) return e;
    switch (W) {
        case 1: hipLaunchKernelGGL(psort_scatter_kernel<1>, dim3(grid_of(B)), dim3(256), 0, s, occU, rankU, occV,
                                   rankV, B, offP, srec); break;
        case 5: hipLaunchKernelGGL(psort_scatter_kernel<5>, dim3(grid_of(B)), dim3(256), 0, s, occU, rankU, occV,
                                   rankV, B, offP, srec); break;
        default: return hipErrorInvalidValue;   // pos_sort runs at W in {1, 5}
    }
    return hipGetLastError();
}

size_t det_ranks_scratch(int64_t n_occ, int64_t n_rows) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)n_occ, 0,
                                             key_bits(n_rows));
    return bytes;
}

// keys / vals hold 2 * n_occ int32 each (in + out halves)
hipError_t launch_det_ranks(const int32_t* occU, int64_t nU, const int32_t* occV, int64_t nV,
                            int64_t n_users, int64_t n_rows, int32_t* rankU, int32_t* rankV,
                            int32_t* off, int32_t* keys, int32_t* vals, void* tmp, size_t tmp_bytes,
                            hipStream_t s) {
    const int64_t n = nU + nV;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(det_keys_kernel, dim3(grid_of(n)), dim3(256), 0, s, occU, nU, occV, nV, n_users,
                       keys, vals);
    size_t bytes = tmp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, keys, keys + n, vals, vals + n, (int)n, 0,
                                                      key_bits(n_rows), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(det_heads_kernel, dim3(grid_of(n)), dim3(256), 0, s, keys + n, n, n_users, nU, off);
    hipLaunchKernelGGL(det_rank_kernel, dim3(grid_of(n)), dim3(256), 0, s, keys + n, vals + n, n, n_users, nU,
                       off, rankU, rankV);
    return hipGetLastError();
}

}  // namespace cfk
