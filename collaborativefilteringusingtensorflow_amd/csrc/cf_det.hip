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
#include "cf_device.h"

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
// among the batch's positives of i_p (counting sort by positive item), as one
// record of psort_stride(W) ints (cf_kernels.h): the ids plus every
// occurrence's resolved destination, from the final counts and offsets
template <int W>
__global__ __launch_bounds__(256) void psort_scatter_kernel(PsortArgs a) {
    constexpr int RS = psort_stride(W);
    const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
    const int nt = gridDim.x * blockDim.x;
    const int B = a.B;
    for (int p = t0; p < B; p += nt) {
        // coalesced: the pair's ids and ranks
        const int32_t u = a.occU[p], i = a.occV[p], ru = a.rankU[p], rp = a.rankV[p];
        int32_t j[W], rj[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int64_t q = (int64_t)B + (int64_t)p * W + w;
            j[w] = a.occV[q];
            rj[w] = a.rankV[q];
        }
        // one round of independent random loads: the user's count, and per
        // item two adjacent (offP, offN) entries -- offsets and counts at once
        const int32_t cu = a.cntU[u];
        const int2 i0 = a.offPN[i], i1 = a.offPN[i + 1];
        int2 j0[W], j1[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            j0[w] = a.offPN[j[w]];
            j1[w] = a.offPN[j[w] + 1];
        }
        const int32_t oP = i0.x, ci = (i1.x - i0.x) + (i1.y - i0.y);
        int32_t cj[W], oN[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            cj[w] = (j1[w].x - j0[w].x) + (j1[w].y - j0[w].y);
            oN[w] = j0[w].y;
        }
        int32_t v[RS];
        v[0] = u;
        v[1] = i;
#pragma unroll
        for (int w = 0; w < W; ++w) v[2 + w] = j[w];
        v[2 + W] = cu == 1 ? kSlotApply : ru < a.capU ? u * a.capU + ru : kSlotAtomic;
        // deterministic mode: a user past its cap gets its compact int64 row
        // once, from its rank-capU occurrence (read by the next launches)
        if (a.hotU != nullptr && ru == a.capU) a.hotU[u] = atomicAdd(a.hot_n, 1);
        v[3 + W] = (int32_t)((uint32_t)oP | (ci == 1 ? 0x80000000u : 0u));
#pragma unroll
        for (int w = 0; w < W; ++w) v[4 + W + w] = cj[w] == 1 ? kSlotApply : oN[w] + rj[w];
#pragma unroll
        for (int k = 4 + 2 * W; k < RS; ++k) v[k] = 0;
        int4* r = reinterpret_cast<int4*>(a.srec + (int64_t)(oP + rp) * RS);
#pragma unroll
        for (int k = 0; k < RS / 4; ++k) r[k] = make_int4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    // the draw's phantoms (StepArgs::spec_ph): a speculatively counted first
    // candidate that the row scan rejected holds rank ph.y among item ph.x's
    // negatives.  Its compact slot row is zeroed, so the apply's sum of the
    // item's negative rows is unchanged (x + 0 = x); an item that only the
    // phantom touched (count 1) is applied by no one, so its count is reset
    // here -- nothing reads cntV of this buffer set after the scans
    if (a.spec_n != nullptr) {
        const int np = *a.spec_n;
        for (int k = t0; k < np; k += nt) {
            const int2 ph = a.spec_ph[k];
            const int2 o0 = a.offPN[ph.x], o1 = a.offPN[ph.x + 1];
            if ((o1.x - o0.x) + (o1.y - o0.y) == 1) {
                a.cntVw[ph.x] = 0;
            } else {
                float* row = a.slotN + ((int64_t)o0.y + ph.y) * a.d;
                for (int e = 0; e < a.d; ++e) row[e] = 0.f;
            }
        }
    }
}

// offPN[r] = (offP[r], offN[r]), the exclusive scans of cntP (positives per
// item) and cntV (negatives per item), r <= n items (the last entry holds the
// totals), in two launches of our own: per-tile sums
// of both arrays, then every tile adds the sums of the tiles before it (read
// by the whole block, O(tiles) per block -- ~50 tiles at 100K items) to its
// local scan.  No cross-block publication inside a launch (the look-back
// forms' XCD-coherence hazards), no library scan's init launch.
constexpr int kScanThreads = 256;
constexpr int kScanPer = 8;
constexpr int kScanTile = kScanThreads * kScanPer;   // 2,048 items per block

__global__ __launch_bounds__(kScanThreads) void psort_tile_sum_kernel(const int32_t* __restrict__ cntP,
                                                                      const int32_t* __restrict__ cntV,
                                                                      int64_t n, int2* __restrict__ tiles) {
    __shared__ int s_p[kScanThreads / 64], s_n[kScanThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    int sp = 0, sn = 0;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        const int64_t k = base + (int64_t)q * kScanThreads + threadIdx.x;   // coalesced
        if (k < n) {
            sp += cntP[k];
            sn += cntV[k];
        }
    }
    sp = wave_sum_i(sp);
    sn = wave_sum_i(sn);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_p[w] = sp;
        s_n[w] = sn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tp = 0, tn = 0;
        for (int k = 0; k < kScanThreads / 64; ++k) {
            tp += s_p[k];
            tn += s_n[k];
        }
        tiles[blockIdx.x] = make_int2(tp, tn);
    }
}

__global__ __launch_bounds__(kScanThreads) void psort_tile_scan_kernel(const int32_t* __restrict__ cntP,
                                                                       const int32_t* __restrict__ cntV,
                                                                       int64_t n, const int2* __restrict__ tiles,
                                                                       int2* __restrict__ offPN) {
    __shared__ int s_p[kScanThreads / 64], s_n[kScanThreads / 64];
    __shared__ int s_bp, s_bn;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the tiles before this one, summed by the whole block
    int bp = 0, bn = 0;
    for (int t = threadIdx.x; t < (int)blockIdx.x; t += kScanThreads) {
        const int2 v = tiles[t];
        bp += v.x;
        bn += v.y;
    }
    bp = wave_sum_i(bp);
    bn = wave_sum_i(bn);
    if (lane == 0) {
        s_p[w] = bp;
        s_n[w] = bn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tp = 0, tn = 0;
        for (int k = 0; k < kScanThreads / 64; ++k) {
            tp += s_p[k];
            tn += s_n[k];
        }
        s_bp = tp;
        s_bn = tn;
    }
    __syncthreads();
    // this thread's kScanPer consecutive items, scanned locally
    const int64_t k0 = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    int vp[kScanPer], vn[kScanPer];
    int tp = 0, tn = 0;
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        const bool ok = k0 + q < n;
        vp[q] = ok ? cntP[k0 + q] : 0;
        vn[q] = ok ? cntV[k0 + q] : 0;
        tp += vp[q];
        tn += vn[q];
    }
    const int ip = wave_incl_scan(tp), in = wave_incl_scan(tn);
    __syncthreads();   // s_p / s_n reused: wave totals
    if (lane == 63) {
        s_p[w] = ip;
        s_n[w] = in;
    }
    __syncthreads();
    int ep = s_bp + ip - tp, en = s_bn + in - tn;
    for (int k = 0; k < w; ++k) {
        ep += s_p[k];
        en += s_n[k];
    }
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        if (k0 + q <= n) offPN[k0 + q] = make_int2(ep, en);   // [n] = the totals
        ep += vp[q];
        en += vn[q];
    }
}

// n_items + 1 entries: the last one holds the totals
int psort_tiles(int64_t n_items) { return (int)((n_items + 1 + kScanTile - 1) / kScanTile); }

// sorted batches (cf_set_option "sorted_batches"): every pair q gets the
// batch its epoch slot falls in, perm_inverse(q) / B (pairs past the last
// whole batch: bin n_batches), with q as the value -- q ascending, so the
// stable radix sort by batch leaves each batch's pairs in pair (CSR) order
__global__ void epoch_keys_kernel(PermKey p, PermInv v, int64_t nnz, int64_t n_used, int B, int32_t nb,
                                  int32_t* __restrict__ keys, int32_t* __restrict__ vals) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = t0; q < nnz; q += nt) {
        const uint64_t slot = perm_inverse((uint64_t)q, p, v);
        keys[q] = slot < (uint64_t)n_used ? (int32_t)(slot / (uint64_t)B) : nb;
        vals[q] = (int32_t)q;
    }
}

// the records form (sorted_batches 1 / 2): the same keys, with each pair's 16-B record as the
// value (read in pair order: coalesced), so the sort leaves the records
// themselves in batch-then-CSR order and the draw reads them sequentially
__global__ void epoch_rec_keys_kernel(PermKey p, PermInv v, int64_t nnz, int64_t n_used, int B, int32_t nb,
                                      const int4* __restrict__ pairs, int32_t* __restrict__ keys,
                                      int4* __restrict__ recs) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = t0; q < nnz; q += nt) {
        const uint64_t slot = perm_inverse((uint64_t)q, p, v);
        keys[q] = slot < (uint64_t)n_used ? (int32_t)(slot / (uint64_t)B) : nb;
        recs[q] = pairs[q];
    }
}

}  // namespace

size_t epoch_records_scratch(int64_t nnz, int32_t n_batches) {
    size_t bytes = 0;
    hipcub::DoubleBuffer<int32_t> k(nullptr, nullptr);
    hipcub::DoubleBuffer<int4> v(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k, v, (int)nnz, 0, key_bits((int64_t)n_batches + 1));
    return bytes;
}

hipError_t launch_epoch_records(const PermKey& p, int64_t nnz, int B, const int4* pairs, int32_t* keys, int4* recs,
                                void* tmp, size_t tmp_bytes, const int4** recs_out, hipStream_t s) {
    if (nnz <= 0 || nnz > INT32_MAX || B <= 0) return hipErrorInvalidValue;
    const int32_t nb = (int32_t)(nnz / B);
    PermInv v{};
    for (int r = 0; r < 3; ++r) v.mi[r] = perm_mul_inverse(p.m[r]);
    hipLaunchKernelGGL(epoch_rec_keys_kernel, dim3(grid_of(nnz)), dim3(256), 0, s, p, v, nnz, (int64_t)nb * B, B,
                       nb, pairs, keys, recs);
    hipcub::DoubleBuffer<int32_t> dk(keys, keys + nnz);
    hipcub::DoubleBuffer<int4> dv(recs, recs + nnz);
    size_t bytes = tmp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, dk, dv, (int)nnz, 0, key_bits((int64_t)nb + 1), s);
    if (e != hipSuccess) return e;
    *recs_out = dv.Current();
    return hipGetLastError();
}

size_t epoch_order_scratch(int64_t nnz, int32_t n_batches) {
    size_t bytes = 0;
    hipcub::DoubleBuffer<int32_t> k(nullptr, nullptr), v(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k, v, (int)nnz, 0, key_bits((int64_t)n_batches + 1));
    return bytes;
}

hipError_t launch_epoch_order(const PermKey& p, int64_t nnz, int B, int32_t* keys, int32_t* vals, void* tmp,
                              size_t tmp_bytes, const int32_t** order_out, hipStream_t s) {
    if (nnz <= 0 || nnz > INT32_MAX || B <= 0) return hipErrorInvalidValue;
    const int32_t nb = (int32_t)(nnz / B);
    PermInv v{};
    for (int r = 0; r < 3; ++r) v.mi[r] = perm_mul_inverse(p.m[r]);
    hipLaunchKernelGGL(epoch_keys_kernel, dim3(grid_of(nnz)), dim3(256), 0, s, p, v, nnz, (int64_t)nb * B, B, nb,
                       keys, vals);
    hipcub::DoubleBuffer<int32_t> dk(keys, keys + nnz), dv(vals, vals + nnz);
    size_t bytes = tmp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, dk, dv, (int)nnz, 0, key_bits((int64_t)nb + 1), s);
    if (e != hipSuccess) return e;
    *order_out = dv.Current();
    return hipGetLastError();
}

size_t psort_scratch(int64_t n_items) { return (size_t)psort_tiles(n_items) * sizeof(int2); }

hipError_t launch_psort(const PsortArgs& a, void* tmp, size_t tmp_bytes, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    const int nt = psort_tiles(a.n_items);
    if (tmp_bytes < (size_t)nt * sizeof(int2)) return hipErrorInvalidValue;
    int2* tiles = reinterpret_cast<int2*>(tmp);
    hipLaunchKernelGGL(psort_tile_sum_kernel, dim3(nt), dim3(kScanThreads), 0, s, a.cntP, a.cntV, a.n_items, tiles);
    hipLaunchKernelGGL(psort_tile_scan_kernel, dim3(nt), dim3(kScanThreads), 0, s, a.cntP, a.cntV, a.n_items, tiles,
                       a.offPN);
    switch (a.W) {
        case 1: hipLaunchKernelGGL(psort_scatter_kernel<1>, dim3(grid_of(a.B)), dim3(256), 0, s, a); break;
        case 5: hipLaunchKernelGGL(psort_scatter_kernel<5>, dim3(grid_of(a.B)), dim3(256), 0, s, a); break;
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
