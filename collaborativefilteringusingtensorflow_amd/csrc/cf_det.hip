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
// one record (u, rank_u, i, p, (j_w, rank_j_w)...) of psort_stride(W) ints
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

// ---------------------------------------------------------------------------
// psort in ONE launch: the exclusive scan of cntP by decoupled look-back, then
// the record scatter, in the same blocks.
//  * scan: tiles of kPsTile items; a block takes tiles by atomic ticket, so
//    tiles are taken in increasing order and every tile a block looks back on
//    is held by a block that is already running (no residency assumption).
//    A tile publishes its aggregate (flag 1), looks back over its
//    predecessors until an inclusive prefix (flag 2), publishes its own
//    inclusive prefix, writes offP for its items and counts itself done.
//  * scatter: a block scatters pairs once every tile is done (one lane polls
//    a per-call counter; per-pair polls of per-tile flags measured 132 us).
//    Every tile is taken before any block scatters, so every wait ends.
// State words carry the call's generation (host counter), so nothing needs
// a reset; the ticket counter alternates between two words and each launch
// zeroes the one the next launch takes.  Spins are bounded: a give-up leaves
// the previous step's (in-range) records, never an out-of-range id.
// ---------------------------------------------------------------------------
constexpr int kPsTile = 1024;            // items per scan tile (4 per lane)
constexpr int kPsBlock = 256;
#ifdef CF_PSORT_DEBUG
constexpr uint32_t kPsSpinMax = 1u << 12;
#else
constexpr uint32_t kPsSpinMax = 1u << 24;
#endif

// a look-back word carries its value itself, so relaxed agent-scope atomics
// suffice for it; only the done counter guards other data (offP): a release
// add after the tile's offP writes, relaxed polls + one acquire fence before
// reading it
__device__ __forceinline__ uint64_t ps_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ps_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// state word: generation (bits 34..63), flag (32..33), value (0..31)
__device__ __forceinline__ uint64_t ps_word(uint32_t gen, uint32_t flag, uint32_t v) {
    return ((uint64_t)(gen & 0x3FFFFFFFu) << 34) | ((uint64_t)flag << 32) | v;
}

template <int W>
__global__ __launch_bounds__(kPsBlock) void psort_fused_kernel(PsortArgs a) {
    __shared__ uint32_t s_tile;
    __shared__ int s_wsum[kPsBlock / 64];
    __shared__ int s_prefix;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // the next launch's ticket and done words
        a.ctr[(a.gen + 1) & 1] = 0;
        a.ctr[2 + ((a.gen + 1) & 1)] = 0;
    }
#ifdef CF_PSORT_DEBUG
    if (threadIdx.x == 0) printf("psort start block %d gen %u ctr %u %u\n", (int)blockIdx.x, a.gen, a.ctr[0], a.ctr[1]);
#endif
    const uint32_t ntiles = (uint32_t)((a.n_items + kPsTile - 1) / kPsTile);
    // one ticket per block, straight-line (a ticket loop around barriers
    // lets the structurizer split wave 0's lanes across them): blocks that
    // draw a tile scan it, every block then scatters
    if (threadIdx.x == 0) s_tile = atomicAdd(&a.ctr[a.gen & 1], 1u);
    __syncthreads();
    // block-uniform, and readfirstlane lets the compiler see it
    const uint32_t t = __builtin_amdgcn_readfirstlane(s_tile);
#ifdef CF_PSORT_DEBUG
    if (threadIdx.x == 0) printf("psort block %d ticket %u of %u\n", (int)blockIdx.x, t, ntiles);
#endif
    if (t < ntiles) {
        const int64_t base = (int64_t)t * kPsTile + threadIdx.x * 4;
        int c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = base + k < a.n_items ? a.cntP[base + k] : 0;
        const int tsum = c[0] + c[1] + c[2] + c[3];
        int incl = tsum;   // wave inclusive scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        int woff = 0, agg = 0;
#pragma unroll
        for (int w = 0; w < kPsBlock / 64; ++w) {
            if (w < wave) woff += s_wsum[w];
            agg += s_wsum[w];
        }
        if (threadIdx.x == 0) {
            int prefix = 0;
            if (t == 0) {
                ps_store(&a.state[0], ps_word(a.gen, 2, (uint32_t)agg));
            } else {
                ps_store(&a.state[t], ps_word(a.gen, 1, (uint32_t)agg));
                int64_t j = (int64_t)t - 1;
                uint32_t spins = 0;
                while (j >= 0) {
                    const uint64_t st = ps_load(&a.state[j]);
                    const uint32_t flag = (uint32_t)(st >> 32) & 3u;
                    if ((uint32_t)(st >> 34) != (a.gen & 0x3FFFFFFFu) || flag == 0) {
                        if (++spins > kPsSpinMax) {
#ifdef CF_PSORT_DEBUG
                            printf("psort look-back gave up: block %d tile %u j %lld st %llx gen %u\n", (int)blockIdx.x,
                                   t, (long long)j, (unsigned long long)st, a.gen);
#endif
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    prefix += (int)(uint32_t)st;
                    if (flag == 2) break;
                    --j;
                }
                ps_store(&a.state[t], ps_word(a.gen, 2, (uint32_t)(prefix + agg)));
            }
            s_prefix = prefix;
        }
        __syncthreads();
        int run = s_prefix + woff + incl - tsum;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (base + k < a.n_items) a.offP[base + k] = run;
            run += c[k];
        }
        // each wave's offP stores complete (workgroup release: no L2 write-back),
        // then one agent-scope release -- one L2 write-back per tile -- on the add
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_waitcnt(0);   // this wave's stores have reached L2 (the fence alone does not wait here)
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_fetch_add(&a.ctr[2 + (a.gen & 1)], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) {
        s_prefix = 0;   // (every read of the scan's prefix is behind the last barrier)
        for (uint32_t spins = 0;
             __hip_atomic_load(&a.ctr[2 + (a.gen & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ntiles;) {
            if (++spins > kPsSpinMax) {
#ifdef CF_PSORT_DEBUG
                printf("psort scatter gave up: block %d gen %u\n", (int)blockIdx.x, a.gen);
#endif
                s_prefix = -1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    if (s_prefix == -1) return;   // gave up: the previous step's records stay (in range)
    // no acquire fence (an L2 invalidate per block): offP is read with
    // agent-scope atomic loads below
    // scatter (the records as in psort_scatter_kernel)
#ifdef CF_PSORT_DEBUG
    if (threadIdx.x == 0) printf("psort block %d scatter\n", (int)blockIdx.x);
#endif
    constexpr int RS = psort_stride(W);
    const int nt = gridDim.x * blockDim.x;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < a.B; p += nt) {
        const int32_t i = a.occV[p];
        int32_t v[RS], rk[W + 2];
        v[0] = a.occU[p];
        v[1] = i;
        rk[0] = rank16(a.rankU[p]);
        rk[W + 1] = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int64_t q = (int64_t)a.B + (int64_t)p * W + w;
            v[2 + w] = a.occV[q];
            rk[1 + w] = rank16(a.rankV[q]);
        }
#pragma unroll
        for (int k = 0; k < (W + 2) / 2; ++k) v[2 + W + k] = rk[2 * k] | (rk[2 * k + 1] << 16);
#pragma unroll
        for (int k = 2 + W + (W + 2) / 2; k < RS; ++k) v[k] = 0;
        const int32_t o = __hip_atomic_load(&a.offP[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int64_t pos = (int64_t)o + a.rankV[p];
        if (pos < 0 || pos >= a.B) continue;   // only after a given-up look-back
        int4* r = reinterpret_cast<int4*>(a.srec + pos * RS);
#pragma unroll
        for (int k = 0; k < RS / 4; ++k) r[k] = make_int4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
}

}  // namespace

size_t psort_state_words(int64_t n_items) { return (size_t)((n_items + kPsTile - 1) / kPsTile); }

hipError_t launch_psort_fused(const PsortArgs& a, int W, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    // one block per scan tile at least (each block scans at most one); the
    // scatter is grid-stride
    int64_t blocks = ((int64_t)a.B + kPsBlock - 1) / kPsBlock;
    if (blocks > 2048) blocks = 2048;
    const int64_t tiles = (a.n_items + kPsTile - 1) / kPsTile;
    if (blocks < tiles) blocks = tiles;
    switch (W) {
        case 1: hipLaunchKernelGGL(psort_fused_kernel<1>, dim3((unsigned)blocks), dim3(kPsBlock), 0, s, a); break;
        case 5: hipLaunchKernelGGL(psort_fused_kernel<5>, dim3((unsigned)blocks), dim3(kPsBlock), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

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
