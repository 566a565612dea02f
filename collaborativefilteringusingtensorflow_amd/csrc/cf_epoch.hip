// cf_epoch.hip -- the sorted batches' epoch order (cf_set_option
// "sorted_batches") as a hand-written counting sort by batch id.
//
// Batch b of an epoch is the epoch bijection's slots [bB, (b+1)B) -- the
// reference shuffles its pairs and slices consecutive batches
// (sampler_ranking.py:24-27).  Sorted batches visit each batch's pairs in pair
// (CSR) order: pair q belongs to batch perm_inverse(q) / B (pairs past the
// last whole batch: bin nb), and the order is the stable sort of the pair
// indices by that bin.  The bins' sizes are known (B each, nnz - nb B for the
// last), so the sort is a counting sort over tiles of kEpochTile consecutive
// pairs:
//
//   1. epoch_bins_kernel: every pair's bin (the bijection's inverse, cycle
//      walking lane by lane -- a lane that finishes a pair takes its next one,
//      so a wave pays the lanes' mean walk, not the longest) -> bins[q]
//      (uint16) and the tile's histogram cnt[tile][bin];
//   2. the column scan over the tiles (three small launches: chunk sums, a
//      wave per bin scanning the chunk sums, the tiles' offsets), in place:
//      cnt[tile][bin] <- bin B + the bin's pairs in earlier tiles;
//   3. epoch_scatter_kernel: a block stably ranks its tile's pairs by bin in
//      LDS (each wave ranks its 512 pairs with ballots over the bin's bits,
//      lower lane = lower pair, on top of the earlier waves' counts), stages
//      the pair indices bin-contiguous in LDS and writes each bin's run with
//      consecutive lanes: coalesced stores (a scattered 16-B store per pair
//      measured 0.9-1.2 ms per 50M-pair epoch, profiles/r06/r06b).
//
// The output is bitwise the stable radix sort's (cf_det.hip
// launch_epoch_records / launch_epoch_order, kept for more than
// kEpochMaxBins bins and as cf_set_option("epoch_sort", 1)), without its key
// arrays: HBM traffic per pair = 2 B bin written + read, 16 B record read,
// 16 B record written (records form; 4 B index written in the index form).
#include "cf_kernels.h"
#include "cf_device.h"

namespace cfk {

namespace {

// consecutive pairs per block (1,024 measured slower: records 0.71 vs 0.70 ms,
// index form 0.33 vs 0.26 ms per 50M-pair epoch, profiles/r06/r06e)
constexpr int kEpochTile = 2048;
constexpr int kEpochItems = kEpochTile / kBlock;  // 8 per thread
constexpr int kEpochWaveSpan = kEpochTile / kWavesPerBlock;   // 512 consecutive pairs per wave (scatter)
constexpr int kEpochChunkTiles = 32;              // tiles per chunk of the column scan

struct EpochCtx {
    uint32_t n, mask, shift, B;
    uint32_t k[3], mi[3];
    uint64_t magic;      // B > 1: slot / B == umulhi64(slot, magic) for slot < 2^32
    uint32_t nb, n_used;
    int32_t n_bins, nbits;
    int32_t xs_steps;    // doubling steps that undo one round's xorshift
    int32_t pad;
    int64_t n_tiles;
};

// one application of the inverse of the 2^bits bijection (perm_rounds_inv,
// cf_device.h) with every value below 2^bits <= 2^31: the products modulo
// 2^bits see only the low 32 bits of the multipliers, and x ^= x >> s is
// undone by doubling, y ^= y >> s; y ^= y >> 2s; .. while the shift < bits
__device__ __forceinline__ uint32_t rounds_inv32(uint32_t q, const EpochCtx& c) {
#pragma unroll
    for (int r = 2; r >= 0; --r) {
        uint32_t z = q;
        uint32_t t = c.shift;
        for (int s = 0; s < c.xs_steps; ++s, t <<= 1) z ^= z >> t;
        q = (z * c.mi[r]) & c.mask;
        q = (q ^ c.k[r]) & c.mask;
    }
    return q;
}

__device__ __forceinline__ int bin_of_slot(uint32_t slot, const EpochCtx& c) {
    if (slot >= c.n_used) return (int)c.nb;
    return c.B == 1 ? (int)slot : (int)__umul64hi((uint64_t)slot, c.magic);
}

// pass 1: bins of a tile's pairs (q = tile0 + k kBlock + tid, k < kEpochItems)
__global__ void __launch_bounds__(kBlock) epoch_bins_kernel(EpochCtx c, uint16_t* __restrict__ bins,
                                                            int32_t* __restrict__ cnt) {
    extern __shared__ int32_t lds[];
    int32_t* hist = lds;                                              // [n_bins]
    uint16_t* stage = reinterpret_cast<uint16_t*>(lds + c.n_bins);   // [kEpochTile]
    const int tid = threadIdx.x;
    const uint32_t tile0 = (uint32_t)blockIdx.x * kEpochTile;
    const uint32_t qend = min(tile0 + (uint32_t)kEpochTile, c.n);
    for (int b = tid; b < c.n_bins; b += kBlock) hist[b] = 0;
    __syncthreads();
    // cycle walking, lane by lane: a pair whose inverse leaves [0, n) walks on;
    // a lane done with a pair starts its next one in the same iteration
    int k = 0;
    uint32_t q = tile0 + (uint32_t)tid, x = q;
    bool live = q < qend;
    while (live) {
        x = rounds_inv32(x, c);
        if (x < c.n) {
            const int b = bin_of_slot(x, c);
            stage[k * kBlock + tid] = (uint16_t)b;
            atomicAdd(&hist[b], 1);
            ++k;
            q += kBlock;
            x = q;
            live = k < kEpochItems && q < qend;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kEpochItems; ++i) {
        const uint32_t qq = tile0 + (uint32_t)(i * kBlock + tid);
        if (qq < qend) bins[qq] = stage[i * kBlock + tid];
    }
    for (int b = tid; b < c.n_bins; b += kBlock) cnt[(int64_t)blockIdx.x * c.n_bins + b] = hist[b];
}

// chunk sums: csum[ch][bin] = sum of cnt[tile][bin] over the chunk's tiles
__global__ void __launch_bounds__(kBlock) epoch_chunk_sum_kernel(EpochCtx c, const int32_t* __restrict__ cnt,
                                                                 int32_t* __restrict__ csum) {
    const int64_t t0 = (int64_t)blockIdx.x * kEpochChunkTiles;
    const int64_t t1 = min(t0 + (int64_t)kEpochChunkTiles, c.n_tiles);
    for (int b = threadIdx.x; b < c.n_bins; b += kBlock) {
        int32_t s = 0;
#pragma unroll 8
        for (int64_t g = t0; g < t1; ++g) s += cnt[g * c.n_bins + b];
        csum[(int64_t)blockIdx.x * c.n_bins + b] = s;
    }
}

// a wave per bin: exclusive scan of its chunk sums, from the bin's first
// output position bin * B (the leftover bin nb starts at nb B = n_used)
__global__ void __launch_bounds__(kBlock) epoch_chunk_scan_kernel(EpochCtx c, int32_t* __restrict__ csum,
                                                                  int64_t n_chunks) {
    const int b = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (b >= c.n_bins) return;
    int32_t run = (int32_t)((uint32_t)b * c.B);
    for (int64_t r = 0; r < n_chunks; r += kWave) {
        const int64_t ch = r + lane;
        const int32_t v = ch < n_chunks ? csum[ch * c.n_bins + b] : 0;
        const int32_t inc = wave_incl_scan(v);
        if (ch < n_chunks) csum[ch * c.n_bins + b] = run + inc - v;
        run += __shfl(inc, kWave - 1, kWave);
    }
}

// the tiles' offsets, in place: cnt[tile][bin] <- csum[chunk][bin] + the
// bin's pairs in the chunk's earlier tiles
__global__ void __launch_bounds__(kBlock) epoch_tile_offsets_kernel(EpochCtx c, int32_t* __restrict__ cnt,
                                                                    const int32_t* __restrict__ csum) {
    const int64_t t0 = (int64_t)blockIdx.x * kEpochChunkTiles;
    const int64_t t1 = min(t0 + (int64_t)kEpochChunkTiles, c.n_tiles);
    for (int b = threadIdx.x; b < c.n_bins; b += kBlock) {
        int32_t run = csum[(int64_t)blockIdx.x * c.n_bins + b];
        for (int64_t g = t0; g < t1; ++g) {
            const int32_t t = cnt[g * c.n_bins + b];
            cnt[g * c.n_bins + b] = run;
            run += t;
        }
    }
}

// exclusive scan of one value per thread over the block
__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t* wtot) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t inc = wave_incl_scan(v);
    if (lane == kWave - 1) wtot[w] = inc;
    __syncthreads();
    int32_t before = 0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) before += i < w ? wtot[i] : 0;
    return before + inc - v;
}

// pass 3.  RECS: out_recs[pos] = pairs[q] (the records form, sorted_batches
// 1 / 2); else out_idx[pos] = q (the index form, sorted_batches 3).  The
// tile is staged as pair indices (4 B): staging the 16-B records themselves
// in LDS measured 0.68-0.91 ms per 50M-pair epoch against 0.12-0.26 ms for
// the index form (profiles/r06/r06c) -- 44 KB of LDS per block (3 blocks per
// CU) and random 16-B LDS writes; the copy-out gathers each record from the
// tile's 32 KB instead, whose lines the block's other lanes read too (L2)
template <bool RECS>
__global__ void __launch_bounds__(kBlock) epoch_scatter_kernel(EpochCtx c, const uint16_t* __restrict__ bins,
                                                               const int32_t* __restrict__ off,
                                                               const int4* __restrict__ pairs,
                                                               int4* __restrict__ out_recs,
                                                               int32_t* __restrict__ out_idx) {
    extern __shared__ int32_t lds[];
    const int nbn = c.n_bins;
    int32_t* stage = lds;                        // [kEpochTile] pair index of each tile position
    int32_t* gstage = stage + kEpochTile;        // [kEpochTile] its global position
    int32_t* wtot = gstage + kEpochTile;         // [4] wave totals of the bin scan
    int32_t* wcnt = wtot + kWavesPerBlock;       // [4][n_bins] each wave's count per bin, then its
                                                 //   next tile position per bin (in place)
    int32_t* delta = wcnt + kWavesPerBlock * nbn;   // [n_bins] global - tile position
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t tile0 = (uint32_t)blockIdx.x * kEpochTile;
    const uint32_t qend = min(tile0 + (uint32_t)kEpochTile, c.n);
    const int tile_len = (int)(qend - tile0);
    for (int b = tid; b < kWavesPerBlock * nbn; b += kBlock) wcnt[b] = 0;
    __syncthreads();
    // this wave's 512 consecutive pairs' bins
    const uint32_t w0 = tile0 + (uint32_t)(w * kEpochWaveSpan);
    constexpr int KC = kEpochWaveSpan / kWave;   // 8 chunks of 64 pairs
    int key[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) {
        const uint32_t q = w0 + (uint32_t)(k * kWave + lane);
        key[k] = q < qend ? (int)bins[q] : nbn;   // sentinel: no bin
    }
#pragma unroll
    for (int k = 0; k < KC; ++k)
        if (key[k] < nbn) atomicAdd(&wcnt[w * nbn + key[k]], 1);
    __syncthreads();
    // the tile's bin starts (exclusive scan over bins), each wave's first
    // position per bin, and the bins' global offsets (pass 2)
    constexpr int kMaxPer = kEpochMaxBins / kBlock;
    const int per = (nbn + kBlock - 1) / kBlock;   // consecutive bins per thread (<= kMaxPer)
    int32_t tot[kMaxPer];
    int32_t mine = 0;
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i) {
        const int b = tid * per + i;
        tot[i] = 0;
        if (i < per && b < nbn) {
#pragma unroll
            for (int v = 0; v < kWavesPerBlock; ++v) tot[i] += wcnt[v * nbn + b];
        }
        mine += tot[i];
    }
    int32_t start = block_excl_scan(mine, wtot);
#pragma unroll
    for (int i = 0; i < kMaxPer; ++i) {
        const int b = tid * per + i;
        if (i < per && b < nbn) {
            int32_t s = start;
#pragma unroll
            for (int v = 0; v < kWavesPerBlock; ++v) {   // this thread's column only: in place
                const int32_t t = wcnt[v * nbn + b];
                wcnt[v * nbn + b] = s;
                s += t;
            }
            delta[b] = off[(int64_t)blockIdx.x * nbn + b] - start;
            start += tot[i];
        }
    }
    __syncthreads();
    // stable ranks: the wave's chunks in pair order, the lanes of a chunk
    // sharing a bin by ballots (lower lane = lower pair)
    const uint64_t below = (1ull << lane) - 1ull;
    int32_t* pos = wcnt + w * nbn;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
        uint64_t peers = ~0ull;
        for (int bit = 0; bit < c.nbits; ++bit) {
            const bool s = (key[k] >> bit) & 1;
            const uint64_t m = __ballot(s);
            peers &= s ? m : ~m;
        }
        const int rank = __popcll(peers & below);
        if (key[k] < nbn) {
            // every lane reads the bin's position before its first lane moves
            // it on (a wave's LDS instructions execute in order)
            const int32_t lp = pos[key[k]] + rank;
            if (rank == 0) pos[key[k]] = lp + __popcll(peers);
            gstage[lp] = lp + delta[key[k]];
            stage[lp] = (int32_t)(w0 + (uint32_t)(k * kWave + lane));
        }
    }
    __syncthreads();
    // each bin's run with consecutive lanes; the records form issues all of a
    // thread's gathers before its first store (one memory round trip, not
    // kEpochItems)
    if (RECS) {
        int4 r[kEpochItems];
        int32_t g[kEpochItems];
#pragma unroll
        for (int i = 0; i < kEpochItems; ++i) {
            // past the tile's end (its last, partial tile only): entry 0 again,
            // an identical second store of the same record -- every load and
            // store stays unconditional, so the compiler cannot sink each load
            // into its store's branch and wait for it there (kEpochItems round
            // trips instead of one, seen in the ISA)
            const int L = tid + i * kBlock;
            const int Lc = L < tile_len ? L : 0;
            g[i] = gstage[Lc];
            r[i] = pairs[stage[Lc]];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < kEpochItems; ++i) out_recs[g[i]] = r[i];
    } else {
#pragma unroll
        for (int i = 0; i < kEpochItems; ++i) {
            const int L = tid + i * kBlock;
            if (L < tile_len) out_idx[gstage[L]] = stage[L];
        }
    }
}

EpochCtx epoch_ctx(const PermKey& p, int64_t nnz, int B) {
    EpochCtx c{};
    c.n = (uint32_t)p.n;
    c.mask = (uint32_t)p.mask;
    c.shift = p.shift;
    c.B = (uint32_t)B;
    for (int r = 0; r < 3; ++r) {
        c.k[r] = (uint32_t)p.k[r];
        c.mi[r] = (uint32_t)perm_mul_inverse(p.m[r]);
    }
    int bits = 0;
    while (bits < 32 && (1ull << bits) - 1ull < (uint64_t)p.mask) ++bits;
    int steps = 0;
    for (uint64_t t = p.shift; t < (uint64_t)bits; t <<= 1) ++steps;
    c.xs_steps = steps;
    c.magic = B > 1 ? ~0ull / (uint64_t)B + 1ull : 0ull;
    c.nb = (uint32_t)(nnz / B);
    c.n_used = c.nb * (uint32_t)B;
    c.n_bins = (int32_t)c.nb + 1;
    int nbits = 0;
    while ((1 << nbits) <= c.n_bins) ++nbits;   // the sentinel n_bins needs its own code
    c.nbits = nbits;
    c.n_tiles = (nnz + kEpochTile - 1) / kEpochTile;
    return c;
}

int64_t n_chunks_of(int64_t n_tiles) { return (n_tiles + kEpochChunkTiles - 1) / kEpochChunkTiles; }

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace

bool epoch_count_ok(int64_t nnz, int B) {
    return nnz > 0 && nnz <= INT32_MAX && B > 0 && nnz / B + 1 <= kEpochMaxBins;
}

// bins uint16[nnz], then cnt / offsets int32[n_tiles][n_bins], chunk sums int32[n_chunks][n_bins]
size_t epoch_count_scratch(int64_t nnz, int B) {
    if (!epoch_count_ok(nnz, B)) return 0;
    const int64_t n_bins = nnz / B + 1;
    const int64_t n_tiles = (nnz + kEpochTile - 1) / kEpochTile;
    return align16((size_t)nnz * sizeof(uint16_t)) +
           (size_t)((n_tiles + n_chunks_of(n_tiles)) * n_bins) * sizeof(int32_t);
}

hipError_t launch_epoch_count(const PermKey& p, int64_t nnz, int B, const int4* pairs, int4* out_recs,
                              int32_t* out_idx, void* tmp, size_t tmp_bytes, hipStream_t s) {
    if (!epoch_count_ok(nnz, B) || (uint64_t)nnz != p.n || p.mask > 0xFFFFFFFFull) return hipErrorInvalidValue;
    if ((pairs == nullptr) != (out_recs == nullptr) || (out_recs == nullptr) == (out_idx == nullptr))
        return hipErrorInvalidValue;
    if (tmp_bytes < epoch_count_scratch(nnz, B)) return hipErrorInvalidValue;
    const EpochCtx c = epoch_ctx(p, nnz, B);
    const int64_t n_chunks = n_chunks_of(c.n_tiles);
    uint16_t* bins = static_cast<uint16_t*>(tmp);
    int32_t* cnt = reinterpret_cast<int32_t*>(static_cast<char*>(tmp) + align16((size_t)nnz * sizeof(uint16_t)));
    int32_t* csum = cnt + c.n_tiles * c.n_bins;
    const dim3 grid((unsigned)c.n_tiles);
    const size_t lds1 = (size_t)c.n_bins * sizeof(int32_t) + kEpochTile * sizeof(uint16_t);
    hipLaunchKernelGGL(epoch_bins_kernel, grid, dim3(kBlock), lds1, s, c, bins, cnt);
    hipLaunchKernelGGL(epoch_chunk_sum_kernel, dim3((unsigned)n_chunks), dim3(kBlock), 0, s, c, cnt, csum);
    hipLaunchKernelGGL(epoch_chunk_scan_kernel, dim3((unsigned)((c.n_bins + kWavesPerBlock - 1) / kWavesPerBlock)),
                       dim3(kBlock), 0, s, c, csum, n_chunks);
    hipLaunchKernelGGL(epoch_tile_offsets_kernel, dim3((unsigned)n_chunks), dim3(kBlock), 0, s, c, cnt, csum);
    // <= 36 KB at kEpochMaxBins bins; 19.5 KB (8 blocks per CU) at cfg2's 96
    size_t lds3 = (size_t)(kWavesPerBlock + 1) * c.n_bins * sizeof(int32_t) +
                  (size_t)(2 * kEpochTile + kWavesPerBlock) * sizeof(int32_t);
    // (fewer blocks per CU -- LDS padded to 40 / 54 / 80 KB -- measured
    // slower: records 0.72 / 0.75 / 0.75 vs 0.70 ms, profiles/r06/r06g)
    if (out_recs)
        hipLaunchKernelGGL(epoch_scatter_kernel<true>, grid, dim3(kBlock), lds3, s, c, bins, cnt, pairs, out_recs,
                           nullptr);
    else
        hipLaunchKernelGGL(epoch_scatter_kernel<false>, grid, dim3(kBlock), lds3, s, c, bins, cnt, nullptr, nullptr,
                           out_idx);
    return hipGetLastError();
}

}  // namespace cfk
