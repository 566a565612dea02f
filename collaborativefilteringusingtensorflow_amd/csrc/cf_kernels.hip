// cf_kernels.hip -- the engine's non-gradient launches for gfx950: the draw
// (prep), the duplicate apply and its fused next draw, the dense item apply,
// the clip / init / fill / pair-record builders, the group exchange, and the
// exported launchers.  The device code itself is in cf_kernels_impl.h; the
// gradient kernels are instantiated per model in cf_grad_<model>.hip.
#include "cf_kernels_impl.h"

namespace cfk {

__global__ void init_normal_kernel(float* __restrict__ X, int64_t n, float mean, float stddev,
                                   int truncated, uint64_t seed) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = t0; k < n; k += nt) {
        uint64_t ctr = 0;
        float z;
        do {
            const uint64_t h = mix64(seed ^ mix64((uint64_t)k * 0x9E3779B97F4A7C15ull + ctr++));
            const float u1 = ((uint32_t)(h >> 40) + 0.5f) * (1.f / 16777216.f);  // (0,1)
            const float u2 = ((uint32_t)(h & 0xFFFFFF)) * (1.f / 16777216.f);
            z = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
        } while (truncated && fabsf(z) > 2.f);
        X[k] = mean + stddev * z;
    }
}

__global__ void fill_kernel(float* __restrict__ X, int64_t n, float v) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = t0; k < n; k += nt) X[k] = v;
}

// the Pos(u) set: one insert per interaction (64-bit CAS, linear probing)
__global__ void build_pos_set_kernel(const int4* __restrict__ pairs, int64_t nnz,
                                     unsigned long long* __restrict__ set, uint64_t mask) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t k = t0; k < nnz; k += nt) {
        const int4 pr = pairs[k];
        const unsigned long long key = ((unsigned long long)(uint32_t)pr.x << 32) | (uint32_t)pr.y;
        uint64_t s = pos_slot(key, mask);
        while (true) {
            const unsigned long long prev = atomicCAS(set + s, kPosEmpty, key);
            if (prev == kPosEmpty || prev == key) break;
            s = (s + 1) & mask;
        }
    }
}

__global__ void build_pairs_kernel(const int64_t* __restrict__ indptr,
                                   const int32_t* __restrict__ indices, int64_t n_users,
                                   int4* __restrict__ pairs) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t u = t0; u < n_users; u += nt)
        for (int64_t k = indptr[u]; k < indptr[u + 1]; ++k)
            pairs[k] = make_int4((int)u, indices[k], (int)(uint32_t)indptr[u],
                                 (int)(indptr[u + 1] - indptr[u]));
}

// ---------------------------------------------------------------------------
// GBPR group exchange (user-sharded engine).  Group members are drawn from
// the item's users over ALL ranks (sampler_gbpr.py:41); a member owned by
// another rank is fetched from its owner and its gradient row sent back
// (DESIGN 5).  Pack: histogram the remote members per (block, owner), scan
// owner-major, scatter each id to its packed position (deterministic: ballot
// ranks inside the block) and recode the occurrence as -1 - position.
// ---------------------------------------------------------------------------
constexpr int kMaxWorld = 64;

__device__ __forceinline__ int owner_of(const int64_t* __restrict__ bounds, int world, int64_t g) {
    int o = 0;
    for (int k = 1; k < world; ++k) o += (g >= bounds[k]) ? 1 : 0;
    return o;
}

__global__ __launch_bounds__(kBlock) void xchg_hist_kernel(XchgArgs a) {
    __shared__ int s_h[kMaxWorld];
    for (int k = threadIdx.x; k < a.world; k += kBlock) s_h[k] = 0;
    __syncthreads();
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q < a.n) {
        const int v = a.occ[q];
        if (v < 0) atomicAdd(&s_h[owner_of(a.bounds, a.world, (int64_t)(-1 - v))], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.world; k += kBlock) a.hist[blockIdx.x * a.world + k] = s_h[k];
}

// one block: exclusive scan of hist in owner-major order (owner o's ids are
// contiguous, blocks in order inside it); per-owner totals into counts
__global__ __launch_bounds__(kBlock) void xchg_scan_kernel(XchgArgs a, int nblk) {
    __shared__ int s_w[kWavesPerBlock];
    __shared__ int s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    for (int o = 0; o < a.world; ++o) {
        const int start = s_carry;
        for (int b0 = 0; b0 < nblk; b0 += kBlock) {
            const int b = b0 + threadIdx.x;
            const int v = (b < nblk) ? a.hist[b * a.world + o] : 0;
            const int inc = wave_incl_scan(v);
            if (lane == 63) s_w[wv] = inc;
            __syncthreads();
            int base = s_carry;
            for (int k = 0; k < wv; ++k) base += s_w[k];
            if (b < nblk) a.hist[b * a.world + o] = base + inc - v;
            __syncthreads();
            if (threadIdx.x == 0) s_carry += s_w[0] + s_w[1] + s_w[2] + s_w[3];
            __syncthreads();
        }
        if (threadIdx.x == 0) a.counts[o] = s_carry - start;
        __syncthreads();
    }
    if (threadIdx.x == 0) a.counts[a.world] = s_carry;
}

__global__ __launch_bounds__(kBlock) void xchg_scatter_kernel(XchgArgs a) {
    __shared__ int s_cnt[kWavesPerBlock][kMaxWorld];
    const int q = blockIdx.x * kBlock + threadIdx.x;
    const int v = (q < a.n) ? a.occ[q] : 0;
    const int o = (v < 0) ? owner_of(a.bounds, a.world, (int64_t)(-1 - v)) : -1;
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int my_rank = 0;
    for (int k = 0; k < a.world; ++k) {
        const unsigned long long m = __ballot(o == k);
        if (o == k) my_rank = __popcll(m & lt);
        if (lane == 0) s_cnt[wv][k] = __popcll(m);
    }
    __syncthreads();
    if (o >= 0) {
        int pos = a.hist[blockIdx.x * a.world + o] + my_rank;
        for (int k = 0; k < wv; ++k) pos += s_cnt[k][o];
        a.send_ids[pos] = -1 - v;
        a.occ[q] = -1 - pos;
    }
}

// owner side, per requested row: flag its count word (it takes the summed
// path, see kRemoteFlag) and copy its pre-update value out
template <int EPL>
__global__ __launch_bounds__(kBlock) void xchg_serve_kernel(const int32_t* __restrict__ ids, int64_t n,
                                                            int64_t u0, int32_t* __restrict__ cntU,
                                                            int32_t* __restrict__ own,
                                                            const float* __restrict__ U,
                                                            float* __restrict__ rows, int d) {
    const int gl = threadIdx.x & (kGL - 1);
    const int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
    if (j >= n) return;
    const int64_t r = (int64_t)ids[j] - u0;
    if (gl == 0) {
        // the first server of a row with no local occurrence applies it
        const int32_t old = atomicOr(&cntU[r], kRemoteFlag);
        own[j] = (old == 0) ? 1 : 0;
    }
    float x[EPL];
    gload<EPL>(U, r, d, gl, x);
    gstore<EPL>(rows, j, d, gl, x);
}

template <int EPL>
__global__ __launch_bounds__(kBlock) void xchg_accumulate_kernel(const int32_t* __restrict__ ids,
                                                                 int64_t n, int64_t u0,
                                                                 const float* __restrict__ grads,
                                                                 float* __restrict__ GU, int d) {
    const int gl = threadIdx.x & (kGL - 1);
    const int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
    if (j >= n) return;
    float g[EPL];
    gload<EPL>(grads, j, d, gl, g);
    gatomic<EPL>(GU, (int64_t)ids[j] - u0, d, gl, g);
}

int grad_fast_w(const StepArgs& a) { return fast_w(a); }
bool grad_lds(const StepArgs& a) { return lds_path(a); }

int grad_blocks(const StepArgs& a, bool with_draw) {
    if (!with_draw && lds_path(a)) return (a.B + kGroupsPerBlock - 1) / kGroupsPerBlock;
    if (a.srec != nullptr)   // grad_sort_kernel: CF_SORT_TILES tiles of kPsortPPB positions per block
        return (a.B + CF_SORT_TILES * kPsortPPB - 1) / (CF_SORT_TILES * kPsortPPB);
    const int fw = fast_w(a);
    const int B = a.B;
    const int gpb = (CF_GRAD_WAVE_BLOCKS && !with_draw) ? kWave / kGL : kGroupsPerBlock;
    const int p5 = (a.model == GBPR && epl_for(a.d) <= 4) ? CF_FAST_PAIRS_GBPR_W5 : CF_FAST_PAIRS_W5;
    const int ppb = fw == 1 ? CF_FAST_PAIRS_W1 * gpb
                  : fw == 5 ? p5 * gpb : kPairsPerBlock;
    return (B + ppb - 1) / ppb;
}

int grad_blocks_max(int B) { return (B + kWave / kGL - 1) / (kWave / kGL); }

hipError_t launch_prep(const StepArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    const int ppb = prep_pairs_per_block(a);
    const int blocks = (a.B + ppb - 1) / ppb;
    switch (a.model) {
        case GBPR: hipLaunchKernelGGL(prep_kernel<GBPR>, dim3(blocks), dim3(kBlock), 0, s, a); break;
        default: hipLaunchKernelGGL(prep_kernel<BPR>, dim3(blocks), dim3(kBlock), 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_grad(const StepArgs& a, hipStream_t s, const StepArgs* next) {
    if (a.B <= 0) return next ? launch_prep(*next, s) : hipSuccess;
    if (next && next->model != a.model) return hipErrorInvalidValue;
    if (a.srec != nullptr && fast_w(a) == 0) return hipErrorInvalidValue;   // pos_sort: phased kernel only
    if (a.pf_out != nullptr && a.srec == nullptr) return hipErrorInvalidValue;   // only grad_sort_kernel prefetches
    switch (a.model) {
        case BPR: return launch_grad_bpr(a, next, s);
        case GBPR: return launch_grad_gbpr(a, next, s);
        case CML: return launch_grad_cml(a, next, s);
        case PLR: return next ? hipErrorInvalidValue : launch_grad_plr_t(a, s);
        default: return launch_grad_amf(a, next, s);
    }
}

static int apply_grid(const ApplyArgs& a) {
    // 64 work items (user occurrences, item occurrences, served rows) per
    // detecting wave
    const int64_t items = (a.count_users ? a.nU : 0) + (a.count_items ? a.nV : 0) + a.nS;
    const int64_t per = (int64_t)kApplyDetectWaves * kApplyChunk;
    int64_t blocks = (items + per - 1) / per;
    if (blocks > 16384) blocks = 16384;  // grid-stride over the work items
    if (blocks < 1) blocks = 1;        // block 0 still reduces the loss
    return (int)blocks;
}

#ifndef CF_APPLY_WAVE_BLOCKS
#define CF_APPLY_WAVE_BLOCKS 0
#endif

template <bool HOT>
static hipError_t launch_apply_h(const ApplyArgs& a, hipStream_t s) {
    const dim3 grid(apply_grid(a)), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((apply_kernel<1, HOT>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((apply_kernel<2, HOT>), grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL((apply_kernel<4, HOT>), grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL((apply_kernel<8, HOT>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((apply_kernel<16, HOT>), grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

// the pos_sort apply (+ the next step's draw when nx is given); PS false: the
// dense item rows of the slot-row / record path (apply_rows_item_block); FX:
// the deterministic pos_sort path's fixed-point sums (ApplyArgs::det_fx)
template <bool PS = true, bool FX = false>
static hipError_t launch_apply_ps_t(const ApplyArgs& p, const StepArgs* nx, hipStream_t s) {
    const int64_t nUw = !p.count_users ? 0 : p.dense_users ? p.n_users : p.nU;
    const int64_t nVw = (p.count_items && !p.dense_items) ? p.nV : 0;
    const int64_t nbI64 = (p.count_items && p.dense_items)
                              ? (p.item_r1 - p.item_r0 + kGroupsPerBlock - 1) / kGroupsPerBlock : 0;
    const int64_t nbW64 = (nUw + nVw + kBlock - 1) / kBlock;
    const int np = prep_blocks(nx);
    if (nbI64 + nbW64 + np > INT32_MAX) return hipErrorInvalidValue;
    const int nbI = (int)nbI64, nbW = (int)std::max<int64_t>(nbW64, nbI64 == 0 ? 1 : 0);   // block 0 folds the loss
    const dim3 grid(nbI + nbW + np), block(kBlock);
    const StepArgs n = nx ? *nx : StepArgs{};
    const bool full = CF_ASSUME_FULL_APPLY && p.d == kGL * epl_for(p.d);
    if (np > 0) {
        switch (epl_for(p.d)) {
            case 1: hipLaunchKernelGGL((apply_ps_kernel<1, true, PS, FX>), grid, block, 0, s, p, n, nbI, nbW); break;
            case 2: hipLaunchKernelGGL((apply_ps_kernel<2, true, PS, FX>), grid, block, 0, s, p, n, nbI, nbW); break;
            case 4:
                if (full) hipLaunchKernelGGL((apply_ps_kernel<4, true, PS, FX, true>), grid, block, 0, s, p, n, nbI, nbW);
                else hipLaunchKernelGGL((apply_ps_kernel<4, true, PS, FX>), grid, block, 0, s, p, n, nbI, nbW);
                break;
            default:
                if (full) hipLaunchKernelGGL((apply_ps_kernel<8, true, PS, FX, true>), grid, block, 0, s, p, n, nbI, nbW);
                else hipLaunchKernelGGL((apply_ps_kernel<8, true, PS, FX>), grid, block, 0, s, p, n, nbI, nbW);
                break;
        }
    } else {
        switch (epl_for(p.d)) {
            case 1: hipLaunchKernelGGL((apply_ps_kernel<1, false, PS, FX>), grid, block, 0, s, p, n, nbI, nbW); break;
            case 2: hipLaunchKernelGGL((apply_ps_kernel<2, false, PS, FX>), grid, block, 0, s, p, n, nbI, nbW); break;
            case 4:
                if (full) hipLaunchKernelGGL((apply_ps_kernel<4, false, PS, FX, true>), grid, block, 0, s, p, n, nbI, nbW);
                else hipLaunchKernelGGL((apply_ps_kernel<4, false, PS, FX>), grid, block, 0, s, p, n, nbI, nbW);
                break;
            default:
                if (full) hipLaunchKernelGGL((apply_ps_kernel<8, false, PS, FX, true>), grid, block, 0, s, p, n, nbI, nbW);
                else hipLaunchKernelGGL((apply_ps_kernel<8, false, PS, FX>), grid, block, 0, s, p, n, nbI, nbW);
                break;
        }
    }
    return hipGetLastError();
}

template <bool PS = true>
static hipError_t launch_apply_ps(const ApplyArgs& p, const StepArgs* nx, hipStream_t s) {
    if constexpr (PS) {
        if (p.det_fx) return launch_apply_ps_t<true, true>(p, nx, s);
    }
    return launch_apply_ps_t<PS, false>(p, nx, s);
}

// the slot-row / record path's dense item apply applies (the engine sets
// dense_items only outside pos_sort and deterministic mode, for a table not
// much larger than the batch's item occurrences)
static bool dense_rows_apply(const ApplyArgs& a) {
    return a.cntP == nullptr && a.dense_items && a.count_items && a.nS == 0 && a.hotP == nullptr &&
           a.offV == nullptr && epl_for(a.d) <= 8;
}

hipError_t launch_apply(const ApplyArgs& a, hipStream_t s) {
    if (CF_APPLY_WAVE_BLOCKS) {
        // one-wave apply blocks have no pos_sort owner rule: refuse rather
        // than skip or double-apply an item whose positives count in cntP
        if (a.cntP != nullptr || a.hotP != nullptr) return hipErrorInvalidValue;
        const dim3 grid(apply_grid(a)), block(kWave);
        switch (epl_for(a.d)) {
            case 1: hipLaunchKernelGGL(apply_wave_kernel<1>, grid, block, 0, s, a); break;
            case 2: hipLaunchKernelGGL(apply_wave_kernel<2>, grid, block, 0, s, a); break;
            case 4: hipLaunchKernelGGL(apply_wave_kernel<4>, grid, block, 0, s, a); break;
            case 8: hipLaunchKernelGGL(apply_wave_kernel<8>, grid, block, 0, s, a); break;
            default: hipLaunchKernelGGL(apply_wave_kernel<16>, grid, block, 0, s, a); break;
        }
        return hipGetLastError();
    }
    if (a.cntP != nullptr) {   // pos_sort (d <= 128, no served rows, no deterministic tiles)
        if (a.hotP != nullptr || a.nS > 0 || epl_for(a.d) > 8) return hipErrorInvalidValue;
        return launch_apply_ps(a, nullptr, s);
    }
    if (dense_rows_apply(a)) return launch_apply_ps<false>(a, nullptr, s);
    return a.hotP != nullptr ? launch_apply_h<true>(a, s) : launch_apply_h<false>(a, s);
}

template <int MODEL, bool HOT>
static hipError_t launch_apply_prep_m(const ApplyArgs& p, const StepArgs& a, hipStream_t s) {
    const int na = apply_grid(p);
    const int np = prep_blocks(&a);
    const dim3 grid(na + np), block(kBlock);
    switch (epl_for(p.d)) {
        case 1: hipLaunchKernelGGL((apply_prep_kernel<1, MODEL, HOT>), grid, block, 0, s, p, a, na); break;
        case 2: hipLaunchKernelGGL((apply_prep_kernel<2, MODEL, HOT>), grid, block, 0, s, p, a, na); break;
        case 4: hipLaunchKernelGGL((apply_prep_kernel<4, MODEL, HOT>), grid, block, 0, s, p, a, na); break;
        case 8: hipLaunchKernelGGL((apply_prep_kernel<8, MODEL, HOT>), grid, block, 0, s, p, a, na); break;
        default: hipLaunchKernelGGL((apply_prep_kernel<16, MODEL, HOT>), grid, block, 0, s, p, a, na); break;
    }
    return hipGetLastError();
}

hipError_t launch_apply_prep(const ApplyArgs& p, const StepArgs& a, hipStream_t s) {
    if (a.B <= 0) return launch_apply(p, s);
    if (p.cntP != nullptr)   // pos_sort: BPR / AMF / CML (their draw is prep_body<BPR>)
        return (p.hotP != nullptr || p.nS > 0 || a.model == GBPR || epl_for(p.d) > 8)
                   ? hipErrorInvalidValue : launch_apply_ps(p, &a, s);
    if (p.hotP != nullptr)
        return a.model == GBPR ? launch_apply_prep_m<GBPR, true>(p, a, s) : launch_apply_prep_m<BPR, true>(p, a, s);
    if (a.model != GBPR && dense_rows_apply(p)) return launch_apply_ps<false>(p, &a, s);   // draw is prep_body<BPR>
    return a.model == GBPR ? launch_apply_prep_m<GBPR, false>(p, a, s) : launch_apply_prep_m<BPR, false>(p, a, s);
}

static int row_grid(int64_t n_rows) {
    int64_t b = (n_rows + kGroupsPerBlock - 1) / kGroupsPerBlock;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_apply_dense(const DenseArgs& a, hipStream_t s) {
    const dim3 grid(row_grid(a.n_rows)), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL(apply_dense_kernel<1>, grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL(apply_dense_kernel<2>, grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL(apply_dense_kernel<4>, grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL(apply_dense_kernel<8>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(apply_dense_kernel<16>, grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_zero_rows(const int32_t* occ, int64_t n, float* G, float* Gb, int d, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid(row_grid(n)), block(kBlock);
    switch (epl_for(d)) {
        case 1: hipLaunchKernelGGL(zero_rows_kernel<1>, grid, block, 0, s, occ, n, G, Gb, d); break;
        case 2: hipLaunchKernelGGL(zero_rows_kernel<2>, grid, block, 0, s, occ, n, G, Gb, d); break;
        case 4: hipLaunchKernelGGL(zero_rows_kernel<4>, grid, block, 0, s, occ, n, G, Gb, d); break;
        case 8: hipLaunchKernelGGL(zero_rows_kernel<8>, grid, block, 0, s, occ, n, G, Gb, d); break;
        default: hipLaunchKernelGGL(zero_rows_kernel<16>, grid, block, 0, s, occ, n, G, Gb, d); break;
    }
    return hipGetLastError();
}

hipError_t launch_clip_full(float* X, int64_t n_rows, int d, float c, hipStream_t s) {
    const dim3 grid(row_grid(n_rows)), block(kBlock);
    switch (epl_for(d)) {
        case 1: hipLaunchKernelGGL(clip_full_kernel<1>, grid, block, 0, s, X, n_rows, d, c); break;
        case 2: hipLaunchKernelGGL(clip_full_kernel<2>, grid, block, 0, s, X, n_rows, d, c); break;
        case 4: hipLaunchKernelGGL(clip_full_kernel<4>, grid, block, 0, s, X, n_rows, d, c); break;
        case 8: hipLaunchKernelGGL(clip_full_kernel<8>, grid, block, 0, s, X, n_rows, d, c); break;
        default: hipLaunchKernelGGL(clip_full_kernel<16>, grid, block, 0, s, X, n_rows, d, c); break;
    }
    return hipGetLastError();
}

static int grid_for(int64_t n) {
    int64_t b = (n + kBlock - 1) / kBlock;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_init_normal(float* X, int64_t n, float mean, float stddev, int truncated,
                              uint64_t seed, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(init_normal_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, X, n, mean,
                       stddev, truncated, seed);
    return hipGetLastError();
}

hipError_t launch_fill(float* X, int64_t n, float v, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, X, n, v);
    return hipGetLastError();
}

hipError_t launch_build_pos_set(const int4* pairs, int64_t nnz, unsigned long long* set,
                                uint64_t mask, hipStream_t s) {
    hipError_t e = hipMemsetAsync(set, 0xFF, (mask + 1) * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    if (nnz <= 0) return hipSuccess;
    hipLaunchKernelGGL(build_pos_set_kernel, dim3(grid_for(nnz)), dim3(kBlock), 0, s, pairs, nnz, set,
                       mask);
    return hipGetLastError();
}

hipError_t launch_build_pairs(const int64_t* indptr, const int32_t* indices, int64_t n_users,
                              int4* pairs, hipStream_t s) {
    if (n_users <= 0) return hipSuccess;
    hipLaunchKernelGGL(build_pairs_kernel, dim3(grid_for(n_users)), dim3(kBlock), 0, s, indptr,
                       indices, n_users, pairs);
    return hipGetLastError();
}

hipError_t launch_xchg_pack(const XchgArgs& a, hipStream_t s) {
    if (a.world < 1 || a.world > kMaxWorld) return hipErrorInvalidValue;
    const int nblk = a.n > 0 ? (a.n + kBlock - 1) / kBlock : 0;
    if (nblk > 0) hipLaunchKernelGGL(xchg_hist_kernel, dim3(nblk), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(xchg_scan_kernel, dim3(1), dim3(kBlock), 0, s, a, nblk);
    if (nblk > 0) hipLaunchKernelGGL(xchg_scatter_kernel, dim3(nblk), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_xchg_serve(const int32_t* ids, int64_t n, int64_t u0, int32_t* cntU, int32_t* own,
                             const float* U, float* rows, int d, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + kGroupsPerBlock - 1) / kGroupsPerBlock)), block(kBlock);
    switch (epl_for(d)) {
        case 1: hipLaunchKernelGGL(xchg_serve_kernel<1>, grid, block, 0, s, ids, n, u0, cntU, own, U, rows, d); break;
        case 2: hipLaunchKernelGGL(xchg_serve_kernel<2>, grid, block, 0, s, ids, n, u0, cntU, own, U, rows, d); break;
        case 4: hipLaunchKernelGGL(xchg_serve_kernel<4>, grid, block, 0, s, ids, n, u0, cntU, own, U, rows, d); break;
        case 8: hipLaunchKernelGGL(xchg_serve_kernel<8>, grid, block, 0, s, ids, n, u0, cntU, own, U, rows, d); break;
        default: hipLaunchKernelGGL(xchg_serve_kernel<16>, grid, block, 0, s, ids, n, u0, cntU, own, U, rows, d); break;
    }
    return hipGetLastError();
}

hipError_t launch_xchg_accumulate(const int32_t* ids, int64_t n, int64_t u0, const float* grads,
                                  float* GU, int d, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n + kGroupsPerBlock - 1) / kGroupsPerBlock)), block(kBlock);
    switch (epl_for(d)) {
        case 1: hipLaunchKernelGGL(xchg_accumulate_kernel<1>, grid, block, 0, s, ids, n, u0, grads, GU, d); break;
        case 2: hipLaunchKernelGGL(xchg_accumulate_kernel<2>, grid, block, 0, s, ids, n, u0, grads, GU, d); break;
        case 4: hipLaunchKernelGGL(xchg_accumulate_kernel<4>, grid, block, 0, s, ids, n, u0, grads, GU, d); break;
        case 8: hipLaunchKernelGGL(xchg_accumulate_kernel<8>, grid, block, 0, s, ids, n, u0, grads, GU, d); break;
        default: hipLaunchKernelGGL(xchg_accumulate_kernel<16>, grid, block, 0, s, ids, n, u0, grads, GU, d); break;
    }
    return hipGetLastError();
}

__global__ void uncount_kernel(const int32_t* __restrict__ occ, int64_t n, int32_t* __restrict__ cnt) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nt = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = t0; q < n; q += nt) {
        const int32_t r = occ[q];
        if (r >= 0) cnt[r] = 0;
    }
}

// a discarded draw's phantoms (StepArgs::spec_ph): one block uncounts them,
// then re-zeroes the phantom count after every lane has read it
__global__ __launch_bounds__(kBlock) void uncount_spec_kernel(const int2* __restrict__ ph, int* __restrict__ n,
                                                               int32_t* __restrict__ cnt) {
    const int np = *n;
    for (int k = threadIdx.x; k < np; k += kBlock) atomicSub(&cnt[ph[k].x], 1);
    __syncthreads();
    if (threadIdx.x == 0) *n = 0;
}

hipError_t launch_uncount_spec(const int2* ph, int* n, int32_t* cnt, hipStream_t s) {
    hipLaunchKernelGGL(uncount_spec_kernel, dim3(1), dim3(kBlock), 0, s, ph, n, cnt);
    return hipGetLastError();
}

bool pair_prefetch_built() { return CF_PAIR_PREFETCH != 0; }

hipError_t launch_uncount(const int32_t* occ, int64_t n, int32_t* cnt, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(uncount_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, occ, n, cnt);
    return hipGetLastError();
}

__global__ void pack_batch_kernel(PackArgs a) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.B) return;
    bool ok = true;
    const int32_t u = a.u[(int64_t)p * a.us], i = a.u[(int64_t)p * a.us + 1];
    const bool uok = u >= 0 && u < a.n_users, iok = i >= 0 && i < a.n_items;
    ok = uok && iok;
    a.occU[p] = uok ? u : 0;
    a.occV[p] = iok ? i : 0;
    for (int w = 0; w < a.W; ++w) {
        const int32_t j = a.j[(int64_t)p * a.js + w];
        const bool jok = j >= 0 && j < a.n_items;
        ok = ok && jok;
        a.occV[a.B + (int64_t)p * a.W + w] = jok ? j : 0;
    }
    for (int k = 0; k < a.G; ++k) {
        const int32_t g = a.g[(int64_t)p * a.gs + k];
        int32_t v;
        if (a.sharded) {
            const bool gok = g >= 0 && g < a.total_users;
            ok = ok && gok;
            v = !gok ? 0 : (g >= a.shard_u0 && g < a.shard_u1) ? (int32_t)(g - a.shard_u0) : -1 - g;
        } else {
            const bool gok = g >= 0 && g < a.n_users;
            ok = ok && gok;
            v = gok ? g : 0;
        }
        a.occU[a.B + (int64_t)p * a.G + k] = v;
    }
    if (!ok) atomicMin(a.bad, p);
}

hipError_t launch_pack_batch(const PackArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    hipLaunchKernelGGL(pack_batch_kernel, dim3((a.B + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

uint64_t mix64_host(uint64_t z) { return mix64(z); }

PermKey make_perm_key(uint64_t n, uint64_t seed, uint64_t epoch) {
    PermKey p{};
    p.n = n;
    uint32_t bits = 1;
    while (bits < 63 && (1ull << bits) < n) ++bits;
    p.mask = (1ull << bits) - 1ull;
    p.shift = bits / 2 > 0 ? bits / 2 : 1;
    uint64_t h = mix64(seed ^ mix64(epoch + 0x5851F42D4C957F2Dull));
    for (int r = 0; r < 3; ++r) {
        h = mix64(h + (uint64_t)r);
        p.k[r] = h & p.mask;
        p.m[r] = (mix64(h ^ 0xA0761D6478BD642Full) | 1ull);
    }
    return p;
}

hipError_t launch_det_hot(const HotArgs& h, hipStream_t s) {
    const int64_t ntiles = h.n / kDetTile;
    if (ntiles <= 0) return hipSuccess;
    const dim3 grid((unsigned)(ntiles < 16384 ? ntiles : 16384)), block(kBlock);
    switch (epl_for(h.d)) {
        case 1: hipLaunchKernelGGL(det_hot_kernel<1>, grid, block, 0, s, h); break;
        case 2: hipLaunchKernelGGL(det_hot_kernel<2>, grid, block, 0, s, h); break;
        case 4: hipLaunchKernelGGL(det_hot_kernel<4>, grid, block, 0, s, h); break;
        case 8: hipLaunchKernelGGL(det_hot_kernel<8>, grid, block, 0, s, h); break;
        default: hipLaunchKernelGGL(det_hot_kernel<16>, grid, block, 0, s, h); break;
    }
    return hipGetLastError();
}

}  // namespace cfk
