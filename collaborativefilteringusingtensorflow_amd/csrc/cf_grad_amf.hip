// cf_grad_amf.hip -- the AMF gradient kernels' instantiations (launch_grad_m<AMF>);
// one translation unit per model so that the build compiles them in parallel.
// Also the two launches of the apr mode (cf_config.amf_mode 1) around it.
#include "cf_kernels_impl.h"

namespace cfk {

// Rows in the interleaved lane layout (element s * 16 + gl in lane gl, slot
// s): every wave instruction touches 64 contiguous bytes per row, so a float
// atomic leaves L2 as one 64-B request per row instead of the 32-B-strided
// requests of the vector layout (vec_rows; apr_embed_kernel took 699 us at
// cfg5 with it).  Rows sit in memory in element order either way; the
// kernel's dot products and gradient rows only need every row it holds in
// one layout.
template <int EPL>
__device__ __forceinline__ void il_load(const float* __restrict__ X, int64_t r, int d, int gl, float (&x)[EPL]) {
    const float* row = X + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        x[s] = e < d ? row[e] : 0.f;
    }
}

template <int EPL>
__device__ __forceinline__ void il_atomic(float* __restrict__ G, int64_t r, int d, int gl, const float (&g)[EPL]) {
    float* row = G + r * (int64_t)d;
#pragma unroll
    for (int s = 0; s < EPL; ++s) {
        const int e = s * kGL + gl;
        if (e < d) unsafeAtomicAdd(row + e, g[s]);
    }
}

// AMF apr, before the gradient launch: the batch's embedding-loss gradient
// dL_embed/dX (amf.py:130: tf.gradients of __embed_loss__, densified by
// stop_gradient = summed per row) for every DUPLICATED row, by float atomics
// into Gadv.  Rows seen once are skipped: apr_pair takes theirs from its own
// registers.  A pair whose rows are all seen once loads nothing past its ids
// and counts.
template <int EPL, int WT>
__global__ __launch_bounds__(kBlock) void apr_embed_kernel(StepArgs a) {
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    const int d = a.d;
    const int W = WT > 0 ? WT : a.W;
    for (int k = 0; k < kPairsPerGroup; ++k) {
        const int p = (blockIdx.x * kPairsPerGroup + k) * kGroupsPerBlock + grp;
        if (p >= a.B) break;   // group-uniform
        const int u = a.occU[p];
        const int i = a.occV[p];
        const int cu = a.cntU[u];
        const int ci = a.cntV[i];
        // multi-rank (apr_global): every item occurrence adds, a row seen once
        // here may be seen on another rank
        bool dup = cu >= 2 || ci >= 2 || a.apr_global;
        for (int w = 0; w < W && !dup; ++w) dup |= a.cntV[a.occV[a.B + p * W + w]] >= 2;
        if (!dup) continue;
        float uu[EPL], vi[EPL], gu[EPL];
        il_load<EPL>(a.U, u, d, gl, uu);
        il_load<EPL>(a.V, i, d, gl, vi);
        const float ui = gdot<EPL>(uu, vi);
#pragma unroll
        for (int s = 0; s < EPL; ++s) gu[s] = 0.f;
        float sc = 0.f;
        for (int w = 0; w < W; ++w) {
            const int j = a.occV[a.B + p * W + w];
            float vj[EPL];
            il_load<EPL>(a.V, j, d, gl, vj);
            const float c = -rcp_1p(expf(ui - gdot<EPL>(uu, vj)));
            sc += c;
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = fmaf(c, vi[s] - vj[s], gu[s]);
            if (a.apr_global || a.cntV[j] >= 2) {
#pragma unroll
                for (int s = 0; s < EPL; ++s) vj[s] = -c * uu[s];
                il_atomic<EPL>(a.GadvV, j, d, gl, vj);
            }
        }
        if (cu >= 2) il_atomic<EPL>(a.GadvU, u, d, gl, gu);
        if (a.apr_global || ci >= 2) {
#pragma unroll
            for (int s = 0; s < EPL; ++s) gu[s] = sc * uu[s];
            il_atomic<EPL>(a.GadvV, i, d, gl, gu);
        }
    }
}

// AMF apr, after the gradient launch: zero the Gadv rows apr_embed_kernel
// wrote, once per row (its rank-0 occurrence).  The gradient launch resets
// the counts of rows seen once only, so a duplicated row still reads >= 2.
template <int EPL>
__global__ __launch_bounds__(kBlock) void apr_zero_kernel(StepArgs a, int64_t nU, int64_t n) {
    const int gl = threadIdx.x & (kGL - 1);
    const int64_t q = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 4;
    if (q >= n) return;
    const bool user = q < nU;
    if (!user && a.apr_global) return;   // the item buffer is cleared whole (launch_grad_amf)
    const int64_t o = user ? q : q - nU;
    const int r = user ? a.occU[o] : a.occV[o];
    const int rank = user ? a.rankU[o] : a.rankV[o];
    const int cnt = user ? a.cntU[r] : a.cntV[r];
    if (rank != 0 || cnt < 2) return;
    float z[EPL];
#pragma unroll
    for (int s = 0; s < EPL; ++s) z[s] = 0.f;
    gstore<EPL>(user ? a.GadvU : a.GadvV, r, a.d, gl, z);
}

// AMF apr, the gradient launch: grad_kernel's pair loop and loss partials
// (one 16-lane group per pair, kPairsPerBlock pairs per block = grad_blocks()
// of a generic step) with apr_pair's arithmetic; its own kernel so that the
// generic AMF kernel keeps its registers.  DRAW: pipeline 2's draw blocks.
template <int EPL, int WT, bool DRAW>
__global__ __launch_bounds__(kBlock) void apr_grad_kernel(StepArgs a, StepArgs nx, int ng, int np) {
    int block = blockIdx.x;
    if (DRAW && minor_block(blockIdx.x, ng, np, block)) {
        prep_any<BPR>(nx, block);
        return;
    }
    __shared__ double s_loss[kGroupsPerBlock];
    const int gl = threadIdx.x & (kGL - 1);
    const int grp = threadIdx.x >> 4;
    const int d = a.d;
    float loss_g = 0.f, sq = 0.f;
    for (int k = 0; k < kPairsPerGroup; ++k) {
        const int p = (block * kPairsPerGroup + k) * kGroupsPerBlock + grp;
        if (p >= a.B) break;   // group-uniform
        const int u = a.occU[p];
        const int i = a.occV[p];
        NegRows<EPL, WT> J;
        J.prefetch(a, p, gl);
        const int cu = a.cntU[u];
        const int ci = a.cntV[i];
        const int64_t su = slot_of(cu, u, a.rankU[p], a.capU, 0, a.offU);
        const int64_t si = slot_of(ci, i, a.rankV[p], a.capV, a.repV, a.offV);
        float uu[EPL], vi[EPL];
        gload<EPL>(a.U, u, d, gl, uu);
        gload<EPL>(a.V, i, d, gl, vi);
        apr_pair<EPL, WT>(a, p, gl, u, i, cu, ci, su, si, uu, vi, J, loss_g, sq);
    }
    const float sq_g = gsum(sq);
    if (gl == 0) s_loss[grp] = (double)loss_g + 0.5 * (double)a.reg * (double)sq_g;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < kGroupsPerBlock; ++k) t += s_loss[k];
        a.loss_partial[block] = t;
    }
}

template <int WT, bool DRAW>
static hipError_t launch_apr_grad_w(const StepArgs& a, const StepArgs& n, int ng, int np, hipStream_t s) {
    const dim3 grid(ng + np), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((apr_grad_kernel<1, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 2: hipLaunchKernelGGL((apr_grad_kernel<2, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 4: hipLaunchKernelGGL((apr_grad_kernel<4, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        case 8: hipLaunchKernelGGL((apr_grad_kernel<8, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
        default: hipLaunchKernelGGL((apr_grad_kernel<16, WT, DRAW>), grid, block, 0, s, a, n, ng, np); break;
    }
    return hipGetLastError();
}

template <int WT>
static hipError_t launch_apr_grad(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    const int ng = (a.B + kPairsPerBlock - 1) / kPairsPerBlock, np = prep_blocks(nx);
    const StepArgs n = nx ? *nx : a;
    return np > 0 ? launch_apr_grad_w<WT, true>(a, n, ng, np, s) : launch_apr_grad_w<WT, false>(a, n, ng, 0, s);
}

template <int WT>
static hipError_t launch_apr_embed_w(const StepArgs& a, hipStream_t s) {
    const dim3 grid((a.B + kPairsPerBlock - 1) / kPairsPerBlock), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((apr_embed_kernel<1, WT>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((apr_embed_kernel<2, WT>), grid, block, 0, s, a); break;
        case 4: hipLaunchKernelGGL((apr_embed_kernel<4, WT>), grid, block, 0, s, a); break;
        case 8: hipLaunchKernelGGL((apr_embed_kernel<8, WT>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((apr_embed_kernel<16, WT>), grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

static hipError_t launch_apr_zero(const StepArgs& a, hipStream_t s) {
    const int64_t nU = a.B, n = nU + (int64_t)a.B * (1 + a.W);
    const dim3 grid((unsigned)((n * kGL + kBlock - 1) / kBlock)), block(kBlock);
    switch (epl_for(a.d)) {
        case 1: hipLaunchKernelGGL((apr_zero_kernel<1>), grid, block, 0, s, a, nU, n); break;
        case 2: hipLaunchKernelGGL((apr_zero_kernel<2>), grid, block, 0, s, a, nU, n); break;
        case 4: hipLaunchKernelGGL((apr_zero_kernel<4>), grid, block, 0, s, a, nU, n); break;
        case 8: hipLaunchKernelGGL((apr_zero_kernel<8>), grid, block, 0, s, a, nU, n); break;
        default: hipLaunchKernelGGL((apr_zero_kernel<16>), grid, block, 0, s, a, nU, n); break;
    }
    return hipGetLastError();
}

hipError_t launch_apr_embed(const StepArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (!a.apr || a.GadvU == nullptr || a.GadvV == nullptr || !a.count_users) return hipErrorInvalidValue;
    return a.W == 1 ? launch_apr_embed_w<1>(a, s) : a.W == 5 ? launch_apr_embed_w<5>(a, s) : launch_apr_embed_w<0>(a, s);
}

hipError_t launch_grad_amf(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    if (!a.apr || a.B <= 0) return launch_grad_m<AMF>(a, nx, s);
    // apr runs on slot rows with counted users: no pos_sort, item records or
    // deterministic compact slots; items counted too unless every item row
    // reads the all-reduced buffer (apr_global, the multi-rank item reduce)
    if (a.srec != nullptr || a.recV != nullptr || a.det_fx || a.offU != nullptr || !a.count_users ||
        (!a.apr_global && (a.items_grad_only || !a.count_items)) || a.GadvU == nullptr || a.GadvV == nullptr)
        return hipErrorInvalidValue;
    hipError_t err = hipSuccess;
    if (!a.apr_embed_done && (err = launch_apr_embed(a, s)) != hipSuccess) return err;
    err = a.W == 1 ? launch_apr_grad<1>(a, nx, s)
        : (a.W == 5 && epl_for(a.d) <= 8) ? launch_apr_grad<5>(a, nx, s) : launch_apr_grad<0>(a, nx, s);
    if (err != hipSuccess) return err;
    if ((err = launch_apr_zero(a, s)) != hipSuccess) return err;
    if (a.apr_global)   // rows of every rank's batch are set after the all-reduce
        return hipMemsetAsync(a.GadvV, 0, (size_t)a.n_items * a.d * sizeof(float), s);
    return hipSuccess;
}

}  // namespace cfk
