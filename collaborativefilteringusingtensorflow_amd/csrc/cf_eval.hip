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
            // key 0 = excluded: the caller's item mask here, train items by mask_train_kernel
            const bool off = a.item_mask != nullptr && ((a.item_mask[ii >> 6] >> (ii & 63)) & 1ull);
            a.keys[(int64_t)uu * a.n_items + ii] = off ? 0u : float_key(s);
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

// ---------------------------------------------------------------------------
// Fused scoring GEMM + streaming top-k (no score matrix in HBM).
//
// One block = 64 users; it sweeps all items in steps of 64.  Per step the
// four waves compute a 2 x 2 arrangement of 32 x 32 score tiles with
// v_mfma_f32_32x32x2_f32 (exact f32, a k-ordered fmaf chain): lane l feeds
// A = U[row l&31][k] and B = V[k][col l&31] where lane half h = l>>5 walks
// the k-half [h*Dh, (h+1)*Dh) -- so each lane streams contiguous k and reads
// its operands four MFMAs at a time with ds_read_b128 from LDS tiles whose
// row stride (Dp+4 floats == 4*odd mod 64 banks) is conflict-free.
// The train items of each user are excluded with a 64-bit mask per user and
// step, built by advancing a cursor through the user's sorted CSR row as the
// sweep moves (items are visited in increasing order).  Every surviving
// score becomes a 64-bit key (order-preserving score bits, then ~item id: ties
// go to the lower id, as TopKV2); keys above the user's running threshold
// are appended to its LDS candidate list, which a wave bitonic-sorts down to
// k entries (and raises the threshold) whenever fewer than 64 slots remain.
// ---------------------------------------------------------------------------
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    const int lo = __shfl_xor((int)(v & 0xFFFFFFFFull), m, 64);
    const int hi = __shfl_xor((int)(v >> 32), m, 64);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
    const int lo = __shfl((int)(v & 0xFFFFFFFFull), src, 64);
    const int hi = __shfl((int)(v >> 32), src, 64);
    return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}

#ifndef CF_FUSED_DPP_SORT
// 1 (round 6): the compaction's bitonic exchanges read lane ^ s through DPP
// (s <= 8, inside a 16-lane row) and gfx950's permlane16 / permlane32 swaps
// (s = 16, 32) instead of ds_bpermute round trips through the LDS crossbar,
// and a list of <= 64 entries is sorted in one register per lane.  Phase
// stamps of the cfg5 pass (CF_FUSED_STAMPS, profiles/r06/r06s) put the
// compactions and the waits they cause the block's other waves at ~18 % of
// the wave cycles; measured cfg5 86.0 -> 89.8 TFLOP/s (same box,
// tools/score_ab.py); 0: the shuffle form
#define CF_FUSED_DPP_SORT 1
#endif

// the value lane ^ s holds (s < 64, a constant after unrolling), all lanes
// active: DPP quad_perm for s = 1, 2; row_shr / row_shl with bank masks for
// s = 4, 8 (the partner is in the same 16-lane row); permlane16_swap /
// permlane32_swap for s = 16, 32 (rows 2r, 2r+1 and the wave's halves swap
// in one instruction: one result holds the even rows' / lower half's values,
// the other the odd rows' / upper half's)
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int s) {
    switch (s) {
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]
        case 4: {
            const int t = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xF, 0xA, false);   // banks 1,3 <- lane-4
            return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x104, 0xF, 0x5, false);     // banks 0,2 <- lane+4
        }
        case 8: {
            const int t = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xF, 0xC, false);   // banks 2,3 <- lane-8
            return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x108, 0xF, 0x3, false);     // banks 0,1 <- lane+8
        }
        case 16: {
            const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            return (lane_id() & 16) ? r[0] : r[1];
        }
        default: {
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return (lane_id() & 32) ? r[0] : r[1];
        }
    }
}

__device__ __forceinline__ unsigned long long xor_lane_u64(unsigned long long v, int s) {
    return ((unsigned long long)xor_lane((uint32_t)(v >> 32), s) << 32) | xor_lane((uint32_t)v, s);
}

// one wave sorts a user's <= 64 R candidates descending (R registers per
// lane: entry e = lane + 64 r), keeps the best `keep` (<= 64 R - 64) in place
// and returns how many it kept; the k-th best becomes the row's threshold
template <int R>
__device__ int wave_compact(unsigned long long* __restrict__ buf, int* cnt,
                            unsigned long long* thr, int keep, int k) {
    const int lane = lane_id();
    const int n = *cnt;
#if CF_FUSED_DPP_SORT
    if (R >= 2 && n <= 64 && keep <= 64) {   // wave-uniform: one register per lane
        unsigned long long x = lane < n ? buf[lane] : 0ull;
#pragma unroll
        for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const unsigned long long y = xor_lane_u64(x, stride);
                const bool lower = (lane & stride) == 0;
                const bool desc = (lane & size) == 0;
                const unsigned long long mx = x > y ? x : y, mn = x > y ? y : x;
                x = (desc == lower) ? mx : mn;
            }
        }
        const int m = n < keep ? n : keep;
        if (lane < m) buf[lane] = x;
        const unsigned long long kth = shfl_u64(x, k - 1);
        if (lane == 0) {
            *cnt = m;
            if (m >= k) *thr = kth;
        }
        return m;
    }
    if constexpr (R == 2) {
        unsigned long long x0 = lane < n ? buf[lane] : 0ull;
        unsigned long long x1 = lane + 64 < n ? buf[lane + 64] : 0ull;
#pragma unroll
        for (int size = 2; size <= 128; size <<= 1) {
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                if (stride == 64) {  // partner is the lane's other register; size == 128
                    if (x0 < x1) { const unsigned long long t = x0; x0 = x1; x1 = t; }
                    continue;
                }
                const bool lower = (lane & stride) == 0;
                {
                    const unsigned long long y = xor_lane_u64(x0, stride);
                    const bool desc = (lane & size) == 0;
                    const unsigned long long mx = x0 > y ? x0 : y, mn = x0 > y ? y : x0;
                    x0 = (desc == lower) ? mx : mn;
                }
                {
                    const unsigned long long y = xor_lane_u64(x1, stride);
                    const bool desc = ((lane + 64) & size) == 0;
                    const unsigned long long mx = x1 > y ? x1 : y, mn = x1 > y ? y : x1;
                    x1 = (desc == lower) ? mx : mn;
                }
            }
        }
        const int m = n < keep ? n : keep;
        if (lane < m) buf[lane] = x0;            // keep <= 64
        const unsigned long long kth = shfl_u64(x0, k - 1);
        if (lane == 0) {
            *cnt = m;
            if (m >= k) *thr = kth;
        }
        return m;
    }
#endif
    if constexpr (R == 2) {   // the two-block-per-CU kernel's form (its register budget is tight)
        unsigned long long x0 = lane < n ? buf[lane] : 0ull;
        unsigned long long x1 = lane + 64 < n ? buf[lane + 64] : 0ull;
        for (int size = 2; size <= 128; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                if (stride == 64) {  // partner is the lane's other register; size == 128
                    if (x0 < x1) { const unsigned long long t = x0; x0 = x1; x1 = t; }
                    continue;
                }
                const bool lower = (lane & stride) == 0;
                {
                    const unsigned long long y = shfl_xor_u64(x0, stride);
                    const bool desc = (lane & size) == 0;
                    const unsigned long long mx = x0 > y ? x0 : y, mn = x0 > y ? y : x0;
                    x0 = (desc == lower) ? mx : mn;
                }
                {
                    const unsigned long long y = shfl_xor_u64(x1, stride);
                    const bool desc = ((lane + 64) & size) == 0;
                    const unsigned long long mx = x1 > y ? x1 : y, mn = x1 > y ? y : x1;
                    x1 = (desc == lower) ? mx : mn;
                }
            }
        }
        const int m = n < keep ? n : keep;
        if (lane < m) buf[lane] = x0;            // keep <= 64
        const unsigned long long kth = shfl_u64(x0, k - 1);
        if (lane == 0) {
            *cnt = m;
            if (m >= k) *thr = kth;
        }
        return m;
    }
    unsigned long long x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lane + 64 * r < n ? buf[lane + 64 * r] : 0ull;
    for (int size = 2; size <= 64 * R; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 64) {   // partners in the lane's own registers r, r | rs
                const int rs = stride >> 6;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if ((r & rs) != 0) continue;
#pragma unroll
                    for (int r2 = 0; r2 < R; ++r2) {
                        if (r2 != (r | rs)) continue;
                        const bool desc = ((lane + 64 * r) & size) == 0;
                        const unsigned long long mx = x[r] > x[r2] ? x[r] : x[r2];
                        const unsigned long long mn = x[r] > x[r2] ? x[r2] : x[r];
                        x[r] = desc ? mx : mn;
                        x[r2] = desc ? mn : mx;
                    }
                }
                continue;
            }
            const bool lower = (lane & stride) == 0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const unsigned long long y = shfl_xor_u64(x[r], stride);
                const bool desc = ((lane + 64 * r) & size) == 0;
                const unsigned long long mx = x[r] > y ? x[r] : y, mn = x[r] > y ? y : x[r];
                x[r] = (desc == lower) ? mx : mn;
            }
        }
    }
    const int m = n < keep ? n : keep;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (lane + 64 * r < m) buf[lane + 64 * r] = x[r];
    unsigned long long xk = x[0];
#pragma unroll
    for (int r = 1; r < R; ++r)
        if (r == ((k - 1) >> 6)) xk = x[r];
    const unsigned long long kth = shfl_u64(xk, (k - 1) & 63);
    if (lane == 0) {
        *cnt = m;
        if (m >= k) *thr = kth;
    }
    return m;
}

// sort registers per lane for a candidate list of CAP slots
__host__ __device__ constexpr int fused_sort_regs(int cap) { return cap <= 64 ? 1 : cap <= 128 ? 2 : 4; }

// V tile in LDS: 64 rows x 128 floats, no padding; the 16-B chunk q of row r
// sits at chunk q ^ (r & 31), so the 16 lanes of a ds_read_b128 phase (rows
// c .. c+15 at one k offset) land on 16 different chunks: conflict-free.
__device__ __forceinline__ int vs_off(int r, int kk) {
    return r * kFusedMaxD + ((((kk >> 2) ^ (r & 31)) << 2) | (kk & 3));
}

#ifndef CF_FUSED_PREFILTER
// 1: the 16 prefilter compares first, the LDS reads only where a lane of the
// wave passed -- measured even (cfg5 83.5 vs 84.8, cfg3 77.8 vs 75.9 TFLOP/s,
// r04k; it spills 16-80 B at the 256-VGPR limit), so 0: the cost of the
// candidate phase (84.7 -> 112.5 without it, CF_FUSED_EXP_NOCAND) is not the
// mask reads
#define CF_FUSED_PREFILTER 0
#endif
#ifndef CF_FUSED_FCMP
// 1 (round 4): the register prefilter compares the float score against the
// float form of its row's threshold word -- one v_cmp per score, no key
// conversion, no per-row (R < nu) mask -- and the wave takes the exact path
// only when some lane passed some score (rare once the thresholds have
// risen); 0: the key-word prefilter per score, each with its own branch
#define CF_FUSED_FCMP 1
#endif
#ifndef CF_FUSED_BPREFETCH
#define CF_FUSED_BPREFETCH 0   // 1: read each MFMA group's B operand one group ahead (measured slower: 74 vs 84.5 TF)
#endif
#ifndef CF_FUSED_STRICT
// 1 (round 6): the exact candidate test reads thr[R] only for a score equal
// to its row's threshold float; 0: every prefilter pass reads it.  Measured
// even (89.7 vs 89.8 TFLOP/s): the exact path's cost is not that read.  (Slots
// from one LDS atomic per row and half-wave, ballot ranks and readlanes,
// measured slower: cfg5 86.8 vs 89.5 TFLOP/s, profiles/r06/r06s/r06s7)
#define CF_FUSED_STRICT 1
#endif
#ifndef CF_FUSED_MASK_AHEAD
// 1 (round 6): the users' threads build the next tile's train masks during
// this tile's candidate phase (two mask buffers, +512 B of LDS), so the
// cursor walk no longer holds the other waves at the staging barrier, and
// with the prefetched tile that barrier goes (two per step instead of
// three): cfg5 89.7 -> 91.2 TFLOP/s; 0: the masks are built in the staging
// phase of their own tile
#define CF_FUSED_MASK_AHEAD 1
#endif
#ifndef CF_FUSED_CURSOR2
// 1 (round 6): the train-row cursor keeps the next TWO items in registers, so
// consuming one issues the load of the one after without waiting for it;
// 0: each consumption waits for its dependent load (wave 0 of the block, at
// nearly every step of a 64-user block).  Measured even (86.1 vs 85.9,
// 90.7 vs 91.2 TFLOP/s with the masks built ahead), so 0
#define CF_FUSED_CURSOR2 0
#endif
#ifndef CF_FUSED_SETPRIO
// 1 (round 5 experiment): a wave raises its issue priority for its MFMA
// stream (s_setprio 3) and drops it for the candidate phase, so the SIMD's
// other wave -- of the other block -- fills the gaps instead of both waves'
// MFMA streams and candidate phases lining up
#define CF_FUSED_SETPRIO 0
#endif
// CAP: candidate slots per user.  kFusedCap (92, k <= 28): ~80 KB of LDS,
// two blocks per CU.  kFusedCapWide (192, k <= 128; round 5, GBPR's topN =
// 100): ~130 KB, one block per CU.
// MASK: the caller's item mask is read (a.item_mask may still be null); the
// narrow kernel without it keeps its register budget (GBPR: 16 B less spill)
template <int MODEL, int CAP = kFusedCap, bool MASK = false, int NU = kFusedUsers>
__global__ __launch_bounds__(4 * NU, (CAP <= kFusedCap && NU == kFusedUsers) ? 2 : 1)
void fused_topk_kernel(FusedTopkArgs a) {
    // The user operands live in registers.
    constexpr int SR = fused_sort_regs(CAP);
    constexpr int NT = 4 * NU;        // threads: one wave per 32 x 32 score tile
    constexpr int NW = NT / kWave;
    __shared__ __attribute__((aligned(16))) float Vs[kFusedItems * kFusedMaxD];
    __shared__ unsigned long long buf[NU * CAP];
    __shared__ unsigned long long thr[NU];
    // the train masks: AHEAD keeps two tiles' (the next one is built by the
    // users' threads during this tile's candidate phase).  BPR only: GBPR's
    // bias tile and CML's norms leave no room for the second buffer beside
    // two blocks per CU (81,928 B > 80 KiB)
    constexpr bool AHEAD = CF_FUSED_MASK_AHEAD && MODEL == BPR;
    __shared__ unsigned long long mask_buf[AHEAD ? 2 : 1][NU];
    __shared__ int cnt[NU];
    __shared__ float unorm[NU];
    __shared__ float bt[kFusedItems];
    __shared__ int thr_ver;                  // bumped whenever a compaction raised thresholds

    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;     // 32-row user block, 32-col item block
    const int h = lane >> 5, c = lane & 31;
    const int d = a.d, Dp = a.Dp, Dh = a.Dh;
    const int u0 = blockIdx.x * NU;
    if (tid == 0) thr_ver = 0;
    // the score words of the thresholds of this lane's 16 output rows, kept in
    // registers: a score whose key word is below its row's cannot enter the
    // list, so most scores are rejected without touching LDS
#if CF_FUSED_FCMP
    float thf[16];   // key_float of the threshold word; +inf for rows past nu
#else
    uint32_t thi[16];
#endif
    int thi_ver = -1;
    const int nu = (a.n_users - u0) < NU ? (a.n_users - u0) : NU;

    // A operand of lane (c, h): U[row wr*32 + c][h*Dh, (h+1)*Dh), zero-padded
    constexpr int kAH = kFusedMaxD / 2;
    float ua[kAH];
    {
        const int r = wr * 32 + c;
        const float* urow = a.U + (int64_t)a.users[u0 + (r < nu ? r : 0)] * d;
#pragma unroll
        for (int t = 0; t < kAH; ++t) {
            const int kk = h * Dh + t;
            ua[t] = (r < nu && t < Dh && kk < d) ? urow[kk] : 0.f;
        }
        if (MODEL == CML) {
            float sq = 0.f;
#pragma unroll
            for (int t = 0; t < kAH; ++t) sq = fmaf(ua[t], ua[t], sq);
            sq += __shfl_xor(sq, 32, 64);
            if (wc == 0 && h == 0) unorm[r] = sq;   // |u|^2 of row r
        }
        // the A operands are complete before the sweep: otherwise the
        // wait-count model merges them with the in-flight tile prefetch at the
        // loop header and every step's first MFMA waits for that prefetch
        __builtin_amdgcn_s_waitcnt(0);
    }
    int64_t cur = 0, end = 0;                // train-row cursor of user `tid` (tid < 64)
    int64_t nxt = INT64_MAX;                 // the train item at the cursor, kept in a register
#if CF_FUSED_CURSOR2
    int nxt2 = INT_MAX;                      // the one after it, loaded a consumption ahead
#endif
    if (tid < NU) {
        thr[tid] = 0ull;
        cnt[tid] = 0;
        if (a.exclude_train && tid < nu) {
            const int u = a.users[u0 + tid];
            cur = a.indptr[u];
            end = a.indptr[u + 1];
            if (cur < end) nxt = a.indices[cur];
#if CF_FUSED_CURSOR2
            if (cur + 1 < end) nxt2 = a.indices[cur + 1];
#endif
        }
    }
    // the next item tile is loaded into registers during this tile's MFMA and
    // candidate phases and written to LDS after them (d % 4 == 0)
    const bool vec = (d & 3) == 0;
    const int q4 = Dp >> 2;
    constexpr int kPre = (kFusedItems * (kFusedMaxD / 4) + NT - 1) / NT;
    float4 pre[kPre];
    auto load_tile = [&](int64_t jt) {   // 16-B loads; rows are 16-B aligned when d % 4 == 0
#pragma unroll
        for (int q = 0; q < kPre; ++q) {
            const int t = tid + q * NT;
            const int r = t / q4, kk = (t - r * q4) * 4;
            const int64_t j = jt + r;
            pre[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t < kFusedItems * q4 && j < a.n_items && kk < d)
                pre[q] = *reinterpret_cast<const float4*>(a.V + j * d + kk);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int q = 0; q < kPre; ++q) {
            const int t = tid + q * NT;
            const int r = t / q4, kk = (t - r * q4) * 4;
            if (t < kFusedItems * q4) *reinterpret_cast<float4*>(Vs + vs_off(r, kk)) = pre[q];
        }
    };
    if (vec) {
        load_tile(0);
        store_tile();
    }
    // tile jt's train mask of user tid (tid < NU): the caller's item
    // exclusions (one word per 64-item tile), then the user's train items
    auto build_mask = [&](int64_t jt, int slot) {
        unsigned long long m = (MASK && a.item_mask != nullptr) ? a.item_mask[jt >> 6] : 0ull;
        while (nxt < jt + kFusedItems) {   // sorted row: no load unless an item is consumed
            m |= 1ull << (int)(nxt - jt);
            ++cur;
#if CF_FUSED_CURSOR2
            // the next item is already in a register; the load issued
            // here is waited on only at a later consumption
            nxt = nxt2 == INT_MAX ? INT64_MAX : (int64_t)nxt2;
            nxt2 = cur + 1 < end ? a.indices[cur + 1] : INT_MAX;
#else
            nxt = cur < end ? (int64_t)a.indices[cur] : INT64_MAX;
#endif
        }
        mask_buf[slot][tid] = m;
    };
    if (AHEAD && tid < NU) build_mask(0, 0);
    if (AHEAD && vec) __syncthreads();         // tile 0 and its masks, before the first MFMA
    int mslot = 0;                                            // mask_buf slot of the current tile
#ifdef CF_FUSED_STAMPS
    // diagnostic builds (cf_engine.cpp score_topk_fused): cycles per phase of
    // the sweep, per wave ([0..8], in the order of the CF_STAMP sites; the
    // candidate phase split as [11] prefilter, [12] exact path, [3] the rest); [9]
    // steps that took the exact candidate path, [10] steps with a compaction
    unsigned long long st_acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#define CF_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
                         st_acc[i] += t_ - st_last; st_last = t_; } while (0)
#define CF_STAMP_COUNT(i) (st_acc[i] += 1)
#else
#define CF_STAMP(i) do {} while (0)
#define CF_STAMP_COUNT(i) do {} while (0)
#endif

    for (int64_t j0 = 0; j0 < a.n_items; j0 += kFusedItems) {
        // ---- stage the item tile (unless prefetched), its bias, the train mask --
        if (!vec) {
            for (int t = tid; t < kFusedItems * Dp; t += NT) {
                const int r = t / Dp, kk = t - r * Dp;
                const int64_t j = j0 + r;
                Vs[vs_off(r, kk)] = (j < a.n_items && kk < d) ? a.V[j * d + kk] : 0.f;
            }
        }
        if (MODEL == GBPR && tid < kFusedItems)
            bt[tid] = (j0 + tid < a.n_items) ? a.b[j0 + tid] : 0.f;
        if (!AHEAD && tid < NU) build_mask(j0, 0);
        CF_STAMP(0);
        // AHEAD with the prefetched tile: nothing is staged here (the masks
        // and the tile were written before the previous step's last barrier),
        // so that barrier is this step's
        if (!AHEAD || !vec) __syncthreads();
        CF_STAMP(1);
#ifdef CF_FUSED_EXP_NOLOAD   // attribution: no tile streaming (stale tile)
        const bool more = false;
#else
        const bool more = vec && j0 + kFusedItems < a.n_items;
#endif
        if (more) load_tile(j0 + kFusedItems);
        // ---- 32 x 32 tile per wave on the matrix cores --------------------------
        if (CF_FUSED_SETPRIO) __builtin_amdgcn_s_setprio(3);
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        float vsq = 0.f;
        const int br = wc * 32 + c;              // B operand row (item) of this lane
#ifndef CF_FUSED_EXP_NOMFMA   // attribution builds (wrong results by design)
#if CF_FUSED_BPREFETCH
        auto bop = [&](int t0) {   // address formed at use (hoisted: 16 VGPRs)
            int r = br, hd = h * Dh;
            asm volatile("" : "+v"(r), "+v"(hd));
            return *reinterpret_cast<const float4*>(Vs + vs_off(r, hd + t0));
        };
#else
        auto bop = [&](int t0) { return *reinterpret_cast<const float4*>(Vs + vs_off(br, h * Dh + t0)); };
#endif
        auto mfma4b = [&](int t0, const float4 b4) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 0], b4.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 1], b4.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 2], b4.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 3], b4.w, acc, 0, 0, 0);
            if (MODEL == CML) vsq += b4.x * b4.x + b4.y * b4.y + b4.z * b4.z + b4.w * b4.w;
        };
        auto mfma4 = [&](int t0) {
            const float4 b4 = bop(t0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 0], b4.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 1], b4.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 2], b4.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 3], b4.w, acc, 0, 0, 0);
            if (MODEL == CML) vsq += b4.x * b4.x + b4.y * b4.y + b4.z * b4.z + b4.w * b4.w;
        };
        if (Dh == kAH) {
            // branch-free: a conditional per k-chunk made the compiler wait
            // for every outstanding global load (the prefetched next tile)
            // at each chunk (s_waitcnt vmcnt(0) before the LDS reads)
#if CF_FUSED_BPREFETCH
            // the next group's B operand is read before this group's MFMAs,
            // so no MFMA group waits on its own LDS read
            float4 bc = bop(0);
#pragma unroll
            for (int t0 = 0; t0 < kAH; t0 += 4) {
                const float4 bn4 = bop(t0 + 4 < kAH ? t0 + 4 : t0);
                mfma4b(t0, bc);
                bc = bn4;
            }
#else
#pragma unroll
            for (int t0 = 0; t0 < kAH; t0 += 4) mfma4(t0);
#endif
        } else {
#pragma unroll
            for (int t0 = 0; t0 < kAH; t0 += 4)
                if (t0 < Dh) mfma4(t0);   // block-uniform
        }
#endif
        if (CF_FUSED_SETPRIO) __builtin_amdgcn_s_setprio(0);
        CF_STAMP(2);
        float vnorm = 0.f;
        if (MODEL == CML) vnorm = vsq + __shfl_xor(vsq, 32, 64);   // |v_col|^2
        // ---- candidates above each user's threshold -------------------------------
        const int jl = wc * 32 + c;
        const int64_t J = j0 + jl;
        const unsigned long long* __restrict__ mask = mask_buf[mslot];
#ifndef CF_FUSED_EXP_NOCAND
#if CF_FUSED_FCMP
        if (thi_ver != thr_ver) {   // block-uniform (thr_ver changes only between barriers)
            thi_ver = thr_ver;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;   // < NU
                const float t = key_float((uint32_t)(thr[R] >> 32));
                thf[q] = R < nu ? t : INFINITY;
            }
        }
        // key(s) > thr[R] implies s >= key_float(thr word) in float order; a
        // NaN score or threshold passes (!(s < t)), so this only prefilters
        const float bj_ = (MODEL == GBPR) ? bt[jl] : 0.f;
        bool anyp = false;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            float s = acc[q];
            if (MODEL == GBPR) s += bj_;
            if (MODEL == CML) {
                const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                s = 2.f * s - vnorm - unorm[R];   // -|u - v|^2
            }
            anyp |= !(s < thf[q]);
        }
        CF_STAMP(11);
        if (__ballot(anyp) != 0ull) {   // wave-uniform
            CF_STAMP_COUNT(9);
#if CF_FUSED_STRICT
            // a score strictly above its row's threshold float has a key above
            // the threshold key (float_key is order-preserving; thf is the
            // float of thr[R]'s high word, refreshed with it): only an equal
            // score (or +-0, NaN) needs thr[R] itself -- one LDS round trip
            // per active q fewer (mask read, then the slot atomic)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                float s = acc[q];
                if (MODEL == GBPR) s += bj_;
                if (MODEL == CML) s = 2.f * s - vnorm - unorm[R];
                if (!(s < thf[q]) && R < nu && J < a.n_items && !((mask[R] >> jl) & 1ull)) {
                    const unsigned long long key = ((unsigned long long)float_key(s) << 32) |
                                                   (0xFFFFFFFFull - (unsigned long long)J);
                    if (s > thf[q] || key > thr[R]) {
                        const int pos = atomicAdd(&cnt[R], 1);
                        buf[R * CAP + pos] = key;
                    }
                }
            }
#else
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                float s = acc[q];
                if (MODEL == GBPR) s += bj_;
                if (MODEL == CML) s = 2.f * s - vnorm - unorm[R];
                if (!(s < thf[q]) && R < nu && J < a.n_items && !((mask[R] >> jl) & 1ull)) {
                    const unsigned long long key = ((unsigned long long)float_key(s) << 32) |
                                                   (0xFFFFFFFFull - (unsigned long long)J);
                    if (key > thr[R]) {
                        const int pos = atomicAdd(&cnt[R], 1);
                        buf[R * CAP + pos] = key;
                    }
                }
            }
#endif
        }
        CF_STAMP(12);
#else
        if (thi_ver != thr_ver) {   // block-uniform (thr_ver changes only between barriers)
            thi_ver = thr_ver;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                thi[q] = R < nu ? (uint32_t)(thr[R] >> 32) : 0xFFFFFFFFu;
            }
        }
#endif
#if CF_FUSED_FCMP
        // (above)
#elif CF_FUSED_PREFILTER
        // round 4: the register prefilter for all 16 scores first -- no LDS
        // read -- and the train mask, the exact threshold and the insertion
        // only where some lane of the wave passed (rare once the thresholds
        // have risen).  Attribution: the candidate phase cost the pass 84.7 ->
        // 112.5 TFLOP/s (CF_FUSED_EXP_NOCAND), its 16 mask reads per lane
        // per tile were issued whatever the prefilter said.
        const float bj_ = (MODEL == GBPR) ? bt[jl] : 0.f;
        uint32_t pass = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
            float s = acc[q];
            if (MODEL == GBPR) s += bj_;
            if (MODEL == CML) s = 2.f * s - vnorm - unorm[R];   // -|u - v|^2
            // key > thr[R] implies fk >= thi[q]: a pure prefilter
            pass |= (float_key(s) >= thi[q]) ? (1u << q) : 0u;
        }
        if (__ballot(pass != 0u) != 0ull) {   // wave-uniform
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                if (!((pass >> q) & 1u)) continue;
                const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                float s = acc[q];
                if (MODEL == GBPR) s += bj_;
                if (MODEL == CML) s = 2.f * s - vnorm - unorm[R];
                const uint32_t fk = float_key(s);
                if (R < nu && J < a.n_items && !((mask[R] >> jl) & 1ull)) {
                    const unsigned long long key = ((unsigned long long)fk << 32) |
                                                   (0xFFFFFFFFull - (unsigned long long)J);
                    if (key > thr[R]) {
                        const int pos = atomicAdd(&cnt[R], 1);
                        buf[R * CAP + pos] = key;
                    }
                }
            }
        }
#else
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
            float s = acc[q];
            if (MODEL == GBPR) s += bt[jl];
            if (MODEL == CML) s = 2.f * s - vnorm - unorm[R];   // -|u - v|^2
            const uint32_t fk = float_key(s);
            // key > thr[R] implies fk >= thi[q]: a pure prefilter
            if (fk >= thi[q] && R < nu && J < a.n_items && !((mask[R] >> jl) & 1ull)) {
                const unsigned long long key = ((unsigned long long)fk << 32) |
                                               (0xFFFFFFFFull - (unsigned long long)J);
                if (key > thr[R]) {
                    const int pos = atomicAdd(&cnt[R], 1);
                    buf[R * CAP + pos] = key;
                }
            }
        }
#endif
#else
        if (acc[0] == 12345.f && J == 7) cnt[0] = 1;   // keep the MFMA result live
#endif
        if (AHEAD && tid < NU && j0 + kFusedItems < a.n_items)
            build_mask(j0 + kFusedItems, mslot ^ 1);   // read after this tile's barriers
        if (AHEAD) mslot ^= 1;
        CF_STAMP(3);
        __syncthreads();
        CF_STAMP(4);
#ifdef CF_FUSED_STAMPS
        if (more) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the tile's loads
        CF_STAMP(5);
#endif
        if (more) store_tile();   // every wave is past its MFMA reads of this tile
#ifdef CF_FUSED_STAMPS
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the tile's LDS stores
        CF_STAMP(6);
#endif
        // ---- shrink lists that could overflow at the next step ---------------------
        // the wave's 16 rows (wv, wv + 4, ..) are checked with one LDS read and
        // a ballot, not 16 dependent reads
        {
            constexpr int kRowsPerWave = NU / NW;
            const int Rl = wv + NW * lane;
            unsigned long long need = __ballot(lane < kRowsPerWave && Rl < nu &&
                                               cnt[lane < kRowsPerWave ? Rl : 0] > CAP - kFusedItems);
            if (need != 0ull) {
                CF_STAMP_COUNT(10);
                if (lane == 0) atomicAdd(&thr_ver, 1);
                while (need != 0ull) {
                    const int l = __ffsll((long long)need) - 1;
                    need &= need - 1ull;
                    const int R = wv + NW * l;
                    wave_compact<SR>(buf + R * CAP, &cnt[R], &thr[R], a.k, a.k);
                }
            }
        }
        CF_STAMP(7);
        __syncthreads();
        CF_STAMP(8);
    }
#ifdef CF_FUSED_STAMPS
    if (a.stamps != nullptr && lane == 0 && NW <= 8) {
#pragma unroll
        for (int q = 0; q < 14; ++q) a.stamps[((size_t)blockIdx.x * 8 + wv) * 16 + q] = st_acc[q];
    }
#endif
    // ---- final sort and output -------------------------------------------------------
    for (int R = wv; R < nu; R += NW) {
        const int n = wave_compact<SR>(buf + R * CAP, &cnt[R], &thr[R], a.k, a.k);
        const int64_t orow = (int64_t)(u0 + R) * a.k;
        for (int o = lane; o < a.k; o += (CAP <= kFusedCap ? a.k : kWave)) {   // k <= 28: one pass
            int id = -1;
            float v = __int_as_float(0x7fc00000);
            if (o < n) {
                const unsigned long long e = buf[R * CAP + o];
                id = (int)(0xFFFFFFFFull - (e & 0xFFFFFFFFull));
                v = key_float((uint32_t)(e >> 32));
            }
            a.idx_out[orow + o] = id;
            if (a.val_out) a.val_out[orow + o] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// The same pass software-pipelined across item tiles (fused_variant 1;
// measured SLOWER than the sequential kernel, 63 vs 85.6 TFLOP/s at cfg5 on
// one box, profiles/r03/score_pass/ -- kept for A/B, not the default):
// while a wave's MFMAs build tile t's scores in one accumulator set, the
// candidate test of tile t-1 runs on the other set, one row (q) per group of
// four MFMAs -- the VALU work issues in the shadow of the matrix core instead
// of after it.  Tile t's train-mask bits, bias and (CML) |v|^2 are taken
// into registers while tile t is current, so the LDS image is unchanged
// (two blocks per CU).  Insertions (rare once the thresholds have risen) run
// after the MFMA loop; every list still receives at most one tile's 64 keys
// between compaction checks.  Same keys, same lists, same output as
// fused_topk_kernel.
// ---------------------------------------------------------------------------
template <int MODEL>
__global__ __launch_bounds__(kBlock, 2) void fused_topk_pipe_kernel(FusedTopkArgs a) {
    __shared__ __attribute__((aligned(16))) float Vs[kFusedItems * kFusedMaxD];
    __shared__ unsigned long long buf[kFusedUsers * kFusedCap];
    __shared__ unsigned long long thr[kFusedUsers];
    __shared__ unsigned long long mask[kFusedUsers];
    __shared__ int cnt[kFusedUsers];
    __shared__ float unorm[kFusedUsers];
    __shared__ float bt[kFusedItems];
    __shared__ int thr_ver;

    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int h = lane >> 5, c = lane & 31;
    const int d = a.d, Dp = a.Dp, Dh = a.Dh;
    const int u0 = blockIdx.x * kFusedUsers;
    if (tid == 0) thr_ver = 0;
    const int nu = (a.n_users - u0) < kFusedUsers ? (a.n_users - u0) : kFusedUsers;

    constexpr int kAH = kFusedMaxD / 2;
    float ua[kAH];
    {
        const int r = wr * 32 + c;
        const float* urow = a.U + (int64_t)a.users[u0 + (r < nu ? r : 0)] * d;
#pragma unroll
        for (int t = 0; t < kAH; ++t) {
            const int kk = h * Dh + t;
            ua[t] = (r < nu && t < Dh && kk < d) ? urow[kk] : 0.f;
        }
        if (MODEL == CML) {
            float sq = 0.f;
#pragma unroll
            for (int t = 0; t < kAH; ++t) sq = fmaf(ua[t], ua[t], sq);
            sq += __shfl_xor(sq, 32, 64);
            if (wc == 0 && h == 0) unorm[r] = sq;
        }
        __builtin_amdgcn_s_waitcnt(0);
    }
    int64_t cur = 0, end = 0;
    int64_t nxt = INT64_MAX;
    if (tid < kFusedUsers) {
        thr[tid] = 0ull;
        cnt[tid] = 0;
        if (a.exclude_train && tid < nu) {
            const int u = a.users[u0 + tid];
            cur = a.indptr[u];
            end = a.indptr[u + 1];
            if (cur < end) nxt = a.indices[cur];
        }
    }
    const bool vec = (d & 3) == 0;
    const int q4 = Dp >> 2;
    constexpr int kPre = (kFusedItems * (kFusedMaxD / 4) + kBlock - 1) / kBlock;
    float4 pre[kPre];
    // (tile-loop-invariant addresses are formed where they are used, behind
    // an opaque copy of tid: hoisted, they would hold ~30 VGPRs all sweep)
    auto load_tile = [&](int64_t jt) {
        int tid_ = tid;
        asm volatile("" : "+v"(tid_));
#pragma unroll
        for (int q = 0; q < kPre; ++q) {
            const int t = tid_ + q * kBlock;
            const int r = t / q4, kk = (t - r * q4) * 4;
            const int64_t j = jt + r;
            pre[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t < kFusedItems * q4 && j < a.n_items && kk < d)
                pre[q] = *reinterpret_cast<const float4*>(a.V + j * d + kk);
        }
    };
    auto store_tile = [&]() {
        int tid_ = tid;
        asm volatile("" : "+v"(tid_));
#pragma unroll
        for (int q = 0; q < kPre; ++q) {
            const int t = tid_ + q * kBlock;
            const int r = t / q4, kk = (t - r * q4) * 4;
            if (t < kFusedItems * q4) *reinterpret_cast<float4*>(Vs + vs_off(r, kk)) = pre[q];
        }
    };
    if (vec) {
        load_tile(0);
        store_tile();
    }
    const int jl = wc * 32 + c;              // this lane's item column in a tile
    // row q of this lane's 16 accumulator rows
    auto row_of = [&](int q) { return wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h; };
    // the previous tile's scores, train-mask bits, bias, |v|^2 and column
    floatx16 accp;
#pragma unroll
    for (int q = 0; q < 16; ++q) accp[q] = 0.f;
    uint32_t mbp = 0;
    float bp = 0.f, vnp = 0.f;
    int64_t Jp = -1;                         // -1: no previous tile
    auto score = [&](int q, float accv) {
        float s = accv;
        if (MODEL == GBPR) s += bp;
        if (MODEL == CML) {   // |u|^2 re-read each time (hoisted: 16 VGPRs)
            int R = row_of(q);
            asm volatile("" : "+v"(R));
            s = 2.f * s - vnp - unorm[R];
        }
        return float_key(s);
    };
    // a score whose key word is below its row's threshold word cannot enter
    // the list: the test reads that word from LDS (the row's 64-bit threshold,
    // high half), no registers held across tiles
    const uint32_t* thr_hi = reinterpret_cast<const uint32_t*>(thr) + 1;
    // branch-free (every operand read unconditionally, R < 64 always), so the
    // scheduler can spread the tests between the MFMAs
    const bool jp_ok_init = false;
    bool jp_ok = jp_ok_init;   // Jp is a column of a real previous tile
    auto pass_of = [&](int q) -> uint32_t {
        const int R = row_of(q);
        const uint32_t fk = score(q, accp[q]);
        const uint32_t ok = (uint32_t)(R < nu) & (uint32_t)(fk >= thr_hi[2 * R]) & (uint32_t)jp_ok &
                            ~(mbp >> q) & 1u;
        return ok << q;
    };
    auto insert = [&](uint32_t pass) {
        while (pass != 0u) {
            const int q = __ffs(pass) - 1;
            pass &= pass - 1u;
            const int R = row_of(q);
            const unsigned long long key = ((unsigned long long)score(q, accp[q]) << 32) |
                                           (0xFFFFFFFFull - (unsigned long long)Jp);
            if (key > thr[R]) {
                const int pos = atomicAdd(&cnt[R], 1);
                buf[R * kFusedCap + pos] = key;
            }
        }
    };
    auto compact_check = [&]() {
        constexpr int kRowsPerWave = kFusedUsers / kWavesPerBlock;
        const int Rl = wv + kWavesPerBlock * lane;
        unsigned long long need = __ballot(lane < kRowsPerWave && Rl < nu &&
                                           cnt[lane < kRowsPerWave ? Rl : 0] > kFusedCap - kFusedItems);
        if (need != 0ull) {
            while (need != 0ull) {
                const int l = __ffsll((long long)need) - 1;
                need &= need - 1ull;
                const int R = wv + kWavesPerBlock * l;
                wave_compact<fused_sort_regs(kFusedCap)>(buf + R * kFusedCap, &cnt[R], &thr[R], a.k, a.k);
            }
        }
    };

    for (int64_t j0 = 0; j0 < a.n_items; j0 += kFusedItems) {
        if (!vec) {
            for (int t = tid; t < kFusedItems * Dp; t += kBlock) {
                const int r = t / Dp, kk = t - r * Dp;
                const int64_t j = j0 + r;
                Vs[vs_off(r, kk)] = (j < a.n_items && kk < d) ? a.V[j * d + kk] : 0.f;
            }
        }
        if (MODEL == GBPR && tid < kFusedItems)
            bt[tid] = (j0 + tid < a.n_items) ? a.b[j0 + tid] : 0.f;
        if (tid < kFusedUsers) {
            unsigned long long m = a.item_mask != nullptr ? a.item_mask[j0 >> 6] : 0ull;
            while (nxt < j0 + kFusedItems) {
                m |= 1ull << (int)(nxt - j0);
                ++cur;
                nxt = cur < end ? (int64_t)a.indices[cur] : INT64_MAX;
            }
            mask[tid] = m;
        }
        __syncthreads();
        const bool more = vec && j0 + kFusedItems < a.n_items;
        if (more) load_tile(j0 + kFusedItems);
        // this tile's mask bits and bias, kept for its candidate test next step
        uint32_t mbn = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) mbn |= (uint32_t)((mask[row_of(q)] >> jl) & 1ull) << q;
        const float bn = (MODEL == GBPR) ? bt[jl] : 0.f;
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        float vsq = 0.f;
        const int br = wc * 32 + c;
        uint32_t pass = 0;
        // the swizzled B-operand address is formed where it is used: hoisted,
        // its 16 values would hold 16 VGPRs through the whole sweep
        auto bop = [&](int t0) {
            int r = br, hd = h * Dh;
            asm volatile("" : "+v"(r), "+v"(hd));
            return *reinterpret_cast<const float4*>(Vs + vs_off(r, hd + t0));
        };
        auto mfma4 = [&](int t0, const float4 b4) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 0], b4.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 1], b4.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 2], b4.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 3], b4.w, acc, 0, 0, 0);
            if (MODEL == CML) vsq += b4.x * b4.x + b4.y * b4.y + b4.z * b4.z + b4.w * b4.w;
        };
        if (Dh == kAH) {
            // one previous-tile row test per group of four MFMAs (16 and 16)
#if CF_FUSED_BPREFETCH
            float4 bc = bop(0);   // the next group's B operand read ahead
#pragma unroll
            for (int t0 = 0; t0 < kAH; t0 += 4) {
                const float4 bn4 = bop(t0 + 4 < kAH ? t0 + 4 : t0);
                mfma4(t0, bc);
                pass |= pass_of(t0 >> 2);
                bc = bn4;
            }
#else
#pragma unroll
            for (int t0 = 0; t0 < kAH; t0 += 4) {
                mfma4(t0, bop(t0));
                pass |= pass_of(t0 >> 2);
            }
#endif
        } else {
#pragma unroll
            for (int t0 = 0; t0 < kAH; t0 += 4)
                if (t0 < Dh) mfma4(t0, bop(t0));   // block-uniform
#pragma unroll
            for (int q = 0; q < 16; ++q) pass |= pass_of(q);
        }
        insert(pass);
        float vnorm = 0.f;
        if (MODEL == CML) vnorm = vsq + __shfl_xor(vsq, 32, 64);
        __syncthreads();
        if (more) store_tile();
        compact_check();
        __syncthreads();
        accp = acc;
        mbp = mbn;
        bp = bn;
        vnp = vnorm;
        Jp = j0 + jl;
        jp_ok = Jp < a.n_items;
    }
    // the last tile's candidates
    {
        uint32_t pass = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) pass |= pass_of(q);
        insert(pass);
    }
    __syncthreads();
    for (int R = wv; R < nu; R += kWavesPerBlock) {
        const int n = wave_compact<fused_sort_regs(kFusedCap)>(buf + R * kFusedCap, &cnt[R], &thr[R], a.k, a.k);
        const int64_t orow = (int64_t)(u0 + R) * a.k;
        if (lane < a.k) {
            int id = -1;
            float v = __int_as_float(0x7fc00000);
            if (lane < n) {
                const unsigned long long e = buf[R * kFusedCap + lane];
                id = (int)(0xFFFFFFFFull - (e & 0xFFFFFFFFull));
                v = key_float((uint32_t)(e >> 32));
            }
            a.idx_out[orow + lane] = id;
            if (a.val_out) a.val_out[orow + lane] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// The same pass with specialised waves (fused_variant 2; round 5, verdict item
// 5).  In fused_topk_kernel every wave computes its MFMA tile, then tests its
// own scores; counter passes showed the matrix cores busy 54 % of the time,
// the waves of a SIMD lining their MFMA streams and candidate phases up.
// Here a block of 512 threads (64 users) splits the work:
//  * waves 0-3 ("MFMA waves") only compute: tile t's 2 x 2 arrangement of
//    32 x 32 score tiles from the V tile in LDS, the model transform (GBPR
//    bias, CML distance), and the scores into an LDS score tile Sc[t & 1];
//    they run at raised issue priority;
//  * waves 4-7 ("candidate waves"), in the same step: stage V tile t+1 (its
//    bias and its train-mask words) into the other LDS buffers, issue the
//    loads of tile t+2, and test tile t-1's scores against their rows'
//    thresholds -- lane (w, l) owns row 16 (w - 4) + (l & 15) and 16 of its
//    64 columns -- appending keys to the row's list and compacting the lists
//    of the rows this wave owns.
// One barrier per step.  Per SIMD one wave of each kind, so the candidate
// phase runs beside the MFMA stream instead of after it.  ~150 KB of LDS:
// one block per CU.  Same keys, same lists, same output as fused_topk_kernel
// (k <= 28).
// ---------------------------------------------------------------------------
constexpr int kWsThreads = 512;
constexpr int kWsSP = kFusedItems + 4;   // score-tile row stride (floats): 16-B rows, staggered banks

template <int MODEL>
__global__ __launch_bounds__(kWsThreads, 1) void fused_topk_ws_kernel(FusedTopkArgs a) {
    constexpr int CAP = kFusedCap;
    __shared__ __attribute__((aligned(16))) float Vs[2][kFusedItems * kFusedMaxD];
    __shared__ __attribute__((aligned(16))) float Sc[2][kFusedUsers * kWsSP];
    __shared__ unsigned long long buf[kFusedUsers * CAP];
    __shared__ unsigned long long thr[kFusedUsers];
    __shared__ unsigned long long maskb[3][kFusedUsers];
    __shared__ int cnt[kFusedUsers];
    __shared__ float unorm[kFusedUsers];
    __shared__ float bt[2][kFusedItems];

    const int tid = threadIdx.x;
    const int lane = lane_id();
    const int wv = tid >> 6;
    const bool mw = wv < 4;                  // MFMA wave
    const int d = a.d, Dp = a.Dp, Dh = a.Dh;
    const int u0 = blockIdx.x * kFusedUsers;
    const int nu = (a.n_users - u0) < kFusedUsers ? (a.n_users - u0) : kFusedUsers;
    const int64_t ntile = (a.n_items + kFusedItems - 1) / kFusedItems;
    constexpr int kAH = kFusedMaxD / 2;

    // ---- MFMA waves: their A operands (U rows) in registers -----------------
    const int wr = (wv & 3) >> 1, wc = wv & 1;
    const int h = lane >> 5, c = lane & 31;
    float ua[kAH];
    if (mw) {
        const int r = wr * 32 + c;
        const float* urow = a.U + (int64_t)a.users[u0 + (r < nu ? r : 0)] * d;
#pragma unroll
        for (int t = 0; t < kAH; ++t) {
            const int kk = h * Dh + t;
            ua[t] = (r < nu && t < Dh && kk < d) ? urow[kk] : 0.f;
        }
        if (MODEL == CML) {
            float sq = 0.f;
#pragma unroll
            for (int t = 0; t < kAH; ++t) sq = fmaf(ua[t], ua[t], sq);
            sq += __shfl_xor(sq, 32, 64);
            if (wc == 0 && h == 0) unorm[r] = sq;
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_s_setprio(2);
    }

    // ---- candidate waves: tile staging, train cursors, candidate rows -------
    const int ct = tid - 4 * kWave;          // 0..255 on candidate waves
    int64_t cur = 0, end = 0, nxt = INT64_MAX;   // train cursor of user ct (ct < 64)
    if (!mw && ct < kFusedUsers) {
        thr[ct] = 0ull;
        cnt[ct] = 0;
        if (a.exclude_train && ct < nu) {
            const int u = a.users[u0 + ct];
            cur = a.indptr[u];
            end = a.indptr[u + 1];
            if (cur < end) nxt = a.indices[cur];
        }
    }
    const bool vec = (d & 3) == 0;
    const int q4 = Dp >> 2;
    constexpr int kPre = (kFusedItems * (kFusedMaxD / 4) + 255) / 256;
    float4 pre[kPre];
    auto load_tile = [&](int64_t jt) {
#pragma unroll
        for (int q = 0; q < kPre; ++q) {
            const int t = ct + q * 256;
            const int r = t / q4, kk = (t - r * q4) * 4;
            const int64_t j = jt + r;
            pre[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t < kFusedItems * q4 && j < a.n_items && kk < d)
                pre[q] = *reinterpret_cast<const float4*>(a.V + j * d + kk);
        }
    };
    // stage tile ti (items j0 .. j0 + 63) into buffer ti & 1: V rows (from
    // the prefetch registers when vec), bias, and the train / caller mask
    // words into maskb[ti % 3]
    auto stage_tile = [&](int64_t ti) {
        const int64_t j0 = ti * kFusedItems;
        float* V_ = Vs[ti & 1];
        if (vec) {
#pragma unroll
            for (int q = 0; q < kPre; ++q) {
                const int t = ct + q * 256;
                const int r = t / q4, kk = (t - r * q4) * 4;
                if (t < kFusedItems * q4) *reinterpret_cast<float4*>(V_ + vs_off(r, kk)) = pre[q];
            }
        } else {
            for (int t = ct; t < kFusedItems * Dp; t += 256) {
                const int r = t / Dp, kk = t - r * Dp;
                const int64_t j = j0 + r;
                V_[vs_off(r, kk)] = (j < a.n_items && kk < d) ? a.V[j * d + kk] : 0.f;
            }
        }
        if (ct < kFusedItems) {
            if (MODEL == GBPR) bt[ti & 1][ct] = (j0 + ct < a.n_items) ? a.b[j0 + ct] : 0.f;
            unsigned long long m = a.item_mask != nullptr ? a.item_mask[j0 >> 6] : 0ull;
            while (nxt < j0 + kFusedItems) {
                m |= 1ull << (int)(nxt - j0);
                ++cur;
                nxt = cur < end ? (int64_t)a.indices[cur] : INT64_MAX;
            }
            maskb[ti % 3][ct] = m;
        }
    };
    const int Rc = ((wv - 4) & 3) * 16 + (lane & 15);   // candidate row of this lane
    const int ch = lane >> 4;                           // its 16-column chunk
    if (!mw) {
        if (vec) load_tile(0);
        stage_tile(0);
        if (vec && ntile > 1) load_tile(kFusedItems);
    }
    __syncthreads();

    for (int64_t t = 0; t <= ntile; ++t) {
        if (mw) {
            if (t < ntile) {
                const float* V_ = Vs[t & 1];
                // one MFMA wave per SIMD: two independent accumulator chains
                // (alternate groups of four k-steps), so a dependent MFMA
                // never waits on the previous one's result; summed at the end
                floatx16 acc, acc2;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    acc[q] = 0.f;
                    acc2[q] = 0.f;
                }
                float vsq = 0.f;
                const int br = wc * 32 + c;
                auto mfma4 = [&](floatx16& A, int t0) {
                    const float4 b4 = *reinterpret_cast<const float4*>(V_ + vs_off(br, h * Dh + t0));
                    A = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 0], b4.x, A, 0, 0, 0);
                    A = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 1], b4.y, A, 0, 0, 0);
                    A = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 2], b4.z, A, 0, 0, 0);
                    A = __builtin_amdgcn_mfma_f32_32x32x2f32(ua[t0 + 3], b4.w, A, 0, 0, 0);
                    if (MODEL == CML) vsq += b4.x * b4.x + b4.y * b4.y + b4.z * b4.z + b4.w * b4.w;
                };
                if (Dh == kAH) {
#pragma unroll
                    for (int t0 = 0; t0 < kAH; t0 += 8) {
                        mfma4(acc, t0);
                        mfma4(acc2, t0 + 4);
                    }
                } else {
#pragma unroll
                    for (int t0 = 0; t0 < kAH; t0 += 8) {
                        if (t0 < Dh) mfma4(acc, t0);          // block-uniform
                        if (t0 + 4 < Dh) mfma4(acc2, t0 + 4);
                    }
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[q] += acc2[q];
                const int jl = wc * 32 + c;
                float vnorm = 0.f;
                if (MODEL == CML) vnorm = vsq + __shfl_xor(vsq, 32, 64);   // |v_col|^2
                const float bj = (MODEL == GBPR) ? bt[t & 1][jl] : 0.f;
                float* S_ = Sc[t & 1];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int R = wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                    float sv = acc[q];
                    if (MODEL == GBPR) sv += bj;
                    if (MODEL == CML) sv = 2.f * sv - vnorm - unorm[R];   // -|u - v|^2
                    S_[R * kWsSP + jl] = sv;
                }
            }
        } else {
#ifndef CF_WS_EXP_NOSTAGE   // attribution only (stale tiles, wrong results)
            if (t + 1 < ntile) stage_tile(t + 1);
            if (vec && t + 2 < ntile) load_tile((t + 2) * kFusedItems);
#endif
#ifdef CF_WS_EXP_NOCAND   // attribution only (no candidates)
            if (false) {
#else
            if (t >= 1 && Rc < nu) {
#endif
                // tile t-1's scores of this lane's row, columns ch*16 .. +16
                const int64_t jb = (t - 1) * kFusedItems + ch * 16;
                const float* S_ = Sc[(t - 1) & 1] + Rc * kWsSP + ch * 16;
                float sv[16];
#pragma unroll
                for (int e = 0; e < 16; e += 4) {
                    const float4 v4 = *reinterpret_cast<const float4*>(S_ + e);
                    sv[e] = v4.x; sv[e + 1] = v4.y; sv[e + 2] = v4.z; sv[e + 3] = v4.w;
                }
                const uint32_t mb = (uint32_t)(maskb[(t - 1) % 3][Rc] >> (ch * 16)) & 0xFFFFu;
                const unsigned long long th = thr[Rc];
                const float thf = key_float((uint32_t)(th >> 32));
                // key > th implies s >= key_float(th word); NaN passes the prefilter
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int64_t J = jb + e;
                    if (!(sv[e] < thf) && J < a.n_items && !((mb >> e) & 1u)) {
                        const unsigned long long key = ((unsigned long long)float_key(sv[e]) << 32) |
                                                       (0xFFFFFFFFull - (unsigned long long)J);
                        if (key > th) {
                            const int pos = atomicAdd(&cnt[Rc], 1);
                            buf[Rc * CAP + pos] = key;
                        }
                    }
                }
            }
            // this wave's 16 rows: shrink the lists that could overflow at
            // the next step (only this wave touches them)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            const int Rl = ((wv - 4) & 3) * 16 + (lane & 15);
            unsigned long long need = __ballot(lane < 16 && Rl < nu && cnt[Rl] > CAP - kFusedItems);
            while (need != 0ull) {
                const int l = __ffsll((long long)need) - 1;
                need &= need - 1ull;
                const int R = ((wv - 4) & 3) * 16 + l;
                wave_compact<fused_sort_regs(CAP)>(buf + R * CAP, &cnt[R], &thr[R], a.k, a.k);
            }
        }
        __syncthreads();
    }
    // ---- final sort and output (all eight waves) --------------------------------
    for (int R = wv; R < nu; R += kWsThreads / kWave) {
        const int n = wave_compact<fused_sort_regs(CAP)>(buf + R * CAP, &cnt[R], &thr[R], a.k, a.k);
        const int64_t orow = (int64_t)(u0 + R) * a.k;
        if (lane < a.k) {
            int id = -1;
            float v = __int_as_float(0x7fc00000);
            if (lane < n) {
                const unsigned long long e = buf[R * CAP + lane];
                id = (int)(0xFFFFFFFFull - (e & 0xFFFFFFFFull));
                v = key_float((uint32_t)(e >> 32));
            }
            a.idx_out[orow + lane] = id;
            if (a.val_out) a.val_out[orow + lane] = v;
        }
    }
}

hipError_t launch_fused_topk(const FusedTopkArgs& a, hipStream_t s) {
    if (a.n_users <= 0) return hipSuccess;
    const dim3 grid((a.n_users + kFusedUsers - 1) / kFusedUsers), block(kBlock);
    // CML's distance transform does not fit the pipelined kernel's registers
    // at two blocks per CU (its A operands spill): it keeps the sequential one
    if (a.k > kFusedMaxWideK) return hipErrorInvalidValue;   // the host checks first
    if (a.variant == 2 && a.k <= kFusedMaxK) {   // specialised waves
        const dim3 wgrid(grid.x), wblock(kWsThreads);
        switch (a.model) {
            case GBPR: hipLaunchKernelGGL(fused_topk_ws_kernel<GBPR>, wgrid, wblock, 0, s, a); break;
            case CML: hipLaunchKernelGGL(fused_topk_ws_kernel<CML>, wgrid, wblock, 0, s, a); break;
            default: hipLaunchKernelGGL(fused_topk_ws_kernel<BPR>, wgrid, wblock, 0, s, a); break;
        }
        return hipGetLastError();
    }
    if (a.variant == 1 && a.model != CML && a.k <= kFusedMaxK && a.item_mask == nullptr) {
        if (a.model == GBPR)
            hipLaunchKernelGGL(fused_topk_pipe_kernel<GBPR>, grid, block, 0, s, a);
        else
            hipLaunchKernelGGL(fused_topk_pipe_kernel<BPR>, grid, block, 0, s, a);
        return hipGetLastError();
    }
    if (a.variant == 3 && a.k <= kFusedMaxK) {   // 128 users per block, one block per CU
        const dim3 g2((a.n_users + 2 * kFusedUsers - 1) / (2 * kFusedUsers)), b2(8 * kFusedUsers);
        const bool m = a.item_mask != nullptr;
        switch (a.model) {
            case GBPR:
                if (m) hipLaunchKernelGGL((fused_topk_kernel<GBPR, kFusedCap, true, 2 * kFusedUsers>), g2, b2, 0, s, a);
                else hipLaunchKernelGGL((fused_topk_kernel<GBPR, kFusedCap, false, 2 * kFusedUsers>), g2, b2, 0, s, a);
                break;
            case CML:
                if (m) hipLaunchKernelGGL((fused_topk_kernel<CML, kFusedCap, true, 2 * kFusedUsers>), g2, b2, 0, s, a);
                else hipLaunchKernelGGL((fused_topk_kernel<CML, kFusedCap, false, 2 * kFusedUsers>), g2, b2, 0, s, a);
                break;
            default:
                if (m) hipLaunchKernelGGL((fused_topk_kernel<BPR, kFusedCap, true, 2 * kFusedUsers>), g2, b2, 0, s, a);
                else hipLaunchKernelGGL((fused_topk_kernel<BPR, kFusedCap, false, 2 * kFusedUsers>), g2, b2, 0, s, a);
                break;
        }
        return hipGetLastError();
    }
    if (a.k > kFusedMaxK) {   // 28 < k <= 128: the wide lists, one block per CU
        switch (a.model) {
            case GBPR: hipLaunchKernelGGL((fused_topk_kernel<GBPR, kFusedCapWide, true>), grid, block, 0, s, a); break;
            case CML: hipLaunchKernelGGL((fused_topk_kernel<CML, kFusedCapWide, true>), grid, block, 0, s, a); break;
            default: hipLaunchKernelGGL((fused_topk_kernel<BPR, kFusedCapWide, true>), grid, block, 0, s, a); break;
        }
        return hipGetLastError();
    }
    if (a.item_mask != nullptr) {
        switch (a.model) {
            case GBPR: hipLaunchKernelGGL((fused_topk_kernel<GBPR, kFusedCap, true>), grid, block, 0, s, a); break;
            case CML: hipLaunchKernelGGL((fused_topk_kernel<CML, kFusedCap, true>), grid, block, 0, s, a); break;
            default: hipLaunchKernelGGL((fused_topk_kernel<BPR, kFusedCap, true>), grid, block, 0, s, a); break;
        }
        return hipGetLastError();
    }
    switch (a.model) {
        case GBPR: hipLaunchKernelGGL(fused_topk_kernel<GBPR>, grid, block, 0, s, a); break;
        case CML: hipLaunchKernelGGL(fused_topk_kernel<CML>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(fused_topk_kernel<BPR>, grid, block, 0, s, a); break;
    }
    return hipGetLastError();
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
