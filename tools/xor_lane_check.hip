// Checks on the GPU that cf_eval.hip's xor_lane (DPP / permlane-swap lane
// exchange, CF_FUSED_DPP_SORT) returns lane ^ s's value for s = 1 .. 32:
//   hipcc -O3 --offload-arch=gfx950 tools/xor_lane_check.hip -o /tmp/xlc && /tmp/xlc
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int s) {
    switch (s) {
        case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
        case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
        case 4: {
            const int t = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xF, 0xA, false);
            return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x104, 0xF, 0x5, false);
        }
        case 8: {
            const int t = __builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xF, 0xC, false);
            return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x108, 0xF, 0x3, false);
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

__global__ void k(uint32_t* out) {
    const uint32_t v = 1000u + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 6; ++i) out[i * 64 + threadIdx.x] = xor_lane(v, 1 << i);
}

int main() {
    uint32_t* d = nullptr;
    uint32_t h[6 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int i = 0; i < 6; ++i)
        for (int l = 0; l < 64; ++l) {
            const uint32_t want = 1000u + (uint32_t)(l ^ (1 << i));
            if (h[i * 64 + l] != want) {
                if (bad < 10) std::printf("s=%d lane %d: got %u want %u\n", 1 << i, l, h[i * 64 + l], want);
                ++bad;
            }
        }
    std::printf("xor_lane check: %s (%d wrong)\n", bad ? "FAIL" : "OK", bad);
    (void)hipFree(d);
    return bad ? 1 : 0;
}
