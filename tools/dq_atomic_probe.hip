// What it would cost a ONE-pass attention backward to accumulate dQ across key blocks in HBM:
// the dK/dV pass's grid (B*H heads x 33 workgroups of 256 keys, 4 waves) walks the 8193
// queries in 32-row tiles, and per tile each workgroup adds a 32 x 64 fp32 dQ partial into the
// head's dQ buffer.  No attention arithmetic runs: this prices the accumulation alone.
//   mode 0: every wave adds its own partial (no-return global f32 atomics, 4x the traffic)
//   mode 1: the 4 waves' partials summed in LDS first, one atomic set per workgroup
//   mode 2: mode 1's partial written with plain stores into a per-key-block slab (a later
//           reduce would read them back; not timed)
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/dq_atomic_probe tools/dq_atomic_probe.hip && /tmp/dq_atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / 8, r = nblk % 8;
    const int xcd = bid % 8, loc = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

template <int MODE>
__global__ __launch_bounds__(256) void dq_accum(float* __restrict__ dq, float* __restrict__ slab, int N, int nkb,
                                                int ntiles) {
    __shared__ float red[4][32 * 64];
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kblk = tile % nkb, bh = tile / nkb;
    float* D = dq + (size_t)bh * N * 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = 1e-3f * (float)(kblk + 1) * (float)(i + 1 + wave);
    for (int t = 0; t < ntiles; ++t) {
        const int q0 = 1 + t * 32;
        if constexpr (MODE == 0) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
                if (q0 + i < N)
                    __hip_atomic_fetch_add(D + (size_t)(q0 + i) * 64 + lane, v[i], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        } else {
#pragma unroll
            for (int i = 0; i < 32; ++i) red[wave][i * 64 + lane] = v[i];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int r = wave * 8 + j;
                const float s = red[0][r * 64 + lane] + red[1][r * 64 + lane] + red[2][r * 64 + lane] +
                                red[3][r * 64 + lane];
                if (q0 + r < N) {
                    if constexpr (MODE == 1)
                        __hip_atomic_fetch_add(D + (size_t)(q0 + r) * 64 + lane, s, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    else
                        slab[(((size_t)bh * nkb + kblk) * N + q0 + r) * 64 + lane] = s;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] += 1e-6f;
    }
}

int main() {
    const int B = 8, H = 12, N = 8193, nkb = (N - 1 + 255) / 256, ntiles = (N - 1 + 31) / 32;
    const int grid = B * H * nkb;
    const size_t dq_floats = (size_t)B * H * N * 64;
    const size_t slab_floats = (size_t)B * H * nkb * N * 64;
    float *dq, *slab;
    CK(hipMalloc(&dq, dq_floats * 4));
    CK(hipMalloc(&slab, slab_floats * 4));
    CK(hipMemset(dq, 0, dq_floats * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes1 = (double)grid * ntiles * 32 * 64 * 4;  // one partial per workgroup per tile
    printf("grid %d workgroups, %d query tiles each; per layer: %.2f GB of fp32 partials (mode 1/2), %.2f GB (mode 0)\n",
           grid, ntiles, bytes1 / 1e9, 4 * bytes1 / 1e9);
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 3; ++mode) {
            CK(hipEventRecord(e0, 0));
            if (mode == 0) dq_accum<0><<<grid, 256>>>(dq, slab, N, nkb, ntiles);
            else if (mode == 1) dq_accum<1><<<grid, 256>>>(dq, slab, N, nkb, ntiles);
            else dq_accum<2><<<grid, 256>>>(dq, slab, N, nkb, ntiles);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double b = mode == 0 ? 4 * bytes1 : bytes1;
            printf("rep %d mode %d: %8.3f ms per layer  (%.2f TB/s of partials)\n", rep, mode, ms, b / ms / 1e9);
        }
    }
    std::vector<float> h(64);
    CK(hipMemcpy(h.data(), dq + 64, 64 * 4, hipMemcpyDeviceToHost));
    printf("dq[1][0..3] = %g %g %g %g\n", h[0], h[1], h[2], h[3]);
    CK(hipFree(dq));
    CK(hipFree(slab));
    return 0;
}
