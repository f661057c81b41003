// Operand feed rate per CU: how many bytes per clock a CU can pull into LDS by LDS-DMA
// (global_load_lds, 1 KiB per wave-instruction, the GEMMs' staging) or into VGPRs by 16-byte
// loads, with every CU streaming, from an L2-resident region (every workgroup of an XCD re-reads
// the same MiBs, as the GEMM tiles of one K-step do) and from HBM (a 4 GiB region).
// 8 waves per workgroup, one workgroup per CU, each wave keeping DEPTH pieces in flight.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/feed_probe tools/feed_probe.hip && /tmp/feed_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
#define LDS_PTR(p) ((lds_ptr_t)(uintptr_t)(p))
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int DEPTH>
__global__ __launch_bounds__(512, 1) void feed_lds(const char* __restrict__ src, size_t region, int iters,
                                                   float* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) char ring[DEPTH][8][1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    size_t off = ((size_t)blockIdx.x * 8 + wave) * 1024 * 64 % region;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const char* p = src + (off + (size_t)lane * 16) % region;
            __builtin_amdgcn_global_load_lds((const void*)p, LDS_PTR(&ring[d][wave][0]), 16, 0, 0);
            off += 8 * 1024 * 37;  // a different 1 KiB piece per issue
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (lane == 0 && sink) sink[blockIdx.x * 8 + wave] = *(const float*)&ring[0][wave][0];
}

template <int DEPTH>
__global__ __launch_bounds__(512, 1) void feed_vgpr(const char* __restrict__ src, size_t region, int iters,
                                                    float* __restrict__ sink) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    size_t off = ((size_t)blockIdx.x * 8 + wave) * 1024 * 64 % region;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
        f32x4 v[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            v[d] = *(const f32x4*)(src + (off + (size_t)lane * 16) % region);
            off += 8 * 1024 * 37;
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) acc += v[d];
    }
    if (sink) sink[blockIdx.x * 512 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
    int dev = 0, cus = 0, clk = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
    const size_t big = (size_t)4 << 30;
    char* src;
    float* sink;
    CK(hipMalloc(&src, big));
    CK(hipMemset(src, 1, big));
    CK(hipMalloc(&sink, (size_t)cus * 512 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("%d CUs, nominal clock %d MHz\n", cus, clk / 1000);
    const int iters = 2000;
    for (size_t region : {(size_t)2 << 20, big}) {
        for (int kind = 0; kind < 2; ++kind) {
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0, 0));
                if (kind == 0) feed_lds<8><<<cus, 512>>>(src, region, iters, sink);
                else feed_vgpr<8><<<cus, 512>>>(src, region, iters, sink);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double bytes = (double)cus * 8 * iters * 8 * 1024;
                const double tbs = bytes / ms / 1e9;
                printf("%-9s region %6zu MiB  rep %d: %7.3f ms  %6.2f TB/s  %5.1f B/clk/CU at 2.1 GHz\n",
                       kind == 0 ? "LDS-DMA" : "to VGPR", region >> 20, rep, ms, tbs, tbs * 1e12 / cus / 2.1e9);
            }
        }
    }
    CK(hipFree(src));
    CK(hipFree(sink));
    return 0;
}
