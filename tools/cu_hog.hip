// Diagnostic: hold `blocks` CUs for `usec` microseconds from a side stream (tools/ab_gemm_sched.py).
// Each workgroup is one wave with 96 KiB of LDS, so no two share a CU and no 160-KiB GEMM
// workgroup fits beside one — the footprint of a foreign kernel (RCCL's channel kernels, a
// side-stream graph) that displaces a persistent kernel's workgroups.  Every wave leaves when the
// 100 MHz constant clock says its time is up.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void cu_hog_kernel(unsigned long long ticks, int* sink) {
    __shared__ char lds[96 * 1024];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = (char)threadIdx.x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
    if (threadIdx.x == 0 && lds[5] == 77) sink[blockIdx.x] = 1;  // keeps the LDS allocation (never true)
}

extern "C" int cu_hog(int blocks, double usec, void* sink, void* stream) {
    if (blocks <= 0) return 0;
    hipLaunchKernelGGL(cu_hog_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream,
                       (unsigned long long)(usec * 100.0), (int*)sink);
    return (int)hipGetLastError();
}
