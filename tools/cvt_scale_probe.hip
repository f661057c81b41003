// Probe: semantics of v_cvt_scalef32_pk_fp8_f32 (does the f32 scale multiply or divide?) and of
// v_cvt_pk_fp8_f32 on the same inputs.  Prints the bytes for a few values and scales.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s2 __attribute__((ext_vector_type(2)));
__global__ void probe(const float* x, const float* sc, int* out) {
    const int i = threadIdx.x;
    s2 o = {0, 0};
    s2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, x[2 * i], x[2 * i + 1], sc[i], false);
    out[2 * i] = __builtin_bit_cast(int, r);
    out[2 * i + 1] = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}
int main() {
    const int n = 6;
    float hx[2 * n] = {1.f, 2.f, 1.f, 2.f, 1.f, 2.f, 0.5f, 3.f, 100.f, 200.f, 1.f, -1.f};
    float hs[n] = {1.f, 2.f, 0.5f, 4.f, 0.25f, 1024.f};
    float *dx, *ds;
    int* dout;
    hipMalloc(&dx, sizeof(hx)); hipMalloc(&ds, sizeof(hs)); hipMalloc(&dout, 2 * n * sizeof(int));
    hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
    hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice);
    probe<<<1, n>>>(dx, ds, dout);
    int h[2 * n];
    hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i)
        printf("x=(%g,%g) scale=%g  scalef32 bytes=%02x %02x   plain bytes=%02x %02x\n", hx[2 * i], hx[2 * i + 1], hs[i],
               h[2 * i] & 0xff, (h[2 * i] >> 8) & 0xff, h[2 * i + 1] & 0xff, (h[2 * i + 1] >> 8) & 0xff);
    return 0;
}
