// Probe of the E8M0 scale operands of v_mfma_scale_f32_32x32x64_f8f6f4 (one wave): which lane's
// scale (and which byte, op_sel) applies to which (row, K block) of A and (column, K block) of B.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_scale_probe.hip -o tools/mfma_scale_probe
// Case a: A = 1.0 in the 32 bytes of lanes `half` only, B = 1.0 everywhere, scale_b = 1, lane l's
// scale_a byte `sel` = 2^(l - 32) (other bytes 2^20): D[i][j] = sum over the nonzero A elements
// of their block's scale, printed as log2(D / 32) + 32 per output row i (and checked constant
// over j).  Case b: the same with the roles of A and B swapped (per output column j).
// Case c (which = 2): A = 1.0 only in bytes 8g .. 8g+7 of BOTH halves (16 elements of a row):
// log2(D / 16) + 32 names the lane whose scale the byte group's block takes.
// Measured (r03k): in cases a / b every row takes 16 elements at lane i's scale and 16 at lane
// i + 32's: a lane's 32 bytes are NOT one scale block.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int SEL>
__global__ void probe(float* out, int which, int half) {
    const int lane = threadIdx.x;
    const int one4 = 0x38383838;  // four e4m3 1.0
    i32x8 ones, part;
    for (int i = 0; i < 8; ++i) {
        ones[i] = one4;
        part[i] = which == 2 ? ((i >> 1) == half ? one4 : 0) : ((lane >> 5) == half ? one4 : 0);
    }
    int sc = 0;
    for (int b = 0; b < 4; ++b) sc |= (b == SEL ? (127 + lane - 32) : (127 + 20)) << (8 * b);
    f32x16 acc = {};
    if (which != 1)
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(part, ones, acc, 0, 0, SEL, sc, 0, 127);
    else
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones, part, acc, 0, 0, 0, 127, SEL, sc);
    // D layout: lane = column j (lane & 31), register r -> row (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), col = lane & 31;
        out[row * 32 + col] = acc[r];
    }
}

int main() {
    float* d;
    float h[1024];
    hipMalloc(&d, 4096);
    int bad = 0;
    for (int which = 0; which < 3; ++which)
        for (int sel = 0; sel < (which == 2 ? 1 : 4); ++sel)
            for (int half = 0; half < (which == 2 ? 4 : 2); ++half) {
                switch (sel) {
                    case 0: probe<0><<<1, 64>>>(d, which, half); break;
                    case 1: probe<1><<<1, 64>>>(d, which, half); break;
                    case 2: probe<2><<<1, 64>>>(d, which, half); break;
                    default: probe<3><<<1, 64>>>(d, which, half); break;
                }
                hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost);
                if (which == 2)
                    printf("A bytes %d-%d of both halves: applied scale lane (per row 0..31):", 8 * half, 8 * half + 7);
                else
                    printf("%s op_sel %d, bytes of lanes %s: log2(D/32)+32 (per %s 0..31):", which ? "B" : "A", sel,
                           half ? "32-63" : "0-31", which ? "column" : "row");
                for (int i = 0; i < 32; ++i) {
                    const float v = which == 1 ? h[0 * 32 + i] : h[i * 32 + 0];
                    const int e = (int)lrintf(log2f(v / (which == 2 ? 16.f : 32.f)));
                    printf(" %d", e + 32);
                    for (int j = 0; j < 32; ++j) {
                        const float w = which == 1 ? h[j * 32 + i] : h[i * 32 + j];
                        if (w != v) bad++;
                    }
                }
                printf("\n");
            }
    printf("non-constant entries: %d\n", bad);
    return 0;
}
