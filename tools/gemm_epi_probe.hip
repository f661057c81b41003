// Where the persistent NT GEMM's time goes (profiles/r03/r03q_*, r03r_*).  Modes:
//   gemm_epi_probe [reps]        dclip_gemm (the shipped host path and kernels, compiled in) at
//                                M = 65536, N = 3072, K = 768 / 1536 / 3072 (12 / 24 / 48 K-steps per
//                                256 x 256 tile, 12 tiles per CU), bias epilogue, bf16 and fp32 output,
//                                for both epilogues (DCLIP_OPT_GEMM_EPI), outputs compared bitwise; a fit
//                                of time against K-steps per tile separates the per-K-step time from
//                                the per-tile cost
//   gemm_epi_probe reps epi      the epilogue alone (no K-loop) on 256 / 128 / 64 / 32 workgroups and
//                                four store patterns: the per-CU store rate by access shape
//   gemm_epi_probe reps model    one ViT-B/16 block's eight NT GEMMs at the bench shape, both epilogues
// Built with -DDCLIP_GEMM_DIAG_NOSTORE the epilogue returns at once (wrong results): the K-loop alone.
#include "../denseclip_vit_multimodal_amd/csrc/capi.hip"
#include "../denseclip_vit_multimodal_amd/csrc/gemm.hip"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__global__ void fill_bf16(bf16* p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        h ^= h >> 15;
        p[i] = (bf16)(((int)(h & 0xffff) - 32768) * (1.0f / 32768.0f));
    }
}

__global__ void count_diff(const unsigned* a, const unsigned* b, int64_t n, unsigned* bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) atomicAdd(bad, 1u);
}


// the persistent kernel's tile loop without the K-loop: every wave stores made-up accumulators
// through pers_epilogue for its tiles (G workgroups, tiles u = r, r + G, ...); l2 = 1 maps every
// tile to row block 0 (the stores stay in a 256 x N region that the XCD L2s hold)
template <typename OutT>
__global__ __launch_bounds__(512, 1) void epi_only_kernel(void* C, int64_t ldc, const float* bias, int tiles_m,
                                                          int tiles_n, int l2) {
    typedef BigCfg<256, 256, 2, 4, 2, 64> Cfg;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / 4, wn = wave % 4;
    const int l16 = lane & 15, lq = lane >> 4;
    const int ntiles = tiles_m * tiles_n;
    const int G = gridDim.x;
    for (int u = blockIdx.x; u < ntiles; u += G) {
        const int m0 = l2 == 1 ? 0 : (u / tiles_n) * 256, n0 = (u % tiles_n) * 256;
        if (l2 >= 2) {  // the same bytes as whole 1-KiB contiguous pieces per store instruction
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const int per_wave = 128 * 64 * (int)sizeof(OutT);
            char* base = (char*)C + ((int64_t)u * 8 + wave) * per_wave;
            const u32x4 v = {(unsigned)lane, (unsigned)u, (unsigned)wave, 7u};
            if (l2 == 2) {
#pragma unroll 4
                for (int o = 0; o < per_wave; o += 1024) *(u32x4*)(base + o + lane * 16) = v;
            } else if (l2 == 4) {  // 16 rows x 64 B per instruction (pers_epilogue's pattern), no VALU
                char* rb = (char*)C + ((int64_t)m0 + wm * 128) * ldc * sizeof(OutT) + (int64_t)(n0 + wn * 64) * sizeof(OutT);
                const int rowb = 64 * (int)sizeof(OutT);
#pragma unroll 4
                for (int o = 0; o < 128 * rowb; o += 1024) {
                    const int r = (o / rowb) / 16 * 16 + (o / 64) % 16 / (rowb / 64) * 0 + (lane & 15);
                    const int cb = (o % rowb) / 64 * 64;  // 64-B column piece of the row
                    *(u32x4*)(rb + (int64_t)((o / (16 * 64)) * 16 % 128 + (lane & 15)) * ldc * sizeof(OutT) + ((o / 1024) % (rowb / 64)) * 64 + (lane >> 4) * 16) = v;
                    (void)r;
                    (void)cb;
                }
            } else {  // 3: two 512-B rows per instruction with the tile's row pitch (ldc)
                char* rb = (char*)C + ((int64_t)m0 + wm * 128) * ldc * sizeof(OutT) + (int64_t)(n0 + wn * 64) * sizeof(OutT);
                const int rowb = 64 * (int)sizeof(OutT), lanes_per_row = rowb / 16;
#pragma unroll 4
                for (int r = 0; r < 128; r += 64 / lanes_per_row)
                    *(u32x4*)(rb + (int64_t)(r + lane / lanes_per_row) * ldc * sizeof(OutT) + (lane % lanes_per_row) * 16) = v;
            }
            continue;
        }
        f32x4 acc[Cfg::NB][Cfg::MB];
#pragma unroll
        for (int i = 0; i < Cfg::NB; ++i)
#pragma unroll
            for (int j = 0; j < Cfg::MB; ++j) acc[i][j] = f32x4{(float)lane, (float)i, (float)j, (float)u};
        PersCols<DCLIP_EPI_STORE, Cfg::NB> pc;
        pers_cols<DCLIP_EPI_STORE, Cfg::NB>(pc, bias, nullptr, n0 + wn * Cfg::WTN, lq);
        pers_epilogue<bf16, DCLIP_EPI_STORE, OutT, Cfg>(acc, pc, m0 + wm * 128, n0 + wn * Cfg::WTN, l16, lq, 1.0f,
                                                        nullptr, 0, C, ldc, nullptr, 0);
    }
}

int main(int argc, char** argv) {
    const int64_t M = 65536, N = 3072, KMAX = 3072;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    bf16 *A, *B;
    void* C;
    float* bias;
    CK(hipMalloc(&A, M * KMAX * 2));
    CK(hipMalloc(&B, N * KMAX * 2));
    CK(hipMalloc(&C, M * N * 4));
    CK(hipMalloc(&bias, N * 4));
    CK(hipMemset(bias, 0, N * 4));
    fill_bf16<<<4096, 256>>>(A, M * KMAX, 1);
    fill_bf16<<<4096, 256>>>(B, N * KMAX, 2);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (argc > 2 && strcmp(argv[2], "model") == 0) {
        // one ViT-B/16 block's eight NT GEMMs at the bench shape (M = 8 x 8193), per configuration
        const int64_t Mm = 65544;
        bf16 *X, *Z;
        float *R, *Y32, *sc;
        void *Y16, *Y16b;
        CK(hipMalloc(&X, Mm * 3072 * 2));
        CK(hipMalloc(&Z, Mm * 3072 * 2));
        CK(hipMalloc(&R, Mm * 768 * 4));
        CK(hipMalloc(&Y32, Mm * 768 * 4));
        CK(hipMalloc(&Y16, Mm * 3072 * 2));
        CK(hipMalloc(&Y16b, Mm * 3072 * 2));
        CK(hipMalloc(&sc, 3072 * 4));
        fill_bf16<<<4096, 256>>>(X, Mm * 3072, 3);
        fill_bf16<<<4096, 256>>>(Z, Mm * 3072, 4);
        CK(hipMemset(R, 0, Mm * 768 * 4));
        CK(hipMemset(sc, 0, 3072 * 4));
        CK(hipDeviceSynchronize());
        struct G8 { const char* name; int epi, n, k, cdt; };
        const G8 g8[8] = {{"qkv      STORE_SCALED", DCLIP_EPI_STORE_SCALED, 2304, 768, DCLIP_BF16},
                          {"out_proj RESIDUAL    ", DCLIP_EPI_RESIDUAL, 768, 768, DCLIP_F32},
                          {"c_fc     GELU        ", DCLIP_EPI_GELU, 3072, 768, DCLIP_BF16},
                          {"c_proj   RESIDUAL+lp ", DCLIP_EPI_RESIDUAL, 768, 3072, DCLIP_F32},
                          {"dz       GELU_BWD    ", DCLIP_EPI_GELU_BWD, 3072, 768, DCLIP_BF16},
                          {"dxh2     STORE f32   ", DCLIP_EPI_STORE, 768, 3072, DCLIP_F32},
                          {"do       STORE bf16  ", DCLIP_EPI_STORE, 768, 768, DCLIP_BF16},
                          {"dxh1     STORE f32   ", DCLIP_EPI_STORE, 768, 2304, DCLIP_F32}};
        const int cfgm[4] = {1, 0, 1, 0};  // DCLIP_OPT_GEMM_EPI, alternated
        for (int c = 0; c < 4; ++c) {
            dclip_set_option(DCLIP_OPT_GEMM_EPI, cfgm[c]);
            double tot = 0;
            for (int g = 0; g < 8; ++g) {
                const G8& q = g8[g];
                auto run = [&]() {
                    const bool res = q.epi == DCLIP_EPI_RESIDUAL, lp = res && q.k == 3072;
                    const void* aux = q.epi == DCLIP_EPI_STORE_SCALED ? (const void*)sc
                                    : res ? (const void*)R : q.epi == DCLIP_EPI_GELU_BWD ? (const void*)Z : nullptr;
                    const int adt = q.epi == DCLIP_EPI_GELU_BWD ? DCLIP_BF16 : DCLIP_F32;
                    void* Cp = q.cdt == DCLIP_F32 ? (void*)Y32 : Y16;
                    void* C2p = q.epi == DCLIP_EPI_GELU ? Y16b : lp ? Y16 : nullptr;
                    return dclip_gemm(q.epi, DCLIP_BF16, X, q.k, X, q.k, Mm, q.n, q.k, 1, 1.0f, nullptr,
                                      q.epi == DCLIP_EPI_GELU_BWD ? nullptr : sc, aux, adt, q.n, Cp, q.cdt, q.n, C2p,
                                      q.n, nullptr);
                };
                if (run() != 0) {
                    fprintf(stderr, "dclip_gemm %s: %s\n", q.name, dclip_last_error());
                    return 1;
                }
                std::vector<float> ms;
                for (int r = 0; r < 5; ++r) {
                    CK(hipEventRecord(e0, nullptr));
                    for (int i = 0; i < reps; ++i) run();
                    CK(hipEventRecord(e1, nullptr));
                    CK(hipEventSynchronize(e1));
                    float x;
                    CK(hipEventElapsedTime(&x, e0, e1));
                    ms.push_back(x / reps);
                }
                std::sort(ms.begin(), ms.end());
                tot += ms[2];
                printf("epi %d  %s N=%5d K=%5d  %8.4f ms  %7.1f TF/s\n", cfgm[c], q.name, q.n, q.k, ms[2], 2.0 * Mm * q.n * q.k / (ms[2] * 1e9));
            }
            printf("epi %d  block total %.4f ms\n", cfgm[c], tot);
            fflush(stdout);
        }
        return 0;
    }
    if (argc > 2 && strcmp(argv[2], "epi") == 0) {
        const int tiles_m = 256, tiles_n = 12;  // the K = 768 problem's 3072 tiles
        for (int l2 = 0; l2 < 5; ++l2)
            for (int out = 0; out < 2; ++out)
                for (int G : {256, 128, 64, 32}) {
                    auto run = [&]() {
                        if (out == 0)
                            epi_only_kernel<bf16><<<G, 512>>>(C, N, bias, tiles_m, tiles_n, l2);
                        else
                            epi_only_kernel<float><<<G, 512>>>(C, N, bias, tiles_m, tiles_n, l2);
                    };
                    run();
                    CK(hipDeviceSynchronize());
                    std::vector<float> ms;
                    for (int r = 0; r < 5; ++r) {
                        CK(hipEventRecord(e0, nullptr));
                        for (int i = 0; i < reps; ++i) run();
                        CK(hipEventRecord(e1, nullptr));
                        CK(hipEventSynchronize(e1));
                        float x;
                        CK(hipEventElapsedTime(&x, e0, e1));
                        ms.push_back(x / reps);
                    }
                    std::sort(ms.begin(), ms.end());
                    const double per_tile_us = ms[2] * 1e3 / ((tiles_m * tiles_n + G - 1) / G);
                    const double bytes = (double)tiles_m * tiles_n * 65536 * (out == 0 ? 2 : 4);
                    printf("epilogue only, %s, out %s, %3d workgroups: %8.4f ms, %6.2f us per tile, %6.2f TB/s, %6.1f GB/s per CU\n",
                           l2 == 0 ? "all rows        " : l2 == 1 ? "L2-resident rows" : l2 == 2 ? "contiguous 1 KiB" : l2 == 3 ? "row-major pieces" : "16 x 64 B, no VALU", out == 0 ? "bf16" : "f32 ", G, ms[2], per_tile_us,
                           bytes / (ms[2] * 1e9), bytes / (ms[2] * 1e6) / G);
                    fflush(stdout);
                }
        return 0;
    }
    const int ks[3] = {768, 1536, 3072};
    // DCLIP_OPT_GEMM_EPI settings; the first (the accumulator-layout stores) is the reference output
    const int cfg[][3] = {{0, 0, 1}, {0, 0, 0}};  // {-, -, DCLIP_OPT_GEMM_EPI}; the first is the reference output
    const int ncfg = (int)(sizeof(cfg) / sizeof(cfg[0]));
    void* Cref;
    unsigned* bad;
    CK(hipMalloc(&Cref, M * N * 4));
    CK(hipMalloc(&bad, 4));
    for (int out = 0; out < 2; ++out)
    for (int c = 0; c < ncfg; ++c) {
        dclip_set_option(DCLIP_OPT_GEMM_EPI, cfg[c][2]);
        const int cdt = out == 0 ? DCLIP_BF16 : DCLIP_F32;
        const char* on = out == 0 ? "bf16" : "f32 ";
        double t[3];
        for (int ki = 0; ki < 3; ++ki) {
            const int64_t K = ks[ki];
            auto run = [&]() {
                return dclip_gemm(DCLIP_EPI_STORE, DCLIP_BF16, A, K, B, K, M, N, K, 1, 1.0f, nullptr, bias, nullptr,
                                  DCLIP_F32, 0, C, cdt, N, nullptr, 0, nullptr);
            };
            if (run() != 0) {
                fprintf(stderr, "dclip_gemm: %s\n", dclip_last_error());
                return 1;
            }
            if (ki == 0) {  // bitwise against the default configuration's output
                CK(hipDeviceSynchronize());
                if (c == 0) CK(hipMemcpy(Cref, C, M * N * (out == 0 ? 2 : 4), hipMemcpyDeviceToDevice));
                CK(hipMemset(bad, 0, 4));
                count_diff<<<4096, 256>>>((const unsigned*)C, (const unsigned*)Cref, M * N * (out == 0 ? 2 : 4) / 4, bad);
                unsigned nb;
                CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
                printf("epi %d out %s: %u words differ from epi 1\n", cfg[c][2], on, nb);
            }
            std::vector<float> ms;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0, nullptr));
                for (int i = 0; i < reps; ++i) run();
                CK(hipEventRecord(e1, nullptr));
                CK(hipEventSynchronize(e1));
                float x;
                CK(hipEventElapsedTime(&x, e0, e1));
                ms.push_back(x / reps);
            }
            std::sort(ms.begin(), ms.end());
            t[ki] = ms[2];
            printf("epi %d out %s K=%5lld  %8.4f ms  %7.1f TF/s\n", cfg[c][2], on, (long long)K,
                   t[ki], 2.0 * M * N * K / (t[ki] * 1e9));
        }
        // t = rounds * (ksteps * s + E), rounds = 12 tiles per CU
        const double s = (t[2] - t[0]) / 12.0 / (48 - 12);
        const double E = t[0] / 12.0 - 12 * s;
        printf("epi %d out %s  per K-step %.2f us, per-tile cost beyond the K-steps %.2f us (= %.1f K-steps)\n",
               cfg[c][2], on, s * 1e3, E * 1e3, E / s);
        fflush(stdout);
    }
    return 0;
}
