// MFMA GEMM for every linear layer of the ViT path and their gradients.
//
//   C[m][n] = sum_k A[m][k] * B[n][k]       (A: activations, B: nn.Linear weight [out][in])
//
// Replaces the addmm calls of nn.MultiheadAttention in/out projections and the MLP
// (reference seg/denseclip/models.py:275-281, 289), conv1-as-GEMM (models.py:407,546),
// vis_proj/global_proj (denseclip.py:605-616) and, with transposed operands, their
// weight/input gradients.
//
// Tile 128(m) x 128(n) x 64(k), 256 threads = 4 waves (2 x 2), each wave 64 x 64 =
// 2 x 2 v_mfma_f32_32x32x16 accumulators.  The MFMA is issued "swapped"
// (A-operand = B rows, B-operand = A rows) so the accumulator holds C^T: the lane
// owns one output row m and registers run along n, giving 4-wide contiguous stores and
// per-lane fused epilogues.  Operands are staged global->LDS with 16-byte
// global_load_lds (no VGPR round trip) into a double-buffered LDS image whose 16-byte
// chunks are XOR-swizzled by ((row>>1)&7) — applied to the per-lane SOURCE address
// since LDS-DMA writes lane-linearly — which makes the ds_read_b128 fragment reads
// bank-conflict free.  Block ids are remapped XCD-aware so the tiles of one A row
// panel run on one XCD and share its L2.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = 128 * BK * 2;      // 16 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;   // A + B

template <typename T>
__device__ __forceinline__ void stage_tile(const T* __restrict__ X, int64_t ldx, int row0, int rows,
                                           int k0, char* lds_tile, int wave, int lane) {
    // 16 wave-instructions of 1 KiB cover the 128 x 128 B tile; wave w issues 4 of them.
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int inst = wave * 4 + i;
        const int r = inst * 8 + (lane >> 3);
        const int p = lane & 7;
        const int c = p ^ ((r >> 1) & 7);
        int gr = row0 + r;
        gr = gr < rows ? gr : rows - 1;
        const T* src = X + (int64_t)gr * ldx + k0 + c * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + inst * 1024), 16, 0, 0);
    }
}

template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag read_frag(const char* lds_tile, int r, int chunk) {
    const int p = chunk ^ ((r >> 1) & 7);
    return *(const typename Mfma<T>::frag*)(lds_tile + r * 128 + p * 16);
}

template <typename T, int EPI, typename OutT>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    int M, int N, int k_chunk, int tiles_m, int tiles_n,
    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux,
    void* __restrict__ C, int64_t ldc, void* __restrict__ C2, int64_t ldc2, int64_t slab) {
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;

    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int m0 = (t / tiles_n) * BM;
    const int n0 = (t % tiles_n) * BN;
    const int kbeg = blockIdx.y * k_chunk;
    const int nk = k_chunk / BK;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    stage_tile<T>(A, lda, m0, M, kbeg, smem, wave, lane);
    stage_tile<T>(B, ldb, n0, N, kbeg, smem + TILE_BYTES, wave, lane);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const char* At = smem + cur * STAGE_BYTES;
        const char* Bt = At + TILE_BYTES;
        if (kt + 1 < nk) {
            char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
            stage_tile<T>(A, lda, m0, M, kbeg + (kt + 1) * BK, nxt, wave, lane);
            stage_tile<T>(B, ldb, n0, N, kbeg + (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            typename Mfma<T>::frag fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = read_frag<T>(Bt, wn * 64 + i * 32 + l32, 2 * s + h);
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = read_frag<T>(At, wm * 64 + j * 32 + l32, 2 * s + h);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = Mfma<T>::mma(fa[i], fb[j], acc[i][j]);
        }
        __syncthreads();
    }

    // ---------------------------------------------------------------- epilogue
    // acc[i][j][4q+e] = C[m][n],  m = m0 + 64wm + 32j + l32,  n = n0 + 64wn + 32i + 8q + 4h + e
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = m0 + wm * 64 + j * 32 + l32;
        if (m >= M) continue;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int nb = n0 + wn * 64 + i * 32 + q * 8 + h * 4;
                if (nb >= N) continue;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
                const bool full = nb + 3 < N;
                if (bias != nullptr && EPI != DCLIP_EPI_SPLITK && EPI != DCLIP_EPI_GELU_BWD) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += (nb + e < N) ? bias[nb + e] : 0.f;
                }
                if constexpr (EPI == DCLIP_EPI_STORE) {
                    OutT* c = (OutT*)C + (int64_t)m * ldc + nb;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (full || nb + e < N) c[e] = (OutT)v[e];
                } else if constexpr (EPI == DCLIP_EPI_GELU) {
                    OutT* z = (OutT*)C + (int64_t)m * ldc + nb;
                    OutT* g = (OutT*)C2 + (int64_t)m * ldc2 + nb;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (full || nb + e < N) {
                            // the activation is applied to the rounded pre-activation, so
                            // that forward and backward see the same z
                            const OutT zr = (OutT)v[e];
                            z[e] = zr;
                            g[e] = (OutT)quick_gelu((float)zr);
                        }
                } else if constexpr (EPI == DCLIP_EPI_RESIDUAL) {
                    const float* r = (const float*)aux + (int64_t)m * ld_aux + nb;
                    float* c = (float*)C + (int64_t)m * ldc + nb;
                    if (full) {
                        f32x4 rv = *(const f32x4*)r;
                        f32x4 o;
#pragma unroll
                        for (int e = 0; e < 4; ++e) o[e] = rv[e] + v[e];
                        *(f32x4*)c = o;
                    } else {
                        for (int e = 0; e < 4; ++e)
                            if (nb + e < N) c[e] = r[e] + v[e];
                    }
                } else if constexpr (EPI == DCLIP_EPI_GELU_BWD) {
                    const T* z = (const T*)aux + (int64_t)m * ld_aux + nb;
                    OutT* c = (OutT*)C + (int64_t)m * ldc + nb;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (full || nb + e < N) c[e] = (OutT)(v[e] * quick_gelu_grad((float)z[e]));
                } else {  // SPLITK: plain f32 partial slab per K split
                    float* c = (float*)C + blockIdx.y * slab + (int64_t)m * ldc + nb;
                    if (full) {
                        f32x4 o;
#pragma unroll
                        for (int e = 0; e < 4; ++e) o[e] = v[e];
                        *(f32x4*)c = o;
                    } else {
                        for (int e = 0; e < 4; ++e)
                            if (nb + e < N) c[e] = v[e];
                    }
                }
            }
        }
    }
}

// out[m][n] = sum_z ws[z][m][n] (+ bias[n]) — the split-K combine (deterministic order)
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int64_t slab,
                                     int M, int N, const float* __restrict__ bias,
                                     float* __restrict__ out, int64_t ldo) {
    const int64_t total4 = (int64_t)M * (N / 4);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / (N / 4));
        const int n = (int)(i % (N / 4)) * 4;
        f32x4 s = *(const f32x4*)(ws + (int64_t)m * N + n);
        for (int z = 1; z < splits; ++z) {
            f32x4 v = *(const f32x4*)(ws + z * slab + (int64_t)m * N + n);
            s += v;
        }
        if (bias) {
            s[0] += bias[n]; s[1] += bias[n + 1]; s[2] += bias[n + 2]; s[3] += bias[n + 3];
        }
        *(f32x4*)(out + (int64_t)m * ldo + n) = s;
    }
}

template <typename T, int EPI, typename OutT>
int launch(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
           int splits, const float* bias, const void* aux, int64_t ld_aux, void* C, int64_t ldc,
           void* C2, int64_t ldc2, hipStream_t st) {
    const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
    const int k_chunk = (int)(K / splits);
    dim3 grid(tiles_m * tiles_n, splits);
    gemm_nt_kernel<T, EPI, OutT><<<grid, 256, 0, st>>>(
        (const T*)A, lda, (const T*)B, ldb, (int)M, (int)N, k_chunk, tiles_m, tiles_n, bias, aux,
        ld_aux, C, ldc, C2, ldc2, (int64_t)M * N);
    return 0;
}

template <typename T>
int dispatch(int epi, int c_dt, const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M,
             int64_t N, int64_t K, int splits, const float* bias, const void* aux, int64_t ld_aux,
             void* C, int64_t ldc, void* C2, int64_t ldc2, hipStream_t st) {
    switch (epi) {
        case DCLIP_EPI_STORE:
            if (c_dt == DCLIP_F32)
                return launch<T, DCLIP_EPI_STORE, float>(A, lda, B, ldb, M, N, K, 1, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
            return launch<T, DCLIP_EPI_STORE, T>(A, lda, B, ldb, M, N, K, 1, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_GELU:
            return launch<T, DCLIP_EPI_GELU, T>(A, lda, B, ldb, M, N, K, 1, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_RESIDUAL:
            return launch<T, DCLIP_EPI_RESIDUAL, float>(A, lda, B, ldb, M, N, K, 1, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_GELU_BWD:
            return launch<T, DCLIP_EPI_GELU_BWD, T>(A, lda, B, ldb, M, N, K, 1, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_SPLITK: {
            // partial slabs in the caller's workspace (aux), then one combine pass
            float* ws = (float*)const_cast<void*>(aux);
            launch<T, DCLIP_EPI_SPLITK, float>(A, lda, B, ldb, M, N, K, splits, nullptr, nullptr, 0,
                                               ws, N, nullptr, 0, st);
            const int64_t total4 = M * (N / 4);
            int blocks = (int)((total4 + 255) / 256);
            blocks = blocks > 4096 ? 4096 : blocks;
            splitk_reduce_kernel<<<blocks, 256, 0, st>>>(ws, splits, M * N, (int)M, (int)N, bias,
                                                         (float*)C, ldc);
            return 0;
        }
    }
    return DCLIP_ERR_ARG;
}

}  // namespace

extern "C" int dclip_gemm(int epilogue, int ab_dt, const void* A, int64_t lda, const void* B,
                          int64_t ldb, int64_t M, int64_t N, int64_t K, int splits,
                          const float* bias, const void* aux, int aux_dt, int64_t ld_aux, void* C,
                          int c_dt, int64_t ldc, void* C2, int64_t ldc2, void* stream) {
    DCLIP_HOST_CHECK(ab_dt == DCLIP_BF16 || ab_dt == DCLIP_F16, "dclip_gemm: operands must be f16/bf16");
    DCLIP_HOST_CHECK(M > 0 && N > 0 && K > 0, "dclip_gemm: empty problem M=%lld N=%lld K=%lld",
                     (long long)M, (long long)N, (long long)K);
    DCLIP_HOST_CHECK(M < (1ll << 31) && N < (1ll << 31), "dclip_gemm: M/N too large");
    DCLIP_HOST_CHECK(splits >= 1, "dclip_gemm: splits must be >= 1");
    DCLIP_HOST_CHECK(K % (BK * splits) == 0, "dclip_gemm: K=%lld must be a multiple of 64*splits", (long long)K);
    DCLIP_HOST_CHECK(lda % 8 == 0 && ldb % 8 == 0 && lda >= K && ldb >= K,
                     "dclip_gemm: lda/ldb must be >= K and multiples of 8");
    DCLIP_HOST_CHECK(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "dclip_gemm: A/B must be 16-byte aligned");
    DCLIP_HOST_CHECK(splits == 1 || epilogue == DCLIP_EPI_SPLITK, "dclip_gemm: splits > 1 needs EPI_SPLITK");
    switch (epilogue) {
        case DCLIP_EPI_STORE:
            DCLIP_HOST_CHECK(c_dt == DCLIP_F32 || c_dt == ab_dt, "dclip_gemm: STORE output must be f32 or the operand dtype");
            break;
        case DCLIP_EPI_GELU:
            DCLIP_HOST_CHECK(c_dt == ab_dt && C2 != nullptr, "dclip_gemm: GELU needs C and C2 of the operand dtype");
            break;
        case DCLIP_EPI_RESIDUAL:
            DCLIP_HOST_CHECK(c_dt == DCLIP_F32 && aux_dt == DCLIP_F32 && aux != nullptr && ldc % 4 == 0 && ld_aux % 4 == 0,
                             "dclip_gemm: RESIDUAL needs f32 C and aux (ld %% 4 == 0)");
            break;
        case DCLIP_EPI_GELU_BWD:
            DCLIP_HOST_CHECK(c_dt == ab_dt && aux_dt == ab_dt && aux != nullptr, "dclip_gemm: GELU_BWD needs aux=z and C of the operand dtype");
            break;
        case DCLIP_EPI_SPLITK:
            DCLIP_HOST_CHECK(c_dt == DCLIP_F32 && aux != nullptr && N % 4 == 0 && ldc % 4 == 0,
                             "dclip_gemm: SPLITK needs f32 C, an f32 workspace aux of splits*M*N and N %% 4 == 0");
            break;
        default:
            DCLIP_HOST_CHECK(false, "dclip_gemm: unknown epilogue %d", epilogue);
    }
    hipStream_t st = (hipStream_t)stream;
    int rc = ab_dt == DCLIP_BF16
                 ? dispatch<bf16>(epilogue, c_dt, A, lda, B, ldb, M, N, K, splits, bias, aux, ld_aux, C, ldc, C2, ldc2, st)
                 : dispatch<f16>(epilogue, c_dt, A, lda, B, ldb, M, N, K, splits, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
    if (rc) return rc;
    DCLIP_LAUNCH_CHECK();
    return 0;
}
