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
#include <mutex>
#include <type_traits>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = 128 * BK * 2;      // 16 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;   // A + B
constexpr int EP_LD = 68;                     // epilogue LDS row stride (floats): 64 + 4 pad
constexpr int SMEM_BYTES = 4 * 64 * EP_LD * 4 > 2 * STAGE_BYTES ? 4 * 64 * EP_LD * 4 : 2 * STAGE_BYTES;

// 8 consecutive elements of a row: one 16-byte (16-bit types) or two (f32) accesses when
// the row segment is complete, element-wise otherwise
template <typename T>
__device__ __forceinline__ void store8(T* p, const float* v, bool full, int rem) {
    if (full) {
        if constexpr (sizeof(T) == 4) {
            f32x4 a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
            *(f32x4*)p = a;
            *(f32x4*)(p + 4) = b;
        } else {
            typedef T t8 __attribute__((ext_vector_type(8)));
            t8 x;
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = (T)v[e];
            *(t8*)p = x;
        }
    } else {
        for (int e = 0; e < rem && e < 8; ++e) p[e] = (T)v[e];
    }
}
template <typename T>
__device__ __forceinline__ void load8(const T* p, float* v, bool full, int rem) {
    if (full) {
        if constexpr (sizeof(T) == 4) {
            const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
            v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
            v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
        } else {
            typedef T t8 __attribute__((ext_vector_type(8)));
            const t8 x = *(const t8*)p;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
        }
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = e < rem ? (float)p[e] : 0.f;
    }
}

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

// Shared epilogue of both GEMM kernels.  acc[i][j][4q+e] = C[m][n] with
// m = m0 + 64wm + 32j + (lane & 31), n = n0 + 64wn + 32i + 8q + 4h + e.
template <typename T, int EPI, typename OutT>
__device__ __forceinline__ void gemm_epilogue(f32x16 (&acc)[2][2], char* smem, int M, int N, int m0, int n0,
                                              const float* __restrict__ bias, const void* __restrict__ aux,
                                              int64_t ld_aux, void* __restrict__ C, int64_t ldc,
                                              void* __restrict__ C2, int64_t ldc2, int64_t slab, float alpha) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    // The accumulator holds C^T (lane = row m, registers along n), so direct stores would
    // scatter each store instruction over 64 rows.  Instead each wave stages its 64 x 64
    // fp32 sub-tile (+ bias) in LDS (272-byte padded rows: conflict-free ds_write_b128)
    // and re-reads it row-contiguous: every global load/store of the epilogue is then a
    // full 8-element row segment per lane (8 lanes cover one 64-column row).
    __syncthreads();  // operand LDS no longer needed by any wave
    float* ep = (float*)smem + wave * (64 * EP_LD);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int col = i * 32 + q * 8 + h * 4;
                f32x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e] * alpha;
                if (bias != nullptr && EPI != DCLIP_EPI_SPLITK && EPI != DCLIP_EPI_GELU_BWD) {
                    const int n = n0 + wn * 64 + col;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += (n + e < N) ? bias[n + e] : 0.f;
                }
                if constexpr (EPI == DCLIP_EPI_STORE_SCALED) {
                    const int n = n0 + wn * 64 + col;
                    const float* sc = (const float*)aux;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] *= (n + e < N) ? sc[n + e] : 1.f;
                }
                *(f32x4*)(ep + (j * 32 + l32) * EP_LD + col) = v;
            }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    const int c8 = (lane & 7) * 8;
    const int nb = n0 + wn * 64 + c8;
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
        const int r = it * 8 + (lane >> 3);
        const int m = m0 + wm * 64 + r;
        if (m >= M || nb >= N) continue;
        float v[8];
        {
            const f32x4 a = *(const f32x4*)(ep + r * EP_LD + c8);
            const f32x4 b = *(const f32x4*)(ep + r * EP_LD + c8 + 4);
            v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
            v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
        }
        const bool full = nb + 8 <= N;
        if constexpr (EPI == DCLIP_EPI_STORE || EPI == DCLIP_EPI_STORE_SCALED) {
            store8<OutT>((OutT*)C + (int64_t)m * ldc + nb, v, full, N - nb);
        } else if constexpr (EPI == DCLIP_EPI_GELU) {
            float g[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                // the activation sees the rounded pre-activation, so forward and backward
                // use the same z
                v[e] = (float)(OutT)v[e];
                g[e] = quick_gelu(v[e]);
            }
            if (C != nullptr) store8<OutT>((OutT*)C + (int64_t)m * ldc + nb, v, full, N - nb);  // z: optional
            store8<OutT>((OutT*)C2 + (int64_t)m * ldc2 + nb, g, full, N - nb);
        } else if constexpr (EPI == DCLIP_EPI_RESIDUAL) {
            float rsd[8];
            load8<float>((const float*)aux + (int64_t)m * ld_aux + nb, rsd, full, N - nb);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += rsd[e];
            store8<float>((float*)C + (int64_t)m * ldc + nb, v, full, N - nb);
            if (C2 != nullptr) store8<T>((T*)C2 + (int64_t)m * ldc2 + nb, v, full, N - nb);  // 16-bit copy
        } else if constexpr (EPI == DCLIP_EPI_GELU_BWD) {
            float z[8];
            load8<T>((const T*)aux + (int64_t)m * ld_aux + nb, z, full, N - nb);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= quick_gelu_grad(z[e]);
            store8<OutT>((OutT*)C + (int64_t)m * ldc + nb, v, full, N - nb);
        } else {  // SPLITK: plain f32 partial slab per K split
            store8<float>((float*)C + blockIdx.y * slab + (int64_t)m * ldc + nb, v, full, N - nb);
        }
    }
}


template <typename T, int EPI, typename OutT>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    int M, int N, int k_chunk, int tiles_m, int tiles_n,
    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux,
    void* __restrict__ C, int64_t ldc, void* __restrict__ C2, int64_t ldc2, int64_t slab, Alpha alpha_arg) {
    const float alpha = alpha_arg.get();
    __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
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

    gemm_epilogue<T, EPI, OutT>(acc, smem, M, N, m0, n0, bias, aux, ld_aux, C, ldc, C2, ldc2, slab, alpha);
}

// ---------------------------------------------------------------------------- large tiles
// The production NT kernel for the token GEMMs (M = B*N ~ 65k rows): BM x BN x 64 tiles,
// 8 waves (WM x WN), MFMA v_mfma_f32_16x16x32 issued swapped (A-operand = B rows) so the
// accumulator holds C^T.  Operands move global -> LDS by 16-byte global_load_lds into a
// STAGES-deep ring (XOR swizzle applied to the per-lane SOURCE address, conflict-free
// ds_read_b128 fragment reads); one raw s_barrier per K-step with a COUNTED vmcnt, so up
// to STAGES-2 future tiles stay in flight across the barrier (a __syncthreads() would
// drain them: it waits vmcnt(0)).  Epilogue: each wave stages 32-row slices of its fp32
// sub-tile in LDS and re-reads them row-contiguous (8 columns per lane) for the fused
// bias / scale / QuickGELU / residual / QuickGELU' / split-K stores.

// one row segment of 8 columns [nb, nb + 8) of output row m: v = alpha * acc
template <typename T, int EPI, typename OutT>
__device__ __forceinline__ void epi_row8(float (&v)[8], int m, int nb, int N, const float* __restrict__ bias,
                                         const void* __restrict__ aux, int64_t ld_aux, void* __restrict__ C,
                                         int64_t ldc, void* __restrict__ C2, int64_t ldc2, int64_t slab) {
    const bool full = nb + 8 <= N;
    const int rem = N - nb;
    if (bias != nullptr && EPI != DCLIP_EPI_SPLITK && EPI != DCLIP_EPI_GELU_BWD) {
        float bv[8];
        load8<float>(bias + nb, bv, full, rem);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bv[e];
    }
    if constexpr (EPI == DCLIP_EPI_STORE_SCALED) {
        float sv[8];
        load8<float>((const float*)aux + nb, sv, full, rem);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= sv[e];
    }
    if constexpr (EPI == DCLIP_EPI_STORE || EPI == DCLIP_EPI_STORE_SCALED) {
        store8<OutT>((OutT*)C + (int64_t)m * ldc + nb, v, full, rem);
    } else if constexpr (EPI == DCLIP_EPI_GELU) {
        float g[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            v[e] = (float)(OutT)v[e];  // the activation sees the rounded pre-activation
            g[e] = quick_gelu(v[e]);
        }
        if (C != nullptr) store8<OutT>((OutT*)C + (int64_t)m * ldc + nb, v, full, rem);  // z: optional
        store8<OutT>((OutT*)C2 + (int64_t)m * ldc2 + nb, g, full, rem);
    } else if constexpr (EPI == DCLIP_EPI_RESIDUAL) {
        float rsd[8];
        load8<float>((const float*)aux + (int64_t)m * ld_aux + nb, rsd, full, rem);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rsd[e];
        store8<float>((float*)C + (int64_t)m * ldc + nb, v, full, rem);
        if (C2 != nullptr) store8<T>((T*)C2 + (int64_t)m * ldc2 + nb, v, full, rem);  // 16-bit copy
    } else if constexpr (EPI == DCLIP_EPI_GELU_BWD) {
        float z[8];
        load8<T>((const T*)aux + (int64_t)m * ld_aux + nb, z, full, rem);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= quick_gelu_grad(z[e]);
        store8<OutT>((OutT*)C + (int64_t)m * ldc + nb, v, full, rem);
    } else {  // SPLITK: plain f32 partial slab per K split
        store8<float>((float*)C + blockIdx.y * slab + (int64_t)m * ldc + nb, v, full, rem);
    }
}

template <int BM, int BN, int WM, int WN, int STAGES, int BKT = 64>
struct BigCfg {
    static constexpr int NW = WM * WN, NT = 64 * NW;
    static constexpr int WTM = BM / WM, WTN = BN / WN;  // per-wave output tile
    static constexpr int MB = WTM / 16, NB = WTN / 16;   // 16x16 blocks per wave
    static constexpr int KB = BKT, ROWB = 2 * BKT;       // k per stage, LDS bytes per row
    static constexpr int RPI = 1024 / ROWB;              // rows per 1-KiB glds piece
    static constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE_BYTES = A_BYTES + B_BYTES;
    static constexpr int A_INST = BM / RPI / NW, B_INST = BN / RPI / NW;  // 1-KiB glds per wave per stage
    static constexpr int G = A_INST + B_INST;                          // glds per thread per stage
    static constexpr int EP_LD = WTN + 4;                              // epilogue row stride (floats)
    static constexpr int EP_BYTES = NW * 32 * EP_LD * 4;
    static constexpr int SMEM = STAGES * STAGE_BYTES > EP_BYTES ? STAGES * STAGE_BYTES : EP_BYTES;
    static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "staging split");
    static_assert(BKT == 64 || BKT == 32, "k per stage");
    static_assert(WTM % 32 == 0 && WTN % 16 == 0 && WTN <= 128, "wave tile");
};

// Epilogue of the large-tile kernels: 32-row slices of the wave's WTM x WTN tile go through
// LDS (f32, padded rows) and are re-read row-contiguous, 8 columns per lane.
// acc[i][j] holds C[mw + 16 j + (lane & 15)][nw + 16 i + 4 (lane >> 4) + e].
template <typename T, int EPI, typename OutT, typename Cfg>
__device__ __forceinline__ void big_epilogue(f32x4 (&acc)[Cfg::NB][Cfg::MB], char* smem, int M, int N, int mw, int nw,
                                             const float* __restrict__ bias, const void* __restrict__ aux,
                                             int64_t ld_aux, void* __restrict__ C, int64_t ldc, void* __restrict__ C2,
                                             int64_t ldc2, int64_t slab, float alpha, int map_hw = 0,
                                             int map_gap = 0, int map_off = 0) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int l16 = lane & 15, lq = lane >> 4;
    __syncthreads();  // every wave is done with the operand ring
    float* ep = (float*)smem + wave * (32 * Cfg::EP_LD);
    constexpr int LPR = Cfg::WTN / 8;  // lanes per output row
    constexpr int RPP = 64 / LPR;      // rows per pass
    const int c8 = (lane % LPR) * 8;
    const int nb = nw + c8;
#pragma unroll
    for (int sl = 0; sl < Cfg::MB / 2; ++sl) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i) {
                f32x4 v = acc[i][2 * sl + jj];
                v *= alpha;
                *(f32x4*)(ep + (jj * 16 + l16) * Cfg::EP_LD + i * 16 + 4 * lq) = v;
            }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 32 / RPP; ++it) {
            const int r = it * RPP + lane / LPR;
            const int m = mw + sl * 32 + r;
            if (m < M && nb < N) {
                float v[8];
                const f32x4 a = *(const f32x4*)(ep + r * Cfg::EP_LD + c8);
                const f32x4 b = *(const f32x4*)(ep + r * Cfg::EP_LD + c8 + 4);
                v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
                v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
                // output row: m, or (map_hw > 0) pixel m of a channels-last image whose batches of
                // map_hw pixels are separated by map_gap rows and start map_off rows in
                const int row = map_hw ? m + (m / map_hw) * map_gap + map_off : m;
                epi_row8<T, EPI, OutT>(v, row, nb, N, bias, aux, ld_aux, C, ldc, C2, ldc2, slab);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();  // reads of this slice done before the next slice's writes
    }
}

// chunk XOR of LDS row r: 128-B rows (BK 64): (r >> 1) & 7; 64-B rows (BK 32): ((r >> 3) & 1) << 1
// — both make the 16x16x32 fragment reads (16 rows x one chunk per 16 lanes) conflict-free
template <int BKT>
__device__ __forceinline__ int big_sw(int r) {
    if constexpr (BKT == 64) return (r >> 1) & 7;
    else return ((r >> 3) & 1) << 1;
}

template <typename T, int ROWS_INST, int BKT>
__device__ __forceinline__ void stage_rows(const T* __restrict__ X, int64_t ldx, int row0, int rows, int k0,
                                           char* lds, int wave, int lane) {
    constexpr int CPR = BKT / 8;  // 16-B chunks per row
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i) {
        const int inst = wave * ROWS_INST + i;
        const int r = inst * (64 / CPR) + lane / CPR;
        const int c = (lane % CPR) ^ big_sw<BKT>(r);
        int gr = row0 + r;
        gr = gr < rows ? gr : rows - 1;
        __builtin_amdgcn_global_load_lds((const void*)(X + (int64_t)gr * ldx + k0 + c * 8), LDS_PTR(lds + inst * 1024),
                                         16, 0, 0);
    }
}

// stage_rows as buffer loads: per-lane byte offsets of this thread's pieces (rows row0.., clamped
// to rows - 1, swizzled chunk) computed once per tile by rows_voff, plus the K-step's byte offset:
// one add per load instead of the ~11 address instructions (3 of them 64-bit multiplies) of
// stage_rows, which sat between every K-step's barrier and its first MFMA
template <typename T, int ROWS_INST, int BKT>
__device__ __forceinline__ void rows_voff(int64_t ldx, int row0, int rows, int wave, int lane,
                                          uint32_t (&voff)[ROWS_INST]) {
    constexpr int CPR = BKT / 8;
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i) {
        const int inst = wave * ROWS_INST + i;
        const int r = inst * (64 / CPR) + lane / CPR;
        const int c = (lane % CPR) ^ big_sw<BKT>(r);
        int gr = row0 + r;
        gr = gr < rows ? gr : rows - 1;
        voff[i] = (uint32_t)((gr * ldx + c * 8) * (int64_t)sizeof(T));
    }
}

template <typename T, int ROWS_INST>
__device__ __forceinline__ void stage_rows_buf(const T* X, uint32_t bytes, const uint32_t (&voff)[ROWS_INST],
                                               uint32_t kbyte, char* lds, int wave) {
#if defined(__HIP_DEVICE_COMPILE__)  // the buffer-resource type exists only for the device target
    const rsrc_t rs = make_rsrc(X, bytes);
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(lds + (wave * ROWS_INST + i) * 1024), 16, voff[i] + kbyte,
                                                 0, 0, 0);
#endif
}

// stage_rows_buf with the per-tile and per-piece parts of the source offset in the SCALAR
// offset: piece i of wave w covers rows 8 (w RI + i) .. + 7 of the tile; lane l reads row
// l / 8 of it, chunk (l % 8) ^ big_sw(row), and for BKT 64 and an even RI that swizzle depends
// on the piece only through its parity.  Two offset VGPRs per operand, none per tile.
template <int ROWS_INST>
__device__ __forceinline__ void rows_voff2(uint32_t ldbytes, int lane, uint32_t (&v2)[2]) {
    static_assert(ROWS_INST % 2 == 0, "piece parity");
#pragma unroll
    for (int p = 0; p < 2; ++p)
        v2[p] = (uint32_t)(lane >> 3) * ldbytes + (uint32_t)(((lane & 7) ^ ((4 * p + (lane >> 4)) & 7)) << 4);
}

template <typename T, int ROWS_INST>
__device__ __forceinline__ void stage_rows_sbuf(const T* X, uint32_t bytes, const uint32_t (&v2)[2], uint32_t s0,
                                                uint32_t s8, char* lds, int wave) {
#if defined(__HIP_DEVICE_COMPILE__)
    const rsrc_t rs = make_rsrc(X, bytes);
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(lds + (wave * ROWS_INST + i) * 1024), 16, v2[i & 1],
                                                 s0 + (uint32_t)i * s8, 0, 0);
#endif
}

template <typename T, int BKT>
__device__ __forceinline__ typename Mfma<T>::frag big_frag(const char* img, int r, int chunk) {
    return *(const typename Mfma<T>::frag*)(img + r * (2 * BKT) + ((chunk ^ big_sw<BKT>(r)) << 4));
}

template <typename T, int EPI, typename OutT, int BM, int BN, int WM, int WN, int STAGES, int BKT>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_nt_big_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    int M, int N, int k_chunk, int tiles_m, int tiles_n,
    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux,
    void* __restrict__ C, int64_t ldc, void* __restrict__ C2, int64_t ldc2, int64_t slab, Alpha alpha_arg) {
    const float alpha = alpha_arg.get();
    typedef BigCfg<BM, BN, WM, WN, STAGES, BKT> Cfg;
    typedef typename Mfma<T>::frag frag;
    __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int l16 = lane & 15, lq = lane >> 4;

    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int m0 = (t / tiles_n) * BM;
    const int n0 = (t % tiles_n) * BN;
    const int kbeg = blockIdx.y * k_chunk;
    const int nk = k_chunk / BKT;

    f32x4 acc[Cfg::NB][Cfg::MB];
#pragma unroll
    for (int i = 0; i < Cfg::NB; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto stage = [&](int kt, int slot) {
        char* base = smem + slot * Cfg::STAGE_BYTES;
        stage_rows<T, Cfg::A_INST, BKT>(A, lda, m0, M, kbeg + kt * BKT, base, wave, lane);
        stage_rows<T, Cfg::B_INST, BKT>(B, ldb, n0, N, kbeg + kt * BKT, base + Cfg::A_BYTES, wave, lane);
    };
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) stage(s, s);

    for (int kt = 0; kt < nk; ++kt) {
        // tile kt has landed when at most min(STAGES-2, nk-1-kt) younger tiles are in flight
        if (kt + STAGES - 2 <= nk - 1) wait_vmcnt<Cfg::G * (STAGES - 2)>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // tile kt visible to every wave; slot of tile kt-1 free
        __builtin_amdgcn_sched_barrier(0);
        if (kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
        const char* At = smem + (kt % STAGES) * Cfg::STAGE_BYTES;
        const char* Bt = At + Cfg::A_BYTES;
#pragma unroll
        for (int ks = 0; ks < BKT / 32; ++ks) {
            frag fb[Cfg::NB], fa[Cfg::MB];
            const int ch = ks * 4 + lq;
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i) fb[i] = big_frag<T, BKT>(Bt, wn * Cfg::WTN + i * 16 + l16, ch);
#pragma unroll
            for (int j = 0; j < Cfg::MB; ++j) fa[j] = big_frag<T, BKT>(At, wm * Cfg::WTM + j * 16 + l16, ch);
#pragma unroll
            for (int j = 0; j < Cfg::MB; ++j)
#pragma unroll
                for (int i = 0; i < Cfg::NB; ++i) acc[i][j] = Mfma16<T>::mma(fb[i], fa[j], acc[i][j]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    big_epilogue<T, EPI, OutT, Cfg>(acc, smem, M, N, m0 + wm * Cfg::WTM, n0 + wn * Cfg::WTN, bias, aux, ld_aux,
                                     C, ldc, C2, ldc2, slab, alpha);
}

// ---------------------------------------------------------------------------- ping-pong 256x256
// The same 256x256 tile, 8 waves (2 x 4, 128 x 64 per wave) and 128 KiB of LDS as
// gemm_nt_big_kernel, with the K-loop cut into phases of 16 MFMAs and the two wave groups
// (rows 0-127 / 128-255 of the tile) run one barrier apart, so that on every SIMD (one wave
// of each group) one wave's MFMAs overlap the other's fragment reads.
//   * a 64-deep K-tile lives in the LDS as two K-halves of 32 (A 256 x 64 B + B 256 x 64 B
//     each), 2 tiles resident: 4 half-slots of 32 KiB;
//   * phases per K-tile: (rows 0-63 of the wave tile, K-half 0), (rows 64-127, K-half 0),
//     (rows 0-63, K-half 1), (rows 64-127, K-half 1): 4 x 4 MFMA 16x16x32 each; B fragments
//     are read at the first phase of a K-half and reused by the second;
//   * K-half 0 of tile t+1 is issued (LDS-DMA, 4 per thread) at phase 0 of tile t, K-half 1
//     at phase 2; each is retired by a counted vmcnt(4) two phases later — one phase before
//     it is read — so the next K-half stays in flight across every barrier, and every
//     half-slot is rewritten 3 phases after its last read (safe under the one-barrier stagger).
template <typename T, int QM, bool LOADB>
__device__ __forceinline__ void pp_phase(f32x4 (&acc)[4][8], typename Mfma<T>::frag (&fa)[4],
                                         typename Mfma<T>::frag (&fb)[4], const char* half, int arow, int brow,
                                         int lq) {
    if constexpr (LOADB) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fb[i] = big_frag<T, 32>(half + 16384, brow + i * 16, lq);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) fa[j] = big_frag<T, 32>(half, arow + QM * 64 + j * 16, lq);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this phase's fragments are in registers
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][QM * 4 + j] = Mfma16<T>::mma(fb[i], fa[j], acc[i][QM * 4 + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <typename T, int EPI, typename OutT>
__global__ __launch_bounds__(512, 1) void gemm_nt_pp_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    int M, int N, int k_chunk, int tiles_m, int tiles_n,
    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux,
    void* __restrict__ C, int64_t ldc, void* __restrict__ C2, int64_t ldc2, int64_t slab, Alpha alpha_arg) {
    const float alpha = alpha_arg.get();
    typedef BigCfg<256, 256, 2, 4, 2, 64> Cfg;
    typedef typename Mfma<T>::frag frag;
    constexpr int HALF = 32768;
    __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int l16 = lane & 15, lq = lane >> 4;
    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int m0 = (t / tiles_n) * 256;
    const int n0 = (t % tiles_n) * 256;
    const int kbeg = blockIdx.y * k_chunk;
    const int nk = k_chunk / 64;
    const int arow = wr * 128 + l16, brow = wc * 64 + l16;

    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    frag fa[4], fb[4];

    auto stage = [&](int kt, int kh) {
        char* base = smem + ((kt & 1) * 2 + kh) * HALF;
        const int k0 = kbeg + kt * 64 + kh * 32;
        stage_rows<T, 2, 32>(A, lda, m0, M, k0, base, wave, lane);
        stage_rows<T, 2, 32>(B, ldb, n0, N, k0, base + 16384, wave, lane);
    };
    stage(0, 0);
    stage(0, 1);
    wait_vmcnt<4>();  // K-half 0 of tile 0 landed (K-half 1 in flight)
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0

    for (int kt = 0; kt < nk; ++kt) {
        const char* h0 = smem + (kt & 1) * 2 * HALF;
        const char* h1 = h0 + HALF;
        const bool more = kt + 1 < nk;
        if (more) stage(kt + 1, 0);
        pp_phase<T, 0, true>(acc, fa, fb, h0, arow, brow, lq);
        if (more) wait_vmcnt<4>();  // K-half 1 of tile kt (read from the next phase on)
        else wait_vmcnt<0>();
        pp_phase<T, 1, false>(acc, fa, fb, h0, arow, brow, lq);
        if (more) stage(kt + 1, 1);
        pp_phase<T, 0, true>(acc, fa, fb, h1, arow, brow, lq);
        if (more) wait_vmcnt<4>();  // K-half 0 of tile kt+1
        pp_phase<T, 1, false>(acc, fa, fb, h1, arow, brow, lq);
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups

    big_epilogue<T, EPI, OutT, Cfg>(acc, smem, M, N, m0 + wr * 128, n0 + wc * 64, bias, aux, ld_aux, C, ldc, C2, ldc2,
                                     slab, alpha);
}

// ---------------------------------------------------------------------------- persistent 256x256
// One workgroup per CU walks its tiles (u = round * G + xcd_remap(block), G = grid size) as ONE
// continuous K-stream over the 2-slot LDS ring of gemm_nt_big_kernel: the last K-step of a
// tile already stages K-step 0 of the next, and the epilogue runs from the accumulators
// straight to global memory (no LDS, no barrier) while those loads fly, so neither the
// epilogue's stores nor the next tile's first load latency stall the MFMA pipe the way a
// grid of one-tile workgroups does (whose epilogues all run at once, round after round).
// Full tiles only (M % 256 == 0, N % 256 == 0; the launcher peels an M tail): no masks, so the
// epilogue issues at least 16 row-segment stores of C per lane after those loads, which lets
// the next tile's first wait count them (vmcnt(PERS_EPI_MIN)) instead of draining them.
// 16-bit outputs pair lanes l and l + 16 (adjacent 4-column groups) with one exchange so that
// every store is 16 contiguous bytes.
constexpr int PERS_EPI_MIN = 16;

// 16-bit row segments: v0 / v1 = this lane's 4 columns of blocks i and i + 1 (columns
// 16 i + 4 lq + e); after the exchange with lane ^ 16 an even-lq lane stores block i's columns
// 4 lq .. 4 lq + 7 and an odd-lq lane block i+1's columns 4 (lq - 1) .. 4 lq + 3.
template <typename OutT>
__device__ __forceinline__ void store_pair16(OutT* row_base, int col_i, const f32x4& v0, const f32x4& v1, int lq) {
    typedef OutT t2 __attribute__((ext_vector_type(2)));
    const t2 a0 = {(OutT)v0[0], (OutT)v0[1]}, a1 = {(OutT)v0[2], (OutT)v0[3]};
    const t2 b0 = {(OutT)v1[0], (OutT)v1[1]}, b1 = {(OutT)v1[2], (OutT)v1[3]};
    const unsigned p0x = __builtin_bit_cast(unsigned, a0), p0y = __builtin_bit_cast(unsigned, a1);
    const unsigned p1x = __builtin_bit_cast(unsigned, b0), p1y = __builtin_bit_cast(unsigned, b1);
    const bool odd = lq & 1;
    const unsigned rx = __shfl_xor(odd ? p0x : p1x, 16, 64), ry = __shfl_xor(odd ? p0y : p1y, 16, 64);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 w = odd ? u32x4{rx, ry, p1x, p1y} : u32x4{p0x, p0y, rx, ry};
    const int col = odd ? col_i + 16 - 4 : col_i;  // col_i = 16 i + 4 lq (+ tile offset)
    *(u32x4*)(row_base + col) = w;
}

// a 16-byte global store, with the streaming (nontemporal) hint when NTS
template <bool NTS, typename V>
__device__ __forceinline__ void st16(V* p, const V& v) {
    if constexpr (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <typename OutT>
__device__ __forceinline__ void store4_out(OutT* p, const f32x4& v) {
    if constexpr (sizeof(OutT) == 4) {
        *(f32x4*)p = v;
    } else {
        typedef OutT t4 __attribute__((ext_vector_type(4)));
        const t4 x = {(OutT)v[0], (OutT)v[1], (OutT)v[2], (OutT)v[3]};
        *(t4*)p = x;
    }
}

// acc[j] += b . a[j] for j < 8 (v_mfma_f32_16x16x32, accumulators in AGPRs).  Opens with s_nop 1:
// a fragment (or a zeroed accumulator) may have been written by VALU just before (the compiler pads
// no hazard into an asm statement).
template <typename T>
__device__ __forceinline__ void tn_mfma_row(f32x4 (&acc)[8], const typename Mfma<T>::frag& b,
                                            const typename Mfma<T>::frag (&a)[8]) {
#define TN_MFMA8(OP)                                                                                         \
    asm volatile("s_nop 1\n\t" OP " %0, %8, %9, %0\n\t" OP " %1, %8, %10, %1\n\t" OP " %2, %8, %11, %2\n\t" OP \
                 " %3, %8, %12, %3\n\t" OP " %4, %8, %13, %4\n\t" OP " %5, %8, %14, %5\n\t" OP                   \
                 " %6, %8, %15, %6\n\t" OP " %7, %8, %16, %7"                                                   \
                 : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]), "+a"(acc[4]), "+a"(acc[5]),         \
                   "+a"(acc[6]), "+a"(acc[7])                                                                  \
                 : "v"(b), "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),         \
                   "v"(a[7]))
    if constexpr (std::is_same<T, bf16>::value) TN_MFMA8("v_mfma_f32_16x16x32_bf16");
    else TN_MFMA8("v_mfma_f32_16x16x32_f16");
#undef TN_MFMA8
}

// the accumulators' last asm MFMA results: wait states before anything reads them (one group)
__device__ __forceinline__ void tn_acc_fence(f32x4 (&acc)[8], bool nops) {
    if (nops)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                     : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]), "+a"(acc[4]), "+a"(acc[5]),
                       "+a"(acc[6]), "+a"(acc[7]));
    else
        asm volatile(""
                     : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]), "+a"(acc[4]), "+a"(acc[5]),
                       "+a"(acc[6]), "+a"(acc[7]));
}

// epilogue of the persistent kernels, from the accumulators straight to global memory:
// acc[i][j] = C[mw + 16 j + l16][nw + 16 i + 4 lq + e]
// the per-column constants (bias, QKV scale) of a wave's columns, loaded when its tile starts so
// that their latency hides behind the K-loop instead of stalling the epilogue
template <int EPI, int NB>
struct PersCols {
    f32x4 bv[NB], sv[NB];
};

template <int EPI, int NB>
__device__ __forceinline__ void pers_cols(PersCols<EPI, NB>& pc, const float* __restrict__ bias,
                                          const void* __restrict__ aux, int nw, int lq) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int col = nw + 16 * i + 4 * lq;
        pc.bv[i] = (bias != nullptr && EPI != DCLIP_EPI_GELU_BWD) ? *(const f32x4*)(bias + col)
                                                                 : f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (EPI == DCLIP_EPI_STORE_SCALED) pc.sv[i] = *(const f32x4*)((const float*)aux + col);
    }
}

template <typename T, int EPI, typename OutT, typename Cfg>
__device__ __forceinline__ void pers_epilogue(const f32x4 (&acc)[Cfg::NB][Cfg::MB], const PersCols<EPI, Cfg::NB>& pc,
                                              int mw, int nw, int l16, int lq, float alpha,
                                              const void* __restrict__ aux, int64_t ld_aux, void* __restrict__ C,
                                              int64_t ldc, void* __restrict__ C2, int64_t ldc2) {
#ifdef DCLIP_GEMM_DIAG_NOSTORE
    if (alpha != 12345.0f) return;  // tools/gemm_epi_probe.hip only: the K-loop without its epilogue
#endif
    // rows outer, column pairs inner (a row's segments stored back to back)
#pragma unroll
    for (int j = 0; j < Cfg::MB; ++j) {
        const int64_t row = mw + 16 * j + l16;
#pragma unroll
        for (int i = 0; i < Cfg::NB; i += 2) {
            const f32x4 bv[2] = {pc.bv[i], pc.bv[i + 1]};
            f32x4 sv[2];
            if constexpr (EPI == DCLIP_EPI_STORE_SCALED) {
                sv[0] = pc.sv[i];
                sv[1] = pc.sv[i + 1];
            }
            const int col = nw + 16 * i + 4 * lq;
            f32x4 v[2] = {acc[i][j] * alpha + bv[0], acc[i + 1][j] * alpha + bv[1]};
            if constexpr (EPI == DCLIP_EPI_RESIDUAL || sizeof(OutT) == 4) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if constexpr (EPI == DCLIP_EPI_RESIDUAL)
                        v[h] += *(const f32x4*)((const float*)aux + row * ld_aux + col + 16 * h);
                    store4_out<OutT>((OutT*)C + row * ldc + col + 16 * h, v[h]);
                }
                if constexpr (EPI == DCLIP_EPI_RESIDUAL) {
                    // the 16-bit copy of the new residual (a read-out map's token buffer): C2 is
                    // null or set for the whole launch, so every lane takes the pair exchange
                    if (C2 != nullptr) store_pair16<T>((T*)C2 + row * ldc2, col, v[0], v[1], lq);
                }
            } else if constexpr (EPI == DCLIP_EPI_STORE) {
                store_pair16<OutT>((OutT*)C + row * ldc, col, v[0], v[1], lq);
            } else if constexpr (EPI == DCLIP_EPI_STORE_SCALED) {
                store_pair16<OutT>((OutT*)C + row * ldc, col, v[0] * sv[0], v[1] * sv[1], lq);
            } else if constexpr (EPI == DCLIP_EPI_GELU) {
                f32x4 g[2];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[h][e] = (float)(OutT)v[h][e];  // the activation sees the rounded pre-activation
                        g[h][e] = quick_gelu(v[h][e]);
                    }
                if (C != nullptr) store_pair16<OutT>((OutT*)C + row * ldc, col, v[0], v[1], lq);  // z: optional
                store_pair16<OutT>((OutT*)C2 + row * ldc2, col, g[0], g[1], lq);
            } else if constexpr (EPI == DCLIP_EPI_GELU_BWD) {
                typedef T t4 __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const t4 z = *(const t4*)((const T*)aux + row * ld_aux + col + 16 * h);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[h][e] *= quick_gelu_grad((float)z[e]);
                }
                store_pair16<OutT>((OutT*)C + row * ldc, col, v[0], v[1], lq);
            }
        }
    }
}

// The same epilogue with every global access a run of whole 128-B lines: a store instruction of
// the accumulator layout above covers 16 rows x 64 B, and one CU issues those at ~32 GB/s
// (4.3 us for a 256 x 256 bf16 tile), while 8 rows x 128 B per instruction go at ~120 GB/s
// (tools/gemm_epi_probe.hip, profiles/r03/r03q_*).  Each wave turns its 128 x 64 tile around
// in 16-row chunks through its own 4 KiB of LDS (past the staging ring): the accumulator-layout
// values go in (16-bit for the bf16 / fp16 outputs, f32 where the row-major side still adds or
// multiplies: RESIDUAL, GELU_BWD, f32 outputs) and come back out row-major, 16 B per lane.
// XOR swizzles keep both sides free of bank conflicts:
//   16-bit image (128-B rows, 16-B chunks c): physical chunk c ^ ((row >> 1) & 7)
//   f32 image    (256-B rows, 16-B chunks c): physical chunk c ^ (row & 15)
template <typename T, int EPI, typename OutT, typename Cfg, bool NTS = false>
__device__ __forceinline__ void pers_epilogue_lds(const f32x4 (&acc)[Cfg::NB][Cfg::MB],
                                                  const PersCols<EPI, Cfg::NB>& pc, int mw, int nw, int l16, int lq,
                                                  int lane, float alpha, const void* __restrict__ aux, int64_t ld_aux,
                                                  void* __restrict__ C, int64_t ldc, void* __restrict__ C2,
                                                  int64_t ldc2, char* __restrict__ img) {
    static_assert(Cfg::NB == 4 && Cfg::MB == 8, "128 x 64 wave tiles");
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    constexpr bool F32IMG = sizeof(OutT) == 4 || EPI == DCLIP_EPI_RESIDUAL || EPI == DCLIP_EPI_GELU_BWD;
    // the row-major side input (residual rows / GELU' pre-activations), one chunk ahead: the loads
    // of chunk j + 1 are issued before chunk j's LDS round trip, so their latency is not exposed
    // once per chunk (the memory clobbers below keep the compiler from hoisting them itself)
    constexpr bool AUX = EPI == DCLIP_EPI_RESIDUAL || EPI == DCLIP_EPI_GELU_BWD;
    typedef T t4 __attribute__((ext_vector_type(4)));
    typedef typename std::conditional<EPI == DCLIP_EPI_RESIDUAL, f32x4, t4>::type auxv;
    auxv cur[4], nxt[4];
    auto aux_load = [&](auxv (&dst)[4], int jj) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t row = mw + 16 * jj + (lane >> 4) + 4 * q;
            const int col = nw + 4 * (lane & 15);
            if constexpr (EPI == DCLIP_EPI_RESIDUAL) dst[q] = *(const f32x4*)((const float*)aux + row * ld_aux + col);
            else dst[q] = *(const t4*)((const T*)aux + row * ld_aux + col);
        }
    };
    if constexpr (AUX) aux_load(cur, 0);
    // unrolled: a runtime chunk index into acc[][] would move the accumulators to scratch
#pragma unroll
    for (int j = 0; j < Cfg::MB; ++j) {
        if constexpr (AUX) {
            if (j + 1 < Cfg::MB) aux_load(nxt, j + 1);
        }
        // ---- in: this lane's row l16 of the chunk, 4 columns per 16-column block i
        if constexpr (F32IMG) {
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i) {
                const f32x4 v = acc[i][j] * alpha + pc.bv[i];  // bv = 0 for GELU_BWD (as pers_epilogue)
                const int c = (4 * i + lq) ^ (l16 & 15);
                *(f32x4*)(img + l16 * 256 + c * 16) = v;
            }
        } else {
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i) {
                f32x4 v = acc[i][j] * alpha + pc.bv[i];
                if constexpr (EPI == DCLIP_EPI_STORE_SCALED) v *= pc.sv[i];
                typedef OutT t4 __attribute__((ext_vector_type(4)));
                const int c = (2 * i + (lq >> 1)) ^ ((l16 >> 1) & 7);
                const int off = l16 * 128 + c * 16 + 8 * (lq & 1);
                t4 z = {(OutT)v[0], (OutT)v[1], (OutT)v[2], (OutT)v[3]};
                *(u32x2*)(img + off) = __builtin_bit_cast(u32x2, z);
                if constexpr (EPI == DCLIP_EPI_GELU) {  // the activation sees the rounded pre-activation
                    t4 g;
#pragma unroll
                    for (int e = 0; e < 4; ++e) g[e] = (OutT)quick_gelu((float)z[e]);
                    *(u32x2*)(img + 2048 + off) = __builtin_bit_cast(u32x2, g);
                }
            }
        }
        // one wave's LDS accesses execute in order; this keeps the compiler from hoisting the
        // reads above the writes
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // ---- out: whole rows, 16 B per lane
        const int64_t row0 = mw + 16 * j;
        if constexpr (F32IMG) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = (lane >> 4) + 4 * q, cc = lane & 15;
                f32x4 x = *(const f32x4*)(img + rr * 256 + ((cc ^ (rr & 15)) * 16));
                const int64_t row = row0 + rr;
                const int col = nw + 4 * cc;
                if constexpr (EPI == DCLIP_EPI_RESIDUAL) {
                    x += cur[q];
                    st16<NTS>((f32x4*)((float*)C + row * ldc + col), x);
                    if (C2 != nullptr) {
                        const t4 y = {(T)x[0], (T)x[1], (T)x[2], (T)x[3]};
                        *(t4*)((T*)C2 + row * ldc2 + col) = y;
                    }
                } else if constexpr (EPI == DCLIP_EPI_GELU_BWD) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) x[e] *= quick_gelu_grad((float)cur[q][e]);
                    store4_out<OutT>((OutT*)C + row * ldc + col, x);
                } else {
                    store4_out<OutT>((OutT*)C + row * ldc + col, x);
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int rr = (lane >> 3) + 8 * q, cc = lane & 7;
                const int off = rr * 128 + ((cc ^ ((rr >> 1) & 7)) * 16);
                const int64_t row = row0 + rr;
                const int col = nw + 8 * cc;
                if (EPI != DCLIP_EPI_GELU || C != nullptr)  // GELU: z optional
                    st16<NTS>((u32x4*)((OutT*)C + row * ldc + col), *(const u32x4*)(img + off));
                if constexpr (EPI == DCLIP_EPI_GELU)
                    st16<NTS>((u32x4*)((OutT*)C2 + row * ldc2 + col), *(const u32x4*)(img + 2048 + off));
            }
        }
        asm volatile("" ::: "memory");  // the next chunk's writes stay behind these reads
        if constexpr (AUX) {
            if (j + 1 < Cfg::MB) {
#pragma unroll
                for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
            }
        }
    }
}

// NW = 8: 2 x 4 waves of 128 x 64 (two waves per SIMD); NW = 4: 2 x 2 waves of 128 x 128 (one
// wave per SIMD, the accumulators in AGPRs: 2/3 of the fragment reads per MFMA)
// Work-conserving tile walk (DYN, sched != null): every tile is claimed, none is tied to a
// workgroup.  Round 0: workgroup b takes tile r = xcd_remap(b) by setting its bit in a bitmap
// (atomicOr, issued beside the first K-step's loads, read behind their wait); a workgroup that
// starts late — its CU held by RCCL's channel kernels or a side-stream graph — finds its bit already
// set by a thief and goes straight to the next claim.  Later tiles: the tiles past round 0 are cut
// into 8 XCD-contiguous ranges; a workgroup takes the next tile of its own XCD's range (L2 locality
// as in the static walk), then steals from the other ranges, then steals round-0 tiles whose
// workgroups have not started.  So a displaced workgroup costs its share of the work, not the
// launch's length.
// Off the critical path: the claim for the tile after the current one is an atomicAdd on the own
// range counter issued by thread 0 at the start of the current tile's epilogue (or at launch), not
// inspected until the next tile's K-step nk - 3 (the next tile's first K-step waits only for loads
// older than the epilogue's stores, so it has the whole epilogue to return); thread 0 then resolves
// it (stealing only when its range is empty) and publishes it in the first word of wave 0's epilogue
// image (the 160 KiB of LDS are all taken; that word is free until wave 0's epilogue); the waves
// read it behind K-step nk - 2's barrier, so K-step nk - 1's barrier orders every read before wave
// 0's epilogue overwrites it.  Needs nk >= 2 and ntiles >= G (launch_pers).
// sched (zero on entry): the 8 range counters at words 0, 32, .., 224 (one 128-B line each: the
// claims of one XCD never queue behind another's), finished workgroups at 256, the round-0 bitmap at
// [288, 296).  Each workgroup's claims end with exactly one that fails; the last workgroup to
// fail zeroes the set again (every claim has returned by then), so the next launch on the stream
// finds it zero (gemm_sched_counters gives each stream its own set).
__device__ __forceinline__ void pers_range(int x, int G, int ntiles, int& lo, int& hi) {
    const int rest = ntiles - G;
    lo = G + (int)((int64_t)rest * x / 8);
    hi = G + (int)((int64_t)rest * (x + 1) / 8);
}

// thread 0: the tile of claim v on the own range counter, else a stolen one, else ntiles
__device__ __forceinline__ int pers_resolve(unsigned* __restrict__ sched, int v, int xcd, int G, int ntiles) {
    int lo, hi;
    pers_range(xcd, G, ntiles, lo, hi);
    if (lo + v < hi) return lo + v;
#pragma unroll 1
    for (int k = 1; k < 8; ++k) {
        const int x = (xcd + k) & 7;
        pers_range(x, G, ntiles, lo, hi);
        if (lo >= hi) continue;
        const int w = (int)atomicAdd(sched + 32 * x, 1u);
        if (lo + w < hi) return lo + w;
    }
    unsigned* const bm = sched + 288;  // round-0 tiles whose workgroups have not started
#pragma unroll 1
    for (int w = 0; w < (G + 31) / 32; ++w) {
        const unsigned valid = (w * 32 + 32 <= G) ? 0xffffffffu : ((1u << (G - w * 32)) - 1u);
        unsigned bits = atomicOr(bm + w, 0u);
        while ((~bits & valid) != 0u) {
            const int bit = __builtin_ctz(~bits & valid);
            const unsigned old = atomicOr(bm + w, 1u << bit);
            if (!(old & (1u << bit))) return w * 32 + bit;
            bits |= old;
        }
    }
    if ((int)atomicAdd(sched + 256, 1u) == G - 1) {  // the last workgroup out: re-arm for the next launch
#pragma unroll 1
        for (int i = 0; i < 8; ++i) atomicExch(sched + 32 * i, 0u);
        atomicExch(sched + 256, 0u);
#pragma unroll 1
        for (int i = 288; i < 296; ++i) atomicExch(sched + i, 0u);
    }
    return ntiles;
}

template <typename T, int EPI, typename OutT, int NW = 8, bool ELDS = false, bool DYN = false, bool NTS = false,
          bool PF = false>
__global__ __launch_bounds__(64 * NW, 1) void gemm_nt_pers_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb, int K, int tiles_m, int tiles_n,
    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux, void* __restrict__ C, int64_t ldc,
    void* __restrict__ C2, int64_t ldc2, Alpha alpha_arg, unsigned* __restrict__ sched = nullptr) {
    const float alpha = alpha_arg.get();
    typedef BigCfg<256, 256, 2, NW / 2, 2, 64> Cfg;
    typedef typename Mfma<T>::frag frag;
    // the staging ring, then (NW = 8) each wave's 4 KiB epilogue image (pers_epilogue_lds)
    constexpr int EPI_IMG = (NW == 8 && ELDS) ? 4096 : 0;
    __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM + NW * EPI_IMG];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / (NW / 2), wn = wave % (NW / 2);
    constexpr bool epi_lds = NW == 8 && ELDS;
    const int l16 = lane & 15, lq = lane >> 4;
    const int ntiles = tiles_m * tiles_n;
    const int G = gridDim.x;
    const int r = xcd_remap(blockIdx.x, G);  // the G tiles of a round in XCD-contiguous ranges
    const int nk = K / 64;
    const int M = tiles_m * 256, N = tiles_n * 256;

    // buffer-load staging (stage_rows_sbuf): two per-lane offsets per operand, the rest scalar
    const uint32_t abytes = (uint32_t)((int64_t)M * lda * sizeof(T)), bbytes = (uint32_t)((int64_t)N * ldb * sizeof(T));
    const uint32_t lda_b = (uint32_t)(lda * sizeof(T)), ldb_b = (uint32_t)(ldb * sizeof(T));
    uint32_t va[2], vb[2];
    rows_voff2<Cfg::A_INST>(lda_b, lane, va);
    rows_voff2<Cfg::B_INST>(ldb_b, lane, vb);
#define PERS_STAGE(M0, N0, KT, SLOT)                                                                                 \
    do {                                                                                                             \
        char* base_ = smem + (SLOT) * Cfg::STAGE_BYTES;                                                              \
        const uint32_t kb_ = (uint32_t)((KT) * 64 * sizeof(T));                                                      \
        stage_rows_sbuf<T, Cfg::A_INST>(A, abytes, va, (uint32_t)((M0) + 8 * wave * Cfg::A_INST) * lda_b + kb_,     \
                                        8 * lda_b, base_, wave);                                                     \
        stage_rows_sbuf<T, Cfg::B_INST>(B, bbytes, vb, (uint32_t)((N0) + 8 * wave * Cfg::B_INST) * ldb_b + kb_,     \
                                        8 * ldb_b, base_ + Cfg::A_BYTES, wave);                                      \
    } while (0)
    int u = r;
    if (u >= ntiles) return;
    int m0 = (u / tiles_n) * 256, n0 = (u % tiles_n) * 256;
    int* const pub = (int*)(smem + Cfg::SMEM);  // DYN: [0] next tile, [1] round-0 ownership (wave 0's image)
    const int xcd = blockIdx.x & 7;
    unsigned own_old = 0;  // thread 0 (DYN): the round-0 bitmap word before this workgroup's bit
    int pend = 0;          // thread 0 (DYN): the claim in flight on the own range counter
    if constexpr (DYN) {
        static_assert(!DYN || (NW == 8 && ELDS), "the claim words live in wave 0's epilogue image");
        if (threadIdx.x == 0) {
            own_old = atomicOr(sched + 288 + (r >> 5), 1u << (r & 31));
            pend = (int)atomicAdd(sched + 32 * xcd, 1u);
        }
    }
    PERS_STAGE(m0, n0, 0, 0);
    int slot = 0;
    bool first = true;
    while (true) {
        f32x4 acc[Cfg::NB][Cfg::MB];
#pragma unroll
        for (int i = 0; i < Cfg::NB; ++i)
#pragma unroll
            for (int j = 0; j < Cfg::MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        PersCols<EPI, Cfg::NB> pc;
        pers_cols<EPI, Cfg::NB>(pc, bias, aux, n0 + wn * Cfg::WTN, lq);
        int un = u + G;
        if constexpr (DYN) {
            if (nk == 2 && threadIdx.x == 0) {  // no K-step nk - 3: the next tile published before the loop
                pub[0] = pers_resolve(sched, pend, xcd, G, ntiles);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
        int nm0 = (un / tiles_n) * 256, nn0 = (un % tiles_n) * 256;
        bool skip = false;
        for (int kt = 0; kt < nk; ++kt) {
            if (kt == 0 && !first) wait_vmcnt<PERS_EPI_MIN>();  // this K-step's loads, not the epilogue's stores
            else wait_vmcnt<0>();
            if constexpr (DYN) {
                if (kt == 0 && first && u == r && threadIdx.x == 0) {  // round-0 ownership (the atomicOr has returned)
                    pub[1] = (own_old >> (r & 31)) & 1u;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
            }
            __builtin_amdgcn_s_barrier();  // K-step kt visible to every wave; the other slot free
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DYN) {
                if (kt == 0 && first && u == r && __builtin_amdgcn_readfirstlane(pub[1]) != 0) {
                    skip = true;  // a thief took tile r before this workgroup started
                    break;
                }
                if (kt == nk - 2) {  // the claim, published behind K-step nk - 3 (or before the loop)
                    un = __builtin_amdgcn_readfirstlane(pub[0]);
                    nm0 = (un / tiles_n) * 256;
                    nn0 = (un % tiles_n) * 256;
                }
            }
            if (kt + 1 < nk) {
                PERS_STAGE(m0, n0, kt + 1, slot ^ 1);
            } else if (un < ntiles) {  // the next tile's first K-step
                PERS_STAGE(nm0, nn0, 0, slot ^ 1);
            }
            const char* At = smem + slot * Cfg::STAGE_BYTES;
            const char* Bt = At + Cfg::A_BYTES;
            if constexpr (PF && NW == 8) {
                // fragment reads one group ahead: a group = the 8 MFMAs of one pair of A fragments
                // (both 32-deep halves of the K-step: 8 groups); each group's reads are issued before
                // the previous group's MFMAs, so a read has 8 MFMAs (~128 cycles) to land instead of
                // the 4 hipcc leaves it when it streams the A fragments two at a time
                frag fb[2][Cfg::NB], fa[4];
                auto rd_b = [&](int ks) {
#pragma unroll
                    for (int i = 0; i < Cfg::NB; ++i)
                        fb[ks][i] = big_frag<T, 64>(Bt, wn * Cfg::WTN + i * 16 + l16, ks * 4 + lq);
                };
                auto rd_a = [&](int ks, int p) {
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        fa[(2 * p + h) & 3] = big_frag<T, 64>(At, wm * Cfg::WTM + (2 * p + h) * 16 + l16, ks * 4 + lq);
                };
                rd_b(0);
                rd_a(0, 0);
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const int ks = g >> 2, p = g & 3;
                    if (g + 1 < 8) {
                        if (((g + 1) & 3) == 0) rd_b((g + 1) >> 2);
                        rd_a((g + 1) >> 2, (g + 1) & 3);
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int i = 0; i < Cfg::NB; ++i)
                            acc[i][2 * p + h] = Mfma16<T>::mma(fb[ks][i], fa[(2 * p + h) & 3], acc[i][2 * p + h]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                frag fb[Cfg::NB], fa[Cfg::MB];
                const int ch = ks * 4 + lq;
#pragma unroll
                for (int i = 0; i < Cfg::NB; ++i) fb[i] = big_frag<T, 64>(Bt, wn * Cfg::WTN + i * 16 + l16, ch);
#pragma unroll
                for (int j = 0; j < Cfg::MB; ++j) fa[j] = big_frag<T, 64>(At, wm * Cfg::WTM + j * 16 + l16, ch);
                if constexpr (NW == 4) {  // 128 x 128 per wave: the accumulators as AGPR asm operands
#pragma unroll
                    for (int i = 0; i < Cfg::NB; ++i) tn_mfma_row<T>(acc[i], fb[i], fa);
                } else {
#pragma unroll
                    for (int j = 0; j < Cfg::MB; ++j)
#pragma unroll
                        for (int i = 0; i < Cfg::NB; ++i) acc[i][j] = Mfma16<T>::mma(fb[i], fa[j], acc[i][j]);
                }
            }
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (DYN) {
                if (kt == nk - 3 && threadIdx.x == 0) {
                    pub[0] = pers_resolve(sched, pend, xcd, G, ntiles);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible at the next barrier
                }
            }
            slot ^= 1;
        }
        if constexpr (DYN) {
            if (skip) {  // nothing computed: resolve the pending claim now and start over on that tile
                if (threadIdx.x == 0) {
                    pub[0] = pers_resolve(sched, pend, xcd, G, ntiles);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_s_barrier();
                un = __builtin_amdgcn_readfirstlane(pub[0]);
                __builtin_amdgcn_s_barrier();  // every wave has read it before it can be rewritten
                if (un >= ntiles) break;
                if (threadIdx.x == 0) pend = (int)atomicAdd(sched + 32 * xcd, 1u);
                u = un;
                m0 = (u / tiles_n) * 256;
                n0 = (u % tiles_n) * 256;
                PERS_STAGE(m0, n0, 0, slot);  // the slot K-step 0 of tile r landed in (waited for)
                continue;                     // `first` stays: the next K-step 0 waits for everything
            }
        }
        if constexpr (NW == 4) {
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i) tn_acc_fence(acc[i], i == 0);
        }
        if constexpr (DYN) {  // the claim for the tile after the next one, while the epilogue runs
            if (un < ntiles && threadIdx.x == 0) pend = (int)atomicAdd(sched + 32 * xcd, 1u);
        }
        if constexpr (NW == 8) {
            if constexpr (epi_lds)
                pers_epilogue_lds<T, EPI, OutT, Cfg, NTS>(acc, pc, m0 + wm * 128, n0 + wn * Cfg::WTN, l16, lq, lane, alpha,
                                                     aux, ld_aux, C, ldc, C2, ldc2, smem + Cfg::SMEM + wave * EPI_IMG);
            else
                pers_epilogue<T, EPI, OutT, Cfg>(acc, pc, m0 + wm * 128, n0 + wn * Cfg::WTN, l16, lq, alpha, aux, ld_aux,
                                                 C, ldc, C2, ldc2);
        } else {
            pers_epilogue<T, EPI, OutT, Cfg>(acc, pc, m0 + wm * 128, n0 + wn * Cfg::WTN, l16, lq, alpha, aux, ld_aux, C,
                                             ldc, C2, ldc2);
        }
        if (un >= ntiles) break;
        u = un;
        m0 = nm0;
        n0 = nn0;
        first = false;
    }
#undef PERS_STAGE
}

// ---------------------------------------------------------------------------- persistent, pipelined fragments
// gemm_nt_pers_kernel with the LDS fragment reads software-pipelined across the MFMA stream:
// the K-stream is cut into 32-deep phases (two per 64-deep K-step) and two fragment register
// sets alternate, so the reads of phase p+1 are issued between the MFMAs of phase p
// (sched_group_barrier interleave) instead of just in time behind an lgkmcnt wait.  One
// barrier per K-step sits between its two phases: by then every wave holds both phases of the
// step in registers (slot free for the step two ahead) and the next step has landed.
// Needs K >= 128 (the DMA for step g + 2 may already belong to the next tile).
template <typename T, int NB, int MB>
__device__ __forceinline__ void pipe_frags(typename Mfma<T>::frag (&fb)[NB], typename Mfma<T>::frag (&fa)[MB],
                                           const char* At, const char* Bt, int arow, int brow, int ch) {
#pragma unroll
    for (int i = 0; i < NB; ++i) fb[i] = big_frag<T, 64>(Bt, brow + i * 16, ch);
#pragma unroll
    for (int j = 0; j < MB; ++j) fa[j] = big_frag<T, 64>(At, arow + j * 16, ch);
}

template <typename T, int NB, int MB>
__device__ __forceinline__ void pipe_mfma(f32x4 (&acc)[NB][MB], const typename Mfma<T>::frag (&fb)[NB],
                                          const typename Mfma<T>::frag (&fa)[MB]) {
#pragma unroll
    for (int j = 0; j < MB; ++j)
#pragma unroll
        for (int i = 0; i < NB; ++i) acc[i][j] = Mfma16<T>::mma(fb[i], fa[j], acc[i][j]);
}

// MB*NB MFMAs with the phase's MB+NB fragment reads spread between them
template <int NB, int MB>
__device__ __forceinline__ void pipe_interleave() {
    constexpr int D = NB + MB, F = NB * MB, PER = F / D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, F - PER * D, 0);
}

template <typename T, int EPI, typename OutT, int NW>
__global__ __launch_bounds__(64 * NW, 1) void gemm_nt_pipe_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb, int K, int tiles_m, int tiles_n,
    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux, void* __restrict__ C, int64_t ldc,
    void* __restrict__ C2, int64_t ldc2, Alpha alpha_arg) {
    const float alpha = alpha_arg.get();
    typedef BigCfg<256, 256, 2, NW / 2, 2, 64> Cfg;
    constexpr int NB = Cfg::NB, MB = Cfg::MB;
    typedef typename Mfma<T>::frag frag;
    __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / (NW / 2), wn = wave % (NW / 2);
    const int l16 = lane & 15, lq = lane >> 4;
    const int ntiles = tiles_m * tiles_n;
    const int G = gridDim.x;
    const int nk = K / 64;
    const int M = tiles_m * 256, N = tiles_n * 256;
    const int arow = wm * Cfg::WTM + l16, brow = wn * Cfg::WTN + l16;
    const uint32_t abytes = (uint32_t)((int64_t)M * lda * sizeof(T)), bbytes = (uint32_t)((int64_t)N * ldb * sizeof(T));
    const uint32_t lda_b = (uint32_t)(lda * sizeof(T)), ldb_b = (uint32_t)(ldb * sizeof(T));
    uint32_t va[2], vb[2];
    rows_voff2<Cfg::A_INST>(lda_b, lane, va);
    rows_voff2<Cfg::B_INST>(ldb_b, lane, vb);
#define stage(M0_, N0_, KT_, SLOT_)                                                                                    \
    do {                                                                                                               \
        char* base_ = smem + (SLOT_) * Cfg::STAGE_BYTES;                                                               \
        const uint32_t kb_ = (uint32_t)((KT_) * 64 * sizeof(T));                                                       \
        stage_rows_sbuf<T, Cfg::A_INST>(A, abytes, va, (uint32_t)((M0_) + 8 * wave * Cfg::A_INST) * lda_b + kb_,       \
                                        8 * lda_b, base_, wave);                                                       \
        stage_rows_sbuf<T, Cfg::B_INST>(B, bbytes, vb, (uint32_t)((N0_) + 8 * wave * Cfg::B_INST) * ldb_b + kb_,       \
                                        8 * ldb_b, base_ + Cfg::A_BYTES, wave);                                        \
    } while (0)
    int u = xcd_remap(blockIdx.x, G);  // the G tiles of a round in XCD-contiguous ranges
    if (u >= ntiles) return;
    int m0 = (u / tiles_n) * 256, n0 = (u % tiles_n) * 256;
    stage(m0, n0, 0, 0);
    stage(m0, n0, 1, 1);
    wait_vmcnt<Cfg::G>();  // step 0 landed (step 1 in flight)
    __builtin_amdgcn_s_barrier();
    frag fb0[NB], fa0[MB], fb1[NB], fa1[MB];
    pipe_frags<T, NB, MB>(fb0, fa0, smem, smem + Cfg::A_BYTES, arow, brow, lq);
    int slot = 0;
    bool first = true;
    while (true) {
        f32x4 acc[NB][MB];
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = 0; j < MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        PersCols<EPI, Cfg::NB> pc;
        pers_cols<EPI, Cfg::NB>(pc, bias, aux, n0 + wn * Cfg::WTN, lq);
        const int un = u + G;
        const bool more = un < ntiles;
        const int nm0 = (un / tiles_n) * 256, nn0 = (un % tiles_n) * 256;
        // one 64-deep K-step (a macro: a lambda over these register arrays sends them to scratch);
        // VMWAIT: the DMA of step g + 1 is the youngest load, or (first step of a tile after the
        // first) older than the previous tile's epilogue stores, which are counted out, not drained
#define PIPE_STEP(KT, VMWAIT)                                                                                          \
    do {                                                                                                               \
        const int kt_ = (KT);                                                                                          \
        const char* At = smem + slot * Cfg::STAGE_BYTES;                                                               \
        const char* An = smem + (slot ^ 1) * Cfg::STAGE_BYTES;                                                         \
        /* phase (kt, 0): MFMAs on set 0, reads of (kt, 1) into set 1 */                                               \
        __builtin_amdgcn_sched_barrier(0);                                                                             \
        pipe_frags<T, NB, MB>(fb1, fa1, At, At + Cfg::A_BYTES, arow, brow, 4 + lq);                                    \
        pipe_mfma<T, NB, MB>(acc, fb0, fa0);                                                                           \
        pipe_interleave<NB, MB>();                                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                                             \
        wait_vmcnt<VMWAIT>();                                                                                          \
        __builtin_amdgcn_s_waitcnt(0xc07f); /* lgkmcnt(0): this wave is done reading slot `slot` */                    \
        __builtin_amdgcn_s_barrier();                                                                                  \
        /* set 1 pinned behind the barrier (the MFMA builtins are pure: without this the compiler */                   \
        /* hoists phase (kt, 1) above it and leaves the reads below with nothing beside them) */                       \
        for (int i = 0; i < NB; ++i) asm volatile("" : "+v"(fb1[i]));                                                  \
        for (int j = 0; j < MB; ++j) asm volatile("" : "+v"(fa1[j]));                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                                             \
        /* step g + 2 into the slot just read (branch-free: past the last tile a harmless re-load of */                \
        /* this tile's step 0 into a slot nobody reads again) */                                                       \
        const bool in_tile = kt_ + 2 < nk;                                                                             \
        stage(in_tile ? m0 : (more ? nm0 : m0), in_tile ? n0 : (more ? nn0 : n0),                                      \
              in_tile ? kt_ + 2 : (more ? kt_ + 2 - nk : 0), slot);                                                    \
        /* phase (kt, 1): MFMAs on set 1, reads of (kt + 1, 0) (or the next tile's first) into set 0 */                \
        __builtin_amdgcn_sched_barrier(0);                                                                             \
        pipe_frags<T, NB, MB>(fb0, fa0, An, An + Cfg::A_BYTES, arow, brow, lq);                                        \
        pipe_mfma<T, NB, MB>(acc, fb1, fa1);                                                                           \
        pipe_interleave<NB, MB>();                                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                                             \
        slot ^= 1;                                                                                                     \
    } while (0)
        if (first) PIPE_STEP(0, 0);
        else PIPE_STEP(0, PERS_EPI_MIN);
        for (int kt = 1; kt < nk; ++kt) PIPE_STEP(kt, 0);
#undef PIPE_STEP
        pers_epilogue<T, EPI, OutT, Cfg>(acc, pc, m0 + wm * 128, n0 + wn * Cfg::WTN, l16, lq, alpha, aux, ld_aux, C,
                                         ldc, C2, ldc2);
        if (!more) break;
        u = un;
        m0 = nm0;
        n0 = nn0;
        first = false;
    }
    wait_vmcnt<0>();
#undef stage
}

// ---------------------------------------------------------------------------- "TN"
// C[m][n] = sum_k A[k][m] * B[k][n]: both operands row-major with the reduction index on
// the ROWS — the weight-gradient shape dW = dY^T X (k = token, m/n = features).  Tiles of
// 64 k-rows x 128 columns are staged by global_load_lds (1 KiB = 4 rows x 256 B per
// wave-instruction, 16-byte chunks XOR-swizzled by (row & 3) << 2 so the transposing
// reads below are bank-conflict free) and the MFMA fragments (8 consecutive k for one
// column) are gathered with ds_read_b64_tr_b16.  No transposed copies in HBM.
//
// One 16-byte LDS-DMA per lane (global_load_lds_dwordx4) written as an asm statement: invisible to
// the compiler's LDS alias analysis, which otherwise waits vmcnt(0) before the first transposed
// fragment read (ds_read_b64_tr_b16 builtin) after any LDS-DMA builtin — the next K-step's staging
// then never overlaps this one's MFMAs.  The caller orders the ring with its own vmcnt wait before
// the barrier that publishes a stage.  M0 = the wave's 1-KiB LDS piece (one wait state after it).
__device__ __forceinline__ void glds16_asm(const void* src, const char* lds) {
    const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(lds));
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(la), "v"(src) : "memory", "m0");
}

template <typename T, bool AD = false>
__device__ __forceinline__ void stage_tile_tn(const T* __restrict__ X, int64_t ldx, int k0, int krows,
                                              int col0, int cols, char* lds_tile, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int inst = wave * 4 + i;
        const int r = inst * 4 + (lane >> 4);
        const int p = lane & 15;
        const int c = p ^ ((r & 3) << 2);
        int gr = k0 + r;
        gr = gr < krows ? gr : krows - 1;
        int gc = col0 + c * 8;
        gc = gc + 8 <= cols ? gc : cols - 8;  // tail columns: any in-bounds data, masked later
        const T* src = X + (int64_t)gr * ldx + gc;
        if constexpr (AD) glds16_asm(src, lds_tile + inst * 1024);
        else __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + inst * 1024), 16, 0, 0);
    }
}

// fragment of 8 consecutive k rows (k = 16s + 8h + j) for column cb*32 + (lane & 31)
template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag tr_frag_tn(const char* img, int s, int col_base, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4, h = lane >> 5;
    const int row = 16 * s + 8 * h + q;
    const int col = col_base + (g & 1) * 16 + 4 * p;
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    auto off = [](int r, int c) { return r * 256 + (((c >> 3) ^ ((r & 3) << 2)) << 4) + ((c & 7) << 1); };
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + off(row, col)));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + off(row + 4, col)));
    typedef short s8 __attribute__((ext_vector_type(8)));
    s8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(typename Mfma<T>::frag, v);
}

// AD: asm LDS-DMA staging and a bare barrier behind a vmcnt wait per K-step (as conv_wgrad_kernel)
template <typename T, int EPI, typename OutT, bool AD = false>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    int M, int N, int Kreal, int k_chunk, int tiles_m, int tiles_n, const float* __restrict__ bias,
    void* __restrict__ C, int64_t ldc, int64_t slab, Alpha alpha_arg) {
    const float alpha = alpha_arg.get();
    __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5;

    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int m0 = (t / tiles_n) * BM;
    const int n0 = (t % tiles_n) * BN;
    const int kbeg = blockIdx.y * k_chunk;
    int nk = k_chunk / BK;
    if (kbeg + nk * BK > Kreal) nk = (Kreal - kbeg + BK - 1) / BK;  // fully padded tiles skipped
    nk = nk < 0 ? 0 : nk;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    if (nk > 0) {
        stage_tile_tn<T>(A, lda, kbeg, Kreal, m0, M, smem, wave, lane);
        stage_tile_tn<T>(B, ldb, kbeg, Kreal, n0, N, smem + TILE_BYTES, wave, lane);
    }
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const char* At = smem + cur * STAGE_BYTES;
        const char* Bt = At + TILE_BYTES;
        const int k0 = kbeg + kt * BK;
        if (kt + 1 < nk) {
            char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
            stage_tile_tn<T, AD>(A, lda, k0 + BK, Kreal, m0, M, nxt, wave, lane);
            stage_tile_tn<T, AD>(B, ldb, k0 + BK, Kreal, n0, N, nxt + TILE_BYTES, wave, lane);
        }
        const bool ragged = k0 + BK > Kreal;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            typename Mfma<T>::frag fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = tr_frag_tn<T>(Bt, s, wn * 64 + i * 32, lane);
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = tr_frag_tn<T>(At, s, wm * 64 + j * 32, lane);
            if (ragged) {  // rows past the true K were clamped duplicates: zero them (A side)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        if (k0 + 16 * s + 8 * h + e >= Kreal) fb[j][e] = (T)0.f;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = Mfma<T>::mma(fa[i], fb[j], acc[i][j]);
        }
        if constexpr (AD) {
            wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();
        } else {
            __syncthreads();
        }
    }
    if constexpr (AD) __syncthreads();  // the epilogue reuses the ring
    gemm_epilogue<T, EPI, OutT>(acc, smem, M, N, m0, n0, bias, nullptr, 0, C, ldc, nullptr, 0, slab, alpha);
}

// ---------------------------------------------------------------------------- "TN", large tiles
// Weight-gradient GEMM on 256 x 256 output tiles, 8 waves (2 x 4), 16x16x32 MFMA.  A K-tile is
// 64 token rows x 256 feature columns of each operand (512-B rows in LDS), staged by
// global_load_lds in 1-KiB pieces (2 rows); fragments of 8 consecutive tokens for one column
// come from two ds_read_b64_tr_b16.  The 16-byte chunks of an LDS row are XOR-swizzled by
// 2 * tn_sw(row) so each half-wave's transposed reads (rows {0-3, 8-11} or {4-7, 12-15} of a
// 16-row group, 32 bytes each) hit 64 distinct banks; the swizzle is applied to the per-lane
// source address (LDS-DMA writes lane-linearly).
__device__ __forceinline__ int tn_sw(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int tn_off(int r, int col) {
    return r * 512 + ((((col >> 3) ^ (2 * tn_sw(r)))) << 4) + ((col & 7) << 1);
}

// fragment: element j = row (ks*32 + 8 (lane >> 4) + j), column col0 + (lane & 15)
template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag tn_frag(const char* img, int ks, int col0, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int row = ks * 32 + 8 * g + q;
    const int col = col0 + 4 * p;
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + tn_off(row, col)));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + tn_off(row + 4, col)));
    typedef short s8 __attribute__((ext_vector_type(8)));
    s8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(typename Mfma<T>::frag, v);
}

// BKT rows x 256 columns (clamped: rows to krows - 1, columns to cols - 8) -> [BKT][512 B] image
template <typename T, int BKT = 64>
__device__ __forceinline__ void stage_tn_big(const T* __restrict__ X, int64_t ldx, int k0, int krows, int col0,
                                             int cols, char* lds, int wave, int lane) {
    constexpr int PW = BKT / 16;  // 1-KiB pieces (2 rows) per wave
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int piece = wave * PW + i;  // BKT / 2 pieces of 2 rows
        const int r = piece * 2 + (lane >> 5);
        const int c = (lane & 31) ^ (2 * tn_sw(r));
        int gr = k0 + r;
        gr = gr < krows ? gr : krows - 1;
        int gc = col0 + c * 8;
        gc = gc + 8 <= cols ? gc : cols - 8;
        __builtin_amdgcn_global_load_lds((const void*)(X + (int64_t)gr * ldx + gc), LDS_PTR(lds + piece * 1024), 16,
                                         0, 0);
    }
}

// BKT-row K-steps in a STAGES-deep ring; a counted vmcnt keeps STAGES - 2 younger K-steps in
// flight across each barrier (BKT 64 / 2 stages: the original one-step-ahead loop).
// one K-step's LDS-DMA: this thread's PW pieces of A and of B (byte offsets va / vb + the step's
// row offset ka / kb), as buffer loads (rows past the buffers' ends read 0)
//
// AD: the LDS-DMA as an asm statement.  The compiler cannot tell a transposed fragment read
// (ds_read_b64_tr_b16 builtin) from the ring slot an LDS-DMA builtin is filling, so with the builtin
// it waits vmcnt(0) before the first fragment read of every K-step: the next K-step's staging never
// overlaps this one's MFMAs.  The asm form is invisible to that analysis; the K-loop's own counted
// wait before each barrier is what orders the ring (the slot read in step kt was filled in step
// kt - 1 and waited for before step kt's barrier; nothing else in the loop touches vmcnt).
template <int PW, int BKT, bool AD = false>
__device__ __forceinline__ void tn_stage_buf(const void* A, uint32_t abytes, const void* B, uint32_t bbytes, char* base,
                                             const uint32_t (&va)[PW], const uint32_t (&vb)[PW], uint32_t ka,
                                             uint32_t kb, int wave) {
#if defined(__HIP_DEVICE_COMPILE__)  // the buffer-resource type exists only for the device target
    const rsrc_t ra = make_rsrc(A, abytes), rb = make_rsrc(B, bbytes);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        if constexpr (AD) {
            // M0 = the wave's 1-KiB LDS piece; one wait state between the M0 write and the DMA
            const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(base + (wave * PW + i) * 1024));
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(la),
                         "v"(va[i] + ka), "s"(ra)
                         : "memory", "m0");
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(la + BKT * 512),
                         "v"(vb[i] + kb), "s"(rb)
                         : "memory", "m0");
        } else {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, LDS_PTR(base + (wave * PW + i) * 1024), 16, va[i] + ka, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, LDS_PTR(base + BKT * 512 + (wave * PW + i) * 1024), 16,
                                                     vb[i] + kb, 0, 0, 0);
        }
    }
#endif
}

// One full 64-token K-step of the 8-wave TN kernel with the transposed fragment reads issued one
// group ahead (a group = the 8 MFMAs of one pair of A fragments; 8 groups per K-step), as
// gemm_nt_pers_kernel's PF K-loop; the fused column sums (CS, do_cs waves) take each A pair right
// after its MFMAs.
template <typename T, typename Cfg, bool CS>
__device__ __forceinline__ void tn_kstep_pf(f32x4 (&acc)[Cfg::NB][Cfg::MB], float (&cs)[Cfg::MB], const char* At,
                                            const char* Bt, int wm, int wn, int lane, bool do_cs) {
    typedef typename Mfma<T>::frag frag;
    frag fb[2][Cfg::NB], fa[4];
    auto rd_b = [&](int ks) {
#pragma unroll
        for (int i = 0; i < Cfg::NB; ++i) fb[ks][i] = tn_frag<T>(Bt, ks, wn * Cfg::WTN + i * 16, lane);
    };
    auto rd_a = [&](int ks, int p) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fa[(2 * p + h) & 3] = tn_frag<T>(At, ks, wm * Cfg::WTM + (2 * p + h) * 16, lane);
    };
    rd_b(0);
    rd_a(0, 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const int ks = g >> 2, p = g & 3;
        if (g + 1 < 8) {
            if (((g + 1) & 3) == 0) rd_b((g + 1) >> 2);
            rd_a((g + 1) >> 2, (g + 1) & 3);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i)
                acc[i][2 * p + h] = Mfma16<T>::mma(fb[ks][i], fa[(2 * p + h) & 3], acc[i][2 * p + h]);
        if (CS && do_cs) {
#pragma unroll
            for (int h = 0; h < 2; ++h) cs[2 * p + h] = frag_sum8(fa[(2 * p + h) & 3], cs[2 * p + h]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// CS: also accumulate the column sums of A over the K range (alpha * sum_k A[k][m] into colsum,
// the bias gradient when A is dY): the tiles in column 0 of the tile grid own them, and of their
// waves the ones with wn == 0 (the other three hold the same A fragments) add their fragments
// with v_dot2c beside the MFMAs -- no separate pass re-reading A from HBM.
//
// NW = 8: 2 x 4 waves of 128 x 64 (two waves per SIMD); NW = 4: 2 x 2 waves of 128 x 128 (one wave
// per SIMD): each transposed fragment read then feeds 8 MFMAs instead of 4 or 8 — 0.5 instead of
// 0.75 LDS reads per MFMA (this pass is LDS-bound).  Its 256 accumulator registers
// live in AGPRs as "+a" operands of inline-asm MFMAs (tn_mfma_row): left to itself, hipcc shuttled
// them between the two files (~300 v_accvgpr copies per 128 MFMAs).
template <typename T, int EPI, int BKT = 64, int STAGES = 2, bool CS = false, int NW = 8, bool PF = false,
          bool AD = false>
__global__ __launch_bounds__(64 * NW, 1) void gemm_tn_big_kernel(const T* __restrict__ A, int64_t lda,
                                                             const T* __restrict__ B, int64_t ldb, int M, int N,
                                                             int Kreal, int k_chunk, int tiles_m, int tiles_n,
                                                             void* __restrict__ C, int64_t ldc, int64_t slab,
                                                             Alpha alpha_arg, float* __restrict__ colsum) {
    const float alpha = alpha_arg.get();
    typedef BigCfg<256, 256, 2, NW / 2, 2> Cfg;
    typedef typename Mfma<T>::frag frag;
    constexpr int STAGE = 2 * BKT * 512;  // A | B
    constexpr int PW = BKT / (2 * NW);    // 1-KiB pieces (2 rows) of each operand per wave per K-step
    constexpr int G = 2 * PW;             // LDS-DMA instructions per thread per K-step
    __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE > Cfg::EP_BYTES ? STAGES * STAGE : Cfg::EP_BYTES];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / (NW / 2), wn = wave % (NW / 2);
    const int lq = lane >> 4;

    // one-dimensional grid over (K split, tile), split-major, in XCD-contiguous ranges: the
    // workgroups that share a split's token rows (every tile of it reads the same K range of both
    // operands) run on one XCD and meet in its L2 (a (tiles, splits) grid spread each split over
    // all eight XCDs: 46 % L2 hits)
    const int ntile = tiles_m * tiles_n;
    const int lin = xcd_remap(blockIdx.x, gridDim.x);
    const int split = lin / ntile;
    const int t = lin - split * ntile;
    const int m0 = (t / tiles_n) * 256;
    const int n0 = (t % tiles_n) * 256;
    const int kbeg = split * k_chunk;
    int nk = k_chunk / BKT;
    if (kbeg + nk * BKT > Kreal) nk = (Kreal - kbeg + BKT - 1) / BKT;  // fully padded tiles skipped
    nk = nk < 0 ? 0 : nk;

    f32x4 acc[Cfg::NB][Cfg::MB];
#pragma unroll
    for (int i = 0; i < Cfg::NB; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool do_cs = CS && t % tiles_n == 0 && wn == 0;  // wave-uniform
    float cs[Cfg::MB];
#pragma unroll
    for (int j = 0; j < Cfg::MB; ++j) cs[j] = 0.f;

    // LDS-DMA sources as buffer loads: a per-lane byte offset of each of this thread's pieces,
    // fixed for the launch, plus the K-step's row offset (one add per piece; the address
    // arithmetic of a pointer per piece cost ~11 VALU instructions, 3 of them 64-bit multiplies,
    // per load, all of them between the barrier and the first MFMA).  Rows past Kreal fall
    // outside the buffer and read 0.
    const uint32_t abytes = (uint32_t)((int64_t)Kreal * lda * sizeof(T));
    const uint32_t bbytes = (uint32_t)((int64_t)Kreal * ldb * sizeof(T));
    uint32_t va[PW], vb[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int r = (wave * PW + i) * 2 + (lane >> 5);
        const int c = (lane & 31) ^ (2 * tn_sw(r));
        const int gca = m0 + c * 8 + 8 <= M ? m0 + c * 8 : M - 8;
        const int gcb = n0 + c * 8 + 8 <= N ? n0 + c * 8 : N - 8;
        va[i] = (uint32_t)(((int64_t)r * lda + gca) * sizeof(T));
        vb[i] = (uint32_t)(((int64_t)r * ldb + gcb) * sizeof(T));
    }
    // (the buffer resources live only inside tn_stage_buf, compiled for the device alone: a template
    // kernel body holding the device-only resource type makes hipcc drop the kernel's host stub)
#define TN_STAGE(KT, SLOT)                                                                                          \
    tn_stage_buf<PW, BKT, AD>(A, abytes, B, bbytes, smem + (SLOT) * STAGE, va, vb,                                  \
                          (uint32_t)((int64_t)(kbeg + (KT) * BKT) * lda * sizeof(T)),                               \
                          (uint32_t)((int64_t)(kbeg + (KT) * BKT) * ldb * sizeof(T)), wave)
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) TN_STAGE(s, s);
    // one K-step; RAGGED (only the last step of the last split can be) masks the token rows past
    // Kreal.  The ragged step is peeled off the loop so the steady-state body has no branch between
    // its fragment reads and its MFMAs.
#define TN_KSTEP(KT, RAGGED)                                                                                        \
    do {                                                                                                            \
        const int kt_ = (KT);                                                                                       \
        if (kt_ + STAGES - 2 <= nk - 1) wait_vmcnt<G * (STAGES - 2)>();                                             \
        else wait_vmcnt<0>();                                                                                       \
        __builtin_amdgcn_s_barrier(); /* K-step kt visible to every wave; the slot of kt - 1 free */               \
        __builtin_amdgcn_sched_barrier(0);                                                                          \
        if (kt_ + STAGES - 1 < nk) TN_STAGE(kt_ + STAGES - 1, (kt_ + STAGES - 1) % STAGES);                         \
        const char* At = smem + (kt_ % STAGES) * STAGE;                                                             \
        const char* Bt = At + BKT * 512;                                                                            \
        const int k0 = kbeg + kt_ * BKT;                                                                            \
        if (PF && NW == 8 && BKT == 64 && !(RAGGED)) {                                                              \
            tn_kstep_pf<T, Cfg, CS>(acc, cs, At, Bt, wm, wn, lane, do_cs);                                          \
        } else                                                                                                      \
        _Pragma("unroll") for (int ks = 0; ks < BKT / 32; ++ks) {                                                   \
            frag fb[Cfg::NB], fa[Cfg::MB];                                                                          \
            _Pragma("unroll") for (int i = 0; i < Cfg::NB; ++i) fb[i] = tn_frag<T>(Bt, ks, wn * Cfg::WTN + i * 16, lane); \
            _Pragma("unroll") for (int j = 0; j < Cfg::MB; ++j) fa[j] = tn_frag<T>(At, ks, wm * Cfg::WTM + j * 16, lane); \
            if (RAGGED) {                                                                                           \
                _Pragma("unroll") for (int j = 0; j < Cfg::MB; ++j)                                                 \
                    _Pragma("unroll") for (int e = 0; e < 8; ++e)                                                   \
                        if (k0 + ks * 32 + 8 * lq + e >= Kreal) fa[j][e] = (T)0.f;                                  \
            }                                                                                                       \
            if (CS && do_cs) {                                                                                      \
                _Pragma("unroll") for (int j = 0; j < Cfg::MB; ++j) cs[j] = frag_sum8(fa[j], cs[j]);               \
            }                                                                                                       \
            if constexpr (NW == 4) {                                                                                \
                _Pragma("unroll") for (int i = 0; i < Cfg::NB; ++i) tn_mfma_row<T>(acc[i], fb[i], fa);               \
            } else {                                                                                                \
                _Pragma("unroll") for (int j = 0; j < Cfg::MB; ++j)                                                 \
                    _Pragma("unroll") for (int i = 0; i < Cfg::NB; ++i) acc[i][j] = Mfma16<T>::mma(fb[i], fa[j], acc[i][j]); \
            }                                                                                                       \
        }                                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                                          \
    } while (0)
    const bool last_ragged = nk > 0 && kbeg + nk * BKT > Kreal;
    const int nfull = last_ragged ? nk - 1 : nk;
    for (int kt = 0; kt < nfull; ++kt) TN_KSTEP(kt, false);
    if (last_ragged) TN_KSTEP(nk - 1, true);
#undef TN_KSTEP
#undef TN_STAGE
    if (CS && do_cs) {  // fragment lane l: column (l & 15), tokens 8 (l >> 4) .. +7 of each 32-row step
#pragma unroll
        for (int j = 0; j < Cfg::MB; ++j) {
            float v = cs[j];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            const int col = m0 + wm * Cfg::WTM + j * 16 + (lane & 15);
            // columns past M: clamped copies.  SPLITK: this split's partial, summed in split order by
            // splitk_reduce_kernel (deterministic); STORE has one split, so one add per column
            if (lq == 0 && col < M) {
                if constexpr (EPI == DCLIP_EPI_SPLITK) colsum[(int64_t)split * M + col] = v * alpha;
                else colsum[col] += v * alpha;
            }
        }
    }
    if constexpr (NW == 4) {
#pragma unroll
        for (int i = 0; i < Cfg::NB; ++i) tn_acc_fence(acc[i], i == 0);
    }
    // the split's slab (blockIdx.y is 0 on this grid, so the epilogue's own slab offset vanishes)
    float* Cs = (float*)C + (EPI == DCLIP_EPI_SPLITK ? (int64_t)split * slab : 0);
    big_epilogue<T, EPI, float, Cfg>(acc, smem, M, N, m0 + wm * Cfg::WTM, n0 + wn * Cfg::WTN, nullptr, nullptr, 0,
                                     Cs, ldc, nullptr, 0, slab, alpha);
}

// per-column sums of a row-major (rows x cols) matrix (f32): a block covers 64 columns (8 lanes
// x 8 columns, 16-byte loads) x a chunk of rows (32 row lanes) and reduces its 32 partial sums
// per column in LDS in a fixed order.  With part, block row z writes part[z][c] (summed in z
// order by the split-K combine); without, one block row adds into out (gridDim.y == 1).  No
// float atomics: the column sums repeat bit for bit run to run.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ x, int64_t ld, int64_t rows, int cols,
                                                     int64_t rows_per_block, Alpha alpha_arg, float* __restrict__ out,
                                                     float* __restrict__ part) {
    const float alpha = alpha_arg.get();
    __shared__ float red[32][65];
    const int cx = threadIdx.x & 7, ry = threadIdx.x >> 3;
    const int c0 = blockIdx.x * 64 + cx * 8;
    const int64_t r0 = blockIdx.y * rows_per_block;
    int64_t r1 = r0 + rows_per_block;
    r1 = r1 < rows ? r1 : rows;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c0 + 8 <= cols) {
        typedef T t8 __attribute__((ext_vector_type(8)));
        int64_t r = r0 + ry;
        // 8 rows per thread in flight (independent 16-byte loads), then the remainder
        for (; r + 7 * 32 < r1; r += 8 * 32) {
            t8 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *(const t8*)(x + (r + 32 * u) * ld + c0);
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int e = 0; e < 8; ++e) s[e] += (float)v[u][e];
        }
        for (; r < r1; r += 32) {
            const t8 v = *(const t8*)(x + r * ld + c0);
#pragma unroll
            for (int e = 0; e < 8; ++e) s[e] += (float)v[e];
        }
    } else {
        for (int64_t r = r0 + ry; r < r1; r += 32)
            for (int e = 0; e < 8 && c0 + e < cols; ++e) s[e] += (float)x[r * ld + c0 + e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[ry][cx * 8 + e] = s[e];
    __syncthreads();
    if (threadIdx.x < 64) {
        float t = 0.f;
        for (int k = 0; k < 32; ++k) t += red[k][threadIdx.x];
        const int c = blockIdx.x * 64 + threadIdx.x;
        if (c < cols) {
            if (part != nullptr) part[(int64_t)blockIdx.y * cols + c] = t * alpha;
            else out[c] += t * alpha;
        }
    }
}

// out[m][n] = sum_z ws[z][m][n] (+ bias[n]) — the split-K combine (deterministic order); with
// cs_part (the fused column sums' per-split partials [splits][M]) also colsum[m] += sum_z cs_part[z][m]
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int64_t slab,
                                     int M, int N, const float* __restrict__ bias,
                                     float* __restrict__ out, int64_t ldo, const float* __restrict__ cs_part = nullptr,
                                     float* __restrict__ colsum = nullptr) {
    const int64_t total4 = (int64_t)M * (N / 4);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / (N / 4));
        const int n = (int)(i % (N / 4)) * 4;
        if (cs_part != nullptr && n == 0) {
            float c = cs_part[m];
            for (int z = 1; z < splits; ++z) c += cs_part[(int64_t)z * M + m];
            colsum[m] += c;
        }
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

// the conv weight gradient's split-K slabs ([co][tap][ci], K = 9 Cin) summed in a fixed order
// and written in torch's (Cout, Cin, 3, 3) layout, times alpha (the 1/s of an fp16 gradient
// scale): one thread per (co, ci), 9 taps each — no permute copy and no separate unscale
__global__ void conv_wgrad_reduce_oihw_kernel(const float* __restrict__ ws, int splits, int64_t slab, int M, int Cin,
                                              Alpha alpha, float* __restrict__ out) {
    const int64_t total = (int64_t)M * Cin;
    const float a = alpha.get();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int co = (int)(i / Cin), ci = (int)(i % Cin);
        const float* src = ws + (int64_t)co * 9 * Cin + ci;
        float v[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) v[t] = src[(int64_t)t * Cin];
        for (int z = 1; z < splits; ++z)
#pragma unroll
            for (int t = 0; t < 9; ++t) v[t] += src[z * slab + (int64_t)t * Cin];
#pragma unroll
        for (int t = 0; t < 9; ++t) out[i * 9 + t] = v[t] * a;
    }
}

// ---------------------------------------------------------------------------- 3x3 convolution
// Implicit-GEMM 3x3 / stride 1 / pad 1 convolution on channels-last pixel rows — the
// ViTFeatureFusionNeck's per-level ConvBNReLU convs (reference models.py:741-745, 13-20) run
// straight on the ViT's token-major read-out: pixel (b, y, x) of a map is the row
//   base + b * bstride + off + (y * W + x) * ld
// (for a token buffer: bstride = N * C, off = C (the CLS row), ld = C), so the NCHW
// materialisation and the NHWC transposes around a library conv disappear.
//   forward: out[m][co] = sum_{tap, ci} in[m + d(tap)][ci] w[co][tap][ci]   (M = B H W pixels)
//   dgrad:   din[m][ci] = sum_{tap, co} dout[m - d(tap)][co] w[co][tap][ci] (the same kernel
//            with dir = -1 and the weights re-laid out as [ci][tap][co])
//   wgrad:   dw[co][tap][ci] = sum_m dout[m][co] in[m + d(tap)][ci]          ("TN", below)
// d(tap) = (tap / 3 - 1, tap % 3 - 1) in (y, x); taps outside the image read a zero row.
// A k-block of 64 channels never straddles two taps (Cin % 64 == 0).
struct PixGeo {
    int64_t bstride, off;  // elements
    int ld, H, W;
};

// p = q * d + r for 0 <= p < 2^24 via a float reciprocal and one correction step each way
__device__ __forceinline__ int fdiv(int p, int d, float inv) {
    int q = (int)((float)p * inv);
    const int r = p - q * d;
    q += (r >= d) - (r < 0);
    return q;
}

// per-lane row (pixel) coordinates of the A rows this lane stages: ROWS_INST rows
template <int ROWS_INST, int BKT>
struct ConvRows {
    int64_t base[ROWS_INST];  // element offset of the pixel
    int y[ROWS_INST], x[ROWS_INST];
};

template <typename T, int ROWS_INST, int BKT>
__device__ __forceinline__ void conv_rows_init(ConvRows<ROWS_INST, BKT>& R, const PixGeo g, int M, int m0, int wave,
                                               int lane) {
    constexpr int CPR = BKT / 8;
    const int HW = g.H * g.W;
    const float invHW = 1.0f / (float)HW, invW = 1.0f / (float)g.W;
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i) {
        const int inst = wave * ROWS_INST + i;
        int m = m0 + inst * (64 / CPR) + lane / CPR;
        m = m < M ? m : M - 1;
        const int b = fdiv(m, HW, invHW);
        const int p = m - b * HW;
        const int y = fdiv(p, g.W, invW);
        R.y[i] = y;
        R.x[i] = p - y * g.W;
        R.base[i] = (int64_t)b * g.bstride + g.off + (int64_t)p * g.ld;
    }
}

template <typename T, int ROWS_INST, int BKT>
__device__ __forceinline__ void stage_conv_rows(const T* __restrict__ X, const T* __restrict__ zero,
                                                const ConvRows<ROWS_INST, BKT>& R, const PixGeo g, int Cin, int dir,
                                                int k0, char* lds, int wave, int lane) {
    constexpr int CPR = BKT / 8;
    const int tap = k0 / Cin, ci = k0 - tap * Cin;  // wave-uniform
    const int dy = (tap / 3 - 1) * dir, dx = (tap % 3 - 1) * dir;
    const int64_t shift = ((int64_t)dy * g.W + dx) * g.ld + ci;
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i) {
        const int inst = wave * ROWS_INST + i;
        const int r = inst * (64 / CPR) + lane / CPR;
        const int c = (lane % CPR) ^ big_sw<BKT>(r);
        const int yy = R.y[i] + dy, xx = R.x[i] + dx;
        const bool ok = yy >= 0 && yy < g.H && xx >= 0 && xx < g.W;
        const T* src = ok ? X + R.base[i] + shift + c * 8 : zero + c * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds + inst * 1024), 16, 0, 0);
    }
}

// stage_conv_rows as buffer loads from X (xbytes bytes from X): a pixel row's byte offset per lane
// (R.base), the tap's shift added per K-step; an out-of-image tap gets an offset past the buffer,
// which reads 0 (no zero row, no 64-bit address arithmetic per load)
template <typename T, int ROWS_INST, int BKT>
__device__ __forceinline__ void stage_conv_rows_buf(const T* X, uint32_t xbytes, const ConvRows<ROWS_INST, BKT>& R,
                                                    const PixGeo g, int Cin, int dir, int k0, char* lds, int wave,
                                                    int lane) {
#if defined(__HIP_DEVICE_COMPILE__)  // the buffer-resource type exists only for the device target
    constexpr int CPR = BKT / 8;
    const rsrc_t rs = make_rsrc(X, xbytes);
    const int tap = k0 / Cin, ci = k0 - tap * Cin;  // wave-uniform
    const int dy = (tap / 3 - 1) * dir, dx = (tap % 3 - 1) * dir;
    const int shift = (int)((((int64_t)dy * g.W + dx) * g.ld + ci) * (int64_t)sizeof(T));
#pragma unroll
    for (int i = 0; i < ROWS_INST; ++i) {
        const int inst = wave * ROWS_INST + i;
        const int r = inst * (64 / CPR) + lane / CPR;
        const int c = (lane % CPR) ^ big_sw<BKT>(r);
        const int yy = R.y[i] + dy, xx = R.x[i] + dx;
        const bool ok = yy >= 0 && yy < g.H && xx >= 0 && xx < g.W;
        const uint32_t voff = ok ? (uint32_t)((int64_t)R.base[i] * (int64_t)sizeof(T) + shift + c * 16) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(lds + inst * 1024), 16, voff, 0, 0, 0);
    }
#endif
}

// out (row-mapped, see big_epilogue) = implicit-GEMM conv; B: weights [Nout][9 * Cin] in (tap, ci) order
template <typename T, int EPI, typename OutT, int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_nt_kernel(
    const T* __restrict__ X, const T* __restrict__ zero, PixGeo g, int Cin, int dir, const T* __restrict__ Bw,
    int64_t ldb, int M, int N, int tiles_m, int tiles_n, const void* __restrict__ aux, int64_t ld_aux,
    void* __restrict__ C, int64_t ldc, int map_hw, int map_gap, int map_off, uint32_t xbytes) {
    constexpr int BKT = 64;
    typedef BigCfg<BM, BN, WM, WN, STAGES, BKT> Cfg;
    typedef typename Mfma<T>::frag frag;
    __shared__ __attribute__((aligned(16))) char smem[Cfg::SMEM];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int l16 = lane & 15, lq = lane >> 4;

    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int m0 = (t / tiles_n) * BM;
    const int n0 = (t % tiles_n) * BN;
    const int nk = 9 * Cin / BKT;

    ConvRows<Cfg::A_INST, BKT> R;
    conv_rows_init<T, Cfg::A_INST, BKT>(R, g, M, m0, wave, lane);
    f32x4 acc[Cfg::NB][Cfg::MB];
#pragma unroll
    for (int i = 0; i < Cfg::NB; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::MB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // buffer-load staging when the input fits 32-bit byte offsets (xbytes > 0); weights always
    uint32_t vb[Cfg::B_INST];
    rows_voff<T, Cfg::B_INST, BKT>(ldb, n0, N, wave, lane, vb);
    const uint32_t bbytes = (uint32_t)((int64_t)N * ldb * sizeof(T));
    auto stage = [&](int kt, int slot) {
        char* base = smem + slot * Cfg::STAGE_BYTES;
        if (xbytes) stage_conv_rows_buf<T, Cfg::A_INST, BKT>(X, xbytes, R, g, Cin, dir, kt * BKT, base, wave, lane);
        else stage_conv_rows<T, Cfg::A_INST, BKT>(X, zero, R, g, Cin, dir, kt * BKT, base, wave, lane);
        stage_rows_buf<T, Cfg::B_INST>(Bw, bbytes, vb, (uint32_t)(kt * BKT * sizeof(T)), base + Cfg::A_BYTES, wave);
    };
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) stage(s, s);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + STAGES - 2 <= nk - 1) wait_vmcnt<Cfg::G * (STAGES - 2)>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
        const char* At = smem + (kt % STAGES) * Cfg::STAGE_BYTES;
        const char* Bt = At + Cfg::A_BYTES;
#pragma unroll
        for (int ks = 0; ks < BKT / 32; ++ks) {
            frag fb[Cfg::NB], fa[Cfg::MB];
            const int ch = ks * 4 + lq;
#pragma unroll
            for (int i = 0; i < Cfg::NB; ++i) fb[i] = big_frag<T, BKT>(Bt, wn * Cfg::WTN + i * 16 + l16, ch);
#pragma unroll
            for (int j = 0; j < Cfg::MB; ++j) fa[j] = big_frag<T, BKT>(At, wm * Cfg::WTM + j * 16 + l16, ch);
#pragma unroll
            for (int j = 0; j < Cfg::MB; ++j)
#pragma unroll
                for (int i = 0; i < Cfg::NB; ++i) acc[i][j] = Mfma16<T>::mma(fb[i], fa[j], acc[i][j]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    big_epilogue<T, EPI, OutT, Cfg>(acc, smem, M, N, m0 + wm * Cfg::WTM, n0 + wn * Cfg::WTN, nullptr, aux, ld_aux, C,
                                     ldc, nullptr, 0, 0, 1.0f, map_hw, map_gap, map_off);
}

// wgrad: dw[n = tap * Cin + ci][co]^T ... computed as C[m = co][n] = sum_p dout[p][co] * in[p + d(tap)][ci]
// with the 128 x 128 "TN" tile (both operands staged as 64 pixel rows x 128 columns; the B
// rows of a tile are the input pixels shifted by the tile's tap, zero rows outside the image).
template <typename T, bool AD = false>
__device__ __forceinline__ void stage_tile_tn_conv(const T* __restrict__ X, const T* __restrict__ zero, const PixGeo g,
                                                   int tap, int ci0, int k0, int krows, char* lds_tile, int wave,
                                                   int lane) {
    const int HW = g.H * g.W;
    const float invHW = 1.0f / (float)HW, invW = 1.0f / (float)g.W;
    const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int inst = wave * 4 + i;
        const int r = inst * 4 + (lane >> 4);
        const int pc = lane & 15;
        const int c = pc ^ ((r & 3) << 2);
        int m = k0 + r;
        const bool in_k = m < krows;
        m = in_k ? m : krows - 1;
        const int b = fdiv(m, HW, invHW);
        const int p = m - b * HW;
        const int y = fdiv(p, g.W, invW);
        const int yy = y + dy, xx = p - y * g.W + dx;
        const bool ok = in_k && yy >= 0 && yy < g.H && xx >= 0 && xx < g.W;
        const T* src = ok ? X + (int64_t)b * g.bstride + g.off + ((int64_t)yy * g.W + xx) * g.ld + ci0 + c * 8
                          : zero + (c & 7) * 8;
        if constexpr (AD) glds16_asm(src, lds_tile + inst * 1024);
        else __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + inst * 1024), 16, 0, 0);
    }
}

// AD: the staging as asm LDS-DMA (glds16_asm) and a bare barrier behind a vmcnt wait at the end of
// each K-step instead of __syncthreads (whose release fence drains the LDS-DMA as well, but the
// compiler's own vmcnt(0) before the first fragment read had already serialised every K-step)
template <typename T, bool AD = false>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(const T* __restrict__ dY, int64_t ldy,
                                                            const T* __restrict__ X, const T* __restrict__ zero,
                                                            PixGeo g, int Cin, int M, int N, int Kpix, int k_chunk,
                                                            int tiles_m, int tiles_n, float* __restrict__ C,
                                                            int64_t slab) {
    __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int m0 = (t / tiles_n) * BM;
    const int n0 = (t % tiles_n) * BN;
    const int tap = n0 / Cin, ci0 = n0 - tap * Cin;  // a tile's 128 columns lie in one tap
    const int kbeg = blockIdx.y * k_chunk;
    int nk = k_chunk / BK;
    if (kbeg + nk * BK > Kpix) nk = (Kpix - kbeg + BK - 1) / BK;
    nk = nk < 0 ? 0 : nk;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    if (nk > 0) {
        stage_tile_tn<T>(dY, ldy, kbeg, Kpix, m0, M, smem, wave, lane);
        stage_tile_tn_conv<T>(X, zero, g, tap, ci0, kbeg, Kpix, smem + TILE_BYTES, wave, lane);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const char* At = smem + cur * STAGE_BYTES;
        const char* Bt = At + TILE_BYTES;
        const int k0 = kbeg + kt * BK;
        if (kt + 1 < nk) {
            char* nxt = smem + (cur ^ 1) * STAGE_BYTES;
            stage_tile_tn<T, AD>(dY, ldy, k0 + BK, Kpix, m0, M, nxt, wave, lane);
            stage_tile_tn_conv<T, AD>(X, zero, g, tap, ci0, k0 + BK, Kpix, nxt + TILE_BYTES, wave, lane);
        }
        // pixel rows past Kpix: the B rows are zero, so the clamped A duplicates add nothing
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            typename Mfma<T>::frag fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = tr_frag_tn<T>(Bt, s, wn * 64 + i * 32, lane);
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = tr_frag_tn<T>(At, s, wm * 64 + j * 32, lane);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = Mfma<T>::mma(fa[i], fb[j], acc[i][j]);
        }
        if constexpr (AD) {  // the next stage landed (this wave's pieces), then everyone's; cur is free
            wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();
        } else {
            __syncthreads();
        }
    }
    if constexpr (AD) __syncthreads();  // the epilogue reuses the ring
    gemm_epilogue<T, DCLIP_EPI_SPLITK, float>(acc, smem, M, N, m0, n0, nullptr, nullptr, 0, C, N, nullptr, 0, slab,
                                               1.0f);
}

// 256 bytes of zeros in device memory: the source of every out-of-image tap
const void* conv_zero_row() {
    static void* z = nullptr;
    if (!z) {
        if (hipMalloc(&z, 256) != hipSuccess) return nullptr;
        if (hipMemset(z, 0, 256) != hipSuccess) return nullptr;
    }
    return z;
}

// grow-only device scratch for the M-tail split (one stream at a time: the library's ops are
// stream-ordered on the caller's stream)
float* tail_scratch(size_t floats) {
    static float* buf = nullptr;
    static size_t cap = 0;
    if (floats > cap) {
        if (buf) (void)hipFree(buf);
        buf = nullptr;
        cap = 0;
        if (hipMalloc(&buf, floats * sizeof(float)) != hipSuccess) return nullptr;
        cap = floats;
    }
    return buf;
}

// sum of the tail's split-K slabs + the GEMM's epilogue for rows m0 + r (r < rows), 8 columns
// per thread
// The M tail of a persistent NT GEMM (M = 256k + mt, mt <= 16: the 8 rows of 8 x 8193 tokens) in
// ONE launch: a workgroup per 64 output columns, its 8 waves each summing a K / 8 slice of the
// 16 x 64 block with 16x16x32 MFMAs on fragments loaded straight from global memory (the mt rows
// of A are read by every workgroup from L2; rows >= mt are zero fragments), the slices added in
// LDS in a fixed order and the epilogue applied per 8-column row segment (epi_row8).  Replaces the
// 256-row split-K tile kernel + combine launch pair (8 + 6 us per GEMM, 97 GEMMs per step).
template <typename T, int EPI, typename OutT>
__global__ __launch_bounds__(512) void gemm_tail16_kernel(const T* __restrict__ A, int64_t lda, const T* __restrict__ B,
                                                          int64_t ldb, int mt, int N, int K, int m0,
                                                          const float* __restrict__ bias, const void* __restrict__ aux,
                                                          int64_t ld_aux, void* __restrict__ C, int64_t ldc,
                                                          void* __restrict__ C2, int64_t ldc2, Alpha alpha_arg) {
    typedef typename Mfma<T>::frag frag;
    __shared__ float red[8][16][68];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, lq = lane >> 4;
    const int n0 = blockIdx.x * 64;
    const int ks = K / 8, kbeg = wave * ks;
    const bool rowok = l16 < mt;
    const T* arow = A + (int64_t)(rowok ? l16 : 0) * lda + kbeg + 8 * lq;
    const T* brow = B + (int64_t)(n0 + l16) * ldb + kbeg + 8 * lq;
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    frag zf;
#pragma unroll
    for (int j = 0; j < 8; ++j) zf[j] = (T)0.f;
#pragma unroll 4
    for (int k = 0; k < ks; k += 32) {
        const frag a = rowok ? *(const frag*)(arow + k) : zf;
        frag b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = *(const frag*)(brow + (int64_t)16 * i * ldb + k);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = Mfma16<T>::mma(a, b[i], acc[i]);  // D[4 lq + e][16 i + l16]
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wave][4 * lq + e][16 * i + l16] = acc[i][e];
    __syncthreads();
    const int t = threadIdx.x;
    if (t < 128) {
        const int r = t >> 3, cb = (t & 7) * 8;
        if (r < mt) {
            const float alpha = alpha_arg.get();
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float sum = 0.f;
#pragma unroll
                for (int w = 0; w < 8; ++w) sum += red[w][r][cb + e];
                v[e] = sum * alpha;
            }
            epi_row8<T, EPI, OutT>(v, m0 + r, n0 + cb, N, bias, aux, ld_aux, C, ldc, C2, ldc2, 0);
        }
    }
}

// The same M tail shaped for latency (round 5, the default): the tail kernel is ~1 % of the step
// (97 launches of 8-15 us) and its time is global-memory round trips, not work.  A workgroup per 16
// output columns (N / 16 workgroups: 48-192, not 12-48), W <= 16 waves each summing a K / W slice of
// IT <= 6 32-deep steps with EVERY fragment load issued before the first MFMA (one round trip
// instead of one per unrolled group of four), and the epilogue's side inputs (bias, column scales,
// residual rows, GELU' pre-activations) loaded at launch by the threads that apply them, so their
// latency hides behind the K loads.  The W slices are added in LDS in wave order (deterministic).
// Needs N % 16 == 0 and W * IT = K / 32 (the launcher picks them).
template <typename T, int EPI, typename OutT>
__global__ __launch_bounds__(1024) void gemm_tail16x16_kernel(const T* __restrict__ A, int64_t lda,
                                                              const T* __restrict__ B, int64_t ldb, int mt, int N,
                                                              int W, int IT, int m0, const float* __restrict__ bias,
                                                              const void* __restrict__ aux, int64_t ld_aux,
                                                              void* __restrict__ C, int64_t ldc, void* __restrict__ C2,
                                                              int64_t ldc2, Alpha alpha_arg) {
    typedef typename Mfma<T>::frag frag;
    constexpr int ITMAX = 6;
    __shared__ float red[16][16][17];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, lq = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int t = threadIdx.x;
    // the epilogue threads (row r, 8-column segment cb) fetch their side inputs first
    const int er = t >> 1, ecb = (t & 1) * 8;
    const bool epi = t < 2 * mt;
    float bv[8], pre[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = pre[e] = 0.f;
    if (epi) {
        const int nb = n0 + ecb;
        if (bias != nullptr && EPI != DCLIP_EPI_GELU_BWD) load8<float>(bias + nb, bv, true, 8);
        if constexpr (EPI == DCLIP_EPI_STORE_SCALED) load8<float>((const float*)aux + nb, pre, true, 8);
        if constexpr (EPI == DCLIP_EPI_RESIDUAL)
            load8<float>((const float*)aux + (int64_t)(m0 + er) * ld_aux + nb, pre, true, 8);
        if constexpr (EPI == DCLIP_EPI_GELU_BWD) load8<T>((const T*)aux + (int64_t)(m0 + er) * ld_aux + nb, pre, true, 8);
    }
    const bool rowok = l16 < mt;
    const int kbeg = wave * IT * 32;
    const T* arow = A + (int64_t)(rowok ? l16 : 0) * lda + kbeg + 8 * lq;
    const T* brow = B + (int64_t)(n0 + l16) * ldb + kbeg + 8 * lq;
    frag zf;
#pragma unroll
    for (int j = 0; j < 8; ++j) zf[j] = (T)0.f;
    frag a[ITMAX], b[ITMAX];
#pragma unroll
    for (int it = 0; it < ITMAX; ++it) {
        if (it < IT) {
            a[it] = rowok ? *(const frag*)(arow + 32 * it) : zf;
            b[it] = *(const frag*)(brow + 32 * it);
        }
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < ITMAX; ++it)
        if (it < IT) acc = Mfma16<T>::mma(a[it], b[it], acc);  // D[4 lq + e][l16]
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave][4 * lq + e][l16] = acc[e];
    __syncthreads();
    if (epi) {
        const float alpha = alpha_arg.get();
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float sum = 0.f;
            for (int w = 0; w < W; ++w) sum += red[w][er][ecb + e];
            v[e] = sum * alpha + bv[e];
        }
        const int64_t m = m0 + er;
        const int nb = n0 + ecb;
        if constexpr (EPI == DCLIP_EPI_STORE) {
            store8<OutT>((OutT*)C + m * ldc + nb, v, true, 8);
        } else if constexpr (EPI == DCLIP_EPI_STORE_SCALED) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= pre[e];
            store8<OutT>((OutT*)C + m * ldc + nb, v, true, 8);
        } else if constexpr (EPI == DCLIP_EPI_GELU) {
            float g[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[e] = (float)(OutT)v[e];  // the activation sees the rounded pre-activation
                g[e] = quick_gelu(v[e]);
            }
            if (C != nullptr) store8<OutT>((OutT*)C + m * ldc + nb, v, true, 8);
            store8<OutT>((OutT*)C2 + m * ldc2 + nb, g, true, 8);
        } else if constexpr (EPI == DCLIP_EPI_RESIDUAL) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += pre[e];
            store8<float>((float*)C + m * ldc + nb, v, true, 8);
            if (C2 != nullptr) store8<T>((T*)C2 + m * ldc2 + nb, v, true, 8);
        } else if constexpr (EPI == DCLIP_EPI_GELU_BWD) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= quick_gelu_grad(pre[e]);
            store8<OutT>((OutT*)C + m * ldc + nb, v, true, 8);
        }
    }
}

// (W, IT) of gemm_tail16x16_kernel for K: the most waves (<= 16) whose slices are <= 6 steps of 32
inline bool tail16x16_plan(int64_t K, int& W, int& IT) {
    if (K % 32 != 0) return false;
    const int s = (int)(K / 32);
    for (int w = 16; w >= 1; --w)
        if (s % w == 0 && s / w <= 6) {
            W = w;
            IT = s / w;
            return true;
        }
    return false;
}

template <typename T, int EPI, typename OutT>
__global__ void tail_combine_kernel(const float* __restrict__ ws, int splits, int rows, int N, int64_t m0,
                                    const float* __restrict__ bias, const void* __restrict__ aux, int64_t ld_aux,
                                    void* __restrict__ C, int64_t ldc, void* __restrict__ C2, int64_t ldc2) {
    const int n8 = (N + 7) / 8;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * n8) return;
    const int r = i / n8, nb = (i % n8) * 8;
    const bool full = nb + 8 <= N;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < splits; ++sp) {
        float t[8];
        load8<float>(ws + ((int64_t)sp * rows + r) * N + nb, t, full, N - nb);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    epi_row8<T, EPI, OutT>(v, (int)(m0 + r), nb, N, bias, aux, ld_aux, C, ldc, C2, ldc2, 0);
}

template <typename T, int EPI, typename OutT, int TBM, int TBN, int WM, int WN, int STAGES, int BKT = 64,
          bool PP = false>
void launch_big(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                int splits, Alpha alpha, const float* bias, const void* aux, int64_t ld_aux, void* C, int64_t ldc,
                void* C2, int64_t ldc2, hipStream_t st) {
    int tiles_m = (int)((M + TBM - 1) / TBM);
    const int tiles_n = (int)((N + TBN - 1) / TBN);
    // M-tail split: the token GEMMs have M = B*(1 + HW) = 256k + B rows, so the last, nearly
    // empty row of tiles adds a whole extra round of workgroups (e.g. 771 tiles on 256 CUs).
    // When it does, the full row tiles run here and the tail rows as K-split slabs over many
    // workgroups plus a combine that applies the epilogue.
    const int64_t Mfull = (M / TBM) * TBM, tail = M - Mfull;
    auto rounds = [](int64_t t) { return (t + 255) / 256; };
    // Only for long K: the tail launch + combine cost ~20-30 us, about one round of a K = 768
    // tile (measured: no gain there), against ~80 us for a round at K = 3072.
    if (EPI != DCLIP_EPI_SPLITK && splits == 1 && tail > 0 && tail <= 64 && Mfull > 0 && K >= 1536 &&
        rounds((int64_t)tiles_m * tiles_n) > rounds((Mfull / TBM) * tiles_n)) {
        const int ksteps = (int)(K / BKT);
        int ts = 1;
        for (int c = 16; c >= 1; --c)
            if (ksteps % c == 0) {
                ts = c;
                break;
            }
        float* ws = tail_scratch((size_t)ts * tail * N);
        if (ws != nullptr) {
            tiles_m = (int)(Mfull / TBM);
            const int ttm = 1;
            gemm_nt_big_kernel<T, DCLIP_EPI_SPLITK, float, TBM, TBN, WM, WN, STAGES, BKT>
                <<<dim3(ttm * tiles_n, ts), 64 * WM * WN, 0, st>>>(
                    (const T*)A + Mfull * lda, lda, (const T*)B, ldb, (int)tail, (int)N, (int)(K / ts), ttm, tiles_n,
                    nullptr, nullptr, 0, ws, N, nullptr, 0, tail * N, alpha);
            const int threads = (int)(tail * ((N + 7) / 8));
            tail_combine_kernel<T, EPI, OutT><<<(threads + 255) / 256, 256, 0, st>>>(
                ws, ts, (int)tail, (int)N, Mfull, bias, aux, ld_aux, C, ldc, C2, ldc2);
            M = Mfull;
        }
    }
    dim3 grid(tiles_m * tiles_n, splits);
    if constexpr (PP) {
        static_assert(TBM == 256 && TBN == 256 && WM == 2 && WN == 4, "ping-pong geometry");
        gemm_nt_pp_kernel<T, EPI, OutT><<<grid, 512, 0, st>>>(
            (const T*)A, lda, (const T*)B, ldb, (int)M, (int)N, (int)(K / splits), tiles_m, tiles_n, bias, aux, ld_aux,
            C, ldc, C2, ldc2, (int64_t)M * N, alpha);
    } else {
        gemm_nt_big_kernel<T, EPI, OutT, TBM, TBN, WM, WN, STAGES, BKT><<<grid, 64 * WM * WN, 0, st>>>(
            (const T*)A, lda, (const T*)B, ldb, (int)M, (int)N, (int)(K / splits), tiles_m, tiles_n, bias, aux,
            ld_aux, C, ldc, C2, ldc2, (int64_t)M * N, alpha);
    }
}

// persistent path (gemm_nt_pers_kernel) for the full 256-row tiles; an M tail of <= 64 rows by
// K-split slabs + an epilogue-applying combine.  Returns false when the shape does not fit it.
int cu_count() {
    static int n[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return 256;
    if (n[dev] == 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        n[dev] = c;
    }
    return n[dev];
}

// the persistent GEMM's tile-claim counters (gemm_nt_pers_kernel DYN): one zeroed set of 512 words per
// stream per device, so launches that may run concurrently (different streams) never share one; a
// launch on a capturing stream (a graph replay may run beside eager work on that stream) or past
// the 64 sets of a device takes the static walk (null)
unsigned* gemm_sched_counters(hipStream_t st) {
    static std::mutex mu;
    static unsigned* base[64] = {nullptr};
    static hipStream_t owner[64][64];
    static int used[64] = {0};
    if (dclip_option(DCLIP_OPT_GEMM_SCHED) != 1) return nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    if (base[dev] == nullptr) {
        unsigned* p = nullptr;
        const size_t bytes = 64 * 512 * sizeof(unsigned);
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        if (hipMemset(p, 0, bytes) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        base[dev] = p;
    }
    for (int i = 0; i < used[dev]; ++i)
        if (owner[dev][i] == st) return base[dev] + 512 * i;
    if (used[dev] == 64) return nullptr;
    owner[dev][used[dev]] = st;
    return base[dev] + 512 * used[dev]++;
}

// Streaming (nontemporal) epilogue stores for the wide forward outputs (qkv, the MLP's z / h:
// N >= 2048): they leave L2 to the operands the K-loop re-reads (B, the weight, by every row of
// tiles; A by the N / 256 column tiles of a row) instead of evicting them — qkv -11 %, c_fc -14 %
// per call, the 7-GEMM set -4.2 %, the step -0.2 % (bf16 and fp16; profiles/r05/r5p: the consumers
// read them from HBM rather than the Infinity Cache, which takes back most of it).  The residual
// stream (read by the LayerNorm right after), the narrow dX outputs and the GELU' epilogue (which
// reads its pre-activations beside the stores) measured equal or slower and keep plain stores.
// DCLIP_OPT_GEMM_EPI: 0 this rule, 2 always, 3 never.
inline bool pers_streaming_stores(int epi, int64_t N) {
    const int o = dclip_option(DCLIP_OPT_GEMM_EPI);
    if (o == 2) return true;
    if (o != 0) return false;
    return N >= 2048 && epi != DCLIP_EPI_GELU_BWD && epi != DCLIP_EPI_RESIDUAL;
}

// The K-loop with the fragment reads one group ahead (gemm_nt_pers_kernel PF) on every epilogue but
// GELU: c_proj -6 %, the dX GEMMs -3..-6 %, out_proj -4 %, qkv -1 %, but the MLP-up GEMM with the
// GELU epilogue +3 % (profiles/r05/r5u).  DCLIP_OPT_GEMM_KLOOP: 0 this rule, 1 every NT and TN
// 8-wave K-loop (the TN kernel measured 1-5 % slower with it), 2 none.
inline bool pers_prefetch_kloop(int epi) {
    const int o = dclip_option(DCLIP_OPT_GEMM_KLOOP);
    if (o == 1) return true;
    if (o != 0) return false;
    return epi != DCLIP_EPI_GELU;
}

template <typename T, int EPI, typename OutT, int NW = 8, bool PIPE = false>
bool launch_pers(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
                 Alpha alpha, const float* bias, const void* aux, int64_t ld_aux, void* C, int64_t ldc, void* C2,
                 int64_t ldc2, hipStream_t st) {
    if constexpr (EPI == DCLIP_EPI_SPLITK) {
        return false;
    } else {
        const int64_t Mfull = (M / 256) * 256, tail = M - Mfull;
        const int G = cu_count();
        if (N % 256 != 0 || tail > 64 || (Mfull / 256) * (N / 256) < 2 * G) return false;
        if (PIPE && K < 128) return false;
        // buffer-load staging addresses each operand with 32-bit byte offsets
        if (Mfull * lda * (int64_t)sizeof(T) >= (1ll << 32) || N * ldb * (int64_t)sizeof(T) >= (1ll << 32)) return false;
        if (EPI == DCLIP_EPI_STORE_SCALED || (bias != nullptr && EPI != DCLIP_EPI_GELU_BWD)) {
            // 16-byte per-column vector loads
            if (((uintptr_t)(EPI == DCLIP_EPI_STORE_SCALED ? aux : bias) % 16) != 0) return false;
            if (bias != nullptr && ((uintptr_t)bias % 16) != 0) return false;
        }
        if (ldc % 4 != 0 || (C2 != nullptr && ldc2 % 4 != 0) || (EPI == DCLIP_EPI_RESIDUAL && ld_aux % 4 != 0) ||
            (EPI == DCLIP_EPI_GELU_BWD && ld_aux % 4 != 0))
            return false;
        const int tail_opt = dclip_option(DCLIP_OPT_GEMM_TAIL);
        int tw = 0, tit = 0;
        if (tail > 0 && tail <= 16 && tail_opt == 0 && tail16x16_plan(K, tw, tit)) {
            gemm_tail16x16_kernel<T, EPI, OutT><<<(unsigned)(N / 16), 64 * tw, 0, st>>>(
                (const T*)A + Mfull * lda, lda, (const T*)B, ldb, (int)tail, (int)N, tw, tit, (int)Mfull, bias, aux,
                ld_aux, C, ldc, C2, ldc2, alpha);
        } else if (tail > 0 && tail <= 16 && K % 256 == 0 && tail_opt != 1) {
            gemm_tail16_kernel<T, EPI, OutT><<<(unsigned)(N / 64), 512, 0, st>>>(
                (const T*)A + Mfull * lda, lda, (const T*)B, ldb, (int)tail, (int)N, (int)K, (int)Mfull, bias, aux,
                ld_aux, C, ldc, C2, ldc2, alpha);
        } else if (tail > 0) {
            const int tiles_n = (int)(N / 256);
            const int ksteps = (int)(K / 64);
            int ts = 1;
            for (int c = 16; c >= 1; --c)
                if (ksteps % c == 0) {
                    ts = c;
                    break;
                }
            float* ws = tail_scratch((size_t)ts * tail * N);
            if (ws == nullptr) return false;
            gemm_nt_big_kernel<T, DCLIP_EPI_SPLITK, float, 256, 256, 2, 4, 2, 64>
                <<<dim3(tiles_n, ts), 512, 0, st>>>((const T*)A + Mfull * lda, lda, (const T*)B, ldb, (int)tail, (int)N,
                                                    (int)(K / ts), 1, tiles_n, nullptr, nullptr, 0, ws, N, nullptr, 0,
                                                    tail * N, alpha);
            const int threads = (int)(tail * ((N + 7) / 8));
            tail_combine_kernel<T, EPI, OutT><<<(threads + 255) / 256, 256, 0, st>>>(
                ws, ts, (int)tail, (int)N, Mfull, bias, aux, ld_aux, C, ldc, C2, ldc2);
        }
        if constexpr (PIPE)
            gemm_nt_pipe_kernel<T, EPI, OutT, NW><<<G, 64 * NW, 0, st>>>((const T*)A, lda, (const T*)B, ldb, (int)K,
                                                                         (int)(Mfull / 256), (int)(N / 256), bias, aux,
                                                                         ld_aux, C, ldc, C2, ldc2, alpha);
        else
        {
            // the row-major LDS epilogue (default) or, DCLIP_OPT_GEMM_EPI 1, the accumulator-layout stores
            // (launch_pers runs only with >= 2 G full tiles; the round-0 bitmap holds up to 256 workgroups)
            unsigned* sched = (NW == 8 && dclip_option(DCLIP_OPT_GEMM_EPI) != 1 && K >= 128 && G <= 256)
                                  ? gemm_sched_counters(st)
                                  : nullptr;
            if (sched != nullptr)  // work-conserving: tiles past round 0 claimed (default)
                gemm_nt_pers_kernel<T, EPI, OutT, NW, true, NW == 8><<<G, 64 * NW, 0, st>>>(
                    (const T*)A, lda, (const T*)B, ldb, (int)K, (int)(Mfull / 256), (int)(N / 256), bias, aux, ld_aux, C,
                    ldc, C2, ldc2, alpha, sched);
#define PERS_LAUNCH(NTS_, PF_)                                                                                  \
    gemm_nt_pers_kernel<T, EPI, OutT, NW, true, false, NTS_, PF_><<<G, 64 * NW, 0, st>>>(                        \
        (const T*)A, lda, (const T*)B, ldb, (int)K, (int)(Mfull / 256), (int)(N / 256), bias, aux, ld_aux, C, ldc, C2, \
        ldc2, alpha)
            else if (NW == 8 && dclip_option(DCLIP_OPT_GEMM_EPI) != 1) {
                const bool nts = pers_streaming_stores(EPI, N), pf = pers_prefetch_kloop(EPI);
                if (nts && pf) PERS_LAUNCH(true, true);
                else if (nts) PERS_LAUNCH(true, false);
                else if (pf) PERS_LAUNCH(false, true);
                else PERS_LAUNCH(false, false);
            }
#undef PERS_LAUNCH
            else
                gemm_nt_pers_kernel<T, EPI, OutT, NW, false><<<G, 64 * NW, 0, st>>>(
                    (const T*)A, lda, (const T*)B, ldb, (int)K, (int)(Mfull / 256), (int)(N / 256), bias, aux, ld_aux, C,
                    ldc, C2, ldc2, alpha);
        }
        return true;
    }
}

// tile configuration: DCLIP_OPT_GEMM_TILE 1 = 128x128 (4 waves, 2 workgroups/CU), 2 = 256x256
// (8 waves, 2-stage ring of 64-deep k-tiles), 3 = 256x128 (8 waves, 3-stage ring),
// 4 = 256x256 with a 4-stage ring of 32-deep k-tiles, 5 = 256x256 ping-pong (gemm_nt_pp_kernel),
// 6 = persistent 256x256 (gemm_nt_pers_kernel) where the shape allows it, 7 = the same with 4
// waves of 128x128, 8 / 9 = the persistent kernel with pipelined fragment reads
// (gemm_nt_pipe_kernel) with 8 / 4 waves, 0 = automatic
inline int gemm_tile_choice(int64_t M, int64_t N) {
    const int opt = dclip_option(DCLIP_OPT_GEMM_TILE);
    if (opt != 0) return opt;
    if (M < 4096) return 1;
    return 6;  // persistent where the shape allows it (falls back to the 256x256 grid kernel)
}

template <typename T, int EPI, typename OutT>
int launch(const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
           int splits, Alpha alpha, const float* bias, const void* aux, int64_t ld_aux, void* C, int64_t ldc,
           void* C2, int64_t ldc2, hipStream_t st) {
    const int choice = gemm_tile_choice(M, N);
    if (choice == 2) {
        launch_big<T, EPI, OutT, 256, 256, 2, 4, 2>(A, lda, B, ldb, M, N, K, splits, alpha, bias, aux, ld_aux, C,
                                                    ldc, C2, ldc2, st);
        return 0;
    }
    if (choice == 3) {
        launch_big<T, EPI, OutT, 256, 128, 4, 2, 3>(A, lda, B, ldb, M, N, K, splits, alpha, bias, aux, ld_aux, C,
                                                    ldc, C2, ldc2, st);
        return 0;
    }
    if (choice == 6 && splits == 1 &&
        launch_pers<T, EPI, OutT>(A, lda, B, ldb, M, N, K, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st))
        return 0;
    if (choice == 7 && splits == 1 &&
        launch_pers<T, EPI, OutT, 4>(A, lda, B, ldb, M, N, K, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st))
        return 0;
    if (choice == 8 && splits == 1 &&
        launch_pers<T, EPI, OutT, 8, true>(A, lda, B, ldb, M, N, K, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st))
        return 0;
    if (choice == 9 && splits == 1 &&
        launch_pers<T, EPI, OutT, 4, true>(A, lda, B, ldb, M, N, K, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st))
        return 0;
    if (choice >= 6) {
        launch_big<T, EPI, OutT, 256, 256, 2, 4, 2>(A, lda, B, ldb, M, N, K, splits, alpha, bias, aux, ld_aux, C,
                                                    ldc, C2, ldc2, st);
        return 0;
    }
    if (choice == 5) {
        launch_big<T, EPI, OutT, 256, 256, 2, 4, 2, 64, true>(A, lda, B, ldb, M, N, K, splits, alpha, bias, aux,
                                                              ld_aux, C, ldc, C2, ldc2, st);
        return 0;
    }
    if (choice == 4) {
        launch_big<T, EPI, OutT, 256, 256, 2, 4, 4, 32>(A, lda, B, ldb, M, N, K, splits, alpha, bias, aux, ld_aux, C,
                                                        ldc, C2, ldc2, st);
        return 0;
    }
    const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
    const int k_chunk = (int)(K / splits);
    dim3 grid(tiles_m * tiles_n, splits);
    gemm_nt_kernel<T, EPI, OutT><<<grid, 256, 0, st>>>(
        (const T*)A, lda, (const T*)B, ldb, (int)M, (int)N, k_chunk, tiles_m, tiles_n, bias, aux,
        ld_aux, C, ldc, C2, ldc2, (int64_t)M * N, alpha);
    return 0;
}

template <typename T>
int dispatch(int epi, int c_dt, const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M,
             int64_t N, int64_t K, int splits, Alpha alpha, const float* bias, const void* aux, int64_t ld_aux,
             void* C, int64_t ldc, void* C2, int64_t ldc2, hipStream_t st) {
    switch (epi) {
        case DCLIP_EPI_STORE:
            if (c_dt == DCLIP_F32)
                return launch<T, DCLIP_EPI_STORE, float>(A, lda, B, ldb, M, N, K, 1, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
            return launch<T, DCLIP_EPI_STORE, T>(A, lda, B, ldb, M, N, K, 1, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_STORE_SCALED:
            return launch<T, DCLIP_EPI_STORE_SCALED, T>(A, lda, B, ldb, M, N, K, 1, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_GELU:
            return launch<T, DCLIP_EPI_GELU, T>(A, lda, B, ldb, M, N, K, 1, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_RESIDUAL:
            return launch<T, DCLIP_EPI_RESIDUAL, float>(A, lda, B, ldb, M, N, K, 1, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_GELU_BWD:
            return launch<T, DCLIP_EPI_GELU_BWD, T>(A, lda, B, ldb, M, N, K, 1, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
        case DCLIP_EPI_SPLITK: {
            // partial slabs in the caller's workspace (aux), then one combine pass
            float* ws = (float*)const_cast<void*>(aux);
            launch<T, DCLIP_EPI_SPLITK, float>(A, lda, B, ldb, M, N, K, splits, alpha, nullptr, nullptr, 0,
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
                          int64_t ldb, int64_t M, int64_t N, int64_t K, int splits, float alpha_v, const float* alpha_ptr,
                          const float* bias, const void* aux, int aux_dt, int64_t ld_aux, void* C,
                          int c_dt, int64_t ldc, void* C2, int64_t ldc2, void* stream) {
    const Alpha alpha(alpha_v, alpha_ptr);
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
        case DCLIP_EPI_STORE_SCALED:
            DCLIP_HOST_CHECK(c_dt == ab_dt && aux != nullptr && aux_dt == DCLIP_F32,
                             "dclip_gemm: STORE_SCALED needs an f32 per-column scale vector in aux and C of the operand dtype");
            break;
        case DCLIP_EPI_GELU:
            DCLIP_HOST_CHECK(c_dt == ab_dt && C2 != nullptr,
                             "dclip_gemm: GELU needs C2 (and C, when z is wanted) of the operand dtype");
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
                 ? dispatch<bf16>(epilogue, c_dt, A, lda, B, ldb, M, N, K, splits, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st)
                 : dispatch<f16>(epilogue, c_dt, A, lda, B, ldb, M, N, K, splits, alpha, bias, aux, ld_aux, C, ldc, C2, ldc2, st);
    if (rc) return rc;
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// K-split plan of dclip_gemm_tn: minimise (rounds of resident workgroups x k-rows per split) x
// tile time + the f32 partial-slab round trip through HBM (write + combine read), with at
// least 4 64-row k-tiles per split.  Slots: 256 CUs x 1 workgroup (256x256 kernel) or x 2
// (128x128); tile time at ~5 TFLOP/s per CU, slabs at ~5 TB/s.
extern "C" int dclip_gemm_tn_plan(int64_t M, int64_t N, int64_t K, int* splits_out, int64_t* k_pad_out) {
    DCLIP_HOST_CHECK(M > 0 && N > 0 && K > 0 && splits_out && k_pad_out, "dclip_gemm_tn_plan: bad arguments");
    const bool big = dclip_option(DCLIP_OPT_GEMM_TN_TILE) != 1 && M >= 256 && N >= 256;
    const int64_t tile = big ? 256 : 128;
    const int64_t tiles = ((M + tile - 1) / tile) * ((N + tile - 1) / tile);
    const int64_t slots = big ? 256 : 512;
    int best = 1;
    double best_t = 1e30;
    for (int sp = 1; sp <= 32; ++sp) {
        if (sp > 1 && K < 64 * 4 * (int64_t)sp) break;
        const int64_t blocks = tiles * sp;
        const double rounds = (double)((blocks + slots - 1) / slots);
        const double krows = (double)((K + 64 * sp - 1) / (64 * sp) * 64);
        const double t = rounds * krows * (2.0 * tile * tile / 5e12) + (sp > 1 ? sp * 8.0 * M * N / 5e12 : 0.0);
        if (t < best_t * 0.98) {
            best = sp;
            best_t = t;
        }
    }
    *splits_out = best;
    *k_pad_out = ((K + 64 * best - 1) / (64 * best)) * 64 * best;
    return 0;
}

extern "C" int dclip_gemm_tn(int epilogue, int ab_dt, const void* A, int64_t lda, const void* B, int64_t ldb,
                             int64_t M, int64_t N, int64_t K, int64_t K_pad, int splits, float alpha_v, const float* alpha_ptr, const float* bias,
                             void* ws, void* C, int64_t ldc, float* colsum_a, void* stream) {
    const Alpha alpha(alpha_v, alpha_ptr);
    DCLIP_HOST_CHECK(ab_dt == DCLIP_BF16 || ab_dt == DCLIP_F16, "dclip_gemm_tn: operands must be f16/bf16");
    DCLIP_HOST_CHECK(M > 0 && N > 0 && K > 0 && M % 8 == 0 && N % 8 == 0,
                     "dclip_gemm_tn: M, N must be positive multiples of 8 (M=%lld N=%lld)", (long long)M, (long long)N);
    DCLIP_HOST_CHECK(splits >= 1 && K_pad >= K && K_pad % (BK * splits) == 0,
                     "dclip_gemm_tn: K_pad must be >= K and a multiple of 64*splits");
    DCLIP_HOST_CHECK(lda >= M && ldb >= N && lda % 8 == 0 && ldb % 8 == 0, "dclip_gemm_tn: bad leading dims");
    DCLIP_HOST_CHECK(((uintptr_t)A % 16) == 0 && ((uintptr_t)B % 16) == 0, "dclip_gemm_tn: A/B must be 16-byte aligned");
    DCLIP_HOST_CHECK(epilogue == DCLIP_EPI_STORE || epilogue == DCLIP_EPI_SPLITK,
                     "dclip_gemm_tn: epilogue must be STORE or SPLITK (f32 output)");
    DCLIP_HOST_CHECK(epilogue == DCLIP_EPI_STORE ? splits == 1 : ws != nullptr,
                     "dclip_gemm_tn: STORE needs splits == 1; SPLITK needs a workspace of splits*(M*N + M) f32");
    DCLIP_HOST_CHECK(ldc % 4 == 0, "dclip_gemm_tn: ldc %% 4 != 0");
    DCLIP_HOST_CHECK(K * lda * 2 < (1ll << 32) && K * ldb * 2 < (1ll << 32),
                     "dclip_gemm_tn: operands must stay below 4 GiB (buffer-load staging)");
    hipStream_t st = (hipStream_t)stream;
    const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
    const int k_chunk = (int)(K_pad / splits);
    dim3 grid(tiles_m * tiles_n, splits);
    const int tn_opt = dclip_option(DCLIP_OPT_GEMM_TN_TILE);
    const bool tn_pf = dclip_option(DCLIP_OPT_GEMM_KLOOP) == 1;
    const bool big = tn_opt != 1 && M >= 256 && N >= 256;
    // the big kernel sums A's columns itself (DCLIP_OPT_GEMM_TN_COLSUM 1: the separate pass)
    const bool fused_cs = colsum_a && big && dclip_option(DCLIP_OPT_GEMM_TN_COLSUM) != 1;
    // the separate column-sum pass: per-split partials into ws's column-sum region (summed in
    // split order by the combine), or, for STORE (splits == 1), one block row over all K
    float* cs_sep = (colsum_a && !fused_cs && epilogue == DCLIP_EPI_SPLITK) ? (float*)ws + (int64_t)splits * M * N
                                                                           : nullptr;
    if (colsum_a && !fused_cs) {
        const int64_t rpb = cs_sep != nullptr ? K_pad / splits : K;
        dim3 cg((unsigned)((M + 63) / 64), (unsigned)(cs_sep != nullptr ? splits : 1));
        if (ab_dt == DCLIP_BF16)
            colsum_kernel<bf16><<<cg, 256, 0, st>>>((const bf16*)A, lda, K, (int)M, rpb, alpha, colsum_a, cs_sep);
        else colsum_kernel<f16><<<cg, 256, 0, st>>>((const f16*)A, lda, K, (int)M, rpb, alpha, colsum_a, cs_sep);
    }
#define TN_LAUNCH_V(T, EPI, OUT, AD)                                                                              \
    gemm_tn_kernel<T, EPI, float, AD><<<grid, 256, 0, st>>>((const T*)A, lda, (const T*)B, ldb, (int)M, (int)N,    \
                                                            (int)K, k_chunk, tiles_m, tiles_n, nullptr, OUT,         \
                                                            EPI == DCLIP_EPI_SPLITK ? N : ldc, (int64_t)M * N, alpha)
#define TN_LAUNCH(T, EPI, OUT)                                                                                    \
    do {                                                                                                          \
        if (tn_opt == 5) TN_LAUNCH_V(T, EPI, OUT, false);                                                         \
        else TN_LAUNCH_V(T, EPI, OUT, true);                                                                      \
    } while (0)
#define TN_BIG_V(T, EPI, OUT, BKT, STG, CS, NW, ...)                                                           \
    gemm_tn_big_kernel<T, EPI, BKT, STG, CS, NW, ##__VA_ARGS__><<<dim3(tm2 * tn2 * splits), 64 * NW, 0, st>>>( \
        (const T*)A, lda, (const T*)B, ldb, (int)M, (int)N, (int)K, k_chunk, tm2, tn2, OUT,                     \
        EPI == DCLIP_EPI_SPLITK ? N : ldc, (int64_t)M * N, alpha, EPI == DCLIP_EPI_SPLITK ? cs_part : colsum_a)
#define TN_BIG(T, EPI, OUT)                                                                                    \
    do {                                                                                                       \
        if (tn_opt == 2) TN_BIG_V(T, EPI, OUT, 32, 4, false, 8);                                               \
        else if (tn_opt == 3) TN_BIG_V(T, EPI, OUT, 32, 5, false, 8);                                          \
        else if (tn_opt == 4 && fused_cs) TN_BIG_V(T, EPI, OUT, 64, 2, true, 4);                               \
        else if (tn_opt == 4) TN_BIG_V(T, EPI, OUT, 64, 2, false, 4);                                          \
        else if (tn_opt == 5 && fused_cs) TN_BIG_V(T, EPI, OUT, 64, 2, true, 8);                               \
        else if (tn_opt == 5) TN_BIG_V(T, EPI, OUT, 64, 2, false, 8);                                          \
        else if (fused_cs && tn_pf) TN_BIG_V(T, EPI, OUT, 64, 2, true, 8, true, true);                         \
        else if (tn_pf) TN_BIG_V(T, EPI, OUT, 64, 2, false, 8, true, true);                                    \
        else if (fused_cs) TN_BIG_V(T, EPI, OUT, 64, 2, true, 8, false, true);                                 \
        else TN_BIG_V(T, EPI, OUT, 64, 2, false, 8, false, true);                                              \
    } while (0)
    const int tm2 = (int)((M + 255) / 256), tn2 = (int)((N + 255) / 256);
    // the fused column sums' per-split partials, past the slabs (SPLITK): summed in split order
    float* cs_part = (fused_cs && epilogue == DCLIP_EPI_SPLITK) ? (float*)ws + (int64_t)splits * M * N : cs_sep;
    if (epilogue == DCLIP_EPI_STORE) {
        DCLIP_HOST_CHECK(bias == nullptr, "dclip_gemm_tn: bias only with SPLITK");
        if (big) {
            if (ab_dt == DCLIP_BF16) TN_BIG(bf16, DCLIP_EPI_STORE, C);
            else TN_BIG(f16, DCLIP_EPI_STORE, C);
        } else {
            if (ab_dt == DCLIP_BF16) TN_LAUNCH(bf16, DCLIP_EPI_STORE, C);
            else TN_LAUNCH(f16, DCLIP_EPI_STORE, C);
        }
    } else {
        if (big) {
            if (ab_dt == DCLIP_BF16) TN_BIG(bf16, DCLIP_EPI_SPLITK, ws);
            else TN_BIG(f16, DCLIP_EPI_SPLITK, ws);
        } else {
            if (ab_dt == DCLIP_BF16) TN_LAUNCH(bf16, DCLIP_EPI_SPLITK, ws);
            else TN_LAUNCH(f16, DCLIP_EPI_SPLITK, ws);
        }
        const int64_t total4 = M * (N / 4);
        int blocks = (int)((total4 + 255) / 256);
        blocks = blocks > 4096 ? 4096 : blocks;
        splitk_reduce_kernel<<<blocks, 256, 0, st>>>((const float*)ws, splits, M * N, (int)M, (int)N, bias,
                                                     (float*)C, ldc, cs_part, colsum_a);
    }
#undef TN_LAUNCH
#undef TN_LAUNCH_V
#undef TN_BIG
#undef TN_BIG_V
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------- conv ABI
extern "C" int dclip_conv3x3(int mode, int ab_dt, const void* X, int64_t x_bstride, int64_t x_off, int64_t x_ld,
                             int B, int H, int W, int Cin, const void* Wt, int Nout, void* out, int out_dt,
                             int64_t out_ld, int out_gap, int out_off, int accumulate, void* stream) {
    DCLIP_HOST_CHECK(ab_dt == DCLIP_BF16 || ab_dt == DCLIP_F16, "dclip_conv3x3: operands must be f16/bf16");
    DCLIP_HOST_CHECK(mode == 0 || mode == 1, "dclip_conv3x3: mode 0 (forward) or 1 (input gradient)");
    DCLIP_HOST_CHECK(B > 0 && H > 0 && W > 0 && Cin > 0 && Nout > 0 && Cin % 64 == 0 && Nout % 8 == 0,
                     "dclip_conv3x3: Cin %% 64 == 0 and Nout %% 8 == 0 required (Cin=%d Nout=%d)", Cin, Nout);
    DCLIP_HOST_CHECK((int64_t)B * H * W < (1ll << 24), "dclip_conv3x3: too many pixels");
    DCLIP_HOST_CHECK(x_ld % 8 == 0 && x_bstride % 8 == 0 && x_off % 8 == 0 && x_ld >= Cin,
                     "dclip_conv3x3: input strides must be multiples of 8 elements");
    DCLIP_HOST_CHECK(((uintptr_t)X % 16) == 0 && ((uintptr_t)Wt % 16) == 0, "dclip_conv3x3: unaligned operands");
    DCLIP_HOST_CHECK(out_dt == ab_dt || out_dt == DCLIP_F32, "dclip_conv3x3: output must be f32 or the operand dtype");
    DCLIP_HOST_CHECK(!accumulate || out_dt == DCLIP_F32, "dclip_conv3x3: accumulate needs an f32 output");
    const void* zero = conv_zero_row();
    DCLIP_HOST_CHECK(zero != nullptr, "dclip_conv3x3: zero row allocation failed");
    hipStream_t st = (hipStream_t)stream;
    const PixGeo g{x_bstride, x_off, (int)x_ld, H, W};
    const int M = B * H * W;
    const int dir = mode == 0 ? 1 : -1;
    constexpr int TBM = 256, TBN = 128;
    const int tiles_m = (M + TBM - 1) / TBM, tiles_n = (Nout + TBN - 1) / TBN;
    const int map_hw = out_gap ? H * W : 0;
    // the input's extent in bytes for the buffer-load staging (0: too large for 32-bit offsets ->
    // pointer staging with the zero row)
    const int64_t xext = ((int64_t)(B - 1) * x_bstride + x_off + (int64_t)H * W * x_ld) * 2;
    const uint32_t xbytes = xext < (1ll << 32) - 4096 ? (uint32_t)xext : 0u;
#define CONV_LAUNCH(T, EPI, OUTT)                                                                                    \
    conv_nt_kernel<T, EPI, OUTT, TBM, TBN, 4, 2, 3><<<tiles_m * tiles_n, 512, 0, st>>>(                             \
        (const T*)X, (const T*)zero, g, Cin, dir, (const T*)Wt, 9 * (int64_t)Cin, M, Nout, tiles_m, tiles_n, out,    \
        out_ld, out, out_ld, map_hw, out_gap, out_off, xbytes)
    if (ab_dt == DCLIP_BF16) {
        if (accumulate) CONV_LAUNCH(bf16, DCLIP_EPI_RESIDUAL, float);
        else if (out_dt == DCLIP_F32) CONV_LAUNCH(bf16, DCLIP_EPI_STORE, float);
        else CONV_LAUNCH(bf16, DCLIP_EPI_STORE, bf16);
    } else {
        if (accumulate) CONV_LAUNCH(f16, DCLIP_EPI_RESIDUAL, float);
        else if (out_dt == DCLIP_F32) CONV_LAUNCH(f16, DCLIP_EPI_STORE, float);
        else CONV_LAUNCH(f16, DCLIP_EPI_STORE, f16);
    }
#undef CONV_LAUNCH
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_conv3x3_wgrad(int ab_dt, const void* dY, int64_t ldy, int Nout, const void* X, int64_t x_bstride,
                                   int64_t x_off, int64_t x_ld, int B, int H, int W, int Cin, float* dW, void* ws,
                                   int splits, int oihw, const float* alpha_ptr, void* stream) {
    DCLIP_HOST_CHECK(ab_dt == DCLIP_BF16 || ab_dt == DCLIP_F16, "dclip_conv3x3_wgrad: operands must be f16/bf16");
    DCLIP_HOST_CHECK(Cin % 128 == 0 && Nout % 8 == 0 && Nout > 0 && ldy % 8 == 0 && ldy >= Nout,
                     "dclip_conv3x3_wgrad: Cin %% 128 == 0 and Nout %% 8 == 0 required");
    DCLIP_HOST_CHECK(x_ld % 8 == 0 && x_bstride % 8 == 0 && x_off % 8 == 0, "dclip_conv3x3_wgrad: bad strides");
    DCLIP_HOST_CHECK(splits >= 1 && ws != nullptr, "dclip_conv3x3_wgrad: workspace of splits * Nout * 9 * Cin f32");
    DCLIP_HOST_CHECK((int64_t)B * H * W < (1ll << 24), "dclip_conv3x3_wgrad: too many pixels");
    const void* zero = conv_zero_row();
    DCLIP_HOST_CHECK(zero != nullptr, "dclip_conv3x3_wgrad: zero row allocation failed");
    hipStream_t st = (hipStream_t)stream;
    const PixGeo g{x_bstride, x_off, (int)x_ld, H, W};
    const int Kpix = B * H * W;
    const int N = 9 * Cin;
    const int kp = (Kpix + 64 * splits - 1) / (64 * splits) * 64;  // pixel rows per split
    const int tiles_m = (Nout + BM - 1) / BM, tiles_n = N / BN;
    dim3 grid(tiles_m * tiles_n, splits);
    // DCLIP_OPT_GEMM_TN_TILE 5: the LDS-DMA builtin form (each K-step's staging serialised)
#define WG_LAUNCH(T, AD)                                                                                        \
    conv_wgrad_kernel<T, AD><<<grid, 256, 0, st>>>((const T*)dY, ldy, (const T*)X, (const T*)zero, g, Cin, Nout, N, \
                                                   Kpix, kp, tiles_m, tiles_n, (float*)ws, (int64_t)Nout * N)
    const bool ad = dclip_option(DCLIP_OPT_GEMM_TN_TILE) != 5;
    if (ab_dt == DCLIP_BF16) {
        if (ad) WG_LAUNCH(bf16, true);
        else WG_LAUNCH(bf16, false);
    } else {
        if (ad) WG_LAUNCH(f16, true);
        else WG_LAUNCH(f16, false);
    }
#undef WG_LAUNCH
    if (oihw || alpha_ptr != nullptr) {
        const int64_t total = (int64_t)Nout * Cin;
        const int blocks = (int)((total + 255) / 256 > 4096 ? 4096 : (total + 255) / 256);
        if (oihw) {
            conv_wgrad_reduce_oihw_kernel<<<blocks, 256, 0, st>>>((const float*)ws, splits, (int64_t)Nout * N, Nout, Cin,
                                                                  Alpha(1.f, alpha_ptr), dW);
            DCLIP_LAUNCH_CHECK();
            return 0;
        }
        DCLIP_HOST_CHECK(false, "dclip_conv3x3_wgrad: alpha_ptr needs the OIHW output");
    }
    const int64_t total4 = (int64_t)Nout * (N / 4);
    int blocks = (int)((total4 + 255) / 256);
    blocks = blocks > 4096 ? 4096 : blocks;
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>((const float*)ws, splits, (int64_t)Nout * N, Nout, N, nullptr, dW,
                                                 N);
    DCLIP_LAUNCH_CHECK();
    return 0;
}
