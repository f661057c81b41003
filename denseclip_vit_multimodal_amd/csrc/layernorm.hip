// LayerNorm forward/backward with fp32 statistics (reference seg/denseclip/models.py:243-249:
// the reference casts to fp32, runs nn.LayerNorm (eps 1e-5, biased variance) and casts
// back).  One wave per row, the row held in registers, wave-shuffle reductions.
// HBM-bound: forward reads the row once (f32) and writes it once (bf16/f16/f32);
// backward reads dy and x once and writes dx once, with dw/db summed in registers over a
// grid-strided set of rows and flushed once per block.
#include <type_traits>

#include "common.h"

namespace {

constexpr int MAXV = 32;  // elements per lane => cols <= 2048

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* v) {
    if constexpr (sizeof(T) == 4) {
        f32x4 x = *(const f32x4*)p;
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    } else {
        typedef T t4 __attribute__((ext_vector_type(4)));
        t4 x = *(const t4*)p;
        v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3];
    }
}
template <typename T>
__device__ __forceinline__ void store4(T* p, const float* v) {
    if constexpr (sizeof(T) == 4) {
        f32x4 x = {v[0], v[1], v[2], v[3]};
        *(f32x4*)p = x;
    } else {
        typedef T t4 __attribute__((ext_vector_type(4)));
        t4 x = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
        *(t4*)p = x;
    }
}

// cols % 4 == 0; lane owns columns 4*lane + 256*i .. +3
template <typename TX, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const TX* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, TY* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t rows, int cols, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const TX* xr = x + row * cols;
    float v[MAXV];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < cols) {
            load4(xr + c, v + 4 * i);
            s += v[4 * i] + v[4 * i + 1] + v[4 * i + 2] + v[4 * i + 3];
        }
    }
    const float mu = wave_sum(s) / cols;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < cols) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float d = v[4 * i + e] - mu;
                ss += d * d;
            }
        }
    }
    const float rs = rsqrtf(wave_sum(ss) / cols + eps);
    TY* yr = y + row * cols;
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < cols) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (v[4 * i + e] - mu) * rs * w[c + e] + b[c + e];
            store4(yr + c, o);
        }
    }
    if (lane == 0) {
        if (mean_out) mean_out[row] = mu;
        if (rstd_out) rstd_out[row] = rs;
    }
}

// optional 16-bit copy of the backward's output (the next GEMM's operand): lp_dt F16 / BF16
__device__ __forceinline__ void store_lp(void* lp, int lp_dt, int64_t off, const float* o) {
    if (lp_dt == DCLIP_BF16) store4((bf16*)lp + off, o);
    else store4((f16*)lp + off, o);
}

template <typename TDY, typename TX>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* res, float* dx,
                                                     void* __restrict__ lp, int lp_dt, float* __restrict__ dw,
                                                     float* __restrict__ db, int64_t rows, int cols) {
    __shared__ float red[2][4][64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float aw[MAXV], ab[MAXV];
#pragma unroll
    for (int i = 0; i < MAXV; ++i) { aw[i] = 0.f; ab[i] = 0.f; }
    float wl[MAXV];
#pragma unroll
    for (int i = 0; i < MAXV / 4; ++i) {
        const int c = 4 * lane + 256 * i;
#pragma unroll
        for (int e = 0; e < 4; ++e) wl[4 * i + e] = c < cols ? w[c + e] : 0.f;
    }
    for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < rows; row += (int64_t)gridDim.x * 4) {
        const float mu = mean[row], rs = rstd[row];
        float xh[MAXV], g[MAXV];
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int i = 0; i < MAXV / 4; ++i) {
            const int c = 4 * lane + 256 * i;
            if (c < cols) {
                float dv[4], xv[4];
                load4(dy + row * cols + c, dv);
                load4(x + row * cols + c, xv);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = 4 * i + e;
                    xh[k] = (xv[e] - mu) * rs;
                    g[k] = dv[e] * wl[k];
                    sg += g[k];
                    sgx += g[k] * xh[k];
                    aw[k] += dv[e] * xh[k];
                    ab[k] += dv[e];
                }
            }
        }
        const float mg = wave_sum(sg) / cols;
        const float mgx = wave_sum(sgx) / cols;
#pragma unroll
        for (int i = 0; i < MAXV / 4; ++i) {
            const int c = 4 * lane + 256 * i;
            if (c < cols) {
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = 4 * i + e;
                    o[e] = rs * (g[k] - mg - xh[k] * mgx);
                }
                if (res) {
                    const f32x4 old = *(const f32x4*)(res + row * cols + c);
                    o[0] += old[0]; o[1] += old[1]; o[2] += old[2]; o[3] += old[3];
                }
                store4(dx + row * cols + c, o);
                if (lp) store_lp(lp, lp_dt, row * cols + c, o);
            }
        }
    }
    // block reduction of dw/db (one column group at a time through a small LDS
    // buffer), then one atomic per column per block
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (256 * (i / 4) >= cols) break;  // block-uniform
        red[0][wave][lane] = aw[i];
        red[1][wave][lane] = ab[i];
        __syncthreads();
        if (wave == 0) {
            const int c = 4 * lane + 256 * (i / 4) + (i % 4);
            if (c < cols) {
                const float sw = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
                const float sb = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
                if (dw) atomicAdd(dw + c, sw);
                if (db) atomicAdd(db + c, sb);
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------- fast path
// cols = 256 * NV (768 = ViT-B, 1024 = ViT-L): persistent waves walk rows grid-strided with
// the NEXT row's loads issued before the current row is reduced (one row of loads always in
// flight per wave), w / b held in registers, register arrays sized exactly (no MAXV
// footprint, so occupancy is not register-bound).
template <typename TX, typename TY, int NV>
__global__ __launch_bounds__(256) void ln_fwd_fast(const TX* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ b, TY* __restrict__ y,
                                                   float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                   int64_t rows, float eps) {
    constexpr int cols = 256 * NV;
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    float wl[4 * NV], bl[4 * NV], v[4 * NV], nv[4 * NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        load4(w + 4 * lane + 256 * i, wl + 4 * i);
        load4(b + 4 * lane + 256 * i, bl + 4 * i);
        load4(x + row * cols + 4 * lane + 256 * i, v + 4 * i);
    }
    while (true) {
        const int64_t nrow = row + stride;
        if (nrow < rows) {
#pragma unroll
            for (int i = 0; i < NV; ++i) load4(x + nrow * cols + 4 * lane + 256 * i, nv + 4 * i);
        }
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4 * NV; ++k) s += v[k];
        const float mu = wave_sum(s) * (1.0f / cols);
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < 4 * NV; ++k) {
            const float d = v[k] - mu;
            ss += d * d;
        }
        const float rs = rsqrtf(wave_sum(ss) * (1.0f / cols) + eps);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (v[4 * i + e] - mu) * rs * wl[4 * i + e] + bl[4 * i + e];
            store4(y + row * cols + 4 * lane + 256 * i, o);
        }
        if (lane == 0) {
            if (mean_out) mean_out[row] = mu;
            if (rstd_out) rstd_out[row] = rs;
        }
        if (nrow >= rows) break;
        row = nrow;
        for (int k = 0; k < 4 * NV; ++k) v[k] = nv[k];
    }
}

// 8 waves per block and at most 512 blocks: the dw / db partial sums of a block are reduced
// in LDS and stored as the block's row of the caller's partials table `part` ([block][2][cols],
// dclip_layernorm_bwd_ws_floats), which ln_dwdb_reduce_kernel sums in block order into dw / db —
// deterministic, and private to the call (no state shared between streams or graph replays).
// Without a table the blocks add atomically into dw / db (512 adds per address: 16-23 us of a
// 112-190 us pass, tools/ln_probe.py)
//
// DS (delayed scale, fp16 lp): lp = (f16)(dx * s), s the power-of-two scale of this gradient
// site's previous use (common.h ds_*: use `use` of the state st), (s, 1/s) to spair for the
// consumers of lp, and this use's |dx| maximum joined into st for the next.
//
// TA (dclip_layernorm_bwd_add / _scaled_add): dx = (res + LN^T(dy)) + add * (*add_scale), add a
// 16-bit (TA) token buffer whose rows with row % ntok == 0 (the CLS rows) read as 0 — the previous
// block's read-out map gradient, so the sum and its 16-bit copy lp come out of this pass instead
// of a dclip_add_readout_cast(_scaled) pass over the written dx (the same fp32 arithmetic in the
// same order: bitwise its result)
template <typename TDY, typename TX, int NV, bool DS = false, typename TA = void>
__global__ __launch_bounds__(512) void ln_bwd_fast(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                   const float* __restrict__ w, const float* __restrict__ mean,
                                                   const float* __restrict__ rstd, const float* res, float* dx,
                                                   void* __restrict__ lp, int lp_dt, float* __restrict__ dw,
                                                   float* __restrict__ db, int64_t rows, float* part,
                                                   float* st = nullptr, int use = 0, float* spair = nullptr,
                                                   float target = 0.f, const void* __restrict__ add = nullptr,
                                                   int ntok = 1, const float* __restrict__ add_scale = nullptr,
                                                   const float* __restrict__ dy_scale = nullptr, int64_t dy_ntok = 0) {
    constexpr int cols = 256 * NV;
    constexpr bool ADD = !std::is_void<TA>::value;
    typedef typename std::conditional<ADD, TA, bf16>::type TAV;  // (a loadable type when ADD is off)
    const TAV* addp = (const TAV*)add;
    float sb = 1.f;
    if constexpr (ADD) sb = add_scale != nullptr ? *add_scale : 1.f;
    // dy_scale: dy arrives on a gradient scale (fp16: the dX GEMM's output left on its operand's s),
    // times *dy_scale (= 1/s) on load; dy_ntok > 0: dy's rows with row % dy_ntok == 0 (CLS) read as 0
    const float dsc = dy_scale != nullptr ? *dy_scale : 1.f;
    __shared__ float red[8][2][4 * NV][64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float ls = 1.f;
    uint32_t amax = 0;
    if constexpr (DS) {
        ls = ds_scale_of_use(st, use, target);
        ds_begin(st, use, ls, spair);
    }
    const int64_t stride = (int64_t)gridDim.x * 8;
    float aw[4 * NV], ab[4 * NV], wl[4 * NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) load4(w + 4 * lane + 256 * i, wl + 4 * i);
#pragma unroll
    for (int k = 0; k < 4 * NV; ++k) aw[k] = ab[k] = 0.f;
    int64_t row = (int64_t)blockIdx.x * 8 + wave;
    // everything a row needs (dy, x, the accumulated dx, its statistics) is loaded one row
    // ahead, so no load latency is exposed per row
    float dv[4 * NV], xv[4 * NV], old[4 * NV], ndv[4 * NV], nxv[4 * NV], nold[4 * NV];
    float av[ADD ? 4 * NV : 1], nav[ADD ? 4 * NV : 1];
    float mu = 0.f, rs = 0.f, nmu = 0.f, nrs = 0.f;
    if (row < rows) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            load4(dy + row * cols + 4 * lane + 256 * i, dv + 4 * i);
            load4(x + row * cols + 4 * lane + 256 * i, xv + 4 * i);
            if (res) load4(res + row * cols + 4 * lane + 256 * i, old + 4 * i);
            if constexpr (ADD) {
                if (row % ntok != 0) load4(addp + row * cols + 4 * lane + 256 * i, av + 4 * i);
                else
#pragma unroll
                    for (int e = 0; e < 4; ++e) av[4 * i + e] = 0.f;
            }
        }
        mu = mean[row];
        rs = rstd[row];
    }
    while (row < rows) {
        const int64_t nrow = row + stride;
        if (nrow < rows) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                load4(dy + nrow * cols + 4 * lane + 256 * i, ndv + 4 * i);
                load4(x + nrow * cols + 4 * lane + 256 * i, nxv + 4 * i);
                if (res) load4(res + nrow * cols + 4 * lane + 256 * i, nold + 4 * i);
                if constexpr (ADD) {
                    if (nrow % ntok != 0) load4(addp + nrow * cols + 4 * lane + 256 * i, nav + 4 * i);
                    else
#pragma unroll
                        for (int e = 0; e < 4; ++e) nav[4 * i + e] = 0.f;
                }
            }
            nmu = mean[nrow];
            nrs = rstd[nrow];
        }
        if (dy_scale != nullptr) {
#pragma unroll
            for (int k = 0; k < 4 * NV; ++k) dv[k] *= dsc;
        }
        if (dy_ntok > 0 && row % dy_ntok == 0) {
#pragma unroll
            for (int k = 0; k < 4 * NV; ++k) dv[k] = 0.f;
        }
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int k = 0; k < 4 * NV; ++k) {
            const float xh = (xv[k] - mu) * rs;
            const float g = dv[k] * wl[k];
            sg += g;
            sgx += g * xh;
            aw[k] += dv[k] * xh;
            ab[k] += dv[k];
            xv[k] = xh;  // keep x-hat
        }
        const float mg = wave_sum(sg) * (1.0f / cols);
        const float mgx = wave_sum(sgx) * (1.0f / cols);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = 4 * i + e;
                o[e] = rs * (dv[k] * wl[k] - mg - xv[k] * mgx);
                if (res) o[e] += old[k];
                if constexpr (ADD) o[e] += av[k] * sb;
            }
            store4(dx + row * cols + 4 * lane + 256 * i, o);
            if constexpr (DS) {
                float q[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    amax = max(amax, __float_as_uint(o[e]) & 0x7fffffffu);
                    q[e] = o[e] * ls;
                }
                store4((f16*)lp + row * cols + 4 * lane + 256 * i, q);
            } else {
                if (lp) store_lp(lp, lp_dt, row * cols + 4 * lane + 256 * i, o);
            }
        }
        row = nrow;
        mu = nmu;
        rs = nrs;
#pragma unroll
        for (int k = 0; k < 4 * NV; ++k) {
            dv[k] = ndv[k];
            xv[k] = nxv[k];
            old[k] = nold[k];
            if constexpr (ADD) av[k] = nav[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 4 * NV; ++k) {
        red[wave][0][k][lane] = aw[k];
        red[wave][1][k][lane] = ab[k];
    }
    __syncthreads();
    // thread t sums the 8 waves' partials of entries t, t + 512, ... of the [2][4NV][64] table
    // into this block's row [dw | db] of the partials table (or, without one, atomically into dw / db)
    for (int e = threadIdx.x; e < 2 * 4 * NV * 64; e += 512) {
        const int which = e / (4 * NV * 64), k = (e / 64) % (4 * NV), l = e % 64;
        float sum = 0.f;
#pragma unroll
        for (int wv = 0; wv < 8; ++wv) sum += red[wv][which][k][l];
        const int c = 4 * l + 256 * (k / 4) + (k % 4);
        if (part != nullptr) {
            part[((int64_t)blockIdx.x * 2 + which) * cols + c] = sum;
        } else {
            float* out = which ? db : dw;
            if (out) atomicAdd(out + c, sum);
        }
    }
    if constexpr (DS) ds_end<8>(amax, st, use);
}

// dw[c] += sum_b part[b][0][c], db[c] += sum_b part[b][1][c] over the nblk blocks' rows, in
// block order (deterministic): a workgroup per 32 consecutive entries of the [2][cols] row, 8 row
// slices of 32 lanes (128-B row segments), the slices added in LDS in slice order
__global__ __launch_bounds__(256) void ln_dwdb_reduce_kernel(const float* __restrict__ part, int cols, int nblk,
                                                             float* __restrict__ dw, float* __restrict__ db) {
    __shared__ float red[8][32];
    const int l = threadIdx.x & 31, sl = threadIdx.x >> 5;
    const int e = blockIdx.x * 32 + l;  // which * cols + c
    float sum = 0.f;
    if (e < 2 * cols) {
#pragma unroll 8
        for (int b = sl; b < nblk; b += 8) sum += part[(int64_t)b * 2 * cols + e];
    }
    red[sl][l] = sum;
    __syncthreads();
    if (sl == 0 && e < 2 * cols) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += red[k][l];
        float* out = e < cols ? dw : db;
        if (out != nullptr) out[e % cols] += t;
    }
}

inline int64_t ln_bwd_blocks(int64_t rows) {
    const int64_t blocks = (rows + 7) / 8;
    return blocks > 512 ? 512 : blocks;
}

// the partials table (ws) sum, when the caller gave one and the pass has dw / db
inline void ln_dwdb_reduce(float* part, int cols, int64_t blocks, float* dw, float* db, hipStream_t st) {
    if (part) ln_dwdb_reduce_kernel<<<(2 * cols + 31) / 32, 256, 0, st>>>(part, cols, (int)blocks, dw, db);
}

// blocks of 4 waves: enough persistent waves to fill the chip (8 per SIMD), fewer for small inputs
inline int64_t ln_blocks(int64_t rows, int64_t cap) {
    int64_t blocks = (rows + 3) / 4;
    return blocks > cap ? cap : blocks;
}

template <typename TX, typename TY, int NV>
void fwd_fast(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd, int64_t rows,
              float eps, hipStream_t st) {
    ln_fwd_fast<TX, TY, NV><<<(unsigned)ln_blocks(rows, 2048), 256, 0, st>>>((const TX*)x, w, b, (TY*)y, mean, rstd,
                                                                            rows, eps);
}

template <typename TDY, typename TX, int NV>
void bwd_fast(const void* dy, const float* dy_scale, int64_t dy_ntok, const void* x, const float* w, const float* mean,
              const float* rstd, const float* res, float* dx, void* lp, int lp_dt, float* dw, float* db, float* ws,
              int64_t rows, hipStream_t st) {
    const int64_t blocks = ln_bwd_blocks(rows);
    float* part = (dw || db) ? ws : nullptr;
    ln_bwd_fast<TDY, TX, NV><<<(unsigned)blocks, 512, 0, st>>>((const TDY*)dy, (const TX*)x, w, mean, rstd, res, dx,
                                                              lp, lp_dt, dw, db, rows, part, nullptr, 0, nullptr, 0.f,
                                                              nullptr, 1, nullptr, dy_scale, dy_ntok);
    ln_dwdb_reduce(part, 256 * NV, blocks, dw, db, st);
}

template <typename TX, typename TY>
void fwd_launch(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                int64_t rows, int cols, float eps, hipStream_t st) {
    switch (cols) {
        case 512: return fwd_fast<TX, TY, 2>(x, w, b, y, mean, rstd, rows, eps, st);
        case 768: return fwd_fast<TX, TY, 3>(x, w, b, y, mean, rstd, rows, eps, st);
        case 1024: return fwd_fast<TX, TY, 4>(x, w, b, y, mean, rstd, rows, eps, st);
        default: break;
    }
    dim3 grid((unsigned)((rows + 3) / 4));
    ln_fwd_kernel<TX, TY><<<grid, 256, 0, st>>>((const TX*)x, w, b, (TY*)y, mean, rstd, rows, cols, eps);
}

template <typename TX>
void fwd_dispatch_y(int y_dt, const void* x, const float* w, const float* b, void* y, float* mean,
                    float* rstd, int64_t rows, int cols, float eps, hipStream_t st) {
    if (y_dt == DCLIP_F32) fwd_launch<TX, float>(x, w, b, y, mean, rstd, rows, cols, eps, st);
    else if (y_dt == DCLIP_F16) fwd_launch<TX, f16>(x, w, b, y, mean, rstd, rows, cols, eps, st);
    else fwd_launch<TX, bf16>(x, w, b, y, mean, rstd, rows, cols, eps, st);
}

template <typename TDY, typename TX>
void bwd_launch(const void* dy, const float* dy_scale, int64_t dy_ntok, const void* x, const float* w,
                const float* mean, const float* rstd, const float* res, float* dx, void* lp, int lp_dt, float* dw,
                float* db, float* ws, int64_t rows, int cols, hipStream_t st) {
    switch (cols) {
        case 512:
            return bwd_fast<TDY, TX, 2>(dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows, st);
        case 768:
            return bwd_fast<TDY, TX, 3>(dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows, st);
        case 1024:
            return bwd_fast<TDY, TX, 4>(dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows, st);
        default: break;
    }
    int64_t blocks = (rows + 3) / 4;
    if (blocks > 1024) blocks = 1024;
    ln_bwd_kernel<TDY, TX><<<(unsigned)blocks, 256, 0, st>>>((const TDY*)dy, (const TX*)x, w, mean, rstd,
                                                             res, dx, lp, lp_dt, dw, db, rows, cols);
}

template <typename TDY>
void bwd_dispatch_x(int x_dt, const void* dy, const float* dy_scale, int64_t dy_ntok, const void* x, const float* w,
                    const float* mean, const float* rstd, const float* res, float* dx, void* lp, int lp_dt, float* dw,
                    float* db, float* ws, int64_t rows, int cols, hipStream_t st) {
    if (x_dt == DCLIP_F32)
        bwd_launch<TDY, float>(dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows, cols, st);
    else if (x_dt == DCLIP_F16)
        bwd_launch<TDY, f16>(dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows, cols, st);
    else bwd_launch<TDY, bf16>(dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows, cols, st);
}

template <typename TDY, int NV>
void bwd_fast_ds(const void* dy, const float* dy_scale, const float* x, const float* w, const float* mean,
                 const float* rstd, const float* res, float* dx, void* lp, float* dw, float* db, float* ws, int64_t rows,
                 float* st, int use, float* spair, float target, hipStream_t s) {
    const int64_t blocks = ln_bwd_blocks(rows);
    float* part = (dw || db) ? ws : nullptr;
    ln_bwd_fast<TDY, float, NV, true><<<(unsigned)blocks, 512, 0, s>>>(
        (const TDY*)dy, x, w, mean, rstd, res, dx, lp, DCLIP_F16, dw, db, rows, part, st, use, spair, target, nullptr, 1,
        nullptr, dy_scale, 0);
    ln_dwdb_reduce(part, 256 * NV, blocks, dw, db, s);
}

template <typename TDY>
void bwd_ds_cols(const void* dy, const float* dy_scale, const float* x, const float* w, const float* mean,
                 const float* rstd, const float* res, float* dx, void* lp, float* dw, float* db, float* ws, int64_t rows,
                 int64_t cols, float* st, int use, float* spair, float target, hipStream_t s) {
    if (cols == 512)
        bwd_fast_ds<TDY, 2>(dy, dy_scale, x, w, mean, rstd, res, dx, lp, dw, db, ws, rows, st, use, spair, target, s);
    else if (cols == 768)
        bwd_fast_ds<TDY, 3>(dy, dy_scale, x, w, mean, rstd, res, dx, lp, dw, db, ws, rows, st, use, spair, target, s);
    else bwd_fast_ds<TDY, 4>(dy, dy_scale, x, w, mean, rstd, res, dx, lp, dw, db, ws, rows, st, use, spair, target, s);
}

template <typename TDY, int NV>
void bwd_fast_add(const void* dy, const float* x, const float* w, const float* mean, const float* rstd,
                  const float* res, const bf16* add, int ntok, float* dx, void* lp, int lp_dt, float* dw, float* db,
                  float* ws, int64_t rows, hipStream_t s) {
    const int64_t blocks = ln_bwd_blocks(rows);
    float* part = (dw || db) ? ws : nullptr;
    ln_bwd_fast<TDY, float, NV, false, bf16><<<(unsigned)blocks, 512, 0, s>>>(
        (const TDY*)dy, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, rows, part, nullptr, 0, nullptr, 0.f, add, ntok);
    ln_dwdb_reduce(part, 256 * NV, blocks, dw, db, s);
}

template <typename TDY>
void bwd_add_cols(const void* dy, const float* x, const float* w, const float* mean, const float* rstd,
                  const float* res, const bf16* add, int ntok, float* dx, void* lp, int lp_dt, float* dw, float* db,
                  float* ws, int64_t rows, int64_t cols, hipStream_t s) {
    if (cols == 512) bwd_fast_add<TDY, 2>(dy, x, w, mean, rstd, res, add, ntok, dx, lp, lp_dt, dw, db, ws, rows, s);
    else if (cols == 768) bwd_fast_add<TDY, 3>(dy, x, w, mean, rstd, res, add, ntok, dx, lp, lp_dt, dw, db, ws, rows, s);
    else bwd_fast_add<TDY, 4>(dy, x, w, mean, rstd, res, add, ntok, dx, lp, lp_dt, dw, db, ws, rows, s);
}

template <typename TDY, typename TA, int NV>
void bwd_fast_ds_add(const void* dy, const float* dy_scale, const float* x, const float* w, const float* mean,
                     const float* rstd, const float* res, const void* add, const float* add_scale, int ntok, float* dx,
                     void* lp, float* dw, float* db, float* ws, int64_t rows, float* st, int use, float* spair,
                     float target, hipStream_t s) {
    const int64_t blocks = ln_bwd_blocks(rows);
    float* part = (dw || db) ? ws : nullptr;
    ln_bwd_fast<TDY, float, NV, true, TA><<<(unsigned)blocks, 512, 0, s>>>(
        (const TDY*)dy, x, w, mean, rstd, res, dx, lp, DCLIP_F16, dw, db, rows, part, st, use, spair, target, add, ntok,
        add_scale, dy_scale, 0);
    ln_dwdb_reduce(part, 256 * NV, blocks, dw, db, s);
}

template <typename TDY, typename TA>
void bwd_ds_add_cols(const void* dy, const float* dy_scale, const float* x, const float* w, const float* mean,
                     const float* rstd, const float* res, const void* add, const float* add_scale, int ntok, float* dx,
                     void* lp, float* dw, float* db, float* ws, int64_t rows, int64_t cols, float* st, int use,
                     float* spair, float target, hipStream_t s) {
    if (cols == 512)
        bwd_fast_ds_add<TDY, TA, 2>(dy, dy_scale, x, w, mean, rstd, res, add, add_scale, ntok, dx, lp, dw, db, ws, rows,
                                    st, use, spair, target, s);
    else if (cols == 768)
        bwd_fast_ds_add<TDY, TA, 3>(dy, dy_scale, x, w, mean, rstd, res, add, add_scale, ntok, dx, lp, dw, db, ws, rows,
                                    st, use, spair, target, s);
    else
        bwd_fast_ds_add<TDY, TA, 4>(dy, dy_scale, x, w, mean, rstd, res, add, add_scale, ntok, dx, lp, dw, db, ws, rows,
                                    st, use, spair, target, s);
}

}  // namespace

extern "C" int dclip_layernorm_bwd_add(const void* dy, int dy_dt, const float* x, const float* w, const float* mean,
                                       const float* rstd, const float* res, const void* add, int ntok, float* dx,
                                       void* lp, int lp_dt, float* dw, float* db, float* ws, int64_t rows, int64_t cols,
                                       void* stream) {
    DCLIP_HOST_CHECK(cols == 512 || cols == 768 || cols == 1024,
                     "dclip_layernorm_bwd_add: cols must be 512, 768 or 1024 (got %lld)", (long long)cols);
    DCLIP_HOST_CHECK(dy_dt == DCLIP_F32 || dy_dt == DCLIP_BF16, "dclip_layernorm_bwd_add: dy must be f32 or bf16");
    DCLIP_HOST_CHECK(add != nullptr && ntok > 0, "dclip_layernorm_bwd_add: the bf16 add buffer and ntok > 0");
    DCLIP_HOST_CHECK(lp != nullptr && (lp_dt == DCLIP_BF16 || lp_dt == DCLIP_F16),
                     "dclip_layernorm_bwd_add: lp (F16 or BF16) is required");
    DCLIP_HOST_CHECK(rows >= 0, "dclip_layernorm_bwd_add: rows < 0");
    if (rows == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (dy_dt == DCLIP_F32)
        bwd_add_cols<float>(dy, x, w, mean, rstd, res, (const bf16*)add, ntok, dx, lp, lp_dt, dw, db, ws, rows, cols, s);
    else bwd_add_cols<bf16>(dy, x, w, mean, rstd, res, (const bf16*)add, ntok, dx, lp, lp_dt, dw, db, ws, rows, cols, s);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_layernorm_bwd_scaled_add(const void* dy, int dy_dt, const float* dy_scale, const float* x,
                                              const float* w, const float* mean, const float* rstd, const float* res,
                                              const void* add, int add_dt, const float* add_scale, int ntok, float* dx,
                                              void* lp, float* dw, float* db, float* ws, int64_t rows, int64_t cols,
                                              float target, float* st, int use, float* spair, void* stream) {
    DCLIP_HOST_CHECK(cols == 512 || cols == 768 || cols == 1024,
                     "dclip_layernorm_bwd_scaled_add: cols must be 512, 768 or 1024 (got %lld)", (long long)cols);
    DCLIP_HOST_CHECK(dy_dt == DCLIP_F32 || dy_dt == DCLIP_F16, "dclip_layernorm_bwd_scaled_add: dy must be f32 or f16");
    DCLIP_HOST_CHECK(add != nullptr && ntok > 0 && (add_dt == DCLIP_F16 || add_dt == DCLIP_BF16),
                     "dclip_layernorm_bwd_scaled_add: a 16-bit add buffer and ntok > 0");
    DCLIP_HOST_CHECK(lp != nullptr && st != nullptr && spair != nullptr && target > 0.f && use >= 1,
                     "dclip_layernorm_bwd_scaled_add: lp, the scale state, use >= 1, the scale pair and target > 0");
    DCLIP_HOST_CHECK(rows > 0, "dclip_layernorm_bwd_scaled_add: rows must be > 0");
    hipStream_t s = (hipStream_t)stream;
#define DS_ADD(TDY, TA)                                                                                       \
    bwd_ds_add_cols<TDY, TA>(dy, dy_scale, x, w, mean, rstd, res, add, add_scale, ntok, dx, lp, dw, db, ws, rows, cols, st, \
                             use, spair, target, s)
    if (dy_dt == DCLIP_F32) {
        if (add_dt == DCLIP_F16) DS_ADD(float, f16);
        else DS_ADD(float, bf16);
    } else {
        if (add_dt == DCLIP_F16) DS_ADD(f16, f16);
        else DS_ADD(f16, bf16);
    }
#undef DS_ADD
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_layernorm_bwd_scaled(const void* dy, int dy_dt, const float* dy_scale, const void* x, int x_dt,
                                          const float* w, const float* mean, const float* rstd, const float* res,
                                          float* dx, void* lp, float* dw, float* db, float* ws, int64_t rows,
                                          int64_t cols, float target, float* st, int use, float* spair, void* stream) {
    DCLIP_HOST_CHECK(cols == 512 || cols == 768 || cols == 1024,
                     "dclip_layernorm_bwd_scaled: cols must be 512, 768 or 1024 (got %lld)", (long long)cols);
    DCLIP_HOST_CHECK(x_dt == DCLIP_F32, "dclip_layernorm_bwd_scaled: x must be f32 (the residual stream)");
    DCLIP_HOST_CHECK(dy_dt == DCLIP_F32 || dy_dt == DCLIP_F16, "dclip_layernorm_bwd_scaled: dy must be f32 or f16");
    DCLIP_HOST_CHECK(lp != nullptr && st != nullptr && spair != nullptr && target > 0.f && use >= 1,
                     "dclip_layernorm_bwd_scaled: lp, the scale state, use >= 1, the scale pair and target > 0");
    DCLIP_HOST_CHECK(rows > 0, "dclip_layernorm_bwd_scaled: rows must be > 0");
    hipStream_t s = (hipStream_t)stream;
    if (dy_dt == DCLIP_F32)
        bwd_ds_cols<float>(dy, dy_scale, (const float*)x, w, mean, rstd, res, dx, lp, dw, db, ws, rows, cols, st, use,
                           spair, target, s);
    else
        bwd_ds_cols<f16>(dy, dy_scale, (const float*)x, w, mean, rstd, res, dx, lp, dw, db, ws, rows, cols, st, use, spair,
                         target, s);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_layernorm_fwd(const void* x, int x_dt, const float* w, const float* b, void* y,
                                   int y_dt, float* mean, float* rstd, int64_t rows, int64_t cols,
                                   float eps, void* stream) {
    DCLIP_HOST_CHECK(cols > 0 && cols % 4 == 0 && cols <= 64 * MAXV,
                     "dclip_layernorm_fwd: cols=%lld must be a multiple of 4 and <= %d", (long long)cols, 64 * MAXV);
    DCLIP_HOST_CHECK(rows >= 0, "dclip_layernorm_fwd: rows < 0");
    if (rows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (x_dt == DCLIP_F32) fwd_dispatch_y<float>(y_dt, x, w, b, y, mean, rstd, rows, (int)cols, eps, st);
    else if (x_dt == DCLIP_F16) fwd_dispatch_y<f16>(y_dt, x, w, b, y, mean, rstd, rows, (int)cols, eps, st);
    else fwd_dispatch_y<bf16>(y_dt, x, w, b, y, mean, rstd, rows, (int)cols, eps, st);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int64_t dclip_layernorm_bwd_ws_floats(int64_t rows, int64_t cols) {
    if (rows <= 0 || !(cols == 512 || cols == 768 || cols == 1024)) return 0;
    return ln_bwd_blocks(rows) * 2 * cols;
}

extern "C" int dclip_layernorm_bwd_res(const void* dy, int dy_dt, const float* dy_scale, int64_t dy_ntok, const void* x,
                                       int x_dt, const float* w, const float* mean, const float* rstd, const float* res,
                                       float* dx, void* lp, int lp_dt, float* dw, float* db, float* ws, int64_t rows,
                                       int64_t cols, void* stream) {
    DCLIP_HOST_CHECK(cols > 0 && cols % 4 == 0 && cols <= 64 * MAXV,
                     "dclip_layernorm_bwd: cols=%lld must be a multiple of 4 and <= %d", (long long)cols, 64 * MAXV);
    DCLIP_HOST_CHECK((dy_scale == nullptr && dy_ntok == 0) || cols == 512 || cols == 768 || cols == 1024,
                     "dclip_layernorm_bwd_res: dy_scale / dy_ntok need cols 512, 768 or 1024 (got %lld)", (long long)cols);
    DCLIP_HOST_CHECK(dy_ntok >= 0, "dclip_layernorm_bwd_res: dy_ntok < 0");
    DCLIP_HOST_CHECK(lp == nullptr || lp_dt == DCLIP_BF16 || lp_dt == DCLIP_F16,
                     "dclip_layernorm_bwd_res: lp_dt must be F16 or BF16");
    if (rows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (dy_dt == DCLIP_F32)
        bwd_dispatch_x<float>(x_dt, dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows,
                              (int)cols, st);
    else if (dy_dt == DCLIP_F16)
        bwd_dispatch_x<f16>(x_dt, dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows,
                            (int)cols, st);
    else
        bwd_dispatch_x<bf16>(x_dt, dy, dy_scale, dy_ntok, x, w, mean, rstd, res, dx, lp, lp_dt, dw, db, ws, rows,
                             (int)cols, st);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_layernorm_bwd(const void* dy, int dy_dt, const void* x, int x_dt, const float* w,
                                   const float* mean, const float* rstd, float* dx, int accumulate,
                                   float* dw, float* db, int64_t rows, int64_t cols, void* stream) {
    return dclip_layernorm_bwd_res(dy, dy_dt, nullptr, 0, x, x_dt, w, mean, rstd, accumulate ? dx : nullptr, dx, nullptr,
                                   0, dw, db, nullptr, rows, cols, stream);
}
