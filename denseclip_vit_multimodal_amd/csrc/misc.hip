// HBM-bound kernels around the ViT blocks: patchify (im2col), token assembly, positional
// embedding interpolation, the per-layer read-out transpose, global average pool, the
// pixel-text score map, bilinear resize and dtype casts — forward and backward.
// All loads/stores are 8-16 bytes per lane where the layout allows (Guideline 13).
#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ T cvt(float v) { return (T)v; }

// ---------------------------------------------------------------------------- im2col
// out[(b*gh + py)*gw + px][(c*p + ky)*p + kx] = img[b][c][py*p + ky][px*p + kx], rows of ldo
// elements whose columns K = Cin*p*p .. ldo-1 are zero (the GEMM's K padding: p = 14 gives
// K = 588, padded to 640).  p % 4 == 0: one thread per 4 consecutive kx; otherwise one thread
// per output element (patchify is ~0.3 % of the step either way).
template <typename TI, typename TO>
__global__ void im2col_kernel(const TI* __restrict__ img, TO* __restrict__ out, int B, int Cin, int Hin, int Win,
                              int p, int gh, int gw, int64_t ldo, int64_t total4) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int64_t l4 = ldo / 4;
    const int64_t row = i / l4;
    const int col = (int)(i % l4) * 4;
    TO* dst = out + row * ldo + col;
    if (col >= Cin * p * p) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e] = (TO)0.0f;
        return;
    }
    const int kx = col % p, ky = (col / p) % p, cc = col / (p * p);
    const int px = (int)(row % gw);
    const int py = (int)((row / gw) % gh);
    const int b = (int)(row / ((int64_t)gw * gh));
    const TI* src = img + (((int64_t)b * Cin + cc) * Hin + (py * p + ky)) * Win + px * p + kx;
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[e] = (TO)(float)src[e];
}

template <typename TI, typename TO>
__global__ void im2col_any_kernel(const TI* __restrict__ img, TO* __restrict__ out, int B, int Cin, int Hin, int Win,
                                  int p, int gh, int gw, int64_t ldo, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t row = i / ldo;
    const int col = (int)(i % ldo);
    if (col >= Cin * p * p) {
        out[i] = (TO)0.0f;
        return;
    }
    const int kx = col % p, ky = (col / p) % p, cc = col / (p * p);
    const int px = (int)(row % gw);
    const int py = (int)((row / gw) % gh);
    const int b = (int)(row / ((int64_t)gw * gh));
    out[i] = (TO)(float)img[(((int64_t)b * Cin + cc) * Hin + (py * p + ky)) * Win + px * p + kx];
}

// ---------------------------------------------------------------------------- tokens
template <typename TP>
__global__ void tokens_fwd_kernel(const TP* __restrict__ patch, const float* __restrict__ cls,
                                  const float* __restrict__ pos, float* __restrict__ x, int B, int P, int C,
                                  int64_t total4) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int c4 = C / 4;
    const int c = (int)(i % c4) * 4;
    const int64_t row = i / c4;  // b*(P+1) + t
    const int t = (int)(row % (P + 1));
    const int64_t b = row / (P + 1);
    f32x4 pv = *(const f32x4*)(pos + (int64_t)t * C + c);
    f32x4 v;
    if (t == 0) {
        v = *(const f32x4*)(cls + c);
    } else {
        const TP* s = patch + (b * P + (t - 1)) * C + c;
        v[0] = (float)s[0]; v[1] = (float)s[1]; v[2] = (float)s[2]; v[3] = (float)s[3];
    }
    *(f32x4*)(x + row * C + c) = v + pv;
}

template <typename TP>
__global__ void tokens_bwd_kernel(const float* __restrict__ dx, TP* __restrict__ dpatch, Alpha dpatch_scale_arg,
                                  float* __restrict__ dcls, float* __restrict__ dpos, int B, int P, int C,
                                  int64_t total4) {
    const float dpatch_scale = dpatch_scale_arg.get();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (P+1) * C/4
    if (i >= total4) return;
    const int c4 = C / 4;
    const int c = (int)(i % c4) * 4;
    const int t = (int)(i / c4);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
        const f32x4 g = *(const f32x4*)(dx + ((int64_t)b * (P + 1) + t) * C + c);
        acc += g;
        if (t > 0 && dpatch) {
            TP* d = dpatch + ((int64_t)b * P + (t - 1)) * C + c;
            d[0] = (TP)(g[0] * dpatch_scale); d[1] = (TP)(g[1] * dpatch_scale);
            d[2] = (TP)(g[2] * dpatch_scale); d[3] = (TP)(g[3] * dpatch_scale);
        }
    }
    if (dpos) *(f32x4*)(dpos + (int64_t)t * C + c) += acc;
    if (t == 0 && dcls) *(f32x4*)(dcls + c) += acc;
}

// ---------------------------------------------------------------------------- bilinear
// PyTorch upsample_bilinear2d, align_corners=False, output size given:
//   scale = in/out (fp32); src = max(scale*(dst+0.5)-0.5, 0); i0 = (int)src;
//   i1 = i0 + (i0 < in-1); l1 = src - i0; l0 = 1 - l1
struct Lerp {
    int i0, i1;
    float l0, l1;
};
__device__ __forceinline__ Lerp lerp_index(int dst, int in, int out) {
    const float scale = (float)in / (float)out;
    float src = scale * ((float)dst + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    Lerp r;
    r.i0 = (int)src;
    if (r.i0 > in - 1) r.i0 = in - 1;
    r.i1 = r.i0 + (r.i0 < in - 1 ? 1 : 0);
    r.l1 = src - (float)r.i0;
    r.l0 = 1.f - r.l1;
    return r;
}
// weight of source index `i` in the interpolation for output index `dst`
__device__ __forceinline__ float lerp_weight(int dst, int i, int in, int out) {
    const Lerp L = lerp_index(dst, in, out);
    return (L.i0 == i ? L.l0 : 0.f) + (L.i1 == i ? L.l1 : 0.f);
}
// conservative range of output indices whose interpolation touches source index i
__device__ __forceinline__ void lerp_range(int i, int in, int out, int* lo, int* hi) {
    const float inv = (float)out / (float)in;
    int a = (int)floorf(((float)i - 1.f + 0.5f) * inv - 0.5f) - 2;
    int b = (int)ceilf(((float)i + 1.f + 0.5f) * inv - 0.5f) + 2;
    *lo = a < 0 ? 0 : a;
    *hi = b > out - 1 ? out - 1 : b;
}

// one workgroup per (output row, 1024-column segment): the row's vertical lerp once per workgroup
// (scalar), 4 consecutive outputs per thread, 16-byte stores when the row pitch allows.  The
// element-per-thread form (64-bit div / mod per output, 4-byte stores) ran at ~1.1 TB/s on the
// eval-mode 8 x 19 x 1024 x 2048 fp32 logits (`profiles/r03/r04i_*`); the arithmetic per output is
// unchanged (same lerp, same evaluation order: bitwise the same values).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void bilinear_fwd_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t NC,
                                                           int Hi, int Wi, int Ho, int Wo) {
    const int xblocks = (Wo + 1023) / 1024;
    const int64_t row = blockIdx.x / xblocks;  // nc * Ho + y
    const int xb = blockIdx.x - (int)(row * xblocks);
    const int64_t nc = row / Ho;
    const int y = (int)(row - nc * Ho);
    const Lerp ly = lerp_index(y, Hi, Ho);
    const TI* p0 = in + (nc * Hi + ly.i0) * Wi;
    const TI* p1 = in + (nc * Hi + ly.i1) * Wi;
    TO* o = out + row * Wo;
    const int x0 = xb * 1024 + 4 * (int)threadIdx.x;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int x = x0 + e < Wo ? x0 + e : Wo - 1;
        const Lerp lx = lerp_index(x, Wi, Wo);
        const float v00 = (float)p0[lx.i0], v01 = (float)p0[lx.i1];
        const float v10 = (float)p1[lx.i0], v11 = (float)p1[lx.i1];
        v[e] = ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11);
    }
    if (x0 + 4 <= Wo && (Wo & 3) == 0) {
        typedef TO to4 __attribute__((ext_vector_type(4)));
        const to4 w = {(TO)v[0], (TO)v[1], (TO)v[2], (TO)v[3]};
        *(to4*)(o + x0) = w;
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (x0 + e < Wo) o[x0 + e] = (TO)v[e];
    }
}

// pass 1: ws[nc][y][ix] = sum_x w_x(x, ix) dout[nc][y][x]
template <typename TG>
__global__ void bilinear_bwd_w_kernel(const TG* __restrict__ dout, float* __restrict__ ws, int64_t NC, int Wi,
                                      int Ho, int Wo) {
    const int64_t total = NC * Ho * Wi;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int ix = (int)(i % Wi);
        const int64_t row = i / Wi;  // nc*Ho + y
        int lo, hi;
        lerp_range(ix, Wi, Wo, &lo, &hi);
        const TG* g = dout + row * Wo;
        float s = 0.f;
        for (int x = lo; x <= hi; ++x) {
            const float w = lerp_weight(x, ix, Wi, Wo);
            if (w != 0.f) s += w * (float)g[x];
        }
        ws[i] = s;
    }
}
// pass 2: din[nc][iy][ix] = sum_y w_y(y, iy) ws[nc][y][ix]
__global__ void bilinear_bwd_h_kernel(const float* __restrict__ ws, float* __restrict__ din, int64_t NC, int Hi,
                                      int Wi, int Ho) {
    const int64_t total = NC * Hi * Wi;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int ix = (int)(i % Wi);
        const int iy = (int)((i / Wi) % Hi);
        const int64_t nc = i / ((int64_t)Wi * Hi);
        int lo, hi;
        lerp_range(iy, Hi, Ho, &lo, &hi);
        float s = 0.f;
        for (int y = lo; y <= hi; ++y) {
            const float w = lerp_weight(y, iy, Hi, Ho);
            if (w != 0.f) s += w * ws[(nc * Ho + y) * Wi + ix];
        }
        din[i] = s;
    }
}

// ---------------------------------------------------------------------------- pos interp
// out[0] = pos[0]; out[1 + y*W + x][c] = bilinear(pos[1 + (iy*g + ix)][c])
__global__ void pos_interp_fwd_kernel(const float* __restrict__ pos, float* __restrict__ out, int g, int C, int H,
                                      int W) {
    const int64_t total = (int64_t)(H * W + 1) * C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const int t = (int)(i / C);
        if (t == 0) {
            out[i] = pos[c];
            continue;
        }
        const int y = (t - 1) / W, x = (t - 1) % W;
        const Lerp ly = lerp_index(y, g, H), lx = lerp_index(x, g, W);
        const float* p = pos + C;
        const float v00 = p[(ly.i0 * g + lx.i0) * C + c], v01 = p[(ly.i0 * g + lx.i1) * C + c];
        const float v10 = p[(ly.i1 * g + lx.i0) * C + c], v11 = p[(ly.i1 * g + lx.i1) * C + c];
        out[i] = ly.l0 * (lx.l0 * v00 + lx.l1 * v01) + ly.l1 * (lx.l0 * v10 + lx.l1 * v11);
    }
}

__global__ void pos_interp_bwd_kernel(const float* __restrict__ dout, float* __restrict__ dpos, int g, int C, int H,
                                      int W) {
    const int64_t total = (int64_t)(g * g + 1) * C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const int t = (int)(i / C);
        if (t == 0) {
            dpos[i] += dout[c];
            continue;
        }
        const int iy = (t - 1) / g, ix = (t - 1) % g;
        int ylo, yhi, xlo, xhi;
        lerp_range(iy, g, H, &ylo, &yhi);
        lerp_range(ix, g, W, &xlo, &xhi);
        float s = 0.f;
        for (int y = ylo; y <= yhi; ++y) {
            const float wy = lerp_weight(y, iy, g, H);
            if (wy == 0.f) continue;
            for (int x = xlo; x <= xhi; ++x) {
                const float wx = lerp_weight(x, ix, g, W);
                if (wx != 0.f) s += wy * wx * dout[(int64_t)(1 + y * W + x) * C + c];
            }
        }
        dpos[i] += s;
    }
}

// ---------------------------------------------------------------------------- transpose
// out[b][c][r] (=|+=) in[b][r0 + r][c]; zero for rows <= r < rows_pad; colsum[c] += sum
template <typename TI, typename TO, bool ACC>
__global__ __launch_bounds__(256) void transpose_kernel(const TI* __restrict__ in, int64_t in_bs, int64_t in_ld,
                                                        int64_t r0, TO* __restrict__ out, int64_t out_bs,
                                                        int64_t out_ld, int64_t rows, int64_t rows_pad, int64_t cols,
                                                        float* __restrict__ colsum) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z;
    const int64_t rb = (int64_t)blockIdx.y * 64, cb = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    const TI* src = in + b * in_bs;
    for (int k = ty; k < 64; k += 4) {
        const int64_t r = rb + k, c = cb + tx;
        float v = 0.f;
        if (r < rows && c < cols) v = (float)src[(r0 + r) * in_ld + c];
        tile[k][tx] = v;
    }
    __syncthreads();
    if (colsum != nullptr && ty == 0 && cb + tx < cols) {
        float s = 0.f;
        for (int k = 0; k < 64; ++k) s += tile[k][tx];
        atomicAdd(colsum + cb + tx, s);
    }
    TO* dst = out + b * out_bs;
    for (int k = ty; k < 64; k += 4) {
        const int64_t c = cb + k, r = rb + tx;
        if (c < cols && r < rows_pad) {
            const float v = tile[tx][k];
            if constexpr (ACC) dst[c * out_ld + r] += v;
            else dst[c * out_ld + r] = (TO)v;
        }
    }
}

// fp32 (rows, cols) -> 16-bit (cols, rows), both multiples of 64 (the transposed compute-dtype
// weight copies refreshed after every optimizer step): 16-byte loads (4 in flight per thread) and
// 16-byte stores of 8 output elements, through a padded LDS tile.  The generic kernel above moves
// 4 and 2 bytes per lane and reached ~1.3 TB/s on these shapes.
template <typename TO>
__global__ __launch_bounds__(256) void transpose_f32_fast_kernel(const float* __restrict__ in, int64_t in_ld,
                                                                 TO* __restrict__ out, int64_t out_ld) {
    __shared__ float tile[64][65];
    const int64_t rb = (int64_t)blockIdx.y * 64, cb = (int64_t)blockIdx.x * 64;
    const int t = threadIdx.x;
    const int c4 = t & 15, r = t >> 4;
    f32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = *(const f32x4*)(in + (rb + r + 16 * i) * in_ld + cb + 4 * c4);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[r + 16 * i][4 * c4 + e] = v[i][e];
    __syncthreads();
    const int j = t & 7, oc = t >> 3;
    typedef TO to8 __attribute__((ext_vector_type(8)));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int c = oc + 32 * i;
        to8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (TO)tile[8 * j + e][c];
        *(to8*)(out + (cb + c) * out_ld + rb + 8 * j) = o;
    }
}

// ---------------------------------------------------------------------------- weight refresh
// After an optimizer step every cached compute-dtype copy of a stepped fp32 weight (ops.WEIGHTS:
// the plain (rows, cols) copy the forward GEMMs read and the (cols, rows) transposed copy of the
// dX GEMMs) is rewritten in place by ONE launch over all weights: a workgroup per 64 x 64 tile of
// one weight reads the fp32 tile once and writes both copies (the transposed one through LDS).
// Entry e of the device descriptor (8 int64): src, plain dst (0: none), transposed dst (0: none),
// rows, cols, first tile, column tiles, unused.  Replaces ~120 per-weight cast / transpose
// launches per step.
template <typename TO>
__global__ __launch_bounds__(256) void weight_refresh_kernel(const int64_t* __restrict__ desc, int n) {
    __shared__ float tile[64][65];
    const int64_t blk = blockIdx.x;
    int lo = 0, hi = n - 1;  // the entry whose tile range holds this block
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (desc[(int64_t)mid * 8 + 5] <= blk) lo = mid;
        else hi = mid - 1;
    }
    const int64_t* d = desc + (int64_t)lo * 8;
    const float* __restrict__ src = (const float*)d[0];
    TO* __restrict__ dp = (TO*)d[1];
    TO* __restrict__ dt = (TO*)d[2];
    const int64_t rows = d[3], cols = d[4], local = blk - d[5], tcn = d[6];
    const int64_t rb = (local / tcn) * 64, cb = (local % tcn) * 64;
    const int t = threadIdx.x, c4 = t & 15, r = t >> 4;
    const bool vec = (cols & 3) == 0;  // 16-byte source rows / 8-byte plain stores
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t row = rb + r + 16 * i, col = cb + 4 * c4;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (row < rows) {
            if (vec && col + 4 <= cols) {
                v = *(const f32x4*)(src + row * cols + col);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (col + e < cols) v[e] = src[row * cols + col + e];
            }
            if (dp != nullptr) {
                if (vec && col + 4 <= cols) {
                    typedef TO to4 __attribute__((ext_vector_type(4)));
                    const to4 o = {(TO)v[0], (TO)v[1], (TO)v[2], (TO)v[3]};
                    *(to4*)(dp + row * cols + col) = o;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (col + e < cols) dp[row * cols + col + e] = (TO)v[e];
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[r + 16 * i][4 * c4 + e] = v[e];
    }
    if (dt == nullptr) return;  // block-uniform
    __syncthreads();
    // transposed copy (cols, rows): row c of it = column c of the tile, 8 source rows per lane
    const int j = t & 7, oc = t >> 3;
    const bool tvec = (rows & 7) == 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int c = oc + 32 * i;
        const int64_t gc = cb + c, gr = rb + 8 * j;
        if (gc >= cols || gr >= rows) continue;
        if (tvec && gr + 8 <= rows) {
            typedef TO to8 __attribute__((ext_vector_type(8)));
            to8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (TO)tile[8 * j + e][c];
            *(to8*)(dt + gc * rows + gr) = o;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (gr + e < rows) dt[gc * rows + gr + e] = (TO)tile[8 * j + e][c];
        }
    }
}

// ---------------------------------------------------------------------------- row mean
// F.adaptive_avg_pool2d(x, 1) of a pixel-row map (denseclip.py:596) read in place from a strided
// row layout (the ViT token buffer: batch stride N*C, row offset 1 skips CLS).  Stage 1: one
// workgroup per (image, chunk of rows) streams its rows with 16-byte loads (a 768-channel row =
// 96 lanes, 256 / 96 rows per pass), RM_BATCH rows per thread loaded before any is summed so
// that ~24 KiB per workgroup are in flight (HBM rate, not load latency), and writes the chunk's
// column sums; stage 2 sums the chunks in a fixed order (deterministic) and divides.
constexpr int RM_CHUNK = 128;  // rows per workgroup
constexpr int RM_BATCH = 8;    // loads in flight per thread

template <typename TI>
__global__ __launch_bounds__(256) void row_mean_part_kernel(const TI* __restrict__ x, int64_t bstride, int64_t row_off,
                                                            int64_t ld, int64_t rows, int C, float* __restrict__ ws) {
    typedef TI t8 __attribute__((ext_vector_type(8)));
    __shared__ float red[2048 / 8 * 8];
    const int b = blockIdx.y, ch = blockIdx.x, S = gridDim.x;
    const int nc8 = C / 8, nrp = 256 / nc8;
    const int t = threadIdx.x, cc = t % nc8, rp = t / nc8;
    const int64_t r0 = (int64_t)ch * RM_CHUNK;
    const int64_t r1 = r0 + RM_CHUNK < rows ? r0 + RM_CHUNK : rows;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (rp < nrp) {
        const TI* base = x + (int64_t)b * bstride + row_off * ld + cc * 8;
        for (int64_t r = r0 + rp; r < r1; r += RM_BATCH * nrp) {
            t8 v[RM_BATCH];
#pragma unroll
            for (int i = 0; i < RM_BATCH; ++i) {
                const int64_t ri = r + (int64_t)i * nrp;
                v[i] = ri < r1 ? *(const t8*)(base + ri * ld) : t8{};
            }
#pragma unroll
            for (int i = 0; i < RM_BATCH; ++i)
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] += (float)v[i][e];
        }
    }
    // reduce the nrp row phases of each column chunk through LDS (phase 0 keeps, the others add)
    for (int p = 1; p < nrp; ++p) {
        if (rp == p)
#pragma unroll
            for (int e = 0; e < 8; ++e) red[cc * 8 + e] = a[e];
        __syncthreads();
        if (rp == 0)
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] += red[cc * 8 + e];
        __syncthreads();
    }
    if (rp == 0) {
        float* o = ws + ((int64_t)b * S + ch) * C + cc * 8;
        *(f32x4*)o = f32x4{a[0], a[1], a[2], a[3]};
        *(f32x4*)(o + 4) = f32x4{a[4], a[5], a[6], a[7]};
    }
}

__global__ __launch_bounds__(256) void row_mean_final_kernel(const float* __restrict__ ws, int S, int C, int64_t rows,
                                                             int B, float* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= B * C) return;
    const int b = i / C, c = i % C;
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += ws[((int64_t)b * S + k) * C + c];
    out[i] = s / (float)rows;
}

// ---------------------------------------------------------------------------- score map
// s[b][k][p] = <v_p / max(|v_p|, eps), t_k / max(|t_k|, eps)> (F.normalize x2 + einsum
// 'bchw,bkc->bkhw', denseclip.py:672-675) as a batched [K x C] . [C x 32-pixel] MFMA product:
// A = the normalised class embeddings (K <= 32 rows, 16-bit, LDS, rows padded by 16 B so the
// row-fragment reads are bank-conflict free), B = 32 pixel rows of v read in place (strided rows:
// the vis_proj GEMM's output over the token buffer, CLS rows skipped), D[class][pixel] with the
// pixel on the lane, so the pixel norm (accumulated from the same B fragments) is lane-local.
template <typename TV>
__global__ __launch_bounds__(256) void score_map_kernel(const TV* __restrict__ v, int64_t bstride, int64_t row_off,
                                                        int64_t ld, const float* __restrict__ t,
                                                        float* __restrict__ score, int HW, int C, int K, float eps) {
    typedef typename Mfma<TV>::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [32][C + 8] TV
    TV* tn = (TV*)smem;
    const int pitch = C + 8;
    const int b = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l32 = lane & 31, h = lane >> 5;
    // class-embedding norms (a wave per row: each lane's 16-byte chunks in order, then the wave's
    // fixed butterfly; no LDS atomics, so the norms repeat bit for bit), then the normalised
    // 16-bit rows from cache
    __shared__ float nrm[32];
    const f32x4* tb = (const f32x4*)(t + (int64_t)b * K * C);
    const int c4 = C / 4;
    for (int k = wave; k < K; k += 4) {
        float ss = 0.f;
        for (int j = lane; j < c4; j += 64) {
            const f32x4 x = tb[k * c4 + j];
            ss += x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
        }
        ss = wave_sum(ss);
        if (lane == 0) nrm[k] = ss;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * c4; i += 256) {
        const int k = i / c4, c = 4 * (i - k * c4);
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (k < K) x = tb[i] * (1.f / fmaxf(sqrtf(nrm[k]), eps));
        typedef TV t4 __attribute__((ext_vector_type(4)));
        *(t4*)(tn + k * pitch + c) = t4{(TV)x[0], (TV)x[1], (TV)x[2], (TV)x[3]};
    }
    __syncthreads();
    // one 32-pixel group per workgroup, its channels split over the 4 waves (16-channel MFMA steps
    // [w S / 4, (w + 1) S / 4)): 4x the loads in flight of one wave sweeping all C, then the
    // partial products and norms summed through LDS in a fixed order
    float* red = (float*)(smem + (size_t)32 * pitch * sizeof(TV));  // [3][17][64]
    const int nsteps = C / 16, s0 = wave * nsteps / 4, s1 = (wave + 1) * nsteps / 4;
    const int p = blockIdx.x * 32 + l32;
    const int pc = p < HW ? p : HW - 1;
    const TV* row = v + (int64_t)b * bstride + (row_off + pc) * ld + 8 * h;
    const TV* arow = tn + l32 * pitch + 8 * h;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    float ss = 0.f;
#pragma unroll 8
    for (int s = s0; s < s1; ++s) {
        const frag bf = *(const frag*)(row + 16 * s);
        const frag af = *(const frag*)(arow + 16 * s);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += (float)bf[j] * (float)bf[j];
        acc = Mfma<TV>::mma(af, bf, acc);
    }
    if (wave > 0) {
        float* r = red + (wave - 1) * 17 * 64;
#pragma unroll
        for (int e = 0; e < 16; ++e) r[e * 64 + lane] = acc[e];
        r[16 * 64 + lane] = ss;
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
        for (int w = 0; w < 3; ++w) {
            const float* r = red + w * 17 * 64;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] += r[e * 64 + lane];
            ss += r[16 * 64 + lane];
        }
        ss += __shfl_xor(ss, 32, 64);  // the other half-wave holds the pixel's other 8-column chunks
        const float inv = 1.f / fmaxf(sqrtf(ss), eps);
        if (p < HW) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
                if (k < K) score[((int64_t)b * K + k) * HW + p] = acc[r] * inv;
            }
        }
    }
}

// ---------------------------------------------------------------------------- gradient scale
// Power-of-two scale of an fp32 gradient for its fp16 cast, on the device (no host read):
//   ws[0] = s = 2^clamp(floor(log2(target / amax|g|)), -60, 60), ws[1] = 1/s  (s = 1 when amax is
//   0 or not finite); ws[2] = running amax bits, ws[3] = finished-workgroup count (both zero on
//   entry, zero again on exit: the last workgroup to finish computes s and resets them).
// |g| as uint32 bits orders like the float (non-negative), NaN / inf sort above every finite value.
// the workgroup's |x| maximum (as uint32 bits) joined into ws[2]; the last workgroup to finish
// turns it into ws[0] = s, ws[1] = 1/s and clears ws[2], ws[3] for the next use
__device__ __forceinline__ void amax_finish(uint32_t m, float target, float* __restrict__ ws) {
    scale_finish<4>(m, target, ws);
}

// four 16-B loads in flight per thread and iteration (one at a time reached 2.2 TB/s on 201 MB)
__global__ __launch_bounds__(256) void grad_scale_kernel(const float* __restrict__ g, int64_t n, float target,
                                                         float* __restrict__ ws) {
    uint32_t m = 0;
    const int64_t n4 = n / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const f32x4*)(g + 4 * (i + u * stride));
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) m = max(m, __float_as_uint(v[u][e]) & 0x7fffffffu);
    }
    for (; i < n4; i += stride) {
        const f32x4 v = *(const f32x4*)(g + 4 * i);
#pragma unroll
        for (int e = 0; e < 4; ++e) m = max(m, __float_as_uint(v[e]) & 0x7fffffffu);
    }
    if (blockIdx.x == 0)
        for (int64_t j = 4 * n4 + threadIdx.x; j < n; j += blockDim.x) m = max(m, __float_as_uint(g[j]) & 0x7fffffffu);
    amax_finish(m, target, ws);
}

extern "C" int dclip_grad_scale(const float* g, int64_t n, float target, float* ws, void* stream) {
    DCLIP_HOST_CHECK(n >= 0 && ws != nullptr && target > 0.f, "dclip_grad_scale: bad arguments");
    DCLIP_HOST_CHECK(((uintptr_t)g % 16) == 0, "dclip_grad_scale: g must be 16-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    // every workgroup ends in one atomic on the same two words: a few hundred workgroups, not
    // thousands (the fan-in costs ~13 ns per arrival under load)
    int64_t blocks = (n / 4 + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 512 ? 512 : blocks);
    grad_scale_kernel<<<(unsigned)blocks, 256, 0, st>>>(g, n, target, ws);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------- stochastic depth
// out[r][c] = (x ? x[r][c] : 0) + s[r % ntok] * y[r][c]: a residual branch scaled by a per-TOKEN
// keep mask (timm drop_path on the reference's LND layout draws one value per token position,
// shared by the batch: models.py:257-268, 291-294), and the same scaling for its gradient.
__global__ void row_scale_add_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                     const float* __restrict__ s, float* __restrict__ out, int64_t rows, int cols,
                                     int ntok) {
    const int c4 = cols / 4;
    const int64_t total = rows * c4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / c4;
        const float sc = s[r % ntok];
        f32x4 v = *(const f32x4*)(y + 4 * i) * sc;
        if (x) v += *(const f32x4*)(x + 4 * i);
        *(f32x4*)(out + 4 * i) = v;
    }
}

extern "C" int dclip_row_scale_add(const float* x, const float* y, const float* s, int ntok, float* out, int64_t rows,
                                   int cols, void* stream) {
    DCLIP_HOST_CHECK(y && s && out && ntok > 0 && rows >= 0 && cols % 4 == 0 && rows % ntok == 0,
                     "dclip_row_scale_add: bad arguments (cols %% 4 == 0, rows a multiple of ntok)");
    if (rows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int64_t blocks = (rows * (cols / 4) + 255) / 256;
    row_scale_add_kernel<<<(unsigned)(blocks < 65536 ? blocks : 65536), 256, 0, st>>>(x, y, s, out, rows, cols, ntok);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------- cast
template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, int64_t n, Alpha scale_arg) {
    const float scale = scale_arg.get();
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
         i += (int64_t)gridDim.x * blockDim.x * 4) {
        if (i + 3 < n) {
#pragma unroll
            for (int e = 0; e < 4; ++e) out[i + e] = (TO)((float)in[i + e] * scale);
        } else {
            for (int64_t j = i; j < n; ++j) out[j] = (TO)((float)in[j] * scale);
        }
    }
}

inline unsigned grid_for(int64_t n, int64_t cap = 65536) {
    int64_t g = (n + 255) / 256;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}

#define DISPATCH_DT(dt, T, ...)                                  \
    do {                                                         \
        if ((dt) == DCLIP_F32) { typedef float T; __VA_ARGS__; } \
        else if ((dt) == DCLIP_F16) { typedef f16 T; __VA_ARGS__; } \
        else { typedef bf16 T; __VA_ARGS__; }                    \
    } while (0)

}  // namespace

extern "C" int dclip_im2col(const void* img, int img_dt, void* out, int out_dt, int64_t ldo, int B, int Cin, int Hin,
                            int Win, int p, void* stream) {
    DCLIP_HOST_CHECK(p > 0, "dclip_im2col: patch size must be positive");
    const int gh = Hin / p, gw = Win / p;
    DCLIP_HOST_CHECK(gh > 0 && gw > 0, "dclip_im2col: image smaller than one patch");
    DCLIP_HOST_CHECK(ldo >= (int64_t)Cin * p * p && ldo % 4 == 0,
                     "dclip_im2col: ldo must be >= Cin*p*p and a multiple of 4");
    const int64_t rows = (int64_t)B * gh * gw;
    hipStream_t st = (hipStream_t)stream;
    if (p % 4 == 0) {
        const int64_t total4 = rows * ldo / 4;
        DISPATCH_DT(img_dt, TI, DISPATCH_DT(out_dt, TO,
            im2col_kernel<TI, TO><<<(unsigned)((total4 + 255) / 256), 256, 0, st>>>((const TI*)img, (TO*)out, B, Cin,
                                                                                 Hin, Win, p, gh, gw, ldo, total4)));
    } else {
        const int64_t total = rows * ldo;
        DISPATCH_DT(img_dt, TI, DISPATCH_DT(out_dt, TO,
            im2col_any_kernel<TI, TO><<<(unsigned)((total + 255) / 256), 256, 0, st>>>((const TI*)img, (TO*)out, B,
                                                                                    Cin, Hin, Win, p, gh, gw, ldo,
                                                                                    total)));
    }
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_tokens_fwd(const void* patch, int patch_dt, const float* cls, const float* pos, float* x, int B,
                                int P, int C, void* stream) {
    DCLIP_HOST_CHECK(C % 4 == 0, "dclip_tokens_fwd: C %% 4 != 0");
    const int64_t total4 = (int64_t)B * (P + 1) * C / 4;
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_DT(patch_dt, TP,
        tokens_fwd_kernel<TP><<<(unsigned)((total4 + 255) / 256), 256, 0, st>>>((const TP*)patch, cls, pos, x, B, P,
                                                                             C, total4));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_tokens_bwd(const float* dx, void* dpatch, int dpatch_dt, float dpatch_scale_v,
                                const float* dpatch_scale_ptr, float* dcls, float* dpos, int B, int P, int C,
                                void* stream) {
    const Alpha dpatch_scale(dpatch_scale_v, dpatch_scale_ptr);
    DCLIP_HOST_CHECK(C % 4 == 0, "dclip_tokens_bwd: C %% 4 != 0");
    const int64_t total4 = (int64_t)(P + 1) * C / 4;
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_DT(dpatch_dt, TP,
        tokens_bwd_kernel<TP><<<(unsigned)((total4 + 255) / 256), 256, 0, st>>>(dx, (TP*)dpatch, dpatch_scale, dcls, dpos, B, P, C,
                                                                             total4));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_pos_interp_fwd(const float* pos, float* out, int g, int C, int H, int W, void* stream) {
    DCLIP_HOST_CHECK(g > 0 && H > 0 && W > 0, "dclip_pos_interp_fwd: bad sizes");
    const int64_t total = (int64_t)(H * W + 1) * C;
    pos_interp_fwd_kernel<<<grid_for(total), 256, 0, (hipStream_t)stream>>>(pos, out, g, C, H, W);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_pos_interp_bwd(const float* dout, float* dpos, int g, int C, int H, int W, void* stream) {
    DCLIP_HOST_CHECK(g > 0 && H > 0 && W > 0, "dclip_pos_interp_bwd: bad sizes");
    const int64_t total = (int64_t)(g * g + 1) * C;
    pos_interp_bwd_kernel<<<grid_for(total), 256, 0, (hipStream_t)stream>>>(dout, dpos, g, C, H, W);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_weight_refresh(const int64_t* desc, int n, int64_t tiles, int out_dt, void* stream) {
    DCLIP_HOST_CHECK(desc != nullptr && n > 0 && tiles > 0, "dclip_weight_refresh: empty descriptor");
    DCLIP_HOST_CHECK(out_dt == DCLIP_BF16 || out_dt == DCLIP_F16, "dclip_weight_refresh: 16-bit copies only");
    DCLIP_HOST_CHECK(tiles < (1ll << 31), "dclip_weight_refresh: too many tiles");
    hipStream_t st = (hipStream_t)stream;
    if (out_dt == DCLIP_BF16) weight_refresh_kernel<bf16><<<(unsigned)tiles, 256, 0, st>>>(desc, n);
    else weight_refresh_kernel<f16><<<(unsigned)tiles, 256, 0, st>>>(desc, n);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_transpose(const void* in, int in_dt, int64_t in_bstride, int64_t in_ld, int64_t r0, void* out,
                               int out_dt, int64_t out_bstride, int64_t out_ld, int batch, int64_t rows,
                               int64_t rows_pad, int64_t cols, int accumulate, float* colsum, void* stream) {
    DCLIP_HOST_CHECK(rows_pad >= rows && batch > 0, "dclip_transpose: rows_pad < rows");
    DCLIP_HOST_CHECK(!accumulate || out_dt == DCLIP_F32, "dclip_transpose: accumulate needs f32 output");
    if (rows_pad == 0 || cols == 0) return 0;
    dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows_pad + 63) / 64), batch);
    hipStream_t st = (hipStream_t)stream;
    const bool fast = !accumulate && colsum == nullptr && batch == 1 && r0 == 0 && in_dt == DCLIP_F32 &&
                      (out_dt == DCLIP_BF16 || out_dt == DCLIP_F16) && rows == rows_pad && rows % 64 == 0 && cols % 64 == 0 &&
                      in_ld % 4 == 0 && out_ld % 8 == 0 && ((uintptr_t)in | (uintptr_t)out) % 16 == 0;
    if (fast) {
        if (out_dt == DCLIP_BF16)
            transpose_f32_fast_kernel<bf16><<<grid, 256, 0, st>>>((const float*)in, in_ld, (bf16*)out, out_ld);
        else
            transpose_f32_fast_kernel<f16><<<grid, 256, 0, st>>>((const float*)in, in_ld, (f16*)out, out_ld);
    } else if (accumulate) {
        DISPATCH_DT(in_dt, TI,
            transpose_kernel<TI, float, true><<<grid, 256, 0, st>>>((const TI*)in, in_bstride, in_ld, r0, (float*)out,
                                                                   out_bstride, out_ld, rows, rows_pad, cols, colsum));
    } else {
        DISPATCH_DT(in_dt, TI, DISPATCH_DT(out_dt, TO,
            transpose_kernel<TI, TO, false><<<grid, 256, 0, st>>>((const TI*)in, in_bstride, in_ld, r0, (TO*)out,
                                                                 out_bstride, out_ld, rows, rows_pad, cols, colsum)));
    }
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int64_t dclip_row_mean_workspace(int B, int64_t rows, int C) {
    return (int64_t)B * ((rows + RM_CHUNK - 1) / RM_CHUNK) * C;
}

extern "C" int dclip_row_mean(const void* x, int x_dt, int64_t bstride, int64_t row_off, int64_t ld, int B, int64_t rows,
                              int C, float* ws, float* out, void* stream) {
    DCLIP_HOST_CHECK(rows > 0 && C > 0 && B > 0, "dclip_row_mean: empty input");
    DCLIP_HOST_CHECK(x_dt != DCLIP_F32, "dclip_row_mean: 16-bit input");
    DCLIP_HOST_CHECK(C % 8 == 0 && C <= 2048 && ld % 8 == 0 && bstride % 8 == 0 && ((uintptr_t)x % 16) == 0,
                     "dclip_row_mean: C %% 8 == 0, C <= 2048, 16-byte aligned rows");
    const int S = (int)((rows + RM_CHUNK - 1) / RM_CHUNK);
    hipStream_t st = (hipStream_t)stream;
    if (x_dt == DCLIP_BF16)
        row_mean_part_kernel<bf16><<<dim3(S, B), 256, 0, st>>>((const bf16*)x, bstride, row_off, ld, rows, C, ws);
    else
        row_mean_part_kernel<f16><<<dim3(S, B), 256, 0, st>>>((const f16*)x, bstride, row_off, ld, rows, C, ws);
    row_mean_final_kernel<<<(B * C + 255) / 256, 256, 0, st>>>(ws, S, C, rows, B, out);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_score_map(const void* v, int v_dt, int64_t bstride, int64_t row_off, int64_t ld, const float* t,
                               float* score, int B, int HW, int C, int K, float eps, void* stream) {
    DCLIP_HOST_CHECK(K > 0 && K <= 32, "dclip_score_map: K must be in [1, 32] (got %d)", K);
    DCLIP_HOST_CHECK(v_dt == DCLIP_BF16 || v_dt == DCLIP_F16, "dclip_score_map: v must be f16/bf16");
    DCLIP_HOST_CHECK(C % 16 == 0 && C <= 2048 && ld % 8 == 0 && bstride % 8 == 0 && ((uintptr_t)v % 16) == 0,
                     "dclip_score_map: C %% 16 == 0, C <= 2048, 16-byte aligned rows");
    DCLIP_HOST_CHECK(B > 0 && HW > 0, "dclip_score_map: empty input");
    const int bx = (HW + 31) / 32;
    const size_t lds = (size_t)32 * (C + 8) * 2 + 3 * 17 * 64 * sizeof(float);
    hipStream_t st = (hipStream_t)stream;
    if (v_dt == DCLIP_BF16)
        score_map_kernel<bf16><<<dim3(bx, B), 256, lds, st>>>((const bf16*)v, bstride, row_off, ld, t, score, HW, C, K,
                                                              eps);
    else
        score_map_kernel<f16><<<dim3(bx, B), 256, lds, st>>>((const f16*)v, bstride, row_off, ld, t, score, HW, C, K,
                                                             eps);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------- score concat
// torch.cat([x_i, F.interpolate(score, x_i's size, bilinear).to(x_i.dtype)], dim=1) of the
// score_concat_index branch (denseclip.py:684-694) in ONE pass: every output pixel row (channels
// last, C + K wide) gets the read-out map's C channels copied from its strided token row and the K
// score channels interpolated with bilinear_fwd_kernel's arithmetic (bitwise the same values) —
// no resized score map and no separate concatenation copy in HBM.  One wave per pixel row.
template <typename T>
__global__ __launch_bounds__(256) void score_concat_kernel(const T* __restrict__ rows, int64_t bstride, int64_t row_off,
                                                           int64_t ld, int C, const float* __restrict__ score, int K,
                                                           int hs, int ws, T* __restrict__ out, int B, int h, int w) {
    const int64_t npix = (int64_t)B * h * w;
    const int CK = C + K;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t p = (int64_t)blockIdx.x * 4 + wave; p < npix; p += (int64_t)gridDim.x * 4) {
        const int64_t b = p / ((int64_t)h * w);
        const int rem = (int)(p - b * h * w);
        const int y = rem / w, x = rem - y * w;
        const T* src = rows + b * bstride + (row_off + rem) * ld;
        T* dst = out + p * CK;
        for (int c = lane; c < C; c += 64) dst[c] = src[c];
        if (lane < K) {
            const Lerp ly = lerp_index(y, hs, h), lx = lerp_index(x, ws, w);
            const float* pl = score + ((int64_t)b * K + lane) * hs * ws;
            const float* p0 = pl + (int64_t)ly.i0 * ws;
            const float* p1 = pl + (int64_t)ly.i1 * ws;
            const float v = ly.l0 * (lx.l0 * p0[lx.i0] + lx.l1 * p0[lx.i1]) + ly.l1 * (lx.l0 * p1[lx.i0] + lx.l1 * p1[lx.i1]);
            dst[C + lane] = (T)v;
        }
    }
}

extern "C" int dclip_score_concat(const void* rows, int dt, int64_t bstride, int64_t row_off, int64_t ld, int C,
                                  const float* score, int K, int hs, int ws, void* out, int B, int h, int w,
                                  void* stream) {
    DCLIP_HOST_CHECK(rows && score && out && B > 0 && h > 0 && w > 0 && C > 0 && hs > 0 && ws > 0,
                     "dclip_score_concat: bad arguments");
    DCLIP_HOST_CHECK(K > 0 && K <= 64, "dclip_score_concat: 1 <= K <= 64 score channels (one lane each)");
    DCLIP_HOST_CHECK(dt == DCLIP_BF16 || dt == DCLIP_F16, "dclip_score_concat: 16-bit maps");
    const int64_t npix = (int64_t)B * h * w;
    const int blocks = (int)((npix + 3) / 4 > 8192 ? 8192 : (npix + 3) / 4);
    hipStream_t st = (hipStream_t)stream;
    if (dt == DCLIP_BF16)
        score_concat_kernel<bf16><<<blocks, 256, 0, st>>>((const bf16*)rows, bstride, row_off, ld, C, score, K, hs, ws,
                                                          (bf16*)out, B, h, w);
    else
        score_concat_kernel<f16><<<blocks, 256, 0, st>>>((const f16*)rows, bstride, row_off, ld, C, score, K, hs, ws,
                                                         (f16*)out, B, h, w);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_bilinear_fwd(const void* in, int in_dt, void* out, int out_dt, int64_t NC, int Hi, int Wi, int Ho,
                                  int Wo, void* stream) {
    DCLIP_HOST_CHECK(Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "dclip_bilinear_fwd: bad sizes");
    const int64_t blocks = NC * Ho * ((Wo + 1023) / 1024);
    DCLIP_HOST_CHECK(blocks < (1ll << 31), "dclip_bilinear_fwd: output too large");
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_DT(in_dt, TI, DISPATCH_DT(out_dt, TO,
        bilinear_fwd_kernel<TI, TO><<<(unsigned)blocks, 256, 0, st>>>((const TI*)in, (TO*)out, NC, Hi, Wi, Ho, Wo)));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_bilinear_bwd(const void* dout, int dout_dt, float* din, float* ws, int64_t NC, int Hi, int Wi,
                                  int Ho, int Wo, void* stream) {
    DCLIP_HOST_CHECK(Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "dclip_bilinear_bwd: bad sizes");
    hipStream_t st = (hipStream_t)stream;
    const int64_t t1 = NC * Ho * Wi;
    DISPATCH_DT(dout_dt, TG,
        bilinear_bwd_w_kernel<TG><<<grid_for(t1), 256, 0, st>>>((const TG*)dout, ws, NC, Wi, Ho, Wo));
    const int64_t t2 = NC * Hi * Wi;
    bilinear_bwd_h_kernel<<<grid_for(t2), 256, 0, st>>>(ws, din, NC, Hi, Wi, Ho);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// sum = a + b (b's CLS rows, row % ntok == 0, read as 0) and lp = (TO)(sum * scale), 8 columns
// per thread with 16-byte accesses; cols % 8 == 0.  sum may alias a.
template <typename TB, typename TO>
__global__ void add_readout_cast_kernel(const float* a, const TB* __restrict__ b, float* sum, TO* __restrict__ lp,
                                        int64_t rows, int cols, int ntok, float scale) {
    const int c8 = cols / 8;
    const int64_t n8 = rows * c8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / c8;
        const int64_t off = i * 8;
        f32x4 x0 = *(const f32x4*)(a + off), x1 = *(const f32x4*)(a + off + 4);
        if (row % ntok != 0) {
            if constexpr (sizeof(TB) == 4) {
                const f32x4 y0 = *(const f32x4*)(b + off), y1 = *(const f32x4*)(b + off + 4);
                x0 += y0;
                x1 += y1;
            } else {
                typedef TB tb8 __attribute__((ext_vector_type(8)));
                const tb8 y = *(const tb8*)(b + off);
#pragma unroll
                for (int e = 0; e < 4; ++e) x0[e] += (float)y[e], x1[e] += (float)y[4 + e];
            }
        }
        *(f32x4*)(sum + off) = x0;
        *(f32x4*)(sum + off + 4) = x1;
        typedef TO to8 __attribute__((ext_vector_type(8)));
        to8 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (TO)(x0[e] * scale), o[4 + e] = (TO)(x1[e] * scale);
        *(to8*)(lp + off) = o;
    }
}

extern "C" int dclip_add_readout_cast(const float* a, const void* b, int b_dt, float* sum, void* lp, int lp_dt,
                                      int64_t rows, int cols, int ntok, float scale, void* stream) {
    DCLIP_HOST_CHECK(cols % 8 == 0 && ntok > 0, "dclip_add_readout_cast: cols must be a multiple of 8");
    DCLIP_HOST_CHECK(lp_dt == DCLIP_BF16 || lp_dt == DCLIP_F16, "dclip_add_readout_cast: lp must be bf16/f16");
    DCLIP_HOST_CHECK(((uintptr_t)a | (uintptr_t)b | (uintptr_t)sum | (uintptr_t)lp) % 16 == 0,
                     "dclip_add_readout_cast: unaligned buffers");
    if (rows == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = grid_for(rows * (cols / 8), 8192);
    DISPATCH_DT(b_dt, TB, DISPATCH_DT(lp_dt, TO,
        if constexpr (sizeof(TO) == 2)
            add_readout_cast_kernel<TB, TO><<<g, 256, 0, st>>>(a, (const TB*)b, sum, (TO*)lp, rows, cols, ntok, scale)));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// The fp16 backward's block-input gradient: sum = a + b * (*bsc) with b's CLS rows read as 0
// (the read-out map's gradient joining the block output's, as dclip_add_readout_cast) and, in
// the same pass, the power-of-two scale of sum for its fp16 cast (dclip_grad_scale's ws
// protocol).  Replaces a 16->32-bit copy, the CLS zeroing, the HeadScale unscale, the add and
// the separate amax pass over sum.
template <typename TB>
__global__ __launch_bounds__(256) void add_readout_amax_kernel(const float* a, const TB* __restrict__ b,
                                                               const float* __restrict__ bsc, float* sum,
                                                               int64_t rows, int cols, int ntok, float target,
                                                               float* __restrict__ ws) {
    const int c8 = cols / 8;
    const int64_t n8 = rows * c8;
    const float sb = bsc != nullptr ? *bsc : 1.0f;
    uint32_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / c8;
        const int64_t off = i * 8;
        f32x4 x0 = *(const f32x4*)(a + off), x1 = *(const f32x4*)(a + off + 4);
        if (row % ntok != 0) {
            if constexpr (sizeof(TB) == 4) {
                x0 += *(const f32x4*)(b + off) * sb;
                x1 += *(const f32x4*)(b + off + 4) * sb;
            } else {
                typedef TB tb8 __attribute__((ext_vector_type(8)));
                const tb8 y = *(const tb8*)(b + off);
#pragma unroll
                for (int e = 0; e < 4; ++e) x0[e] += (float)y[e] * sb, x1[e] += (float)y[4 + e] * sb;
            }
        }
        *(f32x4*)(sum + off) = x0;
        *(f32x4*)(sum + off + 4) = x1;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            m = max(m, max(__float_as_uint(x0[e]) & 0x7fffffffu, __float_as_uint(x1[e]) & 0x7fffffffu));
    }
    amax_finish(m, target, ws);
}

extern "C" int dclip_add_readout_amax(const float* a, const void* b, int b_dt, const float* b_scale_ptr, float* sum,
                                      int64_t rows, int cols, int ntok, float target, float* ws, void* stream) {
    DCLIP_HOST_CHECK(cols % 8 == 0 && ntok > 0 && rows >= 0 && ws != nullptr && target > 0.f,
                     "dclip_add_readout_amax: cols %% 8 == 0, ntok > 0, a workspace and target > 0");
    DCLIP_HOST_CHECK(((uintptr_t)a | (uintptr_t)b | (uintptr_t)sum) % 16 == 0, "dclip_add_readout_amax: unaligned buffers");
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = rows == 0 ? 1u : grid_for(rows * (cols / 8), 512);  // the fan-in (dclip_grad_scale)
    DISPATCH_DT(b_dt, TB,
        add_readout_amax_kernel<TB><<<g, 256, 0, st>>>(a, (const TB*)b, b_scale_ptr, sum, rows, cols, ntok, target, ws));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// The fp16 backward's block-input gradient on a DELAYED scale: sum = a (+ b * (*bsc), b's CLS
// rows read as 0; b may be null) and lp = (f16)(sum * s) in one pass, s the scale of this
// gradient site's previous use (common.h ds_*: use `use` of the state st), (s, 1/s) to spair
// for lp's consumers and this use's |sum| maximum joined into st for the next use.  One pass
// where the exact scale needs two (the maximum, then the cast); two 8-column chunks per thread
// and iteration, their loads issued together.
template <typename TB>
__device__ __forceinline__ void readout_sum8(const float* a, const TB* b, float sb, int64_t off, bool keep,
                                             f32x4& x0, f32x4& x1) {
    x0 = *(const f32x4*)(a + off);
    x1 = *(const f32x4*)(a + off + 4);
    if (b != nullptr && keep) {
        if constexpr (sizeof(TB) == 4) {
            x0 += *(const f32x4*)(b + off) * sb;
            x1 += *(const f32x4*)(b + off + 4) * sb;
        } else {
            typedef TB tb8 __attribute__((ext_vector_type(8)));
            const tb8 y = *(const tb8*)(b + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) x0[e] += (float)y[e] * sb, x1[e] += (float)y[4 + e] * sb;
        }
    }
}

template <typename TB>
__global__ __launch_bounds__(256) void add_readout_cast_ds_kernel(const float* a, const TB* __restrict__ b,
                                                                  const float* __restrict__ bsc, float* sum,
                                                                  f16* __restrict__ lp, int64_t rows, int cols,
                                                                  int ntok, float target, float* __restrict__ st,
                                                                  int use, float* __restrict__ spair) {
    const int c8 = cols / 8;
    const int64_t n8 = rows * c8;
    const float sb = bsc != nullptr ? *bsc : 1.0f;
    const float ls = ds_scale_of_use(st, use, target);
    ds_begin(st, use, ls, spair);
    uint32_t m = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += 2 * stride) {
        const int64_t i2 = i + stride;
        const bool two = i2 < n8;
        f32x4 x[4];
        readout_sum8<TB>(a, b, sb, i * 8, (i / c8) % ntok != 0, x[0], x[1]);
        if (two) readout_sum8<TB>(a, b, sb, i2 * 8, (i2 / c8) % ntok != 0, x[2], x[3]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h == 1 && !two) break;
            const int64_t off = (h ? i2 : i) * 8;
            if (b != nullptr) {
                *(f32x4*)(sum + off) = x[2 * h];
                *(f32x4*)(sum + off + 4) = x[2 * h + 1];
            }
            f16x8 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                m = max(m, max(__float_as_uint(x[2 * h][e]) & 0x7fffffffu, __float_as_uint(x[2 * h + 1][e]) & 0x7fffffffu));
                o[e] = (f16)(x[2 * h][e] * ls);
                o[4 + e] = (f16)(x[2 * h + 1][e] * ls);
            }
            *(f16x8*)(lp + off) = o;
        }
    }
    ds_end<4>(m, st, use);
}

extern "C" int dclip_add_readout_cast_scaled(const float* a, const void* b, int b_dt, const float* b_scale_ptr,
                                             float* sum, void* lp, int64_t rows, int cols, int ntok, float target,
                                             float* st, int use, float* spair, void* stream) {
    DCLIP_HOST_CHECK(cols % 8 == 0 && ntok > 0 && rows > 0 && target > 0.f && st != nullptr && spair != nullptr &&
                         use >= 1,
                     "dclip_add_readout_cast_scaled: cols %% 8 == 0, ntok > 0, rows > 0, target > 0, st, use >= 1, spair");
    DCLIP_HOST_CHECK(b == nullptr || sum != nullptr, "dclip_add_readout_cast_scaled: sum is required with b");
    DCLIP_HOST_CHECK(((uintptr_t)a | (uintptr_t)b | (uintptr_t)sum | (uintptr_t)lp) % 16 == 0,
                     "dclip_add_readout_cast_scaled: unaligned buffers");
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = grid_for((rows * (cols / 8) + 1) / 2, 4096);
    if (b == nullptr) b_dt = DCLIP_F32;
    DISPATCH_DT(b_dt, TB,
        add_readout_cast_ds_kernel<TB><<<g, 256, 0, s>>>(a, (const TB*)b, b_scale_ptr, sum, (f16*)lp, rows, cols, ntok,
                                                         target, st, use, spair));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_cast(const void* in, int in_dt, void* out, int out_dt, int64_t n, float scale_v,
                          const float* scale_ptr, void* stream) {
    if (n == 0) return 0;
    const Alpha scale(scale_v, scale_ptr);
    hipStream_t st = (hipStream_t)stream;
    DISPATCH_DT(in_dt, TI, DISPATCH_DT(out_dt, TO,
        cast_kernel<TI, TO><<<grid_for((n + 3) / 4), 256, 0, st>>>((const TI*)in, (TO*)out, n, scale)));
    DCLIP_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------- batch norm (train)
// Neck / head BatchNorm2d in train mode on channels-last 16-bit maps (reference
// models.py:13-20 ConvModule, heads' FCNHead BN): x viewed as (rows = B*H*W, C).  torch's native
// channels-last kernels reach ~0.12 TB/s on these maps; here every pass streams the map once at
// 16 B per lane.  Statistics are shifted by row 0 (sum of (x - x0) and (x - x0)^2) so that
// E[d^2] - E[d]^2 does not cancel; per-block partials are reduced in a fixed order
// (deterministic).  One thread owns 8 channels (C / 8 threads per row, 256 / (C / 8) rows per
// pass of a 256-thread block).
namespace {

constexpr int BN_NBLK_MAX = 512;

inline int bn_nblk(int64_t rows, int C) {
    const int rpb = 256 / (C / 8);
    const int64_t need = (rows + rpb - 1) / rpb;
    return (int)(need < BN_NBLK_MAX ? need : BN_NBLK_MAX);
}

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* v) {
    typedef T t8 __attribute__((ext_vector_type(8)));
    const t8 r = *(const t8*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)r[e];
}

// the forward's per-channel affine of BN (scale = w rstd, shift = b - mean scale) for 8 channels
__device__ __forceinline__ void bn_affine8(const float* w, const float* b, const float* mean, const float* rstd, int c0,
                                           float* sc, float* sh) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sc[e] = (w ? w[c0 + e] : 1.f) * rstd[c0 + e];
        sh[e] = (b ? b[c0 + e] : 0.f) - mean[c0 + e] * sc[e];
    }
}

// MODE 0: s += x - x0, q += (x - x0)^2 ;  MODE 1: s += dy, q += dy * (x - mean), with dy masked by
// the fused ReLU's derivative (x sc + sh > 0) when RELU.  Rows of ld elements; threads past the
// last whole row of a pass (C / 8 not dividing 256) idle.
template <typename T, int MODE, bool RELU>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ a, const T* __restrict__ x,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       int64_t rows, int C, int64_t ld, float* __restrict__ part) {
    __shared__ float red[2 * 2048];
    const int tpr = C / 8, rpb = 256 / tpr;
    const int c8 = threadIdx.x % tpr, rr = threadIdx.x / tpr;
    float s[8], q[8], ref[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
    if (rr < rpb) {
        if (MODE == 0) load8(a + c8 * 8, ref);
        else
#pragma unroll
            for (int e = 0; e < 8; ++e) ref[e] = mean[c8 * 8 + e];
        if (RELU) bn_affine8(w, b, mean, rstd, c8 * 8, sc, sh);
#pragma unroll 4
        for (int64_t r = (int64_t)blockIdx.x * rpb + rr; r < rows; r += (int64_t)gridDim.x * rpb) {
            float v[8];
            load8(a + r * ld + c8 * 8, v);
            if (MODE == 0) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float d = v[e] - ref[e];
                    s[e] += d;
                    q[e] += d * d;
                }
            } else {
                float xv[8];
                load8(x + r * ld + c8 * 8, xv);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float g = (!RELU || xv[e] * sc[e] + sh[e] > 0.f) ? v[e] : 0.f;
                    s[e] += g;
                    q[e] += g * (xv[e] - ref[e]);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            red[rr * C + c8 * 8 + e] = s[e];
            red[2048 + rr * C + c8 * 8 + e] = q[e];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
        float ss = 0.f, qq = 0.f;
        for (int k = 0; k < rpb; ++k) {
            ss += red[k * C + c];
            qq += red[2048 + k * C + c];
        }
        part[(int64_t)blockIdx.x * 2 * C + c] = ss;
        part[(int64_t)blockIdx.x * 2 * C + C + c] = qq;
    }
}

// the per-block partials of 8 channels (blockIdx.x * 8 ..) summed by 256 threads: 32 groups
// of 8 channels each take every 32nd partial (loads in flight), then a fixed-order sum of the
// 32 group sums; threads 0..7 return the channel's (S, Q), the others (0, 0)
__device__ __forceinline__ void bn_reduce_parts(const float* __restrict__ part, int nblk, int C, int& c, float& S,
                                                float& Q) {
    __shared__ float red[2][32][8];
    const int lc = threadIdx.x & 7, grp = threadIdx.x >> 3;
    c = blockIdx.x * 8 + lc;
    float s = 0.f, q = 0.f;
    if (c < C) {
#pragma unroll 4
        for (int k = grp; k < nblk; k += 32) {
            s += part[(int64_t)k * 2 * C + c];
            q += part[(int64_t)k * 2 * C + C + c];
        }
    }
    red[0][grp][lc] = s;
    red[1][grp][lc] = q;
    __syncthreads();
    S = Q = 0.f;
    if (threadIdx.x < 8)
        for (int g = 0; g < 32; ++g) {
            S += red[0][g][lc];
            Q += red[1][g][lc];
        }
}

// forward finalize: mean, rstd, scale = w rstd, shift = b - mean scale; running statistics
// (unbiased variance, momentum) as nn.BatchNorm2d updates them
template <typename T>
__global__ void bn_fwd_finalize_kernel(const float* __restrict__ part, int nblk, const T* __restrict__ x, int64_t rows,
                                       int C, const float* __restrict__ w, const float* __restrict__ b, float eps,
                                       float momentum, float* __restrict__ rmean, float* __restrict__ rvar,
                                       float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ ss) {
    int c;
    float S, Q;
    bn_reduce_parts(part, nblk, C, c, S, Q);
    if (threadIdx.x >= 8 || c >= C) return;
    const float n = (float)rows;
    const float md = S / n;
    const float var = fmaxf(Q / n - md * md, 0.f);
    const float mu = (float)x[c] + md;
    const float rs = rsqrtf(var + eps);
    mean[c] = mu;
    rstd[c] = rs;
    const float sc = (w ? w[c] : 1.f) * rs;
    ss[c] = sc;
    ss[C + c] = (b ? b[c] : 0.f) - mu * sc;
    if (rmean) {
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * (rows > 1 ? n / (n - 1.f) : 1.f);
    }
}

// backward finalize: dw = sum dy (x - mean) rstd, db = sum dy; dx = k1 dy + k2 x + k3
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int64_t rows, int C,
                                       const float* __restrict__ w, const float* __restrict__ mean,
                                       const float* __restrict__ rstd, float* __restrict__ dw, float* __restrict__ db,
                                       float* __restrict__ k, const float* __restrict__ gscale) {
    int c;
    float S, Q;
    bn_reduce_parts(part, nblk, C, c, S, Q);
    if (threadIdx.x >= 8 || c >= C) return;
    const float n = (float)rows, rs = rstd[c], wc = w ? w[c] : 1.f;
    // the parameter gradients unscaled by 1/s of the fp16 heads' gradient scale (dx keeps s)
    const float ga = gscale ? *gscale : 1.f;
    if (dw) dw[c] = Q * rs * ga;
    if (db) db[c] = S * ga;
    const float k1 = wc * rs;
    const float k2 = -wc * rs * rs * rs * (Q / n);
    k[c] = k1;
    k[C + c] = k2;
    k[2 * C + c] = -k1 * (S / n) - k2 * mean[c];
}

// y = (T)(x * s1[c] + s2[c])   (forward: s1 = scale, s2 = shift; RELU: max(0, .))
// y = (T)(a * k1[c] + x * k2[c] + k3[c])   (backward: a = dy, masked by the ReLU derivative when RELU;
// k[3C..5C) = the forward's scale / shift)
template <typename T, bool BWD, bool RELU>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ a, const T* __restrict__ x,
                                                       const float* __restrict__ k, int64_t rows, int C, int64_t ld,
                                                       T* __restrict__ y) {
    const int c8n = C / 8;
    const int64_t n8 = rows * c8n;
    typedef T t8 __attribute__((ext_vector_type(8)));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const int c0 = (int)(i % c8n) * 8;
        const int64_t off = (i / c8n) * ld + c0;
        float v[8];
        load8(a + off, v);
        t8 o;
        if (BWD) {
            float xv[8];
            load8(x + off, xv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float g = (!RELU || xv[e] * k[3 * C + c0 + e] + k[4 * C + c0 + e] > 0.f) ? v[e] : 0.f;
                o[e] = (T)(g * k[c0 + e] + xv[e] * k[C + c0 + e] + k[2 * C + c0 + e]);
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float t = v[e] * k[c0 + e] + k[C + c0 + e];
                o[e] = (T)(RELU ? fmaxf(t, 0.f) : t);
            }
        }
        *(t8*)(y + off) = o;
    }
}

// the forward's scale / shift for the backward's ReLU mask, into k[3C..5C)
__global__ void bn_mask_affine_kernel(const float* __restrict__ w, const float* __restrict__ b,
                                      const float* __restrict__ mean, const float* __restrict__ rstd, int C,
                                      float* __restrict__ k) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const float sc = (w ? w[c] : 1.f) * rstd[c];
    k[3 * C + c] = sc;
    k[4 * C + c] = (b ? b[c] : 0.f) - mean[c] * sc;
}

// eval mode: scale = w / sqrt(running_var + eps), shift = b - running_mean * scale into ss[0..2C)
__global__ void bn_eval_affine_kernel(const float* __restrict__ w, const float* __restrict__ b,
                                      const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                                      int C, float* __restrict__ ss) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const float sc = (w ? w[c] : 1.f) / sqrtf(rvar[c] + eps);
    ss[c] = sc;
    ss[C + c] = (b ? b[c] : 0.f) - rmean[c] * sc;
}

bool bn_shape_ok(int64_t rows, int C, int64_t ld) {
    const int tpr = C / 8;
    return rows > 0 && C % 8 == 0 && tpr >= 1 && tpr <= 256 && ld >= C && ld % 8 == 0;
}

}  // namespace

extern "C" int64_t dclip_bn_workspace(int64_t rows, int C) {
    (void)rows;
    return (int64_t)BN_NBLK_MAX * 2 * C + 5 * (int64_t)C;
}

extern "C" int dclip_bn_fwd(int dt, const void* x, int64_t rows, int C, int64_t ld, const float* w, const float* b,
                            float eps, float momentum, float* running_mean, float* running_var, float* ws, float* mean,
                            float* rstd, void* y, int relu, void* stream) {
    DCLIP_HOST_CHECK(dt == DCLIP_BF16 || dt == DCLIP_F16, "dclip_bn_fwd: dtype must be bf16/f16");
    DCLIP_HOST_CHECK(bn_shape_ok(rows, C, ld), "dclip_bn_fwd: need rows > 0, C %% 8 == 0, C <= 2048, ld >= C, "
                     "ld %% 8 == 0 (C = %d)", C);
    DCLIP_HOST_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0, "dclip_bn_fwd: unaligned buffers");
    hipStream_t st = (hipStream_t)stream;
    const int nblk = bn_nblk(rows, C);
    float* ss = ws + (int64_t)BN_NBLK_MAX * 2 * C;
    const unsigned ga = grid_for(rows * (C / 8), 8192);
#define BN_FWD(T)                                                                                                      \
    bn_stats_kernel<T, 0, false><<<nblk, 256, 0, st>>>((const T*)x, nullptr, nullptr, nullptr, nullptr, nullptr, rows, \
                                                       C, ld, ws);                                                     \
    bn_fwd_finalize_kernel<T><<<(C + 7) / 8, 256, 0, st>>>(ws, nblk, (const T*)x, rows, C, w, b, eps, momentum,        \
                                                           running_mean, running_var, mean, rstd, ss);                 \
    if (relu) bn_apply_kernel<T, false, true><<<ga, 256, 0, st>>>((const T*)x, nullptr, ss, rows, C, ld, (T*)y);       \
    else bn_apply_kernel<T, false, false><<<ga, 256, 0, st>>>((const T*)x, nullptr, ss, rows, C, ld, (T*)y);
    if (dt == DCLIP_BF16) {
        BN_FWD(bf16)
    } else {
        BN_FWD(f16)
    }
#undef BN_FWD
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_bn_eval(int dt, const void* x, int64_t rows, int C, int64_t ld, const float* w, const float* b,
                             float eps, const float* running_mean, const float* running_var, float* ws, void* y,
                             int relu, void* stream) {
    DCLIP_HOST_CHECK(dt == DCLIP_BF16 || dt == DCLIP_F16, "dclip_bn_eval: dtype must be bf16/f16");
    DCLIP_HOST_CHECK(bn_shape_ok(rows, C, ld), "dclip_bn_eval: need rows > 0, C %% 8 == 0, C <= 2048, ld >= C, "
                     "ld %% 8 == 0 (C = %d)", C);
    DCLIP_HOST_CHECK(running_mean && running_var && ws, "dclip_bn_eval: running statistics and workspace required");
    DCLIP_HOST_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0, "dclip_bn_eval: unaligned buffers");
    hipStream_t st = (hipStream_t)stream;
    float* ss = ws + (int64_t)BN_NBLK_MAX * 2 * C;
    const unsigned ga = grid_for(rows * (C / 8), 8192);
    bn_eval_affine_kernel<<<(C + 255) / 256, 256, 0, st>>>(w, b, running_mean, running_var, eps, C, ss);
#define BN_EVAL(T)                                                                                                 \
    if (relu) bn_apply_kernel<T, false, true><<<ga, 256, 0, st>>>((const T*)x, nullptr, ss, rows, C, ld, (T*)y);   \
    else bn_apply_kernel<T, false, false><<<ga, 256, 0, st>>>((const T*)x, nullptr, ss, rows, C, ld, (T*)y);
    if (dt == DCLIP_BF16) {
        BN_EVAL(bf16)
    } else {
        BN_EVAL(f16)
    }
#undef BN_EVAL
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_bn_bwd(int dt, const void* dy, const void* x, int64_t rows, int C, int64_t ld, const float* w,
                            const float* b, const float* mean, const float* rstd, float* ws, void* dx, float* dw,
                            float* db, int relu, const float* gscale, void* stream) {
    DCLIP_HOST_CHECK(dt == DCLIP_BF16 || dt == DCLIP_F16, "dclip_bn_bwd: dtype must be bf16/f16");
    DCLIP_HOST_CHECK(bn_shape_ok(rows, C, ld), "dclip_bn_bwd: need rows > 0, C %% 8 == 0, C <= 2048, ld >= C, "
                     "ld %% 8 == 0 (C = %d)", C);
    DCLIP_HOST_CHECK(((uintptr_t)dy % 16) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)dx % 16) == 0,
                     "dclip_bn_bwd: unaligned buffers");
    hipStream_t st = (hipStream_t)stream;
    const int nblk = bn_nblk(rows, C);
    float* k = ws + (int64_t)BN_NBLK_MAX * 2 * C;
    const unsigned ga = grid_for(rows * (C / 8), 8192);
    if (relu) bn_mask_affine_kernel<<<(C + 255) / 256, 256, 0, st>>>(w, b, mean, rstd, C, k);
#define BN_BWD(T)                                                                                                      \
    if (relu) {                                                                                                        \
        bn_stats_kernel<T, 1, true><<<nblk, 256, 0, st>>>((const T*)dy, (const T*)x, w, b, mean, rstd, rows, C, ld, ws); \
        bn_bwd_finalize_kernel<<<(C + 7) / 8, 256, 0, st>>>(ws, nblk, rows, C, w, mean, rstd, dw, db, k, gscale);               \
        bn_apply_kernel<T, true, true><<<ga, 256, 0, st>>>((const T*)dy, (const T*)x, k, rows, C, ld, (T*)dx);          \
    } else {                                                                                                           \
        bn_stats_kernel<T, 1, false><<<nblk, 256, 0, st>>>((const T*)dy, (const T*)x, w, b, mean, rstd, rows, C, ld,   \
                                                           ws);                                                        \
        bn_bwd_finalize_kernel<<<(C + 7) / 8, 256, 0, st>>>(ws, nblk, rows, C, w, mean, rstd, dw, db, k, gscale);               \
        bn_apply_kernel<T, true, false><<<ga, 256, 0, st>>>((const T*)dy, (const T*)x, k, rows, C, ld, (T*)dx);         \
    }
    if (dt == DCLIP_BF16) {
        BN_BWD(bf16)
    } else {
        BN_BWD(f16)
    }
#undef BN_BWD
    DCLIP_LAUNCH_CHECK();
    return 0;
}
