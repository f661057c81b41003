// Fused bilinear upsample + loss (+ gradient) of the two DenseCLIP heads.
//
// The reference upsamples the segmentation logits and the depth prediction to the label size
// (seg/denseclip/denseclip.py:843-868, F.interpolate bilinear align_corners=False) and the
// trainer applies CE(ignore 255) and SILog (train_denseclip.py:1265-1314, losses.py:21-78) to
// the upsampled tensors: at 1024x2048 that is a 19-channel fp32 tensor of 1.27 GB per 8 images
// written, read by log-softmax, re-read by NLL, and the same again for the gradients.  Here
// the upsampled values exist only in registers: each workgroup owns the high-res pixels whose
// upper interpolation row is low-res row i (a "band") and whose left interpolation column
// lies in a 32-column chunk, interpolates along x once per pixel column (two rows of
// K values), along y per pixel, evaluates the loss and its gradient per pixel, and folds the
// gradient back through the transposed interpolation.  HBM traffic is the labels plus the
// (small) low-res maps.
//   CE:    loss = sum_p -log softmax(up(L))_p[t_p] / #valid;  dL/dup = softmax - onehot
//   SILog: d = log(max(up(P), eps)) - log(max(gt, eps)) on the mask;
//          loss = sum d^2 / T - lambda (sum d)^2 / T^2;  pass 0 sums, pass 1 the gradient
//          (2 d / T - 2 lambda S / T^2) / up(P)  where up(P) >= eps
//
// Every sum is taken in a FIXED order (ABI 7), so the loss and its gradient repeat bit for bit
// run to run (round 5 traced the fp16 training step's run-to-run divergence to the float
// atomics these kernels used):
//   * within a thread: its high-res columns and rows in loop order;
//   * within a workgroup: thread (jj, xs) of the 32 x 8 grid owns every 8th high-res column x
//     of low-res column jc + jj; the 8 column slices are summed by a xor butterfly over the 8
//     adjacent lanes, then low-res column jx takes its own left weights plus column jx - 1's
//     right weights, in that order, through LDS (no LDS atomics);
//   * across workgroups: each workgroup writes its 2 x 33 x K gradient tile and its loss
//     partials to the caller's workspace; band_merge_kernel adds the <= 4 tiles that overlap a
//     low-res value (own band / chunk, previous chunk's 33rd column, previous band's lower row)
//     in that order, and band_sums_kernel adds the partials in workgroup order.
#include "common.h"

namespace {

constexpr int JW = 32;   // low-res columns per workgroup chunk
constexpr int NTH = 256;
constexpr int NPART = 4; // doubles of loss partials per workgroup: sum d | -log p, sum d^2, count, (pad)

struct Lerp {
    int i0, i1;
    float l0, l1;
};
// PyTorch upsample_bilinear2d, align_corners=False (same arithmetic as misc.hip's resize)
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

// conservative output range [lo, hi] whose i0 may equal i
__device__ __forceinline__ void band_range(int i, int in, int out, int* lo, int* hi) {
    const float inv = (float)out / (float)in;
    int a = (int)floorf(((float)i + 0.5f) * inv - 0.5f) - 2;
    int b = (int)ceilf(((float)i + 1.5f) * inv - 0.5f) + 2;
    *lo = (a < 0 || i == 0) ? 0 : a;  // i = 0 also owns the outputs whose source is clamped at 0
    *hi = (b > out - 1 || i == in - 1) ? out - 1 : b;
}

template <typename TL>
__device__ __forceinline__ float ld(const TL* p) { return (float)*p; }

__device__ __forceinline__ int load_label(const void* lab, int dt, int64_t i) {
    if (dt == 0) return (int)((const int64_t*)lab)[i];
    if (dt == 1) return ((const int32_t*)lab)[i];
    return ((const uint8_t*)lab)[i];
}

__host__ __device__ __forceinline__ int64_t tile_floats(int K) { return 2 * (JW + 1) * (int64_t)K; }

// MODE 0: cross-entropy (K classes);  MODE 1: SILog pass 0 (sums);  MODE 2: SILog pass 1 (gradient)
// part: [nwg][NPART] f64 loss partials (MODE 0, 1); tiles: [nwg][2][JW + 1][K] f32 gradient (MODE 0, 2)
template <typename TL, int K, int MODE>
__global__ __launch_bounds__(NTH) void band_fold_kernel(const TL* __restrict__ low, int h, int w, int H, int W,
                                                        int chunks, const void* __restrict__ lab, int lab_dt,
                                                        int ignore, const float* __restrict__ gt,
                                                        const uint8_t* __restrict__ mask, float eps, float lambd,
                                                        const double* __restrict__ sums, double* __restrict__ part,
                                                        float* __restrict__ tiles) {
    static_assert(NTH == JW * 8, "32 low-res columns x 8 column slices");
    __shared__ float low_s[2][JW + 1][K];  // the band's two low-res rows over the chunk (+1 column)
    __shared__ float g_s[4][JW][K];        // per low-res column: left-upper, right-upper, left-lower, right-lower
    __shared__ double red_s[NTH / 64][3];
    const int tid = threadIdx.x;
    const int wg = blockIdx.x;
    const int ch = wg % chunks;
    const int i = (wg / chunks) % h;
    const int b = wg / (chunks * h);
    const int jc = ch * JW;
    const int i1 = i + (i < h - 1 ? 1 : 0);
    const int ncol = (jc + JW + 1 <= w ? JW + 1 : w - jc);
    for (int e = tid; e < 2 * (JW + 1) * K; e += NTH) {
        const int r = e / ((JW + 1) * K), jj = (e / K) % (JW + 1), k = e % K;
        const int row = r ? i1 : i;
        low_s[r][jj][k] = jj < ncol ? ld(low + (((int64_t)b * K + k) * h + row) * w + jc + jj) : 0.f;
    }
    __syncthreads();
    // SILog pass 1 needs the global sums of pass 0
    float gS = 0.f, gT = 1.f;
    if constexpr (MODE == 2) {
        gS = (float)sums[0];
        gT = (float)sums[2];
        gT = gT > 0.f ? gT : 1.f;
    }
    const int jj = tid >> 3, xs = tid & 7;
    const int j0 = jc + jj;
    int ylo, yhi;
    band_range(i, h, H, &ylo, &yhi);
    double lsum = 0.0, lsum2 = 0.0;
    unsigned lcnt = 0;
    float g[4][K];  // folded gradient: 0: left-upper, 1: right-upper, 2: left-lower, 3: right-lower
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < K; ++k) g[q][k] = 0.f;
    if (j0 < w) {
        int xlo, xhi;
        band_range(j0, w, W, &xlo, &xhi);
        for (int x = xlo + xs; x <= xhi; x += 8) {
            const Lerp X = lerp_index(x, w, W);
            if (X.i0 != j0) continue;
            const int j1 = X.i1 - jc;
            float ut[K], ub[K], at[K], ab[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                ut[k] = X.l0 * low_s[0][jj][k] + X.l1 * low_s[0][j1][k];
                ub[k] = X.l0 * low_s[1][jj][k] + X.l1 * low_s[1][j1][k];
                at[k] = 0.f;
                ab[k] = 0.f;
            }
            // the column's labels / targets 8 rows at a time, all loads in flight together (one
            // dependent global load per pixel left these kernels latency-bound)
            for (int y0 = ylo; y0 <= yhi; y0 += 8) {
                int tl[8];
                float tg[8];
                bool tm[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int y = y0 + u;
                    const int64_t pix = ((int64_t)b * H + (y <= yhi ? y : yhi)) * W + x;
                    if constexpr (MODE == 0) {
                        tl[u] = y <= yhi ? load_label(lab, lab_dt, pix) : ignore;
                    } else {
                        tm[u] = y <= yhi && (mask == nullptr || mask[pix] != 0);
                        tg[u] = gt[pix];
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int y = y0 + u;
                    if (y > yhi) continue;
                    const Lerp Y = lerp_index(y, h, H);
                    if (Y.i0 != i) continue;
                    if constexpr (MODE == 0) {
                        const int t = tl[u];
                        if (t == ignore || t < 0 || t >= K) continue;
                        float v[K];
#pragma unroll
                        for (int k = 0; k < K; ++k) v[k] = Y.l0 * ut[k] + Y.l1 * ub[k];
                        float m = v[0], vt = 0.f;
#pragma unroll
                        for (int k = 1; k < K; ++k) m = fmaxf(m, v[k]);
#pragma unroll
                        for (int k = 0; k < K; ++k) vt = k == t ? v[k] : vt;
                        float s = 0.f;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            v[k] = __expf(v[k] - m);
                            s += v[k];
                        }
                        lsum += (double)(__logf(s) - (vt - m));  // -log softmax[t]
                        ++lcnt;
                        const float inv = 1.0f / s;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const float d = v[k] * inv - (k == t ? 1.f : 0.f);
                            at[k] += Y.l0 * d;
                            ab[k] += Y.l1 * d;
                        }
                    } else {
                        if (!tm[u]) continue;
                        const float p = Y.l0 * ut[0] + Y.l1 * ub[0];
                        const float d = logf(fmaxf(p, eps)) - logf(fmaxf(tg[u], eps));
                        if constexpr (MODE == 1) {
                            lsum += (double)d;
                            lsum2 += (double)d * (double)d;
                            ++lcnt;
                        } else {
                            const float gd =
                                (2.f * d / gT - 2.f * lambd * gS / (gT * gT)) * (p >= eps ? 1.f / p : 0.f);
                            at[0] += Y.l0 * gd;
                            ab[0] += Y.l1 * gd;
                        }
                    }
                }
            }
            if constexpr (MODE != 1) {
                if (j1 == jj) {  // clamped right edge: both weights on one column
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        g[0][k] += at[k];
                        g[2][k] += ab[k];
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        g[0][k] += X.l0 * at[k];
                        g[1][k] += X.l1 * at[k];
                        g[2][k] += X.l0 * ab[k];
                        g[3][k] += X.l1 * ab[k];
                    }
                }
            }
        }
    }
    if constexpr (MODE != 1) {
        // the column's 8 slices (8 adjacent lanes): a xor butterfly, the same order on every run
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int k = 0; k < K; ++k) {
                float v = g[q][k];
                v += __shfl_xor(v, 1, 64);
                v += __shfl_xor(v, 2, 64);
                v += __shfl_xor(v, 4, 64);
                g[q][k] = v;
            }
        if (xs == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < K; ++k) g_s[q][jj][k] = g[q][k];
        }
    }
    if constexpr (MODE != 2) {  // loss partials: wave sums (fixed butterfly), then the 4 waves in order
        double a = lsum, a2 = lsum2, c = (double)lcnt;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a += __shfl_xor(a, o, 64);
            a2 += __shfl_xor(a2, o, 64);
            c += __shfl_xor(c, o, 64);
        }
        if ((tid & 63) == 0) {
            red_s[tid >> 6][0] = a;
            red_s[tid >> 6][1] = a2;
            red_s[tid >> 6][2] = c;
        }
    }
    __syncthreads();
    if constexpr (MODE != 2) {
        if (tid < 3) {
            double s = 0.0;
            for (int wv = 0; wv < NTH / 64; ++wv) s += red_s[wv][tid];
            part[(int64_t)wg * NPART + tid] = s;
        }
    }
    if constexpr (MODE != 1) {  // the chunk's gradient tile (rows i, i1 x columns jc .. jc + JW)
        float* tile = tiles + (int64_t)wg * tile_floats(K);
        for (int e = tid; e < 2 * (JW + 1) * K; e += NTH) {
            const int r = e / ((JW + 1) * K), jx = (e / K) % (JW + 1), k = e % K;
            float v = 0.f;
            if (!(r == 1 && i1 == i)) {
                // low-res column jx: its own left weights, then column jx - 1's right weights
                v = (jx < JW ? g_s[2 * r][jx][k] : 0.f) + (jx > 0 ? g_s[2 * r + 1][jx - 1][k] : 0.f);
                if (r == 0 && i1 == i)  // last band: the lower row is the upper row
                    v += (jx < JW ? g_s[2][jx][k] : 0.f) + (jx > 0 ? g_s[3][jx - 1][k] : 0.f);
            }
            tile[e] = v;
        }
    }
}

// grad[b][k][y][x] += the <= 4 tiles covering it, in a fixed order: band y / chunk x / 32 (upper
// row), chunk x / 32 - 1's 33rd column, band y - 1 (lower row), band y - 1's previous chunk
__global__ __launch_bounds__(256) void band_merge_kernel(const float* __restrict__ tiles, int B, int K, int h, int w,
                                                         int chunks, float* __restrict__ grad) {
    const int64_t total = (int64_t)B * K * h * w;
    const int64_t tf = tile_floats(K);
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(idx % w);
        const int y = (int)((idx / w) % h);
        const int k = (int)((idx / ((int64_t)w * h)) % K);
        const int b = (int)(idx / ((int64_t)w * h * K));
        const int c0 = x / JW, jx = x % JW;
        auto at = [&](int band, int c, int r, int j) {
            return tiles[((int64_t)b * h + band) * chunks * tf + (int64_t)c * tf + ((int64_t)r * (JW + 1) + j) * K + k];
        };
        float v = at(y, c0, 0, jx);
        if (jx == 0 && c0 > 0) v += at(y, c0 - 1, 0, JW);
        if (y > 0) {
            v += at(y - 1, c0, 1, jx);
            if (jx == 0 && c0 > 0) v += at(y - 1, c0 - 1, 1, JW);
        }
        grad[idx] += v;
    }
}

// sums[0..2] (SILog) or loss_sum / count (CE) += the workgroups' partials, in workgroup order
// within each thread's stripe, then a fixed LDS tree
__global__ __launch_bounds__(256) void band_sums_kernel(const double* __restrict__ part, int nwg, int ce,
                                                        double* __restrict__ sums, unsigned* __restrict__ count) {
    __shared__ double red[3][256];
    const int t = threadIdx.x;
    double s[3] = {0.0, 0.0, 0.0};
    for (int e = t; e < nwg; e += 256)
#pragma unroll
        for (int c = 0; c < 3; ++c) s[c] += part[(int64_t)e * NPART + c];
#pragma unroll
    for (int c = 0; c < 3; ++c) red[c][t] = s[c];
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o)
#pragma unroll
            for (int c = 0; c < 3; ++c) red[c][t] += red[c][t + o];
        __syncthreads();
    }
    if (t == 0) {
        if (ce) {
            sums[0] += red[0][0];
            count[0] += (unsigned)(red[2][0] + 0.5);
        } else {
            sums[0] += red[0][0];
            sums[1] += red[1][0];
            sums[2] += red[2][0];
        }
    }
}

int64_t ws_floats(int B, int K, int h, int w) {
    const int64_t nwg = (int64_t)B * h * ((w + JW - 1) / JW);
    return nwg * (2 * NPART + tile_floats(K));  // the f64 partials first (8-byte aligned), then the tiles
}

template <typename TL, int K, int MODE>
void launch_band(const void* low, int B, int h, int w, int H, int W, const void* lab, int lab_dt, int ignore,
                 const float* gt, const uint8_t* mask, float eps, float lambd, double* sums, unsigned* count,
                 float* grad, float* ws, hipStream_t st) {
    const int chunks = (w + JW - 1) / JW;
    const int nwg = B * h * chunks;
    double* part = (double*)ws;
    float* tiles = ws + (int64_t)nwg * 2 * NPART;
    band_fold_kernel<TL, K, MODE><<<nwg, NTH, 0, st>>>((const TL*)low, h, w, H, W, chunks, lab, lab_dt, ignore, gt,
                                                        mask, eps, lambd, sums, part, tiles);
    if constexpr (MODE != 2) band_sums_kernel<<<1, 256, 0, st>>>(part, nwg, MODE == 0, sums, count);
    if constexpr (MODE != 1) {
        const int64_t total = (int64_t)B * K * h * w;
        int64_t blocks = (total + 255) / 256;
        blocks = blocks > 4096 ? 4096 : blocks;
        band_merge_kernel<<<(unsigned)blocks, 256, 0, st>>>(tiles, B, K, h, w, chunks, grad);
    }
}

}  // namespace

extern "C" int64_t dclip_upsample_ws_floats(int B, int K, int h, int w) {
    if (B <= 0 || K <= 0 || h <= 0 || w <= 0) return 0;
    return ws_floats(B, K, h, w);
}

extern "C" int dclip_upsample_ce(int low_dt, const void* logits, int B, int K, int h, int w, const void* labels,
                                 int lab_dt, int H, int W, int ignore_index, double* loss_sum, unsigned* count,
                                 float* grad, float* ws, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && h > 0 && w > 0 && H > 0 && W > 0, "dclip_upsample_ce: bad sizes");
    DCLIP_HOST_CHECK(K == 19, "dclip_upsample_ce: K=%d (built for the 19 Cityscapes classes)", K);
    DCLIP_HOST_CHECK(lab_dt >= 0 && lab_dt <= 2, "dclip_upsample_ce: labels int64 (0), int32 (1) or uint8 (2)");
    DCLIP_HOST_CHECK(loss_sum && count && grad, "dclip_upsample_ce: outputs required");
    DCLIP_HOST_CHECK(ws != nullptr && ((uintptr_t)ws % 8) == 0,
                     "dclip_upsample_ce: ws (dclip_upsample_ws_floats(B, K, h, w) f32, 8-byte aligned) required");
    hipStream_t st = (hipStream_t)stream;
    if (low_dt == DCLIP_F32)
        launch_band<float, 19, 0>(logits, B, h, w, H, W, labels, lab_dt, ignore_index, nullptr, nullptr, 0.f, 0.f,
                                  loss_sum, count, grad, ws, st);
    else if (low_dt == DCLIP_BF16)
        launch_band<bf16, 19, 0>(logits, B, h, w, H, W, labels, lab_dt, ignore_index, nullptr, nullptr, 0.f, 0.f,
                                 loss_sum, count, grad, ws, st);
    else
        launch_band<f16, 19, 0>(logits, B, h, w, H, W, labels, lab_dt, ignore_index, nullptr, nullptr, 0.f, 0.f,
                                loss_sum, count, grad, ws, st);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_upsample_silog(int pass, int low_dt, const void* pred, int B, int h, int w, const float* target,
                                    const uint8_t* mask, int H, int W, float eps, float lambd, double* sums,
                                    float* grad, float* ws, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && h > 0 && w > 0 && H > 0 && W > 0, "dclip_upsample_silog: bad sizes");
    DCLIP_HOST_CHECK(pass == 0 || pass == 1, "dclip_upsample_silog: pass 0 (sums) or 1 (gradient)");
    DCLIP_HOST_CHECK(target && sums && (pass == 0 || grad), "dclip_upsample_silog: missing buffers");
    DCLIP_HOST_CHECK(ws != nullptr && ((uintptr_t)ws % 8) == 0,
                     "dclip_upsample_silog: ws (dclip_upsample_ws_floats(B, 1, h, w) f32, 8-byte aligned) required");
    hipStream_t st = (hipStream_t)stream;
#define SILOG(TL)                                                                                                \
    if (pass == 0)                                                                                               \
        launch_band<TL, 1, 1>(pred, B, h, w, H, W, nullptr, 0, 0, target, mask, eps, lambd, sums, nullptr, nullptr, \
                              ws, st);                                                                           \
    else                                                                                                         \
        launch_band<TL, 1, 2>(pred, B, h, w, H, W, nullptr, 0, 0, target, mask, eps, lambd, sums, nullptr, grad, ws, st)
    if (low_dt == DCLIP_F32) SILOG(float);
    else if (low_dt == DCLIP_BF16) SILOG(bf16);
    else SILOG(f16);
#undef SILOG
    DCLIP_LAUNCH_CHECK();
    return 0;
}
