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
// gradient back through the transposed interpolation (per column over the band's rows in
// registers, across columns in LDS, across workgroups with one global atomic per low-res
// value and workgroup).  HBM traffic is the labels plus the (small) low-res maps.
//   CE:    loss = sum_p -log softmax(up(L))_p[t_p] / #valid;  dL/dup = softmax - onehot
//   SILog: d = log(max(up(P), eps)) - log(max(gt, eps)) on the mask;
//          loss = sum d^2 / T - lambda (sum d)^2 / T^2;  pass 0 sums, pass 1 the gradient
//          (2 d / T - 2 lambda S / T^2) / up(P)  where up(P) >= eps
#include "common.h"

namespace {

constexpr int JW = 32;   // low-res columns per workgroup chunk
constexpr int NTH = 256;

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

// MODE 0: cross-entropy (K classes);  MODE 1: SILog pass 0 (sums);  MODE 2: SILog pass 1 (gradient)
template <typename TL, int K, int MODE>
__global__ __launch_bounds__(NTH) void band_loss_kernel(const TL* __restrict__ low, int h, int w, int H, int W,
                                                        int chunks, const void* __restrict__ lab, int lab_dt,
                                                        int ignore, const float* __restrict__ gt,
                                                        const uint8_t* __restrict__ mask, float eps, float lambd,
                                                        double* __restrict__ sums, unsigned* __restrict__ count,
                                                        float* __restrict__ grad) {
    __shared__ float low_s[2][JW + 1][K];   // the band's two low-res rows over the chunk (+1 column)
    __shared__ float acc_s[2][JW + 1][K];   // transposed-interpolation accumulators
    __shared__ double red_s[NTH / 64][3];
    const int tid = threadIdx.x;
    const int ch = blockIdx.x % chunks;
    const int i = (blockIdx.x / chunks) % h;
    const int b = blockIdx.x / (chunks * h);
    const int jc = ch * JW;
    const int i1 = i + (i < h - 1 ? 1 : 0);
    const int ncol = (jc + JW + 1 <= w ? JW + 1 : w - jc);
    for (int e = tid; e < 2 * (JW + 1) * K; e += NTH) {
        const int r = e / ((JW + 1) * K), jj = (e / K) % (JW + 1), k = e % K;
        const int row = r ? i1 : i;
        low_s[r][jj][k] = jj < ncol ? ld(low + (((int64_t)b * K + k) * h + row) * w + jc + jj) : 0.f;
        acc_s[r][jj][k] = 0.f;
    }
    __syncthreads();
    // SILog pass 1 needs the global sums of pass 0
    float gS = 0.f, gT = 1.f;
    if constexpr (MODE == 2) {
        gS = (float)sums[0];
        gT = (float)sums[2];
        gT = gT > 0.f ? gT : 1.f;
    }
    int ylo, yhi, xlo, xhi, xlo2, xhi2;
    band_range(i, h, H, &ylo, &yhi);
    band_range(jc, w, W, &xlo, &xhi2);
    band_range(jc + JW - 1 < w - 1 ? jc + JW - 1 : w - 1, w, W, &xlo2, &xhi);
    (void)xhi2;
    (void)xlo2;
    double lsum = 0.0, lsum2 = 0.0;
    unsigned lcnt = 0;
    for (int x = xlo + tid; x <= xhi; x += NTH) {
        const Lerp X = lerp_index(x, w, W);
        if (X.i0 < jc || X.i0 >= jc + JW) continue;
        const int j0 = X.i0 - jc, j1 = X.i1 - jc;
        float ut[K], ub[K], at[K], ab[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            ut[k] = X.l0 * low_s[0][j0][k] + X.l1 * low_s[0][j1][k];
            ub[k] = X.l0 * low_s[1][j0][k] + X.l1 * low_s[1][j1][k];
            at[k] = 0.f;
            ab[k] = 0.f;
        }
        for (int y = ylo; y <= yhi; ++y) {
            const Lerp Y = lerp_index(y, h, H);
            if (Y.i0 != i) continue;
            const int64_t pix = ((int64_t)b * H + y) * W + x;
            float v[K];
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = Y.l0 * ut[k] + Y.l1 * ub[k];
            if constexpr (MODE == 0) {
                const int t = load_label(lab, lab_dt, pix);
                if (t == ignore || t < 0 || t >= K) continue;
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
                if (mask && !mask[pix]) continue;
                const float p = v[0];
                const float g = gt[pix];
                const float d = logf(fmaxf(p, eps)) - logf(fmaxf(g, eps));
                if constexpr (MODE == 1) {
                    lsum += (double)d;
                    lsum2 += (double)d * (double)d;
                    ++lcnt;
                } else {
                    const float gd = (2.f * d / gT - 2.f * lambd * gS / (gT * gT)) * (p >= eps ? 1.f / p : 0.f);
                    at[0] += Y.l0 * gd;
                    ab[0] += Y.l1 * gd;
                }
            }
        }
        if constexpr (MODE != 1) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                atomicAdd(&acc_s[0][j0][k], X.l0 * at[k]);
                atomicAdd(&acc_s[0][j1][k], X.l1 * at[k]);
                atomicAdd(&acc_s[1][j0][k], X.l0 * ab[k]);
                atomicAdd(&acc_s[1][j1][k], X.l1 * ab[k]);
            }
        }
    }
    if constexpr (MODE != 2) {  // loss / count partials: wave sums, then one atomic per workgroup
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
        if (tid == 0) {
            double a = 0.0, a2 = 0.0, c = 0.0;
            for (int wv = 0; wv < NTH / 64; ++wv) {
                a += red_s[wv][0];
                a2 += red_s[wv][1];
                c += red_s[wv][2];
            }
            atomicAdd(sums, a);
            if constexpr (MODE == 1) {
                atomicAdd(sums + 1, a2);
                atomicAdd(sums + 2, c);
            } else {
                atomicAdd(count, (unsigned)c);
            }
        }
    }
    if constexpr (MODE != 1) {  // the chunk's low-res gradient: one global atomic per value
        for (int e = tid; e < 2 * (JW + 1) * K; e += NTH) {
            const int r = e / ((JW + 1) * K), jj = (e / K) % (JW + 1), k = e % K;
            if (jj >= ncol || (r == 1 && i1 == i)) continue;
            const float v = acc_s[r][jj][k] + (r == 0 && i1 == i ? acc_s[1][jj][k] : 0.f);
            if (v != 0.f) atomicAdd(grad + (((int64_t)b * K + k) * h + (r ? i1 : i)) * w + jc + jj, v);
        }
    }
}

// Cross-entropy with the gradient folded per LOW-RES column: thread (jj, xs) of the 32 x 8 grid owns
// every 8th high-res column x whose left interpolation column is j0 = jc + jj, runs all the band's
// rows for it, and keeps the four folded sums (left / right column x upper / lower row) of its
// columns in registers; only those go to LDS (8 threads per column instead of one atomic set per
// high-res column: the per-column LDS atomics of band_loss_kernel, 16-way on the same addresses,
// were its cost).  Same arithmetic per pixel as band_loss_kernel MODE 0.
template <typename TL, int K>
__global__ __launch_bounds__(NTH) void band_ce_kernel(const TL* __restrict__ low, int h, int w, int H, int W,
                                                      int chunks, const void* __restrict__ lab, int lab_dt,
                                                      int ignore, double* __restrict__ sums,
                                                      unsigned* __restrict__ count, float* __restrict__ grad) {
    static_assert(NTH == JW * 8, "32 low-res columns x 8 column slices");
    __shared__ float low_s[2][JW + 1][K];
    __shared__ float acc_s[2][JW + 1][K];
    __shared__ double red_s[NTH / 64][2];
    const int tid = threadIdx.x;
    const int ch = blockIdx.x % chunks;
    const int i = (blockIdx.x / chunks) % h;
    const int b = blockIdx.x / (chunks * h);
    const int jc = ch * JW;
    const int i1 = i + (i < h - 1 ? 1 : 0);
    const int ncol = (jc + JW + 1 <= w ? JW + 1 : w - jc);
    for (int e = tid; e < 2 * (JW + 1) * K; e += NTH) {
        const int r = e / ((JW + 1) * K), jj = (e / K) % (JW + 1), k = e % K;
        const int row = r ? i1 : i;
        low_s[r][jj][k] = jj < ncol ? ld(low + (((int64_t)b * K + k) * h + row) * w + jc + jj) : 0.f;
        acc_s[r][jj][k] = 0.f;
    }
    __syncthreads();
    const int jj = tid >> 3, xs = tid & 7;
    const int j0 = jc + jj;
    int ylo, yhi, xlo, xhi;
    band_range(i, h, H, &ylo, &yhi);
    double lsum = 0.0;
    unsigned lcnt = 0;
    float g[4][K];  // folded gradient: [left / right column][upper / lower row] as 0: l-u, 1: r-u, 2: l-b, 3: r-b
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < K; ++k) g[q][k] = 0.f;
    if (j0 < w) {
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
            // the column's labels 8 rows at a time, all loads in flight together (one dependent
            // global load per pixel left this kernel latency-bound)
            for (int y0 = ylo; y0 <= yhi; y0 += 8) {
            int tl[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int y = y0 + u;
                tl[u] = y <= yhi ? load_label(lab, lab_dt, ((int64_t)b * H + y) * W + x) : ignore;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int y = y0 + u;
                if (y > yhi) continue;
                const Lerp Y = lerp_index(y, h, H);
                if (Y.i0 != i) continue;
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
            }
            }
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
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (g[0][k] != 0.f) atomicAdd(&acc_s[0][jj][k], g[0][k]);
            if (g[1][k] != 0.f) atomicAdd(&acc_s[0][jj + 1][k], g[1][k]);
            if (g[2][k] != 0.f) atomicAdd(&acc_s[1][jj][k], g[2][k]);
            if (g[3][k] != 0.f) atomicAdd(&acc_s[1][jj + 1][k], g[3][k]);
        }
    }
    double a = lsum, c = (double)lcnt;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        c += __shfl_xor(c, o, 64);
    }
    if ((tid & 63) == 0) {
        red_s[tid >> 6][0] = a;
        red_s[tid >> 6][1] = c;
    }
    __syncthreads();
    if (tid == 0) {
        double sa = 0.0, sc = 0.0;
        for (int wv = 0; wv < NTH / 64; ++wv) {
            sa += red_s[wv][0];
            sc += red_s[wv][1];
        }
        atomicAdd(sums, sa);
        atomicAdd(count, (unsigned)sc);
    }
    for (int e = tid; e < 2 * (JW + 1) * K; e += NTH) {
        const int r = e / ((JW + 1) * K), jx = (e / K) % (JW + 1), k = e % K;
        if (jx >= ncol || (r == 1 && i1 == i)) continue;
        const float v = acc_s[r][jx][k] + (r == 0 && i1 == i ? acc_s[1][jx][k] : 0.f);
        if (v != 0.f) atomicAdd(grad + (((int64_t)b * K + k) * h + (r ? i1 : i)) * w + jc + jx, v);
    }
}

template <typename TL, int K, int MODE>
void launch_band(const void* low, int B, int h, int w, int H, int W, const void* lab, int lab_dt, int ignore,
                 const float* gt, const uint8_t* mask, float eps, float lambd, double* sums, unsigned* count,
                 float* grad, hipStream_t st) {
    const int chunks = (w + JW - 1) / JW;
    if constexpr (MODE == 0)
        band_ce_kernel<TL, K><<<B * h * chunks, NTH, 0, st>>>((const TL*)low, h, w, H, W, chunks, lab, lab_dt, ignore,
                                                              sums, count, grad);
    else
        band_loss_kernel<TL, K, MODE><<<B * h * chunks, NTH, 0, st>>>((const TL*)low, h, w, H, W, chunks, lab,
                                                                      lab_dt, ignore, gt, mask, eps, lambd, sums,
                                                                      count, grad);
}

}  // namespace

extern "C" int dclip_upsample_ce(int low_dt, const void* logits, int B, int K, int h, int w, const void* labels,
                                 int lab_dt, int H, int W, int ignore_index, double* loss_sum, unsigned* count,
                                 float* grad, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && h > 0 && w > 0 && H > 0 && W > 0, "dclip_upsample_ce: bad sizes");
    DCLIP_HOST_CHECK(K == 19, "dclip_upsample_ce: K=%d (built for the 19 Cityscapes classes)", K);
    DCLIP_HOST_CHECK(lab_dt >= 0 && lab_dt <= 2, "dclip_upsample_ce: labels int64 (0), int32 (1) or uint8 (2)");
    DCLIP_HOST_CHECK(loss_sum && count && grad, "dclip_upsample_ce: outputs required");
    hipStream_t st = (hipStream_t)stream;
    if (low_dt == DCLIP_F32)
        launch_band<float, 19, 0>(logits, B, h, w, H, W, labels, lab_dt, ignore_index, nullptr, nullptr, 0.f, 0.f,
                                  loss_sum, count, grad, st);
    else if (low_dt == DCLIP_BF16)
        launch_band<bf16, 19, 0>(logits, B, h, w, H, W, labels, lab_dt, ignore_index, nullptr, nullptr, 0.f, 0.f,
                                 loss_sum, count, grad, st);
    else
        launch_band<f16, 19, 0>(logits, B, h, w, H, W, labels, lab_dt, ignore_index, nullptr, nullptr, 0.f, 0.f,
                                loss_sum, count, grad, st);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_upsample_silog(int pass, int low_dt, const void* pred, int B, int h, int w, const float* target,
                                    const uint8_t* mask, int H, int W, float eps, float lambd, double* sums,
                                    float* grad, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && h > 0 && w > 0 && H > 0 && W > 0, "dclip_upsample_silog: bad sizes");
    DCLIP_HOST_CHECK(pass == 0 || pass == 1, "dclip_upsample_silog: pass 0 (sums) or 1 (gradient)");
    DCLIP_HOST_CHECK(target && sums && (pass == 0 || grad), "dclip_upsample_silog: missing buffers");
    hipStream_t st = (hipStream_t)stream;
#define SILOG(TL)                                                                                                \
    if (pass == 0)                                                                                               \
        launch_band<TL, 1, 1>(pred, B, h, w, H, W, nullptr, 0, 0, target, mask, eps, lambd, sums, nullptr, nullptr, st); \
    else                                                                                                         \
        launch_band<TL, 1, 2>(pred, B, h, w, H, W, nullptr, 0, 0, target, mask, eps, lambd, sums, nullptr, grad, st)
    if (low_dt == DCLIP_F32) SILOG(float);
    else if (low_dt == DCLIP_BF16) SILOG(bf16);
    else SILOG(f16);
#undef SILOG
    DCLIP_LAUNCH_CHECK();
    return 0;
}
