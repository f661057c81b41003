// Cityscapes depth + segmentation batch preparation on the GPU.
//
// Replaces the per-sample CPU work of the reference loader and trainer transforms:
//   * label ids -> train ids through the 34-entry table (datasets/cityscapes_depth_seg.py:43-45,
//     map_labels_fast 129-135; ids >= 34 -> 255);
//   * uint16 disparity -> metric depth (disparity_to_depth 137-170): d > 0 is valid,
//     s = (d - 1) / 256, depth = 500 / (s + 1e-6) where s > 1e-3, depth > depth_max or an
//     invalid d -> 0; the validity mask after the transforms is depth > 0 (__getitem__ 218);
//   * the trainer's RandomCrop + HorizontalFlip + Normalize + ToTensorV2
//     (train_denseclip.py:143-149): a crop window inside the image, an optional mirror, and
//     (x - 255 mean) * (1 / (255 std)) in f32, HWC uint8 -> CHW.
// The host uploads the decoded uint8 / uint16 planes (6 bytes per pixel instead of the 25 of
// the prepared f32 / int64 tensors); one thread per output pixel does all four outputs, so
// the pass is one read of the crop window and one write of the batch (HBM-bound, trivial).
// Every step is integer or a correctly rounded f32 operation in the reference's order, so the
// outputs are bit-identical to the NumPy reference.
#include "common.h"

namespace {

__constant__ uint8_t ID_TO_TRAIN_ID[34] = {255, 255, 255, 255, 255, 255, 255, 0,   1,   255, 255, 2,
                                           3,   4,   255, 255, 255, 5,   255, 6,   7,   8,   9,   10,
                                           11,  12,  13,  14,  15,  255, 255, 16,  17,  18};

template <typename TO>
__global__ __launch_bounds__(256) void cityscapes_prepare_kernel(
    const uint8_t* __restrict__ img, const uint8_t* __restrict__ ids, const uint16_t* __restrict__ disp, int H,
    int W, const int* __restrict__ crop, int h, int w, float m0, float m1, float m2, float r0, float r1, float r2,
    float bf, float depth_max, TO* __restrict__ out_img, int64_t* __restrict__ out_seg,
    float* __restrict__ out_depth, uint8_t* __restrict__ out_mask, int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % w);
        const int64_t t = i / w;
        const int y = (int)(t % h);
        const int b = (int)(t / h);
        const int y0 = crop[3 * b], x0 = crop[3 * b + 1], flip = crop[3 * b + 2];
        // the host validates the windows; clamping keeps a bad one from faulting the GPU
        const int sx = min(max(flip ? x0 + w - 1 - x : x0 + x, 0), W - 1);
        const int sy = min(max(y0 + y, 0), H - 1);
        const int64_t src = ((int64_t)b * H + sy) * W + sx;
        const int64_t plane = (int64_t)h * w;
        const int64_t o = (int64_t)y * w + x;
        // image: HWC uint8 -> CHW normalised
        const uint8_t* px = img + src * 3;
        TO* oi = out_img + (int64_t)b * 3 * plane + o;
        oi[0] = (TO)(((float)px[0] - m0) * r0);
        oi[plane] = (TO)(((float)px[1] - m1) * r1);
        oi[2 * plane] = (TO)(((float)px[2] - m2) * r2);
        // segmentation: label id -> train id
        const uint8_t id = ids[src];
        out_seg[(int64_t)b * plane + o] = id < 34 ? ID_TO_TRAIN_ID[id] : 255;
        // depth from disparity
        const float d = (float)disp[src];
        const bool valid0 = d > 0.f;
        const float s = valid0 ? (d - 1.0f) / 256.0f : 0.f;
        float depth = s > 1e-3f ? bf / (s + 1e-6f) : 0.f;
        if (!(valid0 && depth <= depth_max)) depth = 0.f;
        out_depth[(int64_t)b * plane + o] = depth;
        out_mask[(int64_t)b * plane + o] = depth > 0.f;
    }
}

// ---------------------------------------------------------------------------- RandomScale + PadIfNeeded
// The trainer's full spatial pipeline (train_denseclip.py:138-149): RandomScale(0.5..2.0) ->
// PadIfNeeded(crop, image 0 / masks 255) -> RandomCrop -> HorizontalFlip, then Normalize.  The
// scale is cv2.resize to (int(H s), int(W s)): the image with interpolation flag 2 (the
// reference passes PIL's Image.BILINEAR = 2, which cv2 reads as INTER_CUBIC), the label-id
// and depth masks with INTER_NEAREST (albumentations' mask interpolation).  Restated from
// OpenCV's generic resize path for 8-bit images (resize.cpp: interpolateCubic with A = -0.75
// in f32, coefficients rounded to 11-bit fixed point, horizontal pass into int, vertical pass
// with (v + 2^21) >> 22 and saturation; replicated borders) and resizeNN (floor(x * W / Ws)).
// One thread per output pixel gathers its 4 x 4 source window straight from the decoded
// planes: no scaled intermediate image.

// OpenCV interpolateCubic + saturate_cast<short>(c * 2048), f32 with no contraction (the x86
// reference evaluates each operation in single precision)
__device__ __forceinline__ void cubic_coeffs_fx(float x, int (&c)[4]) {
#pragma clang fp contract(off)
    const float A = -0.75f;
    const float c0 = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    const float c1 = ((A + 2) * x - (A + 3)) * x * x + 1;
    const float c2 = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    const float c3 = 1.f - c0 - c1 - c2;
    const float cf[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float v = rintf(cf[k] * 2048.f);
        c[k] = (int)fminf(fmaxf(v, -32768.f), 32767.f);
    }
}

// source position of destination index d for a (src -> dst) resize: sx = floor(fx), fraction
__device__ __forceinline__ int cubic_src(int d, double scale, float& frac) {
    const float fx = (float)((d + 0.5) * scale - 0.5);
    const int sx = (int)floorf(fx);
    frac = fx - (float)sx;
    return sx;
}

// U8OUT: the image is written as the uint8 HWC crop (before ColorJitter / Normalize)
template <typename TO, bool U8OUT = false>
__global__ __launch_bounds__(256) void cityscapes_augment_kernel(
    const uint8_t* __restrict__ img, const uint8_t* __restrict__ ids, const uint16_t* __restrict__ disp, int H, int W,
    const int* __restrict__ prm, int h, int w, float m0, float m1, float m2, float r0, float r1, float r2, float bf,
    float depth_max, TO* __restrict__ out_img, int64_t* __restrict__ out_seg, float* __restrict__ out_depth,
    uint8_t* __restrict__ out_mask, int64_t total) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % w);
        const int64_t t = i / w;
        const int y = (int)(t % h);
        const int b = (int)(t / h);
        const int* p = prm + 7 * b;
        const int Hs = max(p[0], 1), Ws = max(p[1], 1), pt = p[2], pl = p[3], y0 = p[4], x0 = p[5], flip = p[6];
        const int ys = y0 + y - pt;                              // row of the scaled image
        const int xs = (flip ? x0 + w - 1 - x : x0 + x) - pl;    // column of the scaled image
        const int64_t plane = (int64_t)h * w;
        const int64_t o = (int64_t)b * plane + (int64_t)y * w + x;
        TO* oi = U8OUT ? out_img + 3 * o : out_img + (int64_t)b * 3 * plane + (int64_t)y * w + x;
        const int64_t cs = U8OUT ? 1 : plane;  // channel stride: HWC bytes or CHW normalised planes
        if (ys < 0 || ys >= Hs || xs < 0 || xs >= Ws) {  // PadIfNeeded: image 0, both masks 255
            if (U8OUT) {
                oi[0] = oi[1] = oi[2] = (TO)0;
            } else {
                oi[0] = (TO)((0.f - m0) * r0);
                oi[cs] = (TO)((0.f - m1) * r1);
                oi[2 * cs] = (TO)((0.f - m2) * r2);
            }
            out_seg[o] = 255;
            out_depth[o] = 255.f;
            out_mask[o] = 1;  // the reference re-derives validity as depth > 0 after the pad
            continue;
        }
        // cv2: inv_scale = dst / src, scale = 1 / inv_scale (double)
        const double sxs = 1.0 / ((double)Ws / (double)W), sys = 1.0 / ((double)Hs / (double)H);
        // ---- image: INTER_CUBIC, 8-bit fixed point
        float fx, fy;
        const int sx = cubic_src(xs, sxs, fx), sy = cubic_src(ys, sys, fy);
        int ax[4], by[4];
        cubic_coeffs_fx(fx, ax);
        cubic_coeffs_fx(fy, by);
        int acc[3] = {0, 0, 0};
        const uint8_t* base = img + (int64_t)b * H * W * 3;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = min(max(sy - 1 + k, 0), H - 1);
            const uint8_t* row = base + (int64_t)r * W * 3;
            int hv[3] = {0, 0, 0};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = min(max(sx - 1 + j, 0), W - 1);
                hv[0] += (int)row[3 * c] * ax[j];
                hv[1] += (int)row[3 * c + 1] * ax[j];
                hv[2] += (int)row[3 * c + 2] * ax[j];
            }
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) acc[ch] += hv[ch] * by[k];
        }
        float px[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) px[ch] = (float)min(max((acc[ch] + (1 << 21)) >> 22, 0), 255);
        if (U8OUT) {
            oi[0] = (TO)px[0];
            oi[1] = (TO)px[1];
            oi[2] = (TO)px[2];
        } else {
            oi[0] = (TO)((px[0] - m0) * r0);
            oi[cs] = (TO)((px[1] - m1) * r1);
            oi[2 * cs] = (TO)((px[2] - m2) * r2);
        }
        // ---- masks: INTER_NEAREST, x_ofs = min(floor(x * W / Ws), W - 1)
        const int nx = min((int)floor((double)xs * sxs), W - 1);
        const int ny = min((int)floor((double)ys * sys), H - 1);
        const int64_t src = ((int64_t)b * H + ny) * W + nx;
        const uint8_t id = ids[src];
        out_seg[o] = id < 34 ? ID_TO_TRAIN_ID[id] : 255;
        const float d = (float)disp[src];
        const bool valid0 = d > 0.f;
        const float s = valid0 ? (d - 1.0f) / 256.0f : 0.f;
        float depth = s > 1e-3f ? bf / (s + 1e-6f) : 0.f;
        if (!(valid0 && depth <= depth_max)) depth = 0.f;
        out_depth[o] = depth;
        out_mask[o] = depth > 0.f;
    }
}

// ---------------------------------------------------------------------------- ColorJitter
// albumentations ColorJitter(brightness, contrast, saturation, hue) on uint8 RGB
// (train_denseclip.py:152-155, inserted before Normalize), restated from albumentations'
// *_torchvision uint8 functions and OpenCV's 8-bit colour conversions (cv2 / albumentations are
// not installed here: parity against them is unpinned):
//   brightness f: LUT clip(i f, 0, 255) -> uint8 (truncation; f64)
//   contrast f:   m = mean of cvtColor(RGB2GRAY); LUT clip(i f + m (1 - f), 0, 255) -> uint8 (f64)
//   saturation f: addWeighted(img, f, gray3, 1 - f, 0): saturate(cvRound(x f + g (1 - f))) in f32
//   hue f:        RGB2HSV (8-bit, 12-bit fixed-point division tables, hue range 180), hue through
//                 LUT (i + 180 f) mod 180 -> uint8, HSV2RGB (f32, sector table), round to uint8
// each image with its own factors and its own random order of the four (params (B, 8) f64:
// brightness, contrast, saturation, hue, order[4]); one launch per position in the order, the
// gray mean of the image as it stands before each position.
__device__ __forceinline__ int gray_u8(int r, int g, int b) { return (r * 4899 + g * 9617 + b * 1868 + 8192) >> 14; }

__device__ __forceinline__ uint8_t sat_round_u8(float v) {
    const float t = rintf(v);
    return (uint8_t)(t < 0.f ? 0.f : (t > 255.f ? 255.f : t));
}

__global__ __launch_bounds__(256) void gray_sum_kernel(const uint8_t* __restrict__ img, int64_t hw,
                                                       unsigned long long* __restrict__ sums) {
    const int b = blockIdx.y;
    const uint8_t* p = img + (int64_t)b * hw * 3;
    unsigned int s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hw; i += (int64_t)gridDim.x * blockDim.x)
        s += gray_u8(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
    for (int o = 32; o >= 1; o >>= 1) s += (unsigned int)__shfl_xor((int)s, o);
    __shared__ unsigned int red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(sums + b, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

__device__ __forceinline__ void rgb2hsv_u8(int r, int g, int b, int& h, int& s, int& v) {
    v = max(max(b, g), r);
    const int vmin = min(min(b, g), r);
    const int diff = v - vmin;
    const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    // sdiv = round((255 << 12) / v), hdiv = round((180 << 12) / (6 diff)); 0 for v, diff = 0
    const int sdiv = v ? (int)rint((double)(255 << 12) / (double)v) : 0;
    const int hdiv = diff ? (int)rint((double)(180 << 12) / (6.0 * diff)) : 0;
    s = (diff * sdiv + (1 << 11)) >> 12;
    int hh = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
    hh = (hh * hdiv + (1 << 11)) >> 12;
    hh += hh < 0 ? 180 : 0;
    h = min(hh, 255);
}

__device__ __forceinline__ void hsv2rgb_u8(int hi, int si, int vi, int& r, int& g, int& b) {
#pragma clang fp contract(off)
    float h = (float)hi, s = (float)si * (1.0f / 255.0f), v = (float)vi * (1.0f / 255.0f);
    float bb, gg, rr;
    if (s == 0.f) {
        bb = gg = rr = v;
    } else {
        h *= 6.0f / 180.0f;
        while (h < 0.f) h += 6.f;
        while (h >= 6.f) h -= 6.f;
        int sector = (int)floorf(h);
        h -= (float)sector;
        if ((unsigned)sector >= 6u) {
            sector = 0;
            h = 0.f;
        }
        const float tab[4] = {v, v * (1.f - s), v * (1.f - s * h), v * (1.f - s * (1.f - h))};
        const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        bb = tab[sd[sector][0]];
        gg = tab[sd[sector][1]];
        rr = tab[sd[sector][2]];
    }
    r = sat_round_u8(rr * 255.f);
    g = sat_round_u8(gg * 255.f);
    b = sat_round_u8(bb * 255.f);
}

__global__ __launch_bounds__(256) void color_jitter_kernel(uint8_t* __restrict__ img, int64_t hw,
                                                           const double* __restrict__ prm,
                                                           const unsigned long long* __restrict__ sums, int pos) {
#pragma clang fp contract(off)
    const int b = blockIdx.y;
    const double* p = prm + 8 * b;
    const int op = (int)p[4 + pos];
    const double f = p[op];
    if ((op == 3 && f == 0.0) || (op != 3 && f == 1.0)) return;  // the identity factor: untouched
    uint8_t* q = img + (int64_t)b * hw * 3;
    const double mean = (double)sums[b] / (double)hw;
    const float af = (float)f, bf_ = (float)(1.0 - f);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hw; i += (int64_t)gridDim.x * blockDim.x) {
        int c[3] = {q[3 * i], q[3 * i + 1], q[3 * i + 2]};
        if (op == 0 || op == 1) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                double t = (double)c[k] * f;
                if (op == 1) t = t + mean * (1.0 - f);
                t = t < 0.0 ? 0.0 : (t > 255.0 ? 255.0 : t);
                c[k] = (int)t;
            }
        } else if (op == 2) {
            const float g = (float)gray_u8(c[0], c[1], c[2]);
#pragma unroll
            for (int k = 0; k < 3; ++k) c[k] = sat_round_u8((float)c[k] * af + g * bf_ + 0.f);
        } else {
            int h, s, v;
            rgb2hsv_u8(c[0], c[1], c[2], h, s, v);
            double t = fmod((double)h + 180.0 * f, 180.0);
            if (t < 0.0) t += 180.0;
            h = (int)t;
            hsv2rgb_u8(h, s, v, c[0], c[1], c[2]);
        }
        q[3 * i] = (uint8_t)c[0];
        q[3 * i + 1] = (uint8_t)c[1];
        q[3 * i + 2] = (uint8_t)c[2];
    }
}

// Normalize + ToTensorV2 of a uint8 HWC batch: (x - 255 mean) * (1 / (255 std)) -> CHW
template <typename TO>
__global__ __launch_bounds__(256) void normalize_u8_kernel(const uint8_t* __restrict__ img, int64_t hw, int64_t total,
                                                           float m0, float m1, float m2, float r0, float r1,
                                                           float r2, TO* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / hw, o = i - b * hw;
        const uint8_t* px = img + 3 * i;
        TO* oi = out + b * 3 * hw + o;
        oi[0] = (TO)(((float)px[0] - m0) * r0);
        oi[hw] = (TO)(((float)px[1] - m1) * r1);
        oi[2 * hw] = (TO)(((float)px[2] - m2) * r2);
    }
}

}  // namespace

extern "C" int dclip_color_jitter(uint8_t* img, int B, int h, int w, const double* params, unsigned long long* ws,
                                  void* stream) {
    DCLIP_HOST_CHECK(img && params && ws && B > 0 && h > 0 && w > 0, "dclip_color_jitter: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    const int64_t hw = (int64_t)h * w;
    int gx = (int)((hw + 255) / 256);
    gx = gx > 1024 ? 1024 : gx;
    for (int pos = 0; pos < 4; ++pos) {
        if (hipMemsetAsync(ws, 0, sizeof(unsigned long long) * B, st) != hipSuccess) {
            dclip_set_error("dclip_color_jitter: hipMemsetAsync failed");
            return DCLIP_ERR_HIP;
        }
        gray_sum_kernel<<<dim3(gx, B), 256, 0, st>>>(img, hw, ws);
        color_jitter_kernel<<<dim3(gx, B), 256, 0, st>>>(img, hw, params, ws, pos);
    }
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_normalize_u8(const uint8_t* img, int B, int h, int w, const float* mean, const float* stdv,
                                  void* out, int out_dt, void* stream) {
    DCLIP_HOST_CHECK(img && mean && stdv && out && B > 0 && h > 0 && w > 0, "dclip_normalize_u8: bad arguments");
    DCLIP_HOST_CHECK(out_dt == DCLIP_F32 || out_dt == DCLIP_BF16 || out_dt == DCLIP_F16,
                     "dclip_normalize_u8: out_dt must be F32, BF16 or F16");
    float m[3], r[3];
    for (int c = 0; c < 3; ++c) {
        m[c] = mean[c] * 255.0f;
        r[c] = 1.0f / (stdv[c] * 255.0f);
    }
    const int64_t hw = (int64_t)h * w, total = (int64_t)B * hw;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipStream_t st = (hipStream_t)stream;
    if (out_dt == DCLIP_F32)
        normalize_u8_kernel<float><<<(unsigned)blocks, 256, 0, st>>>(img, hw, total, m[0], m[1], m[2], r[0], r[1], r[2],
                                                                     (float*)out);
    else if (out_dt == DCLIP_BF16)
        normalize_u8_kernel<bf16><<<(unsigned)blocks, 256, 0, st>>>(img, hw, total, m[0], m[1], m[2], r[0], r[1], r[2],
                                                                    (bf16*)out);
    else
        normalize_u8_kernel<f16><<<(unsigned)blocks, 256, 0, st>>>(img, hw, total, m[0], m[1], m[2], r[0], r[1], r[2],
                                                                   (f16*)out);
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_cityscapes_augment(const uint8_t* img, const uint8_t* ids, const uint16_t* disp, int B, int H,
                                        int W, const int* params, int h, int w, const float* mean, const float* stdv,
                                        float bf, float depth_max, void* out_img, int out_dt, int64_t* out_seg,
                                        float* out_depth, uint8_t* out_mask, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && H > 0 && W > 0 && h > 0 && w > 0, "dclip_cityscapes_augment: bad sizes B=%d H=%d W=%d "
                     "crop %dx%d", B, H, W, h, w);
    DCLIP_HOST_CHECK((int64_t)H * W * 3 < (1ll << 31), "dclip_cityscapes_augment: image too large");
    DCLIP_HOST_CHECK(img && ids && disp && params && mean && stdv && out_img && out_seg && out_depth && out_mask,
                     "dclip_cityscapes_augment: null pointer");
    DCLIP_HOST_CHECK(out_dt == DCLIP_F32 || out_dt == DCLIP_BF16 || out_dt == DCLIP_F16 || out_dt == DCLIP_U8,
                     "dclip_cityscapes_augment: out_dt must be F32, BF16, F16 or U8 (HWC, not normalised)");
    float m[3], r[3];
    for (int c = 0; c < 3; ++c) {
        m[c] = mean[c] * 255.0f;
        r[c] = 1.0f / (stdv[c] * 255.0f);
    }
    const int64_t total = (int64_t)B * h * w;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipStream_t st = (hipStream_t)stream;
#define DCLIP_AUG(TO)                                                                                               \
    cityscapes_augment_kernel<TO><<<(unsigned)blocks, 256, 0, st>>>(img, ids, disp, H, W, params, h, w, m[0], m[1],  \
                                                                    m[2], r[0], r[1], r[2], bf, depth_max,           \
                                                                    (TO*)out_img, out_seg, out_depth, out_mask, total)
    if (out_dt == DCLIP_F32) DCLIP_AUG(float);
    else if (out_dt == DCLIP_BF16) DCLIP_AUG(bf16);
    else if (out_dt == DCLIP_F16) DCLIP_AUG(f16);
    else
        cityscapes_augment_kernel<uint8_t, true><<<(unsigned)blocks, 256, 0, st>>>(
            img, ids, disp, H, W, params, h, w, m[0], m[1], m[2], r[0], r[1], r[2], bf, depth_max, (uint8_t*)out_img,
            out_seg, out_depth, out_mask, total);
#undef DCLIP_AUG
    DCLIP_LAUNCH_CHECK();
    return 0;
}

extern "C" int dclip_cityscapes_prepare(const uint8_t* img, const uint8_t* ids, const uint16_t* disp, int B, int H,
                                        int W, const int* crop, int h, int w, const float* mean, const float* stdv,
                                        float bf, float depth_max, void* out_img, int out_dt, int64_t* out_seg,
                                        float* out_depth, uint8_t* out_mask, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && H > 0 && W > 0 && h > 0 && w > 0 && h <= H && w <= W,
                     "dclip_cityscapes_prepare: bad sizes B=%d H=%d W=%d crop %dx%d", B, H, W, h, w);
    DCLIP_HOST_CHECK(img && ids && disp && crop && mean && stdv && out_img && out_seg && out_depth && out_mask,
                     "dclip_cityscapes_prepare: null pointer");
    DCLIP_HOST_CHECK(out_dt == DCLIP_F32 || out_dt == DCLIP_BF16 || out_dt == DCLIP_F16,
                     "dclip_cityscapes_prepare: out_dt must be F32, BF16 or F16");
    // the reference's f32 constants: mean * 255 and 1 / (std * 255), each rounded once
    float m[3], r[3];
    for (int c = 0; c < 3; ++c) {
        m[c] = mean[c] * 255.0f;
        r[c] = 1.0f / (stdv[c] * 255.0f);
    }
    const int64_t total = (int64_t)B * h * w;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipStream_t st = (hipStream_t)stream;
#define DCLIP_PREP(TO)                                                                                              \
    cityscapes_prepare_kernel<TO><<<(unsigned)blocks, 256, 0, st>>>(img, ids, disp, H, W, crop, h, w, m[0], m[1],     \
                                                                    m[2], r[0], r[1], r[2], bf, depth_max,           \
                                                                    (TO*)out_img, out_seg, out_depth, out_mask, total)
    if (out_dt == DCLIP_F32) DCLIP_PREP(float);
    else if (out_dt == DCLIP_BF16) DCLIP_PREP(bf16);
    else DCLIP_PREP(f16);
#undef DCLIP_PREP
    DCLIP_LAUNCH_CHECK();
    return 0;
}
