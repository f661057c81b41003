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

template <typename TO>
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
        TO* oi = out_img + (int64_t)b * 3 * plane + (int64_t)y * w + x;
        if (ys < 0 || ys >= Hs || xs < 0 || xs >= Ws) {  // PadIfNeeded: image 0, both masks 255
            oi[0] = (TO)((0.f - m0) * r0);
            oi[plane] = (TO)((0.f - m1) * r1);
            oi[2 * plane] = (TO)((0.f - m2) * r2);
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
        oi[0] = (TO)((px[0] - m0) * r0);
        oi[plane] = (TO)((px[1] - m1) * r1);
        oi[2 * plane] = (TO)((px[2] - m2) * r2);
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

}  // namespace

extern "C" int dclip_cityscapes_augment(const uint8_t* img, const uint8_t* ids, const uint16_t* disp, int B, int H,
                                        int W, const int* params, int h, int w, const float* mean, const float* stdv,
                                        float bf, float depth_max, void* out_img, int out_dt, int64_t* out_seg,
                                        float* out_depth, uint8_t* out_mask, void* stream) {
    DCLIP_HOST_CHECK(B > 0 && H > 0 && W > 0 && h > 0 && w > 0, "dclip_cityscapes_augment: bad sizes B=%d H=%d W=%d "
                     "crop %dx%d", B, H, W, h, w);
    DCLIP_HOST_CHECK((int64_t)H * W * 3 < (1ll << 31), "dclip_cityscapes_augment: image too large");
    DCLIP_HOST_CHECK(img && ids && disp && params && mean && stdv && out_img && out_seg && out_depth && out_mask,
                     "dclip_cityscapes_augment: null pointer");
    DCLIP_HOST_CHECK(out_dt == DCLIP_F32 || out_dt == DCLIP_BF16 || out_dt == DCLIP_F16,
                     "dclip_cityscapes_augment: out_dt must be F32, BF16 or F16");
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
    else DCLIP_AUG(f16);
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
