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

}  // namespace

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
