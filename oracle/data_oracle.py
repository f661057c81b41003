"""CPU restatement of the Cityscapes depth + segmentation sample preparation — TEST
INFRASTRUCTURE ONLY (the checker for dclip_cityscapes_prepare; never imported by the product).

Follows /root/reference/segmentation/datasets/cityscapes_depth_seg.py (NumPy, f32) and the
trainer's RandomCrop / HorizontalFlip / Normalize / ToTensorV2 (train_denseclip.py:143-149).
The label and depth functions are pinned by tests/golden/data_prep.safetensors, produced by
running the reference's own functions (tests/golden/gen_data_golden.py).  The normalisation
restates albumentations' Normalize ((x - 255 mean) * (1 / (255 std)), f32); albumentations is
not installed, so that step is parity unpinned.
"""
import numpy as np

# cityscapes_depth_seg.py:43-45
ID_TO_TRAIN_ID = np.array([255, 255, 255, 255, 255, 255, 255, 0, 1, 255, 255, 2, 3, 4,
                           255, 255, 255, 5, 255, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                           255, 255, 16, 17, 18], dtype=np.uint8)


def map_labels(ids):
    """map_labels_fast (cityscapes_depth_seg.py:129-135): ids < 34 through the table, else 255."""
    out = np.full_like(ids, 255, dtype=np.uint8)
    ok = ids < len(ID_TO_TRAIN_ID)
    out[ok] = ID_TO_TRAIN_ID[ids[ok]]
    return out


def disparity_to_depth(disp, bf=500.0, depth_max=80.0):
    """disparity_to_depth (cityscapes_depth_seg.py:137-170) -> (depth f32, valid uint8)."""
    d = disp.astype(np.float32)
    valid0 = d > 0
    s = np.zeros_like(d)
    s[valid0] = (d[valid0] - np.float32(1.0)) / np.float32(256.0)
    use = s > np.float32(1e-3)
    depth = np.zeros_like(s)
    depth[use] = np.float32(bf) / (s[use] + np.float32(1e-6))
    valid = valid0 & (depth <= np.float32(depth_max))
    depth[~valid] = 0.0
    return depth, valid.astype(np.uint8)


def normalize(img, mean, std):
    """albumentations Normalize(max_pixel_value=255) as used at train_denseclip.py:147, f32."""
    m = np.asarray(mean, np.float32) * np.float32(255.0)
    r = np.float32(1.0) / (np.asarray(std, np.float32) * np.float32(255.0))
    return (img.astype(np.float32) - m) * r


def prepare(samples, crop_hw, crops, mean, std, bf=500.0, depth_max=80.0):
    """The batch dclip_cityscapes_prepare writes: crop window, optional mirror, normalised CHW
    image, train ids, depth and the post-transform mask depth > 0 (cityscapes_depth_seg.py:218)."""
    h, w = crop_hw
    imgs, segs, depths, masks = [], [], [], []
    for (img, ids, disp), (y0, x0, flip) in zip(samples, crops):
        win = (slice(y0, y0 + h), slice(x0, x0 + w))
        im, lab, dp = img[win], ids[win], disp[win]
        if flip:
            im, lab, dp = im[:, ::-1], lab[:, ::-1], dp[:, ::-1]
        depth, _ = disparity_to_depth(dp, bf, depth_max)
        imgs.append(normalize(im, mean, std).transpose(2, 0, 1))
        segs.append(map_labels(lab).astype(np.int64))
        depths.append(depth[None])
        masks.append((depth > 0)[None])
    return np.stack(imgs), np.stack(segs), np.stack(depths), np.stack(masks)


# ---------------------------------------------------------------------------- RandomScale + PadIfNeeded
# train_denseclip.py:138-149.  cv2 is not installed here: the resize below restates OpenCV's generic
# 8-bit resize path (modules/imgproc/src/resize.cpp: interpolateCubic, fixed-point HResizeCubic /
# VResizeCubic, resizeNN) — parity against cv2 itself is UNPINNED; tests/test_data_cpu.py holds it
# within 1 LSB of torch's float bicubic (same A = -0.75 kernel, half-pixel centres, clamped borders).
def _cubic_coeffs(fx):
    """interpolateCubic(fx) (A = -0.75, f32 op by op) rounded to 11-bit fixed point (int32 (n, 4))."""
    f32 = np.float32
    x = fx.astype(f32)
    A = f32(-0.75)
    one = f32(1)
    c0 = ((A * (x + one) - f32(5) * A) * (x + one) + f32(8) * A) * (x + one) - f32(4) * A
    c1 = ((A + f32(2)) * x - (A + f32(3))) * x * x + one
    c2 = ((A + f32(2)) * (one - x) - (A + f32(3))) * (one - x) * (one - x) + one
    c3 = one - c0 - c1 - c2
    c = np.stack([c0, c1, c2, c3], -1) * f32(2048)
    return np.clip(np.rint(c), -32768, 32767).astype(np.int64)


def _cubic_src(n_dst, n_src):
    """sx = floor(fx), frac, fx = (float)((d + 0.5) * scale - 0.5), scale = 1 / (dst / src)."""
    scale = 1.0 / (float(n_dst) / float(n_src))
    fx = ((np.arange(n_dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    return sx, fx - sx.astype(np.float32)


def resize_cubic_u8(img, Hs, Ws):
    """cv2.resize(img (H, W, 3) uint8, (Ws, Hs), INTER_CUBIC) restated (see above)."""
    H, W = img.shape[:2]
    sx, fx = _cubic_src(Ws, W)
    sy, fy = _cubic_src(Hs, H)
    ax, by = _cubic_coeffs(fx), _cubic_coeffs(fy)
    cols = np.clip(sx[:, None] - 1 + np.arange(4), 0, W - 1)  # (Ws, 4)
    rows = np.clip(sy[:, None] - 1 + np.arange(4), 0, H - 1)  # (Hs, 4)
    src = img.astype(np.int64)
    hv = (src[:, cols, :] * ax[None, :, :, None]).sum(2)       # (H, Ws, 3) horizontal pass, int
    v = (hv[rows, :, :] * by[:, :, None, None]).sum(1)          # (Hs, Ws, 3)
    return np.clip((v + (1 << 21)) >> 22, 0, 255).astype(np.uint8)


def resize_nearest(a, Hs, Ws):
    """cv2.resize(a, (Ws, Hs), INTER_NEAREST): index min(floor(d * src / dst), src - 1)."""
    H, W = a.shape[:2]
    ix = np.minimum(np.floor(np.arange(Ws) * (1.0 / (float(Ws) / W))).astype(np.int64), W - 1)
    iy = np.minimum(np.floor(np.arange(Hs) * (1.0 / (float(Hs) / H))).astype(np.int64), H - 1)
    return a[iy][:, ix]


def scale_pad_params(H, W, h, w, scale, h_start, w_start, flip):
    """albumentations RandomScale (int(H s), int(W s)), PadIfNeeded (centred: top = int(pad / 2)),
    RandomCrop (y0 = int((Hp - h + 1) * h_start)) -> (Hs, Ws, pad_top, pad_left, y0, x0, flip)."""
    Hs, Ws = int(H * scale), int(W * scale)
    ph, pw = max(0, h - Hs), max(0, w - Ws)
    pt, pl = int(ph / 2.0), int(pw / 2.0)
    Hp, Wp = Hs + ph, Ws + pw
    return (Hs, Ws, pt, pl, int((Hp - h + 1) * h_start), int((Wp - w + 1) * w_start), int(bool(flip)))


def prepare_augmented(samples, crop_hw, params, mean, std, bf=500.0, depth_max=80.0):
    """dclip_cityscapes_augment: per sample resize (image cubic, label ids / disparity nearest),
    pad (image 0, seg 255, depth 255.0), crop, mirror, then the prepare() outputs."""
    h, w = crop_hw
    imgs, segs, depths, masks = [], [], [], []
    for (img, ids, disp), (Hs, Ws, pt, pl, y0, x0, flip) in zip(samples, params):
        H, W = ids.shape
        im = img if (Hs, Ws) == (H, W) else resize_cubic_u8(img, Hs, Ws)
        lab = map_labels(resize_nearest(ids, Hs, Ws))
        dep, _ = disparity_to_depth(resize_nearest(disp, Hs, Ws), bf, depth_max)
        Hp, Wp = max(Hs + pt, y0 + h), max(Ws + pl, x0 + w)  # a canvas holding the image and the window
        pim = np.zeros((Hp, Wp, 3), np.uint8)
        plab = np.full((Hp, Wp), 255, np.uint8)
        pdep = np.full((Hp, Wp), 255.0, np.float32)
        pim[pt:pt + Hs, pl:pl + Ws], plab[pt:pt + Hs, pl:pl + Ws], pdep[pt:pt + Hs, pl:pl + Ws] = im, lab, dep
        win = (slice(y0, y0 + h), slice(x0, x0 + w))
        im, lab, dep = pim[win], plab[win], pdep[win]
        if flip:
            im, lab, dep = im[:, ::-1], lab[:, ::-1], dep[:, ::-1]
        imgs.append(normalize(im, mean, std).transpose(2, 0, 1))
        segs.append(lab.astype(np.int64))
        depths.append(dep[None])
        masks.append((dep > 0)[None])
    return np.stack(imgs), np.stack(segs), np.stack(depths), np.stack(masks)


# ---------------------------------------------------------------------------- ColorJitter
# albumentations ColorJitter on uint8 RGB (train_denseclip.py:152-155): the *_torchvision uint8
# functions and OpenCV's 8-bit RGB2GRAY / RGB2HSV / HSV2RGB, restated from their published code
# (neither is installed here: parity against them is UNPINNED; the GPU kernel is held to this).
def _gray_u8(img):
    x = img.astype(np.int64)
    return (x[..., 0] * 4899 + x[..., 1] * 9617 + x[..., 2] * 1868 + 8192) >> 14


def _rgb2hsv_u8(img):
    x = img.astype(np.int64)
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    i = np.arange(256, dtype=np.float64)
    with np.errstate(divide="ignore"):
        sdiv = np.where(i > 0, np.rint((255 << 12) / i), 0).astype(np.int64)
        hdiv = np.where(i > 0, np.rint((180 << 12) / (6.0 * i)), 0).astype(np.int64)
    s = (diff * sdiv[v] + (1 << 11)) >> 12
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))))
    h = (h * hdiv[diff] + (1 << 11)) >> 12
    h = np.where(h < 0, h + 180, h)
    return np.minimum(h, 255), s, v


def _hsv2rgb_u8(h, s, v):
    f32 = np.float32
    hf = h.astype(f32)
    sf = s.astype(f32) * f32(1.0 / 255.0)
    vf = v.astype(f32) * f32(1.0 / 255.0)
    hh = hf * (f32(6.0) / f32(180.0))
    hh = np.where(hh >= f32(6), hh - f32(6), hh)
    sector = np.floor(hh).astype(np.int64)
    hh = hh - sector.astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    hh = np.where(bad, f32(0), hh)
    one = f32(1)
    tab = np.stack([vf, vf * (one - sf), vf * (one - sf * hh), vf * (one - sf * (one - hh))], -1)
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sd[sector]                                    # (..., 3): b, g, r table slots
    bgr = np.take_along_axis(tab, idx, -1)
    gray = sf == 0
    bgr = np.where(gray[..., None], vf[..., None], bgr)
    rgb = bgr[..., ::-1] * f32(255)
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)


def color_jitter(img, params):
    """One image (h, w, 3) uint8 through the jitter ops in params' order (see
    data.color_jitter_params)."""
    img = img.copy()
    fac, order = params[:4], [int(o) for o in params[4:]]
    for op in order:
        f = float(fac[op])
        if (op == 3 and f == 0.0) or (op != 3 and f == 1.0):
            continue
        if op in (0, 1):
            lut = np.arange(0, 256) * f
            if op == 1:
                lut = lut + _gray_u8(img).mean() * (1 - f)
            img = np.clip(lut, 0, 255).astype(np.uint8)[img]
        elif op == 2:
            g = _gray_u8(img).astype(np.float32)[..., None]
            t = img.astype(np.float32) * np.float32(f) + g * np.float32(1 - f) + np.float32(0)
            img = np.clip(np.rint(t), 0, 255).astype(np.uint8)
        else:
            h, s, v = _rgb2hsv_u8(img)
            lut = np.mod(np.arange(0, 256, dtype=np.int16) + 180 * f, 180).astype(np.uint8)
            img = _hsv2rgb_u8(lut[h].astype(np.int64), s, v)
    return img


def prepare_augmented_jitter(samples, crop_hw, params, jitter, mean, std, bf=500.0, depth_max=80.0):
    """prepare_augmented with ColorJitter on the uint8 crop before Normalize."""
    h, w = crop_hw
    imgs, segs, depths, masks = prepare_augmented(samples, crop_hw, params, (0.0, 0.0, 0.0), (1 / 255.0,) * 3, bf,
                                                  depth_max)
    out = []
    for b in range(len(samples)):
        # undo the identity normalisation above exactly: it wrote (x - 0) * (1 / (255 / 255)) = x
        u8 = np.rint(imgs[b].transpose(1, 2, 0)).astype(np.uint8)
        out.append(normalize(color_jitter(u8, jitter[b]), mean, std).transpose(2, 0, 1))
    return np.stack(out), segs, depths, masks
