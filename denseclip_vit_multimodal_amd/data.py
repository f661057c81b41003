"""Cityscapes depth + segmentation data path, GPU-side.

The reference loader (seg/datasets/cityscapes_depth_seg.py) decodes three PNGs per sample,
remaps label ids, turns the uint16 disparity into metric depth and runs the trainer's
albumentations pipeline on the CPU, then ships f32 / int64 tensors (25 bytes per pixel).
Here the CPU only scans and decodes (`CityscapesDepthSegDataset`, same file layout, names and
errors as the reference); `prepare_batch` uploads the decoded uint8 / uint16 planes (6 bytes
per pixel) and one HIP kernel does the label remap, the disparity -> depth conversion, the
trainer's spatial augmentation and the normalisation, writing the batch in the layout
`train.train_step` takes:
  * `dclip_cityscapes_augment` (params from `random_scale_crops`): the whole train pipeline of
    train_denseclip.py:138-149, RandomScale(0.5..2.0) -> PadIfNeeded -> RandomCrop ->
    HorizontalFlip -> Normalize, with cv2's 8-bit INTER_CUBIC for the image (the reference's
    interpolation=Image.BILINEAR is the integer 2, which cv2 reads as INTER_CUBIC) and
    INTER_NEAREST for the label ids / disparity, restated from OpenCV's resize (cv2 is not
    installed here: that restatement is parity-unpinned against cv2 itself);
  * `dclip_cityscapes_prepare` (crops from `random_crops`): crop + flip only (no rescale).

  * ColorJitter (the reference's `color_jitter: true`, off in the Cityscapes configs): params from
    `color_jitter_params`, `dclip_color_jitter` between the spatial transforms and Normalize.
"""
import os
import os.path as osp

import numpy as np
import torch



# reference constants (datasets/cityscapes_depth_seg.py:19-23) and CLIP normalisation
# (train_denseclip.py:113-114)
BASELINE_FOCAL_LENGTH = 500.0
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)
SEG_IGNORE_INDEX = 255


class CityscapesDepthSegDataset:
    """File scan and PNG decode of the reference dataset (cityscapes_depth_seg.py:57-126):
    `root/leftImg8bit/<split>/<city>/*_leftImg8bit.png` with `gtFine/..._gtFine_labelIds.png` and
    `disparity/..._disparity.png`.  `__getitem__` returns the DECODED planes (uint8 HxWx3 RGB,
    uint8 HxW label ids, uint16 HxW disparity); `prepare_batch` turns a list of them into the
    training batch on the GPU.  Unlike the reference, a broken file raises instead of
    returning Nones."""

    CLASSES = ('road', 'sidewalk', 'building', 'wall', 'fence', 'pole', 'traffic light', 'traffic sign',
               'vegetation', 'terrain', 'sky', 'person', 'rider', 'car', 'truck', 'bus', 'train', 'motorcycle',
               'bicycle')
    SEG_IGNORE_INDEX = SEG_IGNORE_INDEX

    def __init__(self, root, split="train", depth_max=80.0):
        self.root, self.split, self.depth_max = root, split, depth_max
        self.bf = BASELINE_FOCAL_LENGTH
        self.images_base = osp.join(root, "leftImg8bit", split)
        self.labels_base = osp.join(root, "gtFine", split)
        self.disparity_base = osp.join(root, "disparity", split)
        for d, what in ((self.images_base, "Image"), (self.labels_base, "Label"), (self.disparity_base, "Disparity")):
            if not osp.isdir(d):
                raise RuntimeError(f"{what} dir not found: {d}")
        self.img_files, self.label_files, self.disp_files = [], [], []
        for city in sorted(os.listdir(self.images_base)):
            img_dir = osp.join(self.images_base, city)
            label_dir = osp.join(self.labels_base, city)
            disp_dir = osp.join(self.disparity_base, city)
            if not (osp.isdir(img_dir) and osp.isdir(label_dir) and osp.isdir(disp_dir)):
                continue
            for fn in sorted(os.listdir(img_dir)):
                if not fn.endswith("_leftImg8bit.png"):
                    continue
                base = fn[: -len("_leftImg8bit.png")]
                lp = osp.join(label_dir, f"{base}_gtFine_labelIds.png")
                dp = osp.join(disp_dir, f"{base}_disparity.png")
                if osp.exists(lp) and osp.exists(dp):
                    self.img_files.append(osp.join(img_dir, fn))
                    self.label_files.append(lp)
                    self.disp_files.append(dp)
        if not self.img_files:
            raise RuntimeError(f"No valid data triplets found for split '{split}' in {root}")

    def __len__(self):
        return len(self.img_files)

    def __getitem__(self, idx):
        from PIL import Image
        img = np.asarray(Image.open(self.img_files[idx]).convert("RGB"), dtype=np.uint8)
        ids = np.asarray(Image.open(self.label_files[idx]), dtype=np.uint8)
        disp = np.asarray(Image.open(self.disp_files[idx])).astype(np.uint16)
        if ids.shape != img.shape[:2] or disp.shape != img.shape[:2]:
            raise RuntimeError(f"sample {idx}: image {img.shape[:2]}, labels {ids.shape}, disparity {disp.shape}")
        return img, ids, disp


def random_crops(B, H, W, h, w, generator=None, flip_p=0.5):
    """RandomCrop + HorizontalFlip parameters (y0, x0, flip) per image, int32 (B, 3)."""
    if h > H or w > W:
        raise ValueError(f"crop {h}x{w} larger than the image {H}x{W} (padding is not supported)")
    g = generator
    y0 = torch.randint(0, H - h + 1, (B,), generator=g)
    x0 = torch.randint(0, W - w + 1, (B,), generator=g)
    flip = (torch.rand(B, generator=g) < flip_p).to(torch.int64)
    return torch.stack([y0, x0, flip], 1).to(torch.int32)


def random_scale_crops(B, H, W, h, w, scale_range=(0.5, 2.0), rng=None, flip_p=0.5):
    """RandomScale + PadIfNeeded + RandomCrop + HorizontalFlip parameters per image, int32 (B, 7) =
    (Hs, Ws, pad_top, pad_left, y0, x0, flip), drawn like albumentations (train_denseclip.py:
    138-149): scale ~ U(scale_range), (Hs, Ws) = (int(H s), int(W s)); centred padding up to
    the crop, top = int(pad / 2); y0 = int((Hp - h + 1) u), x0 likewise; flip with flip_p.
    rng: a `random.Random` (albumentations draws from Python's `random`)."""
    import random
    r = rng if rng is not None else random
    out = []
    for _ in range(B):
        s = r.uniform(scale_range[0], scale_range[1])
        Hs, Ws = int(H * s), int(W * s)
        ph, pw = max(0, h - Hs), max(0, w - Ws)
        pt, pl = int(ph / 2.0), int(pw / 2.0)
        Hp, Wp = Hs + ph, Ws + pw
        y0 = int((Hp - h + 1) * r.random())
        x0 = int((Wp - w + 1) * r.random())
        out.append((Hs, Ws, pt, pl, y0, x0, int(r.random() < flip_p)))
    return torch.tensor(out, dtype=torch.int32)


def color_jitter_params(B, rng=None, brightness=0.4, contrast=0.4, saturation=0.4, hue=0.1, p=0.8):
    """ColorJitter(brightness, contrast, saturation, hue, p) parameters per image as albumentations
    draws them (train_denseclip.py:152-155): with probability p, factors U(1 - b, 1 + b) (clipped at
    0) for brightness / contrast / saturation, U(-hue, hue) for hue, and a random order of the four;
    otherwise the identity (1, 1, 1, 0).  float64 (B, 8): factors, then the order (0 brightness,
    1 contrast, 2 saturation, 3 hue).  rng: a `random.Random`."""
    import random
    r = rng if rng is not None else random
    out = []
    for _ in range(B):
        if r.random() < p:
            f = [r.uniform(max(0.0, 1 - brightness), 1 + brightness), r.uniform(max(0.0, 1 - contrast), 1 + contrast),
                 r.uniform(max(0.0, 1 - saturation), 1 + saturation), r.uniform(-hue, hue)]
            order = [0, 1, 2, 3]
            r.shuffle(order)
        else:
            f, order = [1.0, 1.0, 1.0, 0.0], [0, 1, 2, 3]
        out.append(f + [float(o) for o in order])
    return torch.tensor(out, dtype=torch.float64)


def prepare_batch(samples, crop_hw, crops, device, out_dtype=torch.bfloat16, mean=CLIP_MEAN, std=CLIP_STD,
                  depth_max=80.0, bf=BASELINE_FOCAL_LENGTH, jitter=None):
    """samples: list of (img uint8 HxWx3, ids uint8 HxW, disp uint16 HxW) of one size;
    crops: int32 (B, 3) (y0, x0, flip) — a window of the image (`random_crops`) — or (B, 7)
    (Hs, Ws, pad_top, pad_left, y0, x0, flip) — the rescaled / padded pipeline
    (`random_scale_crops`).  Returns (img (B,3,h,w) out_dtype, seg int64 (B,h,w), depth f32
    (B,1,h,w), mask bool (B,1,h,w)) on `device`, ready for train.train_step.  jitter: (B, 8) from
    `color_jitter_params` (needs the (B, 7) parameters) applies ColorJitter before Normalize."""
    if not samples:
        raise ValueError("empty batch")
    H, W = samples[0][1].shape
    h, w = crop_hw
    B = len(samples)
    crops = torch.as_tensor(crops, dtype=torch.int32)
    if crops.dim() == 2 and crops.shape == (B, 7):
        Hs, Ws, pt, pl, y0, x0 = (crops[:, i] for i in range(6))
        bad = (Hs < 1) | (Ws < 1) | (pt < 0) | (pl < 0) | (y0 < 0) | (x0 < 0) | \
              (y0 + h > torch.maximum(Hs + pt, torch.full_like(Hs, h))) | \
              (x0 + w > torch.maximum(Ws + pl, torch.full_like(Ws, w)))
        if bad.any():
            raise ValueError(f"bad scale / pad / crop parameters {crops.tolist()} for a {h}x{w} crop")
    else:
        crops = crops.reshape(B, 3)
        if ((crops[:, 0] < 0) | (crops[:, 0] + h > H) | (crops[:, 1] < 0) | (crops[:, 1] + w > W)).any():
            raise ValueError(f"crop windows must lie inside the {H}x{W} images (got {crops.tolist()})")
    for s in samples:
        if s[0].shape != (H, W, 3) or s[1].shape != (H, W) or s[2].shape != (H, W):
            raise ValueError("all samples of a batch must share one image size")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("prepare_batch runs on the GPU (no CPU fallback)")
    pin = torch.cuda.is_available()

    def up(arrs):
        t = torch.from_numpy(np.ascontiguousarray(np.stack(arrs)))
        return (t.pin_memory() if pin else t).to(dev, non_blocking=True)

    img = up([s[0] for s in samples])
    ids = up([s[1] for s in samples])
    disp = up([s[2].view(np.int16) for s in samples])  # the uint16 bits through an int16 tensor
    cr = crops.to(dev)
    from .ops import D
    jt = None
    if jitter is not None:
        jt = torch.as_tensor(jitter, dtype=torch.float64).reshape(B, 8).to(dev)
    out_img, seg, depth, mask = D().cityscapes_prepare(img, ids, disp, cr, h, w, [float(v) for v in mean],
                                                       [float(v) for v in std], float(bf), float(depth_max), out_dtype,
                                                       jt)
    return out_img, seg, depth, mask.view(torch.bool)
