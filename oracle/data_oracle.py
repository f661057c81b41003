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
