"""Cityscapes data path, CPU side: the oracle's label remap and disparity -> depth against the
reference's own functions (tests/golden/data_prep.safetensors, gen_data_golden.py), and the
dataset's file scan / PNG decode on a synthetic directory tree."""
import os

import numpy as np
import pytest
import torch

from helpers import golden
from oracle import data_oracle as D


def test_label_remap_matches_reference():
    g = golden("data_prep")
    assert np.array_equal(D.map_labels(g["ids"].numpy()), g["train_ids"].numpy())


def test_disparity_to_depth_matches_reference():
    g = golden("data_prep")
    disp = g["disp"].numpy().view(np.uint16)
    depth, valid = D.disparity_to_depth(disp)
    assert np.array_equal(depth.view(np.int32), g["depth"].numpy().view(np.int32))  # bit-exact
    assert np.array_equal(valid, g["valid"].numpy())
    # the fixture holds the edge cases: d = 1 is 'valid' with depth 0 (no-transform mask),
    # which the post-transform mask depth > 0 drops
    assert ((valid == 1) & (depth == 0)).any()


def _png_tree(root, cities=("aachen", "bochum"), per_city=2, H=24, W=40, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    names = []
    for c in cities:
        for sub in ("leftImg8bit", "gtFine", "disparity"):
            os.makedirs(os.path.join(root, sub, "train", c), exist_ok=True)
        for i in range(per_city):
            base = f"{c}_{i:06d}_000019"
            img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
            ids = rng.integers(0, 40, (H, W), dtype=np.uint8)
            disp = rng.integers(0, 30000, (H, W)).astype(np.uint16)
            Image.fromarray(img).save(os.path.join(root, "leftImg8bit", "train", c, base + "_leftImg8bit.png"))
            Image.fromarray(ids).save(os.path.join(root, "gtFine", "train", c, base + "_gtFine_labelIds.png"))
            Image.fromarray(disp).save(os.path.join(root, "disparity", "train", c, base + "_disparity.png"))
            names.append((base, img, ids, disp))
    return names


def test_dataset_scan_and_decode(tmp_path):
    from denseclip_vit_multimodal_amd.data import CityscapesDepthSegDataset
    names = _png_tree(str(tmp_path))
    # a sample without its disparity file is skipped, like the reference's scan
    os.remove(os.path.join(tmp_path, "disparity", "train", "bochum", names[-1][0] + "_disparity.png"))
    ds = CityscapesDepthSegDataset(str(tmp_path), "train")
    assert len(ds) == len(names) - 1
    for i, (base, img, ids, disp) in enumerate(names[:-1]):
        assert os.path.basename(ds.img_files[i]).startswith(base)
        a, b, c = ds[i]
        assert a.dtype == np.uint8 and np.array_equal(a, img)
        assert np.array_equal(b, ids)
        assert c.dtype == np.uint16 and np.array_equal(c, disp)
    with pytest.raises(RuntimeError, match="dir not found"):
        CityscapesDepthSegDataset(str(tmp_path), "val")


def test_random_crops_and_cpu_refusal():
    from denseclip_vit_multimodal_amd.data import random_crops, prepare_batch
    g = torch.Generator().manual_seed(3)
    c = random_crops(16, 1024, 2048, 512, 1024, generator=g)
    assert c.dtype == torch.int32 and c.shape == (16, 3)
    assert (c[:, 0] >= 0).all() and (c[:, 0] <= 512).all() and (c[:, 1] <= 1024).all()
    assert set(c[:, 2].tolist()) <= {0, 1}
    with pytest.raises(ValueError):
        random_crops(1, 100, 100, 200, 50)
    s = (np.zeros((8, 8, 3), np.uint8), np.zeros((8, 8), np.uint8), np.zeros((8, 8), np.uint16))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        prepare_batch([s], (4, 4), [[0, 0, 0]], "cpu")
    with pytest.raises(ValueError, match="inside"):
        prepare_batch([s], (4, 4), [[6, 0, 0]], "cpu")


@pytest.mark.parametrize("H,W,Hs,Ws", [(48, 96, 73, 150), (48, 96, 24, 48), (64, 128, 50, 97), (32, 64, 64, 128)])
def test_cubic_restatement_within_one_lsb_of_torch_bicubic(H, W, Hs, Ws):
    """The oracle's cv2 INTER_CUBIC restatement (fixed point) against torch's float bicubic with the
    same kernel (A = -0.75), centres and clamped borders: the fixed-point rounding moves at most
    1 of 255 (cv2 itself is not installed: this is the available pin)."""
    import torch.nn.functional as F
    from oracle import data_oracle as D
    img = np.random.default_rng(0).integers(0, 256, (H, W, 3), dtype=np.uint8)
    ours = D.resize_cubic_u8(img, Hs, Ws).astype(np.int64)
    t = torch.from_numpy(img).permute(2, 0, 1)[None].double()
    ref = F.interpolate(t, size=(Hs, Ws), mode="bicubic", align_corners=False)[0].permute(1, 2, 0)
    ref = ref.clamp(0, 255).round().numpy().astype(np.int64)
    assert np.abs(ours - ref).max() <= 1
    # 2x upscale: exact; identity size: the input
    if (Hs, Ws) == (2 * H, 2 * W):
        assert np.array_equal(ours, ref)
    assert np.array_equal(D.resize_cubic_u8(img, H, W), img)


def test_nearest_restatement_and_scale_params():
    from oracle import data_oracle as D
    from denseclip_vit_multimodal_amd.data import random_scale_crops
    a = np.arange(6 * 8).reshape(6, 8)
    assert np.array_equal(D.resize_nearest(a, 12, 16), np.repeat(np.repeat(a, 2, 0), 2, 1))
    assert np.array_equal(D.resize_nearest(a, 3, 4), a[::2, ::2])
    import random
    p = random_scale_crops(64, 1024, 2048, 512, 1024, rng=random.Random(0))
    assert p.shape == (64, 7) and p.dtype == torch.int32
    Hs, Ws, pt, pl, y0, x0, fl = (p[:, i] for i in range(7))
    assert ((Hs >= 512) & (Hs <= 2048) & (Ws >= 1024) & (Ws <= 4096)).all()
    assert (pt == 0).all() and (pl == 0).all()  # scale >= 0.5 never needs padding at this crop
    assert ((y0 >= 0) & (y0 + 512 <= Hs) & (x0 >= 0) & (x0 + 1024 <= Ws)).all()
    assert set(fl.tolist()) == {0, 1}
    # a crop larger than the scaled image: centred padding, as PadIfNeeded
    q = random_scale_crops(8, 100, 200, 150, 300, scale_range=(0.5, 0.6), rng=random.Random(1))
    for Hs, Ws, pt, pl, y0, x0, _ in q.tolist():
        assert pt == (150 - Hs) // 2 and pl == (300 - Ws) // 2 and y0 == 0 and x0 == 0
    assert D.scale_pad_params(100, 200, 150, 300, 0.5, 0.0, 0.999, 1) == (50, 100, 50, 100, 0, 0, 1)
