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
