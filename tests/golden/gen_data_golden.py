"""Golden vectors for the Cityscapes sample preparation, produced by the REFERENCE's own
functions (seg/datasets/cityscapes_depth_seg.py: map_labels_fast, disparity_to_depth) on
synthetic label-id and disparity planes.  Run ONLY in the development container:

    python tests/golden/gen_data_golden.py      # writes tests/golden/data_prep.safetensors

The inputs cover every label id 0..255 and the disparity edge cases (0, 1, the 1e-3 scaled
threshold, the depth_max = 80 m boundary, 65535) besides random values.
"""
import os

import numpy as np
import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SEG = "/root/reference/segmentation"


def main():
    # by file path: `datasets` would resolve to the installed HuggingFace package
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "ref_cityscapes_depth_seg", os.path.join(REF_SEG, "datasets", "cityscapes_depth_seg.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    Ref = mod.CityscapesDepthSegDataset
    rng = np.random.default_rng(7)
    H, W = 48, 96
    ids = rng.integers(0, 256, (H, W), dtype=np.uint8)
    ids.flat[:256] = np.arange(256, dtype=np.uint8)
    disp = rng.integers(0, 65536, (H, W), dtype=np.uint16)
    small = rng.integers(0, 3000, (H, W), dtype=np.uint16)  # the depth <= 80 m boundary (d ~ 1601)
    disp[H // 2:] = small[H // 2:]
    edge = np.array([0, 1, 2, 3, 257, 1600, 1601, 1602, 1603, 65535], dtype=np.uint16)
    disp.flat[:len(edge)] = edge
    obj = Ref.__new__(Ref)  # disparity_to_depth only reads these two attributes
    obj.bf, obj.depth_max = 500.0, 80.0
    train_ids = Ref.map_labels_fast(ids)
    depth, valid = obj.disparity_to_depth(disp)
    out = {"ids": torch.from_numpy(ids), "disp": torch.from_numpy(disp.view(np.int16)),
           "train_ids": torch.from_numpy(train_ids), "depth": torch.from_numpy(depth),
           "valid": torch.from_numpy(valid)}
    save_file(out, os.path.join(HERE, "data_prep.safetensors"))
    print("data_prep: valid", int(valid.sum()), "depth>0", int((depth > 0).sum()))


if __name__ == "__main__":
    main()
