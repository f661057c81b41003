"""dclip_cityscapes_prepare on the GPU against the CPU oracle (bit-exact: integer work and
correctly rounded f32 steps in the reference's order) and against the reference's own
label / depth golden vectors."""
import numpy as np
import pytest
import torch

from helpers import golden
from oracle import data_oracle as D

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need(hip):
    pass


def _samples(B, H, W, seed=5):
    rng = np.random.default_rng(seed)
    g = golden("data_prep")
    gh, gw = g["ids"].shape
    out = []
    for b in range(B):
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        ids = rng.integers(0, 256, (H, W), dtype=np.uint8)
        disp = rng.integers(0, 65536, (H, W)).astype(np.uint16)
        ids[:gh, :gw] = g["ids"].numpy()
        disp[:gh, :gw] = g["disp"].numpy().view(np.uint16)
        out.append((img, ids, disp))
    return out


def test_prepare_full_window_matches_reference_vectors():
    from denseclip_vit_multimodal_amd.data import prepare_batch
    g = golden("data_prep")
    H, W = g["ids"].shape
    s = [(np.zeros((H, W, 3), np.uint8), g["ids"].numpy(), g["disp"].numpy().view(np.uint16))]
    _, seg, depth, mask = prepare_batch(s, (H, W), [[0, 0, 0]], "cuda", out_dtype=torch.float32)
    assert torch.equal(seg[0].cpu(), g["train_ids"].to(torch.int64))
    assert torch.equal(depth[0, 0].cpu().view(torch.int32), g["depth"].view(torch.int32))
    assert torch.equal(mask[0, 0].cpu(), g["depth"] > 0)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_prepare_crops_flips_match_oracle(out_dtype):
    from denseclip_vit_multimodal_amd.data import prepare_batch, random_crops, CLIP_MEAN, CLIP_STD
    B, H, W, h, w = 4, 64, 160, 40, 96
    samples = _samples(B, H, W)
    crops = random_crops(B, H, W, h, w, generator=torch.Generator().manual_seed(1))
    crops[0] = torch.tensor([0, 0, 1], dtype=torch.int32)            # flipped, at the origin
    crops[1] = torch.tensor([H - h, W - w, 0], dtype=torch.int32)    # at the far corner
    img, seg, depth, mask = prepare_batch(samples, (h, w), crops, "cuda", out_dtype=out_dtype)
    ri, rs, rd, rm = D.prepare(samples, (h, w), crops.tolist(), CLIP_MEAN, CLIP_STD)
    ref_img = torch.from_numpy(np.ascontiguousarray(ri)).to(out_dtype)
    assert torch.equal(img.cpu(), ref_img)
    assert torch.equal(seg.cpu(), torch.from_numpy(rs))
    assert torch.equal(depth.cpu().view(torch.int32), torch.from_numpy(np.ascontiguousarray(rd)).view(torch.int32))
    assert torch.equal(mask.cpu(), torch.from_numpy(rm))


def test_prepared_batch_trains():
    """The prepared batch is what train.train_step takes (one step of the tiny model)."""
    from denseclip_vit_multimodal_amd import DenseCLIP
    from denseclip_vit_multimodal_amd.data import prepare_batch
    from denseclip_vit_multimodal_amd.train import train_step, make_optimizer, freeze_for_mode
    from helpers import TINY_CFG, CITYSCAPES_CLASSES
    m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **TINY_CFG).cuda().train()
    params = freeze_for_mode(m, "F")
    opt = make_optimizer(params)
    batch = prepare_batch(_samples(2, 64, 160), (64, 128), [[0, 0, 0], [0, 32, 1]], "cuda",
                          out_dtype=torch.bfloat16)
    loss = train_step(m, opt, batch)
    assert torch.isfinite(loss)
