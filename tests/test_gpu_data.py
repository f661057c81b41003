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


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_augment_scale_pad_crop_matches_oracle(out_dtype):
    """dclip_cityscapes_augment (RandomScale + PadIfNeeded + RandomCrop + HorizontalFlip) bit-exact
    against the oracle's restatement: up- and down-scales, a padded case, a flipped case and the
    identity (which must equal dclip_cityscapes_prepare)."""
    import random
    from denseclip_vit_multimodal_amd.data import prepare_batch, random_scale_crops, CLIP_MEAN, CLIP_STD
    B, H, W, h, w = 6, 64, 160, 48, 96
    samples = _samples(B, H, W)
    p = random_scale_crops(B, H, W, h, w, rng=random.Random(4))
    p[0] = torch.tensor([H, W, 0, 0, 3, 7, 1], dtype=torch.int32)                       # identity scale
    p[1] = torch.tensor([40, 60, 4, 18, 0, 0, 0], dtype=torch.int32)                     # padded both ways
    p[2] = torch.tensor([int(H * 1.7), int(W * 1.7), 0, 0, 50, 100, 1], dtype=torch.int32)  # up, flipped
    p[3] = torch.tensor([int(H * 0.8), int(W * 0.8), 0, 0, 2, 20, 0], dtype=torch.int32)    # down
    img, seg, depth, mask = prepare_batch(samples, (h, w), p, "cuda", out_dtype=out_dtype)
    ri, rs, rd, rm = D.prepare_augmented(samples, (h, w), p.tolist(), CLIP_MEAN, CLIP_STD)
    assert torch.equal(img.cpu(), torch.from_numpy(np.ascontiguousarray(ri)).to(out_dtype))
    assert torch.equal(seg.cpu(), torch.from_numpy(rs))
    assert torch.equal(depth.cpu().view(torch.int32), torch.from_numpy(np.ascontiguousarray(rd)).view(torch.int32))
    assert torch.equal(mask.cpu(), torch.from_numpy(rm))
    assert (seg[1] == 255).any() and (depth[1] == 255.0).any()  # the padded border
    # identity parameters = the crop-only kernel
    i2, s2, d2, m2 = prepare_batch(samples[:1], (h, w), [[3, 7, 1]], "cuda", out_dtype=out_dtype)
    assert torch.equal(i2, img[:1]) and torch.equal(s2, seg[:1]) and torch.equal(d2, depth[:1])


def test_augment_full_resolution_batch():
    """The Cityscapes train shape: 8 images 1024x2048 rescaled by U(0.5, 2) and cropped to 512x1024."""
    import random
    from denseclip_vit_multimodal_amd.data import prepare_batch, random_scale_crops
    B, H, W = 8, 1024, 2048
    rng = np.random.default_rng(1)
    s = [(rng.integers(0, 256, (H, W, 3), dtype=np.uint8), rng.integers(0, 34, (H, W), dtype=np.uint8),
          rng.integers(0, 3000, (H, W)).astype(np.uint16)) for _ in range(B)]
    p = random_scale_crops(B, H, W, 512, 1024, rng=random.Random(0))
    img, seg, depth, mask = prepare_batch(s, (512, 1024), p, "cuda")
    assert img.shape == (B, 3, 512, 1024) and torch.isfinite(img.float()).all()
    ri, rs, rd, rm = D.prepare_augmented(s[:1], (512, 1024), p[:1].tolist(), (0.48145466, 0.4578275, 0.40821073),
                                         (0.26862954, 0.26130258, 0.27577711))
    assert torch.equal(seg[:1].cpu(), torch.from_numpy(rs))
    assert torch.equal(img[:1].float().cpu(), torch.from_numpy(np.ascontiguousarray(ri)).to(torch.bfloat16).float())


def test_color_jitter_matches_oracle():
    """ColorJitter (brightness / contrast / saturation / hue in a random order per image, the
    identity for a not-applied image) on the GPU bit-exact against the oracle's restatement of
    albumentations' uint8 functions and OpenCV's 8-bit colour conversions (cv2 itself absent:
    parity against it unpinned), inside the full augmented batch preparation."""
    import random
    from denseclip_vit_multimodal_amd.data import (prepare_batch, random_scale_crops, color_jitter_params,
                                                   CLIP_MEAN, CLIP_STD)
    B, H, W, h, w = 6, 64, 160, 48, 96
    samples = _samples(B, H, W, seed=9)
    # saturated colours, greys and black / white pixels beside the random ones
    for s_ in samples:
        s_[0][:4, :4] = [[255, 0, 0], [0, 255, 0], [0, 0, 255], [128, 128, 128]]
        s_[0][4:8, :4] = [[0, 0, 0], [255, 255, 255], [255, 255, 0], [1, 2, 3]]
    p = random_scale_crops(B, H, W, h, w, rng=random.Random(2))
    p[0] = torch.tensor([H, W, 0, 0, 0, 0, 0], dtype=torch.int32)
    jit = color_jitter_params(B, rng=random.Random(3), p=1.0)
    jit[1] = torch.tensor([1.0, 1.0, 1.0, 0.0, 0, 1, 2, 3], dtype=torch.float64)      # not applied
    jit[2] = torch.tensor([1.37, 0.61, 1.39, -0.099, 3, 2, 1, 0], dtype=torch.float64)
    for out_dtype in (torch.float32, torch.bfloat16):
        img, seg, depth, mask = prepare_batch(samples, (h, w), p, "cuda", out_dtype=out_dtype, jitter=jit)
        ri, rs, rd, rm = D.prepare_augmented_jitter(samples, (h, w), p.tolist(), jit.tolist(), CLIP_MEAN, CLIP_STD)
        assert torch.equal(img.cpu(), torch.from_numpy(np.ascontiguousarray(ri)).to(out_dtype))
        assert torch.equal(seg.cpu(), torch.from_numpy(rs))
    # the not-applied image equals the jitter-free pipeline
    i0, *_ = prepare_batch(samples, (h, w), p, "cuda", out_dtype=torch.float32)
    assert torch.equal(img.float()[1], i0.to(img.dtype).float()[1])
    assert not torch.equal(img[2], i0.to(img.dtype)[2])
