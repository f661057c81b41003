"""DenseCLIP constructor kwargs used by the fixtures and the tests.

CITYSCAPES_CFG is what the reference trainer passes to `DenseCLIP(**...)` for
seg/configs/denseclip_cityscapes.yaml (train_denseclip.py:958-1005): the model
section minus `type`/`clip_pretrained`, with `context_length`, `text_dim`,
`token_embed_dim` passed explicitly and `clip_pretrained_path=None` (the YAML's
absolute weight path does not exist offline).  TINY_CFG is the same structure at
toy widths so full weights/gradients fit in a fixture.
"""

CITYSCAPES_CLASSES = [
    'road', 'sidewalk', 'building', 'wall', 'fence', 'pole',
    'traffic light', 'traffic sign', 'vegetation', 'terrain', 'sky',
    'person', 'rider', 'car', 'truck', 'bus', 'train',
    'motorcycle', 'bicycle',
]

CITYSCAPES_CFG = dict(
    backbone=dict(type='CLIPVisionTransformer', patch_size=16, width=768, layers=12, heads=12,
                  input_resolution=224, output_dim=768,
                  out_indices=[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]),
    text_encoder=dict(type='CLIPTextContextEncoder', context_length=22, vocab_size=49408,
                      transformer_width=512, transformer_heads=8, transformer_layers=12,
                      embed_dim=512),
    decode_head=dict(type='FPNHead', in_channels=256, channels=256, num_classes=19,
                     align_corners=False, dropout_ratio=0.1),
    depth_head=dict(type='FCNHeadDepth', in_channels=256, channels=128, align_corners=False),
    neck=dict(type='ViTFeatureFusionNeck', inter_channels=128, out_channels=256),
    context_decoder=None,
    auxiliary_head=None,
    identity_head=None,
    context_length=6,
    text_dim=512,
    token_embed_dim=512,
    context_feature='attention',
    score_concat_index=-1,
    text_head=False,
    tau=0.05,
    clip_pretrained_path=None,
)

TINY_CFG = dict(
    backbone=dict(type='CLIPVisionTransformer', patch_size=16, width=128, layers=3, heads=2,
                  input_resolution=32, output_dim=128, out_indices=[0, 1, 2]),
    text_encoder=dict(type='CLIPTextContextEncoder', context_length=8, vocab_size=49408,
                      transformer_width=64, transformer_heads=2, transformer_layers=2,
                      embed_dim=32),
    decode_head=dict(type='FPNHead', in_channels=32, channels=16, num_classes=19,
                     align_corners=False),
    depth_head=dict(type='FCNHeadDepth', in_channels=32, channels=8, align_corners=False),
    neck=dict(type='ViTFeatureFusionNeck', inter_channels=16, out_channels=32),
    context_decoder=None,
    context_length=6,
    text_dim=32,
    token_embed_dim=64,
    context_feature='attention',
    score_concat_index=-1,
    text_head=False,
    tau=0.05,
    clip_pretrained_path=None,
)

# TINY_CFG with the ContextDecoder branch (denseclip.py:204-211, 627-665):
# the class embeddings cross-attend over [global; pixel] visual context and the decoder's
# output is added with the learnable gamma before the score map
TINY_CTX_CFG = dict(TINY_CFG, context_decoder=dict(type='ContextDecoder', transformer_width=32,
                                                   transformer_heads=2, transformer_layers=2, dropout=0.1))
# the fixture's gamma (the spec weights' value is ~1e-4 scale, which would leave the branch
# below the comparison tolerance)
CTX_GAMMA = 0.5

# BASELINE config 4: ViT-L/14 (width 1024, 24 layers, 16 heads of 64, patch 14).  The reference
# ships no ViT-L YAML; this is CITYSCAPES_CFG with the backbone swapped and four read-outs (the
# quarter-depth layers, the usual dense-prediction choice for a 24-layer ViT) — the neck's
# in_channels follow from width x len(out_indices) exactly as for ViT-B (denseclip.py:224-262).
VITL14_CFG = dict(CITYSCAPES_CFG,
                  backbone=dict(type='CLIPVisionTransformer', patch_size=14, width=1024, layers=24, heads=16,
                                input_resolution=224, output_dim=1024, out_indices=[5, 11, 17, 23]))

# TINY_CFG at widths every neck / head op of the HIP path takes (ops.neck_heads_hip_capable):
# backbone width 128 (3x3 conv Cin % 128 == 0), 2 levels x 64 -> fusion 128 -> 256, decode head
# 256 -> 64 -> 256 -> 19, depth head 256 -> 64 -> 64 -> 1.  score_concat_index 1 (>= 0): the
# reference concatenates the score map onto a clone it then discards (denseclip.py:684-694, 747),
# so training through this config is pinned too.
MID_CFG = dict(TINY_CFG,
               backbone=dict(type='CLIPVisionTransformer', patch_size=16, width=128, layers=2, heads=2,
                             input_resolution=32, output_dim=128, out_indices=[0, 1]),
               decode_head=dict(type='FPNHead', in_channels=256, channels=256, num_classes=19,
                                align_corners=False),
               depth_head=dict(type='FCNHeadDepth', in_channels=256, channels=64, align_corners=False),
               neck=dict(type='ViTFeatureFusionNeck', inter_channels=64, out_channels=256),
               score_concat_index=1)
