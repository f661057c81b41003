"""MI355X-native DenseCLIP ViT hot path.

Public surface mirrors the reference `denseclip` package (seg/denseclip/__init__.py:1-3,
train_denseclip.py:58-66); the ViT forward/backward, the score map and the logits resize
run on the hand-written gfx950 kernels of libdclip.so (include/dclip.h).
"""
from .denseclip import DenseCLIP
from .heads import IdentityHead
from .models import (CLIPResNet, CLIPResNetWithAttention, CLIPTextContextEncoder, CLIPTextEncoder,
                     CLIPVisionTransformer, ContextDecoder, ViTFeatureFusionNeck)

__all__ = ["DenseCLIP", "CLIPResNet", "CLIPTextEncoder", "CLIPVisionTransformer", "CLIPResNetWithAttention",
           "CLIPTextContextEncoder", "ContextDecoder", "ViTFeatureFusionNeck", "IdentityHead"]
