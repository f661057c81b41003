"""Drop-in alias: `from denseclip import DenseCLIP, ...` as the reference trainer does
(train_denseclip.py:58-66) resolves to the MI355X package."""
import sys as _sys

from denseclip_vit_multimodal_amd import *  # noqa: F401,F403
from denseclip_vit_multimodal_amd import __all__  # noqa: F401
from denseclip_vit_multimodal_amd import denseclip as _dc, data, heads, losses, models, train, utils  # noqa: F401

_sys.modules[__name__ + ".models"] = models
_sys.modules[__name__ + ".heads"] = heads
_sys.modules[__name__ + ".losses"] = losses
_sys.modules[__name__ + ".utils"] = utils
_sys.modules[__name__ + ".denseclip"] = _dc
_sys.modules[__name__ + ".data"] = data
_sys.modules[__name__ + ".train"] = train
