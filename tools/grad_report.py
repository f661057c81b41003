"""Per-parameter gradient error of one tiny fine-tune step vs the reference's golden step
(tests/golden/tiny_train.safetensors): prints norm error and sampled-element error for
every parameter, worst first.  python tools/grad_report.py [f16|bf16]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from helpers import TINY_CFG, CITYSCAPES_CLASSES, spec_state_dict, golden, rel_err  # noqa: E402

cdt = torch.bfloat16 if (len(sys.argv) > 1 and sys.argv[1] == "bf16") else torch.float16
from denseclip_vit_multimodal_amd import DenseCLIP  # noqa: E402
from denseclip_vit_multimodal_amd.losses import SILogLoss  # noqa: E402
g = golden("tiny_train")
m = DenseCLIP(class_names=CITYSCAPES_CLASSES, **TINY_CFG)
m.load_state_dict(spec_state_dict("tiny"))
m.backbone.compute_dtype = cdt
m = m.cuda().train()
for mod in m.modules():
    if isinstance(mod, torch.nn.Dropout):
        mod.eval()
for p in m.parameters():
    p.requires_grad_(True)
x = g["input"].cuda()
seg_t = g["seg_t"].cuda()
out = m(x, gt_semantic_seg=seg_t, gt_depth=g["depth_t"].cuda(), return_loss=True)
loss = F.cross_entropy(out["main_output"], seg_t, ignore_index=255) + \
    0.1 * SILogLoss()(out["depth_output"], g["depth_t"].cuda(), g["depth_m"].bool().cuda())
print("loss", float(loss), "ref", float(g["loss"][0]))
loss.backward()
params = dict(m.named_parameters())
rows = []
for k in g:
    if not k.startswith("gnorm/"):
        continue
    name = k[len("gnorm/"):]
    gr = params[name].grad
    if gr is None:
        rows.append((9.9, 9.9, name))
        continue
    ref = float(g[k])
    en = abs(float(gr.double().norm()) - ref) / (ref + 1e-12)
    ev = rel_err(gr.flatten().cpu()[g["gidx/" + name]], g["gval/" + name])
    rows.append((ev, en, name))
rows.sort(reverse=True)
for ev, en, name in rows:
    print(f"{ev:9.2e} {en:9.2e}  {name}")
