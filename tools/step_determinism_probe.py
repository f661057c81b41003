"""Three-step determinism of the train step across launch contexts (ViT-B/16 mode F, B = 2 @
512x1024, exact fp16 scales): six fresh models from one seed — twice on torch's default stream, the
text path eager on its side stream ("side", as CapturedTrainStep's capture runs it), the step on a
side stream, and both (twice) — each compared parameter by parameter with the first.

  python tools/step_determinism_probe.py fp16|bf16
"""
import os, sys
sys.path.insert(0, os.getcwd())
import torch, bench
from denseclip_vit_multimodal_amd import ops, train
from denseclip_vit_multimodal_amd.train import synth_batch, train_step, make_optimizer
ops.FP16_DELAYED_SCALE = False
dev = torch.device("cuda", 0)
cdt = torch.float16 if sys.argv[1] == "fp16" else torch.bfloat16
def make():
    torch.manual_seed(0)
    m = bench.make_model(dev, "F").train()
    m.backbone.compute_dtype = cdt
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout): mod.p = 0.0
    return m, make_optimizer([p for p in m.parameters() if p.requires_grad], capturable=True)
b1 = synth_batch(2, 512, 1024, dev, 0, image_dtype=torch.float32 if cdt == torch.float16 else torch.bfloat16)
def run(text_side, on_side):
    m, o = make()
    if text_side:
        m.graph_text = "side"
    st = torch.cuda.Stream() if on_side else torch.cuda.current_stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        l = [float(train_step(m, o, b1)) for _ in range(3)]
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    return m, l
def ndiff(ma, mb):
    pa = dict(ma.named_parameters())
    return sum(not torch.equal(p, pa[n]) for n, p in mb.named_parameters())
arms = {}
for name, ts, os_ in (("A default", False, False), ("A2 default", False, False), ("D textside", True, False),
                      ("E sidestream", False, True), ("C both", True, True), ("C2 both", True, True)):
    arms[name] = run(ts, os_)
    print(name, arms[name][1], "params differing from A:", ndiff(arms["A default"][0], arms[name][0]), flush=True)
print("C vs C2 params differing:", ndiff(arms["C both"][0], arms["C2 both"][0]))
print("E vs C params differing:", ndiff(arms["E sidestream"][0], arms["C both"][0]))
