"""Throughput benchmark: DenseCLIP ViT-B/16 fwd+bwd training step at 1024x2048 (BASELINE.json
metric, configs[1] per GPU: batch 8 per GPU, bf16), data-parallel over RCCL for N > 1.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode F|R]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N > 1` without a launcher: this process makes NO HIP call; it starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...` as a child
(one rank per GPU, the reference's mp.spawn world, train_denseclip.py:1649-1657), whose
rank 0 prints the JSON line on the inherited stdout, and exits with the child's status.
Under a launcher `--gpus` must equal WORLD_SIZE; `n_gpus` is the process group's size and
`rccl_ranks` an all-reduce of ones over it.

One step = forward of the whole DenseCLIP (ViT on the HIP kernels, text encoder, neck,
heads, bilinear resize to the label size), CE(ignore 255) + 0.1 SILog, backward,
gradient all-reduce (DDP over RCCL when N > 1) and AdamW.  Mode F (default, full
fine-tune) trains the ViT too, so its backward kernels run; mode R is the reference
trainer's regime (backbone + text encoder frozen, train_denseclip.py:1040-1044) and is
measured as well and reported beside the headline.

rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel of a train step (the
attention backward: dQ + dK/dV passes; `roofline_attn_fwd` for the forward), timed with HIP
events on its launch stream over the timed region; `fp16` repeats the mode-F step with fp32
images and the fp16 compute dtype (the reference trainer's input, the dtype that holds the
north-star 1e-3: the HIP neck / heads run in fp16 with device-side gradient scales);
`cpu_baseline` times the CPU oracle (the reference algorithm restated in torch fp32,
including the same SDPA op the reference calls) on a bounded sample on the host cores.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
PEAK_FP8_TFLOPS = 5000.0  # MI355X dense fp8 (block-scaled f8f6f4 MFMA at 2x the bf16 rate)
# the fp8 attention's mix: QK^T (half the FLOPs) at the bf16 peak, P V at the fp8 one:
# 1 / (0.5 / 2500 + 0.5 / 5000)
PEAK_FP8_MIXED_TFLOPS = 1.0 / (0.5 / PEAK_BF16_TFLOPS + 0.5 / PEAK_FP8_TFLOPS)
# configs[4]'s backward (dclip_attn_bwd_fp8): of its 5 useful N^2 matmuls S, dP, dQ run on the 16-bit MFMA
# and dV, dK on the block-scaled e4m3 one
PEAK_FP8_BWD_TFLOPS = 1.0 / (0.6 / PEAK_BF16_TFLOPS + 0.4 / PEAK_FP8_TFLOPS)
PEAK_HBM_GBS = 8000.0
FUSED_HEAD_LOSS = True  # resize + CE / SILog fused (same loss; no 1024x2048 logits in HBM)
# backbone kwargs per --arch: ViT-B/16 is seg/configs/denseclip_cityscapes.yaml's own backbone;
# ViT-L/14 (BASELINE configs[3]) is tests/golden/model_configs.py's VITL14_CFG backbone
ARCHS = {
    "vitb16": None,
    "vitl14": dict(type="CLIPVisionTransformer", patch_size=14, width=1024, layers=24, heads=16,
                   input_resolution=224, output_dim=1024, out_indices=[5, 11, 17, 23]),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (default: WORLD_SIZE under a launcher, else 1); N > 1 without a "
                         "launcher spawns torch.distributed.run with N ranks")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--mode", choices=["F", "R"], default="F")
    ap.add_argument("--no-mode-r", action="store_true", help="skip the extra mode-R measurement")
    ap.add_argument("--no-fp16", action="store_true", help="skip the extra fp16 (fp32-image) mode-F measurement")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--arch", choices=sorted(ARCHS), default="vitb16",
                    help="vitb16: the headline (BASELINE configs[1]); vitl14: BASELINE configs[3]'s backbone")
    ap.add_argument("--infer", action="store_true",
                    help="inference forward only (eval mode, seg + depth at full resolution, no grad)")
    ap.add_argument("--attn-fp8", action="store_true",
                    help="attention forward on the e4m3 MFMA kernel (BASELINE configs[4]); training runs the 16-bit "
                         "flash backward on its (o, lse)")
    ap.add_argument("--unfused-head-loss", action="store_true",
                    help="materialise the resized logits/depth and use F.cross_entropy + SILogLoss")
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default="bf16",
                    help="image / compute dtype of the ViT and neck operands (fp32 accumulation either way)")
    ap.add_argument("--ddp", action="store_true",
                    help="process group (RCCL) + DDP even at world size 1 (torchrun --nproc-per-node 1)")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="dtype of the DDP gradient all-reduce buckets (bf16: DDP's compression hook)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the BASELINE configs[3] (ViT-L/14) / configs[4] (fp8 attention) sub-measurements "
                         "and the configs[0] CPU forward")
    ap.add_argument("--no-op-timing", action="store_true",
                    help="no per-op HIP-event breakdown (`ops` objects) of the headline and fp16 steps")
    return ap.parse_args(argv)


def progress(msg):
    """A progress line on stderr (the JSON result stays the only stdout line)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def free_port():
    """An unused localhost TCP port for the rendezvous (no GPU involved)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(argv, n, port, script=None):
    """argv of the child that runs N ranks of this benchmark (one process per GPU, RCCL over
    xGMI): torch.distributed.run on one node at 127.0.0.1, the same bench arguments."""
    script = script or os.path.abspath(__file__)
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script] + list(argv)


def launch_env(base=None):
    env = dict(os.environ if base is None else base)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"  # dmabuf IPC only on this host driver (RCCL)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def spawn_ranks(argv, n, script=None):
    """Run N ranks as a CHILD process (never exec: this process stays the parent) and return
    its exit status; rank 0's JSON line reaches our stdout directly."""
    proc = subprocess.run(launch_cmd(argv, n, free_port(), script), env=launch_env())
    return proc.returncode


def resolve_world(args, env=None):
    """(world, spawn): world size this process runs at, and whether it must spawn the ranks
    itself.  Under a launcher (WORLD_SIZE set) --gpus must match it."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        return world, False
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {n})")
    return n, n > 1


def attn_flops_fwd(B, N, H, D=64):
    return 4.0 * B * H * N * N * D  # QK^T and PV


def model_fwd_flops(H, W, arch):
    """Algorithmic forward FLOPs per image (SURVEY 8(d)'s formulas): ViT attention L*4N^2C,
    linears L*24NC^2, patchify 2*P*C*3p^2, neck (3x3 convs C->128 per read-out + 1x1 fusion
    -> 256) and a 12 GFLOP allowance for projections / score map / heads (ViT-B at 1024x2048:
    4.068 TFLOP)."""
    b = ARCHS[arch] or dict(patch_size=16, width=768, layers=12, heads=12, out_indices=list(range(12)))
    p, C, L, nl = b["patch_size"], b["width"], b["layers"], len(b["out_indices"])
    P = (H // p) * (W // p)
    N = P + 1
    vit = L * (4.0 * N * N * C + 24.0 * N * C * C) + 2.0 * P * C * 3 * p * p
    neck = nl * 2.0 * P * 9 * C * 128 + 2.0 * P * 128 * nl * 256
    return vit + neck + 12e9 * P / 8192


def make_model(dev, mode, arch="vitb16"):
    from denseclip_vit_multimodal_amd.config import build_model, load_yaml
    from denseclip_vit_multimodal_amd.train import freeze_for_mode
    cfg = load_yaml("denseclip_cityscapes.yaml")
    if ARCHS[arch] is not None:
        cfg["model"]["backbone"] = dict(ARCHS[arch])
    model = build_model(cfg, clip_path_override="").to(dev)
    freeze_for_mode(model, mode)
    model.fused_head_loss = FUSED_HEAD_LOSS
    return model


def run_steps(model, opt, batch, steps, silog):
    from denseclip_vit_multimodal_amd.train import train_step
    loss = None
    for _ in range(steps):
        if opt is None:  # inference: eval forward, seg + depth resized to the image
            with torch.no_grad():
                out = model(batch[0], return_loss=False)
            loss = out["seg"][0, 0, 0, 0]
        else:
            loss = train_step(model, opt, batch, silog)
    return loss


def timed(model, opt, batch, steps, warmup, silog, world, dist_on=None, op_timing=False):
    """(seconds for `steps` steps, max over ranks; per-op HIP-event summary; last loss).
    op_timing also brackets every torch.ops.dclip launch with events (ops.TIMING_OPS)."""
    from denseclip_vit_multimodal_amd import ops
    dist_on = world > 1 if dist_on is None else dist_on
    run_steps(model, opt, batch, warmup, silog)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    ops.TIMING = {}
    ops.TIMING_OPS = bool(op_timing)
    t0 = time.perf_counter()
    loss = run_steps(model, opt, batch, steps, silog)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    summary = ops.timing_summary()
    ops.TIMING = None
    ops.TIMING_OPS = False
    if dist_on:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    return dt, summary, float(loss)


def op_breakdown(summary, steps, ms_per_step):
    """Per-op device time per step from the `op:` events (every dclip custom-op launch on the
    step's stream) and what is left of the step: torch-native kernels (AdamW, copies, fills),
    the text graph's side-stream share and launch gaps."""
    ops_ms = {k[3:]: round(v[1] / steps, 3) for k, v in summary.items() if k.startswith("op:")}
    if not ops_ms:
        return None
    ops_ms = dict(sorted(ops_ms.items(), key=lambda kv: -kv[1]))
    tot = sum(ops_ms.values())
    return {"ms_per_step": ops_ms, "dclip_ops_ms": round(tot, 2), "step_ms_with_events": round(ms_per_step, 2),
            "not_dclip_ms": round(ms_per_step - tot, 2),
            "what": "a separate 2-step pass after the timed region with HIP events around each torch.ops.dclip "
                    "launch (the events slow the step by ~4 %, so they are kept out of the reported time); "
                    "not_dclip = that pass's step time - the ops' sum (torch-native kernels: fused AdamW, "
                    "copies, fills; launch gaps)"}


def roofline(summary, key, flops, peak):
    n, _, mean = summary.get(key, (0, 0.0, float("nan")))
    if not n:
        return None
    a = flops / (mean * 1e-3) / 1e12
    return {"achieved": round(a, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(a / peak, 4),
            "ms_per_launch": round(mean, 4), "launches": n}


def cpu_baseline(H, W, threads):
    """Oracle (reference algorithm restated in torch fp32 on the host) fwd+bwd, full fine-tune
    (mode F: ViT + neck + heads trainable), ONE image at the benchmark resolution."""
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from helpers import CITYSCAPES_CFG, spec_state_dict, class_tokens, images
    from oracle import denseclip_oracle as O
    torch.set_num_threads(threads)
    O.USE_SDPA = True
    sd = spec_state_dict("cityscapes")
    p = {k: (v.requires_grad_(True) if v.is_floating_point() and not k.startswith("text_encoder.") else v)
         for k, v in sd.items()}
    x = images(1, H, W)
    g = torch.Generator().manual_seed(1235)
    seg = torch.randint(0, 19, (1, H, W), generator=g)
    t0 = time.perf_counter()
    out = O.denseclip_forward(x, p, class_tokens(), CITYSCAPES_CFG, training=True)
    loss = F.cross_entropy(out["seg"], seg, ignore_index=255)
    loss.backward()
    dt = time.perf_counter() - t0
    O.USE_SDPA = False
    return {"value": round(1.0 / dt, 5), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"1 image {H}x{W}, full DenseCLIP fwd+bwd (mode F, text path frozen), torch fp32 CPU "
                      f"oracle with SDPA attention, {dt:.1f} s"}


def cpu_baseline_cfg0(threads):
    """BASELINE configs[0] / SURVEY 8(d): the reference algorithm's DenseCLIP ViT-B/16 eval
    FORWARD on 2x3x512x1024 fp32 (the oracle restatement, SDPA attention as the reference
    calls it), all `threads` host cores."""
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from helpers import CITYSCAPES_CFG, spec_state_dict, class_tokens, images
    from oracle import denseclip_oracle as O
    torch.set_num_threads(threads)
    O.USE_SDPA = True
    sd = spec_state_dict("cityscapes")
    x = images(2, 512, 1024)
    tok = class_tokens()
    with torch.no_grad():
        O.denseclip_forward(x[:1, :, :64, :128], sd, tok, CITYSCAPES_CFG)  # warm the allocator / MKL
        t0 = time.perf_counter()
        O.denseclip_forward(x, sd, tok, CITYSCAPES_CFG)
        dt = time.perf_counter() - t0
    O.USE_SDPA = False
    return {"value": round(2.0 / dt, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"BASELINE configs[0]: DenseCLIP ViT-B/16 eval forward, 2x3x512x1024 fp32, torch CPU oracle "
                      f"with SDPA attention, one timed pass {dt:.2f} s"}


def main():
    global FUSED_HEAD_LOSS
    args = parse()
    world, spawn = resolve_world(args)
    if spawn:  # N ranks as a child process; this parent makes no HIP call at all
        sys.exit(spawn_ranks(sys.argv[1:], world))
    FUSED_HEAD_LOSS = not args.unfused_head_loss
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1 or args.ddp
    rccl_ranks = None
    if dist_on:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL on ROCm (reference utils.py:106)
        world = dist.get_world_size()
        ones = torch.ones(1, device="cuda")
        dist.all_reduce(ones)  # every rank reachable over RCCL: must equal the world size
        rccl_ranks = int(ones.item())
        if rccl_ranks != world:
            raise RuntimeError(f"RCCL all-reduce over {world} ranks gave {rccl_ranks}")
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    from denseclip_vit_multimodal_amd.losses import SILogLoss
    silog = SILogLoss()

    from denseclip_vit_multimodal_amd.train import synth_batch, wrap_ddp, make_optimizer
    from denseclip_vit_multimodal_amd import ops
    B, H, W = args.batch, args.height, args.width
    img_dtype = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    batch = synth_batch(B, H, W, dev, rank, image_dtype=img_dtype)

    def setup(mode, compute_dtype=None, arch=None, attn_fp8=None):
        model = make_model(dev, mode, arch or args.arch)
        model.backbone.attn_fp8 = args.attn_fp8 if attn_fp8 is None else attn_fp8
        if compute_dtype is not None:
            model.backbone.compute_dtype = compute_dtype
        if args.infer:  # replicas: no gradients, no collective
            model.eval()
            return model, None
        model.train()
        if dist_on:
            model = wrap_ddp(model, dev, torch.bfloat16 if args.grad_dtype == "bf16" else None)
        opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
        return model, opt

    def geometry(arch):
        bb = ARCHS[arch] or dict(patch_size=16, heads=12)
        return (H // bb["patch_size"]) * (W // bb["patch_size"]) + 1, bb["heads"]

    op_timing = not args.no_op_timing

    def op_pass(model, opt, batch_, steps=2):
        """The per-op breakdown from its OWN short pass after the timed region: HIP events around
        every launch cost ~4 % of a step, so they never bracket the reported time."""
        if not op_timing:
            return None
        dto, so, _ = timed(model, opt, batch_, steps, 0, silog, world, dist_on, True)
        return op_breakdown(so, steps, dto / steps * 1e3)

    model, opt = setup(args.mode)
    dt, summ, loss = timed(model, opt, batch, args.steps, args.warmup, silog, world, dist_on)
    ops_head = op_pass(model, opt, batch)
    value = world * B * args.steps / dt
    progress(f"headline {dt / args.steps * 1e3:.2f} ms per step")
    N, heads = geometry(args.arch)

    # attention forward roofline (one dclip_attn_fwd launch per layer)
    akey = "attn_fwd_fp8" if args.attn_fp8 else "attn_fwd"
    peak_attn = PEAK_FP8_MIXED_TFLOPS if args.attn_fp8 else PEAK_BF16_TFLOPS
    n_att, tot_att, mean_att = summ.get(akey, (0, 0.0, float("nan")))
    fl = attn_flops_fwd(B, N, heads)
    achieved = fl / (mean_att * 1e-3) / 1e12 if n_att else None
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "attn_fwd_pmc.json")
    probe_shape = args.arch == "vitb16" and B == 8 and (H, W) == (1024, 2048)  # the PMC runs' shape
    if os.path.exists(pmc) and probe_shape and not args.attn_fp8:
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    traffic_b = None
    pmc_b = os.path.join(ROOT, "profiles", "attn_bwd_pmc.json")
    if os.path.exists(pmc_b) and probe_shape and not args.infer:
        with open(pmc_b) as f:
            traffic_b = json.load(f).get("hbm_bytes_per_launch")
    kernels = {k: {"launches": v[0], "ms_total": round(v[1], 3), "ms_mean": round(v[2], 4)}
               for k, v in summ.items() if not k.startswith("op:")}
    # the attention backward (dQ pass + dK/dV pass + the CLS row's merge per launch): useful work = the
    # 5 N^2-matmuls of flash backward (2.5x the forward's), same HIP-event timing
    n_ab, _, mean_ab = summ.get("attn_bwd", (0, 0.0, float("nan")))
    fl_b = 2.5 * fl
    ach_b = fl_b / (mean_ab * 1e-3) / 1e12 if n_ab else None
    # whole-model MFMA utilisation: 3 x 4.068 TFLOP per image fwd+bwd in mode F
    if args.infer:
        model_fl = model_fwd_flops(H, W, args.arch)
    elif args.arch == "vitb16":
        model_fl = (3 * 4.068e12 if args.mode == "F" else 4.44e12) * H * W / (1024 * 2048)
    else:
        model_fl = 3 * model_fwd_flops(H, W, args.arch) if args.mode == "F" else None

    def release():
        nonlocal model, opt
        model = opt = None
        torch.cuda.empty_cache()

    k_sub = max(3, args.steps // 2)
    mode_r = None
    if args.mode == "F" and not args.no_mode_r and not args.infer:
        release()
        model, opt = setup("R")
        dtr, _, _ = timed(model, opt, batch, k_sub, 2, silog, world, dist_on)
        progress(f"mode R {dtr / k_sub * 1e3:.2f} ms per step")
        mode_r = {"value": round(world * B * k_sub / dtr, 4), "unit": "images/sec",
                  "ms_per_step": round(dtr / k_sub * 1e3, 2),
                  "what": "reference regime: backbone + text encoder frozen (train_denseclip.py:1040-1044)"}

    fp16 = None
    if args.mode == "F" and not args.no_fp16 and not args.infer and args.dtype == "bf16" and not args.attn_fp8:
        # the 1e-3 dtype: fp32 images (what the reference trainer feeds), fp16 compute
        release()
        model, opt = setup("F", torch.float16)
        batch16 = synth_batch(B, H, W, dev, rank, image_dtype=torch.float32)
        # 3 untimed steps, as the fp8 line: a fresh fp16 model also primes its delayed gradient scales
        # (exact two-pass scales on step 1, delayed from step 2), and 2 left this line 5-7 % low on
        # some boxes (r5r: 144.8 ms where the steady state is ~135)
        dt16, s16, loss16 = timed(model, opt, batch16, k_sub, 3, silog, world, dist_on)
        ops16 = op_pass(model, opt, batch16)
        progress(f"fp16 {dt16 / k_sub * 1e3:.2f} ms per step")
        del batch16
        fp16 = {"value": round(world * B * k_sub / dt16, 4), "unit": "images/sec",
                "ms_per_step": round(dt16 / k_sub * 1e3, 2),
                "what": "mode F with fp32 images and fp16 compute (neck / heads on the HIP kernels in fp16)",
                "loss": round(loss16, 4), "roofline_attn_bwd": roofline(s16, "attn_bwd", fl_b, PEAK_BF16_TFLOPS),
                "roofline_attn_fwd": roofline(s16, "attn_fwd", fl, PEAK_BF16_TFLOPS),
                "kernels": {k: {"launches": v[0], "ms_total": round(v[1], 3), "ms_mean": round(v[2], 4)}
                            for k, v in s16.items() if not k.startswith("op:")},
                "ops": ops16}

    extras = not args.no_extras and args.mode == "F" and not args.infer and args.arch == "vitb16" \
        and not args.attn_fp8 and args.dtype == "bf16" and (H, W) == (1024, 2048)
    fp8 = None
    vitl14 = None
    if extras:
        # BASELINE configs[4]: seg + depth heads, e4m3 MX-scaled MFMA attention forward (training: the
        # 16-bit flash backward on its (o, lse)), same batch / resolution / dtype otherwise
        release()
        model, opt = setup("F", attn_fp8=True)
        # 3 untimed steps: a fresh model's first steps still build its weight caches, optimizer
        # state and allocator pools (2 left the fp8 line 5-10 % low on some boxes)
        dt8, s8, loss8 = timed(model, opt, batch, k_sub, 3, silog, world, dist_on)
        progress(f"fp8 {dt8 / k_sub * 1e3:.2f} ms per step")
        fp8 = {"value": round(world * B * k_sub / dt8, 4), "unit": "images/sec",
               "ms_per_step": round(dt8 / k_sub * 1e3, 2), "loss": round(loss8, 4),
               "what": "BASELINE configs[4]: mode F, seg + depth heads, attention forward with P V on the e4m3 "
                       "MFMA (MX E8M0 block scales) and the scores on the bf16 MFMA; backward: S, dP and the dQ "
                       "pass on the bf16 MFMA, dV = P^T dO and dK = dS^T q on the block-scaled e4m3 MFMA"
                       + ("" if ops.ATTN_BWD_FP8 else " (disabled: 16-bit flash backward)"),
               "roofline_attn_fwd": roofline(s8, "attn_fwd_fp8", fl, PEAK_FP8_MIXED_TFLOPS),
               "roofline_attn_bwd": roofline(s8, "attn_bwd", fl_b,
                                             PEAK_FP8_BWD_TFLOPS if ops.ATTN_BWD_FP8 else PEAK_BF16_TFLOPS)}
        # BASELINE configs[3]: ViT-L/14 backbone (C 1024, 24 layers, 16 heads, N = 10659)
        release()
        model, opt = setup("F", arch="vitl14")
        kl = max(3, k_sub // 2)
        dtl, sl, lossl = timed(model, opt, batch, kl, 2, silog, world, dist_on)
        NL, hl = geometry("vitl14")
        fll = attn_flops_fwd(B, NL, hl)
        vl_val = world * B * kl / dtl
        progress(f"ViT-L/14 {dtl / kl * 1e3:.2f} ms per step")
        vl_fl = 3 * model_fwd_flops(H, W, "vitl14")
        vitl14 = {"value": round(vl_val, 4), "unit": "images/sec", "ms_per_step": round(dtl / kl * 1e3, 2),
                  "steps": kl, "loss": round(lossl, 4), "tokens_per_image": NL,
                  "what": "BASELINE configs[3]: ViT-L/14 DenseCLIP train step (mode F, bf16), out_indices "
                          "[5, 11, 17, 23]",
                  "roofline_attn_fwd": roofline(sl, "attn_fwd", fll, PEAK_BF16_TFLOPS),
                  "roofline_attn_bwd": roofline(sl, "attn_bwd", 2.5 * fll, PEAK_BF16_TFLOPS),
                  "model_mfma": {"flops_per_image": vl_fl,
                                 "frac": round(vl_val / world * vl_fl / 1e12 / PEAK_BF16_TFLOPS, 4)}}
    infer = None
    if extras:
        # inference forward (eval, seg + depth resized to the image, no grad), bf16 attention vs the
        # configs[4] fp8 attention forward: where the e4m3 P.V pays (no 16-bit backward behind it)
        infer = {}
        k_inf = max(6, args.steps)
        for name, f8 in (("bf16", False), ("fp8", True)):
            release()
            model = make_model(dev, "F", "vitb16").eval()
            model.backbone.attn_fp8 = f8
            opt = None
            dti, si, _ = timed(model, None, batch, k_inf, 3, silog, world, dist_on)
            progress(f"inference {name} {dti / k_inf * 1e3:.2f} ms per step")
            # the serving path: the same forward captured into one HIP graph and replayed (the eager
            # forward's ~620 launches per step take about as long to issue as to run)
            from denseclip_vit_multimodal_amd.serve import CapturedForward
            cf = CapturedForward(model, batch[0], warmup=3)
            for _ in range(3):
                cf(batch[0])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k_inf):
                cf(batch[0])
            torch.cuda.synchronize()
            dtg = time.perf_counter() - t0
            if dist_on:
                tg = torch.tensor([dtg], device="cuda")
                dist.all_reduce(tg, op=dist.ReduceOp.MAX)
                dtg = float(tg)
            del cf
            progress(f"inference {name} graph {dtg / k_inf * 1e3:.2f} ms per step")
            infer[name] = {"value": round(world * B * k_inf / dti, 4), "unit": "images/sec",
                           "ms_per_step": round(dti / k_inf * 1e3, 2), "steps": k_inf,
                           "graph": {"value": round(world * B * k_inf / dtg, 4), "unit": "images/sec",
                                     "ms_per_step": round(dtg / k_inf * 1e3, 2),
                                     "what": "serve.CapturedForward: the step replayed from one HIP graph"},
                           "roofline_attn_fwd": roofline(si, "attn_fwd_fp8" if f8 else "attn_fwd", fl,
                                                         PEAK_FP8_MIXED_TFLOPS if f8 else PEAK_BF16_TFLOPS)}
        infer["fp8_over_bf16"] = round(infer["fp8"]["value"] / infer["bf16"]["value"], 4)
        infer["fp8_over_bf16_graph"] = round(infer["fp8"]["graph"]["value"] / infer["bf16"]["graph"]["value"], 4)
        infer["what"] = ("inference forward (eval, seg + depth at full resolution, no grad), same batch / resolution, "
                         "bf16 attention vs the configs[4] fp8 attention forward; eager launches and HIP-graph replay")
    ddp1 = None
    if extras and world == 1 and not dist_on:
        # the data-parallel wrapper's per-step cost at world size 1: the same mode-F step with the model
        # wrapped (train.wrap_ddp) over an RCCL process group of one rank
        release()
        env_keys = ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK")
        saved = {k: os.environ.get(k) for k in env_keys}
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK=str(local))
        try:
            dist.init_process_group("nccl")
            model, opt = setup("F")
            model = wrap_ddp(model, dev)
            opt = make_optimizer([p for p in model.parameters() if p.requires_grad])
            # the unwrapped step timed in the same process beside it: a box drifts by ~2 % over a
            # bench run (the A/A control), so the overhead is read against blocks of the
            # plain step interleaved with the wrapped ones (P D W W D P: linear drift cancels)
            plain, plain_opt = setup("F")
            run_steps(plain, plain_opt, batch, 3, silog)
            run_steps(model, opt, batch, 3, silog)
            has_skip = hasattr(model, "skip_collectives")
            blocks = {"P": [], "D": [], "W": []}
            for arm in ("P", "D", "W", "W", "D", "P") if has_skip else ("P", "D", "D", "P"):
                if arm == "P":
                    dtb, _, _ = timed(plain, plain_opt, batch, k_sub, 0, silog, 1, True)
                else:
                    # D: the collectives issued even on one rank (GradAllReduce skips the identity
                    # there by default): the wrapper AND RCCL's all-reduce call path; W: the wrapper
                    # alone (hooks, bucket bookkeeping)
                    if has_skip:
                        model.skip_collectives = arm == "W"
                    dtb, _, lossd = timed(model, opt, batch, k_sub, 0, silog, 1, True)
                blocks[arm].append(dtb / k_sub * 1e3)
            ms_p = sum(blocks["P"]) / len(blocks["P"])
            ms_d = sum(blocks["D"]) / len(blocks["D"])
            ms_w = sum(blocks["W"]) / len(blocks["W"]) if blocks["W"] else None
            progress(f"ddp1 {ms_d:.2f} ms per step (plain beside it {ms_p:.2f}, wrapper alone {ms_w})")
            head_ms = dt / args.steps * 1e3
            ddp1 = {"value": round(B * 1e3 / ms_d, 4), "unit": "images/sec", "ms_per_step": round(ms_d, 2),
                    "ms_per_step_plain_interleaved": round(ms_p, 2),
                    "overhead": round(ms_d / ms_p - 1.0, 4),
                    "overhead_vs_headline": round(ms_d / head_ms - 1.0, 4), "loss": round(lossd, 4),
                    "ms_per_step_without_collectives": round(ms_w, 2) if ms_w else None,
                    "overhead_without_collectives": round(ms_w / ms_p - 1.0, 4) if ms_w else None,
                    "blocks_ms": {k: [round(x, 2) for x in v] for k, v in blocks.items()},
                    "what": "mode F under the data-parallel wrapper (train.wrap_ddp: GradAllReduce, in-place "
                            "AVG all-reduces of ~100 MB gradient buckets launched during the backward as each "
                            "bucket's last gradient lands) on an RCCL process group of world size 1, with the "
                            "collectives issued (RCCL's one-rank all-reduce of the 393 MB of gradients) and, "
                            "`_without_collectives`, the wrapper alone (it skips the identity on one rank); "
                            "`overhead` against the unwrapped step timed in blocks interleaved with the wrapped "
                            "ones (P D W W D P, k steps each), `overhead_vs_headline` against the headline run "
                            "minutes earlier"}
            del plain, plain_opt
        finally:
            release()
            if dist.is_initialized():
                dist.destroy_process_group()
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    release()

    cpu = cpu0 = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto" and args.arch == "vitb16" and not args.infer:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        try:
            progress("cpu baseline")
            cpu = cpu_baseline(H, W, threads)
        except Exception as e:  # report, do not hide
            cpu = {"value": None, "error": repr(e)[:300]}
        if not args.no_extras:
            try:
                cpu0 = cpu_baseline_cfg0(threads)
            except Exception as e:
                cpu0 = {"value": None, "error": repr(e)[:300]}

    if rank == 0:
        # N >= 257 runs the CLS-split attention kernels (attention.hip bwd2_launch / fwd3 when N - 1 is a
        # multiple of 256, else fwd2 with a ragged N - 1); the fp8 forward splits CLS for N = 1 + 256k only
        cls_split = N >= 257
        fp8_split = N >= 257 and (N - 1) % 256 == 0
        rf_fwd = {"kernel": ("attn_fp8mx_kernel (+ pack%s)" % (" / row-0 pass" if fp8_split else "")
                             if args.attn_fp8 else
                             ("attn_fwd3_kernel (+ row-0 pass)" if (N - 1) % 256 == 0 else
                              "attn_fwd2_kernel (+ row-0 pass)") if cls_split else "attn_fwd_kernel"),
                  "bound": "mfma",
                  "achieved": round(achieved, 2) if achieved else None, "peak": peak_attn,
                  "unit": "TFLOP/s", "frac": round(achieved / peak_attn, 4) if achieved else None,
                  "traffic": traffic, "flops_per_launch": fl, "launches": n_att,
                  "ms_per_launch": round(mean_att, 4) if n_att else None}
        # the dominant op of a train step is the attention backward (5 N^2-matmuls
        # per launch, 2.5x the forward's): it is the headline roofline whenever it ran
        rf_bwd = None
        if n_ab:
            fp8_bwd = args.attn_fp8 and ops.ATTN_BWD_FP8
            rf_bwd = {"kernel": "attn_bwd1_prep_kernel + attn_bwd1b_kernel + attn_bwd1_dq_reduce (+ CLS-row fold merge)"
                      if cls_split and not fp8_bwd else
                      "attn_bwd_dq2_kernel + attn_bwd_dkdv8_kernel (+ pack, CLS-row fold merge)" if cls_split
                      else "attn_bwd_dq_kernel + attn_bwd_dkdv_kernel",
                      "bound": "mfma", "achieved": round(ach_b, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(ach_b / PEAK_BF16_TFLOPS, 4), "traffic": traffic_b,
                      "flops_per_launch": fl_b, "launches": n_ab, "ms_per_launch": round(mean_ab, 4)}
        line = {
            "metric": "images/sec (%s) %s DenseCLIP @%dx%d" % (
                "fwd, inference" if args.infer else "fwd+bwd",
                {"vitb16": "ViT-B/16", "vitl14": "ViT-L/14"}[args.arch], H, W),
            "value": round(value, 4),
            "unit": "images/sec",
            "n_gpus": world,
            "rccl_ranks": rccl_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype + (" (attention e4m3)" if args.attn_fp8 else ""),
            "data": "synthetic (randn images, random labels/depth; random-init weights)",
            "config": {"workload": "DenseCLIP %s seg+depth %s, %dx%d" % (
                           {"vitb16": "ViT-B/16", "vitl14": "ViT-L/14"}[args.arch],
                           ("inference forward" if args.infer else "train step (mode %s)" % args.mode)
                           + (" (fp8 attention forward)" if args.attn_fp8 else ""), H, W),
                       "per_gpu_batch": B, "global_batch": B * world, "tokens_per_image": N,
                       "parallelism": f"dp{world}", "mode": args.mode, "ddp": dist_on,
                       "grad_allreduce_dtype": args.grad_dtype if dist_on else None,
                       "head_loss": "fused resize+CE/SILog" if FUSED_HEAD_LOSS else "materialised resize"},
            "roofline": rf_bwd if rf_bwd is not None else rf_fwd,
            "roofline_attn_fwd": rf_fwd,
            "model_mfma": {"flops_per_image": model_fl, "peak_tflops": PEAK_BF16_TFLOPS, "achieved_tflops": round(value / world * model_fl / 1e12, 1),
                           "frac": round(value / world * model_fl / 1e12 / PEAK_BF16_TFLOPS, 4)} if model_fl else None,
            "kernels": kernels,
            "ops": ops_head,
            "mode_R": mode_r,
            "fp16": fp16,
            "fp8": fp8,
            "vitl14": vitl14,
            "infer": infer,
            "ddp1": ddp1,
            "cpu_baseline": cpu,
            "cpu_baseline_cfg0": cpu0,
            "loss": round(loss, 4),
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
