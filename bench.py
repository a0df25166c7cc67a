#!/usr/bin/env python3
"""ACC-UNet training-throughput benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 16] [--size 256]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` (N > 1) without a launcher around it (no WORLD_SIZE in the environment)
starts `python -m torch.distributed.run --nnodes 1 --nproc-per-node N` on this same
command line as a child process before anything touches the GPU, relays rank 0's
JSON line and exits with the launcher's status (non-zero if any rank failed). Under
a launcher the world size must equal --gpus.

One step = forward + WeightedDiceBCE(0.5, 0.5) + backward (+ RCCL bucketed
all-reduce for N > 1) + Adam(lr 1e-3) step of the canonical ACC_UNet (16.77 M
params, ACC_UNet/ACC_UNet.py) on a per-GPU batch of 16 x 3 x 256 x 256 fp32
synthetic images resident in HBM (BASELINE configs[1]; configs[2] at N = 8).
Rank 0 prints one JSON line; `value` = images/s over all ranks (weak scaling).

Each step replays one HIP graph holding forward + loss + backward (captured on the
first call, accunet/train.py), then the RCCL all-reduce (N > 1) and the fused Adam
launch; --eager launches every kernel from Python instead.

`--model unext` runs BASELINE configs[4] instead: UNeXt (Experiments/nets/UNext.py,
1.47 M params) at 32 x 3 x 224 x 224 per GPU, same step and line format (no
roofline probes; accunet/unext.py).

Extra objects on the line:
  roofline     — the HANC depthwise stage (K1, the depthwise kernel of cnv12 and
                 cnv92, B x 256^2 x 96) timed inside the replayed training graph of
                 every timed step: event-record nodes stand around those launches
                 (accunet/profile.py), on the stream they run on; algorithmic bytes
                 (2 x B*H*W*C*4) / average launch time vs the 8 TB/s HBM3E peak.
                 `probe`: the same kernel re-launched back-to-back at that shape after
                 the timed steps, beside the fastest copy of the same bytes
                 (accunet/probe.py). `rooflines` adds K3 (the SE layer, timed the
                 same two ways) and the largest MFMA GEMM (cnv72's HANC x-branch,
                 probe only); `roofline_dw_se` reads K1 + K3
                 together;
  cpu_baseline — the CPU oracle (oracle/accunet_oracle.py, plain PyTorch-CPU, same op
                 sequence as the reference) timed on this host on a bounded sample;
                 its `parity` object runs the HIP model and the CPU path on the same
                 fixed inputs (Cfg1 Lite 1x3x128^2, canonical 1x3x256^2, eval mode) and
                 reports max |prob| difference, _show_dice and dice_on_batch of both.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec fwd+bwd, ACC-UNet 3×256×256 bs=16/GPU, 1→8 MI355X"
METRIC_UNEXT = "images/sec fwd+bwd, UNeXt 3×224×224 bs=32/GPU"
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="acc_unet", choices=["acc_unet", "unext"],
                    help="acc_unet: the headline (BASELINE configs[1]); unext: configs[4]")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (16; unext 32)")
    ap.add_argument("--size", type=int, default=None, help="image size (256; unext 224)")
    ap.add_argument("--variant", default="canonical")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="activation storage: fp32 (configs[1], the reference's precision) or "
                         "bf16 (configs[2]: bf16 activations, fp32 master weights / Adam / "
                         "BN statistics)")
    ap.add_argument("--comm-dtype", default=None, choices=["fp32", "bf16"],
                    help="gradient all-reduce wire format for N > 1 (default: bf16 with --dtype "
                         "bf16, else fp32)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python (default: replay one HIP graph per step)")
    ap.add_argument("--no-probe", action="store_true", help="skip the roofline probes")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the same-run forward parity vs the CPU path (cpu_baseline.parity)")
    ap.add_argument("--dp-world1", action="store_true",
                    help="time the data-parallel step itself (world-1 RCCL group) as the main "
                         "step, for kernel traces of the DP path; not a headline line")
    ap.add_argument("--dp-path", action="store_true",
                    help="N = 1 only: also time the data-parallel step (graph-mode event-gated "
                         "gradient buckets all-reduced by RCCL over a world-1 process group) "
                         "against the plain step, same box, and report dp_overhead_ms")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="images per timed CPU step (2; unext 16)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv, gpus, port=None):
    """The torch.distributed.run command that runs this bench on `gpus` ranks of one
    node (Experiments/Train_one_epoch.py:107,126-129 is the reference's single-process
    caller; the reference has no DP launcher at all). None when no child launch is due:
    --gpus 1, or already under a launcher (WORLD_SIZE set)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
            "--nproc-per-node", str(gpus), "--master-addr", "127.0.0.1",
            "--master-port", str(port or _free_port()),
            os.path.abspath(__file__)] + list(argv)


def relay(cmd) -> int:
    """Run the launcher as a child (never exec: see the module docstring), stream its
    stderr through, print exactly one JSON line (rank 0's) and return its exit status."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for ln in p.stdout:
        if ln.startswith('{"metric"'):
            lines.append(ln.strip())
        else:
            sys.stderr.write(ln)
    rc = p.wait()
    if rc == 0 and len(lines) != 1:
        sys.stderr.write(f"bench launcher: expected one JSON line from rank 0, got {len(lines)}\n")
        rc = 1
    if rc == 0:
        print(lines[0], flush=True)
    return rc


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import accunet_oracle as O
    return O


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_WARM, CPU_TIMED = 2, 3  # 2 warm + 3 timed steps


def cpu_baseline(variant, size, n_img, model="acc_unet"):
    """Time the CPU oracle on a bounded sample of the same workload, SURVEY 8(d)'s CPU
    protocol: two untimed warm-up steps on 1 image (first-touch allocation, thread-pool
    start), then three timed steps of n_img images each: forward + WeightedDiceBCE +
    backward + torch.optim.Adam(lr 1e-3) step. `value` is the images of the three steps
    over their summed time; the per-step rates give the spread."""
    O = _oracle()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(threads)
    spec = O.unext_param_spec(3, 1) if model == "unext" else O.param_spec(variant, 3, 1, 32)
    sd = O.det_state_dict(spec, seed=0)
    params = [v.requires_grad_(True) for k, v in sd.items()
              if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
    opt = torch.optim.Adam(params, lr=1e-3)
    name = "UNeXt" if model == "unext" else variant

    def step(n, key):
        x = O.det_input((n, 3, size, size), f"{key}-x")
        m = O.det_mask((n, 1, size, size), f"{key}-mask", p=0.3)
        opt.zero_grad(set_to_none=True)
        out = (O.unext_forward(sd, x, training=True) if model == "unext" else
               O.forward(sd, x, variant, training=True))
        loss = O.dice_bce_loss(out, m)
        loss.backward()
        opt.step()

    t0 = time.perf_counter()
    for i in range(CPU_WARM):
        step(1, f"bench-cpu-warm{i}")
    t_warm = time.perf_counter() - t0
    dts = []
    for i in range(CPU_TIMED):
        t0 = time.perf_counter()
        step(n_img, f"bench-cpu{i}")
        dts.append(time.perf_counter() - t0)
    del params, opt
    rates = [n_img / d for d in dts]
    return {"value": CPU_TIMED * n_img / sum(dts), "unit": "images/s", "cores": threads,
            "kind": "port", "steps_images_per_s": [round(r, 4) for r in rates],
            "spread": round((max(rates) - min(rates)) / (sum(rates) / len(rates)), 4),
            "sample": f"{CPU_WARM} untimed warm-up steps (1 image each, {t_warm:.1f} s), then "
                      f"{CPU_TIMED} timed steps of {n_img} image(s) each: {name} "
                      f"3x{size}x{size} fwd + WeightedDiceBCE + bwd + Adam, fp32, torch-CPU "
                      f"oracle, {sum(dts):.1f} s",
            "cpu_model": _cpu_model()}


# (variant, image size, weight seed, input key): configs[0] is the reference's own
# golden case (tests/golden/cfg1_lite.npz holds the reference's output for it), then
# configs[1]'s image at batch 1
PARITY_CASES = (("lite", 128, 1, "cfg1"), ("canonical", 256, 0, "bench-parity-256"))
PARITY_TOL = 1e-4  # north_star: forward Dice on fixed inputs within 1e-4 of the CPU path, fp32
SPREAD_LOGITS = 4.0  # the spread-head check: logits rescaled to span ~4 (probs ~0.12..0.88)


def forward_parity(dev, cases=PARITY_CASES, n_filts=32):
    """Same-run forward parity against the reference CPU path (north_star; SURVEY 8(c),
    8(d) Cfg1): for each case one fixed 1x3xSxS image and mask; the HIP model (fp32,
    eval mode, the oracle's deterministic weights) and the CPU oracle (the reference's
    op sequence) run on the same input. Reported per case:

    - the probabilities: max|prob_hip - prob_cpu|, the logged Dice
      (WeightedDiceBCE._show_dice, Experiments/utils.py:149-158) and dice_on_batch
      (utils.py:503-519) of both sides, all within 1e-4 (the north-star bound); for the
      Cfg1 case also against the reference's own recorded output
      (tests/golden/cfg1_lite.npz);
    - the pre-sigmoid logits: max|logit_hip - logit_cpu| and that divided by the logits'
      spread, and both sides against an fp64 run of the oracle: the HIP error must stay
      within 4x the reference's own fp32 error (the CPU fp32 path vs fp64) + 1e-6 of the
      logits' scale -- the yardstick of the -m gpu parity suite. With the deterministic
      weights the output is nearly constant (prob spread ~2e-4: the north-star 1e-4
      bound alone would pass a constant 0.5), so this is the check that can fail;
    - a spread head: the same network with its 1x1 head rescaled (w' = s*w,
      b' = s*(b - median logit), s = 4 / logit spread) so that the probabilities span
      ~0.12..0.88; max|prob_hip - prob_cpu| there and both sides against fp64, under
      the same yardstick.
    Both Dice values are degenerate for sigmoid-output presets (the reference applies a
    second sigmoid, so every pixel thresholds to 1); they are reported, not relied on."""
    import numpy as np
    O = _oracle()
    from accunet import model as M
    from accunet.loss import WeightedDiceBCE
    from accunet.trainer import dice_on_batch
    threads = torch.get_num_threads()
    rows = []

    def hip_run(variant, sd, x, mask, logits):
        net = M.VARIANTS[variant](3, 1, n_filts=n_filts)
        net.load_state_dict(sd)
        net = net.to(dev).eval()
        if logits:
            net.last_activation = None  # the head without its Sigmoid
        with torch.no_grad():
            y = net(x.to(dev)).float()
            torch.cuda.synchronize()
            if logits:
                return y.cpu(), None, None
            sdice = float(WeightedDiceBCE(0.5, 0.5)._show_dice(y, mask.to(dev).clone()))
            db = dice_on_batch(mask.to(dev), y)
        return y.cpu(), sdice, db

    def fp32_noise(sd_, x_, variant, l64, post):
        """the reference's own fp32 error vs fp64: the max over the plain fp32 run and
        three runs on weights and input perturbed by one fp32 rounding (relative 2^-24
        noise; a single run under-states cancellation-dominated outputs, the ensemble of
        tests/parity_util.py)"""
        e = 0.0
        for seed in (None, 1, 2, 3):
            if seed is None:
                sdp, xp = sd_, x_
            else:
                g = torch.Generator().manual_seed(seed)

                def jit(t):
                    u = torch.rand(t.shape, generator=g, dtype=torch.float64) * 2 - 1
                    return (t.double() * (1 + u * 2.0 ** -24)).float()
                sdp = {k: (jit(v) if v.is_floating_point() and not k.endswith(
                    ("running_mean", "running_var")) else v) for k, v in sd_.items()}
                xp = jit(x_)
            with torch.no_grad():
                y = post(O.forward(sdp, xp, variant, training=False, return_logits=True))
            e = max(e, float((y.double() - l64).abs().max()))
        return e

    def yard(hip, e_ref, c64, scale_of):
        e_hip = float((hip.double() - c64).abs().max())
        tol = 4.0 * e_ref + 1e-6 * float(scale_of.abs().max())
        return e_hip, tol

    for variant, S, seed, key in cases:
        sd = O.det_state_dict(O.param_spec(variant, 3, 1, n_filts), seed=seed)
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        x = O.det_input((1, 3, S, S), f"{key}-x")
        mask = O.det_mask((1, 1, S, S), f"{key}-mask", p=0.5)
        p_hip, sd_hip, db_hip = hip_run(variant, sd, x, mask, False)
        l_hip = hip_run(variant, sd, x, mask, True)[0]
        t0 = time.perf_counter()
        with torch.no_grad():
            l_cpu = O.forward(sd, x, variant, training=False, return_logits=True)
        t_cpu = time.perf_counter() - t0
        with torch.no_grad():
            l_64 = O.forward(sd64, x.double(), variant, training=False, return_logits=True)
        p_cpu = torch.sigmoid(l_cpu)
        sd_cpu = float(O.show_dice(p_cpu, mask.clone()))
        db_cpu = O.dice_on_batch(mask, p_cpu)
        spread = float(l_64.max() - l_64.min())
        e_ref = fp32_noise(sd, x, variant, l_64, lambda t: t)
        e_hip, tol = yard(l_hip, e_ref, l_64, l_64)
        row = {"case": f"{variant} n_filts {n_filts} 1x3x{S}x{S} eval",
               "max_abs_prob": float((p_hip - p_cpu).abs().max()),
               # the probabilities' own range: the scale the difference is read against
               "prob_spread": float(p_cpu.max() - p_cpu.min()),
               "show_dice": [sd_hip, sd_cpu], "dice_on_batch": [db_hip, db_cpu],
               "cpu_forward_s": round(t_cpu, 3),
               "logits": {"max_abs": float((l_hip - l_cpu).abs().max()), "spread": spread,
                          "rel_to_spread": float((l_hip - l_cpu).abs().max()) / spread,
                          "hip_vs_fp64": e_hip, "cpu32_vs_fp64": e_ref, "tol_vs_fp64": tol}}
        ok = (row["max_abs_prob"] <= PARITY_TOL and abs(sd_hip - sd_cpu) <= PARITY_TOL
              and abs(db_hip - db_cpu) <= PARITY_TOL and e_hip <= tol)
        # the spread head: probabilities across ~0.12 .. 0.88
        s = SPREAD_LOGITS / spread
        med = float(l_64.median())
        sds = dict(sd)
        sds["out.weight"] = sd["out.weight"] * s
        sds["out.bias"] = (sd["out.bias"].double() - med).float() * s
        sds64 = dict(sd64)
        sds64["out.weight"] = sds["out.weight"].double()
        sds64["out.bias"] = sds["out.bias"].double()
        ps_hip, ssd_hip, sdb_hip = hip_run(variant, sds, x, mask, False)
        with torch.no_grad():
            ps_cpu = torch.sigmoid(O.forward(sds, x, variant, training=False, return_logits=True))
            ps_64 = torch.sigmoid(O.forward(sds64, x.double(), variant, training=False,
                                            return_logits=True))
        es_ref = fp32_noise(sds, x, variant, ps_64, torch.sigmoid)
        es_hip, stol = yard(ps_hip, es_ref, ps_64, torch.ones(1))
        row["spread_head"] = {
            "scale": s, "prob_spread": float(ps_64.max() - ps_64.min()),
            "max_abs_prob": float((ps_hip - ps_cpu).abs().max()),
            "hip_vs_fp64": es_hip, "cpu32_vs_fp64": es_ref, "tol_vs_fp64": stol,
            "show_dice": [ssd_hip, float(O.show_dice(ps_cpu.float(), mask.clone()))],
            "dice_on_batch": [sdb_hip, O.dice_on_batch(mask, ps_cpu.float())]}
        ok = ok and es_hip <= stol and row["spread_head"]["prob_spread"] > 0.1
        gold = os.path.join(ROOT, "tests", "golden", "cfg1_lite.npz")
        if key == "cfg1" and os.path.exists(gold):
            g = np.load(gold)
            row["max_abs_prob_vs_reference_golden"] = float(
                np.abs(p_hip.double().numpy() - g["probs_eval"]).max())
            ok = ok and row["max_abs_prob_vs_reference_golden"] <= PARITY_TOL
        row["ok"] = ok
        rows.append(row)
    return {"tol": PARITY_TOL, "cores": threads, "cpu_model": _cpu_model(), "cases": rows,
            "ok": all(r["ok"] for r in rows)}


def dp_path_overhead(args, step, x, mask, dev, prec, reps=4):
    """The per-rank cost of the data-parallel machinery, measured at world 1 on the
    hardware clock: a second model (same init) stepped by TrainStep(graph=True,
    process_group=WORLD) over a world-1 RCCL group -- bucket packing into the flat
    all-reduce buffer, per-bucket batched weight-gradient relayouts, the marker / event
    nodes, the side-stream RCCL all-reduces (identities at world 1, but launched and
    synchronised like at world 8) and, with the bf16 wire, the widening copies --
    against the plain step, alternating blocks of --steps steps (reference caller:
    Experiments/Train_one_epoch.py:107,126-129; the reference has no DP)."""
    from accunet import model as M
    from accunet.train import TrainStep
    if dist.is_initialized():
        raise SystemExit("--dp-path runs at N = 1 (it creates its own world-1 RCCL group)")
    dist.init_process_group("nccl", rank=0, world_size=1,
                            init_method=f"tcp://127.0.0.1:{_free_port()}")
    torch.manual_seed(0)
    m2 = M.VARIANTS[args.variant](3, 1, n_filts=32).to(dev).train()
    wire = args.comm_dtype or ("bf16" if args.dtype == "bf16" else "fp32")
    sdp = TrainStep(m2, lr=1e-3, graph=True, precision=prec, process_group=dist.group.WORLD,
                    comm_dtype="bf16" if wire == "bf16" else None)
    for _ in range(args.warmup):
        sdp(x, mask)
    torch.cuda.synchronize()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn(x, mask)
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / args.steps

    plain, dp = [], []
    for _ in range(reps):
        plain.append(timed(step))
        dp.append(timed(sdp))
    mp, md = min(plain), min(dp)
    row = {"ms_per_step_plain": [round(v, 3) for v in plain],
           "ms_per_step_dp": [round(v, 3) for v in dp],
           "dp_overhead_ms": round(md - mp, 3), "dp_overhead_frac": round((md - mp) / mp, 4),
           "buckets": len(sdp._buckets.buckets), "wire": wire, "backend": "nccl (RCCL), world 1",
           "relayout_launches": sdp._defer.launches if sdp._defer is not None else None}
    del sdp, m2
    dist.destroy_process_group()
    return row


def main():
    args = parse()
    cmd = launcher_cmd(sys.argv[1:], args.gpus)
    if cmd is not None:  # before any GPU call: the ranks are children of this process
        sys.exit(relay(cmd))
    from accunet import dist as adist
    from accunet import model as M
    from accunet import profile as prof
    from accunet.train import TrainStep

    rank, world = adist.init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s)")
    local = adist.local_device()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    unext = args.model == "unext"
    if args.batch is None:
        args.batch = 32 if unext else 16
    if args.size is None:
        args.size = 224 if unext else 256
    if args.cpu_sample is None:
        args.cpu_sample = 16 if unext else 2
    torch.manual_seed(0)
    if unext:
        from accunet.unext import UNext
        model = UNext(3, 1, img_size=args.size).to(dev).train()
    else:
        model = M.VARIANTS[args.variant](3, 1, n_filts=32).to(dev).train()
    prec = None if unext else args.dtype
    if unext and args.dtype != "fp32":
        raise SystemExit("--dtype bf16 is the ACC_UNet configs[2] mode")
    if args.eager:
        reducer = adist.GradBucketReducer(model) if world > 1 else None
        step = TrainStep(model, lr=1e-3, reducer=reducer, precision=prec)
    else:
        # configs[2]: bf16 activations AND bf16 gradient buckets over xGMI (--comm-dtype)
        wire = args.comm_dtype or ("bf16" if args.dtype == "bf16" else "fp32")
        pg = None
        if args.dp_world1:
            if world > 1 or args.dp_path:
                raise SystemExit("--dp-world1: N = 1, without --dp-path")
            dist.init_process_group("nccl", rank=0, world_size=1,
                                    init_method=f"tcp://127.0.0.1:{_free_port()}")
            pg = dist.group.WORLD
        step = TrainStep(model, lr=1e-3, graph=True, precision=prec, process_group=pg,
                         comm_dtype="bf16" if wire == "bf16" else None)

    g = torch.Generator(device="cpu").manual_seed(1000 + rank)
    B, S = args.batch, args.size
    x = torch.randn(B, 3, S, S, generator=g).to(dev)
    mask = (torch.rand(B, 1, S, S, generator=g) < 0.3).float().to(dev)

    # K1 once more BEFORE any training step (the GPU not yet under sustained load), for
    # context only: the line's roofline is the probe right after the timed steps
    k1_before = None
    if not args.no_probe and not unext:
        from accunet import probe
        blk = model.cnv12
        k1_before = probe.k1_dw3x3(B, S, S, blk.conv2.weight.shape[0], blk.conv2.weight,
                                   blk.conv2.bias, dtype=model.act_dtype)
        torch.cuda.synchronize()

    # K1 / K3 timed INSIDE the captured training step: the first two launches of each
    # (cnv12's / cnv92's depthwise stage at B x 256^2 x 96, the first two SE layers at
    # B x 256^2 x 32) get event-record nodes around them (accunet/profile.py), re-pointed
    # at a fresh event pair for every replay of the timed region
    in_graph = not args.eager and not unext and not args.no_probe
    if in_graph:
        blk = model.cnv12
        k1_tag = f"dw3x3_fwd B{B} {S}x{S} C{blk.conv2.weight.shape[0]}"
        k3_tag = f"se_fwd B{B} HW{S * S} C{blk.sqe.fc2.weight.shape[0]}"
        prof.graph_time(k1_tag, 2)
        prof.graph_time(k3_tag, 2)

    for _ in range(args.warmup):
        step(x, mask)
    torch.cuda.synchronize()

    prof.enable(args.eager)  # per-launch events only make sense for eager launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    prof.graph_window(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(x, mask)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    prof.graph_window(False)
    prof.enable(False)
    graph_rows = {r["tag"]: r for r in prof.graph_rows(HBM_PEAK_GBS)} if in_graph else {}
    dt = t1 - t0
    per_rank = [dt]
    if world > 1:
        tt = torch.zeros(world, dtype=torch.float64, device=dev)
        tt[rank] = dt
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)  # every rank's time, in rank order
        per_rank = tt.tolist()
        dt = max(per_rank)
    imgs = B * world * args.steps
    dp_row = None
    if args.dp_path:
        dp_row = dp_path_overhead(args, step, x, mask, dev, prec)
    line = {
        "metric": METRIC_UNEXT if unext else METRIC,
        "value": imgs / dt,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * dt / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (x ~ N(0,1), mask ~ Bernoulli(0.3), per-rank seed 1000+rank); "
                "torch.manual_seed(0) default init",
        "config": {"workload": (f"UNext fwd+WeightedDiceBCE+bwd+Adam, {B}x3x{S}x{S} per GPU"
                                if unext else
                                f"ACC_UNet {args.variant} fwd+WeightedDiceBCE+bwd+Adam, "
                                f"{B}x3x{S}x{S} per GPU"
                                + (", bf16 activations / fp32 master weights"
                                   if args.dtype == "bf16" else "")),
                   "model": ("UNext (1.47M)" if unext else
                             "ACC_UNet (16.77M)" if args.variant == "canonical" else args.variant),
                   "global_batch": B * world, "per_gpu_batch": B, "image": [3, S, S],
                   "parallelism": f"dp{world}",
                   "grad_allreduce": (None if (world == 1 and not args.dp_world1) or args.eager else
                                      args.comm_dtype or ("bf16" if args.dtype == "bf16"
                                                          else "fp32"))},
        "final_loss": float(loss.item()),
        "ranks_seen": world,
        "ms_per_step_per_rank": [round(1000.0 * t / args.steps, 3) for t in per_rank],
    }
    # roofline: K1, the HANC depthwise stage at the north-star instance (cnv12's
    # dw3x3 over B x 256^2 x 96; cnv92 has the same shape), SURVEY.md 8(d), plus K3
    # (the SE layer) and the largest MFMA GEMM. K1 and K3: their in-model launches of
    # the timed steps (event-record nodes in the graph, above); each is also
    # re-launched back-to-back at its in-model shape right after the timed steps
    # (accunet/probe.py: `probe`, with the copy ceiling), the GEMM only that way
    if not args.no_probe and not unext:
        from accunet import probe
        blk = model.cnv12
        adt = model.act_dtype
        rl = [probe.k1_dw3x3(B, S, S, blk.conv2.weight.shape[0], blk.conv2.weight, blk.conv2.bias,
                             dtype=adt),
              probe.k3_se(B, S, S, blk.sqe.fc2.weight.shape[0], blk.sqe, dtype=adt),
              probe.hanc_gemm(B * (S // 4) ** 2, model.cnv72.hnc.cnv.weight.shape[0],
                              model.cnv72.conv1.weight.shape[0], dtype=adt)]
        if k1_before is not None:
            rl[0]["before_steps"] = {k: k1_before[k] for k in
                                     ("avg_us", "median_us", "frac", "copy_us", "frac_of_copy")}
        # K1 / K3: the launches of the timed steps are the row, the probe is kept beside
        # it. (K3's probe re-reads one 134 MB input back to back, which can partly stay in
        # the 256 MB Infinity Cache; in the step its launches ran ~25 % longer.)
        notes = {0: "cnv12's and cnv92's depthwise launch", 1: "the first two SE launches of this shape"}
        for i, tag in ((0, k1_tag if in_graph else None), (1, k3_tag if in_graph else None)):
            row = graph_rows.get(tag)
            if row is None:
                continue
            row.pop("tag")
            row["timing"] = f"in-graph: event-record nodes around {notes[i]} in every timed step"
            row["probe"] = {k: v for k, v in rl[i].items()
                            if k in ("avg_us", "median_us", "frac", "launch_us", "copy_us",
                                     "copy_median_us", "frac_of_copy", "before_steps")}
            rl[i] = row
        if in_graph and prof.graph_error():
            line["graph_timing_error"] = prof.graph_error()
        # HBM traffic of K1 / K3 from the committed PMC passes of this same bench command
        # (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs; tools/pmc_traffic.py),
        # only when taken on this tree's kernel sources
        probe.attach_traffic(rl[0], os.path.join(ROOT, "profiles", "k1_traffic.json"),
                             args.dtype, probe.K1_SOURCES)
        probe.attach_traffic(rl[1], os.path.join(ROOT, "profiles", "k3_traffic.json"),
                             args.dtype, probe.K3_SOURCES)
        line["roofline"] = rl[0]
        line["rooflines"] = rl
        # the HANC depthwise + SE reading, (bytes K1 + bytes K3) over the sum
        # of their average launch times (two launch chains, no fused kernel)
        k1, k3 = rl[0], rl[1]
        by = k1["bytes_alg_per_launch"] + k3["bytes_alg_per_launch"]
        us = k1["avg_us"] + k3["avg_us"]
        gbs = by / (us * 1e-6) / 1e9
        line["roofline_dw_se"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                                  "kernels": [k1["kernel"], k3["kernel"]],
                                  "bytes_alg": by, "us": round(us, 2)}
        if "probe" in k1 and "probe" in k3:
            pus = k1["probe"]["avg_us"] + k3["probe"]["avg_us"]
            line["roofline_dw_se"]["probe"] = {"us": round(pus, 2),
                                               "frac": round(by / (pus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
    if args.eager:
        line["rooflines_in_model"] = prof.rooflines(HBM_PEAK_GBS)
    line["mode"] = "eager" if args.eager else "hipgraph"
    if dp_row is not None:
        line["dp_path"] = dp_row
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.variant, S, args.cpu_sample, args.model)
        if not unext and not args.no_parity:
            line["cpu_baseline"]["parity"] = forward_parity(dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
