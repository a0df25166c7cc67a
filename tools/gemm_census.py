"""GEMM census of one training step: every accunet_gemm call of the canonical
ACC_UNet at B16 256^2 timed in isolation (synchronise before/after), grouped by
shape and mode, with achieved TFLOP/s against the 157.3 TFLOP/s fp32 MFMA peak.

    python tools/gemm_census.py [--batch 16] [--size 256] [--top 40]
    python tools/gemm_census.py --replay I [--reps 20]   (PMC passes: re-launch the
        I-th GEMM of the census, by total time, REPS times at the end of the run)
"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--replay", type=int, default=-1)
    ap.add_argument("--replay-key", default="",
                    help="M,N,K,amode,bmode[,pro_a]: replay the GEMM with this key (largest total if several)")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from accunet import kern
    from accunet import model as M
    from accunet.train import TrainStep

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = M.VARIANTS["canonical"](3, 1, n_filts=32).to(dev).train()
    step = TrainStep(model, lr=1e-3, precision=a.dtype)
    x = torch.randn(a.batch, 3, a.size, a.size, device=dev)
    m = (torch.rand(a.batch, 1, a.size, a.size, device=dev) < 0.3).float()
    step(x, m)
    torch.cuda.synchronize()

    rec = collections.defaultdict(list)
    first = {}
    orig = kern.gemm

    REP = 5

    def timed(M_, N_, K_, **kw):
        # the call itself, then REP back-to-back repeats between HIP events on the
        # launch stream (every GEMM here overwrites its output: repeats are idempotent)
        r = orig(M_, N_, K_, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REP):
            orig(M_, N_, K_, **kw)
        e1.record()
        torch.cuda.synchronize()
        dt = e0.elapsed_time(e1) / 1e3 / REP
        key = (M_, N_, K_, kw.get("amode", 0), kw.get("bmode", 0), kw.get("pro_a", 0),
               kw.get("pro_b", 0), len(kw.get("a", [])), len(kw.get("ups", ())),
               bool(kw.get("allow_split")), kw.get("stats") is not None,
               kw.get("pyr") is not None)
        rec[key].append(dt)
        first.setdefault(key, ((M_, N_, K_), kw))
        return r

    kern.gemm = timed
    try:
        step(x, m)
    finally:
        kern.gemm = orig
    rows = []
    for k, v in rec.items():
        t = sum(v) / len(v)
        fl = 2.0 * k[0] * k[1] * k[2]
        rows.append((t * len(v), len(v), t, fl / t / 1e12, k))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"total GEMM time (HIP events, back-to-back repeats) {tot * 1e3:.2f} ms over {sum(r[1] for r in rows)} calls")
    print(f"{'ms':>8} {'n':>3} {'us/call':>9} {'TF/s':>7} {'/ideal':>6}  M N K amode bmode proA proB nsrc nup split stats pyr")
    for tt, n, t, tf, k in rows[:a.top]:
        M_, N_, K_ = k[:3]
        # roofline: fp32 MFMA 155 TF/s measured (bf16 ~2.5 PF), HBM 6.3 TB/s measured
        # (A + B + C only, at the activation storage width)
        es = 2.0 if a.dtype == "bf16" else 4.0
        pk = 2500e12 if a.dtype == "bf16" else 155e12
        ideal = max(2.0 * M_ * N_ * K_ / pk, es * (M_ * K_ + K_ * N_ + M_ * N_) / 6.3e12)
        print(f"{tt * 1e3:8.3f} {n:3d} {t * 1e6:9.1f} {tf:7.1f} {t / ideal:5.1f}x  {k}")
    if a.replay_key:
        want = tuple(int(v) for v in a.replay_key.split(","))
        cand = [r for r in rows if tuple(r[4][:len(want)]) == want]
        if not cand:
            raise SystemExit(f"no GEMM with key {want}")
        a.replay = rows.index(cand[0])
    if a.replay >= 0:
        k = rows[a.replay][4]
        (M_, N_, K_), kw = first[k]
        torch.cuda.synchronize()
        for _ in range(a.reps):
            orig(M_, N_, K_, **kw)
        torch.cuda.synchronize()
        print(f"replayed #{a.replay} {k} x{a.reps}: {2.0 * M_ * N_ * K_:.6e} flop per call")


if __name__ == "__main__":
    main()
