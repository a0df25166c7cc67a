"""kernels/dwconv2d benchmark at the reference's test.py shape (64 x 384 x 64 x 64, padding
k//2, no bias; its kernel sizes): one DwConv2d layer through csrc/dwconvk.hip, forward and
forward+backward (x and weight gradients), median of per-iteration HIP-event times, against
MIOpen's depthwise convolution (torch nn.Conv2d groups=C, zero padding) on the same tensors.

    python tools/dwk_bench.py [--ks 3,7,13,31] [--iters 10] [--no-miopen-bwd]

Prints one JSON line per kernel size (the format of profiles/r01_dwconvk_bench.txt).
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="3,7,13,31")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-miopen-bwd", action="store_true")
    a = ap.parse_args()
    from accunet.dwconv2d import DwConv2d
    N, C, H, W = 64, 384, 64, 64
    torch.manual_seed(0)
    x = torch.rand(N, C, H, W, device="cuda", requires_grad=True)
    gy = torch.rand(N, C, H, W, device="cuda")
    for k in [int(v) for v in a.ks.split(",")]:
        m = DwConv2d(C, (k, k), (k // 2, k // 2), bias=False).cuda()
        with torch.no_grad():
            fwd = timed(lambda: m(x), a.iters)

        def fb():
            x.grad = None
            m.weight.grad = None
            m(x).backward(gy)
        fwd_bwd = timed(fb, a.iters)
        ref = torch.nn.Conv2d(C, C, k, padding=k // 2, groups=C, bias=False).cuda()
        with torch.no_grad():
            mio = timed(lambda: ref(x), a.iters)
        row = {"k": k, "shape": f"{N}x{C}x{H}x{W}", "fwd_us": round(fwd, 1),
               "fwd_GBps": round(2 * x.numel() * 4 / fwd / 1e3, 1),
               "fwd_TFLOPs": round(2 * x.numel() * k * k / fwd / 1e6, 2),
               "fwd_bwd_us": round(fwd_bwd, 1), "miopen_zero_pad_fwd_us": round(mio, 1)}
        if not a.no_miopen_bwd:
            def rfb():
                x.grad = None
                ref.weight.grad = None
                ref(x).backward(gy)
            row["miopen_zero_pad_fwd_bwd_us"] = round(timed(rfb, max(3, a.iters // 3)), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
