"""Large-kernel depthwise conv (accunet/dwconv2d.py) at the reference's benchmark
shape (kernels/dwconv2d/test.py:11-25: 64 x 384 x 64 x 64, padding k // 2, no
bias), per layer: forward, and forward + backward, for several kernel sizes; MIOpen's
zero-padded depthwise nn.Conv2d on the same tensors as a reference point.

    python tools/dwconvk_bench.py [--iters 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
import torch  # noqa: E402

from accunet.dwconv2d import DepthwiseFunction  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return 1000.0 * s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    N, C, S = a.batch, 384, 64
    x = torch.rand(N, C, S, S, device="cuda")
    gy = torch.rand(N, C, S, S, device="cuda")
    for k in (3, 7, 13, 31):
        w = (torch.randn(C, 1, k, k, device="cuda") * 0.1).requires_grad_(True)
        xg = x.clone().requires_grad_(True)
        p = k // 2
        fwd = timeit(lambda: DepthwiseFunction.apply(x, w, None, p, p, False), a.iters)

        def fb():
            y = DepthwiseFunction.apply(xg, w, None, p, p, False)
            y.backward(gy)
        fwdbwd = timeit(fb, a.iters)
        conv = torch.nn.Conv2d(C, C, k, padding=p, groups=C, bias=False).cuda()
        mio = timeit(lambda: conv(x), a.iters)
        nbytes = 2.0 * x.numel() * 4
        flops = 2.0 * x.numel() * k * k
        print(json.dumps({"k": k, "shape": f"{N}x{C}x{S}x{S}", "fwd_us": round(fwd, 1),
                          "fwd_GBps": round(nbytes / fwd / 1e3, 1),
                          "fwd_TFLOPs": round(flops / fwd / 1e6, 2),
                          "fwd_bwd_us": round(fwdbwd, 1), "miopen_zero_pad_fwd_us": round(mio, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
