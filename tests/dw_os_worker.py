"""Child process of test_kernels_gpu.py::test_dw3x3_one_shot_matches_strip_bitwise: runs
the depthwise forward (+ norm2 statistics), the flipped-kernel data gradient and the
BatchNorm-backward data gradient (bz / bst: the partials of accunet_bn_bwd_part) with
whatever ACCUNET_DW_OS the parent set -- the one-shot tile kernel (1) or the strip
kernel (0) -- in fp32 and bf16, and saves the outputs with the statistics TOTALS (the
two kernels cut the partial rows differently)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "acc-unet-unext_amd"))
from accunet import _lib, kern  # noqa: E402

SHAPES = [(2, 16, 64, 96), (1, 13, 35, 96), (2, 9, 21, 192), (2, 16, 16, 128), (1, 24, 40, 64)]
if os.environ.get("DW_WORKER_K1"):  # the north-star K1 shape (402 MB fp32: one-shot by default)
    SHAPES = [(16, 256, 256, 96)]


def main(out_path):
    dev = "cuda"
    lib = _lib.load()
    res = {"variant": torch.tensor(lib.accunet_dw3x3_variant(2, 16, 64, 96, 0)),
           "variant_bf16": torch.tensor(lib.accunet_dw3x3_variant(2, 16, 64, 96, 1))}
    for (B, H, W, C) in SHAPES:
        for dt in ((torch.float32,) if os.environ.get("DW_WORKER_K1") else
                   (torch.float32, torch.bfloat16)):
            g = torch.Generator().manual_seed(B * 100 + H * 7 + C)
            x = torch.randn(B, H, W, C, generator=g).to(dev, dt)
            bz = torch.randn(B, H, W, C, generator=g).to(dev, dt)
            wt = (torch.randn(C, 1, 3, 3, generator=g) * 0.3).to(dev)
            bias = (torch.randn(C, generator=g) * 0.1).to(dev)
            sc = (torch.rand(C, generator=g) + 0.5).to(dev)
            sh = (torch.randn(C, generator=g) * 0.2).to(dev)
            bst = torch.zeros(4, C, device=dev)  # mean, rstd, scale, shift
            bst[0] = torch.randn(C, generator=g).to(dev) * 0.1
            bst[1] = 1.0
            bst[2] = sc
            bst[3] = sh
            rows = kern.dw3x3_rows(B, H, W, C, x)
            st = torch.zeros(rows, 2, C, dtype=torch.float64, device=dev)
            rows_b = kern.dw3x3_rows(B, H, W, C, x, bnb=True)
            z = torch.empty_like(x)
            kern.dw3x3_fwd(x, wt, bias, sc, sh, 1, 0, z, st, B, H, W, C)
            zf = torch.empty_like(x)
            kern.dw3x3_fwd(x, wt, None, None, None, 0, 1, zf, None, B, H, W, C)
            zb = torch.empty_like(x)
            sb = torch.zeros(rows_b, 2, C, dtype=torch.float64, device=dev)
            kern.dw3x3_fwd(x, wt, None, None, None, 0, 1, zb, sb, B, H, W, C, bnb=(bz, bst, 1))
            torch.cuda.synchronize()
            tag = f"{'f32' if dt == torch.float32 else 'bf16'}_{B}x{H}x{W}x{C}"
            res[tag + "_z"] = z.float().cpu()
            res[tag + "_zf"] = zf.float().cpu()
            res[tag + "_zb"] = zb.float().cpu()
            res[tag + "_st"] = st.sum(0).cpu()
            res[tag + "_sb"] = sb.sum(0).cpu()
    torch.save(res, out_path)


if __name__ == "__main__":
    main(sys.argv[1])
