"""Child process of test_gemm_gpu.py::test_conv3x3_halo_matches_engine_bitwise: runs the
32-channel 3x3 forward (+ statistics) and data gradient (in-place addend) through
accunet_gemm in fp32 and in bf16 activation mode, with whatever ACCUNET_CONV3_HALO the
parent set (the halo kernels or the implicit-GEMM engine), and saves the outputs with
the number of halo-kernel launches the library made (accunet_conv3x3_halo_launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "acc-unet-unext_amd"))
from accunet import _lib, kern  # noqa: E402


def main(out_path):
    torch.manual_seed(21)
    dev = "cuda"
    lib = _lib.load()
    n0 = lib.accunet_conv3x3_halo_launches(0)
    res = {}
    # 256 tiles of 128 pixels (the few-tiles threshold: still 128x32 engine tiles) and
    # 1024 tiles, well above it
    for (B, H, W, C), dt in [(s, d) for s in ((4, 64, 128, 32), (8, 128, 128, 32))
                             for d in (torch.float32, torch.bfloat16)]:
        P = B * H * W
        x = torch.randn(P, C, device=dev).to(dt)
        wr = torch.randn(C, 9 * C, device=dev) * 0.1
        bias = torch.randn(C, device=dev)
        out = torch.empty(P, C, device=dev, dtype=dt)
        rows = kern.gemm_stats_rows(P, C, 9 * C, _lib.AMODE_SHIFT3, _lib.BMODE_NT, C)
        st = torch.zeros(rows, 2, C, device=dev, dtype=torch.float64)
        kern.gemm(P, C, 9 * C, a=[x], lda=[C], amode=_lib.AMODE_SHIFT3, b=wr, ldb=9 * C, c=out,
                  ldc=C, bias=bias, stats=st, H=H, W=W, cin=C)
        dx = torch.randn(P, C, device=dev).to(dt)
        kern.gemm(P, C, 9 * C, a=[x], lda=[C], amode=_lib.AMODE_SHIFT3, b=wr, ldb=9 * C, c=dx,
                  ldc=C, H=H, W=W, cin=C, ups=[(dx, C, 0, 0)])
        torch.cuda.synchronize()
        tag = ("f32" if dt == torch.float32 else "bf16") + f"_{P}"
        res[f"{tag}_out"] = out.float().cpu()
        res[f"{tag}_stats"] = st.cpu()
        res[f"{tag}_dx"] = dx.float().cpu()
    # which implementation ran: 2 GEMMs x 2 shapes x 2 dtypes on the halo kernels, or none
    res["halo_launches"] = torch.tensor(lib.accunet_conv3x3_halo_launches(0) - n0)
    torch.save(res, out_path)


if __name__ == "__main__":
    main(sys.argv[1])
