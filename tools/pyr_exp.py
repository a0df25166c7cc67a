"""Epilogue-cost experiment for the HANCLayer x-branch data-gradient GEMM
(cnv12 shape: P = 16*256*256, C = 96 out, K = N_hanc = 32): time the GEMM with
none / pyramid / BN-backward-stats / both epilogue features (HIP events)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
import torch  # noqa: E402
from accunet import kern  # noqa: E402
from accunet._lib import BMODE_NN  # noqa: E402


def timeit(fn, it=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    dev = "cuda"
    B, H, W = 16, 256, 256
    for (C, N) in [(96, 32), (192, 64)]:
        P = B * H * W
        J = 5
        dZ = torch.randn(P, N, device=dev)
        Wp = torch.randn(N, J * C, device=dev)
        dA = torch.empty(P, C, device=dev)
        dP2 = torch.randn(P // 4, 2 * C, device=dev)
        dP4 = torch.randn(P // 16, 2 * C, device=dev)
        mk2 = torch.randint(0, 4, (P // 4, C), dtype=torch.uint8, device=dev)
        mk4 = torch.randint(0, 16, (P // 16, C), dtype=torch.uint8, device=dev)
        z = torch.randn(P, C, device=dev)
        st = torch.rand(4, C, device=dev) + 0.5
        R = kern.gemm_stats_rows(P, C, N)
        part = torch.empty(R, 2, C, dtype=torch.float64, device=dev)
        base = dict(a=[dZ], lda=[N], b=Wp, ldb=J * C, bmode=BMODE_NN, c=dA, ldc=C, H=H, W=W)
        r = {}
        r["plain"] = timeit(lambda: kern.gemm(P, C, N, **base))
        r["pyr"] = timeit(lambda: kern.gemm(P, C, N, pyr=(dP2, dP4, mk2, mk4), **base))
        r["bnb"] = timeit(lambda: kern.gemm(P, C, N, stats=part, bnb=(z, st, 1), **base))
        r["pyr+bnb"] = timeit(lambda: kern.gemm(P, C, N, pyr=(dP2, dP4, mk2, mk4), stats=part,
                                                bnb=(z, st, 1), **base))
        mb = 4 * (P * N + P * C) / 1e6
        print(f"P{P} C{C} N{N} (A+C {mb:.0f} MB): " + " ".join(f"{k} {v:.0f}us" for k, v in r.items()),
              flush=True)


if __name__ == "__main__":
    main()
