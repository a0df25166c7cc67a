"""GEMM engine experiments: time one shape under epilogue variants (HIP events).

    python tools/gemm_exp.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
import torch  # noqa: E402
from accunet import kern  # noqa: E402
from accunet._lib import BMODE_NN  # noqa: E402


def timeit(fn, it=20):
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
    for (M, N, K) in [(1048576, 192, 64), (1048576, 64, 192), (1048576, 32, 32), (65536, 4352, 128),
                      (65536, 128, 4352)]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        c = torch.empty(M, N, device=dev)
        bias = torch.randn(N, device=dev)
        st = torch.empty(kern.gemm_stats_rows(M, N, K), 2, N, dtype=torch.float64, device=dev)
        ideal_m = 4.0 * (M * K + M * N) / 6.3e12 * 1e6
        ideal_c = 2.0 * M * N * K / 155e12 * 1e6
        r = {}
        r["plain"] = timeit(lambda: kern.gemm(M, N, K, a=[a], lda=[K], b=w, ldb=K, c=c, ldc=N))
        r["bias"] = timeit(lambda: kern.gemm(M, N, K, a=[a], lda=[K], b=w, ldb=K, c=c, ldc=N,
                                             bias=bias))
        r["bias+stats"] = timeit(lambda: kern.gemm(M, N, K, a=[a], lda=[K], b=w, ldb=K, c=c, ldc=N,
                                                   bias=bias, stats=st))
        wn = torch.randn(K, N, device=dev)
        r["NN"] = timeit(lambda: kern.gemm(M, N, K, a=[a], lda=[K], b=wn, ldb=N, bmode=BMODE_NN,
                                           c=c, ldc=N))
        cp = torch.empty_like(c)
        r["copy C"] = timeit(lambda: cp.copy_(c))
        print(f"M{M} N{N} K{K}: ideal mem {ideal_m:.0f} us, mfma {ideal_c:.0f} us | " +
              " ".join(f"{k} {v:.0f}" for k, v in r.items()), flush=True)
        del a, w, c, st, cp


if __name__ == "__main__":
    main()
