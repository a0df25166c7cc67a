"""Roofline probes: the bench's hot kernels re-launched in isolation at their
in-model shapes, timed with HIP events recorded on the stream they are launched
on (torch's current stream, which every accunet kernel uses). Inside a replayed
HIP graph individual launches cannot be bracketed by events, and in eager mode an
event pair around one launch also times the host's launch latency whenever the
GPU is starved; back-to-back launches of one kernel between two events give its
true average duration, which is what rocprofv3 --kernel-trace reports for the
same grid (profiles/ keeps both).

Algorithmic bytes follow SURVEY.md 8(d): K1 (HANC depthwise) and K3 (SE) move
one read + one write of their activation, 2 * B*H*W*C * s bytes (s = 4 fp32, 2 in
the bf16 activation mode); weights and statistics are excluded.
"""
from __future__ import annotations

import torch

from . import kern

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md)
FP32_MFMA_TFLOPS = 157.3   # dense fp32 MFMA
BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA (~2.5 PF, MI355X_MICROARCH.md "Matrix cores")


def _time(fn, iters):
    fn()  # first launch outside the timed window
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return 1000.0 * s.elapsed_time(e) / iters  # us per launch


def _hbm_row(kernel, shape, bytes_alg, avg_us, launches):
    ach = bytes_alg / (avg_us * 1e-6) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kernel,
            "shape": shape, "avg_us": round(avg_us, 2), "launches": launches,
            "bytes_alg_per_launch": bytes_alg}


def k1_dw3x3(B, H, W, C, weight, bias, iters=20, device="cuda", dtype=torch.float32):
    """K1: HANCBlock depthwise stage as the model launches it (conv1 output with its
    pending BN1+LeakyReLU applied in the prologue, norm2 fp64 partials written)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(B, H, W, C, generator=g).to(device=device, dtype=dtype)
    sc = (torch.rand(C, generator=g) + 0.5).to(device)
    sh = (torch.randn(C, generator=g) * 0.1).to(device)
    z = torch.empty_like(x)
    st = torch.empty(kern.dw3x3_rows(B, H, W, C), 2, C, dtype=torch.float64, device=device)
    w = weight.detach().contiguous()
    b = bias.detach().contiguous()

    def run():
        kern.dw3x3_fwd(x, w, b, sc, sh, 1, 0, z, st, B, H, W, C)
    us = _time(run, iters)
    name = "dw3x3_tile_fwd_kernel" if C % 32 == 0 else "dw3x3_fwd_kernel"
    return _hbm_row(name, f"{B}x{H}x{W}x{C}", 2.0 * x.element_size() * B * H * W * C, us, iters)


def k3_se(B, H, W, C, se_mod, iters=20, device="cuda", dtype=torch.float32):
    """K3: ChannelSELayer fused with its preceding BN3+LeakyReLU (one reduce pass,
    gate + analytic BN statistics, one apply pass) as the model launches it."""
    g = torch.Generator(device="cpu").manual_seed(8)
    HW = H * W
    Cr = se_mod.fc1.weight.shape[0]
    z = torch.randn(B, H, W, C, generator=g).to(device=device, dtype=dtype)
    sc = (torch.rand(C, generator=g) + 0.5).to(device)
    sh = (torch.randn(C, generator=g) * 0.1).to(device)
    out = torch.empty_like(z)
    save = torch.empty(kern.se_save_elems(B, C, Cr), device=device)
    rm = torch.zeros(C, device=device)
    rv = torch.ones(C, device=device)
    p = {k: v.detach().contiguous() for k, v in se_mod.named_parameters()}

    def run():
        kern.se_fwd(z, sc, sh, 1, B, HW, C, Cr, p["fc1.weight"], p["fc1.bias"], p["fc2.weight"],
                    p["fc2.bias"], p["bn.weight"], p["bn.bias"], rm, rv, None, 0.1, 1e-5, True,
                    out, save, None)
    us = _time(run, iters)
    return _hbm_row("se_reduce+se_mid_sample+se_mid_bn+se_apply", f"{B}x{HW}x{C}",
                    2.0 * z.element_size() * B * HW * C, us, iters)


def hanc_gemm(P, N, K, iters=10, device="cuda", dtype=torch.float32):
    """The largest MFMA GEMM of the step: HANCLayer x-branch 1x1 conv of cnv72
    (P = B*64*64 pixels, K = 128*34 inputs, N = 128 outputs) with fp64 output stats.
    dtype = activation storage (fp32 engine / bf16 engine; fp32 weights either way)."""
    g = torch.Generator(device="cpu").manual_seed(9)
    a = torch.randn(P, K, generator=g).to(device=device, dtype=dtype)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(device)
    bias = torch.zeros(N, device=device)
    c = torch.empty(P, N, device=device, dtype=dtype)
    st = torch.empty(kern.gemm_stats_rows(P, N, K), 2, N, dtype=torch.float64, device=device)

    def run():
        kern.gemm(P, N, K, a=[a], lda=[K], b=w, ldb=K, c=c, ldc=N, bias=bias, stats=st)
    us = _time(run, iters)
    fl = 2.0 * P * N * K
    ach = fl / (us * 1e-6) / 1e12
    bf = dtype == torch.bfloat16
    peak = BF16_MFMA_TFLOPS if bf else FP32_MFMA_TFLOPS
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None,
            "kernel": "gemm_bf16_kernel" if bf else "gemm_f32_kernel",
            "shape": f"M{P} N{N} K{K}", "avg_us": round(us, 2),
            "launches": iters, "flops_alg_per_launch": fl}
