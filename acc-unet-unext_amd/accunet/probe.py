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

import hashlib
import os
import statistics

import torch

from . import kern

_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
# sources that decide K1's instruction stream (profiles/k1_traffic.json is only
# attached to a bench line whose tree has the same bytes here)
K1_SOURCES = ("dwconv.hip", "common.h", "chan.h")
K3_SOURCES = ("se.hip", "common.h", "chan.h")  # the same rule for K3's traffic


def src_hash(files=K1_SOURCES) -> str:
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(_CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]

def attach_traffic(row: dict, path: str, dtype: str, sources=K1_SOURCES) -> dict:
    """Set row["traffic"] from a committed PMC summary (profiles/k1_traffic.json,
    k3_traffic.json: FETCH_SIZE / WRITE_SIZE passes of the bench command, per launch)
    when it describes this row: same shape, same storage dtype, and taken on the same
    kernel sources as this tree (src_sha == src_hash(sources)). A summary of other
    sources is reported as traffic_stale instead; a missing one leaves traffic None."""
    if not os.path.exists(path):
        return row
    import json
    with open(path) as f:
        t = json.load(f)
    if t.get("shape") != row.get("shape") or t.get("dtype", "fp32") != dtype:
        return row
    here = src_hash(sources)
    if t.get("src_sha") == here:
        row["traffic"] = t["traffic_bytes"]
        row["traffic_source"] = t.get("source", t.get("stamp", path))
    else:
        row["traffic_stale"] = {"pmc_src_sha": t.get("src_sha"), "tree_src_sha": here}
    return row


HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md)
FP32_MFMA_TFLOPS = 157.3   # dense fp32 MFMA
BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA (~2.5 PF, MI355X_MICROARCH.md "Matrix cores")


def _time(fn, iters):
    """(mean us per launch over `iters` back-to-back launches, the per-launch times).
    An event pair brackets every launch: consecutive launches still run back to back
    (events are stream markers), and the per-launch list shows the clock's give-back
    under sustained load (MI355X DVFS: the same kernel slows as the chip heats, so
    the mean and the median are both reported)."""
    fn()  # first launch outside the timed window
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    ev[0].record()
    for i in range(iters):
        fn()
        ev[i + 1].record()
    ev[-1].synchronize()
    per = [1000.0 * ev[i].elapsed_time(ev[i + 1]) for i in range(iters)]
    total = 1000.0 * ev[0].elapsed_time(ev[-1])
    return total / iters, per


def _hbm_row(kernel, shape, bytes_alg, timing, launches):
    avg_us, per = timing
    ach = bytes_alg / (avg_us * 1e-6) / 1e9
    med = statistics.median(per)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kernel,
            "shape": shape, "avg_us": round(avg_us, 2), "median_us": round(med, 2),
            "frac_median": round(bytes_alg / (med * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "launch_us": [round(v, 1) for v in per], "launches": launches,
            "bytes_alg_per_launch": bytes_alg}


def k1_dw3x3(B, H, W, C, weight, bias, iters=20, device="cuda", dtype=torch.float32):
    """K1: HANCBlock depthwise stage as the model launches it (conv1 output with its
    pending BN1+LeakyReLU applied in the prologue, norm2 fp64 partials written)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(B, H, W, C, generator=g).to(device=device, dtype=dtype)
    sc = (torch.rand(C, generator=g) + 0.5).to(device)
    sh = (torch.randn(C, generator=g) * 0.1).to(device)
    z = torch.empty_like(x)
    st = torch.empty(kern.dw3x3_rows(B, H, W, C, x), 2, C, dtype=torch.float64, device=device)
    w = weight.detach().contiguous()
    b = bias.detach().contiguous()

    def run():
        kern.dw3x3_fwd(x, w, b, sc, sh, 1, 0, z, st, B, H, W, C)
    t = _time(run, iters)
    name = kern.dw3x3_kernel_name(B, H, W, C, x)
    row = _hbm_row(name, f"{B}x{H}x{W}x{C}", 2.0 * x.element_size() * B * H * W * C, t, iters)
    # context for the rate: the fastest device copy of the same bytes (x read once, z
    # written once; non-temporal float4 loads and stores, 4 per thread: accunet_copy_nt,
    # tools/kbench "x4/thread nt") timed the same way right after K1, so the line shows
    # what streaming reaches on this GPU in this state (the clocks under sustained load
    # move both)
    c_us, c_per = _time(lambda: kern.copy_nt(x, z), iters)
    row["copy_us"] = round(c_us, 2)
    row["copy_median_us"] = round(statistics.median(c_per), 2)
    row["frac_of_copy"] = round(c_us / t[0], 4)
    return row


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
    t = _time(run, iters)
    return _hbm_row("se_reduce+se_mid_sample+se_apply", f"{B}x{HW}x{C}",
                    2.0 * z.element_size() * B * HW * C, t, iters)


def hanc_gemm(P, N, K, iters=10, device="cuda", dtype=torch.float32):
    """The largest MFMA GEMM of the step: HANCLayer x-branch 1x1 conv of cnv72
    (P = B*64*64 pixels, K = 128*34 inputs, N = 128 outputs) with fp64 output stats.
    dtype = activation storage (fp32 engine / bf16 engine; fp32 weights either way).

    The row reports the roofline that binds this shape: MFMA time 2PNK / peak vs HBM
    time (A + B + C bytes) / 8 TB/s. fp32: 465 us vs 147 us -> "mfma"; bf16 (2.5 PF
    dense, half the A bytes): 29 us vs 74 us -> "hbm". Both fractions are kept."""
    g = torch.Generator(device="cpu").manual_seed(9)
    a = torch.randn(P, K, generator=g).to(device=device, dtype=dtype)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).to(device)
    bias = torch.zeros(N, device=device)
    c = torch.empty(P, N, device=device, dtype=dtype)
    st = torch.empty(kern.gemm_stats_rows(P, N, K), 2, N, dtype=torch.float64, device=device)

    def run():
        kern.gemm(P, N, K, a=[a], lda=[K], b=w, ldb=K, c=c, ldc=N, bias=bias, stats=st)
    us, per = _time(run, iters)
    fl = 2.0 * P * N * K
    by = float(a.element_size() * P * K + w.element_size() * N * K + c.element_size() * P * N)
    bf = dtype == torch.bfloat16
    peak = BF16_MFMA_TFLOPS if bf else FP32_MFMA_TFLOPS
    t_mfma = fl / (peak * 1e12)
    t_hbm = by / (HBM_PEAK_GBS * 1e9)
    tflops = fl / (us * 1e-6) / 1e12
    gbs = by / (us * 1e-6) / 1e9
    # fp32: the LDS-DMA engine (gemm_f32g.h) unless ACCUNET_GEMM_G=0
    kname = ("gemm_bf16_kernel" if bf else
             "gemm_f32_kernel" if os.environ.get("ACCUNET_GEMM_G", "1") == "0" else "gemm_f32g_kernel")
    row = {"kernel": kname, "shape": f"M{P} N{N} K{K}", "avg_us": round(us, 2),
           "median_us": round(statistics.median(per), 2), "launches": iters,
           "flops_alg_per_launch": fl, "bytes_alg_per_launch": by, "traffic": None,
           "frac_mfma": round(tflops / peak, 4), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)}
    if t_mfma >= t_hbm:
        row.update({"bound": "mfma", "achieved": round(tflops, 2), "peak": peak,
                    "unit": "TFLOP/s", "frac": row["frac_mfma"]})
    else:
        row.update({"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": row["frac_hbm"]})
    return row
