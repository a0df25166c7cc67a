"""Kernel-level parity of the streaming HANC kernels against fp64 torch restatements
of the reference ops (the depthwise conv + norm2 statistics of HANCBlock,
ACC_UNet/ACC_UNet.py:240-247,273-275, and ChannelSELayer :37-49), called through
the C ABI (accunet.kern) so every tile variant / fallback path is exercised:
    dw3x3: forward / data gradient on the LDS-tiled TCQ=8 / TCQ=16 kernels
           (C % 32 == 0) or the register-window fallback (incl. cnv11's C = 9); the
           weight gradient on the whole-pixel span kernel (C % 8 == 0, C <= 128:
           256-thread blocks, ragged spans and row bands) or the tile kernels. The
           span FORWARD kernel (ACCUNET_DW_SPAN bit 2, off by default; 256- and 512-
           thread blocks) runs the same checks in a child process with the knob set."""
import os
import sys

import pytest
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "acc-unet-unext_amd"))

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _kern():
    from accunet import kern
    return kern


def _lrelu(t):
    return torch.where(t > 0, t, 0.01 * t)


DW_SHAPES = [
    (2, 16, 16, 96),     # TCQ 16 tile, W = TP; wgrad span, 10-pixel spans (last 6)
    (2, 24, 40, 64),     # TCQ 8 tile, ragged H and W; wgrad 16-pixel spans
    (1, 13, 35, 32),     # ragged everything
    (3, 8, 8, 128),      # W < TP / PX
    (1, 13, 35, 96),     # wgrad span, ragged H (13) and W (35 = 3 x 10 + 5)
    (2, 9, 21, 192),     # tile kernels (span forward knob: 512 threads, PX 10)
    (1, 8, 17, 256),     # tile kernels (span forward knob: 512 threads, PX 8)
    (2, 6, 300, 8),      # register kernel; wgrad span with 2 quads per pixel (PX 128)
    (2, 16, 24, 384),    # TCQ 8 tile (C > 256, wgrad too)
    (2, 16, 16, 320),    # TCQ 16 tile (W <= 16)
    (2, 17, 19, 36),     # fallback register-window kernel, V = 4
    (2, 12, 12, 9),      # fallback, V = 1 (cnv11's hidden width)
]


@pytest.mark.parametrize("B,H,W,C", DW_SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_dw3x3_fwd_stats_wgrad_vs_fp64(B, H, W, C, pro):
    kern = _kern()
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + C)
    x = torch.randn(B, H, W, C, generator=g, dtype=torch.float64)
    wt = torch.randn(C, 1, 3, 3, generator=g, dtype=torch.float64) * 0.3
    bias = torch.randn(C, generator=g, dtype=torch.float64) * 0.1
    sc = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(C, generator=g, dtype=torch.float64) * 0.2
    dz = torch.randn(B, H, W, C, generator=g, dtype=torch.float64)
    a = _lrelu(x * sc + sh) if pro else x
    a_nchw = a.permute(0, 3, 1, 2)
    z_ref = F.conv2d(a_nchw, wt, bias, padding=1, groups=C).permute(0, 2, 3, 1)
    # flipped-kernel correlation = data gradient of the conv
    zf_ref = F.conv2d(a_nchw, wt.flip(-1).flip(-2), None, padding=1, groups=C).permute(0, 2, 3, 1)
    # weight / bias gradient for upstream dz
    a_req = a_nchw.clone().requires_grad_(False)
    w_req = wt.clone().requires_grad_(True)
    b_req = bias.clone().requires_grad_(True)
    zz = F.conv2d(a_req, w_req, b_req, padding=1, groups=C)
    (zz * dz.permute(0, 3, 1, 2)).sum().backward()

    f = lambda t: t.float().contiguous().to(DEV)  # noqa: E731
    xd, wd, bd, scd, shd, dzd = f(x), f(wt), f(bias), f(sc), f(sh), f(dz)
    rows = kern.dw3x3_rows(B, H, W, C, xd)
    st = torch.zeros(rows, 2 * C, dtype=torch.float64, device=DEV)
    z = torch.empty(B, H, W, C, device=DEV)
    act = 1 if pro else 0
    kern.dw3x3_fwd(xd, wd, bd, scd if pro else None, shd if pro else None, act, 0, z, st, B, H, W, C)
    zf = torch.empty_like(z)
    kern.dw3x3_fwd(xd, wd, None, scd if pro else None, shd if pro else None, act, 1, zf, None,
                   B, H, W, C)
    dw = torch.empty(C, 1, 3, 3, device=DEV)
    db = torch.empty(C, device=DEV)
    kern.dw3x3_wgrad(xd, dzd, scd if pro else None, shd if pro else None, act, dw, db, B, H, W, C)
    torch.cuda.synchronize()
    scale = z_ref.abs().max().item()
    assert (z.double().cpu() - z_ref).abs().max().item() <= 2e-6 * scale
    assert (zf.double().cpu() - zf_ref).abs().max().item() <= 2e-6 * scale
    s = st.sum(0).cpu()
    zr = z_ref.reshape(-1, C)
    assert torch.allclose(s[:C], zr.sum(0), rtol=1e-6, atol=1e-6 * zr.abs().sum(0).max().item())
    assert torch.allclose(s[C:], (zr * zr).sum(0), rtol=1e-6)
    gw = w_req.grad
    assert (dw.double().cpu() - gw).abs().max().item() <= 1e-5 * gw.abs().max().item() + 1e-5
    gb = b_req.grad
    assert (db.double().cpu() - gb).abs().max().item() <= 1e-5 * gb.abs().max().item() + 1e-5


def _dw_compare(outs, a_key, b_key):
    for k in outs[a_key]:
        a, b = outs[a_key][k], outs[b_key][k]
        if k.endswith("_sb"):  # BN-backward partials: fp64 per element in both kernels
            assert torch.allclose(a, b, rtol=1e-9, atol=1e-9 * float(b.abs().max())), k
        elif k.endswith("_st"):  # (sum z, sum z^2): fp32 over 4-row chunks vs 8-row tiles
            C = a.shape[-1]
            zabs = outs[b_key][k[:-3] + "_z"].double().abs().reshape(-1, C).sum(0)
            assert bool(((a[0] - b[0]).abs() <= 1e-6 * zabs).all()), k
            assert torch.allclose(a[1], b[1], rtol=1e-6), k
        else:
            assert torch.equal(a, b), (k, float((a - b).abs().max()))


def _dw_runs(tmp_path, settings, extra_env=None):
    import subprocess
    outs = {}
    for v in settings:
        env = dict(os.environ, ACCUNET_DW_OS=v, **(extra_env or {}))
        path = tmp_path / f"dw_{v}.pt"
        subprocess.run([sys.executable, os.path.join(HERE, "dw_os_worker.py"), str(path)], env=env,
                       check=True, timeout=240)
        outs[v] = torch.load(path, weights_only=True)
    return outs


@pytest.mark.parametrize("os16", ["1", "0"])
def test_dw3x3_one_shot_k1_shape_matches_strip(tmp_path, os16):
    """The default kernel choice at the north-star K1 shape (16 x 256^2 x 96 fp32, 402 MB:
    one-shot tiles for the forward and the plain data gradient -- 16-row 512-thread tiles,
    or with ACCUNET_DW_OS16=0 the 8-row tiles -- the strip for the BN-backward data
    gradient) against the strip everywhere (ACCUNET_DW_OS=0): z and both data gradients
    bit for bit, statistics totals to summation order."""
    outs = _dw_runs(tmp_path, ("1", "0"), {"DW_WORKER_K1": "1", "ACCUNET_DW_OS16": os16})
    assert int(outs["1"].pop("variant")) == 1  # (the worker's 2 x 16 x 64 probe shape)
    outs["0"].pop("variant")
    outs["1"].pop("variant_bf16")
    outs["0"].pop("variant_bf16")
    _dw_compare(outs, "1", "0")


@pytest.mark.parametrize("os16", ["1", "0"])
def test_dw3x3_one_shot_matches_strip_bitwise(tmp_path, os16):
    """The one-shot tile kernel and the strip kernel sum every output in the same order
    (bias, then the taps row-major), so forward z, the flipped-kernel data gradient and
    the BatchNorm-backward data gradient are bit-identical, and their statistics totals
    (the partial rows are cut differently: one per 8-row tile vs one per 32-row strip)
    agree to summation order. ACCUNET_DW_OS=2 (one-shot tiles for every tile shape,
    dtype and launch kind) against 0 (the strip everywhere) on ragged and channel-group
    shapes, fp32 and bf16, each in a child process (the knob is read once per process;
    tests/dw_os_worker.py)."""
    outs = _dw_runs(tmp_path, ("2", "0"), {"ACCUNET_DW_OS16": os16})
    one_shot = 4 if os16 == "1" else 3  # 16-row 512-thread tiles / 8-row tiles
    assert int(outs["2"].pop("variant")) == one_shot and int(outs["0"].pop("variant")) == 1
    assert int(outs["2"].pop("variant_bf16")) == one_shot and int(outs["0"].pop("variant_bf16")) == 1
    _dw_compare(outs, "2", "0")


@pytest.mark.parametrize("B,H,W,C", [(2, 16, 64, 96), (1, 13, 35, 96), (2, 24, 40, 192),
                                     (1, 16, 16, 64), (2, 9, 20, 128)])
@pytest.mark.parametrize("pro", [False, True])
def test_dw3x3_bf16_fwd_vs_fp64(B, H, W, C, pro):
    """bf16 storage (BASELINE configs[2]): the depthwise forward reads bf16 x, computes
    in fp32 (prologue, 9 taps) and stores z rounded to bf16; its norm2 statistics are
    those of the stored values. Against an fp64 restatement of the same rounding: z
    within one bf16 rounding (2^-8 relative, plus the fp32 arithmetic), statistics of
    the stored z within fp32 accumulation noise. Covers 32- and 64-channel tiles
    (C % 64 == 0) and ragged images (the register-staged strip kernel)."""
    kern = _kern()
    g = torch.Generator().manual_seed(B * 7 + H * 3 + C)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    wt = torch.randn(C, 1, 3, 3, generator=g, dtype=torch.float64) * 0.3
    bias = torch.randn(C, generator=g, dtype=torch.float64) * 0.1
    sc = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(C, generator=g, dtype=torch.float64) * 0.2
    xd = x.double()
    a = _lrelu(xd * sc.float().double() + sh.float().double()) if pro else xd
    z_ref = F.conv2d(a.permute(0, 3, 1, 2), wt.float().double(), bias.float().double(), padding=1,
                     groups=C).permute(0, 2, 3, 1)
    xg = x.to(DEV)
    wd = wt.float().to(DEV)
    rows = kern.dw3x3_rows(B, H, W, C, xg)
    st = torch.zeros(rows, 2, C, dtype=torch.float64, device=DEV)
    z = torch.empty(B, H, W, C, device=DEV, dtype=torch.bfloat16)
    kern.dw3x3_fwd(xg, wd, bias.float().to(DEV), sc.float().to(DEV) if pro else None,
                   sh.float().to(DEV) if pro else None, 1 if pro else 0, 0, z, st, B, H, W, C)
    torch.cuda.synchronize()
    zh = z.double().cpu()
    scale = z_ref.abs().max().item()
    assert (zh - z_ref).abs().max().item() <= 2.0 ** -8 * z_ref.abs().max().item() * 1.01 + 1e-6 * scale
    # statistics describe the stored (rounded) values
    s_ = st.sum(0).cpu()  # [2][C]: sum z, sum z^2
    zr = zh.reshape(-1, C)
    assert torch.allclose(s_[0], zr.sum(0), rtol=1e-6, atol=1e-6 * zr.abs().sum(0).max().item())
    assert torch.allclose(s_[1], (zr * zr).sum(0), rtol=1e-6)


def test_dw3x3_span_forward_knob_vs_fp64():
    """The span forward / data-gradient kernel ships behind ACCUNET_DW_SPAN bit 2 (read
    once per process by the library): a child process with ACCUNET_DW_SPAN=3 runs the
    forward + statistics + flipped-kernel + weight-gradient checks above on shapes that
    select it with 256-thread (C/4 <= 32) and 512-thread (C/4 33..64) blocks."""
    import subprocess
    code = (
        "import sys; sys.path.insert(0, %r); import test_kernels_gpu as T\n"
        "from accunet import _lib\n"
        "lib = _lib.load()\n"
        "for (B, H, W, C) in [(2, 16, 16, 96), (1, 13, 35, 96), (2, 6, 300, 8), (2, 9, 21, 192),\n"
        "                     (1, 8, 17, 256), (2, 24, 40, 64)]:\n"
        "    assert lib.accunet_dw3x3_variant(B, H, W, C, 0) == 2, (B, H, W, C)\n"
        "    for pro in (False, True):\n"
        "        T.test_dw3x3_fwd_stats_wgrad_vs_fp64(B, H, W, C, pro)\n"
        "print('SPAN_OK')\n") % HERE
    env = dict(os.environ, ACCUNET_DW_SPAN="3")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240, cwd=HERE)
    assert r.returncode == 0 and "SPAN_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("B,H,C", [(4, 16, 64), (2, 8, 32), (16, 32, 256), (3, 5, 40), (2, 8, 18),
                                   (2, 8, 512), (16, 64, 32)])
def test_se_layer_vs_fp64_oracle(B, H, C):
    """ChannelSELayer (fused GAP / gate / BN-of-gated / LeakyReLU, and its backward) vs
    the fp64 oracle; tolerance relative to the reference's own fp32 error."""
    sys.path.insert(0, HERE)
    import parity_util as PU
    from parity_util import O
    from accunet import model as M
    torch.manual_seed(0)
    se = M.ChannelSELayer(C)
    spec = [("s." + n, tuple(t.shape)) for n, t in se.state_dict().items()]
    sd = O.det_state_dict(spec, seed=3)
    se.load_state_dict({n[2:]: v for n, v in sd.items()})
    se = se.to(DEV).train()
    x = O.det_input((B, C, H, H), "se-x") * 2 + 0.5
    go = O.det_input((B, C, H, H), "se-go")
    res = {}
    for dt in (torch.float64, torch.float32):
        sdo = {n: (v.to(dt).requires_grad_(not n.endswith(PU.BUFFER_LEAVES))
                   if v.is_floating_point() else v.clone()) for n, v in sd.items()}
        xr = x.detach().clone().to(dt).requires_grad_(True)
        y = O.se(xr, sdo, "s", True)
        (y * go.to(dt)).sum().backward()
        res[dt] = (y.detach(), xr.grad, {n[2:]: v.grad for n, v in sdo.items() if v.grad is not None},
                   {n[2:]: v for n, v in sdo.items()})
    xh = x.detach().to(DEV).requires_grad_(True)
    y = se(xh)
    (y * go.to(DEV)).sum().backward()
    hip = {"out": y, "dx": xh.grad}
    a64 = {"out": res[torch.float64][0], "dx": res[torch.float64][1]}
    a32 = {"out": res[torch.float32][0], "dx": res[torch.float32][1]}
    for n, p in se.named_parameters():
        hip[n] = p.grad
        a64[n] = res[torch.float64][2][n]
        a32[n] = res[torch.float32][2][n]
    sdh = se.state_dict()
    for n in ("bn.running_mean", "bn.running_var"):
        hip[n] = sdh[n]
        a64[n] = res[torch.float64][3][n]
        a32[n] = res[torch.float32][3][n]
    rows = PU.compare_vs_reference_fp32(hip, a64, a32, factor=4.0, rel_floor=1e-5)
    bad = [r for r in rows if not r[4]]
    assert not bad, bad


@pytest.mark.parametrize("B,H,W,C,dt", [(2, 16, 32, 32, torch.float32), (3, 8, 12, 20, torch.float32),
                                        (16, 256, 256, 32, torch.float32),
                                        (2, 16, 32, 64, torch.bfloat16)])
def test_upsample_bwd24_matches_two_blocksums(B, H, W, C, dt):
    """The k = 3 HANCLayer backward's fused pyramid sums (one read of dZ) carry the bits
    of the two separate f = 2 / f = 4 block-sum launches, and match float64."""
    from accunet import kern
    torch.manual_seed(31)
    dz = torch.randn(B, H, W, C, device=DEV).to(dt)
    g2 = torch.empty(B, H // 2, W // 2, C, device=DEV, dtype=dt)
    g4 = torch.empty(B, H // 4, W // 4, C, device=DEV, dtype=dt)
    kern.upsample_bwd24(dz, C, g2, C, g4, C, B, H, W, C)
    r2, r4 = torch.empty_like(g2), torch.empty_like(g4)
    kern.upsample_bwd(dz, C, 0, r2, C, B, H, W, C, 2)
    kern.upsample_bwd(dz, C, 0, r4, C, B, H, W, C, 4)
    assert torch.equal(g2, r2) and torch.equal(g4, r4)
    d = dz.double()
    ref4 = d.view(B, H // 4, 4, W // 4, 4, C).sum((2, 4))
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert ((g4.double() - ref4).abs().max() / ref4.abs().max()).item() < tol


def test_bucket_packing_copies_aligned_and_ragged():
    """relayout_batch_kernel kinds 3 / 4 (the DP bucket packing, ops.DeferredRelayouts
    .copy): the float4 path (16-byte aligned source and destination) and the scalar path
    (destinations at odd element offsets, ragged lengths), times a scale, into fp32 and
    bf16 wires -- bit-equal to torch's (src * scale).to(dtype)."""
    from accunet import ops
    torch.manual_seed(12)
    d = ops.DeferredRelayouts(DEV, cap=8)
    src = [torch.randn(n, device=DEV) for n in (4096, 1031, 7, 5000)]
    wire32 = torch.zeros(16384, device=DEV)
    wire16 = torch.zeros(16384, device=DEV, dtype=torch.bfloat16)
    cases = [(src[0], wire32[0:4096], 1.0), (src[1], wire32[4097:5128], 0.125),
             (src[2], wire16[8:15], 0.5), (src[3], wire16[5001:10001], 0.125)]
    kern = _kern()
    for s_, dst, sc in cases:
        d.copy(s_, dst, scale=sc)
    d.flush()   # (the captured launch; outside a capture its table is not filled yet)
    d.upload()  # the item table, as TrainStep uploads it after the capture
    kern.relayout_batch(d.table, len(d.items), sum(kern.relayout_blocks(it.total) for it in d.items))
    torch.cuda.synchronize()
    for s_, dst, sc in cases:
        assert torch.equal(dst, (s_ * sc).to(dst.dtype)), (dst.dtype, dst.numel(), sc)


def _two_pass(z, C, rv0, mom=0.1, eps=1e-5):
    """ATen's BatchNorm2d training statistics restated in fp64, two passes over the
    stored values: mean, rstd (of the biased variance) and the running_var update with
    the unbiased variance."""
    zz = z.double().reshape(-1, C).cpu()
    n = zz.shape[0]
    m = zz.mean(0)
    v = ((zz - m) ** 2).mean(0)
    rstd = 1.0 / torch.sqrt(v + eps)
    rv = (1 - mom) * rv0.double().cpu() + mom * v * n / (n - 1)
    return m, rstd, rv, v


def _finish_and_compare(st, rows, z, C, tag):
    kern = _kern()
    dev = z.device
    P = z.numel() // C
    gamma = torch.ones(C, device=dev)
    beta = torch.zeros(C, device=dev)
    rmean = torch.zeros(C, device=dev)
    rv0 = torch.linspace(0.5, 2.0, C, device=dev)
    rvar = rv0.clone()
    nbt = torch.zeros((), dtype=torch.long, device=dev)
    out = torch.empty(4, C, device=dev)
    kern.bn_finalize(st, rows, C, float(P), gamma, beta, rmean, rvar, nbt, 0.1, 1e-5, True, out)
    torch.cuda.synchronize()
    m, rstd, rv, v = _two_pass(z, C, rv0)
    # the test is only meaningful if the channels really are offset: mean >= 300 x spread
    assert float((m.abs() / v.sqrt()).min()) >= 300, tag
    got_m, got_r = out[0].double().cpu(), out[1].double().cpu()
    assert float(((got_m - m) / m).abs().max()) <= 1e-6, (tag, "mean")
    rel_r = float(((got_r - rstd) / rstd).abs().max())
    assert rel_r <= 1e-6, (tag, "rstd", rel_r)
    rel_v = float(((rvar.double().cpu() - rv) / rv).abs().max())
    assert rel_v <= 1e-6, (tag, "running_var", rel_v)
    assert int(nbt) == 1


@pytest.mark.parametrize("B,H,W,C", [(2, 32, 48, 96), (16, 256, 256, 96)])
def test_bn_statistics_large_mean_match_two_pass_fp64(B, H, W, C):
    """BatchNorm statistics (ATen's two-pass fp64 BatchNorm at e.g.
    ACC_UNet/ACC_UNet.py:274) from the producers' partial sums plus the finish kernel,
    on channels whose mean is ~300-1000x their spread -- the case where sum z^2 - n m^2
    from fp32 partials would cancel: K1 (the depthwise forward, strip kernel at the small
    shape, one-shot tiles at the north-star 16x256^2x96), a GEMM epilogue and the
    materialising affine pass. Mean, rstd and running_var within 1e-6 relative of a
    two-pass fp64 computation over the stored values."""
    kern = _kern()
    g = torch.Generator().manual_seed(7)
    P = B * H * W
    # K1: x ~ N(0,1), weights of norm ~0.35, bias ~300 -> z ~ 300 +- 0.35 (a large bias,
    # not a large input: the zero-padded border keeps the per-channel spread small)
    x = torch.randn(B, H, W, C, generator=g).to(DEV)
    wt = (1.0 / 9 + 0.02 * torch.randn(C, 1, 3, 3, generator=g)).to(DEV)
    bias = (300.0 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    z = torch.empty_like(x)
    rows = kern.dw3x3_rows(B, H, W, C, x)
    st = torch.zeros(rows, 2, C, dtype=torch.float64, device=DEV)
    kern.dw3x3_fwd(x, wt, bias, None, None, 0, 0, z, st, B, H, W, C)
    _finish_and_compare(st, rows, z, C, f"dw3x3 {kern.dw3x3_kernel_name(B, H, W, C)}")
    # GEMM epilogue: z = a W^T + 300, spread ~0.4
    K, N = 64, 96
    a = torch.randn(P, K, generator=g).to(DEV)
    w = (0.05 * torch.randn(N, K, generator=g)).to(DEV)
    b2 = torch.full((N,), 300.0, device=DEV)
    zg = torch.empty(P, N, device=DEV)
    rg = kern.gemm_stats_rows(P, N, K)
    sg = torch.zeros(rg, 2, N, dtype=torch.float64, device=DEV)
    kern.gemm(P, N, K, a=[a], lda=[K], b=w, ldb=K, c=zg, ldc=N, bias=b2, stats=sg)
    _finish_and_compare(sg, rg, zg, N, "gemm epilogue")
    # the materialising BatchNorm+act pass with statistics of its output (y = 0.3 x + 300)
    y = torch.empty_like(x)
    ra = kern.stream_rows(P, C)
    sa = torch.zeros(ra, 2, C, dtype=torch.float64, device=DEV)
    kern.affine_act(x, torch.full((C,), 0.3, device=DEV), torch.full((C,), 300.0, device=DEV), 0,
                    None, y, P, C, sa)
    _finish_and_compare(sa, ra, y, C, "affine_act")
