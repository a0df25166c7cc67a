"""GEMM engine parity (fp32 MFMA) against float64 torch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from accunet import kern  # noqa: E402
from accunet import _lib  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30)).item()


@pytest.mark.parametrize("M,N,K", [(4096, 128, 96), (1000, 64, 45), (777, 32, 18),
                                   (2048, 9, 3), (300, 200, 256), (64, 512, 1536)])
def test_row_nt_bias_stats(M, N, K):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=DEV)
    Wt = torch.randn(N, K, device=DEV)
    b = torch.randn(N, device=DEV)
    C = torch.empty(M, N, device=DEV)
    rows = kern.gemm_stats_rows(M, N, K)
    st = torch.zeros(rows, 2, N, device=DEV, dtype=torch.float64)
    kern.gemm(M, N, K, a=[A], lda=[K], b=Wt, ldb=K, c=C, ldc=N, bias=b, stats=st)
    ref = A.double() @ Wt.double().t() + b.double()
    assert rel(C, ref) < 1e-5
    s = st.double().sum(0)
    assert torch.allclose(s[0], ref.sum(0), rtol=1e-4, atol=1e-2)
    assert torch.allclose(s[1], (ref * ref).sum(0), rtol=1e-4, atol=1e-1)


def test_row_nt_prologue_multisrc_ups():
    torch.manual_seed(1)
    B, H, W = 2, 16, 32
    P = B * H * W
    K1, K2 = 32, 16
    N = 48
    A1 = torch.randn(P, K1, device=DEV)
    A2 = torch.randn(P, 40, device=DEV)[:, 8:24]  # column slice with ld=40
    Wt = torch.randn(N, K1 + K2, device=DEV)
    g2 = torch.randn(B * (H // 2) * (W // 2), N, device=DEV)
    g4 = torch.randn(B * (H // 4) * (W // 4), 64, device=DEV)
    C = torch.empty(P, N, device=DEV)
    A2full = A2.contiguous()
    base = torch.randn(P, 40, device=DEV)
    base[:, 8:24] = A2full
    kern.gemm(P, N, K1 + K2, a=[A1, base], lda=[K1, 40], a_offsets=[0, 8], kbeg=[0, K1, K1 + K2],
              b=Wt, ldb=K1 + K2, c=C, ldc=N, H=H, W=W,
              ups=[(g2, N, 1, 0), (g4, 64, 2, 16)])
    X = torch.cat([A1, A2full], 1).double()
    ref = X @ Wt.double().t()
    up2 = g2.view(B, H // 2, W // 2, N).repeat_interleave(2, 1).repeat_interleave(2, 2).reshape(P, N)
    up4 = g4[:, 16:16 + N].reshape(B, H // 4, W // 4, N).repeat_interleave(4, 1).repeat_interleave(4, 2).reshape(P, N)
    ref = ref + up2.double() + up4.double()
    assert rel(C, ref) < 1e-5

    # prologue (affine + lrelu) on A
    sc = torch.rand(K1, device=DEV) + 0.5
    sh = torch.randn(K1, device=DEV)
    C2 = torch.empty(P, N, device=DEV)
    kern.gemm(P, N, K1, a=[A1], lda=[K1], b=Wt, ldb=K1 + K2, c=C2, ldc=N,
              pro_a=_lib.PRO_AFFINE_LRELU, a_scale=sc, a_shift=sh)
    Xp = F.leaky_relu(A1.double() * sc.double() + sh.double(), 0.01)
    assert rel(C2, Xp @ Wt[:, :K1].double().t()) < 1e-5


@pytest.mark.parametrize("P,N,K", [(5000, 96, 32), (4096, 3, 32), (1024, 1536, 512)])
def test_row_nn_dgrad(P, N, K):
    # dX[P,K] = dZ[P,N] @ W[N,K]  -> GEMM M=P, N=K, K=N with B = W as [K][N] (NN)
    torch.manual_seed(2)
    dZ = torch.randn(P, N, device=DEV)
    Wt = torch.randn(N, K, device=DEV)
    dX = torch.empty(P, K, device=DEV)
    kern.gemm(P, K, N, a=[dZ], lda=[N], b=Wt, ldb=K, bmode=_lib.BMODE_NN, c=dX, ldc=K)
    assert rel(dX, dZ.double() @ Wt.double()) < 1e-5


@pytest.mark.parametrize("P,Co,Ci,pro", [(65536, 96, 32, 0), (20000, 32, 96, 2), (4096, 512, 1536, 1),
                                         (3000, 9, 3, 0)])
def test_col_nn_wgrad_splitk(P, Co, Ci, pro):
    torch.manual_seed(3)
    dZ = torch.randn(P, Co, device=DEV)
    X = torch.randn(P, Ci, device=DEV)
    sc = torch.rand(Ci, device=DEV) + 0.5
    sh = torch.randn(Ci, device=DEV)
    dW = torch.empty(Co, Ci, device=DEV)
    kern.gemm(Co, Ci, P, a=[dZ], lda=[Co], amode=_lib.AMODE_COL, b=X, ldb=Ci,
              bmode=_lib.BMODE_NN, c=dW, ldc=Ci, pro_b=pro,
              b_scale=sc if pro else None, b_shift=sh if pro else None, allow_split=True)
    Xd = X.double()
    if pro == 1:
        Xd = Xd * sc.double() + sh.double()
    elif pro == 2:
        Xd = F.leaky_relu(Xd * sc.double() + sh.double(), 0.01)
    ref = dZ.double().t() @ Xd
    assert rel(dW, ref) < 1e-5


@pytest.mark.parametrize("M,N,K,ldc,off", [(256, 1152, 131072, 1152, 0), (96, 290, 200003, 301, 7),
                                           (128, 640, 65536, 1000, 333), (200, 136, 40000, 136, 0)])
def test_splitk_many_slabs_into_slice(M, N, K, ldc, off):
    """Tiled split-K weight gradients (more than 3 output tiles, tens of slabs): quad and
    non-quad N, output into a column slice of a wider row (unaligned, columns outside the
    slice untouched), ragged M; bitwise reproducible (fixed slab order); against fp64."""
    torch.manual_seed(6)
    A = torch.randn(K, M, device=DEV)
    B = torch.randn(K, N, device=DEV)
    C = torch.full((M + 1, ldc), 7.0, device=DEV)  # (one spare row: the slice is offset)

    def run(c):
        kern.gemm(M, N, K, a=[A], lda=[M], amode=_lib.AMODE_COL, b=B, ldb=N,
                  bmode=_lib.BMODE_NN, c=c, ldc=ldc, c_offset=off, allow_split=True)
    run(C)
    got = torch.as_strided(C.view(-1)[off:], (M, N), (ldc, 1))
    ref = A.double().t() @ B.double()
    assert rel(got, ref) < 2e-5
    mask = torch.ones((M + 1) * ldc, dtype=torch.bool, device=DEV)
    idx = off + torch.arange(M, device=DEV)[:, None] * ldc + torch.arange(N, device=DEV)[None, :]
    mask[idx.reshape(-1)] = False
    assert bool((C.view(-1)[mask] == 7.0).all())
    C2 = torch.full((M + 1, ldc), 7.0, device=DEV)
    run(C2)
    assert torch.equal(C, C2)


@pytest.mark.parametrize("B,H,W,Ci,Co", [(2, 32, 32, 32, 32), (1, 16, 64, 64, 64), (2, 8, 8, 256, 256)])
def test_conv3x3_fwd_dgrad_wgrad(B, H, W, Ci, Co):
    torch.manual_seed(4)
    x = torch.randn(B, Ci, H, W, device=DEV, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Co, Ci, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
    bias = torch.randn(Co, device=DEV, dtype=torch.float64)
    y = F.conv2d(x, w, bias, padding=1)
    gy = torch.randn_like(y)
    y.backward(gy)
    P = B * H * W
    xn = x.detach().permute(0, 2, 3, 1).reshape(P, Ci).float().contiguous()
    wr = w.detach().permute(0, 2, 3, 1).reshape(Co, 9 * Ci).float().contiguous()  # [co][tap][ci]
    out = torch.empty(P, Co, device=DEV)
    kern.gemm(P, Co, 9 * Ci, a=[xn], lda=[Ci], amode=_lib.AMODE_SHIFT3, b=wr, ldb=9 * Ci,
              c=out, ldc=Co, bias=bias.float(), H=H, W=W, cin=Ci)
    ref = y.detach().permute(0, 2, 3, 1).reshape(P, Co)
    assert rel(out, ref) < 1e-5
    # dgrad: conv with flipped, transposed weights W'[ci][tap'][co] = W[co][ci][8-tap']
    gyn = gy.permute(0, 2, 3, 1).reshape(P, Co).float().contiguous()
    wf = w.detach().flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co).float().contiguous()
    dx = torch.empty(P, Ci, device=DEV)
    kern.gemm(P, Ci, 9 * Co, a=[gyn], lda=[Co], amode=_lib.AMODE_SHIFT3, b=wf, ldb=9 * Co,
              c=dx, ldc=Ci, H=H, W=W, cin=Co)
    assert rel(dx, x.grad.permute(0, 2, 3, 1).reshape(P, Ci)) < 1e-5
    # wgrad: dW[co][tap][ci] = sum_p gy[p,co] x[shift_tap(p), ci]
    dw = torch.empty(Co, 9 * Ci, device=DEV)
    kern.gemm(Co, 9 * Ci, P, a=[gyn], lda=[Co], amode=_lib.AMODE_COL, b=xn, ldb=Ci,
              bmode=_lib.BMODE_NN_SHIFT3, c=dw, ldc=9 * Ci, H=H, W=W, cin=Ci, allow_split=True)
    refw = w.grad.permute(0, 2, 3, 1).reshape(Co, 9 * Ci)
    assert rel(dw, refw) < 1e-5


@pytest.mark.parametrize("B,H,W,Co", [(2, 128, 128, 32), (4, 32, 256, 32), (16, 256, 256, 32)])
def test_conv3x3_halo_kernel_c32(B, H, W, Co):
    """The halo-tile 3x3 kernel (csrc/conv3x3.hip; 32 input channels, image rows of whole
    128-pixel tiles: the first ResPath level): forward with bias and the fp64 statistics
    rows (one per 128-pixel tile, as the implicit GEMM's), the data gradient
    accumulated in place onto C (the residual's gradient) and the weight gradient,
    against float64 torch."""
    torch.manual_seed(14)
    Ci = 32
    x = torch.randn(B, Ci, H, W, device=DEV, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Co, Ci, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True) * 0.1
    w.retain_grad()
    bias = torch.randn(Co, device=DEV, dtype=torch.float64)
    y = F.conv2d(x, w, bias, padding=1)
    gy = torch.randn_like(y)
    y.backward(gy)
    P = B * H * W
    xn = x.detach().permute(0, 2, 3, 1).reshape(P, Ci).float().contiguous()
    wr = w.detach().permute(0, 2, 3, 1).reshape(Co, 9 * Ci).float().contiguous()
    out = torch.empty(P, Co, device=DEV)
    rows = kern.gemm_stats_rows(P, Co, 9 * Ci, _lib.AMODE_SHIFT3, _lib.BMODE_NT, Ci)
    # >= 256 tiles of 128x32: the engine's tile there and the halo kernel's (fewer run
    # 64x64 tiles on the engine, pick_tile)
    assert rows == P // 128
    st = torch.zeros(rows, 2, Co, device=DEV, dtype=torch.float64)
    kern.gemm(P, Co, 9 * Ci, a=[xn], lda=[Ci], amode=_lib.AMODE_SHIFT3, b=wr, ldb=9 * Ci,
              c=out, ldc=Co, bias=bias.float(), stats=st, H=H, W=W, cin=Ci)
    ref = y.detach().permute(0, 2, 3, 1).reshape(P, Co)
    assert rel(out, ref) < 1e-5
    s = st.sum(0)
    o = out.double()
    assert torch.allclose(s[0], o.sum(0), rtol=1e-9, atol=1e-6)
    assert torch.allclose(s[1], (o * o).sum(0), rtol=1e-9, atol=1e-6)
    # data gradient (Co = 32 only: the halo kernel's input is 32-channel) onto C in place
    if Co == 32:
        gyn = gy.permute(0, 2, 3, 1).reshape(P, Co).float().contiguous()
        wf = w.detach().flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co).float().contiguous()
        r = torch.randn(P, Ci, device=DEV)
        dx = r.clone()
        kern.gemm(P, Ci, 9 * Co, a=[gyn], lda=[Co], amode=_lib.AMODE_SHIFT3, b=wf, ldb=9 * Co,
                  c=dx, ldc=Ci, H=H, W=W, cin=Co, ups=[(dx, Ci, 0, 0)])
        refx = x.grad.permute(0, 2, 3, 1).reshape(P, Ci) + r.double()
        assert rel(dx, refx) < 1e-5
        # weight gradient (its own halo kernel: one slab per workgroup, split-K reduce)
        def wgrad():
            dw = torch.empty(Co, 9 * Ci, device=DEV)
            kern.gemm(Co, 9 * Ci, P, a=[gyn], lda=[Co], amode=_lib.AMODE_COL, b=xn, ldb=Ci,
                      bmode=_lib.BMODE_NN_SHIFT3, c=dw, ldc=9 * Ci, H=H, W=W, cin=Ci,
                      allow_split=True)
            return dw
        dw = wgrad()
        assert rel(dw, w.grad.permute(0, 2, 3, 1).reshape(Co, 9 * Ci)) < 1e-5
        assert torch.equal(dw, wgrad())  # fixed slab order: bitwise reproducible


def test_conv3x3_halo_matches_engine_bitwise(tmp_path):
    """The halo-tile forward / data-gradient kernels (fp32 and bf16 activation mode) use
    the implicit GEMM's MFMA, k pairing, k order and epilogue, so their outputs and fp64
    statistics rows are bit-identical to the engine's (ACCUNET_CONV3_HALO=0), each run in
    a child process (the knob is read once per process)."""
    import os
    import subprocess
    import sys
    outs = {}
    for v in ("1", "0"):
        env = dict(os.environ, ACCUNET_CONV3_HALO=v)
        path = tmp_path / f"c3_{v}.pt"
        subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "conv3x3_worker.py"),
                        str(path)], env=env, check=True, timeout=240)
        outs[v] = torch.load(path, weights_only=True)
    # the knob-on run really took the halo kernels (every launch), the knob-off run never
    assert int(outs["1"].pop("halo_launches")) == 8
    assert int(outs["0"].pop("halo_launches")) == 0
    for k in outs["1"]:
        assert torch.equal(outs["1"][k], outs["0"][k]), k


@pytest.mark.parametrize("B,H,W,Ci,Co", [(2, 24, 128, 64, 64), (1, 8, 256, 32, 96),
                                         (2, 6, 128, 128, 64), (16, 128, 128, 64, 64)])
def test_conv3x3_halo_wgrad_channel_blocks(B, H, W, Ci, Co):
    """The halo weight-gradient kernel on wider layers (32x32 channel blocks per
    workgroup, each writing its part of the [Co][9 Ci] slab): the second ResPath level
    (16 x 128^2 x 64) and non-square channel counts, against float64 torch; bitwise
    reproducible."""
    torch.manual_seed(15)
    x = torch.randn(B, Ci, H, W, device=DEV, dtype=torch.float64)
    gy = torch.randn(B, Co, H, W, device=DEV, dtype=torch.float64)
    w = torch.zeros(Co, Ci, 3, 3, device=DEV, dtype=torch.float64, requires_grad=True)
    F.conv2d(x, w, padding=1).backward(gy)
    P = B * H * W
    xn = x.permute(0, 2, 3, 1).reshape(P, Ci).float().contiguous()
    gyn = gy.permute(0, 2, 3, 1).reshape(P, Co).float().contiguous()

    def wgrad():
        dw = torch.empty(Co, 9 * Ci, device=DEV)
        kern.gemm(Co, 9 * Ci, P, a=[gyn], lda=[Co], amode=_lib.AMODE_COL, b=xn, ldb=Ci,
                  bmode=_lib.BMODE_NN_SHIFT3, c=dw, ldc=9 * Ci, H=H, W=W, cin=Ci,
                  allow_split=True)
        return dw
    lib = _lib.load()
    n0 = lib.accunet_conv3x3_halo_launches(1)
    dw = wgrad()
    assert lib.accunet_conv3x3_halo_launches(1) == n0 + 1  # the halo weight-gradient kernel ran
    assert rel(dw, w.grad.permute(0, 2, 3, 1).reshape(Co, 9 * Ci)) < 1e-5
    assert torch.equal(dw, wgrad())


@pytest.mark.parametrize("M,N,K,lda,pro_b", [(32, 32, 1 << 20, 32, 0), (32, 32, 100003, 48, 1),
                                             (32, 96, 40000, 64, 2), (96, 32, 65536, 96, 0),
                                             (64, 32, 20000, 80, 2), (32, 64, 16384, 32, 1),
                                             (64, 192, 20000, 80, 2)])
def test_skinny_weight_gradient_path(M, N, K, lda, pro_b):
    """csrc/gemm_skinny.hip: AMODE_COL x BMODE_NN with small M, N (multiples of 32, at
    most 3 tiles; the last case takes the tiled path) and K >= 16384 (the 1x1-conv weight gradients over a batch of
    pixels), optional affine(+LeakyReLU) prologue on B's columns, ragged K, lda > M.
    Also bit-reproducible run to run (fixed reduction order)."""
    torch.manual_seed(3)
    A = torch.randn(K, lda, device=DEV)
    B = torch.randn(K, N, device=DEV)
    sc = torch.rand(N, device=DEV) + 0.5
    sh = torch.randn(N, device=DEV) * 0.2
    C = torch.empty(M, N, device=DEV)
    kw = {}
    if pro_b:
        kw = dict(pro_b=pro_b, b_scale=sc, b_shift=sh)
    kern.gemm(M, N, K, a=[A], lda=[lda], amode=_lib.AMODE_COL, b=B, ldb=N, bmode=_lib.BMODE_NN,
              c=C, ldc=N, allow_split=True, **kw)
    Bd = B.double()
    if pro_b:
        Bd = Bd * sc.double() + sh.double()
        if pro_b == 2:
            Bd = torch.where(Bd > 0, Bd, 0.01 * Bd)
    ref = A[:, :M].double().t() @ Bd
    assert rel(C, ref) < 2e-5
    C2 = torch.empty_like(C)
    kern.gemm(M, N, K, a=[A], lda=[lda], amode=_lib.AMODE_COL, b=B, ldb=N, bmode=_lib.BMODE_NN,
              c=C2, ldc=N, allow_split=True, **kw)
    assert torch.equal(C, C2)


@pytest.mark.parametrize("M,N,K", [(9, 3, 100000), (48, 40, 50000), (16, 27, 65536)])
def test_skinny_masked_edges(M, N, K):
    """Skinny path with M, N not multiples of 32 (edge tiles masked)."""
    torch.manual_seed(4)
    A = torch.randn(K, M, device=DEV)
    B = torch.randn(K, N, device=DEV)
    C = torch.empty(M, N, device=DEV)
    kern.gemm(M, N, K, a=[A], lda=[M], amode=_lib.AMODE_COL, b=B, ldb=N, bmode=_lib.BMODE_NN,
              c=C, ldc=N, allow_split=True)
    assert rel(C, A.double().t() @ B.double()) < 2e-5


@pytest.mark.parametrize("Bn,H,W,Co,Ci", [(8, 64, 64, 16, 3), (4, 48, 40, 32, 1), (2, 128, 96, 24, 2),
                                           (4, 64, 96, 32, 32)])
def test_skinny_shift3_weight_gradient(Bn, H, W, Co, Ci):
    """Skinny path for the 3x3 weight gradient (BMODE_NN_SHIFT3, <= 3 output tiles):
    dW[co][tap*Ci + ci] = sum_p dZ[p][co] * X[shift_tap(p)][ci] vs torch's conv2d
    weight gradient."""
    torch.manual_seed(5)
    P = Bn * H * W
    X = torch.randn(Bn, H, W, Ci, device=DEV)
    dZ = torch.randn(Bn, H, W, Co, device=DEV)
    C = torch.empty(Co, 9 * Ci, device=DEV)
    kern.gemm(Co, 9 * Ci, P, a=[dZ], lda=[Co], amode=_lib.AMODE_COL, b=X, ldb=Ci,
              bmode=_lib.BMODE_NN_SHIFT3, c=C, ldc=9 * Ci, H=H, W=W, cin=Ci, allow_split=True)
    xd = X.double().permute(0, 3, 1, 2).cpu()
    gd = dZ.double().permute(0, 3, 1, 2).cpu()
    wref = torch.nn.grad.conv2d_weight(xd, (Co, Ci, 3, 3), gd, padding=1)  # [co][ci][kh][kw]
    ref = wref.permute(0, 2, 3, 1).reshape(Co, 9 * Ci)  # [co][tap][ci]
    assert rel(C.cpu(), ref) < 2e-5


# ---------------------------------------------------------------------------
# The shape-gated paths only the full-size model reaches:
#   * K <= 64 && M >= 65536 small-K tiles (gemm_run.hip pick_tile) with the fused
#     HANCLayer pyramid backward (EPI_PYR) and BatchNorm-backward statistics
#     (EPI_BNB) epilogues, at the HANC x-branch data-gradient shapes of cnv12/cnv92
#     (1x1 GEMM P x 96 x 32) and cnv22/cnv82 (P x 192 x 64);
#   * the "< 128 output tiles -> 64x64 tiles" rule (16^2 / 32^2 levels);
#   * the skinny split-K weight gradient at cnv12's real K = 16 * 256^2 pixels.
# ---------------------------------------------------------------------------
def _pyr_bnb_reference(dZ, Wp, C, B, H, W, dP2, dP4, mk2, mk4, z, st, act):
    """fp64: dA = dZ @ Wp[:, :C] + pyramid backward; BN-backward partial sums."""
    P = B * H * W
    dA = dZ.double() @ Wp[:, :C].double()
    h = torch.arange(H, device=dZ.device).view(1, H, 1, 1)
    w = torch.arange(W, device=dZ.device).view(1, 1, W, 1)
    pos2 = ((h & 1) * 2 + (w & 1)).expand(B, H, W, 1)
    pos4 = ((h & 3) * 4 + (w & 3)).expand(B, H, W, 1)

    def up(t, f):
        return t.repeat_interleave(f, 1).repeat_interleave(f, 2)
    d2 = dP2.double().view(B, H // 2, W // 2, 2 * C)
    g = up(d2[..., :C], 2) * 0.25 + up(d2[..., C:], 2) * (up(mk2.view(B, H // 2, W // 2, C).long(), 2) == pos2)
    if dP4 is not None:
        d4 = dP4.double().view(B, H // 4, W // 4, 2 * C)
        g = g + up(d4[..., :C], 4) / 16.0 + up(d4[..., C:], 4) * (
            up(mk4.view(B, H // 4, W // 4, C).long(), 4) == pos4)
    dA = dA + g.reshape(P, C)
    zd = z.double()
    pre = zd * st[2].double() + st[3].double()
    gg = dA * torch.where(pre > 0, 1.0, 0.01) if act == _lib.ACT_LRELU else dA
    t2 = gg * (zd - st[0].double())
    return dA, gg.sum(0), t2.sum(0), gg.abs().sum(0), t2.abs().sum(0)


@pytest.mark.parametrize("B,H,W,C,N,k", [(2, 256, 256, 96, 32, 3), (4, 128, 128, 192, 64, 3),
                                         (4, 128, 128, 96, 32, 2)])
def test_hanc_dgrad_pyramid_bnb_epilogue_full_size(B, H, W, C, N, k):
    torch.manual_seed(6)
    P = B * H * W
    J = 2 * k - 1
    dZ = torch.randn(P, N, device=DEV)
    Wp = torch.randn(N, J * C, device=DEV) * 0.2
    dP2 = torch.randn(P // 4, 2 * C, device=DEV)
    mk2 = torch.randint(0, 4, (P // 4, C), device=DEV, dtype=torch.uint8)
    mk2[::7] = 255  # windows without a maximum (NaN input): no max routing
    dP4 = mk4 = None
    if k == 3:
        dP4 = torch.randn(P // 16, 2 * C, device=DEV)
        mk4 = torch.randint(0, 16, (P // 16, C), device=DEV, dtype=torch.uint8)
    z = torch.randn(P, C, device=DEV)
    st = torch.stack([torch.randn(C), torch.rand(C) + 0.5, torch.rand(C) + 0.5,
                      torch.randn(C) * 0.3]).float().to(DEV)
    R = kern.gemm_stats_rows(P, C, N)
    part = torch.empty(R, 2, C, device=DEV, dtype=torch.float64)
    dA = torch.empty(P, C, device=DEV)
    kern.gemm(P, C, N, a=[dZ], lda=[N], b=Wp, ldb=J * C, bmode=_lib.BMODE_NN, c=dA, ldc=C,
              H=H, W=W, pyr=(dP2, dP4, mk2, mk4), stats=part, bnb=(z, st, _lib.ACT_LRELU))
    ref, s1, s2, a1, a2 = _pyr_bnb_reference(dZ, Wp, C, B, H, W, dP2, dP4, mk2, mk4, z, st,
                                             _lib.ACT_LRELU)
    assert rel(dA, ref) < 1e-5
    tot = part.sum(0)
    # fp32 g per element (relative rounding ~6e-8), summed in fp64
    assert bool(((tot[0] - s1).abs() <= 1e-6 * a1 + 1e-9).all())
    assert bool(((tot[1] - s2).abs() <= 1e-6 * a2 + 1e-9).all())
    # deterministic: same bits on a second launch
    dA2 = torch.empty_like(dA)
    part2 = torch.empty_like(part)
    kern.gemm(P, C, N, a=[dZ], lda=[N], b=Wp, ldb=J * C, bmode=_lib.BMODE_NN, c=dA2, ldc=C,
              H=H, W=W, pyr=(dP2, dP4, mk2, mk4), stats=part2, bnb=(z, st, _lib.ACT_LRELU))
    assert torch.equal(dA, dA2) and torch.equal(part, part2)


@pytest.mark.parametrize("P,N,K", [(131072, 96, 32), (65536, 64, 64), (262144, 32, 16)])
def test_small_k_dgrad_full_size(P, N, K):
    """K <= 64, M >= 65536: the small-K tile choice, plain data gradient."""
    torch.manual_seed(7)
    dZ = torch.randn(P, K, device=DEV)
    Wt = torch.randn(K, N, device=DEV)
    dX = torch.empty(P, N, device=DEV)
    kern.gemm(P, N, K, a=[dZ], lda=[K], b=Wt, ldb=N, bmode=_lib.BMODE_NN, c=dX, ldc=N)
    assert rel(dX, dZ.double() @ Wt.double()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(4096, 256, 512), (4096, 128, 1024), (1024, 512, 1536)])
def test_few_tiles_rule_with_prologue_bias_stats(M, N, K):
    """< 128 output tiles of the default size -> 64x64 tiles (16^2 / 32^2 levels), with
    the affine+LeakyReLU prologue, bias and C statistics of the forward GEMMs."""
    torch.manual_seed(8)
    A = torch.randn(M, K, device=DEV)
    Wt = torch.randn(N, K, device=DEV) * 0.1
    b = torch.randn(N, device=DEV)
    sc = torch.rand(K, device=DEV) + 0.5
    sh = torch.randn(K, device=DEV)
    C = torch.empty(M, N, device=DEV)
    rows = kern.gemm_stats_rows(M, N, K)
    st = torch.zeros(rows, 2, N, device=DEV, dtype=torch.float64)
    kern.gemm(M, N, K, a=[A], lda=[K], b=Wt, ldb=K, c=C, ldc=N, bias=b,
              pro_a=_lib.PRO_AFFINE_LRELU, a_scale=sc, a_shift=sh, stats=st)
    X = F.leaky_relu(A.double() * sc.double() + sh.double(), 0.01)
    ref = X @ Wt.double().t() + b.double()
    assert rel(C, ref) < 1e-5
    s = st.sum(0)
    assert torch.allclose(s[0], ref.sum(0), rtol=1e-6, atol=1e-6 * ref.abs().sum().item())
    assert torch.allclose(s[1], (ref * ref).sum(0), rtol=1e-6)


@pytest.mark.parametrize("M,N,lda,pro_b", [(96, 32, 96, 0), (32, 96, 32, 2), (32, 32, 32, 1)])
def test_skinny_weight_gradient_cnv12_shapes(M, N, lda, pro_b):
    """cnv12's 1x1 weight gradients at the bench batch: K = 16 * 256 * 256 pixels
    (conv1 96x32, hnc.cnv x-branch 32x96 with the norm2 prologue, conv3 32x32)."""
    K = 16 * 256 * 256
    torch.manual_seed(9)
    A = torch.randn(K, lda, device=DEV)
    B = torch.randn(K, N, device=DEV)
    sc = torch.rand(N, device=DEV) + 0.5
    sh = torch.randn(N, device=DEV) * 0.2
    C = torch.empty(M, N, device=DEV)
    kw = dict(pro_b=pro_b, b_scale=sc, b_shift=sh) if pro_b else {}
    kern.gemm(M, N, K, a=[A], lda=[lda], amode=_lib.AMODE_COL, b=B, ldb=N, bmode=_lib.BMODE_NN,
              c=C, ldc=N, allow_split=True, **kw)
    Bd = B.double()
    if pro_b:
        Bd = Bd * sc.double() + sh.double()
        if pro_b == 2:
            Bd = torch.where(Bd > 0, Bd, 0.01 * Bd)
    ref = A[:, :M].double().t() @ Bd
    assert rel(C, ref) < 2e-5
