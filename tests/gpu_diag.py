"""Diagnostic driver (GPU box): HIP model vs fp64 oracle, with the reference's own
fp32 error (fp32 oracle) as the yardstick. Prints the worst tensors by ratio.

    python tests/gpu_diag.py variant nf B H
"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.environ.get("ACCUNET_PKG_DIR", os.path.join(os.path.dirname(HERE), "acc-unet-unext_amd")))
sys.path.insert(0, HERE)
import parity_util as PU  # noqa: E402
from parity_util import O  # noqa: E402
from accunet import model as M  # noqa: E402
from accunet.loss import WeightedDiceBCE  # noqa: E402


def run_model(variant, nf, B, H):
    spec = O.param_spec(variant, 3, 1, nf)
    sd = O.det_state_dict(spec, seed=0)
    x = O.det_input((B, 3, H, H), "golden-x")
    mask = O.det_mask((B, 1, H, H), "golden-mask", p=0.4)
    r64 = PU.oracle_run(variant, sd, x, mask)
    r32 = PU.oracle_run(variant, sd, x, mask, dtype=torch.float32)
    m = M.VARIANTS[variant](3, 1, n_filts=nf)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x.cuda())
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.cuda())
    loss.backward()
    torch.cuda.synchronize()
    hip = {"out": out}
    a64 = {"out": r64[0]}
    a32 = {"out": r32[0]}
    for k, p in m.named_parameters():
        hip[k] = p.grad
        a64[k] = r64[2][k]
        a32[k] = r32[2][k]
    rows = PU.compare_vs_reference_fp32(hip, a64, a32)
    rows.sort(key=lambda r: -(r[1] / (r[2] + 1e-30)))
    print(f"== {variant} nf{nf} B{B} {H}x{H}: loss hip {loss.item():.7f} r64 {r64[1].item():.7f} "
          f"r32 {r32[1].item():.7f}")
    for r in rows[:25]:
        sc = a64[r[0]].abs().max().item()
        print("   %-42s hip %.2e ref32 %.2e ratio %6.1f  scale %.2e %s" %
              (r[0], r[1], r[2], r[1] / (r[2] + 1e-30), sc, "" if r[4] else "BAD"))
    print("   bad:", sum(1 for r in rows if not r[4]), "/", len(rows))


def run_se(C, B, H, pre):
    torch.manual_seed(0)
    se = M.ChannelSELayer(C)
    spec = [(n, tuple(t.shape)) for n, t in se.state_dict().items()]
    sd = O.det_state_dict([("s." + n, s) for n, s in spec], seed=3)
    se.load_state_dict({n[2:]: v for n, v in sd.items()})
    se = se.cuda().train()
    x = O.det_input((B, C, H, H), "se-x") * 2 + 0.5
    go = O.det_input((B, C, H, H), "se-go")
    res = {}
    for dt in (torch.float64, torch.float32):
        sdo = {n: (v.to(dt).requires_grad_(not n.endswith(PU.BUFFER_LEAVES)) if v.is_floating_point() else v.clone())
               for n, v in sd.items()}
        xr = x.detach().clone().to(dt).requires_grad_(True)
        y = O.se(xr, sdo, "s", True)
        (y * go.to(dt)).sum().backward()
        res[dt] = (y.detach(), xr.grad, {n[2:]: v.grad for n, v in sdo.items() if v.grad is not None})
    xh = x.detach().cuda().requires_grad_(True)
    y = se(xh)
    (y * go.cuda()).sum().backward()
    print(f"== SE C{C} B{B} {H}x{H}")
    hip = {"out": y, "dx": xh.grad}
    a64 = {"out": res[torch.float64][0], "dx": res[torch.float64][1]}
    a32 = {"out": res[torch.float32][0], "dx": res[torch.float32][1]}
    for n, p in se.named_parameters():
        hip[n] = p.grad
        a64[n] = res[torch.float64][2][n]
        a32[n] = res[torch.float32][2][n]
    for r in PU.compare_vs_reference_fp32(hip, a64, a32):
        print("   %-20s hip %.2e ref32 %.2e ratio %6.1f %s" % (r[0], r[1], r[2], r[1] / (r[2] + 1e-30),
                                                            "" if r[4] else "BAD"))


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "se":
        run_se(int(a[1]), int(a[2]), int(a[3]), None)
    else:
        variant = a[0] if a else "canonical"
        nf = int(a[1]) if len(a) > 1 else 8
        B = int(a[2]) if len(a) > 2 else 2
        H = int(a[3]) if len(a) > 3 else 32
        run_model(variant, nf, B, H)
