"""Diagnostic (not a test): bf16 HIP model vs fp64 oracle vs bf16-emulated oracle."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
import torch
import parity_util as PU
from parity_util import O
from accunet import model as M
from accunet.loss import WeightedDiceBCE

BF = torch.bfloat16
for variant in sys.argv[1:] or ["script", "canonical"]:
    nf, B, S = 8, 4, 64
    sd = O.det_state_dict(O.param_spec(variant, 3, 1, nf), seed=0)
    x = O.det_input((B, 3, S, S), "golden-x")
    mask = O.det_mask((B, 1, S, S), "golden-mask", p=0.4)
    o64, l64, g64, _ = PU.oracle_run(variant, sd, x, mask)
    with O.storage_rounding(BF):
        oe, le, ge, _ = PU.oracle_run(variant, sd, x, mask)
    res = {}
    for prec in ("fp32", "bf16"):
        m = M.VARIANTS[variant](3, 1, n_filts=nf, precision=prec)
        m.load_state_dict(sd)
        m = m.cuda().train()
        out = m(x.cuda())
        loss = WeightedDiceBCE(0.5, 0.5)(out, mask.cuda())
        loss.backward()
        g = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in m.named_parameters()}
        res[prec] = (out.detach().double().cpu(), float(loss), g)
    keys = list(g64)
    print(f"== {variant}: loss64 {float(l64):.6f} emu {float(le):.6f} ({float(le)-float(l64):+.2e})")
    for prec, (o, l, g) in res.items():
        d = o - o64
        print(f"  hip {prec}: loss {l:.6f} ({l-float(l64):+.2e}) out max {d.abs().max():.3e} "
              f"mean {d.abs().mean():.3e} bias {d.mean():+.3e} grad rel {PU.global_rel_err(g, g64, keys):.3e}")
    d = oe - o64
    print(f"  emu     : out max {d.abs().max():.3e} mean {d.abs().mean():.3e} bias {d.mean():+.3e} "
          f"grad rel {PU.global_rel_err(ge, g64, keys):.3e}  |o64| max {o64.abs().max():.2f}")
    # per-sample mean output
    ob = res["bf16"][0]
    print("  per-sample mean out: 64", [round(float(v), 4) for v in o64.mean((1, 2, 3))],
          "bf16", [round(float(v), 4) for v in ob.mean((1, 2, 3))],
          "emu", [round(float(v), 4) for v in oe.mean((1, 2, 3))])

# rounding mode of the kernels' fp32 -> bf16 conversion vs torch (RNE)
from accunet import kern
xs = torch.randn(1 << 20, device="cuda") * 3
y = torch.empty(1 << 20, device="cuda", dtype=BF)
kern.permute4(xs.view(1, 1, 1, -1), y.view(1, 1, 1, -1), (1, 1, 1, 1 << 20), (0, 0, 0, 1))
ref = xs.to(BF)
print("kernel bf16 rounding == torch RNE:", bool(torch.equal(y, ref)),
      "mismatches", int((y != ref).sum()), "mean(y - x)", float((y.double() - xs.double()).mean()))
