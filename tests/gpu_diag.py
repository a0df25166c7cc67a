"""Diagnostic driver (GPU box): HIP model vs fp64 oracle, prints per-check errors.

    python tests/gpu_diag.py [variant ...]
"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "acc-unet-unext_amd"))
sys.path.insert(0, HERE)
import parity_util as PU  # noqa: E402
from parity_util import O  # noqa: E402
from accunet.model import VARIANTS  # noqa: E402
from accunet.loss import WeightedDiceBCE  # noqa: E402


def run(variant, nf=8, B=2, H=32, W=32):
    spec = O.param_spec(variant, 3, 1, nf)
    sd = O.det_state_dict(spec, seed=0)
    x = O.det_input((B, 3, H, W), "golden-x")
    mask = O.det_mask((B, 1, H, W), "golden-mask", p=0.4)
    t0 = time.time()
    ref_out, ref_loss, ref_grads, ref_sd = PU.oracle_run(variant, sd, x, mask)
    t1 = time.time()
    m = VARIANTS[variant](3, 1, n_filts=nf)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x.cuda())
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.cuda())
    loss.backward()
    torch.cuda.synchronize()
    t2 = time.time()
    oerr = (out.detach().double().cpu() - ref_out).abs().max().item()
    lerr = abs(loss.item() - ref_loss.item())
    print(f"[{variant}] oracle {t1 - t0:.2f}s hip {t2 - t1:.2f}s  out max|d|={oerr:.3e} "
          f"loss {loss.item():.6f} vs {ref_loss.item():.6f} d={lerr:.2e}")
    hip_grads = {k: p.grad if p.grad is not None else torch.zeros_like(p)
                 for k, p in m.named_parameters()}
    rows = PU.compare_grads(hip_grads, ref_grads)
    bad = [r for r in rows if not r[4]]
    rows.sort(key=lambda r: -(r[1] / (r[3] + 1e-30)))
    for r in rows[:12]:
        print("   %-45s err=%.3e scale=%.3e tol=%.3e %s" % (r[0], r[1], r[2], r[3], "ok" if r[4] else "BAD"))
    print(f"   grads: {len(rows) - len(bad)}/{len(rows)} ok")
    # running stats
    msd = m.state_dict()
    worst = 0.0
    wname = ""
    for k, v in ref_sd.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            d = (msd[k].double().cpu() - v.double()).abs().max().item()
            if d > worst:
                worst, wname = d, k
        if k.endswith("num_batches_tracked"):
            assert int(msd[k]) == int(v), k
    print(f"   running stats worst |d| = {worst:.3e} ({wname})")
    # eval mode forward
    m.eval()
    with torch.no_grad():
        oe = m(x.cuda()).double().cpu()
    ref_e, _, _, _ = PU.oracle_run(variant, ref_sd, x, None, training=False)
    print(f"   eval out max|d| = {(oe - ref_e).abs().max().item():.3e}")
    return len(bad)


if __name__ == "__main__":
    vs = sys.argv[1:] or ["canonical", "script", "lite", "w"]
    nbad = 0
    for v in vs:
        nbad += run(v)
    print("TOTAL BAD", nbad)
