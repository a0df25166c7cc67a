"""Full-width (n_filts 32, 2x3x256^2) gradient accuracy of the HIP model vs the fp64
oracle, per tensor, against two fp32 yardsticks: the single fp32 oracle run the
test uses and the max over an ensemble of fp32 runs on 2^-24-perturbed inputs
(parity_util.oracle_run_fp32_ensemble). Prints the tensors closest to the bound.

    ACCUNET_GEMM_G=1 python tools/fw_diag.py [--variant script]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import parity_util as PU  # noqa: E402
from parity_util import O  # noqa: E402
from accunet import model as M  # noqa: E402
from accunet.loss import WeightedDiceBCE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="script")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    torch.set_num_threads(16)
    spec = O.param_spec(a.variant, 3, 1, 32)
    sd = O.det_state_dict(spec, seed=7)
    x = O.det_input((2, 3, 256, 256), "fw-x2")
    mask = O.det_mask((2, 1, 256, 256), "fw-mask", p=0.3)
    m = M.VARIANTS[a.variant](3, 1, n_filts=32)
    m.load_state_dict(sd)
    m = m.cuda().train()
    out = m(x.cuda())
    loss = WeightedDiceBCE(0.5, 0.5)(out, mask.cuda())
    loss.backward()
    torch.cuda.synchronize()
    ref_out, _, ref_grads, _ = PU.oracle_run(a.variant, sd, x, mask)
    r32_out, _, r32_grads, _ = PU.oracle_run(a.variant, sd, x, mask, dtype=torch.float32)
    ens = PU.oracle_run_fp32_ensemble(a.variant, sd, x, mask)
    hip, r64, r32 = {"out": out}, {"out": ref_out}, {"out": r32_out}
    for k, p in m.named_parameters():
        hip["grad:" + k] = p.grad if p.grad is not None else torch.zeros_like(p)
        r64["grad:" + k] = ref_grads[k]
        r32["grad:" + k] = r32_grads[k]
    single = PU.compare_vs_reference_fp32(hip, r64, r32)
    both = PU.compare_vs_reference_fp32(hip, r64, r32, ref32_extra=ens)
    ebe = {r[0]: r for r in both}
    keys = list(hip)
    print("global rel err: hip", PU.global_rel_err(hip, r64, keys), "fp32",
          PU.global_rel_err(r32, r64, keys))
    single.sort(key=lambda r: -r[1] / max(r[2], 1e-30))
    print(f"{'tensor':48s} {'err_hip':>10s} {'err_fp32':>10s} {'ratio':>6s} {'err_ens':>10s} {'ratio_ens':>9s}")
    for r in single[:a.top]:
        e = ebe[r[0]]
        print(f"{r[0]:48s} {r[1]:10.3e} {r[2]:10.3e} {r[1] / max(r[2], 1e-30):6.2f} {e[2]:10.3e} "
              f"{r[1] / max(e[2], 1e-30):9.2f}")


if __name__ == "__main__":
    main()
