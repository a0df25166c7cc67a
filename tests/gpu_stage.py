"""Staged GPU bring-up (run with ACCUNET_DEBUG=1 to trace/serialise every kernel call)."""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "acc-unet-unext_amd"))
sys.path.insert(0, HERE)
from parity_util import O  # noqa: E402
from accunet.model import VARIANTS  # noqa: E402
from accunet.loss import WeightedDiceBCE  # noqa: E402


def log(msg):
    sys.stderr.write(f"=== {msg} ({time.strftime('%H:%M:%S')})\n")
    sys.stderr.flush()


variant = sys.argv[1] if len(sys.argv) > 1 else "canonical"
stages = sys.argv[2] if len(sys.argv) > 2 else "fwd,bwd"
nf = 8
spec = O.param_spec(variant, 3, 1, nf)
sd = O.det_state_dict(spec, seed=0)
x = O.det_input((2, 3, 32, 32), "golden-x").cuda()
mask = O.det_mask((2, 1, 32, 32), "golden-mask", p=0.4).cuda()
m = VARIANTS[variant](3, 1, n_filts=nf)
m.load_state_dict(sd)
m = m.cuda().train()
log("forward")
out = m(x)
torch.cuda.synchronize()
log(f"forward done {out.shape} {out.float().mean().item():.6f}")
loss = WeightedDiceBCE(0.5, 0.5)(out, mask)
torch.cuda.synchronize()
log(f"loss {loss.item():.6f}")
if "bwd" in stages:
    loss.backward()
    torch.cuda.synchronize()
    log("backward done")
