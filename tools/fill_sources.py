"""Attribute the small ATen kernels of one eager ACC_UNet training step (zero fills,
gradient-accumulation adds, copies) to the Python stack that caused them, with
torch.profiler (with_stack). Autograd's own adds appear under the backward with no
Python frame; their input shapes are listed instead.

    python tools/fill_sources.py [--batch 16] [--size 256]       (GPU)
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    from accunet import model as M
    from accunet.train import TrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = M.VARIANTS["canonical"](3, 1, n_filts=32).to(dev).train()
    step = TrainStep(model, lr=1e-3)
    x = torch.randn(a.batch, 3, a.size, a.size, device=dev)
    m = (torch.rand(a.batch, 1, a.size, a.size, device=dev) < 0.3).float()
    step(x, m)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        step(x, m)
        torch.cuda.synchronize()
    want = ("aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::copy_")
    by = collections.Counter()
    for ev in prof.events():
        if ev.name not in want:
            continue
        stack = [s for s in (ev.stack or []) if "accunet" in s or "tools/" in s]
        site = " < ".join(s.split("/")[-1] for s in stack[:3]) or "(autograd engine)"
        shp = str(ev.input_shapes[0]) if ev.input_shapes else ""
        by[(ev.name, site, shp if site == "(autograd engine)" else "")] += 1
    for (name, site, shp), c in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"{c:5d}  {name:<12} {site} {shp}")


if __name__ == "__main__":
    main()
