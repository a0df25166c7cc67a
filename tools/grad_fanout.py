"""Where autograd sums gradients: walk the backward graph of one canonical ACC_UNet
training forward and list every (node, output) consumed more than once (each such
output costs one gradient-accumulation add kernel per step), grouped by producer and
consumer Function, with the output's shape (recorded by forward hooks on the ops).

    python tools/grad_fanout.py [--size 256] [--batch 16]     (GPU)
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
    from accunet import ops
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = M.VARIANTS["canonical"](3, 1, n_filts=32).to(dev).train()
    x = torch.randn(a.batch, 3, a.size, a.size, device=dev)
    # shapes: wrap every autograd Function's apply to tag its outputs' grad_fn
    shapes = {}
    for name in dir(ops):
        fn = getattr(ops, name)
        if isinstance(fn, type) and issubclass(fn, torch.autograd.Function) and fn is not torch.autograd.Function:
            orig = fn.apply

            def wrapped(*args, _orig=orig, **kw):
                out = _orig(*args, **kw)
                outs = out if isinstance(out, tuple) else (out,)
                for i, o in enumerate(outs):
                    if isinstance(o, torch.Tensor) and o.grad_fn is not None:
                        shapes[(id(o.grad_fn), i)] = (tuple(o.shape), o.dtype)
                return out
            fn.apply = staticmethod(wrapped) if False else wrapped
    out = model(x)
    loss = out.float().mean()
    uses = collections.Counter()
    consumers = collections.defaultdict(list)
    seen = set()
    stack = [loss.grad_fn]
    while stack:
        n = stack.pop()
        if n is None or id(n) in seen:
            continue
        seen.add(id(n))
        for nxt, idx in n.next_functions:
            if nxt is None or type(nxt).__name__ == "AccumulateGrad":
                continue
            uses[(id(nxt), idx)] += 1
            consumers[(id(nxt), idx)].append(type(n).__name__)
            stack.append(nxt)
    names = {}
    stack = [loss.grad_fn]
    seen = set()
    while stack:
        n = stack.pop()
        if n is None or id(n) in seen:
            continue
        seen.add(id(n))
        names[id(n)] = type(n).__name__
        stack.extend(m for m, _ in n.next_functions)
    groups = collections.Counter()
    elems = collections.Counter()
    total = 0
    for k, c in uses.items():
        if c < 2:
            continue
        shp = shapes.get(k, ((), None))
        ne = 1
        for s in shp[0]:
            ne *= s
        key = (names.get(k[0], "?"), tuple(sorted(consumers[k])))
        groups[key] += c - 1
        elems[key] += (c - 1) * ne
        total += c - 1
    print(f"gradient-accumulation adds per backward: {total}")
    for key, c in sorted(groups.items(), key=lambda kv: -elems[kv[0]]):
        print(f"{c:4d} adds {elems[key] / 1e6:9.1f} M elems  producer {key[0]:<22} consumers {', '.join(key[1])}")


if __name__ == "__main__":
    main()
