"""Host vs GPU time of the graph-mode training step, plain and data-parallel (world-1
RCCL group): how long the host takes to submit the replayed graph, to enqueue the bucket
all-reduces and to prepare Adam, against the GPU time of the graph -- i.e. whether the
all-reduces can start while the backward still runs (they are enqueued only after the
replay call returns). Variants are built once and timed in alternating blocks.

    python tools/dp_host.py [--dtype bf16] [--steps 10] [--reps 3]
"""
import argparse
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "acc-unet-unext_amd"))
from accunet import model as M  # noqa: E402
from accunet.train import TrainStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}")
    g = torch.Generator().manual_seed(1000)
    x = torch.randn(16, 3, 256, 256, generator=g).to(dev)
    m = (torch.rand(16, 1, 256, 256, generator=g) < 0.3).float().to(dev)
    variants = [("plain", None), ("dp", dist.group.WORLD)]
    steps, seg = {}, {}
    for name, pg in variants:
        torch.manual_seed(0)
        model = M.VARIANTS["canonical"](3, 1, n_filts=32).to(dev).train()
        st = TrainStep(model, lr=1e-3, graph=True, precision=a.dtype, process_group=pg,
                       comm_dtype="bf16" if a.dtype == "bf16" else None)
        for _ in range(3):
            st(x, m)
        torch.cuda.synchronize()
        sg = {"replay": [], "reduce": [], "opt": [], "host": [], "graph_gpu": [], "step_gpu": []}
        ev = {}

        def timed(key, fn, sg=sg, ev=ev):
            def w(*args, **kw):
                t0 = time.perf_counter()
                if key == "replay":
                    ev["a"] = torch.cuda.Event(enable_timing=True)
                    ev["a"].record()
                r = fn(*args, **kw)
                if key == "replay":
                    ev["b"] = torch.cuda.Event(enable_timing=True)
                    ev["b"].record()
                sg[key].append(1e3 * (time.perf_counter() - t0))
                return r
            return w

        st._g.replay = timed("replay", st._g.replay)
        st.opt.step = timed("opt", st.opt.step)
        if st.dp:
            st._buckets.reduce = timed("reduce", st._buckets.reduce)
        steps[name], seg[name] = (st, ev), sg
    for _ in range(a.reps):
        for name, _pg in variants:
            st, ev = steps[name]
            sg = seg[name]
            for _ in range(a.steps):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record()
                st(x, m)
                e1.record()
                sg["host"].append(1e3 * (time.perf_counter() - t0))
                torch.cuda.synchronize()
                sg["graph_gpu"].append(ev["a"].elapsed_time(ev["b"]))
                sg["step_gpu"].append(e0.elapsed_time(e1))
    for name, _pg in variants:
        med = {k: sorted(v)[len(v) // 2] for k, v in seg[name].items() if v}
        print(name, " ".join(f"{k} {v:.2f} ms" for k, v in med.items()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
