"""Worker for tests/test_dist_gpu.py::test_rccl_world1_graph_buckets: the RCCL branch
of the graph-mode data-parallel step on the box's one GPU.

Launched by torch.distributed.run with one process and ACCUNET_DIST_BACKEND=nccl, so
the process group is RCCL (torch's "nccl" backend on ROCm). TrainStep(graph=True,
process_group=WORLD, bucket_mb=0.25) takes the data-parallel path even at world 1
(accunet/train.py: an explicit process group selects it): ~16 event-gated buckets,
each all-reduced (AVG) by RCCL on the side stream behind its in-graph event
(_GraphBuckets.reduce, nccl branch), then the fused Adam reads the flat buffer. At
world 1 RCCL's AVG is an identity, so after 3 steps the parameters must equal, bit
for bit, those of the plain world-1 graph step (no process group, no buckets) on the
same data -- in fp32 and in bf16 storage. With the bf16 wire (comm_dtype="bf16", the
bench default for --dtype bf16) every bucket travels as bf16 and is widened back on the
side stream after its reduce: at world 1 the gradient Adam reads must be the graph's
fp32 gradient rounded to bf16 and widened, bit for bit, for every parameter.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import accunet_oracle as O  # noqa: E402
from accunet.model import ACC_UNet  # noqa: E402
from accunet.train import TrainStep  # noqa: E402


def flat_params(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def run(sd, data, dev, pg, prec):
    m = ACC_UNet(3, 1, n_filts=8)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    kw = dict(process_group=pg, bucket_mb=0.25) if pg is not None else {}
    step = TrainStep(m, lr=1e-3, graph=True, precision=prec, **kw)
    return _steps(step, m, data)


def wire16(sd, data, dev, pg, prec):
    """graph DP step over RCCL with bf16 gradient buckets: after each step the fp32
    gradients the optimizer read == bf16(graph gradient) widened, every parameter"""
    m = ACC_UNet(3, 1, n_filts=8)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    step = TrainStep(m, lr=1e-3, graph=True, precision=prec, process_group=pg, bucket_mb=0.25,
                     comm_dtype="bf16")
    nb = 0
    for x, y in data:
        step(x, y)
        torch.cuda.synchronize()
        nb = len(step._buckets.buckets)
        for p, g in zip(step.params, step._graph_grads):
            assert p.grad.data_ptr() != g.data_ptr()
            want = g.to(torch.bfloat16).float()
            assert torch.equal(p.grad, want), float((p.grad - want).abs().max())
    return nb


def _steps(step, m, data):
    losses = [float(step(x, y)) for x, y in data]
    torch.cuda.synchronize()
    nb = len(step._buckets.buckets) if step._buckets is not None else 0
    return flat_params(m), losses, nb


def main():
    assert os.environ.get("WORLD_SIZE") == "1"
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl")
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    dev = torch.device("cuda", 0)
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, 8), seed=0)
    g = torch.Generator().manual_seed(1000)
    data = [(torch.randn(2, 3, 32, 32, generator=g).to(dev),
             (torch.rand(2, 1, 32, 32, generator=g) < 0.3).float().to(dev)) for _ in range(3)]
    for prec in ("fp32", "bf16"):
        p_dp, l_dp, nb = run(sd, data, dev, dist.group.WORLD, prec)
        p_1, l_1, nb1 = run(sd, data, dev, None, prec)
        d = float((p_dp - p_1).abs().max())
        print(f"{prec}: rccl buckets {nb} (plain {nb1}); losses {l_dp} vs {l_1}; "
              f"max|dp| {d:.3e}", flush=True)
        assert nb >= 3 and nb1 == 0, (nb, nb1)
        assert torch.equal(p_dp, p_1), d
        assert l_dp == l_1
        nb16 = wire16(sd, data, dev, dist.group.WORLD, prec)
        print(f"{prec}: bf16-wire buckets {nb16}: reduced gradient == bf16(gradient)", flush=True)
        assert nb16 >= 3
    dist.destroy_process_group()
    print("RCCL_OK", flush=True)


if __name__ == "__main__":
    main()
