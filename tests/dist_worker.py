"""Worker for tests/test_dist_gpu.py: one rank of a world-2 (or world-4) data-parallel run.

Launched by torch.distributed.run with ACCUNET_DIST_BACKEND=gloo so that two ranks
can share the single GPU of a test box (RCCL refuses two ranks on one device); the
data-parallel code path is the one bench.py runs over RCCL on a node:
  1. graph mode: TrainStep(graph=True, bucket_mb=0.25) = HIP-graph replay + the
     event-gated bucketed all-reduce (mean; ~16 buckets of the n_filts=8 model, so
     the multi-bucket marker/event path runs) + fused Adam, 3 steps on rank-specific
     data;
  2. eager mode: TrainStep with GradBucketReducer (bucketed all-reduce overlapped
     with backward through post-accumulate-grad hooks), same start, same data.
  3. the epoch loop: Trainer(reducer=GradBucketReducer) over the same batches.
  4./5. graph and eager again in bf16 storage (BASELINE configs[2]'s precision).
  6. graph mode with bf16 gradient buckets on the wire (TrainStep(comm_dtype="bf16"),
     fp32 storage): within bf16 rounding of the fp32-bucket run.
Checks: parameters identical on both ranks after each mode (bitwise), graph and eager
identical to each other (bitwise, fp32 and bf16: the same kernels in the same order,
and a world-2 sum is order-free), the epoch loop equal to eager, and the parameters
moved. World 4 (check_world4): every rank identical after every mode, and one step's
reduced gradient (fp32 buckets, bf16 buckets, eager reducer) against the fp64 mean of
the four ranks' own gradients.
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "acc-unet-unext_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import accunet_oracle as O  # noqa: E402
from accunet import dist as adist  # noqa: E402
from accunet.model import ACC_UNet  # noqa: E402
from accunet.train import TrainStep  # noqa: E402


def flat_params(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def run(mode, sd, data, dev):
    m = ACC_UNet(3, 1, n_filts=8)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    prec = None
    wire = None
    if mode.endswith("_wire16"):
        mode, wire = mode[:-7], "bf16"
    if mode.endswith("_bf16"):
        mode, prec = mode[:-5], "bf16"
    if mode == "trainer":  # the epoch loop with the bucketed reducer (Trainer(reducer=))
        from accunet.trainer import Trainer
        tr = Trainer(m, lr=1e-3, lr_scheduler=None, device=dev,
                     reducer=adist.GradBucketReducer(m, bucket_mb=0.25))
        tr.train_one_epoch([({"image": x, "label": y}, None) for x, y in data], 0, True)
        torch.cuda.synchronize()
        return flat_params(m), [h["loss"] for h in tr.history]
    if mode == "graph":
        step = TrainStep(m, lr=1e-3, graph=True, bucket_mb=0.25, precision=prec,
                         comm_dtype=wire)
    else:
        step = TrainStep(m, lr=1e-3, reducer=adist.GradBucketReducer(m, bucket_mb=0.25),
                         precision=prec)
    losses = []
    for x, y in data:
        losses.append(float(step(x, y)))
    torch.cuda.synchronize()
    if mode == "graph":
        nb = len(step._buckets.buckets)
        assert nb >= 3, f"graph mode ran {nb} bucket(s); the multi-bucket path needs >= 3"
        want = torch.bfloat16 if wire else torch.float32
        assert step._buckets.wire.dtype == want, step._buckets.wire.dtype
        print(f"graph{'_' + prec if prec else ''}: {nb} buckets", flush=True)
    return flat_params(m), losses


def grads_one_step(sd, batch, dev, wire):
    """the all-reduced fp32 gradient vector after one graph-mode step (bucket wire format
    `wire`): p.grad are the views of the bucket buffer the optimizer read"""
    m = ACC_UNet(3, 1, n_filts=8)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    step = TrainStep(m, lr=1e-3, graph=True, bucket_mb=0.25, comm_dtype=wire)
    step(*batch)
    torch.cuda.synchronize()
    return torch.cat([p.grad.detach().reshape(-1).double() for p in m.parameters()])


def local_grads(sd, batch, dev):
    """this rank's own (un-reduced) fp32 gradient of one step: plain autograd through
    the HIP ops, no process group involved"""
    from accunet.loss import WeightedDiceBCE
    m = ACC_UNet(3, 1, n_filts=8)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    loss = WeightedDiceBCE(0.5, 0.5)(m(batch[0]), batch[1])
    loss.backward()
    torch.cuda.synchronize()
    return torch.cat([p.grad.detach().reshape(-1) for p in m.parameters()])


def eager_grads_one_step(sd, batch, dev):
    """the all-reduced gradient after one eager step with the bucketed hook reducer"""
    m = ACC_UNet(3, 1, n_filts=8)
    m.load_state_dict(sd)
    m = m.to(dev).train()
    step = TrainStep(m, lr=1e-3, reducer=adist.GradBucketReducer(m, bucket_mb=0.25))
    step(*batch)
    torch.cuda.synchronize()
    return torch.cat([p.grad.detach().reshape(-1).double() for p in m.parameters()])


def check_world4(rank, world, sd, data, dev):
    """world > 2: the reduced gradient of one step -- graph mode with fp32 and bf16
    buckets (cut_buckets, 1/world pre-division, SUM), eager hook reducer -- against the
    fp64 mean of the ranks' own fp32 gradients (all-gathered). fp32 wire and eager:
    within fp32 rounding of a world-addend sum (world 4 or 8); bf16 wire: each addend
    rounded to bf16 when packed and the partial sums rounded by the collective, so
    within sqrt(world) * 2^-9 of the mean of |g_r| in norm (2^-8 at world 4)."""
    mine = local_grads(sd, data[0], dev)
    allg = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allg, mine)
    ref = torch.stack([g.double() for g in allg]).mean(0)
    ranks_differ = float(max((allg[r] - allg[0]).abs().max() for r in range(1, world)))
    assert ranks_differ > 0, "rank-specific data should give different local gradients"
    g32 = grads_one_step(sd, data[0], dev, None)
    g16 = grads_one_step(sd, data[0], dev, "bf16")
    ge = eager_grads_one_step(sd, data[0], dev)
    rn = float(ref.norm())
    e32 = float((g32 - ref).norm()) / rn
    e16 = float((g16 - ref).norm()) / rn
    ee = float((ge - ref).norm()) / rn
    dge = float((g32 - ge).abs().max())
    # bf16 wire bound: world roundings of the addends and world - 1 of the partial sums,
    # unit roundoff 2^-8 each, adding like a random walk (sqrt(world) * 2^-9), measured
    # against the mean of |g_r| (cancellation between ranks' gradients magnifies the
    # relative error of the mean): 2^-8 at world 4, as before
    ratio = float(torch.stack([g.double().abs() for g in allg]).mean(0).norm()) / rn
    b16 = 2 ** -9 * math.sqrt(world) * ratio
    print(f"rank {rank} world {world}: reduced gradient vs fp64 mean of {world} ranks: fp32 "
          f"buckets {e32:.3e}, eager reducer {ee:.3e}, bf16 buckets {e16:.3e} (bound {b16:.3e}, "
          f"|g| ratio {ratio:.3f}); graph vs eager max|dg| {dge:.3e}", flush=True)
    assert e32 <= 1e-6 and ee <= 1e-6, (e32, ee)
    assert 0 < e16 <= b16, (e16, b16)
    assert dge <= 1e-6 * float(ref.abs().max()), dge


def main():
    rank, world = adist.init_from_env()
    assert world in (2, 4, 8), world
    dev = torch.device("cuda", adist.local_device())
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, 8), seed=0)
    m0 = ACC_UNet(3, 1, n_filts=8)
    m0.load_state_dict(sd)
    p0 = flat_params(m0).to(dev)
    g = torch.Generator().manual_seed(1000 + rank)
    data = [(torch.randn(2, 3, 32, 32, generator=g).to(dev),
             (torch.rand(2, 1, 32, 32, generator=g) < 0.3).float().to(dev)) for _ in range(3)]
    out = {}
    modes = ("graph", "eager", "trainer", "graph_bf16", "eager_bf16", "graph_wire16")
    if os.environ.get("DIST_MODES"):  # diagnostics: a subset of the modes
        modes = tuple(os.environ["DIST_MODES"].split(","))
    for mode in modes:
        p, losses = run(mode, sd, data, dev)
        other = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(other, p)
        same = all(bool(torch.equal(other[0], o)) for o in other[1:])
        moved = float((p - p0).abs().max())
        out[mode] = (p, losses)
        print(f"rank {rank} {mode}: losses {losses} ranks-identical {same} moved {moved:.3e}",
              flush=True)
        assert same, f"{mode}: parameters differ between ranks"
        assert moved > 1e-5, f"{mode}: parameters did not move"
    if world > 2:
        # a sum of 4 (8) addends depends on the collective's order, which follows the bucket
        # cut (graph and eager buckets differ): compared through one step's gradients
        check_world4(rank, world, sd, data, dev)
        dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            print("DIST_OK", flush=True)
        return
    for sfx in ("", "_bf16"):
        d = float((out["graph" + sfx][0] - out["eager" + sfx][0]).abs().max())
        print(f"rank {rank} graph{sfx} vs eager{sfx} max|dp| {d:.3e}", flush=True)
        assert torch.equal(out["graph" + sfx][0], out["eager" + sfx][0]), d
        assert out["graph" + sfx][1] == out["eager" + sfx][1]
    # the epoch loop runs the same steps (its loss is the epoch average)
    d = float((out["trainer"][0] - out["eager"][0]).abs().max())
    print(f"rank {rank} trainer vs eager max|dp| {d:.3e}", flush=True)
    assert d < 1e-5, d
    # bf16 buckets: the all-reduced gradient of one step (each rank's gradient rounded to
    # bf16 when packed, the pair summed in bf16 by the collective, then halved) against
    # the fp32-bucket run's: within a few bf16 roundings, in norm. (Parameters after
    # several Adam steps are no yardstick: Adam turns the rounding of near-zero gradients
    # into lr-sized steps of either sign.)
    g32, g16 = grads_one_step(sd, data[0], dev, None), grads_one_step(sd, data[0], dev, "bf16")
    rel = float((g16 - g32).norm() / g32.norm())
    dl = max(abs(a - b) for a, b in zip(out["graph_wire16"][1], out["graph"][1]))
    print(f"rank {rank} bf16-bucket gradient vs fp32 buckets: rel {rel:.3e}; 3-step max|dloss| "
          f"{dl:.3e}", flush=True)
    assert 0 < rel <= 2 ** -7, rel
    assert dl <= 1e-2 * abs(out["graph"][1][-1]), dl
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print("DIST_OK", flush=True)


if __name__ == "__main__":
    main()
