"""Training-step harness: the counterpart of Experiments/Train_one_epoch.py:48-201
and train_model.py:269-833 for the ACC-UNet path, without the per-step host
syncs of the reference loop (sklearn IoU on CPU, torch.cuda.empty_cache twice per
step, Train_one_epoch.py:134,167,185): metrics stay on the device and are read
only when logged.

    step = TrainStep(model, lr=1e-3)            # Adam(lr 1e-3), WeightedDiceBCE(0.5, 0.5)
    step = TrainStep(model, precision="bf16")   # BASELINE configs[2]: bf16 activations
    loss = step(images, masks)                  # fwd + loss + bwd (+ RCCL all-reduce) + Adam

Two execution modes, same arithmetic:
  eager (graph=False): every kernel is launched from Python per step; with a
      GradBucketReducer the gradient all-reduce overlaps backward (bucket hooks).
  graph (graph=True): forward + loss + backward (~1.5k kernel launches) are
      captured once into a HIP graph and replayed, removing the host launch cost
      that otherwise leaves the GPU idle between short kernels. For world > 1 the
      graph also packs the gradients into one flat buffer, which is all-reduced
      (AVG, RCCL) as ONE 67 MB collective between the replay and the optimizer
      (~0.3 ms on xGMI vs ~120 ms of compute); Adam is one launch.
      Capture happens on the first call: no autograd graph of an earlier eager
      step may still be alive then (drop references to its outputs / loss), since
      PyTorch keeps the stream of every AccumulateGrad node such a graph holds and
      accumulating through it on the default stream breaks the capture.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .dist import all_reduce_mean
from .loss import WeightedDiceBCE
from .optim import FusedAdam


class TrainStep:
    def __init__(self, model, lr=1e-3, reducer=None, dice_weight=0.5, bce_weight=0.5,
                 graph=False, process_group=None, precision=None):
        if graph and reducer is not None:
            raise ValueError("graph mode does its own single-bucket all-reduce; pass no reducer")
        if precision is not None:  # "fp32" / "bf16": see ACC_UNet.set_precision
            model.set_precision(precision)
        self.model = model
        self.reducer = reducer
        self.graph = graph
        self.pg = process_group
        self.world = (dist.get_world_size(process_group)
                      if dist.is_available() and dist.is_initialized() else 1)
        self.criterion = WeightedDiceBCE(dice_weight, bce_weight)
        self.params = [p for p in model.parameters() if p.requires_grad]
        # eager single GPU: gradients are the tensors the backward kernels produce
        # (AccumulateGrad steals them, no per-parameter add); with a reducer they
        # are views of its flat all-reduce buffer.
        self.opt = FusedAdam(self.params, lr=lr)
        self._g = None
        if graph and self.world > 1:
            # identical replicas to start from (what DDP / GradBucketReducer do at wrap time)
            with torch.no_grad():
                for t in list(self.params) + [b for b in model.buffers()]:
                    dist.broadcast(t, 0, group=process_group)

    def zero_grad(self):
        if self.reducer is not None:
            self.reducer.zero_grad()
        else:
            for p in self.params:
                p.grad = None

    # ------------------------------------------------------------------ eager
    def _eager(self, images, masks):
        self.model.train(True)
        self.zero_grad()
        if self.reducer is not None:
            self.reducer.prepare()
        preds = self.model(images)
        loss = self.criterion(preds, masks)
        loss.backward()
        self.opt.step()
        return loss.detach()

    # ------------------------------------------------------------------ graph
    def _fwd_bwd(self, x, m):
        preds = self.model(x)
        loss = self.criterion(preds, m)
        loss.backward()
        return loss

    def _capture(self, images, masks):
        self.model.train(True)
        self._x = images.detach().clone()
        self._m = masks.detach().clone()
        # one warm-up pass on a side stream (first launches, allocator growth),
        # with the BatchNorm buffers restored afterwards so capturing has no
        # side effect on the training state
        bufs = {k: v.detach().clone() for k, v in self.model.named_buffers()}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for p in self.params:
                p.grad = None
            self._fwd_bwd(self._x, self._m)
        torch.cuda.current_stream().wait_stream(side)
        with torch.no_grad():
            for k, v in self.model.named_buffers():
                v.copy_(bufs[k])
        for p in self.params:
            p.grad = None
        torch.cuda.synchronize()

        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self._fwd_bwd(self._x, self._m)
            live = [p for p in self.params if p.grad is not None]
            if self.world > 1:
                total = sum(p.numel() for p in self.params)
                self._flat = torch.zeros(total, dtype=torch.float32, device=self._x.device)
                views, o = {}, 0
                for p in self.params:
                    views[p] = self._flat[o:o + p.numel()].view_as(p)
                    o += p.numel()
                torch._foreach_copy_([views[p] for p in live], [p.grad for p in live])
        self._g = g
        self._loss = loss.detach()
        # keep the graph-pool gradient tensors alive; the optimizer reads either them
        # (world 1) or the flat all-reduced buffer (world > 1)
        self._graph_grads = [p.grad for p in self.params]
        if self.world > 1:
            for p in self.params:
                p.grad = views[p]
        else:
            for p in self.params:
                if p.grad is None:  # never produced (e.g. Lite's idle MLFC): zero gradient
                    p.grad = torch.zeros_like(p)

    def _replay(self, images, masks):
        if images.shape != self._x.shape or masks.shape != self._m.shape:
            # copy_ would broadcast a smaller batch silently (e.g. a ragged last batch
            # of size 1 replicated over every captured slot)
            raise ValueError(f"TrainStep(graph=True) was captured for images "
                             f"{tuple(self._x.shape)} / masks {tuple(self._m.shape)}, got "
                             f"{tuple(images.shape)} / {tuple(masks.shape)}; use drop_last "
                             f"batching or graph=False for ragged batches")
        if images.data_ptr() != self._x.data_ptr():
            self._x.copy_(images)
        if masks.data_ptr() != self._m.data_ptr():
            self._m.copy_(masks)
        self._g.replay()
        if self.world > 1:
            all_reduce_mean(self._flat, self.pg)
        self.opt.step()
        return self._loss

    def __call__(self, images, masks):
        if not self.graph:
            return self._eager(images, masks)
        if self._g is None:
            self._capture(images, masks)
        return self._replay(images, masks)
