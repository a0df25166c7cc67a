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
      gradients are bucketed (~16 MB, reverse registration order = the order
      backward finishes them). Inside the graph, the moment a bucket's last
      gradient is accumulated its gradients are packed into the flat all-reduce
      buffer and a marker kernel is left in the stream; after capture an
      event-record node is added behind each marker (accunet_graph_events_after_
      markers on the kept hipGraph_t, then instantiate). Each step the host replays
      the graph and, without waiting, enqueues per bucket on a side stream:
      wait(bucket event) -> RCCL all_reduce(SUM) of that slice (packed pre-divided
      by the world, so the sum is the mean). The collectives therefore run over xGMI while the graph is still computing the rest of
      backward; only the last bucket's reduce is exposed before the one-launch Adam.
      The collectives themselves are not captured (they run on RCCL's own stream).
      Capture happens on the first call: no autograd graph of an earlier eager
      step may still be alive then (drop references to its outputs / loss), since
      PyTorch keeps the stream of every AccumulateGrad node such a graph holds and
      accumulating through it on the default stream breaks the capture.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import contextlib
import os

from . import kern, ops
from . import profile as _prof
from .loss import WeightedDiceBCE
from .optim import FusedAdam


def cut_buckets(numels, bucket_mb, tail_mb=1.0):
    """Parameter indices per bucket, in reverse registration order (backward finishes
    the output layer first); each bucket but the last holds >= bucket_mb of fp32. One
    graph marker per bucket, and accunet_graph_marker takes MAX_GRAPH_MARKERS ids, so
    a smaller bucket_mb is raised until the greedy cut yields at most that many."""
    total = sum(numels)
    cap = max(1, int(bucket_mb * (1 << 20) / 4), -(-total // kern.MAX_GRAPH_MARKERS))
    buckets, cur, n = [], [], 0
    for i in reversed(range(len(numels))):
        cur.append(i)
        n += numels[i]
        if n >= cap:
            buckets.append(cur)
            cur, n = [], 0
    if cur:
        buckets.append(cur)
    # The last bucket seals when the backward ends, so its reduce (and, with the bf16
    # wire, its widening copy) is the exposed tail of the step: its first-registered
    # parameters (the encoder's first blocks, whose gradients come last) go into a
    # bucket of their own of at most tail_mb, and the rest seals earlier, while those
    # blocks' backward still runs.
    tail = max(1, int(tail_mb * (1 << 20) / 4))
    last = buckets[-1] if buckets else []
    if len(buckets) < kern.MAX_GRAPH_MARKERS and sum(numels[i] for i in last) > tail:
        k, n = len(last), 0
        while k > 1 and n + numels[last[k - 1]] <= tail:
            k -= 1
            n += numels[last[k]]
        if k < len(last):
            buckets[-1:] = [last[:k], last[k:]]
    return buckets


class _GraphBuckets:
    """Bucketed, event-gated gradient all-reduce for the captured backward (graph mode,
    world > 1; see the module docstring). Built before capture; its hooks run only
    while the backward is being captured."""

    def __init__(self, params, bucket_mb, device, comm_dtype=None, world=1):
        self.params = params
        # the packed gradients are pre-divided by the world (exact for power-of-two
        # worlds), so the all-reduce is a plain SUM -- RCCL's PreMulSum form of AVG, which
        # at world 1 also leaves no reduce kernel behind -- and the reduced buffer holds
        # the mean, as with AVG
        self.scale = 1.0 / world
        # each view starts at a multiple of 4 elements, so the packing copies move whole
        # 16-byte (fp32) / 8-byte (bf16) quads; the pads stay zero
        offs, o = [], 0
        for p in params:
            offs.append(o)
            o += -(-p.numel() // 4) * 4
        total = max(o, 1)
        self.flat = torch.zeros(total, dtype=torch.float32, device=device)
        # comm_dtype bf16: the buckets travel as bf16 (half the bytes over xGMI; the
        # gradients are rounded once when packed, RCCL sums in bf16) and are widened back
        # into the fp32 views the optimizer reads, bucket by bucket, behind each reduce
        self.comm_dtype = comm_dtype
        self.wire = (torch.zeros(total, dtype=comm_dtype, device=device)
                     if comm_dtype not in (None, torch.float32) else self.flat)
        self.views, self.wviews = [], []
        for p, o in zip(params, offs):
            self.views.append(self.flat[o:o + p.numel()].view_as(p))
            self.wviews.append(self.wire[o:o + p.numel()].view_as(p))
        self.buckets = cut_buckets([p.numel() for p in params], bucket_mb)
        self.range = [(min(offs[i] for i in b), max(offs[i] + params[i].numel() for i in b))
                      for b in self.buckets]
        self.bucket_of = {i: k for k, b in enumerate(self.buckets) for i in b}
        self.events = [kern.GraphEvent() for _ in self.buckets]
        self._handles = []
        # every sealed bucket is packed by ONE batched copy launch (fp32, or rounded to
        # bf16 for the bf16 wire) instead of _foreach_copy_ (a mixed-dtype foreach copy
        # falls back to one launch per tensor: ~900 graph nodes per step)
        self.packer = ops.DeferredRelayouts(device, cap=len(params))
        self.seal_stream = None

    # ------------------------------------------------------------ capture side
    def _seal(self, k):
        """pack bucket k's gradients into the flat buffer, then mark it ready -- on a
        stream of its own, forked from the backward at this point, so the packing
        launches run beside the rest of the backward instead of in its chain (every
        source is final here and stays referenced: parameter gradients, the deferred
        relayouts' kept sources); the backward joins it before the capture ends"""
        if self._sealed[k]:
            return
        self._sealed[k] = True
        main = torch.cuda.current_stream()
        if self.seal_stream is None:
            self.seal_stream = torch.cuda.Stream(device=main.device)
        self.seal_stream.wait_stream(main)
        with torch.cuda.stream(self.seal_stream):
            if ops._DEFER is not None:  # pending inverse weight relayouts: final values first
                ops._DEFER.flush()
            for i in self.buckets[k]:
                g = self.params[i].grad
                if g is not None:
                    self.packer.copy(g.contiguous(), self.wviews[i], scale=self.scale)
            self.packer.flush()
            kern.GraphEvent.mark(k)

    def join(self):
        """the capturing stream waits for the packing stream (before the capture ends)"""
        if self.seal_stream is not None:
            torch.cuda.current_stream().wait_stream(self.seal_stream)

    def _hook(self, i):
        def hook(p):
            # one gradient contribution per parameter: a second AccumulateGrad add on the
            # main stream could land after this bucket's seal (packing, and the deferred
            # relayouts the seal stream writes into .grad) -- refuse it at capture time
            self._fired[i] += 1
            if self._fired[i] > 1:
                raise RuntimeError(f"graph-mode data parallelism: parameter {i} received more "
                                   f"than one gradient contribution; its bucket would be "
                                   f"sealed before the last one (use graph=False)")
            if not self._queued:  # buckets with unused parameters close at the end
                self._queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._flush)
            k = self.bucket_of[i]
            self._left[k] -= 1
            if self._left[k] == 0:
                self._seal(k)
        return hook

    def _flush(self):
        for k in range(len(self.buckets)):
            self._seal(k)

    def arm(self):
        self._left = [len(b) for b in self.buckets]
        self._sealed = [False] * len(self.buckets)
        self._fired = [0] * len(self.params)
        self._queued = False
        self._handles = [p.register_post_accumulate_grad_hook(self._hook(i))
                         for i, p in enumerate(self.params)]

    def disarm(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    # -------------------------------------------------------------- step side
    def reduce(self, pg):
        """enqueue every bucket's all-reduce behind its event (no host wait for RCCL)"""
        nccl = dist.get_backend(pg) == "nccl"
        main = torch.cuda.current_stream()
        narrow = self.wire is not self.flat
        if not nccl:  # gloo (tests): host-synchronous collectives on finished buckets
            for k, (lo, hi) in enumerate(self.range):
                self.events[k].synchronize()
                dist.all_reduce(self.wire[lo:hi], op=dist.ReduceOp.SUM, group=pg)
                if narrow:
                    self.flat[lo:hi].copy_(self.wire[lo:hi])
            return
        works = []
        with torch.cuda.stream(self.stream):
            # every reduce first, each behind its own bucket's event only: RCCL's stream
            # waits on this side stream when a collective is enqueued, so a widening copy
            # issued between two reduces would hold the next reduce back
            for k, (lo, hi) in enumerate(self.range):
                self.events[k].wait(self.stream)
                works.append(dist.all_reduce(self.wire[lo:hi], op=dist.ReduceOp.SUM, group=pg,
                                             async_op=True))
            if narrow:  # widen each bucket on the side stream once RCCL is done with it
                for (lo, hi), w in zip(self.range, works):
                    w.wait()
                    self.flat[lo:hi].copy_(self.wire[lo:hi])
        for w in works:  # the main stream (Adam) waits on RCCL's stream
            w.wait()
        main.wait_stream(self.stream)


class TrainStep:
    def __init__(self, model, lr=1e-3, reducer=None, dice_weight=0.5, bce_weight=0.5,
                 graph=False, process_group=None, precision=None, bucket_mb=16.0,
                 comm_dtype=None):
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
        # data-parallel path: world > 1, or an explicitly passed process group (also at
        # world 1, where the all-reduce is an identity: tests run the RCCL branch so)
        self.dp = self.world > 1 or process_group is not None
        self.criterion = WeightedDiceBCE(dice_weight, bce_weight)
        self.params = [p for p in model.parameters() if p.requires_grad]
        # eager single GPU: gradients are the tensors the backward kernels produce
        # (AccumulateGrad steals them, no per-parameter add); with a reducer they
        # are views of its flat all-reduce buffer.
        self.opt = FusedAdam(self.params, lr=lr)
        self._g = None
        self.bucket_mb = bucket_mb
        # graph-mode DP gradient wire format: None / torch.float32, or torch.bfloat16
        # (BASELINE configs[2]: 33.5 MB instead of 67 MB per step over xGMI)
        if comm_dtype == "bf16":
            comm_dtype = torch.bfloat16
        if comm_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError(f"comm_dtype: None, torch.float32 or torch.bfloat16, got {comm_dtype}")
        self.comm_dtype = comm_dtype
        if graph and self.dp:
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
        if ops._DEFER is not None:  # the deferred weight-gradient relayouts, one launch
            ops._DEFER.flush()
        if getattr(self, "_buckets", None) is not None:
            self._buckets.join()
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

        # every forward-layout weight copy in one launch before each replay, read by the
        # captured ops (ops.WeightPrep; ACCUNET_WEIGHT_PREP=0: each op relayouts itself)
        self._prep = None
        if os.environ.get("ACCUNET_WEIGHT_PREP", "1") != "0":
            self._prep = ops.WeightPrep(self.model)
            self._prep.run()
        self._buckets = None
        if self.dp:
            self._buckets = _GraphBuckets(self.params, self.bucket_mb, self._x.device,
                                          self.comm_dtype, world=self.world)
            self._buckets.stream = torch.cuda.Stream()
            self._buckets.seal_stream = torch.cuda.Stream()  # created outside the capture
            self._buckets.arm()
        # the backward's inverse weight relayouts batched: one launch at its end at world 1;
        # with data parallelism one launch per sealed bucket (a gradient bucket must hold
        # final values when it is packed for its all-reduce, _GraphBuckets._seal)
        self._defer = None
        if os.environ.get("ACCUNET_DEFER_RELAYOUT", "1") != "0":
            self._defer = ops.DeferredRelayouts(self._x.device)
        # in-graph timing (accunet/profile.py, bench.py's roofline): marker ids below the
        # bucket count are the buckets'; the timed launches' markers become event-record
        # nodes before the graph is instantiated, so the graph is kept for that too
        _prof.graph_reserve_markers(len(self._buckets.buckets) if self._buckets is not None else 0)
        keep = self._buckets is not None or _prof.graph_timing_requested()
        g = torch.cuda.CUDAGraph(keep_graph=keep)
        try:
            with torch.cuda.graph(g):
                with contextlib.ExitStack() as es:
                    if self._prep is not None:
                        es.enter_context(self._prep.active())
                    if self._defer is not None:
                        es.enter_context(self._defer.active())
                    loss = self._fwd_bwd(self._x, self._m)
        finally:
            if self._buckets is not None:
                self._buckets.disarm()
        if self._defer is not None:
            # every deferred relayout must write a buffer autograd took as a parameter's
            # .grad (not a copy of it, which would have been read before the launch)
            grads = {p.grad.data_ptr() for p in self.params if p.grad is not None}
            lost = [a for a in self._defer.destinations() if a not in grads]
            if lost:
                raise RuntimeError(f"deferred weight-gradient relayouts: {len(lost)} "
                                   f"destination(s) are not parameter gradients")
            self._defer.upload()  # the item table the captured launch reads
        if self._buckets is not None:
            self._buckets.packer.upload()  # the bucket-packing item tables
            # an event-record node behind every bucket's marker, then instantiate
            n = kern.GraphEvent.attach(g.raw_cuda_graph(), self._buckets.events)
            if n != len(self._buckets.buckets):
                raise RuntimeError(f"graph bucket markers: found {n}, expected "
                                   f"{len(self._buckets.buckets)}")
        if _prof.graph_marks_pending():
            _prof.graph_attach(g.raw_cuda_graph())
        if keep:
            g.instantiate()
        self._g = g
        self._loss = loss.detach()
        # keep the graph-pool gradient tensors alive; the optimizer reads either them
        # (world 1) or the flat all-reduced buffer (world > 1)
        self._graph_grads = [p.grad for p in self.params]
        if self.dp:
            for p, v in zip(self.params, self._buckets.views):
                p.grad = v
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
        if self._prep is not None:
            self._prep.run()  # from the weights the last Adam step left
        _prof.graph_before_replay(self._g)
        self._g.replay()
        if self.dp:
            self._buckets.reduce(self.pg)
        self.opt.step()
        return self._loss

    def __call__(self, images, masks):
        if not self.graph:
            return self._eager(images, masks)
        if self._g is None:
            self._capture(images, masks)
        return self._replay(images, masks)
