"""Data-parallel training over RCCL (torch.distributed "nccl" backend = RCCL on ROCm).

One process per GPU; the minibatch is sharded (each rank runs its own B images);
BatchNorm statistics stay per rank, as with torch DDP's default (the reference
has no SyncBN and no distributed code at all — SURVEY §2.1, §8(e)).

GradBucketReducer is the only collective on the path: gradients are views into
one flat fp32 buffer partitioned into ~25 MB buckets in reverse registration
order (the order backward produces them, output layer first). A
post-accumulate-grad hook counts ready parameters per bucket and launches an
async all-reduce (pre-divided by the world, then SUM) of the bucket as soon as it is complete, so RCCL traffic
over xGMI overlaps the rest of backward on RCCL's own stream. A final autograd
callback flushes buckets holding parameters that received no gradient (e.g.
ACC_UNet_Lite's bypassed MLFC convolutions, ACC_UNet_lite.py:422-429) so every
rank issues the same collectives in the same order.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def init_from_env(backend: Optional[str] = None):
    """Initialise the process group from torchrun env vars (RANK, WORLD_SIZE, ...)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return 0, 1
    if backend is None:
        # ACCUNET_DIST_BACKEND=gloo runs the same path over gloo (e.g. several ranks
        # sharing one GPU in tests, where RCCL refuses duplicate devices)
        backend = os.environ.get("ACCUNET_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device())
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def local_device() -> int:
    """GPU index of this rank: LOCAL_RANK (modulo the visible devices, so ranks can
    share a GPU when there are fewer devices than ranks)."""
    n = torch.cuda.device_count()
    return int(os.environ.get("LOCAL_RANK", "0")) % max(n, 1)


def all_reduce_mean(t: torch.Tensor, group=None):
    """In-place mean over ranks: RCCL's AVG, or SUM / world on backends without AVG."""
    if dist.get_backend(group) == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(dist.get_world_size(group))


class GradBucketReducer:
    def __init__(self, module: torch.nn.Module, bucket_mb: float = 25.0, process_group=None,
                 broadcast_params: bool = True):
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # the fp32 value of 1/world the graph-mode packing multiplies by (AccRelayout.scale)
        self.inv_world = float(torch.tensor(1.0 / self.world, dtype=torch.float32))
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = params
        dev = params[0].device
        total = sum(p.numel() for p in params)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        # registration order offsets; buckets are cut in REVERSE order
        offs = []
        o = 0
        for p in params:
            offs.append(o)
            o += p.numel()
        cap = int(bucket_mb * (1 << 20) / 4)
        self.buckets: List[List[int]] = []
        cur, cur_n = [], 0
        for i in reversed(range(len(params))):
            cur.append(i)
            cur_n += params[i].numel()
            if cur_n >= cap:
                self.buckets.append(cur)
                cur, cur_n = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {}
        self.bucket_range = []
        for b, idxs in enumerate(self.buckets):
            lo = min(offs[i] for i in idxs)
            hi = max(offs[i] + params[i].numel() for i in idxs)
            self.bucket_range.append((lo, hi))
            for i in idxs:
                self.bucket_of[i] = b
        self._views = [self.flat[offs[i]:offs[i] + p.numel()].view_as(p)
                       for i, p in enumerate(params)]
        for p, v in zip(params, self._views):
            p.grad = v
        self._reset()
        for i, p in enumerate(params):
            p.register_post_accumulate_grad_hook(self._make_hook(i))
        if broadcast_params and self.world > 1:
            with torch.no_grad():
                for p in params:
                    dist.broadcast(p.data, 0, group=self.pg)
                for b in module.buffers():
                    dist.broadcast(b, 0, group=self.pg)

    def zero_grad(self):
        self.flat.zero_()

    def _reset(self):
        self._pending = [len(idxs) for idxs in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._handles = []
        self._callback_queued = False

    def _launch(self, b):
        if self._launched[b]:
            return
        self._launched[b] = True
        lo, hi = self.bucket_range[b]
        if self.world > 1:
            # pre-divided by the world (fp32), then a plain SUM: the PreMulSum form of
            # AVG the graph-mode step uses (train._GraphBuckets packs gradients times
            # 1/world), so the two modes agree bit for bit at every world size, not only
            # where x/world == x*(1/world) exactly (powers of two)
            seg = self.flat[lo:hi]
            seg.mul_(self.inv_world)
            h = dist.all_reduce(seg, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            self._handles.append((h, lo, hi))

    def _finish(self):
        for b in range(len(self.buckets)):
            self._launch(b)
        for h, lo, hi in self._handles:
            h.wait()
        # ready for the next backward whether or not the caller runs prepare()
        self._reset()

    def _make_hook(self, i):
        def hook(p):
            if not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finish)
            v = self._views[i]
            if p.grad is not v and (p.grad is None or p.grad.data_ptr() != v.data_ptr()):
                # the gradient was detached from the flat buffer (e.g.
                # optimizer.zero_grad()'s set_to_none): move it back in, so the bucket
                # reduces what backward produced instead of stale zeros
                v.copy_(p.grad)
                p.grad = v
            b = self.bucket_of[i]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)
        return hook

    def prepare(self):
        """Optional before a backward (the state also resets after every flush)."""
        self._reset()
