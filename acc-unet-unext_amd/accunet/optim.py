"""Optimizer and LR schedule of the training step.

FusedAdam is torch.optim.Adam's update (the reference's optimizer,
Experiments/train_model.py:647: Adam(lr=1e-3), default betas/eps, no weight decay)
executed as ONE multi-tensor HIP launch over every parameter (libaccunet_hip.so:
accunet_adam_step). It keeps torch.optim.Optimizer's param_groups / state_dict
interface so checkpoints (train_model.py:139-145 stores optimizer.state_dict())
and LR schedulers work unchanged.

CosineAnnealingWarmRestarts restates Experiments/utils.py:668-784 (T_mult = 1 path).
"""
from __future__ import annotations

import math

import torch

from . import kern


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._tables = {}

    def _table(self, group_idx, params):
        # The chunk map depends only on the parameter set; gradient pointers change
        # every step when autograd hands over fresh gradient tensors, so only the
        # pointer table is re-uploaded (pinned, async: no host sync).
        # the moment buffers are part of the key: load_state_dict replaces them
        key = (group_idx, tuple((p.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                                 self.state[p]["exp_avg_sq"].data_ptr()) for p in params))
        gkey = tuple(p.grad.data_ptr() for p in params)
        t = self._tables.get(group_idx)
        if t is not None and t[0] == key:
            tab, ct, cs, n = t[1]
            if t[2] != gkey:
                rows = [[p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                         self.state[p]["exp_avg_sq"].data_ptr(), p.numel()] for p in params]
                host = torch.tensor(rows, dtype=torch.int64).pin_memory()
                tab.copy_(host, non_blocking=True)
                self._tables[group_idx] = (key, t[1], gkey)
            return t[1]
        dev = params[0].device
        rows = []
        chunk_t, chunk_s = [], []
        ce = kern.adam_chunk_elems()
        for i, p in enumerate(params):
            st = self.state[p]
            rows.append([p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                         st["exp_avg_sq"].data_ptr(), p.numel()])
            for s0 in range(0, p.numel(), ce):
                chunk_t.append(i)
                chunk_s.append(s0)
        tab = torch.tensor(rows, dtype=torch.int64).to(dev)
        ct = torch.tensor(chunk_t, dtype=torch.int32).to(dev)
        cs = torch.tensor(chunk_s, dtype=torch.int64).to(dev)
        entry = (tab, ct, cs, len(chunk_t))
        self._tables[group_idx] = (key, entry, gkey)
        return entry

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    raise RuntimeError("FusedAdam: fp32 contiguous gradients expected")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            # one step counter per group (all params of a group step together here):
            # the params share ONE host tensor, incremented in place like
            # torch.optim.Adam's step_t += 1, so the host cost per step is one op
            # instead of one tensor per parameter (918 for ACC-UNet)
            shared = self.state[params[0]]["step"]
            if any(self.state[p]["step"] is not shared for p in params):
                steps = {float(self.state[p]["step"]) for p in params}
                if len(steps) != 1:
                    raise RuntimeError("FusedAdam: parameters of a group have different step counts")
                shared = torch.tensor(steps.pop())
                for p in params:
                    self.state[p]["step"] = shared
            if len(params) != len(group["params"]):
                # a parameter skipped this step (grad None) keeps its own count, as in
                # torch.optim.Adam: it leaves the shared counter before the increment
                live = {id(p) for p in params}
                for p in group["params"]:
                    st = self.state.get(p)
                    if id(p) not in live and st and st.get("step") is shared:
                        st["step"] = shared.clone()
            shared += 1
            step = int(shared)
            tab, ct, cs, n = self._table(gi, params)
            b1, b2 = group["betas"]
            kern.adam_step(tab, ct, cs, n, group["lr"], b1, b2, group["eps"],
                           group["weight_decay"], step)
        return loss


class CosineAnnealingWarmRestarts:
    """eta_t = eta_min + (base_lr - eta_min) * (1 + cos(pi * T_cur / T_i)) / 2,
    stepped once per (validation) epoch (Experiments/Train_one_epoch.py:187-188)."""

    def __init__(self, optimizer, T_0, T_mult=1, eta_min=0.0, last_epoch=-1):
        if T_0 <= 0 or not isinstance(T_0, int):
            raise ValueError(f"Expected positive integer T_0, but got {T_0}")
        if T_mult != 1:
            raise NotImplementedError("T_mult == 1 only (the reference uses T_0=10, T_mult=1)")
        self.optimizer = optimizer
        self.T_0 = T_0
        self.T_i = T_0
        self.T_mult = T_mult
        self.eta_min = eta_min
        self.base_lrs = [g.get("initial_lr", g["lr"]) for g in optimizer.param_groups]
        for g, b in zip(optimizer.param_groups, self.base_lrs):
            g.setdefault("initial_lr", b)
        self.last_epoch = last_epoch
        self.T_cur = last_epoch
        self.step()

    def get_lr(self):
        return [self.eta_min + (b - self.eta_min) * (1 + math.cos(math.pi * self.T_cur / self.T_i)) / 2
                for b in self.base_lrs]

    def step(self, epoch=None):
        if epoch is None and self.last_epoch < 0:
            epoch = 0
        if epoch is None:
            epoch = self.last_epoch + 1
            self.T_cur = self.T_cur + 1
            if self.T_cur >= self.T_i:
                self.T_cur = self.T_cur - self.T_i
        else:
            self.T_cur = epoch % self.T_0 if epoch >= self.T_0 else epoch
        self.last_epoch = math.floor(epoch)
        for g, lr in zip(self.optimizer.param_groups, self.get_lr()):
            g["lr"] = lr
        self._last_lr = [g["lr"] for g in self.optimizer.param_groups]

    def get_last_lr(self):
        return self._last_lr

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, sd):
        self.__dict__.update(sd)
