"""Training-step harness: the counterpart of Experiments/Train_one_epoch.py:48-201
and train_model.py:269-833 for the ACC-UNet path, without the per-step host
syncs of the reference loop (sklearn IoU on CPU, torch.cuda.empty_cache twice per
step, Train_one_epoch.py:134,167,185): metrics stay on the device and are read
only when logged.

    step = TrainStep(model, lr=1e-3)            # Adam(lr 1e-3), WeightedDiceBCE(0.5, 0.5)
    loss = step(images, masks)                  # fwd + loss + bwd (+ RCCL all-reduce) + Adam
"""
from __future__ import annotations

import torch

from .loss import WeightedDiceBCE
from .optim import FusedAdam


class TrainStep:
    def __init__(self, model, lr=1e-3, reducer=None, dice_weight=0.5, bce_weight=0.5):
        self.model = model
        self.reducer = reducer
        self.criterion = WeightedDiceBCE(dice_weight, bce_weight)
        params = [p for p in model.parameters() if p.requires_grad]
        # single GPU: gradients are the tensors the backward kernels produce
        # (AccumulateGrad steals them, no per-parameter add); with a reducer they
        # are views of its flat all-reduce buffer.
        self.opt = FusedAdam(params, lr=lr)

    def zero_grad(self):
        if self.reducer is not None:
            self.reducer.zero_grad()
        else:
            for p in self.opt.param_groups[0]["params"]:
                p.grad = None

    def __call__(self, images, masks):
        self.model.train(True)
        self.zero_grad()
        if self.reducer is not None:
            self.reducer.prepare()
        preds = self.model(images)
        loss = self.criterion(preds, masks)
        loss.backward()
        self.opt.step()
        return loss.detach()
