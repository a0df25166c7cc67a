"""Loss / metrics of the training step (reference Experiments/utils.py).

WeightedDiceBCE keeps the reference's interface (`forward(inputs, targets)`,
`_show_dice`) and semantics, including the double sigmoid the reference applies
to probability outputs (utils.py:124 on top of the model's Sigmoid) and the
in-place binarisation of `targets` in `_show_dice` (utils.py:154-155). The loss
value and its gradient come from one HIP reduction + one elementwise kernel.
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops


class WeightedDiceBCE(nn.Module):
    """Experiments/utils.py:140-171 with WeightedBCE / WeightedDiceLoss weights [0.5, 0.5]."""

    def __init__(self, dice_weight=1, BCE_weight=1, n_labels=1):
        super().__init__()
        if n_labels != 1:
            raise NotImplementedError("WeightedDiceBCE: n_labels == 1 (as in the reference)")
        self.n_labels = n_labels
        self.dice_weight = dice_weight
        self.BCE_weight = BCE_weight

    def forward(self, inputs, targets):
        return ops.weighted_dice_bce(inputs, targets, self.dice_weight, self.BCE_weight)

    @torch.no_grad()
    def _show_dice(self, inputs, targets):
        """Hard Dice as the reference logs it (utils.py:149-158): sigmoid, threshold,
        then the (sigmoid-applying) weighted Dice loss; mutates `targets`."""
        hard = (torch.sigmoid(inputs) >= 0.5).float()
        targets[targets > 0] = 1
        targets[targets <= 0] = 0
        dice = ops.weighted_dice_terms(hard, targets)
        return 1.0 - dice
