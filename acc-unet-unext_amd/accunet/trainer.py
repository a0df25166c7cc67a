"""Epoch loop around the training step: the counterpart of the reference's
Experiments/train_model.py:663-831 (epochs, validation, best-model checkpoint,
early stopping, resume) and Experiments/Train_one_epoch.py:48-201 (one pass over a
loader with loss / IoU / Dice running averages), for the ACC-UNet path.

Differences from the reference loop are confined to host overhead: metrics are
accumulated on the device and read once per epoch (the reference copies every
prediction to the host for sklearn's jaccard_score and calls
torch.cuda.empty_cache() twice per step, Train_one_epoch.py:134,167,185); the
arithmetic and the logged quantities are the same:

  * loss    = WeightedDiceBCE(0.5, 0.5) (train_model.py:718), optimizer Adam(lr)
              over requires_grad parameters (train_model.py:647);
  * IoU     = iou_on_batch (utils.py:478-494): mean over the batch of the Jaccard
              index of (sigmoid(pred) >= 0.5) vs (mask > 0), 0 when both are empty
              (sklearn's zero_division default);
  * Dice    = criterion._show_dice (utils.py:149-158), double-sigmoid quirk kept;
  * epoch averages weight each batch by its size and divide by the images seen
              (Train_one_epoch.py:150-167);
  * the LR schedule (CosineAnnealingWarmRestarts(T_0=10, T_mult=1, eta_min=1e-5),
              train_model.py:740) is stepped once, at the end of the validation
              pass (Train_one_epoch.py:187-188 receives it only for validation);
  * best model: saved when val Dice improves, as
              {save_path}/best_model-{model_type}.pth.tar with the keys epoch,
              best_model, model, state_dict, val_loss, val_dice, optimizer
              (train_model.py:125-145, 796-811);
  * early stopping when epoch - best_epoch + 1 > patience (train_model.py:824-829);
  * resume: weights + optimizer from the best checkpoint, start_epoch = epoch + 1,
              max_dice = val_dice (train_model.py:676-690).
"""
from __future__ import annotations

import os
from typing import Iterable, Optional, Tuple

import torch

from .optim import CosineAnnealingWarmRestarts


# --------------------------------------------------------------------------- metrics
@torch.no_grad()
def iou_terms(masks: torch.Tensor, pred: torch.Tensor) -> torch.Tensor:
    """Per-sample Jaccard of the hard masks (utils.py:478-494) as a device tensor [B]."""
    p = torch.sigmoid(pred[:, 0].float()) >= 0.5
    m = (masks.reshape(p.shape) > 0)
    inter = (p & m).flatten(1).sum(1).double()
    union = (p | m).flatten(1).sum(1).double()
    return torch.where(union > 0, inter / union.clamp_min(1), torch.zeros_like(inter))


@torch.no_grad()
def iou_on_batch(masks: torch.Tensor, pred: torch.Tensor) -> float:
    return float(iou_terms(masks, pred).mean())


@torch.no_grad()
def dice_on_batch(masks: torch.Tensor, pred: torch.Tensor) -> float:
    """utils.py:503-519: mean hard Dice with smooth 1e-5 (float32, as the reference's
    numpy arrays are)."""
    p = (torch.sigmoid(pred[:, 0].float()) >= 0.5).float()
    m = (masks.reshape(p.shape) > 0).float()
    inter = (p * m).flatten(1).sum(1)
    d = (2.0 * inter + 1e-5) / (m.flatten(1).sum(1) + p.flatten(1).sum(1) + 1e-5)
    return float(d.mean())


# ----------------------------------------------------------------------- checkpoints
def checkpoint_filename(save_path: str, model_type: str, epoch: int, best: bool) -> str:
    if best:
        return os.path.join(save_path, f"best_model-{model_type}.pth.tar")
    return os.path.join(save_path, "model-{}-{:02d}.pth.tar".format(model_type, epoch))


def save_checkpoint(state: dict, save_path: str) -> str:
    """train_model.py:125-145: best_model-{model}.pth.tar or model-{model}-{epoch:02d}.pth.tar."""
    os.makedirs(save_path, exist_ok=True)
    fn = checkpoint_filename(save_path, state["model"], state["epoch"], state["best_model"])
    torch.save(state, fn)
    return fn


def load_checkpoint(path: str, map_location=None) -> dict:
    # our own files hold only tensors / numbers / strings: the safe loader suffices
    return torch.load(path, map_location=map_location, weights_only=True)


# --------------------------------------------------------------------------- trainer
class Trainer:
    """train_model.main_loop + Train_one_epoch.train_one_epoch for one model.

    `loader`s yield (sampled_batch, names) with sampled_batch = {'image': [B,C,H,W],
    'label': [B,H,W] or [B,1,H,W]} like the reference's DataLoader over
    ImageToImage2D (Load_Dataset.py:387-487).
    """

    def __init__(self, model: torch.nn.Module, model_type: str = "ACC_UNet",
                 save_path: str = "./models", lr: float = 1e-3, epochs: int = 1000,
                 early_stopping_patience: int = 100, criterion=None, optimizer=None,
                 lr_scheduler="cosine", device: Optional[torch.device] = None, logger=None,
                 reducer=None):
        """reducer: an accunet.dist.GradBucketReducer over `model` for data-parallel
        training (one process per GPU; its hooks all-reduce the gradients during each
        backward). The loop then zeroes gradients through it, keeping them views of
        its flat all-reduce buffer; without one the loop is single-process."""
        self.model = model
        self.reducer = reducer
        self.model_type = model_type
        self.save_path = save_path
        self.epochs = epochs
        self.patience = early_stopping_patience
        self.device = device if device is not None else next(model.parameters()).device
        if criterion is None:
            from .loss import WeightedDiceBCE
            criterion = WeightedDiceBCE(dice_weight=0.5, BCE_weight=0.5)
        self.criterion = criterion
        if optimizer is None:
            from .optim import FusedAdam
            optimizer = FusedAdam([p for p in model.parameters() if p.requires_grad], lr=lr)
        self.optimizer = optimizer
        if lr_scheduler == "cosine":
            lr_scheduler = CosineAnnealingWarmRestarts(optimizer, T_0=10, T_mult=1, eta_min=1e-5)
        self.lr_scheduler = lr_scheduler
        self.log = logger or (lambda msg: None)
        self.start_epoch = 0
        self.max_dice = 0.0
        self.best_epoch = 1
        self.history = []

    # ------------------------------------------------------------------ one pass
    def train_one_epoch(self, loader: Iterable, epoch: int, training: bool) -> Tuple[float, float]:
        """Returns (average_loss, average_dice) over the images of the pass."""
        model, crit = self.model, self.criterion
        model.train(training)
        loss_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        iou_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        dice_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        n = 0
        lr = min(g["lr"] for g in self.optimizer.param_groups)  # the LR this pass runs at
        ctx = torch.enable_grad() if training else torch.no_grad()
        with ctx:
            for sampled_batch, _names in loader:
                images = sampled_batch["image"].to(self.device, non_blocking=True)
                masks = sampled_batch["label"].to(self.device, non_blocking=True)
                if masks.dim() == 3:
                    masks = masks.unsqueeze(1)
                preds = model(images)
                if isinstance(preds, (tuple, list)):
                    preds = preds[0]
                loss = crit(preds, masks.float())
                if training:
                    if self.reducer is not None:
                        self.reducer.zero_grad()
                    else:
                        self.optimizer.zero_grad()
                    loss.backward()
                    self.optimizer.step()
                b = images.shape[0]
                with torch.no_grad():
                    iou_sum += iou_terms(masks, preds).mean() * b
                    dice = crit._show_dice(preds.detach(), masks.float())
                    dice_sum += torch.as_tensor(dice, dtype=torch.float64, device=self.device) * b
                    loss_sum += loss.detach().double() * b
                n += b
        if not training and self.lr_scheduler is not None:
            self.lr_scheduler.step()
        n = max(n, 1)
        avg_loss, avg_iou, avg_dice = (float(v) / n for v in (loss_sum, iou_sum, dice_sum))
        self.history.append(dict(epoch=epoch, mode="Train" if training else "Val", loss=avg_loss,
                                 iou=avg_iou, dice=avg_dice, lr=lr))
        return avg_loss, avg_dice

    # ---------------------------------------------------------------- main loop
    def resume(self, path: Optional[str] = None) -> bool:
        path = path or checkpoint_filename(self.save_path, self.model_type, 0, True)
        if not os.path.isfile(path):
            return False
        ck = load_checkpoint(path, map_location=self.device)
        self.model.load_state_dict(ck["state_dict"])
        self.optimizer.load_state_dict(ck["optimizer"])
        if isinstance(self.lr_scheduler, CosineAnnealingWarmRestarts):
            # the reference builds its scheduler AFTER optimizer.load_state_dict
            # (train_model.py:677 then :738): the fresh scheduler's first step puts every
            # group back at its initial_lr, so the first resumed epoch runs at base LR
            s = self.lr_scheduler
            self.lr_scheduler = CosineAnnealingWarmRestarts(self.optimizer, T_0=s.T_0,
                                                            T_mult=s.T_mult, eta_min=s.eta_min)
        self.start_epoch = ck["epoch"] + 1
        self.max_dice = float(ck.get("val_dice", 0.0))
        self.best_epoch = self.start_epoch
        self.log(f"resuming from epoch {ck['epoch']} (best dice {self.max_dice:.4f})")
        return True

    def fit(self, train_loader: Iterable, val_loader: Iterable) -> torch.nn.Module:
        for epoch in range(self.start_epoch, self.epochs):
            self.train_one_epoch(train_loader, epoch, training=True)
            val_loss, val_dice = self.train_one_epoch(val_loader, epoch, training=False)
            if val_dice > self.max_dice:
                self.log(f"saving best model, mean dice increased from {self.max_dice:.4f} "
                         f"to {val_dice:.4f}")
                self.max_dice = val_dice
                self.best_epoch = epoch + 1
                save_checkpoint({"epoch": epoch, "best_model": True, "model": self.model_type,
                                 "state_dict": self.model.state_dict(), "val_loss": val_loss,
                                 "val_dice": val_dice, "optimizer": self.optimizer.state_dict()},
                                self.save_path)
            early = epoch - self.best_epoch + 1
            if early > self.patience:
                self.log("early stopping")
                break
        return self.model
