"""The epoch loop around the training step (accunet/trainer.py), counterpart of
Experiments/train_model.py:663-831 and Train_one_epoch.py:48-201.

CPU: the device-side IoU / Dice metrics against the oracle restatement of
utils.py:478-519, and the loop logic (LR stepped once per validation pass, best
checkpoint name and keys, early stopping, resume) with a tiny torch model and the
oracle's loss. GPU: two epochs of ACC_UNet through the HIP kernels, checkpoint
round trip."""
import os
import sys

import pytest
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import accunet_oracle as O  # noqa: E402

from accunet import trainer as T  # noqa: E402
from accunet.optim import CosineAnnealingWarmRestarts  # noqa: E402

CK_KEYS = {"epoch", "best_model", "model", "state_dict", "val_loss", "val_dice", "optimizer"}


class OracleLoss(nn.Module):
    """WeightedDiceBCE(0.5, 0.5) as restated by the oracle (CPU criterion for the loop test)."""

    def forward(self, inputs, targets):
        return O.dice_bce_loss(inputs, targets)

    def _show_dice(self, inputs, targets):
        return O.show_dice(inputs, targets)


def _loader(n_batches, B, seed, H=16, ch=1):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n_batches):
        x = torch.randn(B, ch, H, H, generator=g)
        m = (torch.rand(B, H, H, generator=g) < 0.4).long()  # [B,H,W] like Load_Dataset.py:485
        out.append(({"image": x, "label": m}, [f"img{i}_{j}.npy" for j in range(B)]))
    return out


@pytest.mark.parametrize("p_mask", [0.0, 0.3, 1.0])
def test_metrics_match_oracle(p_mask):
    g = torch.Generator().manual_seed(3)
    pred = torch.randn(5, 1, 12, 12, generator=g) * 2
    masks = (torch.rand(5, 1, 12, 12, generator=g) < p_mask).float()
    masks[0] = 0  # an empty mask
    pred[0] = -5  # ... with an empty prediction: IoU 0 (sklearn zero_division)
    assert abs(T.iou_on_batch(masks, pred) - O.iou_on_batch(masks.clone(), pred)) < 1e-12
    assert abs(T.dice_on_batch(masks, pred) - O.dice_on_batch(masks.clone(), pred)) < 1e-6


def test_loop_schedule_checkpoint_early_stop_resume(tmp_path):
    torch.manual_seed(0)
    model = nn.Sequential(nn.Conv2d(1, 4, 3, padding=1), nn.LeakyReLU(), nn.Conv2d(4, 1, 1))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    tr = T.Trainer(model, "TinyNet", str(tmp_path), epochs=40, early_stopping_patience=2,
                   criterion=OracleLoss(), optimizer=opt, device=torch.device("cpu"))
    train, val = _loader(3, 2, 1), _loader(2, 2, 2)
    tr.fit(train, val)
    vals = [h for h in tr.history if h["mode"] == "Val"]
    n_ep = len(vals)
    # early stopping: the loop ends once epoch - best_epoch + 1 > patience (or at 40)
    assert n_ep < 40 or tr.best_epoch >= 38
    assert n_ep - 1 - tr.best_epoch + 1 > 2 or n_ep == 40
    # the LR of validation epoch e is the schedule at e (stepped after each val pass)
    for h in vals:
        assert abs(h["lr"] - O.cosine_warm_restarts_lr(1e-3, 1e-5, 10, h["epoch"])) < 1e-12
    assert abs(opt.param_groups[0]["lr"] - O.cosine_warm_restarts_lr(1e-3, 1e-5, 10, n_ep)) < 1e-12
    # averages weight batches by their size: the train loss is the mean over images
    # best checkpoint: file name and keys of train_model.py:125-145
    fn = os.path.join(str(tmp_path), "best_model-TinyNet.pth.tar")
    assert os.path.isfile(fn)
    ck = T.load_checkpoint(fn)
    assert set(ck) == CK_KEYS
    assert ck["best_model"] is True and ck["model"] == "TinyNet"
    assert ck["epoch"] == tr.best_epoch - 1
    assert abs(ck["val_dice"] - tr.max_dice) < 1e-15
    # resume: weights + optimizer state restored, start epoch after the best one
    torch.manual_seed(1)
    model2 = nn.Sequential(nn.Conv2d(1, 4, 3, padding=1), nn.LeakyReLU(), nn.Conv2d(4, 1, 1))
    opt2 = torch.optim.Adam(model2.parameters(), lr=1e-3)
    tr2 = T.Trainer(model2, "TinyNet", str(tmp_path), criterion=OracleLoss(), optimizer=opt2,
                    lr_scheduler=None, device=torch.device("cpu"))
    assert tr2.resume()
    assert tr2.start_epoch == ck["epoch"] + 1 and tr2.best_epoch == tr2.start_epoch
    for k, v in ck["state_dict"].items():
        assert torch.equal(model2.state_dict()[k], v)
    assert opt2.state_dict()["state"][0]["exp_avg"].shape == model2[0].weight.shape


def test_resume_restarts_cosine_schedule_at_base_lr(tmp_path):
    """train_model.py:677,738: the scheduler is built after optimizer.load_state_dict,
    so a resumed run's first epoch uses initial_lr, not the checkpoint's mid-cycle LR."""
    torch.manual_seed(0)
    model = nn.Conv2d(1, 1, 3, padding=1)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    sched = CosineAnnealingWarmRestarts(opt, T_0=10, T_mult=1, eta_min=1e-5)
    for _ in range(4):
        sched.step()
    assert opt.param_groups[0]["lr"] < 1e-3 * 0.9  # mid-cycle
    T.save_checkpoint({"epoch": 3, "best_model": True, "model": "T",
                       "state_dict": model.state_dict(), "val_loss": 0.0, "val_dice": 0.5,
                       "optimizer": opt.state_dict()}, str(tmp_path))
    model2 = nn.Conv2d(1, 1, 3, padding=1)
    opt2 = torch.optim.Adam(model2.parameters(), lr=1e-3)
    tr = T.Trainer(model2, "T", str(tmp_path), criterion=OracleLoss(), optimizer=opt2,
                   device=torch.device("cpu"))
    assert tr.resume()
    assert opt2.param_groups[0]["lr"] == 1e-3
    assert abs(opt2.param_groups[0]["lr"] - O.cosine_warm_restarts_lr(1e-3, 1e-5, 10, 0)) < 1e-15
    tr.lr_scheduler.step()
    assert abs(opt2.param_groups[0]["lr"] - O.cosine_warm_restarts_lr(1e-3, 1e-5, 10, 1)) < 1e-15


def test_epoch_average_is_per_image(tmp_path):
    model = nn.Conv2d(1, 1, 1)
    crit = OracleLoss()
    tr = T.Trainer(model, "T", str(tmp_path), criterion=crit,
                   optimizer=torch.optim.SGD(model.parameters(), lr=0.0), lr_scheduler=None,
                   device=torch.device("cpu"))
    batches = _loader(2, 3, 5) + _loader(1, 1, 6)  # ragged last batch
    loss, dice = tr.train_one_epoch(batches, 0, training=False)
    want_l = sum(float(crit(model(b["image"]), b["label"].unsqueeze(1).float())) * b["image"].shape[0]
                 for b, _ in batches) / 7
    assert abs(loss - want_l) < 1e-9


@pytest.mark.gpu
def test_trainer_acc_unet_gpu(tmp_path):
    from accunet.model import ACC_UNet
    dev = torch.device("cuda")
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, 8), seed=0)
    model = ACC_UNet(3, 1, n_filts=8)
    model.load_state_dict(sd)
    model = model.to(dev)
    tr = T.Trainer(model, "ACC_UNet", str(tmp_path), epochs=2, early_stopping_patience=100)
    train, val = _loader(2, 2, 11, H=32, ch=3), _loader(1, 2, 12, H=32, ch=3)
    # the first training batch's loss is the oracle's loss on the same weights
    b0 = train[0][0]
    ref = O.dice_bce_loss(O.forward({k: v.double() if v.is_floating_point() else v
                                     for k, v in sd.items()}, b0["image"].double(), "canonical",
                                    training=True), b0["label"].unsqueeze(1).double())
    model.train(True)
    got = tr.criterion(model(b0["image"].to(dev)), b0["label"].unsqueeze(1).float().to(dev))
    assert abs(float(got) - float(ref)) < 1e-5
    model.load_state_dict(sd)  # undo the BN running-stat update of that check
    tr.fit(train, val)
    assert len(tr.history) == 4
    assert all(h["loss"] == h["loss"] for h in tr.history)
    fn = os.path.join(str(tmp_path), "best_model-ACC_UNet.pth.tar")
    # the canonical head outputs probabilities, so _show_dice's second sigmoid makes
    # the hard mask all-ones: val Dice = 2|m|/(|m|+N) > 0 for any
    # non-empty mask, the first validation pass always improves on 0 and saves
    assert tr.max_dice > 0
    ck = T.load_checkpoint(fn)
    assert set(ck) == CK_KEYS
    m2 = ACC_UNet(3, 1, n_filts=8).to(dev)
    tr2 = T.Trainer(m2, "ACC_UNet", str(tmp_path))
    assert tr2.resume()
    for k, v in ck["state_dict"].items():
        assert torch.equal(m2.state_dict()[k].cpu(), v.cpu())
    # the restored optimizer state drives the next HIP Adam step
    tr2.train_one_epoch(train, tr2.start_epoch, training=True)
    assert all(torch.isfinite(p).all() for p in m2.parameters())


def test_eval_metrics_match_test_model_restatement():
    from accunet.evaluate import image_dice_iou
    g = torch.Generator().manual_seed(9)
    out = torch.rand(4, 1, 10, 10, generator=g)
    lab = (torch.rand(4, 10, 10, generator=g) < 0.4).long()
    lab[0] = 0
    out[0] = 0.2  # both empty: dice 0 (no numerator smoothing), IoU 0
    d, i = image_dice_iou(out, lab)
    for b in range(4):
        rd, ri = O.test_image_dice_iou(out[b], lab[b])
        assert abs(float(d[b]) - rd) < 1e-6 and abs(float(i[b]) - ri) < 1e-12


@pytest.mark.gpu
def test_evaluate_acc_unet_gpu(tmp_path):
    from accunet.evaluate import evaluate, image_dice_iou, load_best
    from accunet.model import ACC_UNet
    sd = O.det_state_dict(O.param_spec("canonical", 3, 1, 8), seed=0)
    m = ACC_UNet(3, 1, n_filts=8).cuda()
    m.load_state_dict(sd)
    torch.save({"epoch": 0, "best_model": True, "model": "ACC_UNet", "state_dict": m.state_dict(),
                "val_loss": 0.0, "val_dice": 0.0, "optimizer": {}},
               os.path.join(str(tmp_path), "best_model-ACC_UNet.pth.tar"))
    m2 = load_best(ACC_UNet(3, 1, n_filts=8).cuda(),
                   os.path.join(str(tmp_path), "best_model-ACC_UNet.pth.tar"))
    batches = _loader(3, 2, 21, H=32, ch=3)
    r = evaluate(m2, batches)
    assert r["n"] == 6 and 0 <= r["dice"] <= 1 and 0 <= r["iou"] <= 1
    # the same numbers from the oracle metric on the HIP outputs, one image at a time
    ds, ios = [], []
    with torch.no_grad():
        for b, _ in batches:
            out = m2.eval()(b["image"].cuda())
            for j in range(out.shape[0]):
                dd, ii = O.test_image_dice_iou(out[j], b["label"][j])
                ds.append(dd)
                ios.append(ii)
    assert abs(r["dice"] - sum(ds) / 6) < 1e-6 and abs(r["iou"] - sum(ios) / 6) < 1e-9
