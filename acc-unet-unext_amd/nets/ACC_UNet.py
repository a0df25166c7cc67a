"""Drop-in for the reference's `from nets.ACC_UNet import ACC_UNet`
(Experiments/train_model.py:24, test_model.py:25): the script variant
(Experiments/nets/ACC_UNet.py:530 — cnv72 inv_fctr 3, raw logits), running on the
MI355X kernels of accunet. The canonical model is accunet.model.ACC_UNet.
"""
from accunet.model import (ACC_UNet_Script as ACC_UNet, ChannelSELayer, Conv2d_batchnorm,  # noqa: F401
                           Conv2d_channel, HANCBlock, HANCLayer, MLFC, ResPath)
