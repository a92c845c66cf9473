"""The parts of r2r_src/utils.py the policy path uses (angle features, masks); the tokenizers,
feature readers and graph utilities stay with the reference."""
import math

import numpy as np
import torch

from .param import args

padding_idx = 0   # base_vocab.index('<PAD>') (utils.py:22-24); BERT [PAD] is 0 too


def angle_feature(heading, elevation):
    """utils.py:361-368."""
    return np.array([math.sin(heading), math.cos(heading), math.sin(elevation), math.cos(elevation)]
                    * (args.angle_feat_size // 4), dtype=np.float32)


def length2mask(length, size=None, device=None):
    """utils.py:503-508: True where index > len-1, on the compute device."""
    size = int(max(length)) if size is None else size
    lens = torch.as_tensor(list(length), dtype=torch.int64)
    mask = torch.arange(size, dtype=torch.int64).unsqueeze(0) > (lens - 1).unsqueeze(1)
    # pinned + non_blocking: the copy is queued on the stream instead of syncing the host with it
    return mask.pin_memory().to(device if device is not None else torch.device("cuda"), non_blocking=True)
