#!/usr/bin/env python3
"""GPU box: the engine works when riptide_amd is imported before torch (the
engine library must bind torch's HIP runtime, riptide_amd/_lib.py load)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import riptide_amd  # noqa: E402  (before torch on purpose)
import torch  # noqa: E402

x = np.random.RandomState(3).normal(size=20000).astype(np.float32)
y = riptide_amd.downsample(x, 7.3)
t = torch.ones(4, device="cuda")
print("import order ok", y.shape, float(t.sum()))
