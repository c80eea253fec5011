"""Generate tests/golden/learner_aug_pixels.npz by running the REFERENCE `helper.RandomShiftsAug` in this container.

Run once in the build container (where /root/reference exists):   python tests/golden/make_aug_golden.py
Imports the reference like make_golden.py (rlpyt stub; CPU). Inputs: seeded uint8-valued float frames, a 4-D
batch [2, 9, 84, 84] and a 5-D horizon batch [1, 2, 9, 84, 84]; torch.manual_seed(11) before each call fixes the
shift draw. The .npz holds the inputs and the reference's outputs.
"""
from __future__ import annotations

import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import import_reference  # noqa: E402


def main():
    import_reference()
    import algorithm.helper as h
    cfg = SimpleNamespace(img_size=84, modality="pixels")
    aug = h.RandomShiftsAug(cfg)
    rs = np.random.RandomState(0)
    x4 = rs.randint(0, 256, size=(2, 9, 84, 84)).astype(np.float32)
    x5 = rs.randint(0, 256, size=(1, 2, 9, 84, 84)).astype(np.float32)
    torch.manual_seed(11)
    y4 = aug(torch.from_numpy(x4)).numpy()
    torch.manual_seed(11)
    y5 = aug(torch.from_numpy(x5)).numpy()
    np.savez_compressed(os.path.join(HERE, "learner_aug_pixels.npz"), x4=x4.astype(np.uint8), y4=y4,
                        x5=x5.astype(np.uint8), y5=y5)
    print("wrote learner_aug_pixels.npz", y4.shape, y5.shape)


if __name__ == "__main__":
    main()
