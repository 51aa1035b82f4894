import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def loc_crossing_mask(loc, shapes, eps=1e-4):
    """Bool (N, Lq, M, L, P, 2): samples within `eps` px of a pixel-centre line of their level.

    d value / d loc is discontinuous there (the bilinear corner pair changes).  Kernels derive the pixel
    coordinate in fp32 (loc * W - 0.5, contracted to one FMA as the reference's CUDA build does), the oracle
    in fp64, so such samples can sit on different sides: their grad_loc entries are compared separately
    (expected fraction ~4 eps per coordinate pair)."""
    import numpy as np
    loc = np.asarray(loc, dtype=np.float64)
    L = loc.shape[3]
    wh = np.array([[w, h] for h, w in shapes], dtype=np.float64).reshape((1,) * 3 + (L, 1, 2))
    pix = loc * wh - 0.5
    amb = (np.abs(pix - np.round(pix)) < eps).any(-1, keepdims=True)
    return np.broadcast_to(amb, loc.shape)
