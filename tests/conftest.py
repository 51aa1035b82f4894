import os
import sys

# HIP graph replays need the runtime's graph packet capture off on this ROCm (bm2f_amd/__init__.py); set before any
# test initialises the device
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

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
    in fp64, so such samples can sit on different sides: their grad_loc entries are checked by
    :func:`check_crossing_entries` against the oracle's one-sided values (expected fraction ~4 eps per
    coordinate pair)."""
    import numpy as np
    loc = np.asarray(loc, dtype=np.float64)
    L = loc.shape[3]
    wh = np.array([[w, h] for h, w in shapes], dtype=np.float64).reshape((1,) * 3 + (L, 1, 2))
    pix = loc * wh - 0.5
    amb = (np.abs(pix - np.round(pix)) < eps).any(-1, keepdims=True)
    return np.broadcast_to(amb, loc.shape)


def check_crossing_entries(got, value, shapes, level_start_index, loc, attn, grad_out, amb, to_cmp=None,
                           delta_px=3e-4, rtol=1e-3, atol_frac=1e-4, scale=None, eps=1e-4):
    """Check the grad_loc entries ``loc_crossing_mask`` flags (where d loc jumps at a pixel-centre line) against
    the C oracle evaluated just on either side of the line: each such entry must match one side's value.

    d f / d x is piecewise constant in x across a bilinear cell and continuous across y lines (and vice
    versa), so shifting every coordinate that lies within ``eps`` of a line by -delta and by +delta px gives
    the two one-sided gradients of every flagged entry at once (only those coordinates move: d f / d y
    changes with x inside a cell, so moving a sample's other coordinate would shift its other entry).  The oracle runs only on the queries that hold a flagged
    sample (a sample's grad_loc depends on its own location alone).  ``to_cmp`` maps an oracle grad_loc
    array (n, q, M, L, P, 2) to the layout of ``got`` (e.g. d offsets = d loc / (W, H)); ``got`` is
    (N, Lq, ...) in that layout; ``scale`` (default: the largest one-sided value) is the atol reference, as
    the caller's comparison of the other entries uses the whole tensor's max."""
    import numpy as np
    import torch
    from oracle import msda_ref
    loc = np.asarray(loc, dtype=np.float64)
    amb = np.asarray(amb)
    N, Lq = loc.shape[:2]
    L = loc.shape[3]
    to_cmp = to_cmp or (lambda a: a)
    wh = np.array([[w, h] for h, w in shapes], dtype=np.float64).reshape((1,) * 3 + (L, 1, 2))
    checked = 0
    for n in range(N):
        qs = np.nonzero(amb[n].reshape(Lq, -1).any(-1))[0]
        if len(qs) == 0:
            continue
        sub = loc[n:n + 1, qs]
        a_sub = amb[n:n + 1, qs].astype(np.float64)
        pix = sub * wh - 0.5
        near = (np.abs(pix - np.round(pix)) < eps).astype(np.float64)   # per coordinate
        sides = []
        for sign in (-1.0, 1.0):
            shifted = sub + sign * near * (delta_px / wh)
            _, gl, _ = msda_ref.msda_backward(torch.as_tensor(np.asarray(value[n:n + 1], dtype=np.float64)),
                                              shapes_tensor(shapes), level_start_index,
                                              torch.as_tensor(shifted),
                                              torch.as_tensor(np.asarray(attn[n:n + 1, qs], dtype=np.float64)),
                                              torch.as_tensor(np.asarray(grad_out[n:n + 1, qs], dtype=np.float64)))
            sides.append(np.asarray(to_cmp(gl), dtype=np.float64)[0])
        g = np.asarray(got, dtype=np.float64)[n, qs].reshape(sides[0].shape)
        sel = np.asarray(to_cmp(np.broadcast_to(a_sub, sub.shape).copy()))[0].reshape(sides[0].shape) > 0
        sc = scale if scale is not None else max(max(np.abs(s_).max() for s_ in sides), 1e-30)
        ok = np.zeros(g.shape, dtype=bool)
        for s_ in sides:
            ok |= np.abs(g - s_) <= atol_frac * sc + rtol * np.abs(s_)
        bad = sel & ~ok
        if bad.any():
            err = np.minimum(np.abs(g - sides[0]), np.abs(g - sides[1]))[bad] / sc
            raise AssertionError(f"{int(bad.sum())} of {int(sel.sum())} crossing entries match neither side (image "
                                 f"{n}): nearest-side error / scale {np.sort(err)[-5:]}, got {g[bad][:5]}, sides "
                                 f"{sides[0][bad][:5]} / {sides[1][bad][:5]}")
        checked += int(sel.sum())
    return checked


def shapes_tensor(shapes):
    import torch
    return torch.tensor(shapes, dtype=torch.int64)
