"""The CPU oracle (oracle/) against the golden vectors generated from the reference itself.

Pins both restatements: the C loops (oracle/msda_ref.c) and the grid_sample restatement
(oracle.msda_ref.core_pytorch) of ms_deform_attn_core_pytorch (ops/functions/ms_deform_attn_func.py:52-72).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import msda_ref


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_testpy_fixture(tag):
    g = golden("msda_testpy.npz")
    shapes, lsi = g["shapes"], g["level_start_index"]
    v, loc, a, gout = (g[f"{tag}_{k}"] for k in ("value", "loc", "attn", "grad_out"))
    out = msda_ref.msda_forward(v, shapes, lsi, loc, a)
    # test.py:44 uses allclose defaults in fp64; :57 rtol 1e-2 atol 1e-3 in fp32 -- we hold tighter bounds
    tol = dict(rtol=1e-12, atol=1e-15) if tag == "f64" else dict(rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out, g[f"{tag}_out"], **tol)
    gv, gl, ga = msda_ref.msda_backward(v, shapes, lsi, loc, a, gout)
    np.testing.assert_allclose(gv, g[f"{tag}_grad_value"], **tol)
    np.testing.assert_allclose(gl, g[f"{tag}_grad_loc"], **tol)
    np.testing.assert_allclose(ga, g[f"{tag}_grad_attn"], **tol)


@pytest.mark.parametrize("variant", ["uniform", "local"])
def test_slice_fixture(variant):
    g = golden("msda_slice.npz")
    shapes, lsi = g["shapes"], g["level_start_index"]
    v, loc, a, gout = (g[f"{variant}_{k}"].astype(np.float64) for k in ("value", "loc", "attn", "grad_out"))
    out = msda_ref.msda_forward(v, shapes, lsi, loc, a)
    np.testing.assert_allclose(out, g[f"{variant}_out"], rtol=1e-5, atol=1e-6)
    gv, gl, ga = msda_ref.msda_backward(v, shapes, lsi, loc, a, gout)
    np.testing.assert_allclose(gv, g[f"{variant}_grad_value"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ga, g[f"{variant}_grad_attn"], rtol=1e-5, atol=1e-6)
    # grad wrt location is discontinuous where a sample crosses a pixel centre; the fixtures are random
    # reals so no sample sits on one, and the restatement matches grid_sample's gradient there too
    np.testing.assert_allclose(gl, g[f"{variant}_grad_loc"], rtol=1e-5, atol=1e-5)


def test_core_pytorch_matches_fixture():
    g = golden("msda_slice.npz")
    shapes = torch.from_numpy(g["shapes"])
    v, loc, a = (torch.from_numpy(g[f"uniform_{k}"]).double() for k in ("value", "loc", "attn"))
    out = msda_ref.core_pytorch(v, shapes, loc, a)
    np.testing.assert_allclose(out.numpy(), g["uniform_out"], rtol=1e-5, atol=1e-6)
