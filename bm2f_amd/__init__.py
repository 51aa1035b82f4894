"""bm2f_amd — MI355X-native (gfx950) Mask2Former pixel-decoder + transformer-decoder hot path.

Drop-in for the reference's (wenhe-jia/BM2F) MSDeformAttn op, MSDeformAttnPixelDecoder and
MultiScaleMaskedTransformerDecoder, backed by hand-written HIP kernels in ``bm2f_amd/csrc`` reached
through the C ABI of ``include/bm2f.h``.
"""
from . import _native  # noqa: F401
from .msda import MSDeformAttn, MSDeformAttnFunction, ms_deform_attn_backward, ms_deform_attn_forward  # noqa: F401

__version__ = "0.1.0"
