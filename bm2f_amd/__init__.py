"""bm2f_amd — MI355X-native (gfx950) Mask2Former pixel-decoder + transformer-decoder hot path.

Drop-in for the reference's (wenhe-jia/BM2F) MSDeformAttn op, MSDeformAttnPixelDecoder and
MultiScaleMaskedTransformerDecoder, backed by hand-written HIP kernels in ``bm2f_amd/csrc`` reached
through the C ABI of ``include/bm2f.h``.
"""
import os as _os

# HIP graphs (bench_model.GraphStep): on this ROCm the runtime's graph packet capture replays captured memset nodes
# incorrectly (torch's cross-workgroup reductions zero their semaphores with one), so every replay after the first
# computes wrong sums; with the packet capture off they replay correctly (tools/graph_memset_check.py).  Read when
# the HIP runtime initialises, so it must be set before the first device call; an explicit setting wins.
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from . import _native  # noqa: F401,E402
from .msda import MSDeformAttn, MSDeformAttnFunction, ms_deform_attn_backward, ms_deform_attn_forward  # noqa: F401,E402

__version__ = "0.1.0"
