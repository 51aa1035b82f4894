"""INTEGRATION.md §2 end to end, in a fresh interpreter (tests/registry_dropin_check.py): the reference's own
build_pixel_decoder / build_transformer_decoder return the bm2f classes after the documented import, a
reference state_dict loads strictly, and the outputs match the reference's fixtures.  Needs /root/reference
(this container); skipped where the reference is absent (the GPU box)."""
import os
import subprocess
import sys

import pytest

REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "mask2former")), reason="reference tree absent")
def test_registry_dropin_with_reference_builders():
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "registry_dropin_check.py"), REF], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "registry drop-in ok" in r.stdout
