"""Shipped MIOpen find-db for the benchmark's convolutions (backbone and pixel-decoder FPN).

MIOpen's FAST find mode (no search; the bench's default so a fresh box starts in seconds) falls back
to a heuristic solver choice that is up to 25 % slower on several of this model's convolutions than
what a NORMAL-mode search picks (measured: 278.7 -> 267 ms per step).  FAST mode does consult the user
find-db first, so ``bm2f_amd/miopen_db/`` holds the find-db a NORMAL-mode run wrote on an MI355X with
this image's MIOpen (the file name carries the MIOpen version; other versions or shapes simply miss
and use the heuristic).  Regenerate with::

    MIOPEN_FIND_MODE=NORMAL MIOPEN_USER_DB_PATH=<dir> python bench.py --steps 2 --warmup 1

and copy ``<dir>/*.ufdb.txt`` here.
"""
from __future__ import annotations

import atexit
import glob
import os
import shutil
import tempfile

DB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")


def use_shipped_find_db() -> str | None:
    """Point MIOpen at a private copy of the shipped find-db (FAST mode) unless the caller already chose
    a db path / find mode.  Call before the first convolution.  Returns the db directory in use."""
    os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
    if "MIOPEN_USER_DB_PATH" in os.environ:
        return os.environ["MIOPEN_USER_DB_PATH"]
    files = glob.glob(os.path.join(DB_DIR, "*.ufdb.txt"))
    if not files:
        return None
    tmp = tempfile.mkdtemp(prefix="bm2f_miopen_db_")   # private: MIOpen may touch the db's timestamps
    for f in files:
        shutil.copy(f, tmp)
    atexit.register(shutil.rmtree, tmp, True)
    os.environ["MIOPEN_USER_DB_PATH"] = tmp
    return tmp
