"""Locate the in-tree native libraries (built by __graft_entry__.build())."""
from __future__ import annotations

import os

# BNFLAC_LIB_DIR: a development build variant instead (build.py BNFLAC_VARIANT_DIR)
LIB_DIR = os.environ.get("BNFLAC_LIB_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")


def lib_path(name: str) -> str:
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{name} not built: run `python -c 'import __graft_entry__ as g; g.build()'` (looked in {LIB_DIR})")
    return path
