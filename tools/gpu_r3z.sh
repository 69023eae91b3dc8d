#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PYTHONPATH=. timeout -k 10 120 python tools/dbg_sw_qf.py
