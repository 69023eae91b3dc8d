#!/bin/bash
# Reader open: pageable H2D vs pinned staging (BNFLAC_READER_STAGE chunk KiB), one C2 stream,
# tools/reader_bench best of 20, two interleaved passes; then the reader GPU tests.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python3 - <<'PY'
import sys
sys.path.insert(0, ".")
from birdnest.audio_amd import synth
s = synth.encode(synth.config("C2", nframes=1024, seed=2))
open("gpurun_out/c2_stream.flac", "wb").write(s.data.tobytes())
PY
for pass in 1 2; do
  for st in 0 256 512 1024 2048 4096; do
    echo -n "stage=$st "
    BNFLAC_READER_STAGE=$st timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 20 16384 2
  done
done
BNFLAC_READER_STAGE=1024 BNFLAC_READER_TRACE=1 timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 2 16384 2 2>&1 | tail -8
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "reader or filereader or stream" > gpurun_out/r5stage_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5stage_pytest.log; exit $rc
