#!/bin/bash
# Reader frame records sized from STREAMINFO: the reader GPU tests, then tools/reader_bench on
# one C2 stream (best of 20, twice) and one traced open/close.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "reader or filereader or stream" > gpurun_out/r5cap_pytest.log 2>&1 || { tail -30 gpurun_out/r5cap_pytest.log; exit 1; }
tail -2 gpurun_out/r5cap_pytest.log
python3 - <<'PY'
import sys
sys.path.insert(0, ".")
from birdnest.audio_amd import synth
s = synth.encode(synth.config("C2", nframes=1024, seed=2))
open("gpurun_out/c2_stream.flac", "wb").write(s.data.tobytes())
PY
for pass in 1 2; do
  timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 20 16384 2
done
BNFLAC_READER_TRACE=1 timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 3 16384 2 2>&1 | tail -9
rm -f gpurun_out/c2_stream.flac
