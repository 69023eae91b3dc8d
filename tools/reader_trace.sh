#!/bin/bash
# Streaming-reader phases on one C2 stream (1024 frames): tools/reader_bench best-of-10 totals
# with the decode on the lane kernels and on k_decode_sys, then one traced open per setting
# (BNFLAC_READER_TRACE=1: device-synchronised phase times, so they add up to more than the
# untraced open).  Writes gpurun_out/c2_stream.flac.
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
for e in 0 1; do
  echo "BNFLAC_DECODE_SYS=$e"
  BNFLAC_DECODE_SYS=$e timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 10 16384 2
  BNFLAC_DECODE_SYS=$e BNFLAC_READER_TRACE=1 timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 2 16384 2 2>&1 | tail -8
done
