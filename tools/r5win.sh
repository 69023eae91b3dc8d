#!/bin/bash
# Reader window size (frames per D2H window) A/B on one C2 stream: tools/reader_bench best of 20.
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
  for w in 16 32 64 128 256 512; do
    echo -n "window=$w "
    timeout -k 10 60 tools/reader_bench gpurun_out/c2_stream.flac 20 16384 2 $w
  done
done
rm -f gpurun_out/c2_stream.flac
