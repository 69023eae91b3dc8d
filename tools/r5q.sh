#!/bin/bash
# round 5: is C2's decode bound by HBM traffic?  The same instructions with the PCM stores or the
# CRC re-read moved to L2-resident windows (timing ablations 0x10000000 / 0x40000000), against
# removing them (2 / 1)
mkdir -p gpurun_out
ENVS="BNFLAC_ABLATE=0;BNFLAC_ABLATE=0x10000000;BNFLAC_ABLATE=0x40000000;BNFLAC_ABLATE=0x50000000;BNFLAC_ABLATE=1;BNFLAC_ABLATE=2;BNFLAC_ABLATE=3" CFGS="C2" ROUNDS=1 TAG=ab5q bash tools/ab_env.sh
