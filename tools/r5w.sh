#!/bin/bash
# round 5: C3 (k_decode_sw) -- PCM stores removed (2) against the same stores into an
# L2-resident window (0x10000000) and per-lane 16-byte stores instead of the line flush (0x20000000)
mkdir -p gpurun_out
ENVS="BNFLAC_ABLATE=0;BNFLAC_ABLATE=0x10000000;BNFLAC_ABLATE=2;BNFLAC_ABLATE=0x20000000;BNFLAC_ABLATE=0x40000000" CFGS="C3" ROUNDS=1 TAG=ab5w bash tools/ab_env.sh
