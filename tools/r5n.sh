#!/bin/bash
# round 5: same-box A/B of the committed build (_var/base) against the working tree's
mkdir -p gpurun_out
ENVS="BNFLAC_LIB_DIR=/root/repo/_var/base;BNFLAC_LIB_DIR=/root/repo/birdnest/audio_amd/lib" CFGS="C2 C3 C4" ROUNDS=2 TAG=ab5n bash tools/ab_env.sh
