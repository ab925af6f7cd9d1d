#!/bin/bash
# gpu_final.sh followed by the C2 PMC passes (single stream), for the round's profiles/.
# usage (via gpurun): bash scripts/gpu_final2.sh <tag>
set -e
TAG=${1:-fin}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 bash scripts/gpu_final.sh "$TAG"
timeout -k 10 300 bash scripts/pmc_profile.sh "gpurun_out/$TAG/pmc"
