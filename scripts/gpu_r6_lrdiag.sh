#!/bin/bash
# k_fgs_lr diagnostics: the stamps of the default build, with every chunk preloaded (SDR_LR_PRELOAD)
# and with one solver wave (SDR_LR_ONE_SOLVER)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_lrdiag}
mkdir -p $O
for v in thstamps lrpre lrone; do
  timeout -k 10 120 python -u scripts/lr_stamps.py stereo_depth_ruler_amd/lib/libsdr-$v.so > $O/stamps_$v.txt 2>&1 || exit 1
done
echo diag-done
