#!/bin/bash
# A/B on one box: k_fgs_lr's lines a workgroup capped (SDR_FGS_LR_MAXL 16: the column pass takes 16,
# 8: it takes 8 like the row pass), C4 on one stream, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_maxl}
mkdir -p $O
for rep in 1 2; do
  for m in ${MS:-16 8}; do
    SDR_FGS_LR_MAXL=$m timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 \
        --no-cpu-baseline --no-stream-probe > $O/c4s1_m${m}_$rep.json 2> $O/c4s1_m${m}_$rep.err || exit 1
  done
done
SDR_FGS_LR_MAXL=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_wls.py -m gpu -q -x --timeout 240 \
    --timeout-method thread > $O/tests_m8.log 2>&1
echo maxl-done
