#!/bin/bash
# k_fgs_lr's lines-a-workgroup cap on C4's default line (6 frames in flight), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_maxl6}
mkdir -p $O
for rep in 1 2; do
  for m in 16 8 4; do
    SDR_FGS_LR_MAXL=$m timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --no-cpu-baseline \
        --no-stream-probe --no-kernel-timing > $O/c4_m${m}_$rep.json 2> $O/c4_m${m}_$rep.err || exit 1
  done
done
echo maxl6-done
