#!/bin/bash
# C3 batches in flight (streams) 2 / 3 / 4 on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_c3streams}
mkdir -p $O
for s in 3 4 2 3 4; do
  timeout -k 10 300 python -u bench.py --config c3 --streams $s --steps 60 --warmup 8 --no-cpu-baseline --no-stream-probe \
      --no-kernel-timing > $O/c3_s${s}_$RANDOM.json 2> $O/c3_s$s.err || exit 1
done
echo c3s-done
