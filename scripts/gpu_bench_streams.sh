#!/bin/bash
# Compare frames-in-flight settings of bench.py on one GPU (no CPU baseline).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-bs}
mkdir -p "$O"
for s in 1 2 3; do
  timeout -k 10 200 python3 bench.py --streams $s --no-cpu-baseline > "$O/s$s.json" 2> "$O/s$s.err"
  python3 -c "import json;d=json.load(open('$O/s$s.json'));print('streams',$s,'fps',d['fps'],'paths_us',d['roofline']['avg_launch_us'],'frac',d['roofline']['frac'])"
done
