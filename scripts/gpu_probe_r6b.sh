set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
timeout -k 10 60 scripts/probe/fgs_rows > gpurun_out/r6b/fgs_rows.txt 2>&1 &&
timeout -k 10 120 scripts/probe/copy_rate > gpurun_out/r6b/copy_rate.txt 2>&1
echo done
