set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== prod" >> gpurun_out/dbg.log
timeout -k 5 120 python -u scripts/fold_debug.py >> gpurun_out/dbg.log 2>&1
echo "rc=$?" >> gpurun_out/dbg.log
