#!/bin/bash
# decode / rows tests + figures, then the storage-row kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_dec_figs.sh || exit $?
SERIES=100000 bash scripts/gpu_rows_prof.sh > gpurun_out/rows_prof.out 2>&1 || { tail -5 gpurun_out/rows_prof.out; exit 1; }
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/ks_rows/ks_kernel_stats.csv")))[:6]:
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3))
PY
