#!/bin/bash
# r05u: march phase / event diagnostics at the step-1600 state with the exact empty-block skip off and on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for v in 0 1; do
  NEUS_MARCH_MACRO=$v WARM=1600 timeout -k 10 200 python -u scripts/diag_march_prof.py > gpurun_out/march_prof_m${v}_r05u.log 2>&1 || exit 1
  head -12 gpurun_out/march_prof_m${v}_r05u.log
done
echo ALL_OK
