#!/bin/bash
# End-of-session evidence: __graft_entry__.smoke() on cuda:0, then the full round pass (scripts/gpu_round.sh).
# Usage: bash scripts/gpu_final.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-final}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash scripts/gpu_round.sh $TAG
