#!/bin/bash
# Perf iteration on the box (development): optional bitwise regression check against a golden fingerprint
# (scripts/golden_params.py), then a rocprofv3 kernel-trace summary of the driver-shaped bench.
# Usage: bash scripts/gpu_perf.sh TAG [GOLDEN.npz]  (golden files under golden_ref/: gpurun_out/ does not travel to the box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-perf}
if [ -n "$2" ]; then
  timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_$TAG.npz --compare "$2" > gpurun_out/golden_$TAG.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/golden_$TAG.log
  [ $rc -eq 0 ] || { echo GOLDEN_MISMATCH; [ $rc -eq 1 ] || exit $rc; }
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 > "$R/gpurun_out/prof_${TAG}_drv.log" 2>&1 || { echo PROF_FAIL; exit 1; }
python3 "$R/scripts/prof_summary.py" "$R/gpurun_out/prof_$TAG" "$R/gpurun_out/prof_${TAG}_drv_summary.md" --last-steps 20 > /dev/null && rm -rf "$R/gpurun_out/prof_$TAG"
tail -1 "$R/gpurun_out/prof_${TAG}_drv.log" | cut -c1-200
echo PERF_OK
