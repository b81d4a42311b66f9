#!/bin/bash
# r05mw: the unit box's (p - 0) / 1 skipped in the march write and the occupancy samples, the constant step's warped dt
# folded: march parity tests, fingerprint against the build before, kernel traces of both, alternating benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_progressive.py tests/test_gpu_train_parity.py > gpurun_out/pytest_r05mw.log 2>&1 || { tail -30 gpurun_out/pytest_r05mw.log; exit 1; }
tail -2 gpurun_out/pytest_r05mw.log
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_prev.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_prev_r05mw.npz > gpurun_out/golden_prev_r05mw.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05mw.npz --compare gpurun_out/golden_prev_r05mw.npz > gpurun_out/golden_new_r05mw.log 2>&1 || { tail -5 gpurun_out/golden_new_r05mw.log; exit 1; }
echo "fingerprint: $(grep -c identical gpurun_out/golden_new_r05mw.log) identical of 8"
for v in prev new; do
  if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_prev.so; fi
  (cd /tmp && export TMPDIR=/tmp && NEUS2_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mw_$v" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 5 \
     --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_mw_$v.log" 2>&1) || { echo PROF_FAIL; exit 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_mw_$v gpurun_out/prof_mw_${v}_summary.md --last-steps 40 > /dev/null && rm -rf gpurun_out/prof_mw_$v
  echo "$v: $(grep -E 'k_march_write|k_nerf_density' gpurun_out/prof_mw_${v}_summary.md | tr '\n' ' ')"
done
T=r05mw bash scripts/gpu_r05ab.sh
