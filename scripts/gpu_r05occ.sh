#!/bin/bash
# r05occ: the occupancy samples' retry densities loaded together: fingerprint against the build before it, kernel traces of
# both builds (k_nerf_density per update), alternating benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
NEUS2_HIP_LIB=$PWD/neus2_amd/libneus2_hip_prev.so timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_prev_r05occ.npz > gpurun_out/golden_prev_r05occ.log 2>&1 &&
timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_new_r05occ.npz --compare gpurun_out/golden_prev_r05occ.npz > gpurun_out/golden_new_r05occ.log 2>&1 || { tail -5 gpurun_out/golden_new_r05occ.log; exit 1; }
echo "fingerprint: $(grep -c identical gpurun_out/golden_new_r05occ.log) identical of 8"
for v in prev new; do
  if [ $v = new ]; then L=$PWD/neus2_amd/libneus2_hip.so; else L=$PWD/neus2_amd/libneus2_hip_prev.so; fi
  (cd /tmp && export TMPDIR=/tmp && NEUS2_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_occ_$v" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --warmup 5 \
     --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_occ_$v.log" 2>&1) || { echo PROF_FAIL; exit 1; }
  python3 scripts/prof_summary.py gpurun_out/prof_occ_$v gpurun_out/prof_occ_${v}_summary.md --last-steps 40 > /dev/null && rm -rf gpurun_out/prof_occ_$v
  echo "$v: $(grep 'k_nerf_density' gpurun_out/prof_occ_${v}_summary.md | head -1)"
done
T=r05occ bash scripts/gpu_r05ab.sh
