#!/bin/bash
# Kernel-variant A/B (development): for each library named (golden_ref/<name>.so, "base" first), a bitwise
# fingerprint against the base (scripts/golden_params.py) and a steady-state bench line with its per-kernel rooflines.
# Usage: bash scripts/gpu_lib_ab.sh TAG libneus2_hip_base libneus2_hip_g1 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; shift
BASE=$1
for L in "$@"; do
  LIB="$R/golden_ref/$L.so"
  if [ "$L" = "$BASE" ]; then
    NEUS2_HIP_LIB="$LIB" timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_${TAG}_$L.npz > gpurun_out/golden_${TAG}_$L.log 2>&1 || { echo "GOLDEN_FAIL $L"; exit 1; }
  else
    NEUS2_HIP_LIB="$LIB" timeout -k 10 300 python -u scripts/golden_params.py gpurun_out/golden_${TAG}_$L.npz --compare gpurun_out/golden_${TAG}_$BASE.npz > gpurun_out/golden_${TAG}_$L.log 2>&1
    rc=$?; echo "$L fingerprint rc=$rc"; grep -v amdgpu.ids gpurun_out/golden_${TAG}_$L.log | tail -6
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  fi
  NEUS2_HIP_LIB="$LIB" timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/bench_${TAG}_$L.log 2>&1 || { echo "BENCH_FAIL $L"; exit 1; }
  python3 - "$L" gpurun_out/bench_${TAG}_$L.log <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = d["kernels"]
print(sys.argv[1], "ms/step %.4f" % d["ms_per_step"], " ".join("%s=%.1f" % (n, 1000 * v["ms"]) for n, v in k.items()))
EOF
  if [ -n "$PROF" ]; then  # kernel-trace summary of the steady-state steps with this library
    ( cd /tmp && export TMPDIR=/tmp && NEUS2_HIP_LIB="$LIB" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_$L" -o run -- python3 "$R/bench.py" --steps 50 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > "$R/gpurun_out/prof_${TAG}_$L.log" 2>&1 ) || { echo "PROF_FAIL $L"; exit 1; }
    python3 scripts/prof_summary.py "$R/gpurun_out/prof_${TAG}_$L" "$R/gpurun_out/prof_${TAG}_${L}_summary.md" --last-steps 50 > /dev/null && rm -rf "$R/gpurun_out/prof_${TAG}_$L"
    grep -E "^\| k_|per step" "$R/gpurun_out/prof_${TAG}_${L}_summary.md" | head -${PROF_N:-14}
  fi
done
echo AB_OK
