#!/bin/bash
# Bench sweep over an environment variable (driver shape, main leg only): bash scripts/gpu_sweep_env.sh TAG VAR "v1" "v2" ...
# prints one line per value: VAR=value ms_per_step value(samples/s)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=$1; VAR=$2; shift 2
for V in "$@"; do
  env "$VAR=$V" timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --psnr-steps 0 --cpu-baseline 0 --l16 0 --early 0 --mc-res 0 ${BENCH_ARGS:-} \
    > "gpurun_out/sweep_${TAG}_$(echo "$V" | tr ',/' '__').log" 2>&1 || { echo "bench failed for $VAR=$V"; exit 1; }
  python3 - "$VAR" "$V" "gpurun_out/sweep_${TAG}_$(echo "$V" | tr ',/' '__').log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
k = d.get('kernels', {})
ks = ' '.join(f"{n}={v['ms']:.4f}" for n, v in k.items() if isinstance(v, dict) and 'ms' in v)
print(f"{sys.argv[1]}={sys.argv[2]} ms_per_step={d['ms_per_step']:.4f} value={d['value']:.4g} {ks}", flush=True)
PY
done
echo SWEEP_OK
