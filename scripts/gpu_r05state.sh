#!/bin/bash
# Is the default bench's slower inference launch (182 against 148 us) the training state or the longer run before it?
# The driver shape after a 1020-step prepare (the default run's state, a short run) against after the usual 800.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
F="--cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for p in 1020 800; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --prepare $p $F > gpurun_out/state_$p.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/state_$p.log').read().strip().splitlines()[-1]); r=d['roofline']; print('prepare', $p, 'ms', round(d['ms_per_step'],4), 'launch_ms', r['launch_ms'], 'units', r['units_per_launch'], 'chunk_end', d.get('progressive_chunk_end'), 'replay_ms', d['kernels']['inference']['ms'])"
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --prepare 800 $F > gpurun_out/state_long.log 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/state_long.log').read().strip().splitlines()[-1]); r=d['roofline']; print('prepare 800 steps 200', 'ms', round(d['ms_per_step'],4), 'launch_ms', r['launch_ms'], 'units', r['units_per_launch'], 'chunk_end', d.get('progressive_chunk_end'), 'replay_ms', d['kernels']['inference']['ms'])"
echo ALL_OK
