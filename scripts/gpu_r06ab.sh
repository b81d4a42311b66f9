#!/bin/bash
# Round 6: data-parallel and overlap tests with the group's witness word from the step-counters launch; the bench at step
# 1600 with the cut-march replay (kernel id 13) in the dominant-kernel choice.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06ab}
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_dp.py tests/test_gpu_dp_procs.py -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|^E " gpurun_out/pytest_$TAG.log | tail -8; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --prepare 1600 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0 > gpurun_out/bench_step1600_$TAG.log 2>&1 || { echo BENCH_FAIL; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/bench_step1600_$TAG.log') if l.startswith('{')][-1])
print(d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], json.dumps(d['kernels']['march']), json.dumps(d['kernels']['march_cut']))"
echo ALL_OK
