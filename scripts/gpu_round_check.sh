set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_r01c.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r01c.log 2>&1 || { echo BENCH_FAIL; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_r01c -o run -- python3 /root/repo/bench.py --steps 50 --psnr-steps 2000 --mc-res 1024 --cpu-baseline 0 > /root/repo/gpurun_out/bench_prof_r01c.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
