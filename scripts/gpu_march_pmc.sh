#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
STEPS=5,25,800 timeout -k 10 200 python -u scripts/diag_march.py > gpurun_out/diag_march.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1
cd /tmp
WARM=5 K=0 V=99 ITERS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "k_march" --output-format csv -d "$R/gpurun_out/pmc_march" -o run -- python3 "$R/scripts/diag_one.py" > "$R/gpurun_out/pmc_march.log" 2>&1
echo "pmc rc=$?"
python3 "$R/scripts/pmc_table.py" --last 3 "$R/gpurun_out/pmc_march" > "$R/gpurun_out/pmc_march_table.txt"; rm -rf "$R/gpurun_out/pmc_march"
