#!/bin/bash
# XCD-partitioned inference experiment (scripts/exp_xcd_infer.py): timing with and without NEUS_INFER_XCD_PARTS, then
# one PMC pass (L2 hit / miss, EA reads) per (parts, order). Usage: LIB=neus2_amd/libneus2_hip_x.so bash scripts/gpu_xcd_exp.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export NEUS2_HIP_LIB=${LIB:-neus2_amd/libneus2_hip.so}
for X in 0 1; do
  NEUS_INFER_XCD_PARTS=$X timeout -k 10 300 python -u scripts/exp_xcd_infer.py > gpurun_out/xcd_t$X.log 2>&1 || { echo "timing $X failed"; exit 1; }
  grep ms_per_launch gpurun_out/xcd_t$X.log
done
for X in 0 1; do for O in random morton; do
  (cd /tmp && export TMPDIR=/tmp && NEUS_INFER_XCD_PARTS=$X EXP_ORDERS=$O timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
     --kernel-include-regex k_nerf_infer --output-format csv -d "$R/gpurun_out/pmcx_${X}_$O" -o run -- python3 "$R/scripts/exp_xcd_infer.py" \
     > "$R/gpurun_out/pmcx_${X}_$O.log" 2>&1) || { echo "pmc $X $O failed"; exit 1; }
  python3 scripts/pmc_table.py --last 40 gpurun_out/pmcx_${X}_$O > gpurun_out/pmcx_${X}_${O}_table.txt && echo "== parts=$X order=$O" && cat gpurun_out/pmcx_${X}_${O}_table.txt
done; done
echo XCD_OK
