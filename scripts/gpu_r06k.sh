#!/bin/bash
# Round 6, iteration k: the packed-fp32 reproducer (scripts/repro_pk_f32.hip, built here with packed fp32 on) and where the
# compaction cut falls among the marched slots (scripts/diag_cut_extent.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06k}
hipcc --offload-arch=gfx950 -O3 scripts/repro_pk_f32.hip -o /tmp/repro_pk_f32 > gpurun_out/repro_pk_build_$TAG.log 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 240 /tmp/repro_pk_f32 30 > gpurun_out/repro_pk_f32_$TAG.jsonl 2>&1 || { echo REPRO_FAIL; tail -5 gpurun_out/repro_pk_f32_$TAG.jsonl; exit 1; }
cat gpurun_out/repro_pk_f32_$TAG.jsonl
timeout -k 10 300 python3 -u scripts/diag_cut_extent.py > gpurun_out/diag_cut_extent_$TAG.jsonl 2>&1 || { echo DIAG_FAIL; tail -5 gpurun_out/diag_cut_extent_$TAG.jsonl; exit 1; }
grep '^{' gpurun_out/diag_cut_extent_$TAG.jsonl
echo ALL_OK
