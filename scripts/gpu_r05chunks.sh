#!/bin/bash
# r05chunks: progressive chunk schedules at the bench state with the round-5 kernels (auto = {e, 2e} from the step's rule)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
o=gpurun_out/chunks_${TAG:-r05}.txt
: > $o
B="--gpus 1 --steps 100 --warmup 5 --cpu-baseline 0 --psnr-steps 0 --mc-res 0 --l16 0 --early 0"
for i in 1 2; do
  for v in ${VARIANTS:-auto 40,80,120 48,96,144 56,112,168 32,64,96,128}; do
    if [ $v = auto ]; then unset NEUS_CHUNK_ENDS; else export NEUS_CHUNK_ENDS=$v; fi
    timeout -k 10 200 python -u bench.py $B > gpurun_out/bench_ch_${v}_$i.log 2>&1 || exit 1
    echo "main $v $i $(tail -1 gpurun_out/bench_ch_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["ms_per_step"], r["evaluated_per_step"], d.get("progressive_chunk_end"))')" >> $o
  done
  unset NEUS_CHUNK_ENDS
done
cat $o
echo ALL_OK
