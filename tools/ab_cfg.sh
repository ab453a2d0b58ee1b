#!/bin/bash
# Alternating A/B of bench.py (eager) over environment configurations:
#   bash tools/ab_cfg.sh reps "A=1 B=0" "A=0 B=1" ...
# prints: <config> img/s ms/step host_ms gpu_ms_host_ahead
set -u
reps=$1; shift
mkdir -p gpurun_out
for rep in $(seq 1 "$reps"); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 400 python bench.py --steps 30 --warmup 6 --mode eager ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "[$cfg] failed"; tail -5 gpurun_out/ab.log; exit 1; }
    grep -E "^\{" gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('[$cfg]', d['value'], d['ms_per_step'], c.get('host_ms_per_step'), c.get('gpu_ms_per_step_host_ahead'))"
  done
done
