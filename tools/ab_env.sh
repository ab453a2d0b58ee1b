#!/bin/bash
# Alternating A/B of bench.py (eager) over an environment toggle:
#   bash tools/ab_env.sh VAR "val_a val_b" [reps] [extra bench args...]
# prints: <VAR>=<val> img/s ms/step host_ms gpu_ms_host_ahead
set -u
var=$1; vals=$2; reps=${3:-2}; shift 3 || true
mkdir -p gpurun_out
for rep in $(seq 1 "$reps"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 400 python bench.py --steps 30 --warmup 6 --mode eager "$@" > gpurun_out/ab.log 2>&1 || { echo "$var=$v failed"; tail -5 gpurun_out/ab.log; exit 1; }
    grep -E "^\{" gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$var=$v', d['value'], d['ms_per_step'], c.get('host_ms_per_step'), c.get('gpu_ms_per_step_host_ahead'))"
  done
done
