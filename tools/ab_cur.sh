# repeated bench runs of the current tree (eager)
run() { tag=$1; shift; env "$@" timeout -k 10 400 python bench.py --steps 40 --warmup 6 --mode eager > gpurun_out/ab.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ab.log; exit 1; }; grep -E "^\{" gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['ms_per_step'], c.get('host_ms_per_step'), c.get('gpu_ms_per_step_host_ahead'), c.get('host_ms_per_step_unblocked'))"; }
for rep in 1 2 3; do run cur A=1; done
