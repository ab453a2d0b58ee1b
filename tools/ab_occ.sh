# A/B of the split-K wgrad occupancy candidates (ops/gemm.py WGRAD_OCC): more splits run faster alone
# but move more fp32 partials through HBM while the main stream's BN passes stream.
for o in 1,2,4,8 1 1,2 1,2,4,8 1 1,2; do TONY_WGRAD_OCC=$o timeout -k 10 400 python bench.py --steps 30 --warmup 6 --mode eager > gpurun_out/ab.log 2>&1 || exit 1; grep -E "^\{" gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('occ $o', d['value'], d['ms_per_step'], c['host_ms_per_step'], c['gpu_ms_per_step_host_ahead'])"; done
