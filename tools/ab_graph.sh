# HIP-graph replay of the whole step vs eager, with the HIP runtime's graph execution knobs
run() { tag=$1; shift; env "$@" timeout -k 10 400 python bench.py --steps 30 --warmup 6 --mode $MODE > gpurun_out/ab.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ab.log; exit 1; }; grep -E "^\{" gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['ms_per_step'], c.get('host_ms_per_step'), c.get('gpu_ms_per_step_host_ahead'), c.get('mode'))"; }
MODE=eager run eager A=1
MODE=graph run graph A=1
MODE=graph run graph_pc DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
MODE=graph run graph_q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
MODE=graph run graph_q4_pc DEBUG_HIP_FORCE_GRAPH_QUEUES=4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
MODE=eager run eager A=1
