#!/bin/bash
# Round-2 GPU session steps (see tools/gpu_check.sh for the round-1 set).
set -u
mkdir -p gpurun_out
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -4 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    overlap) step overlap 400 python -u -m pytest tests/test_overlap_gpu.py tests/test_trainer_gpu.py -x -v --timeout 240 --timeout-method thread ;;
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 6 --tune-cache gpurun_out/tune.json ;;
    bench2) step bench2_gloo 900 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 3 --mode eager ;;
    conv) step conv 400 python -u -m pytest tests/test_conv_gpu.py -x -v --timeout 200 --timeout-method thread ;;
    newtests) step newtests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_hvd_gpu.py tests/test_convergence_gpu.py tests/test_model_fp32_gpu.py -x -v -s --timeout 300 --timeout-method thread ;;
    stem) step stem 400 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py -x -v -k "stem or linear or whole_input" --timeout 200 --timeout-method thread ;;
    xgmi) step xgmi 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 200 --timeout-method thread ;;
    bench2_hip) step bench2_hip 900 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 6 --warmup 3 --mode eager --collective hip ;;
    coll2) step coll2 300 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 tools/coll_bench.py --max-mb 64 --json gpurun_out/coll2.json ;;
    bench_fp32) step bench_fp32 900 python bench.py --steps 10 --warmup 4 --dtype fp32 --mode eager ;;
    bench_gradfp32) step bench_gradfp32 900 python bench.py --steps 20 --warmup 6 --grad-dtype fp32 --tune-cache gpurun_out/tune.json ;;
    bench_nooverlap) step bench_nooverlap 900 python bench.py --steps 20 --warmup 6 --no-overlap --mode eager --tune-cache gpurun_out/tune.json ;;
    bench2_ded) step bench2_ded 900 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 2 --mode eager --ps-mode dedicated ;;
    prof) export TMPDIR=/tmp; R=$(pwd)
          step prof 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 --mode eager ${BENCH_ARGS:-}
          python3 tools/prof_summary.py gpurun_out/prof --skip 6 > gpurun_out/prof_summary.md; find gpurun_out/prof -name '*trace*' -delete ;;
    trace) export TMPDIR=/tmp; R=$(pwd)
          step trace 900 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 5 --mode eager ${BENCH_ARGS:-}
          python3 tools/step_union.py gpurun_out/trace --per-queue > gpurun_out/trace_union.txt; ${KEEP_TRACE:+true} find gpurun_out/trace -name "*trace*.csv" -delete ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
