#!/bin/bash
# GPU session steps for one gpurun call:  bash tools/gpu_steps.sh <step> [<step> ...]
# Each step runs under its own time limit and writes gpurun_out/<step>.log; the session stops at the
# first failing step (a GPU fault / abort / timeout must not be followed by more GPU work).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
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
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
for s in "$@"; do
  case $s in
    # ---- test suites
    tests) step gpu_suite 900 $PYT tests -m gpu -q ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    plane) step plane 500 $PYT tests/test_ps_plane_gpu.py tests/test_hvd_gpu.py tests/test_overlap_gpu.py ;;
    plan) step plan_tests 400 $PYT tests/test_plan_gpu.py tests/test_trainer_gpu.py ;;
    dropout) step dropout_tests 300 $PYT tests/test_dropout_gpu.py ;;
    x3) step x3_tests 400 $PYT tests/test_x3_gpu.py ;;
    conv_tests) step conv_tests 400 $PYT tests/test_conv_gpu.py -q ;;
    ops_tests) step ops_tests 400 $PYT tests/test_ops_gpu.py -q ;;
    bn_tests) step bn_tests 400 $PYT tests/test_ops_gpu.py -q -k "bn or batch or residual" ;;
    # ---- benches (one JSON line each, in the step's log)
    bench) step bench 400 python bench.py --steps 20 --warmup 6 ;;
    bench_plan) step bench_plan 400 python bench.py --steps 20 --warmup 6 --mode graph ;;
    bench_eager) step bench_eager 400 python bench.py --steps 20 --warmup 6 --mode eager ;;
    bench_r50) step bench_r50 400 python bench.py --model resnet50 --steps 20 --warmup 6 ;;
    bench_fp32) step bench_fp32 600 python bench.py --steps 10 --warmup 3 --dtype fp32 ;;
    # ---- multi-rank rehearsals on the box's one GPU (gloo only exchanges handles / scalars)
    bench2_auto) step bench2_auto 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 ;;
    bench2_autoplan) step bench2_autoplan 600 env TONY_BENCH_AUTO_PLAN=1 TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29526 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 ;;
    # round 3's failing N > 1 plan form (no bucket markers in the capture): names the op the replay fails on
    bench2_nomarkers) step bench2_nomarkers 600 env TONY_PLAN_MARKERS=0 TONY_BENCH_AUTO_PLAN=1 TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29528 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 ;;
    bench2_graph)step bench2_graph 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29527 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 --mode graph ;;
    bench2_plan) step bench2_plan 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29524 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 --mode graph --collective hip ;;
    bench3_ded) step bench3_ded 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 3 --steps 4 --warmup 2 --batch 32 --mode eager --ps-mode dedicated ;;
    # the paper topology through the launcher (bin/tony: coordinator -> task agents -> TF_CONFIG)
    # (fake inventories map every task to the box's one GPU; --python_binary_path: TonY runs --executes as the
    # command unless a python binary is given, TonyClient.buildTaskCommand)
    ps_job) step ps_job 600 bash bin/tony --src_dir tony_amd/jobs --executes inception_ps.py --python_binary_path python3 \
              --task_params "--ps-mode dedicated --batch-size 32 --steps 6 --warmup 2" \
              --conf tony.ps.instances=1 --conf tony.worker.instances=2 --conf tony.ps.gpus=1 \
              --conf tony.worker.gpus=1 --conf tony.amd.fake-gpus=3 --conf tony.application.security.enabled=false \
              --shell_env TONY_DIST_BACKEND=gloo
            mkdir -p gpurun_out/ps_job_logs; cp -r "$HOME"/.tony/application_*/logs/* gpurun_out/ps_job_logs/ 2>/dev/null || true ;;
    # TonY's default 0-GPU ps placed on worker 0's GPU (tony.amd.ps-share-gpu) owning the variables on the xGMI plane
    ps_job_shared) step ps_job_shared 600 bash bin/tony --src_dir tony_amd/jobs --executes inception_ps.py --python_binary_path python3 \
              --task_params "--ps-mode dedicated --batch-size 32 --steps 6 --warmup 2" \
              --conf tony.ps.instances=1 --conf tony.worker.instances=2 --conf tony.worker.gpus=1 \
              --conf tony.amd.fake-gpus=2 --conf tony.application.security.enabled=false \
              --shell_env TONY_DIST_BACKEND=gloo
            mkdir -p gpurun_out/ps_job_shared_logs; cp -r "$HOME"/.tony/application_*/logs/* gpurun_out/ps_job_shared_logs/ 2>/dev/null || true ;;
    # ---- kernel microbenches
    conv_bench) step conv_bench 400 python tools/conv_bench.py ;;
    bn_bench) step bn_bench 300 python tools/bn_bench.py ;;
    # ---- profiles: steady-state kernel table / per-stream union of a trace
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 --mode eager ${BENCH_ARGS:-}
          python3 tools/prof_summary.py gpurun_out/prof --skip 6 > gpurun_out/prof_summary.md
          python3 tools/prof_summary.py gpurun_out/prof --skip 6 --by-grid --top 120 > gpurun_out/prof_by_grid.md; find gpurun_out/prof -name '*trace*' -delete ;;
    trace) step trace 600 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 5 --mode ${TRACE_MODE:-graph} ${BENCH_ARGS:-}
          python3 tools/step_union.py gpurun_out/trace --per-queue > gpurun_out/trace_union.txt
          f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1); python3 tools/crit_path.py "$f" > gpurun_out/crit_path.txt || true
          find gpurun_out/trace -name "*trace*.csv" -delete ;;
    # ---- A/B of environment toggles against the default step: AB="name=VAR=VAL ..." (tools/ab.py)
    ab) step ab 1000 python tools/ab.py --reps ${AB_REPS:-3} ${AB_ARGS:-} ${AB:-} ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
