#!/bin/bash
# Round-3 GPU session steps.  Each step runs under its own time limit; the session stops at the
# first failing step (a GPU fault / abort / timeout must not be followed by more GPU work).
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
    plane) step plane 500 python -u -m pytest tests/test_ps_plane_gpu.py tests/test_hvd_gpu.py tests/test_overlap_gpu.py -x -v --timeout 240 --timeout-method thread ;;
    plan) step plan_tests 400 python -u -m pytest tests/test_plan_gpu.py tests/test_trainer_gpu.py -x -v --timeout 240 --timeout-method thread ;;
    bench_plan) step bench_plan 400 python bench.py --steps 20 --warmup 6 --mode graph ;;
    bench_graph) step bench_graph 400 env TONY_REPLAY=graph python bench.py --steps 20 --warmup 6 --mode graph ;;
    x3) step x3_tests 400 python -u -m pytest tests/test_x3_gpu.py -x -v --timeout 240 --timeout-method thread ;;
    bench_fp32) step bench_fp32 600 python bench.py --steps 10 --warmup 3 --dtype fp32 --mode eager ;;
    bench_fp32_auto) step bench_fp32_auto 600 python bench.py --steps 10 --warmup 3 --dtype fp32 ;;
    conv_tests) step conv_tests 400 python -u -m pytest tests/test_conv_gpu.py tests/test_x3_gpu.py -x -q --timeout 240 --timeout-method thread ;;
    tbm) step tbm_diag 400 bash tools/diag/wgrad_tbm.sh ;;
    ab_tbm) step ab_tbm 600 python tools/ab_r3.py --reps 3 tbm128=TONY_WGRAD_TBM96=0 ;;
    ab_tbm_fp32) step ab_tbm_fp32 600 python tools/ab_r3.py --reps 2 --steps 10 --bench-args "--dtype fp32" tbm128=TONY_WGRAD_TBM96=0 ;;
    join_tests) step join_tests 400 python -u -m pytest tests/test_resnet_join_gpu.py tests/test_ops_gpu.py -x -q --timeout 240 --timeout-method thread -k "join or resnet or residual or inception" ;;
    ab_join) step ab_join 600 python tools/ab_r3.py --reps 3 --bench-args "--model resnet50" nojoin=TONY_RESNET_JOIN=0 ds_miopen=TONY_RESNET_DS_TONY=0 ;;
    ab_ijoin) step ab_ijoin 600 python tools/ab_r3.py --reps 3 nojoin=TONY_INCEPTION_JOIN=0 ;;
    acc_tests) step acc_tests 400 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_join_gpu.py -x -q --timeout 240 --timeout-method thread -k "accum or join" ;;
    ab_r50) step ab_r50 1000 python tools/ab_r3.py --reps 2 --bench-args "--model resnet50" fused_red=TONY_BN_FUSED_REDUCE=1 onepass16=TONY_BN_ONEPASS=1,TONY_BN_ONEPASS_MAX_MB=16 occ2=TONY_WGRAD_OCC=2 tbm128=TONY_WGRAD_TBM96=0 urgent0=TONY_WGRAD_URGENT_MB=0 ;;
    gemm) step gemm_resnet 300 python tools/gemm_bench.py --resnet
          step gemm_incep 300 python tools/gemm_bench.py ;;
    ab_masked) step ab_masked 700 python tools/ab_r3.py --reps 3 --bench-args "--model resnet50" dres=TONY_MASKED_JOIN=0 ;;
    pool_tests) step pool_tests 400 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py -x -q --timeout 240 --timeout-method thread -k "pool or stem" ;;
    ab_gather) step ab_gather 700 python tools/ab_r3.py --reps 3 dy=TONY_POOL_BN_GATHER=0 ;;
    ab_gather_r50) step ab_gather_r50 700 python tools/ab_r3.py --reps 3 --bench-args "--model resnet50" dy=TONY_POOL_BN_GATHER=0 ;;
    splitk_tests) step splitk_tests 300 python -u -m pytest tests/test_ops_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "splitk or wgrad" ;;
    ab_red) step ab_red 700 python tools/ab_r3.py --reps 3 red1k=TONY_BN_RED_WGS=1024 red2k=TONY_BN_RED_WGS=2048 ;;
    ab_red_r50) step ab_red_r50 700 python tools/ab_r3.py --reps 3 --bench-args "--model resnet50" red1k=TONY_BN_RED_WGS=1024 red2k=TONY_BN_RED_WGS=2048 ;;
    ab_mask) step ab_mask 600 python tools/ab_r3.py --reps 3 --bench-args "--model resnet50" nomask=TONY_RES_MASK=0 ;;
    ab2) step ab2 700 python tools/ab_r3.py --reps 3 fr_auto=TONY_BN_FUSED_REDUCE=auto fr_auto32=TONY_BN_FUSED_REDUCE=auto,TONY_BN_FUSED_REDUCE_MIN_MB=32 urgent0=TONY_WGRAD_URGENT_MB=0 ;;
    ab_so_r50) step ab_so_r50 700 python tools/ab_r3.py --reps 3 --bench-args "--model resnet50" old_so=TONY_KERNELS_SO=$(pwd)/tony_amd/ops/_tony_kernels_ab.so ;;
    bn_tests) step bn_tests 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 240 --timeout-method thread -k "bn or batch or residual" ;;
    ab_so_plan) step ab_so_plan 700 python tools/ab_r3.py --reps 3 --mode graph old_so=TONY_KERNELS_SO=$(pwd)/tony_amd/ops/_tony_kernels_ab.so ;;
    ab_so_plan_r50) step ab_so_plan_r50 700 python tools/ab_r3.py --reps 3 --mode graph --bench-args "--model resnet50" old_so=TONY_KERNELS_SO=$(pwd)/tony_amd/ops/_tony_kernels_ab.so ;;
    ab_so) step ab_so 700 python tools/ab_r3.py --reps 3 old_so=TONY_KERNELS_SO=$(pwd)/tony_amd/ops/_tony_kernels_ab.so ;;
    # alternating A/B of the opt-in environment toggles against the default step (tools/ab_r3.py)
    ab) step ab 1000 python tools/ab_r3.py --reps 2 onepass16=TONY_BN_ONEPASS=1,TONY_BN_ONEPASS_MAX_MB=16 fused_red=TONY_BN_FUSED_REDUCE=1 pool_bnred=TONY_POOL_BNRED=1 occ2=TONY_WGRAD_OCC=2 nobranch=TONY_BRANCH_STREAMS=0 wbatch1=TONY_WGRAD_BATCH=1 ;;
    tests) step gpu_suite 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ;;
    bench) step bench 400 python bench.py --steps 20 --warmup 6 ;;
    bench_r50) step bench_r50 400 python bench.py --model resnet50 --steps 20 --warmup 6 ;;
    bench_r50_b16) step bench_r50_b16 400 python bench.py --model resnet50 --batch 16 --steps 20 --warmup 6 --mode eager ;;
    host) step host_layer 300 python tools/host_layer_bench.py
          step host_micro 300 python tools/host_micro.py ;;
    hostprof) step host_prof_fwd 300 python tools/host_profile.py --steps 5
              step host_prof_bwd 300 python tools/host_profile.py --steps 5 --bwd ;;
    # 1 ps + 2 workers, three processes on the box's one GPU (gloo only exchanges the window handles):
    # the dedicated PS on the xGMI data plane with the real Inception-v3 step
    bench3_ded) step bench3_ded 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 3 --steps 4 --warmup 2 --batch 32 --mode eager --ps-mode dedicated ;;
    # 2 colocated ranks on the box's one GPU (gloo): --mode auto now also times the native plan with
    # per-bucket segments at N > 1; bench2_plan forces it (and the xGMI kernels for the buckets)
    bench2_auto) step bench2_auto 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 ;;
    bench2_plan_gloo) step bench2_plan_gloo 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29525 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 --mode graph ;;
    bench2_plan) step bench2_plan 600 env TONY_BENCH_BACKEND=gloo TONY_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29524 bench.py --gpus 2 --steps 6 --warmup 3 --batch 32 --mode graph --collective hip ;;
    # the same topology through the launcher (bin/tony: coordinator -> task agents -> TF_CONFIG)
    ps_job) step ps_job 600 bash bin/tony --src_dir tony_amd/jobs --executes inception_ps.py \
              --task_params "--ps-mode dedicated --batch-size 32 --steps 6 --warmup 2" \
              --conf tony.ps.instances=1 --conf tony.worker.instances=2 --conf tony.ps.gpus=1 \
              --conf tony.worker.gpus=1 --conf tony.amd.fake-gpus=3 --conf tony.application.security.enabled=false \
              --shell_env TONY_DIST_BACKEND=gloo ;;
    prof) export TMPDIR=/tmp; R=$(pwd)
          step prof 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 --mode eager ${BENCH_ARGS:-}
          python3 tools/prof_summary.py gpurun_out/prof --skip 6 > gpurun_out/prof_summary.md; find gpurun_out/prof -name '*trace*' -delete ;;
    trace) export TMPDIR=/tmp; R=$(pwd)
          step trace 600 rocprofv3 --kernel-trace -d "$R/gpurun_out/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 5 --mode ${TRACE_MODE:-graph} ${BENCH_ARGS:-}
          python3 tools/step_union.py gpurun_out/trace --per-queue > gpurun_out/trace_union.txt; python3 tools/crit_path.py $(find gpurun_out/trace -name "*kernel_trace.csv" | head -1) > gpurun_out/crit_path.txt 2>&1 || true; find gpurun_out/trace -name "*trace*.csv" -delete ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
