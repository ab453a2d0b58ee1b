#!/bin/bash
# Launch the BASELINE configurations through bin/tony (counterpart of
# tony-in-gcp/scripts/launch_jobs.sh).  Usage: launch_jobs.sh [tony.xml | local]
set -u
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
JOBS="$ROOT/tony_amd/jobs"
if [ "${1:-}" = "local" ]; then  # CPU plumbing run: fewer ranks, tiny batches
  SUBMIT=("$ROOT/bin/tony" local)
  COMMON=(--conf tony.amd.fake-gpus=8 --conf tony.amd.visible-devices-mode=none
          --conf tony.application.security.enabled=false --shell_env TONY_DIST_BACKEND=gloo
          --shell_env OMP_NUM_THREADS=1)
  TINY=1
else
  SUBMIT=("$ROOT/bin/tony")
  COMMON=()
  [ -n "${1:-}" ] && COMMON+=(--conf_file "$1")
fi
TINY=${TINY:-0}
W=8; [ "$TINY" = 1 ] && W=2
run() {  # run <name> <script> <task params> <conf...>
  local name=$1 script=$2 params=$3; shift 3
  local confs=()
  for c in "$@"; do confs+=(--conf "$c"); done
  echo "=== $name"
  "${SUBMIT[@]}" --src_dir "$JOBS" --executes "$script" --python_binary_path python3 \
    --task_params "$params" "${COMMON[@]}" "${confs[@]}"
  echo "=== $name exit $?"
}
run "MNIST TF-PS, 1 ps + 2 workers" mnist_tf_ps.py "--steps 20" \
    tony.ps.instances=1 tony.worker.instances=2
if [ "$TINY" = 1 ]; then
  run "Inception-v3 TF-PS (tiny), 1 ps + 2 workers" inception_ps.py \
      "--ps-mode colocated --batch-size 2 --steps 1 --warmup 1" tony.ps.instances=1 tony.worker.instances=2
else
  run "Inception-v3 TF-PS, 1 ps + 4 workers" inception_ps.py "--steps 20" \
      tony.ps.instances=1 tony.worker.instances=4 tony.worker.gpus=1 tony.worker.memory=32g
  run "Horovod ResNet-50 bf16, 8 workers" hvd_resnet50.py "--steps 20" \
      tony.application.framework=horovod tony.ps.instances=0 tony.worker.instances=8 tony.worker.gpus=1 tony.worker.memory=32g
fi
run "MNIST PyTorch DDP, $W workers" mnist_pytorch_ddp.py "--steps-per-epoch 20" \
    tony.application.framework=pytorch tony.ps.instances=0 tony.worker.instances=$W tony.worker.gpus=1 tony.worker.memory=32g
run "MXNet linreg dist_sync, 1 server + $W workers" mxnet_linreg.py "--kvstore dist_sync --epochs 1" \
    tony.application.framework=mxnet tony.scheduler.instances=1 tony.server.instances=1 \
    tony.worker.instances=$W tony.ps.instances=0
