#!/bin/bash
# Write a tony.xml for one MI355X node (counterpart of tony-in-gcp/scripts/tony.sh:104-209, which
# writes ps / worker instances, memory and gpus for the Dataproc samples).  Env overrides:
#   TONY_FRAMEWORK (tensorflow)  TONY_PS (1)  TONY_WORKERS (4)  TONY_WORKER_GPUS (1)
#   TONY_PS_GPUS (0)  TONY_WORKER_MEMORY (32g)  TONY_PS_MEMORY (8g)  TONY_MODE (GANG)
set -eu
out="${1:-tony.xml}"
prop() { printf '  <property>\n    <name>%s</name>\n    <value>%s</value>\n  </property>\n' "$1" "$2"; }
{
  echo '<?xml version="1.0"?>'
  echo '<configuration>'
  prop tony.application.framework "${TONY_FRAMEWORK:-tensorflow}"
  prop tony.application.distributed-mode "${TONY_MODE:-GANG}"
  prop tony.ps.instances "${TONY_PS:-1}"
  prop tony.ps.memory "${TONY_PS_MEMORY:-8g}"
  prop tony.ps.gpus "${TONY_PS_GPUS:-0}"
  prop tony.worker.instances "${TONY_WORKERS:-4}"
  prop tony.worker.memory "${TONY_WORKER_MEMORY:-32g}"
  prop tony.worker.gpus "${TONY_WORKER_GPUS:-1}"
  echo '</configuration>'
} > "$out"
echo "wrote $out"
