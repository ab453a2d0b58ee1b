#!/bin/bash
# Node check for tony_amd on MI355X (counterpart of tony-in-gcp/scripts/create_cluster.sh +
# install_gpu*.sh: there is nothing to install, only to verify).
set -u
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
ok=0
say() { printf '%-28s %s\n' "$1" "$2"; }
for t in hipcc rocminfo amd-smi rocprofv3; do
  if command -v "$t" > /dev/null 2>&1 || [ -x "/opt/rocm/bin/$t" ]; then say "$t" "found"; else say "$t" "MISSING"; ok=1; fi
done
say "HSA_ENABLE_IPC_MODE_LEGACY" "${HSA_ENABLE_IPC_MODE_LEGACY:-unset} (RCCL/IPC need 0: dmabuf IPC)"
[ "${HSA_ENABLE_IPC_MODE_LEGACY:-}" = "0" ] || ok=1
say "gfx950 agents" "$( (/opt/rocm/bin/rocminfo 2>/dev/null || true) | grep -c 'gfx950' )"
if command -v amd-smi > /dev/null 2>&1; then
  amd-smi topology 2>/dev/null | sed -n '1,40p' || true     # xGMI link table (8 GPUs, all-to-all)
fi
say "NUMA nodes" "$(ls -d /sys/devices/system/node/node[0-9]* 2>/dev/null | wc -l)"
cd "$ROOT" || exit 1
python3 - <<'PY' || ok=1
import __graft_entry__ as g
g.build()                                   # hipcc --offload-arch=gfx950, in-tree .so files
from tony_amd.gpu.inventory import discover
devs = discover()
print(f"tony_amd GPU inventory: {len(devs)} device(s)")
for d in devs:
    print("  ", d)
PY
exit $ok
