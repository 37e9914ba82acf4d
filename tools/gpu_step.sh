#!/bin/bash
# Run GPU steps in sequence; stop at the first fault/timeout (exit >= 2 except pytest's 1).
# usage: tools/gpu_step.sh "<cmd1>" "<cmd2>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for c in "$@"; do
  i=$((i+1))
  echo "=== step $i: $c" | tee -a gpurun_out/steps.log
  bash -c "$c"
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
