#!/bin/bash
# Local helper (not run on the GPU box): retry a gpurun call only while the pool
# reports that nothing ran (status=transient); stop at the first real run.
# usage: N=40 GT=1200 tools/gpr_retry.sh '<command>'
for i in $(seq 1 ${N:-40}); do
  out=$(timeout 2400 /usr/local/graft/bin/gpurun --timeout ${GT:-1200} -- "$@" 2>&1)
  echo "$out" | grep -v "^\[gpurun\] every" | tail -15
  if echo "$out" | grep -q "status=transient"; then sleep ${SLEEP:-120}; continue; fi
  break
done
