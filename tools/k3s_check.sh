#!/bin/bash
# K3s (staged) vs K3: CM parity suite with the default, then both benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k3s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/k3s_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1; do
  GNS_K3_STAGED=$v timeout -k 10 200 python bench.py --no-cpu > gpurun_out/k3s_$v.json 2>&1 || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/k3s_$v.json').read().strip().splitlines()[-1]); print('staged=$v', d['value'], d['stage_ms_per_step'])"
done
