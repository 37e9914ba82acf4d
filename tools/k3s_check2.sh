#!/bin/bash
# K3s / K3 parity (both paths), headline bench for both, C5 bench, K3s phase profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k3s_tests.log 2>&1
rc=$?; tail -1 gpurun_out/k3s_tests.log; [ $rc -ne 0 ] && exit $rc
GNS_K3_STAGED=0 timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k3_tests.log 2>&1
rc=$?; tail -1 gpurun_out/k3_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  GNS_K3_STAGED=$v timeout -k 10 200 python bench.py --no-cpu > gpurun_out/k3s_$v.json 2>&1 || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/k3s_$v.json').read().strip().splitlines()[-1]); print('staged=$v', d['value'], d['stage_ms_per_step'])"
done
timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_cm.json 2>&1 || exit 4
python3 -c "import json; d=json.loads(open('gpurun_out/c5_cm.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['stage_ms_per_step'])"
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_k3p.so timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/k3p.json 2>&1
python3 -c "import json; d=json.loads(open('gpurun_out/k3p.json').read().strip().splitlines()[-1]); print('k3p', d['stage_ms_per_step'], d['engine_counters'])"
