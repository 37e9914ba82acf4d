#!/bin/bash
# Count-Min GPU parity tests, then the headline bench (K1 parks displaced flows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cm_gpu.py tests/test_edges_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/park_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/park_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/park_bench.json 2> gpurun_out/park_bench.err || { tail -20 gpurun_out/park_bench.err; exit 2; }
python3 -c "import json; d=json.loads(open('gpurun_out/park_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['stage_ms_per_step'], d['window_exchange'])"
