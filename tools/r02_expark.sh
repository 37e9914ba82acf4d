#!/bin/bash
# Exact-aggregator GPU parity tests, then its bench (X1 pipelined, displaced flows parked).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_thrift_gpu.py tests/test_edges_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/expark_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/expark_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --sketch exact --no-cpu > gpurun_out/expark_bench.json 2> gpurun_out/expark_bench.err || { tail -20 gpurun_out/expark_bench.err; exit 2; }
python3 -c "import json; d=json.loads(open('gpurun_out/expark_bench.json').read().strip().splitlines()[-1]); print(d['value'], d.get('roofline'), d['stage_ms_per_step'])"
