#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cm_gpu.py tests/test_edges_gpu.py tests/test_thrift_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/hh2_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/hh2_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/hh_probe.py 60 > gpurun_out/hh_probe.log 2>&1 || { tail gpurun_out/hh_probe.log; exit 2; }
grep -E "hh|C call" gpurun_out/hh_probe.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/hh2_bench.json 2> gpurun_out/hh2_bench.err || { tail -20 gpurun_out/hh2_bench.err; exit 3; }
python3 -c "import json; d=json.loads(open('gpurun_out/hh2_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['stage_ms_per_step'], d['window_exchange'])"
