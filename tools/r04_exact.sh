#!/bin/bash
# Exact aggregator: GPU tests and the bench line.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/ex
O=gpurun_out/ex
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --sketch exact --no-cpu > $O/bench.json 2> $O/bench.err || exit 3
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d.get('stage_ms_per_step'))"
