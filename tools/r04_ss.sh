#!/bin/bash
# SuperSpread check: GPU tests, bench line, rocprofv3 kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/ss
O=gpurun_out/ss
timeout -k 10 400 python -u -m pytest tests/test_ss_gpu.py tests/test_growth_gpu.py -k "ss or superspread or SuperSpread or spread" -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --sketch superspread --no-cpu > $O/bench.json 2> $O/bench.err || exit 3
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['stage_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ss -- \
    python3 bench.py --sketch superspread --no-cpu --steps 3 --warmup 1 > $O/prof.log 2>&1
