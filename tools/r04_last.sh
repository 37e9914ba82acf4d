#!/bin/bash
# Last check of the round's tree: the whole -m gpu suite, smoke, and the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/last
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/last/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/last/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1 || exit 2
tail -1 gpurun_out/last/smoke.log
timeout -k 10 500 python3 bench.py > gpurun_out/last/bench.json 2> gpurun_out/last/bench.err || exit 3
python3 -c "import json; d=json.loads(open('gpurun_out/last/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['parity']['bit_exact'], d['cpu_baseline']['value'])"
