#!/bin/bash
# Round-4 check run: selected GPU tests (args: pytest selectors), smoke, one headline bench.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SEL=${SEL:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/chk_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/chk_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk_smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/chk_bench.json 2> gpurun_out/chk_bench.err || exit 3
python3 -c "import json; d=json.loads(open('gpurun_out/chk_bench.json').read().strip().splitlines()[-1]); print(d['value'], d.get('stage_ms_per_step'), d['roofline']['frac'])"
