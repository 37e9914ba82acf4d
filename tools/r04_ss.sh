#!/bin/bash
# SuperSpread check: GPU tests, P4 diagnosis (GNS_SS_DEBUG), bench lines at two bin targets, rocprofv3 trace.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/ss
O=gpurun_out/ss
timeout -k 10 400 python -u -m pytest tests/test_ss_gpu.py tests/test_growth_gpu.py -k "ss or superspread or SuperSpread or spread" -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
GNS_SS_DEBUG=1 timeout -k 10 200 python3 bench.py --sketch superspread --no-cpu --steps 3 --warmup 1 > $O/dbg.json 2> $O/dbg.err || exit 3
grep gns_ss $O/dbg.err
for b in 512 256; do
  GNS_SS_BINS=$b timeout -k 10 200 python3 bench.py --sketch superspread --no-cpu > $O/bench_$b.json 2> $O/bench_$b.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/bench_$b.json').read().strip().splitlines()[-1]); print($b, d['value'], d['stage_ms_per_step'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ss -- \
    python3 bench.py --sketch superspread --no-cpu --steps 3 --warmup 1 > $O/prof.log 2>&1
