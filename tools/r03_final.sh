#!/bin/bash
# Round-3 evidence run: GPU suite, smoke, headline bench (with CPU baseline) under rocprofv3 kernel
# stats, exact / SuperSpread / configs[4] / hybrid benches, exact kernel stats, headline PMC traffic.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/fin_pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/fin_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o cm -- python3 bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof_ex -o ex -- python3 bench.py --sketch exact > gpurun_out/fin_exact_bench.json 2> gpurun_out/fin_exact_bench.err || exit 4
timeout -k 10 200 python bench.py --sketch superspread --no-cpu > gpurun_out/fin_ss_bench.json 2>&1 || exit 5
timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/fin_c5_bench.json 2>&1 || exit 6
timeout -k 10 300 python bench.py --sketch hybrid --steps 5 --warmup 1 > gpurun_out/fin_hybrid_bench.json 2>&1 || exit 7
for f in fin_bench fin_exact_bench fin_ss_bench fin_c5_bench fin_hybrid_bench; do
  python3 -c "import json; d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('stage_ms_per_step'))"
done
