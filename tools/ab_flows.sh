#!/bin/bash
# A/B of the flow-dictionary capacity (2*max_flows slots of 64 B) on the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mf in 2097152 1048576 4194304 2097152; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --max-flows $mf > gpurun_out/ab_mf_$mf.json 2> gpurun_out/ab_mf_$mf.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_mf_$mf.json').read()); print('$mf', d['value'], d['stage_ms_per_step'], d['engine_counters'])"
done
