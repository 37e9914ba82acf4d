#!/bin/bash
# Headline bench at several flow-dictionary capacities (max_flows), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for mf in 2097152 4194304 8388608; do
    timeout -k 10 200 python bench.py --no-cpu --windows 0 --max-flows $mf > gpurun_out/abmf_${mf}_$rep.json 2> gpurun_out/abmf_${mf}_$rep.err || { echo "stop $mf"; tail -5 gpurun_out/abmf_${mf}_$rep.err; exit 2; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abmf_${mf}_$rep.json').read().strip().splitlines()[-1]); print('$mf', d['value'], d['stage_ms_per_step'])"
  done
done
