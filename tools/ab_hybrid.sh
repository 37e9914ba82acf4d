#!/bin/bash
# configs[4] hybrid bench: concurrent (two streams, two threads) vs serial ingest, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for mode in conc serial; do
    extra=""; [ $mode = serial ] && extra="--hybrid-serial"
    timeout -k 10 300 python bench.py --sketch hybrid --steps 5 --warmup 1 $extra > gpurun_out/abh_${mode}_$rep.json 2> gpurun_out/abh_${mode}_$rep.err || { echo "stop $mode"; tail -5 gpurun_out/abh_${mode}_$rep.err; exit 2; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abh_${mode}_$rep.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['queries']['latency_ms_avg'], d['stage_ms_per_step'])"
  done
done
