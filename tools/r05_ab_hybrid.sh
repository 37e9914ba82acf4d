#!/bin/bash
# A/B of the configs[4] hybrid line: concurrent ingest (exact and Count-Min on two streams from
# two host threads, the default) vs serial ingest (--hybrid-serial), same box, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in conc serial; do
    A="--sketch hybrid --no-cpu"; [ $v = serial ] && A="$A --hybrid-serial"
    timeout -k 10 400 python3 bench.py $A > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "FAIL $v"; tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['exact_stage_ms_per_step'], d['queries'])"
  done
done
