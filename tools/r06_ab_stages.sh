#!/bin/bash
# Round 6: the benches with HIP events around the main stages only (default) vs every stage
# (GNS_BENCH_ALL_STAGES=1), interleaved, for SuperSpread, the exact aggregator and the headline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_abst}
mkdir -p $O
for r in 1 2 3; do
for sk in superspread exact countmin; do
for all in 0 1; do
  GNS_BENCH_ALL_STAGES=$all timeout -k 10 300 python3 bench.py --sketch $sk --no-cpu --windows 0 --steps 10 --warmup 3 > $O/${sk}_${all}_$r.json 2> $O/${sk}_${all}_$r.err || { echo "FAIL $sk $all"; tail -3 $O/${sk}_${all}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/${sk}_${all}_$r.json').read().strip().splitlines()[-1]); print('$sk all=$all', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done; done; done
