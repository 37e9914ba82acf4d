#!/bin/bash
# A/B of SuperSpread lines: the default library vs a variant library (GNS_LIB), same box,
# interleaved, three rounds.  usage: tools/r05_ab_ss.sh <tag> <variant .so name suffix>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
V=$2
mkdir -p $O
for i in 1 2 3; do
  for v in base $V; do
    if [ $v = base ]; then L=$PWD/go2netspectra_amd/libgns_sketch.so; else L=$PWD/go2netspectra_amd/libgns_sketch_$V.so; fi
    GNS_LIB=$L timeout -k 10 300 python3 bench.py --sketch superspread --no-cpu --steps 10 --warmup 3 > $O/${v}_$i.json 2> $O/${v}_$i.err || { echo "FAIL $v"; tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
