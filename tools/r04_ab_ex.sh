#!/bin/bash
# A/B on one box: the exact aggregator before this round's touched-flow list (libgns_sketch_exold.so) vs now.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/abx
for r in 1 2; do
  for v in base exold; do
    if [ $v = base ]; then L=""; else L="$PWD/go2netspectra_amd/libgns_sketch_$v.so"; fi
    GNS_LIB=$L timeout -k 10 200 python3 bench.py --sketch exact --no-cpu > gpurun_out/abx/${v}_$r.json 2> gpurun_out/abx/${v}_$r.err || exit 3
    python3 -c "import json; d=json.loads(open('gpurun_out/abx/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['stage_ms_per_step'])"
  done
done
