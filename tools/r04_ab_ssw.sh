#!/bin/bash
# A/B on one box: SuperSpread S1 occupancy (GNS_SS_MINW 4 = default build, 6, 7 variant libraries), two rounds.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/abw
for r in 1 2; do
  for v in base w6 w7; do
    if [ $v = base ]; then L=""; else L="$PWD/go2netspectra_amd/libgns_sketch_$v.so"; fi
    GNS_LIB=$L timeout -k 10 200 python3 bench.py --sketch superspread --no-cpu > gpurun_out/abw/${v}_$r.json 2> gpurun_out/abw/${v}_$r.err || exit 3
    python3 -c "import json; d=json.loads(open('gpurun_out/abw/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['stage_ms_per_step'])"
  done
done
