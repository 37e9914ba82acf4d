#!/bin/bash
# A/B on one box: K1 hashing IPv4 waves' keys with constant zero words (default) vs generic
# (libgns_sketch_nov4.so, GNS_K1_V4HASH=0), two interleaved rounds of the headline bench.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in base nov4; do
    if [ $v = base ]; then L=""; else L="$PWD/go2netspectra_amd/libgns_sketch_nov4.so"; fi
    GNS_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu --windows 0 > gpurun_out/ab/${v}_$r.json 2> gpurun_out/ab/${v}_$r.err || exit 3
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['stage_ms_per_step']['extract'], d['ms_per_step'])"
  done
done
