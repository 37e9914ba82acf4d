#!/bin/bash
# A/B of k_subpart's workgroup size at configs[4] geometry (GNS_SUBPART_NT=1024 vs the
# 512-thread default), same box: C5 bench lines, the apply stage = k_subpart + K4.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
for v in 512 1024 512 1024; do
    GNS_SUBPART_NT=$v timeout -k 10 300 python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 > $O/c5_$v.json 2> $O/c5_$v.err || { echo "FAIL $v"; tail -5 $O/c5_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done
