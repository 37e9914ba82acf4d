#!/bin/bash
# A/B: K3s for rows of 512 bins (the configs[4] geometry) as one 1024-thread workgroup with
# 16-bit (wave, bin) counters (k_scatter_st<1024,512,8192,true>, now the default; the run that
# chose it selected it with GNS_K3_STAGED=p) against the 512-thread workgroup (GNS_K3_STAGED=u);
# the Count-Min and configs parity files under the variant
# first, then configs[4] bench lines, interleaved.
# usage: tools/r05_ab_k3pack.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_cm_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 > $O/tests.log 2>&1 || { echo "FAIL tests"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in u 1; do
    GNS_K3_STAGED=$v timeout -k 10 300 python3 bench.py --no-cpu --steps 6 --warmup 2 --windows 0 --width 16777216 --depth 8 > $O/k3${v}_$i.json 2> $O/k3${v}_$i.err || { echo "FAIL $v"; tail -5 $O/k3${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/k3${v}_$i.json').read().strip().splitlines()[-1]); print('k3=$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
