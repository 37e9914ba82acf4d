#!/bin/bash
# A/B: K3s with consecutive K1 blocks mapped to workgroups of one XCD (GNS_K3_XCD=1, now the default), so that
# the partial lines at the boundary of adjacent blocks' runs of a bin are written through one
# L2, against the default round-robin order; parity file under the variant first, then
# headline and configs[4] bench lines, interleaved.
# usage: tools/r05_ab_k3xcd.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
GNS_K3_XCD=1 timeout -k 10 600 python -u -m pytest tests/test_cm_gpu.py -m gpu -x -q --timeout 300 > $O/tests.log 2>&1 || { echo "FAIL tests"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    for w in c2 c5; do
      A="--no-cpu --steps 6 --warmup 2 --windows 0"; [ $w = c5 ] && A="$A --width 16777216 --depth 8"
      GNS_K3_XCD=$v timeout -k 10 300 python3 bench.py $A > $O/x${v}_${w}_$i.json 2> $O/x${v}_${w}_$i.err || { echo "FAIL $v $w"; tail -5 $O/x${v}_${w}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/x${v}_${w}_$i.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('xcd=$v $w', d['value'], d['ms_per_step'], 'scatter', s['scatter'], 'apply', s['apply'])"
    done
  done
done
