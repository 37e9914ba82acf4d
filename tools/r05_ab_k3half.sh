#!/bin/bash
# A/B: K3s as two 512-thread workgroups per CU with 4096-packet sub-passes (GNS_K3_STAGED=h)
# against the default one 1024-thread workgroup per CU with 8192-packet sub-passes; the
# Count-Min parity file under the variant first, then headline bench lines, interleaved.
# usage: tools/r05_ab_k3half.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
GNS_K3_STAGED=h timeout -k 10 600 python -u -m pytest tests/test_cm_gpu.py -m gpu -x -q --timeout 300 > $O/tests.log 2>&1 || { echo "FAIL tests"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in 1 h; do
    GNS_K3_STAGED=$v timeout -k 10 300 python3 bench.py --no-cpu --steps 10 --warmup 2 --windows 0 > $O/k3${v}_$i.json 2> $O/k3${v}_$i.err || { echo "FAIL $v"; tail -5 $O/k3${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/k3${v}_$i.json').read().strip().splitlines()[-1]); print('k3=$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
