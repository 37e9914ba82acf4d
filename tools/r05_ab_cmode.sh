#!/bin/bash
# Round 5 A/B: compact K1 -> K3c streams (GNS_CMODE=1, default) vs the per-packet
# code array (GNS_CMODE=0) on one box: CM parity tests first, then the headline
# bench interleaved (two rounds each).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_ab_cmode; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cm_gpu.py -m gpu \
  > $O/tests_cm.log 2>&1
rc=$?; echo "cm tests rc=$rc"; tail -2 $O/tests_cm.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in 1 0; do
    GNS_CMODE=$m timeout -k 10 300 python3 bench.py --no-cpu --windows 0 --steps 10 --warmup 3 > $O/b_m${m}_$i.json 2> $O/b_m${m}_$i.err || { echo "bench m=$m failed"; tail -3 $O/b_m${m}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_m${m}_$i.json').read().strip().splitlines()[-1]); print('cmode=$m', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
