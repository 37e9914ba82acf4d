#!/bin/bash
# Round 6: the sparse super-bin K4 (k_apply_sparse) -- wide-geometry parity tests, then the
# configs[4] bench with it and without it (GNS_K4_SPARSE=0: k_subpart + tile sweep).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_sparse}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_cm_gpu.py -k "wide or candidates_beyond or c5 or C5" tests/test_configs_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/tests.log | tail -12; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  GNS_K4_SPARSE=$v timeout -k 10 300 python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 --steps 5 --warmup 2 > $O/c5_sp$v.json 2> $O/c5_sp$v.err || { echo "FAIL bench sp=$v"; tail -3 $O/c5_sp$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c5_sp$v.json').read().strip().splitlines()[-1]); print('sparse=$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'], d['engine_counters'])"
done
