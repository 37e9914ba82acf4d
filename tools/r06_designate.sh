#!/bin/bash
# Round 6: designation candidates from the histogram pass -- CM GPU tests, then configs[4]
# and headline benches twice each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_desig}
mkdir -p $O
bash tools/r06_tests.sh $(basename $O)_t tests/test_cm_gpu.py tests/test_configs_gpu.py tests/test_growth_gpu.py || exit 1
for v in a b; do
  timeout -k 10 300 python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 --steps 5 --warmup 2 > $O/c5_$v.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu --windows 0 --steps 10 --warmup 3 > $O/c2_$v.json 2>/dev/null || exit 1
  for w in c5 c2; do python3 -c "
import json; d=json.loads(open('$O/${w}_$v.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"; done
done
