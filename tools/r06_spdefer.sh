#!/bin/bash
# Round 6: k_apply_sparse with the new buckets' state gathered slot-major after the map
# (default) against the gather at insert (libgns_sketch_spold.so, -DGNS_SP_DEFER=0):
# super-bin parity tests on the default library, then configs[4] interleaved A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_spdefer}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_cm_gpu.py -k "wide or candidates_beyond or c5 or C5 or contested or bucket_range" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/tests.log | tail -20; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in new old new old; do
  if [ $v = old ]; then L=$PWD/go2netspectra_amd/libgns_sketch_spold.so; else L=$PWD/go2netspectra_amd/libgns_sketch.so; fi
  GNS_LIB=$L timeout -k 10 300 python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 --steps 5 --warmup 2 > $O/c5_$v.json 2> $O/c5_$v.err || { echo "FAIL bench $v"; tail -3 $O/c5_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
done
