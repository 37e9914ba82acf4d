#!/bin/bash
# Round 6: interleaved configs[4] A/B of library builds (main = libgns_sketch.so, other names =
# libgns_sketch_<name>.so from `make variant`), after the super-bin parity tests on main.
# usage: r06_ab_libs.sh TAG "main v1 v2" [rounds] [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_ab}
mkdir -p $O
if [ -z "$4" ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_cm_gpu.py -k "wide or candidates_beyond or c5 or C5 or contested or bucket_range" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
fi
for r in $(seq ${3:-2}); do
for v in $2; do
  if [ $v = main ]; then L=$PWD/go2netspectra_amd/libgns_sketch.so; else L=$PWD/go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$L timeout -k 10 300 python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 --steps 5 --warmup 2 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { echo "FAIL bench $v"; tail -3 $O/c5_${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c5_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['value'], d['ms_per_step'], 'apply', s['apply'], 'extract', s['extract'], 'scatter', s['scatter'])"
done; done
