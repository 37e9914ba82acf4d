#!/bin/bash
# Round 6: Count-Min engine tests on the main library, then interleaved bench A/B of library
# builds (main = libgns_sketch.so, others libgns_sketch_<name>.so).
# usage: r06_ab_head.sh TAG "main base" ROUNDS "bench args"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_abh}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_cm_gpu.py tests/test_growth_gpu.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for r in $(seq ${3:-2}); do
for v in $2; do
  # a name ending in "+m" runs with GNS_STAGE_MASK=0x39 (events around K1, K3, K4 and the batch only)
  M=; n=${v%+m}; [ "$n" != "$v" ] && M=0x39
  if [ $n = main ]; then L=$PWD/go2netspectra_amd/libgns_sketch.so; else L=$PWD/go2netspectra_amd/libgns_sketch_$n.so; fi
  GNS_STAGE_MASK=$M GNS_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --windows 0 ${4:---steps 10 --warmup 3} > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { echo "FAIL bench $v"; tail -3 $O/b_${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['value'], d['ms_per_step'], 'insert', s['insert'], 'K1', s['extract'], 'K3', s['scatter'], 'K4', s['apply'])"
done; done
