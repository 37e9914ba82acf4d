#!/bin/bash
# Round 5 A/B of K1 (all variants exact): the per-packet code array (GNS_CMODE=0),
# compact streams (GNS_CMODE=1) with K1 at 4 waves per SIMD (128 VGPRs, spills), and
# compact streams with K1 at 3 waves per SIMD (libgns_sketch_w3.so, -DGNS_CM_MINW=3:
# 155 VGPRs, no spills).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_ab_k1b; mkdir -p $O
W3=$GRAFT_REPO_ROOT/go2netspectra_amd/libgns_sketch_w3.so
GNS_LIB=$W3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cm_gpu.py -m gpu -k "zipf or golden or many_calls" > $O/w3_tests.log 2>&1
rc=$?; echo "w3 tests rc=$rc"; tail -2 $O/w3_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in m0 m1 w3; do
    case $v in m0) E="GNS_CMODE=0";; m1) E="GNS_CMODE=1";; w3) E="GNS_CMODE=1 GNS_LIB=$W3";; esac
    env $E timeout -k 10 300 python3 bench.py --no-cpu --windows 0 --steps 8 --warmup 3 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { echo "bench $v failed"; tail -3 $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print('$v', d['value'], d['ms_per_step'], 'K1', s['extract'], 'K3', s['scatter'], 'K4', s['apply'])"
  done
done
