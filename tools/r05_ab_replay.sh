#!/bin/bash
# A/B: K4 replay with a leader lane per bucket walking its peers in registers (default) vs one
# LDS round per same-bucket lane (variant build libgns_sketch_rl0.so: GNS_REPLAY_LEAD=0);
# configs[4] and headline.  The default library runs the whole CM parity file first.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
VAR=$PWD/go2netspectra_amd/libgns_sketch_rl0.so
timeout -k 10 600 python -u -m pytest tests/test_cm_gpu.py -m gpu -x -q --timeout 300 > $O/rl0_tests.log 2>&1 || { echo "FAIL rl0 tests"; tail -20 $O/rl0_tests.log; exit 1; }
tail -1 $O/rl0_tests.log
for i in 1 2; do
  for v in base rl0; do
    for w in c5 c2; do
      A="--no-cpu --steps 6 --warmup 2 --windows 0"; [ $w = c5 ] && A="$A --width 16777216 --depth 8"
      if [ $v = rl0 ]; then L=$VAR; else L=$PWD/go2netspectra_amd/libgns_sketch.so; fi
      GNS_LIB=$L timeout -k 10 300 python3 bench.py $A > $O/${v}_${w}_$i.json 2> $O/${v}_${w}_$i.err || { echo "FAIL $v $w"; tail -5 $O/${v}_${w}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${w}_$i.json').read().strip().splitlines()[-1]); print('$v $w', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
    done
  done
done
