#!/bin/bash
# A/B of the default library against a variant build (make -C go2netspectra_amd/csrc variant
# NAME=<name> VARIANT_FLAGS=...): the whole Count-Min parity file on the default library first,
# then configs[4] and headline bench lines, interleaved, two rounds.
# usage: tools/r05_ab_var.sh <tag> <name>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
V=$2
mkdir -p $O
VAR=$PWD/go2netspectra_amd/libgns_sketch_$V.so
timeout -k 10 600 python -u -m pytest tests/test_cm_gpu.py -m gpu -x -q --timeout 300 > $O/tests.log 2>&1 || { echo "FAIL tests"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in base $V; do
    for w in c5 c2; do
      A="--no-cpu --steps 6 --warmup 2 --windows 0"; [ $w = c5 ] && A="$A --width 16777216 --depth 8"
      if [ $v = base ]; then L=$PWD/go2netspectra_amd/libgns_sketch.so; else L=$VAR; fi
      GNS_LIB=$L timeout -k 10 300 python3 bench.py $A > $O/${v}_${w}_$i.json 2> $O/${v}_${w}_$i.err || { echo "FAIL $v $w"; tail -5 $O/${v}_${w}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${w}_$i.json').read().strip().splitlines()[-1]); print('$v $w', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
    done
  done
done
