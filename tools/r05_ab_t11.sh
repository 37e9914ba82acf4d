#!/bin/bash
# A/B: 2048-bucket K4 tiles with two 512-thread K4 workgroups per CU (variant build
# libgns_sketch_t11.so: GNS_TILE_BITS=11 GNS_AP_THREADS=512 GNS_REP_CAP=512 GNS_SEG_ALL=256)
# vs the default 4096-bucket tiles, one 1024-thread workgroup per CU; configs[4] and headline.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
T11=$PWD/go2netspectra_amd/libgns_sketch_t11.so
GNS_LIB=$T11 timeout -k 10 600 python -u -m pytest tests/test_cm_gpu.py -m gpu -x -q --timeout 300 -k "(wide_rows or superbin or insert_keys) and not 20000000" > $O/t11_tests.log 2>&1 || { echo "FAIL t11 tests"; tail -20 $O/t11_tests.log; exit 1; }
tail -1 $O/t11_tests.log
for i in 1 2; do
  for v in base t11; do
    for w in c5 c2; do
      A="--no-cpu --steps 6 --warmup 2 --windows 0"; [ $w = c5 ] && A="$A --width 16777216 --depth 8"
      if [ $v = t11 ]; then L=$T11; else L=$PWD/go2netspectra_amd/libgns_sketch.so; fi
      GNS_LIB=$L timeout -k 10 300 python3 bench.py $A > $O/${v}_${w}_$i.json 2> $O/${v}_${w}_$i.err || { echo "FAIL $v $w"; tail -5 $O/${v}_${w}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${w}_$i.json').read().strip().splitlines()[-1]); print('$v $w', d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
    done
  done
done
