#!/bin/bash
# A/B of the XCD-contiguous workgroup order (gns_xcd.cuh) in the run-writing partitions (at the
# time of profiles/r05_ab_xcd_all.txt all three; SuperSpread's was then dropped as neutral)
# (Count-Min K3s, exact P3 k_ex_pscatter, SuperSpread P3 k_sp_scatter) against a build with
# -DGNS_NO_XCD_MAP (make -C go2netspectra_amd/csrc variant NAME=noxcd
# VARIANT_FLAGS=-DGNS_NO_XCD_MAP): the SuperSpread and exact parity files first, then
# interleaved bench lines of the headline, SuperSpread, exact and configs[4].
# usage: tools/r05_ab_xcd_all.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ss_gpu.py tests/test_exact_gpu.py -m gpu -x -q --timeout 300 > $O/tests.log 2>&1 || { echo "FAIL tests"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in noxcd base; do
    for w in c2 ss exact c5; do
      A="--no-cpu --steps 6 --warmup 2"
      case $w in c2) A="$A --windows 0";; ss) A="$A --sketch superspread";; exact) A="$A --sketch exact";; c5) A="$A --windows 0 --width 16777216 --depth 8";; esac
      if [ $v = base ]; then L=$PWD/go2netspectra_amd/libgns_sketch.so; else L=$PWD/go2netspectra_amd/libgns_sketch_noxcd.so; fi
      GNS_LIB=$L timeout -k 10 300 python3 bench.py $A > $O/${v}_${w}_$i.json 2> $O/${v}_${w}_$i.err || { echo "FAIL $v $w"; tail -5 $O/${v}_${w}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${w}_$i.json').read().strip().splitlines()[-1]); print('$v $w', d['value'], d['ms_per_step'], d.get('stage_ms_per_step'))"
    done
  done
done
