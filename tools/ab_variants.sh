#!/bin/bash
# A/B the in-tree library variants: parity (CM GPU tests) + bench line each.
# usage: tools/ab_variants.sh name1 name2 ...   (go2netspectra_amd/libgns_sketch_<name>.so; "base" = default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  echo "=== $v" | tee -a gpurun_out/ab.log
  GNS_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_cm_gpu.py -x -q > gpurun_out/ab_test_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/ab_test_$v.log | tee -a gpurun_out/ab.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
  GNS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_bench_$v.json 2> gpurun_out/ab_bench_$v.err
  rc=$?; cat gpurun_out/ab_bench_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step'])" | tee -a gpurun_out/ab.log
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; exit $rc; fi
done
