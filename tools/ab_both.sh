#!/bin/bash
# CM parity tests, then new (base) vs previous library on the headline and the C5 geometry.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py tests/test_edges_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -15 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
run() {  # name lib args...
  local v=$1 lib=$2; shift 2
  GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "stop $v"; exit 2; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['stage_ms_per_step'])"
}
for rep in 1 2; do
  run c2_base go2netspectra_amd/libgns_sketch.so --steps 5 --warmup 2
  run c2_prev go2netspectra_amd/libgns_sketch_prev.so --steps 5 --warmup 2
done
run c5_base go2netspectra_amd/libgns_sketch.so --width 16777216 --depth 8 --steps 3 --warmup 1
run c5_prev go2netspectra_amd/libgns_sketch_prev.so --width 16777216 --depth 8 --steps 3 --warmup 1
