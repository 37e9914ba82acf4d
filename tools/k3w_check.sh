#!/bin/bash
# K3s<512,512> (wide rows): CM parity tests, then C5-geometry and headline benches, new vs prev library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py tests/test_edges_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k3w_tests.log 2>&1 || { tail -15 gpurun_out/k3w_tests.log; exit 1; }
tail -1 gpurun_out/k3w_tests.log
for v in base prev; do
  if [ $v = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/k3w_c5_$v.json 2>&1 || exit 2
  GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/k3w_c2_$v.json 2>&1 || exit 3
done
python3 - <<'PY'
import json
for f in ["k3w_c5_base", "k3w_c5_prev", "k3w_c2_base", "k3w_c2_prev"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d.get("stage_ms_per_step"))
PY
