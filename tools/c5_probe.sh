#!/bin/bash
# C5-geometry (d=8, w=2^24) bench + the K4 phase profile build, and the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 || { tail -5 gpurun_out/c5_tests.log; exit 1; }
tail -1 gpurun_out/c5_tests.log
timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_cm.json 2>&1 || exit 2
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_k4p.so timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_k4p.json 2>&1 || exit 3
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_k4p.so timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/c2_k4p.json 2>&1 || exit 4
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/c2_cm.json 2>&1 || exit 5
python3 - <<'PY'
import json
for f in ["c5_cm", "c5_k4p", "c2_k4p", "c2_cm"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d.get("stage_ms_per_step"), d.get("engine_counters"))
PY
