#!/bin/bash
# Round-2 check: full GPU suite, headline bench, C5 geometry bench (+K4 phase profile), hybrid configs[4] bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r02_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/c2_cm.json 2>&1 || exit 5
timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_cm.json 2>&1 || exit 2
if [ -f go2netspectra_amd/libgns_sketch_k4p.so ]; then
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_k4p.so timeout -k 10 200 python bench.py --width 16777216 --depth 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_k4p.json 2>&1 || exit 3
fi
timeout -k 10 300 python bench.py --sketch hybrid --steps 5 --warmup 1 > gpurun_out/c4_hybrid.json 2>&1 || exit 4
python3 - <<'PY'
import json, os
for f in ["c2_cm", "c5_cm", "c5_k4p", "c4_hybrid"]:
    if not os.path.exists(f"gpurun_out/{f}.json"): continue
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d.get("stage_ms_per_step"), d.get("engine_counters"), d.get("queries"))
PY
