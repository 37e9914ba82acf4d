#!/bin/bash
# Round 6: sparse K4 -- the dense-super-bin stress test (20M unique flows at d=8 w=2^24: the
# hash table fills and pieces are halved), then configs[4] at 100M and 200M packets per step
# under a kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_sparse2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_cm_gpu.py -k "beyond_2p26 or wide" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
for P in 100000000 200000000; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$P -o c5 -- \
    python3 bench.py --width 16777216 --depth 8 --no-cpu --windows 0 --steps 5 --warmup 2 --packets $P > $O/c5_$P.json 2> $O/c5_$P.err || { echo "FAIL $P"; tail -3 $O/c5_$P.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c5_$P.json').read().strip().splitlines()[-1]); print($P, d['value'], d['ms_per_step'], d['stage_ms_per_step'])"
  python3 tools/prof_steady.py --last 5 $O/prof_$P/c5_kernel_trace.csv k_extract k_scatter_st k_apply_sparse k_hot_hist k_resolve
done
