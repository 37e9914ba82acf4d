#!/bin/bash
# Round-4 measurement run (GPU box): the bench lines DESIGN.md §6 quotes, then
# rocprofv3 kernel statistics of the headline and SuperSpread steps.  Every GPU
# step has its own time limit; the script stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r04
O=gpurun_out/r04
run() {  # name, seconds, bench args...
    local n=$1 t=$2
    shift 2
    echo "== $n" && timeout -k 10 "$t" python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n rc=$?"; tail -5 $O/$n.err; exit 1; }
    tail -c 400 $O/$n.json
}
run headline 300 --no-cpu &&
run default 500 &&
run ss 300 --sketch superspread --no-cpu &&
run host_compact 300 --host-input compact --no-cpu &&
run host_headers 300 --host-input headers --no-cpu &&
run c5 400 --width 16777216 --depth 8 --no-cpu &&
run exact 300 --sketch exact --no-cpu &&
run hybrid 500 --sketch hybrid --no-cpu &&
echo "== rocprof headline" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cm -o cm -- \
    python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_cm.log 2>&1 &&
echo "== rocprof ss" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ss -o ss -- \
    python3 bench.py --sketch superspread --no-cpu --steps 3 --warmup 1 > $O/prof_ss.log 2>&1 &&
echo done
