#!/bin/bash
# Round-6 measurement runs (GPU box).  usage: tools/r06_bench.sh <tag> <leg>...
# legs: driver (the driver's exact command: --steps 20 --warmup 5, CPU legs + parity), default,
# headline (--no-cpu), c5 (configs[4] geometry with the CPU leg + in-line parity), c5fast (--no-cpu),
# c5big (configs[4] geometry, 200M-packet steps = device batches, CPU leg + parity),
# ss, exact, hybrid, thrift, srcip, c1, host_compact, prof_cm / prof_c5 / prof_ss (rocprofv3 kernel
# traces, >= 10 steady full-batch launches).  Every GPU step has its own time limit; the
# script stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
run() {  # name, seconds, bench args...
    local n=$1 t=$2
    shift 2
    echo "== $n" && timeout -k 10 "$t" python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n rc=$?"; tail -5 $O/$n.err; exit 1; }
    tail -c 700 $O/$n.json
}
prof() {  # name, seconds, bench args...
    local n=$1 t=$2
    shift 2
    echo "== rocprof $n" && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o $n -- \
        python3 bench.py "$@" > $O/prof_$n.log 2>&1 || { echo "FAIL prof $n rc=$?"; tail -5 $O/prof_$n.log; exit 1; }
    tail -c 300 $O/prof_$n.log
}
for leg in "$@"; do
    case $leg in
        driver) run driver 500 --gpus 1 --steps 20 --warmup 5 ;;
        default) run default 500 ;;
        headline) run headline 300 --no-cpu ;;
        ss) run ss 400 --sketch superspread ;;
        c5) run c5 600 --width 16777216 --depth 8 ;;
        c5fast) run c5fast 400 --width 16777216 --depth 8 --no-cpu ;;
        c5big) run c5big 600 --width 16777216 --depth 8 --packets 200000000 ;;
        exact) run exact 300 --sketch exact --no-cpu ;;
        hybrid) run hybrid 500 --sketch hybrid --no-cpu ;;
        host_compact) run host_compact 300 --host-input compact --no-cpu ;;
        host_compact16) run host_compact16 300 --host-input compact16 --no-cpu ;;
        thrift) run thrift 400 --sketch thrift --no-cpu ;;
        srcip) run srcip 400 --key srcip --no-cpu ;;
        c1) run c1 600 --config c1 ;;
        prof_cm) prof cm 400 --no-cpu --steps 10 --warmup 5 --windows 0 ;;
        prof_ss) prof ss 400 --sketch superspread --no-cpu --steps 10 --warmup 5 ;;
        prof_c5) prof c5 500 --width 16777216 --depth 8 --no-cpu --steps 10 --warmup 5 --windows 0 ;;
        prof_c5big) prof c5big 600 --width 16777216 --depth 8 --packets 200000000 --no-cpu --steps 10 --warmup 3 --windows 0 ;;
        *) echo "unknown leg $leg"; exit 2 ;;
    esac || exit 1
done
echo done
