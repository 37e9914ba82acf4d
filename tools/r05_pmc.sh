#!/bin/bash
# Round 5 rocprofv3 evidence (GPU box): kernel trace + FETCH_SIZE and WRITE_SIZE
# passes (one counter set per run) for one bench workload.
# usage: tools/r05_pmc.sh <c2|c5|hybrid|ss> [extra bench args]
#   then tools/pmc_traffic.py <fetch csv> <write csv> <profiles/traffic_*.json>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
w=$1; shift
case $w in
    c2) A="--steps 3 --warmup 1 --no-cpu --windows 0" ;;
    c5) A="--width 16777216 --depth 8 --steps 3 --warmup 1 --no-cpu --windows 0" ;;
    hybrid) A="--sketch hybrid --steps 3 --warmup 1 --no-cpu" ;;
    ss) A="--sketch superspread --steps 6 --warmup 1 --no-cpu" ;;
    *) echo "unknown workload $w"; exit 2 ;;
esac
O=gpurun_out/pmc_$w
mkdir -p $O
B="python3 bench.py $A $*"
echo "== $w trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o k -- $B > $O/trace.log 2>&1 && \
echo "== $w fetch" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o k -- $B > $O/fetch.log 2>&1 && \
echo "== $w write" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o k -- $B > $O/write.log 2>&1 && \
echo "== $w done"
