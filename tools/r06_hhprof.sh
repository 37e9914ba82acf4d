#!/bin/bash
# Round 6: the heavy-hitter probe (driver shape) under a rocprofv3 kernel trace, so a
# slow call can be attributed to a kernel, a gap before it, or the host.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06_hhprof}
mkdir -p $O
GNS_HH_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O -o hh -- \
  python3 -u tools/hh_probe.py 25 10 > $O/probe.txt 2>&1
rc=$?; echo "rc=$rc"; grep -v "^\[hh\]" $O/probe.txt | tail -12; find $O -name "*.csv" | head; exit $rc
