#!/bin/bash
# SuperSpread counters: SQ passes and FETCH/WRITE traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && PMC_BENCH_ARGS="--sketch superspread" bash tools/pmc_sq.sh && bash tools/pmc_ss.sh && echo pmc-ss-ok
