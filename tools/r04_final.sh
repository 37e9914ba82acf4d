#!/bin/bash
# Round-4 final: whole GPU suite, smoke, bench set with rocprof, then the exact A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && bash tools/r04_full.sh && bash tools/r04_ab_ex.sh
