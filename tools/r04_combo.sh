#!/bin/bash
# SuperSpread check then the K1 A/B, one GPU call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && bash tools/r04_ss.sh && bash tools/r04_ab_v4.sh
