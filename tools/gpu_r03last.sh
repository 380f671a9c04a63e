#!/bin/bash
# Last record of round 3: the branch-free gather A/B, then the closing record
# (GPU suite, smoke, bench, rocprofv3 headline and full-bench kernel stats).
#   usage: tools/gpu_r03last.sh TAG
set -o pipefail
TAG=${1:-r03last}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_patbf.sh "$TAG/patbf" || exit 1
bash tools/gpu_r03final.sh "$TAG"
