#!/bin/bash
# r06: GPU suite + smoke, span kernel timelines (fixture, held-out), Unigram phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
if [ -z "${NO_SUITE:-}" ]; then bash tools/gpu_suite.sh || exit $?; fi
OUT=${OUT:-r06uni} K=16 bash tools/gpu_trace.sh "--task span --no-heldout" "--task span --corpus heldout --no-heldout" || exit $?
bash tools/gpu_uni_stamps.sh
