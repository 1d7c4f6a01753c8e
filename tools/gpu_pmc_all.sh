#!/bin/bash
# PMC passes (tools/pmc.sh) of the tokenize kernels for mlm / clm / span on both
# corpora at the bench arena size; summarise locally with tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CORPORA:-fixture heldout}; do
  for t in ${TASKS:-mlm clm span}; do
    bash tools/pmc.sh $t 256 $c || exit $?
  done
done
echo pmc all done
