#!/bin/bash
# PMC: every task's counter passes at 256 MiB (fixture), mlm/clm/span held-out fetch/write,
# (the stream calibration is tools/gpu_pmc_load.sh).  Summarised on the
# box (gpurun_out/pmcsum/*.json -> profiles/pmc/) and the raw counter CSVs dropped (> 64 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PMC_SUMMARY_DIR=gpurun_out/pmcsum
summ() {  # task corpus
  python tools/pmc_summary.py gpurun_out/pmc_$1_256_$2 $1 256 $2 > /dev/null || return 1
  cp gpurun_out/pmc_$1_256_$2/passes.log $PMC_SUMMARY_DIR/$1_$2_passes.log
}
for t in mlm multi-label clm span; do
  bash tools/pmc.sh $t 256 fixture || exit $?
  summ $t fixture || exit 1
done
for t in mlm clm span; do
  PMC_ONLY=FETCH_SIZE bash tools/pmc.sh $t 256 heldout || exit $?
  PMC_ONLY=WRITE_SIZE bash tools/pmc.sh $t 256 heldout || exit $?
  summ $t heldout || exit 1
done
rm -rf gpurun_out/pmc_*
ls $PMC_SUMMARY_DIR
