#!/bin/bash
# single-class PMC passes (summarised on the box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PMC_SUMMARY_DIR=gpurun_out/pmcsum_sc
bash tools/pmc.sh single-class 256 fixture || exit $?
python tools/pmc_summary.py gpurun_out/pmc_single-class_256_fixture single-class 256 fixture > /dev/null || exit 1
cp gpurun_out/pmc_single-class_256_fixture/passes.log $PMC_SUMMARY_DIR/single-class_fixture_passes.log
rm -rf gpurun_out/pmc_*
timeout -k 10 240 python bench.py --task single-class --no-cpu-baseline > $PMC_SUMMARY_DIR/bench_single-class.json 2>/dev/null || exit $?
