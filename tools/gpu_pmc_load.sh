#!/bin/bash
# the load-only build's FETCH_SIZE (WordPiece text stream calibration) -> gpurun_out/pmcsum/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PMC_SUMMARY_DIR=gpurun_out/pmcsum_load
PMC_TAG=_load PMC_ONLY=FETCH_SIZE PMC_LIB=var/abl3/libsdl_batcher.so bash tools/pmc.sh mlm 256 fixture || exit $?
python tools/pmc_summary.py gpurun_out/pmc_mlm_256_fixture_load mlm 256 fixture > /dev/null || exit 1
rm -rf gpurun_out/pmc_*
