#!/bin/bash
# r06 final, WordPiece tasks again after the last WordPiece change: GPU suite + smoke, PMC passes
# (mlm, multi-label, single-class fixture; mlm held-out FETCH/WRITE) summarised and put in
# profiles/pmc of this box's copy, then the WordPiece bench lines + rocprof stats.
# Output: gpurun_out/pmcsum/, gpurun_out/r06final_wp/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PMC_SUMMARY_DIR=gpurun_out/pmcsum SDL_ROUND=r06
bash tools/gpu_suite.sh || exit $?
summ() {  # task corpus
  python tools/pmc_summary.py gpurun_out/pmc_$1_256_$2 $1 256 $2 > /dev/null || return 1
  cp gpurun_out/pmc_$1_256_$2/passes.log $PMC_SUMMARY_DIR/$1_$2_passes.log
}
for t in mlm multi-label single-class; do
  bash tools/pmc.sh $t 256 fixture || exit $?
  summ $t fixture || exit 1
done
PMC_ONLY=FETCH_SIZE bash tools/pmc.sh mlm 256 heldout || exit $?
PMC_ONLY=WRITE_SIZE bash tools/pmc.sh mlm 256 heldout || exit $?
summ mlm heldout || exit 1
rm -rf gpurun_out/pmc_*
cp $PMC_SUMMARY_DIR/*.json profiles/pmc/
O=gpurun_out/r06final_wp; mkdir -p $O
for t in mlm multi-label single-class; do
  timeout -k 10 240 python bench.py --task $t > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 bench.py --task $t --no-cpu-baseline --no-heldout > $O/prof_$t.out 2>&1 || exit $?
  find $O/prof_$t -name '*kernel_trace.csv' -delete
done
timeout -k 10 240 python bench.py --task mlm --corpus heldout --no-cpu-baseline > $O/heldout_mlm.json 2> $O/heldout_mlm.err || exit $?
timeout -k 10 240 python bench.py --task mlm --rng-mode 1 --no-cpu-baseline > $O/rng1_mlm.json 2> $O/rng1_mlm.err || exit $?
ls $O
