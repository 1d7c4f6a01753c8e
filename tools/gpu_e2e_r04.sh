#!/bin/bash
# r04 re-measure of every end-to-end leg at HEAD: per task the record path +
# channel loops (--e2e), JSON filter (--json), JSON lines -> frames sequential / chunked /
# from BGZF gzip (--e2e-frames), device frames (--frames); multi-label / single-class Arrow
# record path (--e2e); device gzip inflate (--gz).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for t in mlm clm span; do
  TAG=e2e_r04/$t TASK=$t bash tools/gpu_hostpaths.sh || exit $?
done
O=gpurun_out/e2e_r04
for t in multi-label single-class; do
  timeout -k 10 300 python bench.py --task $t --steps 3 --warmup 1 --arena-mib 64 --no-cpu-baseline --e2e > $O/e2e_$t.json 2> $O/e2e_$t.err || exit $?
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --gz --no-cpu-baseline --arena-mib 64 > $O/gz_mlm.json 2> $O/gz_mlm.err || exit $?
echo e2e done
