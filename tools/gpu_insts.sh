#!/bin/bash
# Per-wave instruction mix (SQ_INSTS_*) of each libsdl_batcher.so build:
# one --pmc pass each, kernel trace only.  Usage:
#   TASK=clm tools/gpu_insts.sh lib1 lib2 ...   (then tools/insts_summary.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/insts; rm -rf $O; mkdir -p $O
i=0
for lib in "$@"; do
  i=$((i+1))
  SDL_LIB=$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $O/l$i -o run -- python3 bench.py --task ${TASK:-clm} --steps 2 --warmup 1 --arena-mib 64 --no-cpu-baseline --corpus ${CORPUS:-fixture} > $O/l$i.out 2> $O/l$i.err || exit $?
  echo "$i $lib" >> $O/libs.txt
done
