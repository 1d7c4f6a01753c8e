#!/bin/bash
# One rocprofv3 PMC pass (SQ instruction counts) per library build: where the
# tokenize kernel's instructions go (ablation builds vs the product).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmcvar
mkdir -p $O
i=0
for lib in "$@"; do
  i=$((i+1))
  SDL_LIB=$lib timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --kernel-trace --output-format csv -d $O/v$i -o run -- python3 bench.py --steps 2 --warmup 1 --arena-mib 64 --no-cpu-baseline > $O/v$i.out 2> $O/v$i.err || exit $?
  echo "v$i $lib" >> $O/index.txt
done
