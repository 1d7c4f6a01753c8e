#!/bin/bash
# PMC passes for the tokenize kernel (one counter group per rocprofv3 run,
# kernel-trace/stats only -- no sys/runtime trace with --pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TASK="${1:-mlm}"
ARENA="${2:-256}"
CORPUS="${3:-fixture}"
D=gpurun_out/pmc_${TASK}_${ARENA}_${CORPUS}${PMC_TAG:-}
mkdir -p $D
export TMPDIR=/tmp
ARGS="--task $TASK --steps 2 --warmup 1 --arena-mib $ARENA --corpus $CORPUS --no-cpu-baseline ${PMC_EXTRA:-}"
i=0
while IFS= read -r group; do
  [[ -z "$group" ]] && continue
  i=$((i+1))
  [[ -n "${PMC_ONLY:-}" && "$group" != "$PMC_ONLY" ]] && continue
  SDL_LIB=${PMC_LIB:-} timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $D/p$i -o run -- python3 bench.py $ARGS > $D/p$i.out 2> $D/p$i.err
  rc=$?
  echo "pass $i [$group] exit $rc" | tee -a $D/passes.log
  case $rc in 0) ;; *) exit $rc;; esac
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT
GROUPS
