#!/bin/bash
# bench A/B over environment settings: ENV_SETS="A=1 B=2;A=3" BARGS="--rng-mode 1" bash tools/gpu_env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-envab}; mkdir -p $O; export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${ENV_SETS:-X=1}"
i=0
for e in "${SETS[@]}"; do
  i=$((i+1))
  env $e timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --soak-s 0 ${BARGS:-} > $O/e$i.json 2> $O/e$i.err || { tail -5 $O/e$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/e$i.json')); print('[$e]', d['value'], d['ms_per_step'], d.get('stage_ms'))" | tee -a $O/summary.txt
done
