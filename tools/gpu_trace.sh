#!/bin/bash
# Kernel timeline (last dispatches) of a short bench run per configuration in $@ (bench args, quoted)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-trace}; mkdir -p $O; export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/t$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --soak-s 0 $a > $O/t$i.out 2> $O/t$i.err || { tail -5 $O/t$i.err; exit 1; }
  f=$(find $O/t$i -name '*kernel_trace.csv' | head -1)
  echo "== $a" | tee $O/t$i.txt; python3 tools/trace_timeline.py "$f" ${K:-30} | tee -a $O/t$i.txt
  rm -f "$f"
done
