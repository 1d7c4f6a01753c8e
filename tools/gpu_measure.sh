#!/bin/bash
# Bench lines + rocprof kernel stats on the box.  Each argument is one run:
#   NAME:ARGS      -> gpurun_out/meas/NAME.json (bench.py ARGS)
#   prof/NAME:ARGS -> the same under rocprofv3 --kernel-trace --stats (gpurun_out/meas/prof_NAME/)
# e.g. bash tools/gpu_measure.sh "mlm:" "span_r1:--task span --rng-mode 1 --no-cpu-baseline"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/meas; mkdir -p $O
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  if [[ $name == prof/* ]]; then
    n=${name#prof/}
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 bench.py $args --steps 5 --warmup 2 > $O/prof_$n.json 2> $O/prof_$n.err
  else
    n=$name
    timeout -k 10 500 python bench.py $args > $O/$n.json 2> $O/$n.err
  fi
  rc=$?
  echo "[$name] exit $rc" | tee -a $O/steps.log
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json,sys
d=json.load(open('$O/'+'$([[ $name == prof/* ]] && echo prof_)$n'+'.json'))
r=d['roofline']; print('$n', d['value'], 'MB/s', d['ms_per_step'], 'ms/step', r['avg_launch_ms'], r['bound'], r['frac'], d.get('stage_ms'))
" | tee -a $O/summary.log
done
