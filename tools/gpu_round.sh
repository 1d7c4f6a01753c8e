#!/bin/bash
# Round-end measurement: GPU suite, smoke, the BASELINE configs (fixture + held-out), rocprof
# kernel stats per task, the gzip provider leg.  Output: gpurun_out/round/ (copied to profiles/<round>/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/round; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
step() {  # step NAME LIMIT CMD...: stop on anything but success
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$name] exit $rc" >> $O/steps.log; echo "[$name] exit $rc" >&2
  [ $rc -eq 0 ] || exit $rc
}
step pytest 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step bench_mlm 600 python bench.py > $O/bench_mlm.json 2> $O/bench_mlm.err
for t in span clm; do
  step bench_$t 600 python bench.py --task $t > $O/bench_$t.json 2> $O/bench_$t.err
done
for t in mlm span clm; do
  step heldout_$t 400 python bench.py --task $t --corpus heldout --no-cpu-baseline > $O/heldout_$t.json 2> $O/heldout_$t.err
  step prof_$t 400 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 bench.py --task $t --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$t.json 2> $O/prof_$t.err
done
step gz 400 python bench.py --gz --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_gz.json 2> $O/bench_gz.err
python3 - <<'PY'
import json
for n in ["bench_mlm", "bench_span", "bench_clm", "heldout_mlm", "heldout_span", "heldout_clm"]:
    d = json.load(open(f"gpurun_out/round/{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d.get("cpu_baseline", {}) and d["cpu_baseline"]["value"])
g = json.load(open("gpurun_out/round/bench_gz.json"))["provider_gzip"]
print("gz", g["inflated_MBps"], g["gz_to_text_MBps"], g["members"])
PY
