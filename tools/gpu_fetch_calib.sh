#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_wordpiece_chunks for the product build and the
# load-only ablation (SDL_ABLATE=3: the 16-B text stream and nothing else), mlm 256 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/calib; rm -rf $O; mkdir -p $O
A="bench.py --task mlm --steps 2 --warmup 1 --arena-mib 256 --no-cpu-baseline"
for v in prod abl3; do
  L=streaming_data_loader_amd/libsdl_batcher.so; [ $v = abl3 ] && L=build/abl3/libsdl_batcher.so
  for c in FETCH_SIZE WRITE_SIZE; do
    SDL_LIB=$L timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${v}_$c -o run -- python3 $A > $O/${v}_$c.out 2> $O/${v}_$c.err || exit $?
    f=$(find $O/${v}_$c -name '*counter_collection.csv' | head -1)
    python3 - "$f" "$v" "$c" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_wordpiece_chunks" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
vals = [sum(v) for v in acc.values()]
print(sys.argv[2], sys.argv[3], "per launch (kB):", [round(v) for v in vals])
PY
  done
done
