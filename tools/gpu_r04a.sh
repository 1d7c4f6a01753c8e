set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_inflate.py tests/test_inflate_fuzz.py tests/test_gpu_drop_in.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --gz --no-cpu-baseline > $O/bench_gz.json 2> $O/bench_gz.err || { tail -30 $O/bench_gz.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_gz.json')); print(json.dumps(d.get('provider_gzip'), indent=1)[:3000])"
