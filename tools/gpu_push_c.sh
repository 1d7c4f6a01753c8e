#!/bin/bash
# per-record push at the C ABI (tools/diag/push_bench.cpp -> var/push_bench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/push_c; mkdir -p $O; export TMPDIR=/tmp
python tools/push_latency.py --dump /tmp/sdl_records.bin || exit $?
A=streaming_data_loader_amd/assets
timeout -k 10 120 ./var/push_bench /tmp/sdl_records.bin $A/bert_proxy/tokenizer.json 0 512 256 | tee $O/lat.txt || exit $?
timeout -k 10 120 ./var/push_bench /tmp/sdl_records.bin $A/gpt2_proxy/tokenizer.json 1 1024 128 | tee -a $O/lat.txt || exit $?
timeout -k 10 120 ./var/push_bench /tmp/sdl_records.bin $A/t5_proxy/tokenizer.json 2 512 256 | tee -a $O/lat.txt || exit $?
