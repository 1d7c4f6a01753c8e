#!/bin/bash
# Build the committed tree's library into build/var/prev (stash, build, restore, rebuild).
set -eu
cd "$(dirname "$0")/.."
git stash -q
python -c "import __graft_entry__ as g; g.build()" > /dev/null
mkdir -p build/var/prev && cp streaming_data_loader_amd/libsdl_batcher.so build/var/prev/
git stash pop -q
python -c "import __graft_entry__ as g; g.build()" > /dev/null
