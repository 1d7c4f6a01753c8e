set -u
cd "${GRAFT_REPO_ROOT:-.}"
C=streaming_data_loader_amd/libsdl_batcher.so
CORPORA="fixture heldout" TASK=span tools/gpu_ab.sh $C build/var/wt3/libsdl_batcher.so build/var/wt4/libsdl_batcher.so $C
