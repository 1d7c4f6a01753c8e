"""k_bpe_long's cached-merge LDS path (tokenize_bpe.hip, r04) as a Python model of its wave
steps, against the uncached merge loop it replaced, on random merge tables and pieces of up
to 300 symbols (several 64-symbol tiles).  The GPU tests compare the kernel itself with the
oracle and the tokenizers goldens (test_gpu_gpt2.py, test_gpu_full_size.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "sim"))


def test_cached_merges_equal_uncached_loop():
    import bpe_long_cache_sim as m
    assert m.run(1000, seed=7)
