"""Stream calibration for bench.py pmc_traffic: FETCH_SIZE of the load-only WordPiece build
(SDL_ABLATE=3, tools/gpu_pmc_load.sh) per byte of the text + offsets stream it reads, on the
bench's fixture arena of the same size.

    python tools/pmc_calibration.py gpurun_out/pmcsum_load/mlm_256mib.json [ARENA_MIB]
      -> profiles/pmc/stream_calibration.json
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    src = sys.argv[1]
    arena_mib = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    with open(src) as f:
        summ = json.load(f)
    k = next(v for n, v in summ["kernels"].items() if "k_wordpiece_chunks" in n)
    fetch = k["counters"]["FETCH_SIZE"] * 1024
    _, _, offs, _, _ = bench.shard(0, arena_mib << 20, "fixture", 1)
    R = len(offs) - 1
    stream = int(offs[-1]) + 8 * (R + 1)
    out = {"source": f"{summ['source']} with var/abl3 (SDL_ABLATE=3: windows staged, nothing tokenized)",
           "arena_mib": arena_mib, "text_bytes": int(offs[-1]), "records": R, "stream_bytes": stream,
           "load_only_fetch_bytes": int(fetch), "launches": k["launches"], "ratio": fetch / stream}
    dst = os.path.join(REPO, "profiles", "pmc", "stream_calibration.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
