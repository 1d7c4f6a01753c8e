#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into profiles/pmc/<task>_<arena>mib.json
(bench.py reads it only for the same task and arena size).

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB units), the gfx950
FETCH_SIZE correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half the
bytes of a 16 B/lane streaming read).  Averaged over every launch of a kernel.

    python tools/pmc_summary.py gpurun_out/pmc TASK ARENA_MIB [CORPUS]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    task = sys.argv[2] if len(sys.argv) > 2 else "mlm"
    arena = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    corpus = sys.argv[4] if len(sys.argv) > 4 else "fixture"
    out_dir = os.environ.get("PMC_SUMMARY_DIR", "profiles/pmc")  # (on a GPU box: under gpurun_out/)
    os.makedirs(out_dir, exist_ok=True)
    dst = f"{out_dir}/{task}_{arena}mib" + ("" if corpus == "fixture" else f"_{corpus}") + ".json"
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for f in sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = short(row["Kernel_Name"])
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    out = {"source": f"rocprofv3 --pmc passes of bench.py --task {task} --arena-mib {arena} --corpus {corpus} "
                     "(tools/pmc.sh)",
           "task": task, "arena_mib": arena, "corpus": corpus, "kernels": {}}
    # provenance: the library the passes ran (its embedded source hash) and, when the caller
    # passes it (the GPU box has no .git), the commit
    from streaming_data_loader_amd import build
    out["library_build_id"] = build.embedded_id(os.environ.get("SDL_LIB") or build.LIB)
    if os.environ.get("SDL_HEAD"):
        out["head"] = os.environ["SDL_HEAD"]
    import time
    out["date"] = time.strftime("%Y-%m-%d") + (f" ({os.environ['SDL_ROUND']})" if os.environ.get("SDL_ROUND") else "")
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        ent = {"launches": max(len(v) for v in cs.values()), "counters": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            # (the uniform x2 upper bound; bench.py pmc_traffic splits the stream from the rest)
            ent["hbm_bytes_per_launch"] = int((2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024)
        out["kernels"][k] = ent
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
