#!/usr/bin/env python3
"""Markdown table of a final run's bench lines (tools/gpu_final.sh output dir):
python tools/final_table.py profiles/r06/final"""
import glob
import json
import os
import sys


def line(path):
    t = open(path).read()
    i = t.find('{"metric')
    return json.loads(t[i:].splitlines()[0]) if i >= 0 else None


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r06/final"
    rows = []
    for name in ["mlm", "clm", "span", "multi-label", "single-class"]:
        p = os.path.join(d, f"bench_{name}.json")
        if not os.path.exists(p):
            continue
        j = line(p)
        rf = j.get("roofline", {})
        iss = rf.get("issue") or {}
        cb = j.get("cpu_baseline") or {}
        allc = cb.get("all_cores") or {}
        ref = cb.get("reference_engine") or {}
        ho = j.get("heldout") or {}
        rows.append(f"| {name} | **{j['value']:,.0f}** | {j['ms_per_step']:.3f} | {rf.get('avg_launch_ms', 0):.3f} "
                    f"({rf.get('kernel', '')}) | {rf.get('frac', 0):.3f} / {iss.get('frac', 0):.2f} | "
                    f"{(rf.get('traffic') or 0) / 1e6:,.0f} / {(rf.get('algorithmic_bytes_per_launch') or 0) / 1e6:,.0f} MB | "
                    f"{cb.get('value', 0):.1f} / {allc.get('value', 0):.1f} / {ref.get('value', 0):.1f} MB/s | "
                    f"{ho.get('value', 0) or 0:,.0f} |")
    print("| task (256 MiB arena, fixture) | value MB/s | ms/step | tokenize launch ms (kernel) | HBM frac / issue frac "
          "| traffic / algorithmic | CPU port 1 thr / 16 thr / HF engine | held-out leg MB/s |")
    print("|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))
    print()
    for p in sorted(glob.glob(os.path.join(d, "heldout_*.json")) + glob.glob(os.path.join(d, "rng1_*.json"))):
        j = line(p)
        if j:
            print(f"- {os.path.basename(p)[:-5]}: {j['value']:,.0f} MB/s, {j['ms_per_step']:.3f} ms/step, "
                  f"tokenize {j.get('roofline', {}).get('avg_launch_ms', 0):.3f} ms")


if __name__ == "__main__":
    main()
