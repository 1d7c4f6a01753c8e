"""Per-record push latency (the reference's channel loop, batcher.rs:33-77: one
sdl_batcher_push per ProviderChannel::Data).  Pushes single records of the bench
corpus and prints the mean / median microseconds per push; run under
`rocprofv3 --kernel-trace --stats` it also gives the launches per push.

    python tools/push_latency.py [--task mlm] [--records 2000]
    SDL_HOST_TIMING=1 python tools/push_latency.py --records 5   # host laps per push
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="mlm")
    ap.add_argument("--records", type=int, default=2000)
    ap.add_argument("--dump", help="write the records length-prefixed (for tools/diag/push_bench) and exit")
    a = ap.parse_args()
    import bench
    records = bench.corpus_records("fixture")
    order = bench.build_order(records, 4 << 20, 0x5D1B)
    texts = [records[i] for i in order][:a.records + 1]
    if a.dump:
        import struct
        with open(a.dump, "wb") as f:
            for x in texts:
                b = x.encode()
                f.write(struct.pack("<I", len(b)) + b)
        return
    t = bench.TASKS[a.task]
    from streaming_data_loader_amd import batcher as Bt
    tt = {"mlm": Bt.TaskType.Mlm, "clm": Bt.TaskType.Clm, "span": Bt.TaskType.Span}[a.task]
    gt = Bt.GenTokenizer.from_config(Bt.get_case(tt, False, t["S"], t["B"], 1234))
    gt.create_sync_batch(texts[0])  # warm
    lat = []
    for x in texts[1:]:
        t0 = time.perf_counter()
        gt.create_sync_batch(x)
        lat.append(time.perf_counter() - t0)
    lat.sort()
    n = len(lat)
    nbytes = sum(len(x.encode()) for x in texts[1:])
    print({"task": a.task, "records": n, "mean_us": round(sum(lat) / n * 1e6, 1),
           "median_us": round(lat[n // 2] * 1e6, 1), "p90_us": round(lat[int(n * 0.9)] * 1e6, 1),
           "MBps": round(nbytes / sum(lat) / 1e6, 2), "mean_record_bytes": round(nbytes / n)})


if __name__ == "__main__":
    main()
