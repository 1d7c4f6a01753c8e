// Per-record push latency at the C ABI (what a Rust `impl Batcher` calling sdl_batcher_push
// per ProviderChannel::Data pays, without the Python mirror): records from a length-prefixed
// file (tools/push_latency.py --dump), one sdl_batcher_push each, emitted batches released.
//   push_bench RECORDS.bin TOKENIZER.json TASK(0 mlm, 1 clm, 2 span) S B [N]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "sdl_batcher.h"

int main(int argc, char **argv) {
    if (argc < 6) return 2;
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<std::vector<uint8_t>> recs;
    uint32_t len;
    while (std::fread(&len, 4, 1, f) == 1) {
        std::vector<uint8_t> r(len);
        if (len && std::fread(r.data(), 1, len, f) != len) return 2;
        recs.push_back(std::move(r));
    }
    std::fclose(f);
    sdl_config c;
    sdl_config_default(&c, std::atoi(argv[3]));
    c.sequence_length = std::atoi(argv[4]);
    c.batch_size = std::atoi(argv[5]);
    c.mask_length = (int32_t)((float)c.sequence_length * 0.15f);
    c.seed = 1234;
    sdl_batcher *h = nullptr;
    if (sdl_batcher_create(&c, argv[2], nullptr, &h) != 0) {
        std::fprintf(stderr, "create: %s\n", sdl_last_error());
        return 3;
    }
    const size_t n = argc > 6 ? (size_t)std::atoi(argv[6]) : recs.size() - 1;
    sdl_batch b;
    (void)sdl_batcher_push(h, recs[0].data(), recs[0].size(), nullptr, 0, &b);  // warm
    std::vector<double> us;
    size_t bytes = 0, emitted = 0;
    for (size_t i = 1; i <= n && i < recs.size(); ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = sdl_batcher_push(h, recs[i].data(), recs[i].size(), nullptr, 0, &b);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc < 0) {
            std::fprintf(stderr, "push: %s\n", sdl_last_error());
            return 4;
        }
        if (rc == 1) {
            ++emitted;
            sdl_batch_release(&b);
        }
        us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        bytes += recs[i].size();
    }
    double sum = 0;
    for (double x : us) sum += x;
    std::vector<double> s = us;
    std::sort(s.begin(), s.end());
    std::printf("{\"task\": %s, \"records\": %zu, \"mean_us\": %.1f, \"median_us\": %.1f, \"p90_us\": %.1f, "
                "\"MBps\": %.2f, \"emitted\": %zu}\n",
                argv[3], us.size(), sum / us.size(), s[s.size() / 2], s[s.size() * 9 / 10], bytes / sum, emitted);
    sdl_batcher_destroy(h);
    return 0;
}
