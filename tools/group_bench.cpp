// Concurrent object writers through the C ABI, grouped vs private streaming handles.
// Each of W writer threads feeds its own stream (Go math/rand bytes, kcdc_gorand_read) to
// kcdc_splitter_next in S-byte slices, the way objectWriter.Write does
// (repo/object/object_writer.go:120-136), and records its cut offsets.  Prints one JSON line
// with the aggregate rate of both modes and whether every writer's cuts agree.
//   g++ -O2 -std=c++17 -pthread -Iinclude tools/group_bench.cpp -Lkopia_amd -lkcdc \
//       -Wl,-rpath,'$ORIGIN/../kopia_amd' -o build/group_bench
//   build/group_bench [writers=16] [MiB per writer=64] [slice KiB=64] [name] [wait_us=50] [no_server=0]
// no_server=1: private handles launch one scan per call (KCDC_TEST_NO_SERVER) instead of using
// the resident scan server.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "kcdc.h"

static std::vector<uint64_t> write_object(kcdc_splitter* s, const uint8_t* d, size_t n, size_t slice) {
    std::vector<uint64_t> cuts;
    size_t pos = 0, chunk_start = 0;
    while (pos < n) {
        size_t k = slice < n - pos ? slice : n - pos;
        const uint8_t* p = d + pos;
        size_t base = pos;
        pos += k;
        while (k) {
            const int64_t r = kcdc_splitter_next(s, p, k);
            if (r < -1) {
                std::fprintf(stderr, "kcdc_splitter_next: %s\n", kcdc_last_error());
                std::exit(1);
            }
            if (r < 0) break;
            base += static_cast<size_t>(r);
            cuts.push_back(base);
            chunk_start = base;
            p += r;
            k -= static_cast<size_t>(r);
        }
    }
    if (chunk_start < n) cuts.push_back(n);
    return cuts;
}

int main(int argc, char** argv) {
    const int W = argc > 1 ? std::atoi(argv[1]) : 16;
    const size_t L = (argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 64) << 20;
    const size_t S = (argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 64) << 10;
    const std::string name = argc > 4 ? argv[4] : "DYNAMIC-4M-BUZHASH";
    const uint32_t wait_us = argc > 5 ? static_cast<uint32_t>(std::atoi(argv[5])) : 50;
    const int no_server = argc > 6 ? std::atoi(argv[6]) : 0;
    kcdc_test_set(KCDC_TEST_NO_SERVER, no_server);
    if (kcdc_device_count() < 1) {
        std::fprintf(stderr, "no gfx950 device: %s\n", kcdc_last_error());
        return 1;
    }
    std::vector<std::vector<uint8_t>> data(W, std::vector<uint8_t>(L));
    for (int i = 0; i < W; i++) kcdc_gorand_read(1000 + i, data[i].data(), L);
    auto run = [&](kcdc_group* g, std::vector<std::vector<uint64_t>>& out) {
        std::vector<kcdc_splitter*> hs(W);
        for (int i = 0; i < W; i++) hs[i] = g ? kcdc_group_splitter(g) : kcdc_splitter_new(name.c_str(), 0);
        write_object(hs[0], data[0].data(), 1 << 20, S);  // warm-up (device tables, first launch)
        kcdc_splitter_reset(hs[0]);
        std::vector<std::thread> th;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < W; i++)
            th.emplace_back([&, i] { out[i] = write_object(hs[i], data[i].data(), L, S); });
        for (auto& t : th) t.join();
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (auto* h : hs) kcdc_splitter_close(h);
        return static_cast<double>(W) * L / dt / 1e9;
    };
    std::vector<std::vector<uint64_t>> cg(W), cp(W);
    kcdc_group* g = kcdc_group_new(name.c_str(), 0, 0, wait_us);
    if (!g) {
        std::fprintf(stderr, "kcdc_group_new: %s\n", kcdc_last_error());
        return 1;
    }
    const double grouped = run(g, cg);
    kcdc_group_free(g);
    const double priv = run(nullptr, cp);
    size_t chunks = 0;
    bool same = true;
    for (int i = 0; i < W; i++) {
        same = same && cg[i] == cp[i];
        chunks += cg[i].size();
    }
    std::printf("{\"writers\": %d, \"bytes_per_writer\": %zu, \"slice\": %zu, \"splitter\": \"%s\", \"wait_us\": %u, "
                "\"grouped_gb_s\": %.3f, \"private_gb_s\": %.3f, \"chunks\": %zu, \"identical\": %s}\n",
                W, L, S, name.c_str(), wait_us, grouped, priv, chunks, same ? "true" : "false");
    return same ? 0 : 2;
}
