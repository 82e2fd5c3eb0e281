// Batching object writers through the C ABI (kcdc_bw_*): W writer threads
// each feed their own object in S-byte slices, the way the uploader drives objectWriter.Write
// (snapshot/upload/upload.go:394-407, repo/object/object_writer.go:113-139), poll the final
// cuts as they arrive and finish.  The aggregate rate counts every byte from host memory to
// final cut lists (PCIe included).  The cuts are checked against kcdc_split_batch_host on the
// same objects (the whole-stream path, itself checked against the oracle by the GPU tests).
// Prints one JSON line.
//   build/writer_bench [writers=64] [MiB per writer=64] [slice KiB=64] [name] [round MiB=256] [reps=3] [hash=none]
// hash: a content-hash name (kcdc_bw_batcher_hash with a 32-byte secret): every final chunk is also
// named on the device and the rate counts host bytes to (cut, ID) pairs.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>
#include <algorithm>

#include "kcdc.h"

__attribute__((target("avx2"))) static void nt_copy(uint8_t* d, const uint8_t* s, size_t n) {
    const size_t h = std::min<size_t>(n, (32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31);
    std::memcpy(d, s, h);
    d += h, s += h, n -= h;
    for (; n >= 32; n -= 32, d += 32, s += 32)
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d), _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s)));
    std::memcpy(d, s, n);
    _mm_sfence();
}

int main(int argc, char** argv) {
    const int W = argc > 1 ? std::atoi(argv[1]) : 64;
    const size_t L = (argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 64) << 20;
    const size_t S = (argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 64) << 10;
    const std::string name = argc > 4 ? argv[4] : "DYNAMIC-4M-BUZHASH";
    const uint64_t round = (argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 256) << 20;
    const int reps = argc > 6 ? std::atoi(argv[6]) : 3;
    const std::string hash = argc > 7 ? argv[7] : "none";
    const bool ids = hash != "none";
    if (kcdc_device_count() < 1) {
        std::fprintf(stderr, "no gfx950 device: %s\n", kcdc_last_error());
        return 1;
    }
    std::vector<std::vector<uint8_t>> data(W, std::vector<uint8_t>(L));
    {
        std::vector<std::thread> th;
        for (int i = 0; i < W; i++)
            th.emplace_back([&, i] {
                uint64_t x = 0x9E3779B97F4A7C15ull * (i + 1);
                uint64_t* p = reinterpret_cast<uint64_t*>(data[i].data());
                for (size_t k = 0; k < L / 8; k++) {
                    x ^= x << 13;
                    x ^= x >> 7;
                    x ^= x << 17;
                    p[k] = x;
                }
            });
        for (auto& t : th) t.join();
    }
    // reference cuts: the whole-stream host path
    std::vector<const uint8_t*> ptrs(W);
    std::vector<uint64_t> lens(W, L), base(W), counts(W);
    uint64_t cap = 0;
    for (int i = 0; i < W; i++) {
        ptrs[i] = data[i].data();
        base[i] = cap;
        cap += kcdc_cut_capacity(name.c_str(), L);
    }
    std::vector<uint64_t> ref(cap);
    if (kcdc_split_batch_host(name.c_str(), ptrs.data(), lens.data(), W, ref.data(), cap, base.data(), counts.data(), 0)) {
        std::fprintf(stderr, "kcdc_split_batch_host: %s\n", kcdc_last_error());
        return 1;
    }
    kcdc_bw_batcher* b = kcdc_bw_batcher_new(name.c_str(), 0, round, 2000);
    if (!b) {
        std::fprintf(stderr, "kcdc_bw_batcher_new: %s\n", kcdc_last_error());
        return 1;
    }
    if (ids) {
        uint8_t key[32];
        for (int i = 0; i < 32; i++) key[i] = static_cast<uint8_t>(7 + i);
        if (kcdc_bw_batcher_hash(b, hash.c_str(), key, 32)) {
            std::fprintf(stderr, "kcdc_bw_batcher_hash: %s\n", kcdc_last_error());
            return 1;
        }
    }
    std::vector<double> rates;
    std::vector<double> fin_ms;  // per object: kcdc_bw_finish's latency (what Result() waits on), timed reps
    std::mutex fin_mu;
    double st0[24] = {0};  // the stats after the warm-up rep: the steady-state pool misses are the rest
    bool ok = true;
    for (int r = 0; r < reps + 1; r++) {  // rep 0 warms the pinned pool and device buffers
        std::vector<std::vector<uint64_t>> got(W);
        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        std::vector<std::thread> th;
        for (int i = 0; i < W; i++)
            th.emplace_back([&, i] {
                kcdc_bw* w = kcdc_bw_open(b);
                uint64_t buf[256];
                static thread_local uint8_t idbuf[256 * 32];
                auto take = [&] {
                    if (ids) {
                        for (int64_t n; (n = kcdc_bw_cuts_ids(w, buf, idbuf, 32, 256)) > 0;)
                            got[i].insert(got[i].end(), buf, buf + n);
                    } else {
                        for (int64_t n; (n = kcdc_bw_cuts(w, buf, 256)) > 0;) got[i].insert(got[i].end(), buf, buf + n);
                    }
                };
                ready++;
                while (!go.load()) std::this_thread::yield();
                size_t pos = 0, calls = 0;
                while (pos < L) {
                    const size_t k = S < L - pos ? S : L - pos;
                    if (kcdc_bw_write(w, data[i].data() + pos, k)) {
                        std::fprintf(stderr, "kcdc_bw_write: %s\n", kcdc_last_error());
                        std::exit(1);
                    }
                    pos += k;
                    if (++calls % 16 == 0) take();
                }
                const auto f0 = std::chrono::steady_clock::now();
                if (kcdc_bw_finish(w)) {
                    std::fprintf(stderr, "kcdc_bw_finish: %s\n", kcdc_last_error());
                    std::exit(1);
                }
                if (r > 0) {
                    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count();
                    std::lock_guard<std::mutex> fl(fin_mu);
                    fin_ms.push_back(ms);
                }
                take();
                kcdc_bw_free(w);
            });
        while (ready.load() < W) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        go = true;
        for (auto& t : th) t.join();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (r > 0) rates.push_back(static_cast<double>(W) * L / s / (1ull << 30));
        if (r == 0) kcdc_bw_stats(b, st0, 24);
        for (int i = 0; i < W; i++)
            ok = ok && got[i] == std::vector<uint64_t>(ref.begin() + base[i], ref.begin() + base[i] + counts[i]);
    }
    const int64_t rounds = kcdc_bw_rounds(b);
    double st[24] = {0};
    kcdc_bw_stats(b, st, 24);
    kcdc_bw_batcher_free(b);
    // the host-side ceiling: the same W threads only copying their slices into 4 MiB buffers
    double copy_rate = 0;
    {
        std::vector<std::vector<uint8_t>> stage(W, std::vector<uint8_t>(4u << 20));
        std::vector<std::thread> th;
        std::atomic<bool> go{false};
        for (int i = 0; i < W; i++)
            th.emplace_back([&, i] {
                while (!go.load()) std::this_thread::yield();
                size_t at = 0;
                for (size_t pos = 0; pos < L; pos += S) {
                    const size_t k = S < L - pos ? S : L - pos;
                    if (at + k > stage[i].size()) at = 0;
                    std::memcpy(stage[i].data() + at, data[i].data() + pos, k);
                    at += k;
                }
            });
        const auto t0 = std::chrono::steady_clock::now();
        go = true;
        for (auto& t : th) t.join();
        copy_rate = static_cast<double>(W) * L / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() /
                    (1ull << 30);
    }
    // the same, with non-temporal stores (what the batcher's staging copy uses on AVX2 hosts)
    double copy_nt_rate = 0;
    if (__builtin_cpu_supports("avx2")) {
        std::vector<uint8_t*> stage(W);
        for (auto& p : stage) p = static_cast<uint8_t*>(std::aligned_alloc(64, 4u << 20));
        std::vector<std::thread> th;
        std::atomic<bool> go{false};
        for (int i = 0; i < W; i++)
            th.emplace_back([&, i] {
                while (!go.load()) std::this_thread::yield();
                size_t at = 0;
                for (size_t pos = 0; pos < L; pos += S) {
                    const size_t k = S < L - pos ? S : L - pos;
                    if (at + k > (4u << 20)) at = 0;
                    nt_copy(stage[i] + at, data[i].data() + pos, k);
                    at += k;
                }
            });
        const auto t0 = std::chrono::steady_clock::now();
        go = true;
        for (auto& t : th) t.join();
        copy_nt_rate = static_cast<double>(W) * L / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() /
                       (1ull << 30);
        for (auto& p : stage) std::free(p);
    }
    std::sort(fin_ms.begin(), fin_ms.end());
    auto pct = [&](double q) { return fin_ms.empty() ? 0.0 : fin_ms[std::min(fin_ms.size() - 1, static_cast<size_t>(q * fin_ms.size()))]; };
    double best = 0, sum = 0;
    for (double x : rates) {
        best = x > best ? x : best;
        sum += x;
    }
    std::printf("{\"writers\": %d, \"mib_per_writer\": %zu, \"slice_kib\": %zu, \"name\": \"%s\", \"round_mib\": %llu, "
                "\"gib_s_mean\": %.2f, \"gib_s_best\": %.2f, \"rounds\": %lld, \"round_submit_s\": %.3f, "
                "\"round_wait_s\": %.3f, \"dev_gather_s\": %.3f, \"dev_split_s\": %.3f, \"dev_span_s\": %.3f, "
                "\"dev_busy_s\": %.3f, \"host_s\": [%.3f, %.3f, %.3f, %.3f, %.3f], "
                "\"round_idle_s\": %.3f, \"writer_capped_s\": %.3f, \"writer_block_s\": %.3f, \"pool_misses\": %.0f, \"pool_misses_after_warmup\": %.0f, \"writer_block_s_after_warmup\": %.3f, \"round_lock_s\": %.3f, "
                "\"memcpy_only_gib_s\": %.2f, \"memcpy_nt_only_gib_s\": %.2f, \"hash\": \"%s\", \"ids_named\": %.0f, \"hash_steps\": %.0f, \"hash_dev_s\": %.3f, \"id_space_wait_s\": %.3f, \"hash_idle_s\": %.3f, \"chains_per_step\": %.0f, \"finish_ms_p50\": %.2f, \"finish_ms_p99\": %.2f, \"finish_ms_max\": %.2f, \"parity_ok\": %s}\n",
                W, L >> 20, S >> 10, name.c_str(), static_cast<unsigned long long>(round >> 20),
                rates.empty() ? 0.0 : sum / rates.size(), best, static_cast<long long>(rounds), st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11], st[12], st[13], st[14], st[15], st[16], st[16] - st0[16], st[15] - st0[15], st[17], copy_rate, copy_nt_rate,
                hash.c_str(), st[18], st[19], st[20], st[21], st[22], st[19] > 0 ? st[23] / st[19] : 0.0, pct(0.5), pct(0.99), fin_ms.empty() ? 0.0 : fin_ms.back(), ok ? "true" : "false");
    return ok ? 0 : 2;
}
