// Host memcpy rate into pinned staging (coherent vs default) and kcdc_splitter_next latency
// with the resident scan server on/off, from native code (no Python in the loop).
//   hipcc -O2 -std=c++17 -Iinclude tools/stage_copy.cpp -Lkopia_amd -lkcdc -Wl,-rpath,'$ORIGIN/../kopia_amd' -o build/stage_copy
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "kcdc.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    std::vector<uint8_t> src(8 << 20);
    for (size_t i = 0; i < src.size(); i++) src[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
    for (unsigned flags : {unsigned(hipHostMallocMapped), unsigned(hipHostMallocMapped | hipHostMallocCoherent)}) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 8 << 20, flags) != hipSuccess) return 1;
        for (size_t n : {size_t(64) << 10, size_t(1) << 20}) {
            std::memcpy(p, src.data(), n);
            const double t0 = now_us();
            for (int r = 0; r < 200; r++) std::memcpy(p, src.data() + (r % 7) * 4096, n);
            const double t = (now_us() - t0) / 200;
            std::printf("{\"memcpy_into\": \"%s\", \"bytes\": %zu, \"us\": %.2f, \"gb_s\": %.2f}\n",
                        flags & hipHostMallocCoherent ? "coherent" : "mapped", n, t, n / t / 1e3);
        }
        (void)hipHostFree(p);
    }
    const char* name = "DYNAMIC-8M-BUZHASH";
    for (int off : {0, 1, 0, 1}) {
        kcdc_test_set(KCDC_TEST_NO_SERVER, off);
        for (size_t S : {size_t(64) << 10, size_t(1) << 20}) {
            kcdc_splitter* s = kcdc_splitter_new(name, 0);
            kcdc_splitter_next(s, src.data(), (4 << 20) - 1);  // below min: no GPU
            size_t i = (4 << 20) - 1;
            int calls = 0;
            double t = 0;
            while (i + S <= src.size() && calls < 200) {
                const double t0 = now_us();
                const int64_t r = kcdc_splitter_next(s, src.data() + i, S);
                t += now_us() - t0;
                calls++;
                if (r >= 0) break;
                i += S;
            }
            kcdc_splitter_close(s);
            std::printf("{\"server\": %s, \"slice\": %zu, \"calls\": %d, \"us_per_call\": %.1f, \"gb_s\": %.3f}\n",
                        off ? "false" : "true", S, calls, t / calls, calls * S / t / 1e3);
        }
    }
    return 0;
}
