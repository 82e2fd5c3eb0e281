// Memory-side microbenchmark for the batch splitter's access pattern (no hashing).
// A wave owns tiles of 64 lane segments x L bytes (segment l at tile + l*L) and streams
// them by LDS-DMA in rounds: round r fetches bytes [r*RUN, (r+1)*RUN) of every segment
// (64*RUN bytes per round, contiguous RUN-byte runs), S-deep slot pipeline, W waves/CU.
// Each lane then reads its segment's run back (ds_read_b128) and folds it into a checksum.
// Reports GB/s per configuration, and a plain coalesced streaming read for the peak.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/membench.hip -o build/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// layout 0: tile t at t*64L (linear).  layout 1: 4096 "streams" of 4 MiB, tile t is tile
// t/4096 of stream t%4096 (concurrent tiles share their offset mod 4 MiB, as in the batch
// splitter).  layout 2: as 1 with the tile index skewed by the stream id.
template <int RUN, int S, int W, int AUX, int D = 0>
__global__ __launch_bounds__(W * 64) void seg_kernel(const uint8_t* base, int64_t L, uint32_t ntiles,
                                                     uint32_t* counter, uint32_t* out, int layout) {
    constexpr int kSlot = 64 * RUN;       // bytes per round
    constexpr int kIns = kSlot / 1024;    // DMA instructions per round
    constexpr int kLanesPerSeg = RUN / 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t* sl = smem + static_cast<size_t>(wave) * S * kSlot;
    uint32_t acc = 0;
    const int rounds = static_cast<int>(L / RUN);
    for (;;) {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(counter, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0));
        if (t >= ntiles) break;
        int64_t tb = static_cast<int64_t>(t) * 64 * L;
        if (layout) {
            const int64_t tiles_per_stream = (int64_t(4) << 20) / (64 * L);
            const int64_t sidx = t % 4096, k = t / 4096;
            const int64_t kk = layout == 2 ? (k + sidx) % tiles_per_stream : k;
            tb = sidx * (int64_t(4) << 20) + kk * 64 * L;
        }
        int64_t nrec = 64 * L;
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(base + tb), static_cast<short>(0), static_cast<int>(nrec), 0x00020000);
        auto issue = [&](int r, uint8_t* slot) {
#pragma unroll
            for (int i = 0; i < kIns; i++) {
                const int f = i * 64 + lane;
                const int seg = f / kLanesPerSeg;
                const int within = (f % kLanesPerSeg) * 16;
                const int off = static_cast<int>(seg * L + static_cast<int64_t>(r) * RUN + within);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_ptr_t)(slot + 1024 * i), 16, off, 0, 0, AUX);
            }
        };
#pragma unroll
        for (int j = 0; j < S; j++)
            if (j < rounds) issue(j, sl + kSlot * j);
        int qs = 0;
        for (int r = 0; r < rounds; r++) {
            uint8_t* slot = sl + kSlot * qs;
            if (r + S - 1 < rounds)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kIns * (S - 1) > 63 ? 63 : kIns * (S - 1)) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int k = 0; k < kLanesPerSeg; k++) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(slot + lane * RUN + 16 * k);
                acc += v.x ^ v.y ^ v.z ^ v.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (r + S < rounds) issue(r + S, slot);
            // emulated hashing: D dependent VALU ops (rotate + xor chains, 2 per iteration)
#pragma unroll 16
            for (int k = 0; k < D; k++) {
                acc = __builtin_amdgcn_alignbit(acc, acc, 31) ^ (acc + k);
            }
            qs = qs + 1 == S ? 0 : qs + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (acc == 0x12345678u) out[threadIdx.x] = acc;  // keep the loads alive
}

// Peak reference: every thread streams 16 B per iteration, grid-stride, fully coalesced.
__global__ __launch_bounds__(256) void stream_kernel(const u32x4* p, int64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

struct Cfg {
    const char* name;
    void (*fn)(const uint8_t*, int64_t, uint32_t, uint32_t*, uint32_t*, int);
    int run, s, w;
};

#define CFG(RUN, S, W, AUX) \
    Cfg{"run" #RUN "_s" #S "_w" #W "_aux" #AUX, seg_kernel<RUN, S, W, AUX>, RUN, S, W}
#define CFGD(RUN, S, W, AUX, D) \
    Cfg{"run" #RUN "_s" #S "_w" #W "_aux" #AUX "_d" #D, seg_kernel<RUN, S, W, AUX, D>, RUN, S, W}

int main(int argc, char** argv) {
    const bool calib = argc > 1 && std::string(argv[1]) == "calib";  // one config, 4 launches (FETCH_SIZE calibration)
    const int64_t L = 2048;
    const int64_t total = int64_t(16) << 30;
    const uint32_t ntiles = static_cast<uint32_t>(total / (64 * L));
    uint8_t* buf;
    uint32_t *counter, *out;
    CK(hipMalloc(&buf, total));
    CK(hipMalloc(&counter, 4));
    CK(hipMalloc(&out, 4096));
    CK(hipMemset(buf, 0x5a, total));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::vector<Cfg> cfgs = {
        CFG(64, 2, 8, 0), CFG(64, 4, 8, 0), CFG(128, 2, 8, 0), CFG(128, 2, 8, 2), CFG(128, 4, 4, 0), CFG(256, 2, 4, 0),
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (calib) cfgs = {CFG(128, 2, 8, 2)};
    const bool depth = argc > 1 && std::string(argv[1]) == "depth";  // pipeline depth vs emulated compute
    if (depth)
        cfgs = {CFGD(128, 1, 8, 2, 0),   CFGD(128, 2, 8, 2, 0),   CFGD(128, 1, 8, 2, 200), CFGD(128, 2, 8, 2, 200),
                CFGD(128, 1, 8, 2, 400), CFGD(128, 2, 8, 2, 400), CFGD(64, 3, 8, 0, 200),  CFGD(64, 3, 8, 0, 100),
                CFGD(128, 2, 6, 2, 200), CFGD(128, 2, 6, 2, 400), CFGD(64, 2, 8, 0, 100),  CFGD(64, 4, 8, 0, 100)};
    // occupancy: 128-B runs at 8 waves/CU vs 64-B runs at 12 (the LDS the splitter can afford),
    // emulated hashing ~4 VALU per byte
    const bool occ = argc > 1 && std::string(argv[1]) == "occ";
    if (occ)
        cfgs = {CFGD(128, 1, 8, 2, 250), CFGD(64, 1, 8, 2, 125), CFGD(64, 1, 12, 2, 125), CFGD(64, 1, 16, 2, 125),
                CFGD(128, 1, 12, 2, 250), CFGD(64, 2, 12, 2, 125), CFGD(128, 1, 8, 2, 300), CFGD(64, 1, 12, 2, 150)};
    // Rabin-Karp plan: 64-B runs (two chains per lane, 64 B each per step) vs 128-B runs,
    // 8 waves/CU, emulated hashing of ~10.5 VALU per byte (D = 2 ops per unit)
    const bool rk = argc > 1 && std::string(argv[1]) == "rk";
    if (rk)
        cfgs = {CFGD(128, 1, 8, 2, 672), CFGD(64, 2, 8, 2, 336), CFGD(64, 1, 8, 2, 336), CFGD(128, 1, 8, 2, 0),
                CFGD(64, 2, 8, 2, 0), CFGD(64, 2, 8, 0, 336), CFGD(128, 1, 8, 2, 336), CFGD(64, 2, 8, 2, 168)};
    for (int rep = 0; rep < (calib ? 1 : 2); rep++) {
      for (int layout = (depth || occ || rk ? 1 : 0); layout < (calib ? 1 : depth || occ || rk ? 2 : 3); layout++) {
        for (auto& c : cfgs) {
            const size_t lds = static_cast<size_t>(c.w) * c.s * 64 * c.run;
            if (lds > 160 * 1024) {
                if (rep == 0) printf("%-22s skipped (LDS %zu)\n", c.name, lds);
                continue;
            }
            CK(hipFuncSetAttribute(reinterpret_cast<const void*>(c.fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   static_cast<int>(lds)));
            float best = 1e9f;
            for (int it = 0; it < 4; it++) {
                CK(hipMemset(counter, 0, 4));
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(c.fn, dim3(cus), dim3(c.w * 64), lds, 0, buf, L, ntiles, counter, out, layout);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it > 0 && ms < best) best = ms;
            }
            printf("L%d %-22s lds %6zu  %.3f ms  %.0f GB/s\n", layout, c.name, lds, best, total / (best * 1e-3) / 1e9);
        }
      }
        float best = 1e9f;
        for (int it = 0; it < 4; it++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(stream_kernel, dim3(cus * 16), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(buf),
                               total / 16, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0 && ms < best) best = ms;
        }
        printf("%-22s             %.3f ms  %.0f GB/s\n", "coalesced_stream", best, total / (best * 1e-3) / 1e9);
        fflush(stdout);
    }
    return 0;
}
