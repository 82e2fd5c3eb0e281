// VALU issue rate of the splitters' integer instructions on gfx950 (round 4: every op class an
// inline-asm instruction, so the compiler can neither fold nor reassociate a chain -- round 3's
// plain-C v_xor row was folded and read 0.2 cycles).  W waves per CU (W/4 per SIMD), each running
// 16 independent accumulator chains of one instruction; cycles from s_memtime inside the kernel
// (shader clock).  Prints shader cycles per wave64 instruction per SIMD (4 = one instruction per
// 4 cycles per SIMD; 2 = two waves' instructions issue together), and the s_nop count the
// hazard recognizer put into the timed loop (must be 0 for a clean row).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/valu_rate.hip -o build/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <string>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

// One dependent step of chain `a` (b, c: loop-invariant operands).
#define OPS(X)                                                   \
    X(0, "v_xor_b32 %0, %0, %1")                                 \
    X(1, "v_and_b32 %0, %0, %1")                                 \
    X(2, "v_add_u32 %0, %0, %1")                                 \
    X(3, "v_lshlrev_b32 %0, 3, %0")                              \
    X(4, "v_lshl_or_b32 %0, %0, 8, %1")                          \
    X(5, "v_min3_u32 %0, %0, %1, %2")                            \
    X(6, "v_perm_b32 %0, %0, %1, %2")                            \
    X(7, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")              \
    X(8, "v_alignbit_b32 %0, %0, %1, 8")                         \
    X(9, "v_bfe_u32 %0, %0, 11, 8")                              \
    X(10, "v_lshl_add_u32 %0, %0, 2, %1")                        \
    X(11, "v_mov_b32 %0, %1")                                    \
    X(12, "v_fma_f32 %0, %0, %1, %2")                            \
    X(13, "v_lshrrev_b32 %0, 8, %0")                              \
    X(14, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2") \
    X(15, "v_xor_b32_sdwa %0, %1, %0 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_3") \
    X(16, "v_and_or_b32 %0, %0, %1, %2")                         \
    X(17, "v_min_u32 %0, %0, %1")                                \
    X(18, "v_or3_b32 %0, %0, %1, %2")                            \
    X(19, "v_xor_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD") \
    X(20, "v_bfrev_b32 %0, %0")                                  \
    X(21, "v_lshlrev_b32 %0, %1, %0")                            \
    X(22, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:BYTE_2") \
    X(23, "v_lshrrev_b32 %0, %1, %0")

static const char* kNames[] = {"v_xor_b32",  "v_and_b32",   "v_add_u32",  "v_lshlrev_b32", "v_lshl_or_b32",
                               "v_min3_u32", "v_perm_b32",  "v_bitop3_b32", "v_alignbit_b32", "v_bfe_u32",
                               "v_lshl_add_u32", "v_mov_b32",   "v_fma_f32",  "v_lshrrev_b32",
                               "v_mov_sdwa_pres", "v_xor_sdwa_pres", "v_and_or_b32", "v_min_u32", "v_or3_b32",
                               "v_xor_sdwa_src", "v_bfrev_b32", "v_lshlrev_reg", "v_mov_sdwa_pad", "v_lshrrev_reg"};

template <int KIND>
__device__ __forceinline__ void step(uint32_t& a, uint32_t b, uint32_t c) {
#define X(k, s) \
    if constexpr (KIND == k) asm volatile(s : "+v"(a) : "v"(b), "v"(c));
    OPS(X)
#undef X
}

template <int KIND>
__global__ void rate_kernel(uint32_t iters, uint32_t seed, uint32_t* out, uint64_t* cyc) {
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = seed * (threadIdx.x + 3 * i + 1);
    const uint32_t b = seed ^ threadIdx.x, c = 0x05040100u ^ (seed & 0x03030303u);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t it = 0; it < iters; it++) {
        asm volatile("; VALU_RATE_LOOP_BEGIN");
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int i = 0; i < 16; i++) step<KIND>(acc[i], b, c);
        asm volatile("; VALU_RATE_LOOP_END");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= acc[i];
    if (x == 0x12345678u) out[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int KIND>
int run(int cus, uint32_t* out, uint64_t* cyc) {
    for (int w : {4, 8, 12, 16}) {
        const uint32_t iters = 2000;
        hipLaunchKernelGGL(rate_kernel<KIND>, dim3(cus), dim3(64 * w), 0, 0, iters, 7u, out, cyc);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(rate_kernel<KIND>, dim3(cus), dim3(64 * w), 0, 0, iters, 7u, out, cyc);
        CK(hipDeviceSynchronize());
        static uint64_t h[256 * 16];
        CK(hipMemcpy(h, cyc, sizeof(uint64_t) * cus * w, hipMemcpyDeviceToHost));
        double mx = 0;
        for (int i = 0; i < cus * w; i++) mx = h[i] > mx ? h[i] : mx;
        const double insts_per_simd = double(iters) * 16 * 8 * (w / 4);
        printf("%-15s waves/CU %2d: %.2f cycles per wave64 instruction per SIMD\n", kNames[KIND], w, mx / insts_per_simd);
    }
    return 0;
}

template <int... K>
int run_all(int cus, uint32_t* out, uint64_t* cyc, std::integer_sequence<int, K...>) {
    int rc = 0;
    ((rc |= run<K>(cus, out, cyc)), ...);
    return rc;
}

// The Rabin-Karp batch kernel's hot loop in isolation (a replica of rk_step64 in
// kcdc_kernels.hip: two chains per lane interleaved byte by byte, 16 mod[] replicas and 32 out[]
// replicas in LDS, bit-reversed state, the running v_min3 test, outx[] reads two bytes ahead),
// fed from an LDS step slot (8 ds_read_b128 + 32 v_bfrev per 128 bytes, as the kernel's
// rk_read_step128) instead of the DMA ring, at the kernel's occupancy (one 512-thread workgroup
// per CU, 160 KiB LDS) over config 2's rolled bytes (4096 x 4 MiB).  Its wall time is the hot
// loop's floor on config 2 without HBM, queue, warm-up or tile overheads.
struct RkL {
    uint64_t mod[256 * 16];
    uint64_t out[256 * 32];
    uint32_t slot[8][32][64];  // per wave: 32 dwords per lane, lane-minor (conflict free)
};
__device__ __forceinline__ uint64_t ld64(const char* base, uint32_t a) { return *reinterpret_cast<const uint64_t*>(base + a); }
__global__ __launch_bounds__(512, 2) void rkloop_kernel(uint64_t steps, uint32_t seed, uint32_t* out) {
    __shared__ RkL t;
    for (uint32_t i = threadIdx.x; i < 256u * 16u; i += 512u) t.mod[i] = (i * 0x9E3779B97F4A7C15ull) ^ seed;
    for (uint32_t i = threadIdx.x; i < 256u * 32u; i += 512u) t.out[i] = (i * 0xC2B2AE3D27D4EB4Full) ^ seed;
    const uint32_t wv = threadIdx.x / 64u, lane = threadIdx.x % 64u;
    for (uint32_t i = 0; i < 32u; i++) t.slot[wv][i][lane] = (lane + 1u) * 0x01000193u * (i + seed);
    __syncthreads();
    const char* modb = reinterpret_cast<const char*>(t.mod);
    const char* outb = reinterpret_cast<const char*>(t.out);
    const uint32_t l8o = (lane & 31u) * 8u, l8m = (lane & 15u) * 8u;
    auto maddr = [&](uint32_t lo) { return (__builtin_amdgcn_ubfe(lo, 11, 8) << 7) | l8m; };
    auto oaddr = [&](uint32_t w, int b) { return __builtin_amdgcn_perm(w, l8o, 0x0c0c0000u | ((4u + (3 - b)) << 8)); };
    auto sel = [](int b) { return 0x00030201u | (static_cast<uint32_t>(7 - b) << 24); };
    uint32_t ha = seed, la = seed * 3u, hb = seed * 5u, lb = seed * 7u, ma = ~0u, mb = ~0u;
    uint32_t pa[16], pb[16];
#pragma unroll
    for (int i = 0; i < 16; i++) pa[i] = pb[i] = seed * (i + 1);
    for (uint64_t s = 0; s < steps; s++) {
        uint32_t a[16], b[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            a[i] = __builtin_bitreverse32(t.slot[wv][i][lane]);
            b[i] = __builtin_bitreverse32(t.slot[wv][16 + i][lane]);
        }
        constexpr int W = 2;
        uint64_t oa[64], ob[64];
        uint64_t mA = ld64(modb, maddr(la)), mB;
#pragma unroll
        for (int i = 0; i < W; i++) oa[i] = ld64(outb, oaddr(pa[i >> 2], i & 3));
        mB = ld64(modb, maddr(lb));
#pragma unroll
        for (int i = 0; i < W; i++) ob[i] = ld64(outb, oaddr(pb[i >> 2], i & 3));
        uint32_t pha = ~0u, phb = ~0u;
#pragma unroll
        for (int x = 0; x < 64; x++) {
            __builtin_amdgcn_sched_barrier(0);
            {
                const uint32_t th = __builtin_amdgcn_perm(a[x >> 2], ha, sel(x & 3));
                const uint32_t tl = __builtin_amdgcn_alignbit(ha, la, 8);
                ha = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mA >> 32), static_cast<uint32_t>(oa[x] >> 32), 0x96);
                la = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mA), static_cast<uint32_t>(oa[x]), 0x96);
                __builtin_amdgcn_sched_barrier(0);
                if (x + 1 < 64) mA = ld64(modb, maddr(la));
                if (x + W < 64) oa[x + W] = ld64(outb, oaddr(pa[(x + W) >> 2], (x + W) & 3));
                __builtin_amdgcn_sched_barrier(0);
                if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(ma) : "v"(ma), "v"(pha), "v"(ha));
                else pha = ha;
            }
            {
                const uint32_t th = __builtin_amdgcn_perm(b[x >> 2], hb, sel(x & 3));
                const uint32_t tl = __builtin_amdgcn_alignbit(hb, lb, 8);
                hb = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mB >> 32), static_cast<uint32_t>(ob[x] >> 32), 0x96);
                lb = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mB), static_cast<uint32_t>(ob[x]), 0x96);
                __builtin_amdgcn_sched_barrier(0);
                if (x + 1 < 64) mB = ld64(modb, maddr(lb));
                if (x + W < 64) ob[x + W] = ld64(outb, oaddr(pb[(x + W) >> 2], (x + W) & 3));
                __builtin_amdgcn_sched_barrier(0);
                if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(mb) : "v"(mb), "v"(phb), "v"(hb));
                else phb = hb;
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            pa[i] = a[i];
            pb[i] = b[i];
        }
    }
    if ((ma ^ mb ^ ha ^ la ^ hb ^ lb) == 0x12345678u) out[threadIdx.x] = ma;
}

// Round 5: the same hot loop at 12 waves per CU (three per SIMD: six chains per SIMD instead of
// four).  12 step slots of 8 KiB leave 64 KiB for the tables, so both go to 16 replicas in one
// table of 256-byte rows: mod[] in bytes 0..127 of row r (address: bfe + lshl_or, as now) and
// out[] in bytes 128..255 (address: one v_perm with 128 + lane%16 * 8 as its low byte).  Same
// instruction mix per byte; what changes is the chains in flight per SIMD (and out[]'s 16-replica
// bank conflicts).  "rk12": this variant; "rk": the production layout at 8 waves.
struct RkL12 {
    uint64_t tab[256 * 32];        // row r: mod replicas 0..15, then out replicas 0..15
    uint32_t slot[12][32][64];
};
__global__ __launch_bounds__(768, 1) void rkloop12_kernel(uint64_t steps, uint32_t seed, uint32_t* out) {
    __shared__ RkL12 t;
    for (uint32_t i = threadIdx.x; i < 256u * 32u; i += 768u) t.tab[i] = (i * 0x9E3779B97F4A7C15ull) ^ seed;
    const uint32_t wv = threadIdx.x / 64u, lane = threadIdx.x % 64u;
    for (uint32_t i = 0; i < 32u; i++) t.slot[wv][i][lane] = (lane + 1u) * 0x01000193u * (i + seed);
    __syncthreads();
    const char* tb = reinterpret_cast<const char*>(t.tab);
    const uint32_t l8o = 128u + (lane & 15u) * 8u, l8m = (lane & 15u) * 8u;
    auto maddr = [&](uint32_t lo) { return (__builtin_amdgcn_ubfe(lo, 11, 8) << 8) | l8m; };
    auto oaddr = [&](uint32_t w, int b) { return __builtin_amdgcn_perm(w, l8o, 0x0c0c0000u | ((4u + (3 - b)) << 8)); };
    auto sel = [](int b) { return 0x00030201u | (static_cast<uint32_t>(7 - b) << 24); };
    uint32_t ha = seed, la = seed * 3u, hb = seed * 5u, lb = seed * 7u, ma = ~0u, mb = ~0u;
    uint32_t pa[16], pb[16];
#pragma unroll
    for (int i = 0; i < 16; i++) pa[i] = pb[i] = seed * (i + 1);
    for (uint64_t s = 0; s < steps; s++) {
        uint32_t a[16], b[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            a[i] = __builtin_bitreverse32(t.slot[wv][i][lane]);
            b[i] = __builtin_bitreverse32(t.slot[wv][16 + i][lane]);
        }
        constexpr int W = 2;
        uint64_t oa[64], ob[64];
        uint64_t mA = ld64(tb, maddr(la)), mB;
#pragma unroll
        for (int i = 0; i < W; i++) oa[i] = ld64(tb, oaddr(pa[i >> 2], i & 3));
        mB = ld64(tb, maddr(lb));
#pragma unroll
        for (int i = 0; i < W; i++) ob[i] = ld64(tb, oaddr(pb[i >> 2], i & 3));
        uint32_t pha = ~0u, phb = ~0u;
#pragma unroll
        for (int x = 0; x < 64; x++) {
            __builtin_amdgcn_sched_barrier(0);
            {
                const uint32_t th = __builtin_amdgcn_perm(a[x >> 2], ha, sel(x & 3));
                const uint32_t tl = __builtin_amdgcn_alignbit(ha, la, 8);
                ha = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mA >> 32), static_cast<uint32_t>(oa[x] >> 32), 0x96);
                la = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mA), static_cast<uint32_t>(oa[x]), 0x96);
                __builtin_amdgcn_sched_barrier(0);
                if (x + 1 < 64) mA = ld64(tb, maddr(la));
                if (x + W < 64) oa[x + W] = ld64(tb, oaddr(pa[(x + W) >> 2], (x + W) & 3));
                __builtin_amdgcn_sched_barrier(0);
                if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(ma) : "v"(ma), "v"(pha), "v"(ha));
                else pha = ha;
            }
            {
                const uint32_t th = __builtin_amdgcn_perm(b[x >> 2], hb, sel(x & 3));
                const uint32_t tl = __builtin_amdgcn_alignbit(hb, lb, 8);
                hb = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mB >> 32), static_cast<uint32_t>(ob[x] >> 32), 0x96);
                lb = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mB), static_cast<uint32_t>(ob[x]), 0x96);
                __builtin_amdgcn_sched_barrier(0);
                if (x + 1 < 64) mB = ld64(tb, maddr(lb));
                if (x + W < 64) ob[x + W] = ld64(tb, oaddr(pb[(x + W) >> 2], (x + W) & 3));
                __builtin_amdgcn_sched_barrier(0);
                if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(mb) : "v"(mb), "v"(phb), "v"(hb));
                else phb = hb;
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) {
            pa[i] = a[i];
            pb[i] = b[i];
        }
    }
    if ((ma ^ mb ^ ha ^ la ^ hb ^ lb) == 0x12345678u) out[threadIdx.x] = ma;
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    uint32_t* out;
    uint64_t* cyc;
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&cyc, 256 * 16 * 8));
    if (argc > 1 && std::string(argv[1]) == "rk12") {
        const double bytes = 6.7429e9;
        const int cus = p.multiProcessorCount;
        const uint64_t steps = static_cast<uint64_t>(bytes / (cus * 768.0) / 128.0);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(rkloop12_kernel, dim3(cus), dim3(768), 0, 0, steps, 7u, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("rk hot loop, 12 waves/CU, 64 KiB combined tables: %.3f ms over config 2 (%llu 128-byte steps per lane)\n", ms,
                   static_cast<unsigned long long>(steps));
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "rk") {
        const double bytes = 6.7429e9;  // config 2's rolled bytes under 4M-RABINKARP
        const int cus = p.multiProcessorCount;
        const uint64_t steps = static_cast<uint64_t>(bytes / (cus * 512.0) / 128.0);  // 128 bytes per step per lane
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(rkloop_kernel, dim3(cus), dim3(512), 0, 0, steps, 7u, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("rk hot loop alone: %.3f ms over config 2 (%.0f bytes, %llu 128-byte steps per lane, %d CUs)\n", ms,
                   bytes, static_cast<unsigned long long>(steps), cus);
        }
        return 0;
    }
    return run_all(p.multiProcessorCount, out, cyc, std::make_integer_sequence<int, 24>{});
}
