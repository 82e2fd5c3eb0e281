// Rabin-Karp hot-loop variants in isolation (round 6): what bounds split_batch_rk_kernel's
// per-byte chain, measured rather than argued.  Each variant is a replica of rk_step64
// (kcdc_kernels.hip) fed from an LDS step slot, no DMA, queue, warm-up or tile overhead, over
// config 2's rolled bytes (6.7429e9 B under 4M-RABINKARP), one workgroup per CU.
//
//   NCH     chains per lane (2: production; 4: the lane segment in quarters)
//   MODREP  mod[] replicas (16: 128-byte rows, 2-way conflicts; 32: 256-byte rows, conflict-free)
//   OUTREP  out[] replicas (32: 256-byte rows, address = one v_perm; 16: 128-byte rows)
//   WAVES   waves per CU (8 = 2 per SIMD as in production; 12, 16 for the latency ablation)
//   FL      flags: kNoOut (no out[] read: the leaving byte's term is a register),
//                  kIndep (the mod[] read's address comes from the data, not the chain, and is
//                          issued two bytes ahead: the throughput floor of the same instruction mix),
//                  kBitop (mod[] address as lshrrev + one v_bitop3 instead of the compiler's pick)
//                  kSdwa  (out[] address: one SDWA v_mov of the leaving byte into byte 1 of a register
//                          that keeps lane%32*8 in byte 0, instead of a v_perm)
//                  kB64   (the shift as one v_lshrrev_b64 and the entering byte XORed into byte 3 of hi
//                          by one SDWA v_xor after the xor3s, instead of v_perm + v_alignbit)
//                  kRegData (no step slot: the bytes come from registers, one v_add per dword, so the
//                          tables may take all of LDS -- the layout a feed by global loads would allow)
//
// Bytes per variant are the same, so the times compare directly.  The output only defeats DCE.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/rk_loop.hip -o build/rk_loop
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kNoOut = 1, kIndep = 2, kBitop = 4, kSdwa = 8, kB64 = 16, kRegData = 32;

template <int MODREP, int OUTREP, int NSLOT>
struct Lds {
    uint64_t mod[256 * MODREP];
    uint64_t out[256 * OUTREP];
    uint32_t slot[NSLOT][32][64];
};

template <int NCH, int MODREP, int OUTREP, int WAVES, int FL>
struct V {
    static constexpr int kTab = 256 * 8 * (MODREP + OUTREP);
    static constexpr int kFree = (160 * 1024 - kTab) / 8192;
    static constexpr int kSlots = (FL & kRegData) ? 1 : kFree < WAVES ? kFree : WAVES;
    static_assert((FL & kRegData) || kSlots >= 1, "no room for a step slot");
    using L = Lds<MODREP, OUTREP, (FL & kRegData) ? 0 : kSlots>;
};

__device__ __forceinline__ uint64_t ld64(const char* base, uint32_t a) { return *reinterpret_cast<const uint64_t*>(base + a); }

template <int NCH, int MODREP, int OUTREP, int WAVES, int FL>
__global__ __launch_bounds__(WAVES * 64, 1) void rk_loop_kernel(uint64_t steps, uint32_t seed, uint32_t* out) {
    using Vv = V<NCH, MODREP, OUTREP, WAVES, FL>;
    __shared__ typename Vv::L t;
    for (uint32_t i = threadIdx.x; i < 256u * MODREP; i += blockDim.x) t.mod[i] = (i * 0x9E3779B97F4A7C15ull) ^ seed;
    for (uint32_t i = threadIdx.x; i < 256u * OUTREP; i += blockDim.x) t.out[i] = (i * 0xC2B2AE3D27D4EB4Full) ^ seed;
    const uint32_t wv = threadIdx.x / 64u, lane = threadIdx.x % 64u;
    const uint32_t sv = wv % Vv::kSlots;
    if constexpr ((FL & kRegData) == 0)
        if (wv < Vv::kSlots)
            for (uint32_t i = 0; i < 32u; i++) t.slot[sv][i][lane] = (lane + 1u) * 0x01000193u * (i + seed);
    __syncthreads();
    const char* modb = reinterpret_cast<const char*>(t.mod);
    const char* outb = reinterpret_cast<const char*>(t.out);
    const uint32_t l8o = (lane % OUTREP) * 8u, l8m = (lane % MODREP) * 8u;
    auto maddr = [&](uint32_t lo) -> uint32_t {
        constexpr int sh = MODREP == 16 ? 7 : 8;  // row stride 128 or 256
        if constexpr ((FL & kBitop) != 0) {
            constexpr uint32_t m = 0xFFu << sh;
            return __builtin_amdgcn_bitop3_b32(lo >> (11 - sh), m, l8m, 0xEA);  // (a & m) | l8m
        } else {
            return (__builtin_amdgcn_ubfe(lo, 11, 8) << sh) | l8m;
        }
    };
    auto oaddr = [&](uint32_t w, int b) -> uint32_t {
        const int pos = 3 - b;  // byte position of the (bit-reversed) leaving byte
        if constexpr (OUTREP == 32) {
            return __builtin_amdgcn_perm(w, l8o, 0x0c0c0000u | ((4u + pos) << 8));
        } else {  // 128-byte rows: the byte to bits 7..14
            const uint32_t s = pos == 0 ? (w << 7) : (w >> (8 * pos - 7));
            return __builtin_amdgcn_bitop3_b32(s, 0x7F80u, l8o, 0xEA);
        }
    };
    auto oaddr_sdwa = [&](uint32_t& a, uint32_t w, int b) {
        const int pos = 3 - b;
        if (pos == 0) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(a) : "v"(w));
        else if (pos == 1) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(a) : "v"(w));
        else if (pos == 2) asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a) : "v"(w));
        else asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(a) : "v"(w));
        return a;
    };
    auto xin = [](uint32_t& h, uint32_t w, int b) {  // byte 3 of h ^= the entering byte (byte 3 - b of w)
        const int pos = 3 - b;
        if (pos == 0) asm("v_xor_b32_sdwa %0, %1, %0 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_3" : "+v"(h) : "v"(w));
        else if (pos == 1) asm("v_xor_b32_sdwa %0, %1, %0 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_3" : "+v"(h) : "v"(w));
        else if (pos == 2) asm("v_xor_b32_sdwa %0, %1, %0 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 src1_sel:BYTE_3" : "+v"(h) : "v"(w));
        else asm("v_xor_b32_sdwa %0, %1, %0 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3 src1_sel:BYTE_3" : "+v"(h) : "v"(w));
    };
    uint32_t oad[NCH][2];
#pragma unroll
    for (int c = 0; c < NCH; c++) oad[c][0] = oad[c][1] = l8o;
    auto sel = [](int b) { return 0x00030201u | (static_cast<uint32_t>(7 - b) << 24); };
    uint32_t h[NCH], l[NCH], m[NCH], ph[NCH], p[NCH][16];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        h[c] = seed * (2 * c + 1);
        l[c] = seed * (2 * c + 3);
        m[c] = ~0u;
#pragma unroll
        for (int i = 0; i < 16; i++) p[c][i] = seed * (i + 1 + c);
    }
    for (uint64_t s = 0; s < steps; s++) {
        uint32_t d[NCH][16];
#pragma unroll
        for (int c = 0; c < NCH; c++)
#pragma unroll
            for (int i = 0; i < 16; i++) {
                uint32_t v;
                if constexpr ((FL & kRegData) != 0) v = static_cast<uint32_t>(s) * 0x9E3779B9u + (lane * 16u + i) * 0x01000193u + c;
                else v = t.slot[sv][(16 * c + i) & 31][lane];
                d[c][i] = c < 2 ? __builtin_bitreverse32(v) : __builtin_bitreverse32(v ^ 0x5A5A5A5Au);
            }
        constexpr int W = 2;
        uint64_t o[NCH][64], mr[NCH];
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if constexpr ((FL & kIndep) != 0) {
                mr[c] = ld64(modb, maddr(d[c][0] << 11));
            } else {
                mr[c] = ld64(modb, maddr(l[c]));
            }
#pragma unroll
            for (int i = 0; i < W; i++)
                if constexpr ((FL & kNoOut) == 0) {
                    if constexpr ((FL & kSdwa) != 0) o[c][i] = ld64(outb, oaddr_sdwa(oad[c][i & 1], p[c][i >> 2], i & 3));
                    else o[c][i] = ld64(outb, oaddr(p[c][i >> 2], i & 3));
                }
            ph[c] = ~0u;
        }
        uint64_t mn[NCH];  // kIndep: the next byte's read, issued a byte ahead
#pragma unroll
        for (int x = 0; x < 64; x++) {
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                __builtin_amdgcn_sched_barrier(0);
                uint64_t ox;
                if constexpr ((FL & kNoOut) != 0) ox = (static_cast<uint64_t>(p[c][x >> 2]) << 32) | d[c][x >> 2];
                else ox = o[c][x];
                if constexpr ((FL & kIndep) != 0)
                    if (x + 1 < 64) mn[c] = ld64(modb, maddr(d[c][(x + 1) >> 2] >> (4 * ((x + 1) & 3))));
                if constexpr ((FL & kB64) != 0) {
                    const uint64_t v0 = (static_cast<uint64_t>(h[c]) << 32) | l[c];
                    uint64_t v;
                    asm("v_lshrrev_b64 %0, 8, %1" : "=v"(v) : "v"(v0));
                    h[c] = __builtin_amdgcn_bitop3_b32(static_cast<uint32_t>(v >> 32), static_cast<uint32_t>(mr[c] >> 32), static_cast<uint32_t>(ox >> 32), 0x96);
                    l[c] = __builtin_amdgcn_bitop3_b32(static_cast<uint32_t>(v), static_cast<uint32_t>(mr[c]), static_cast<uint32_t>(ox), 0x96);
                    xin(h[c], d[c][x >> 2], x & 3);
                } else {
                    const uint32_t th = __builtin_amdgcn_perm(d[c][x >> 2], h[c], sel(x & 3));
                    const uint32_t tl = __builtin_amdgcn_alignbit(h[c], l[c], 8);
                    h[c] = __builtin_amdgcn_bitop3_b32(th, static_cast<uint32_t>(mr[c] >> 32), static_cast<uint32_t>(ox >> 32), 0x96);
                    l[c] = __builtin_amdgcn_bitop3_b32(tl, static_cast<uint32_t>(mr[c]), static_cast<uint32_t>(ox), 0x96);
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr ((FL & kIndep) != 0) {
                    if (x + 1 < 64) mr[c] = mn[c];
                } else {
                    if (x + 1 < 64) mr[c] = ld64(modb, maddr(l[c]));
                }
                if constexpr ((FL & kNoOut) == 0)
                    if (x + W < 64) {
                        if constexpr ((FL & kSdwa) != 0) o[c][x + W] = ld64(outb, oaddr_sdwa(oad[c][(x + W) & 1], p[c][(x + W) >> 2], (x + W) & 3));
                        else o[c][x + W] = ld64(outb, oaddr(p[c][(x + W) >> 2], (x + W) & 3));
                    }
                __builtin_amdgcn_sched_barrier(0);
                if (x & 1) asm("v_min3_u32 %0, %1, %2, %3" : "=v"(m[c]) : "v"(m[c]), "v"(ph[c]), "v"(h[c]));
                else ph[c] = h[c];
            }
        }
#pragma unroll
        for (int c = 0; c < NCH; c++)
#pragma unroll
            for (int i = 0; i < 16; i++) p[c][i] = d[c][i];
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) x ^= m[c] ^ h[c] ^ l[c];
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

template <int NCH, int MODREP, int OUTREP, int WAVES, int FL>
int run(const char* name, int cus, uint32_t* out, int reps) {
    const double bytes = 6.7429e9;  // config 2's rolled bytes under 4M-RABINKARP
    const uint64_t steps = static_cast<uint64_t>(bytes / (double(cus) * WAVES * 64) / (NCH * 64.0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9f, last = 0;
    for (int rep = 0; rep < reps; rep++) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((rk_loop_kernel<NCH, MODREP, OUTREP, WAVES, FL>), dim3(cus), dim3(WAVES * 64), 0, 0, steps, 7u + rep, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        last = ms;
    }
    printf("%-34s chains/lane %d mod rep %2d out rep %2d waves/CU %2d flags %d: best %.3f ms last %.3f ms (%llu steps/lane)\n",
           name, NCH, MODREP, OUTREP, WAVES, FL, best, last, static_cast<unsigned long long>(steps));
    fflush(stdout);
    return 0;
}

int main(int argc, char** argv) {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    uint32_t* out;
    CK(hipMalloc(&out, 4096 * 4));
    const int reps = argc > 1 ? std::stoi(argv[1]) : 12;
    // warm the clock on the production replica first
    run<2, 16, 32, 8, 0>("warm (production replica)", cus, out, reps);
    run<2, 16, 32, 8, 0>("production replica", cus, out, reps);
    run<2, 16, 32, 8, kBitop>("mod addr lshrrev+bitop3", cus, out, reps);
    run<2, 32, 16, 8, 0>("mod conflict-free, out 128-B rows", cus, out, reps);
    run<2, 16, 32, 8, kNoOut>("no out[] read", cus, out, reps);
    run<2, 16, 32, 8, kIndep>("mod read off the chain", cus, out, reps);
    run<2, 16, 16, 12, 0>("12 waves/CU", cus, out, reps);
    run<2, 16, 16, 16, 0>("16 waves/CU (ablation)", cus, out, reps);
    run<4, 16, 32, 8, 0>("4 chains/lane", cus, out, reps);
    run<4, 32, 16, 8, 0>("4 chains/lane, mod conflict-free", cus, out, reps);
    run<2, 16, 32, 8, kBitop | kSdwa>("bitop3 mod addr + sdwa out addr", cus, out, reps);
    run<2, 16, 32, 8, kBitop | kSdwa | kRegData>("... data from registers", cus, out, reps);
    run<2, 32, 32, 8, kBitop | kSdwa | kRegData>("... + mod conflict-free (128 KiB tables)", cus, out, reps);
    run<2, 32, 32, 12, kBitop | kSdwa | kRegData>("... + 12 waves/CU", cus, out, reps);
    run<2, 16, 32, 8, kBitop | kB64>("bitop3 mod addr + b64 shift", cus, out, reps);
    run<2, 16, 32, 8, kBitop | kNoOut>("bitop3 mod addr, no out[]", cus, out, reps);
    run<2, 16, 32, 8, 0>("production replica (again)", cus, out, reps);
    return 0;
}
