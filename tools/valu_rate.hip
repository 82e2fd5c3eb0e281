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
    X(13, "v_lshrrev_b32 %0, 8, %0")

static const char* kNames[] = {"v_xor_b32",  "v_and_b32",   "v_add_u32",  "v_lshlrev_b32", "v_lshl_or_b32",
                               "v_min3_u32", "v_perm_b32",  "v_bitop3_b32", "v_alignbit_b32", "v_bfe_u32",
                               "v_lshl_add_u32", "v_mov_b32",   "v_fma_f32",  "v_lshrrev_b32"};

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

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    uint32_t* out;
    uint64_t* cyc;
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&cyc, 256 * 16 * 8));
    return run_all(p.multiProcessorCount, out, cyc, std::make_integer_sequence<int, 14>{});
}
