// VALU issue rate of the splitters' integer instructions on gfx950: W waves per CU (W/4 per
// SIMD), each running 8 independent accumulator chains of one instruction kind; cycles from
// s_memtime inside the kernel (shader clock).  Prints shader cycles per wave64 instruction
// per SIMD: 4 = one instruction per 4 cycles per SIMD, 2 = two waves issue together.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/valu_rate.hip -o build/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int KIND>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b, uint32_t c) {
    if constexpr (KIND == 0) return __builtin_amdgcn_perm(a, b, c);
    if constexpr (KIND == 1) return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
    if constexpr (KIND == 2) return __builtin_amdgcn_alignbit(a, b, c & 31);
    if constexpr (KIND == 3) return a ^ b;
    if constexpr (KIND == 4) return __float_as_uint(__builtin_fmaf(__uint_as_float(a), __uint_as_float(b), __uint_as_float(c)));
    return 0;
}

template <int KIND>
__global__ void rate_kernel(uint32_t iters, uint32_t seed, uint32_t* out, uint64_t* cyc) {
    uint32_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = seed * (threadIdx.x + 3 * i + 1);
    const uint32_t b = seed ^ threadIdx.x, c = 0x05040100u ^ (seed & 0x03030303u);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++)
#pragma unroll
            for (int i = 0; i < 8; i++) acc[i] = op<KIND>(acc[i], b + r, c);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= acc[i];
    if (x == 0x12345678u) out[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int KIND>
int run(const char* name, int cus, uint32_t* out, uint64_t* cyc) {
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
        printf("%-10s waves/CU %2d: %.2f cycles per wave64 instruction per SIMD\n", name, w, mx / insts_per_simd);
    }
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    uint32_t* out;
    uint64_t* cyc;
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&cyc, 256 * 16 * 8));
    const int cus = p.multiProcessorCount;
    run<0>("v_perm", cus, out, cyc);
    run<1>("v_bitop3", cus, out, cyc);
    run<2>("v_alignbit", cus, out, cyc);
    run<3>("v_xor", cus, out, cyc);
    run<4>("v_fma_f32", cus, out, cyc);
    return 0;
}
