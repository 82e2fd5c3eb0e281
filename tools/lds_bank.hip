// ds_read_b64 table reads at random rows, R replicas per row (lane l reads replica l % R at
// byte offset 8 * (l % R) of a row of 8R bytes): issue cost per wave-instruction for R = 8..64,
// independent reads (no chain), 8 waves per CU, 12 reads in flight per wave.  Round 6: why a
// conflict-free 32-replica mod[] table measured slower than the 16-replica one.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/lds_bank.hip -o build/lds_bank
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int R, int ROWS>
__global__ __launch_bounds__(512, 1) void bank_kernel(uint32_t iters, uint32_t seed, uint64_t* out, uint64_t* cyc) {
    __shared__ uint64_t t[ROWS * R];
    for (uint32_t i = threadIdx.x; i < ROWS * R; i += 512) t[i] = i * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t off = (lane % R) * 8u;
    const char* base = reinterpret_cast<const char*>(t);
    // 12 independent random row patterns (per lane); each iteration XORs the same scalar salt into
    // every row index, so the pattern's conflicts are preserved and the VALU cost is one v_xor per read
    uint32_t addr[12];
    uint32_t x = seed * (threadIdx.x + 1) | 1u;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        x = x * 1664525u + 1013904223u;
        addr[k] = ((x >> 16) & (ROWS - 1)) * (8u * R) + off;
    }
    uint64_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t it = 0; it < iters; it++) {
        const uint32_t salt = __builtin_amdgcn_readfirstlane((it * 2654435761u >> 8) & (ROWS - 1)) * (8u * R);
        uint64_t v[12];
#pragma unroll
        for (int k = 0; k < 12; k++) v[k] = *reinterpret_cast<const uint64_t*>(base + (addr[k] ^ salt));
#pragma unroll
        for (int k = 0; k < 12; k++) acc ^= v[k];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (acc == 0x1234) out[threadIdx.x] = acc;
    if (lane == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
}

template <int R, int ROWS>
int run(int cus, uint64_t* out, uint64_t* cyc) {
    const uint32_t iters = 4000;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL((bank_kernel<R, ROWS>), dim3(cus), dim3(512), 0, 0, iters, 7u + rep, out, cyc);
        CK(hipDeviceSynchronize());
    }
    static uint64_t h[256 * 8];
    CK(hipMemcpy(h, cyc, sizeof(uint64_t) * cus * 8, hipMemcpyDeviceToHost));
    double mx = 0;
    for (int i = 0; i < cus * 8; i++) mx = h[i] > mx ? h[i] : mx;
    // per CU: 8 waves x iters x 12 reads
    printf("replicas %2d rows %3d (%3d KiB): %.2f cycles per ds_read_b64 wave-instruction per CU\n", R, ROWS,
           ROWS * R * 8 / 1024, mx / (8.0 * iters * 12));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    uint64_t *out, *cyc;
    CK(hipMalloc(&out, 512 * 8));
    CK(hipMalloc(&cyc, 256 * 8 * 8));
    run<8, 256>(p.multiProcessorCount, out, cyc);
    run<16, 256>(p.multiProcessorCount, out, cyc);
    run<32, 256>(p.multiProcessorCount, out, cyc);
    run<64, 256>(p.multiProcessorCount, out, cyc);
    run<32, 128>(p.multiProcessorCount, out, cyc);
    run<32, 64>(p.multiProcessorCount, out, cyc);
    run<16, 512>(p.multiProcessorCount, out, cyc);
    return 0;
}
