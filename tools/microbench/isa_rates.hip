// Issue rates of the integer / float instructions the walk kernel's Philox and
// geometry use, on one MI355X (gfx950): each thread runs 8 independent chains of
// one operation, the whole chip busy, and the time per wave-instruction per SIMD
// is reported. Build: hipcc --offload-arch=gfx950 -O3 isa_rates.hip -o isa_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int OP>
__global__ void __launch_bounds__(256) rate_kernel(unsigned* out, unsigned seed) {
    unsigned x[8];
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        x[c] = seed + threadIdx.x * 8 + c + blockIdx.x;
        f[c] = (float)x[c] * 1e-9f;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if (OP == 0) {          // v_mad_u64_u32: full 64-bit product
                const unsigned long long p = (unsigned long long)x[c] * 0xD2511F53u;
                x[c] = (unsigned)(p >> 32) ^ (unsigned)p;
            } else if (OP == 1) {   // v_mul_hi_u32 only
                x[c] = __umulhi(x[c], 0xD2511F53u) + x[c];
            } else if (OP == 2) {   // v_mul_lo_u32 only
                x[c] = x[c] * 0xD2511F53u + 1u;
            } else if (OP == 3) {   // v_fma_f32
                f[c] = fmaf(f[c], 1.0001f, 1e-7f);
            } else if (OP == 4) {   // v_exp_f32
                f[c] = __expf(f[c]) * 0.5f;
            } else if (OP == 5) {   // v_bitop3_b32
                x[c] = __builtin_amdgcn_bitop3_b32(x[c], x[(c + 1) & 7], 0x9E3779B9u, 0x96);
            }
        }
    }
    unsigned acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc ^= x[c] ^ __float_as_uint(f[c]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
float run(unsigned* d, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    rate_kernel<OP><<<grid, 256>>>(d, 1);   // warm-up
    hipEventRecord(a);
    rate_kernel<OP><<<grid, 256>>>(d, 2);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
    const int grid = cus * 8;   // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    unsigned* d = nullptr;
    hipMalloc(&d, sizeof(unsigned) * grid * 256);
    const char* names[] = {"v_mad_u64_u32 (+xor)", "v_mul_hi_u32 (+add)", "v_mul_lo_u32 (+add)", "v_fma_f32",
                           "v_exp_f32 (+mul)", "v_bitop3_b32"};
    float ms[6] = {run<0>(d, grid), run<1>(d, grid), run<2>(d, grid), run<3>(d, grid), run<4>(d, grid),
                   run<5>(d, grid)};
    const double waves_per_simd = (double)grid * 4 / (cus * 4);
    for (int k = 0; k < 6; ++k) {
        const double cycles = ms[k] * 1e-3 * clk * 1e3;
        const double per = cycles / (waves_per_simd * kIters * 8);
        std::printf("%-22s %8.3f ms  %6.2f SIMD cycles per wave-op (clock %d MHz)\n", names[k], ms[k], per, clk / 1000);
    }
    hipFree(d);
    return 0;
}
