// alubench.hip -- diagnostic: issue throughput of the integer multiplies Philox
// needs (v_mul_lo_u32 / v_mul_hi_u32 vs v_mad_u64_u32) and a few reference ops.
// Build: hipcc --offload-arch=gfx950 -O3 -o build_abl/alubench tools/alubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
    unsigned a0 = threadIdx.x * 2654435761u + seed, a1 = a0 ^ 0x1234567u, a2 = a0 + 77u, a3 = a0 * 3u;
    const unsigned m = 0xD2511F53u;
    float f0 = (float)a0 * 1e-9f, f1 = f0 + 1.f, f2 = f0 + 2.f, f3 = f0 + 3.f;
    for (int i = 0; i < ITERS; i++) {
        if (OP == 0) {         // mul_hi + mul_lo, 4 independent chains
            a0 = __umulhi(a0, m) ^ (a0 * m); a1 = __umulhi(a1, m) ^ (a1 * m);
            a2 = __umulhi(a2, m) ^ (a2 * m); a3 = __umulhi(a3, m) ^ (a3 * m);
        } else if (OP == 1) {  // 64-bit product (v_mad_u64_u32)
            unsigned long long p0 = (unsigned long long)a0 * m, p1 = (unsigned long long)a1 * m;
            unsigned long long p2 = (unsigned long long)a2 * m, p3 = (unsigned long long)a3 * m;
            a0 = (unsigned)(p0 >> 32) ^ (unsigned)p0; a1 = (unsigned)(p1 >> 32) ^ (unsigned)p1;
            a2 = (unsigned)(p2 >> 32) ^ (unsigned)p2; a3 = (unsigned)(p3 >> 32) ^ (unsigned)p3;
        } else if (OP == 2) {  // xor/add only
            a0 = (a0 ^ m) + 0x9E3779B9u; a1 = (a1 ^ m) + 0x9E3779B9u; a2 = (a2 ^ m) + 0x9E3779B9u; a3 = (a3 ^ m) + 0x9E3779B9u;
        } else if (OP == 3) {  // v_exp_f32
            f0 = __builtin_amdgcn_exp2f(f0) * 0.5f; f1 = __builtin_amdgcn_exp2f(f1) * 0.5f;
            f2 = __builtin_amdgcn_exp2f(f2) * 0.5f; f3 = __builtin_amdgcn_exp2f(f3) * 0.5f;
        } else if (OP == 4) {  // mul_lo only
            a0 = a0 * m + 1u; a1 = a1 * m + 1u; a2 = a2 * m + 1u; a3 = a3 * m + 1u;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ __float_as_uint(f0 + f1 + f2 + f3);
}

template <int OP>
int run(const char* name, unsigned* d) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int blocks = 256 * 8;   // 8 waves per SIMD
    k<OP><<<blocks, 256>>>(d, 1);
    CK(hipEventRecord(a));
    k<OP><<<blocks, 256>>>(d, 2);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    // wave-instructions per SIMD: blocks*4 waves / 1024 SIMDs * ITERS * 4 ops-units
    const double waves_per_simd = blocks * 4.0 / 1024.0;
    printf("%-22s %8.3f ms  %.2f ns per (wave, iteration of 4 chains) per SIMD\n", name, ms,
           ms * 1e6 / (waves_per_simd * ITERS));
    return 0;
}

int main() {
    unsigned* d; CK(hipMalloc(&d, 256 * 8 * 256 * 4));
    run<2>("xor+add", d); run<4>("mul_lo+add", d); run<0>("mul_hi^mul_lo", d);
    run<1>("u64 product", d); run<3>("exp2*0.5", d);
    return 0;
}
