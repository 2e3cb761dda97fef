// fetchbench.hip -- calibration of rocprofv3's FETCH_SIZE for the learners' access shapes
// (MI355X_MICROARCH.md: FETCH_SIZE reads exactly half the bytes of a wide coalesced stream
// on gfx950; other widths are uncalibrated).  Each kernel reads a known number of bytes from
// a 2 GiB table (8x the Infinity Cache), every line once, in one of the shapes the C4 / C5
// table passes use; run under `rocprofv3 --pmc FETCH_SIZE` and divide.
//   stream16   : 16 B per lane, consecutive (the calibrated case)
//   rand64x4   : one random 64-B line per 4 lanes (16 B each): a dense H record
//   rand128x8  : one random 128-B line per 8 lanes
//   rand16     : 16 B at the start of a random 64-B line per lane: a V record
//   rand8      : 8 B at the start of a random 64-B line per lane: a V value / H increment
// Random line orders are a bijection of the line index (odd multiplier mod 2^k), so no
// index array is streamed and no line is read twice.
// Build: hipcc --offload-arch=gfx950 -O3 -o ab/fetchbench tools/fetchbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr unsigned long long kTable = 2ull << 30;       // bytes
constexpr unsigned kMul = 0x9E3779B1u;                    // odd: i -> i * kMul mod 2^k is a bijection

__device__ __forceinline__ unsigned long long perm(unsigned long long i, unsigned long long mask) {
    return (i * kMul + 0x5bd1e995ull) & mask;
}

__global__ __launch_bounds__(256) void stream16(const float4* t, unsigned long long n16, float* out) {
    float acc = 0.f;
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
        const float4 v = t[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

// L bytes per line, G lanes per line (16 B each)
template <int L, int G>
__global__ __launch_bounds__(256) void rand_lines(const float4* t, unsigned long long lines, float* out) {
    float acc = 0.f;
    const unsigned long long mask = lines - 1;
    const unsigned long long nthr = gridDim.x * 256ull;
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < lines * G; i += nthr) {
        const unsigned long long ln = perm(i / G, mask);
        const float4 v = t[ln * (L / 16) + (i % G)];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

// W bytes at the start of a random 64-B line, one line per lane
template <int W>
__global__ __launch_bounds__(256) void rand_head(const char* t, unsigned long long lines, float* out) {
    float acc = 0.f;
    const unsigned long long mask = lines - 1;
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < lines; i += gridDim.x * 256ull) {
        const char* p = t + perm(i, mask) * 64;
        if (W == 16) {
            const float4 v = *reinterpret_cast<const float4*>(p);
            acc += v.x + v.y + v.z + v.w;
        } else {
            const float2 v = *reinterpret_cast<const float2*>(p);
            acc += v.x + v.y;
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main() {
    char* t = nullptr;
    float* out = nullptr;
    CK(hipMalloc(&t, kTable));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(t, 1, kTable));
    CK(hipDeviceSynchronize());
    const unsigned long long l64 = kTable / 64, l128 = kTable / 128;
    const int blocks = 8192;
    // known bytes each kernel reads (the first launch of each is a warmup, the second measured)
    for (int rep = 0; rep < 2; rep++) {
        stream16<<<blocks, 256>>>(reinterpret_cast<const float4*>(t), kTable / 16, out);
        rand_lines<64, 4><<<blocks, 256>>>(reinterpret_cast<const float4*>(t), l64, out);
        rand_lines<128, 8><<<blocks, 256>>>(reinterpret_cast<const float4*>(t), l128, out);
        rand_head<16><<<blocks, 256>>>(t, l64 / 4, out);      // a quarter of the lines: 16 B of each
        rand_head<8><<<blocks, 256>>>(t, l64 / 4, out);
    }
    CK(hipDeviceSynchronize());
    printf("{\"table_bytes\": %llu, \"known_bytes\": {\"stream16\": %llu, \"rand_lines<64, 4>\": %llu, "
           "\"rand_lines<128, 8>\": %llu, \"rand_head<16>\": %llu, \"rand_head<8>\": %llu}, "
           "\"lines_touched\": {\"rand_head<16>\": %llu, \"rand_head<8>\": %llu}}\n",
           kTable, kTable, kTable, kTable, (l64 / 4) * 16, (l64 / 4) * 8, l64 / 4, l64 / 4);
    CK(hipFree(t));
    CK(hipFree(out));
    return 0;
}
