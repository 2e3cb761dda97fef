// membench.hip -- diagnostic: HBM round trip of the batched env state with the
// access pattern of core_wave_kernel (persistent waves, one env pair per wave
// per iteration), to separate memory-system cost from kernel compute.
// Build: hipcc --offload-arch=gfx950 -O3 -o build_abl/membench tools/membench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int HW = 144, A = 32, EW = 2;

// mode bits: 1 = DFF, 2 = positions (full line), 4 = positions partial (half lanes),
// 8 = counts, 16 = one env per thread-group in block order instead of grid-stride
template <int MODE>
__global__ __launch_bounds__(256) void state_copy(float* dff, unsigned short* pos, int* cnt, long long E,
                                                  float scale) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long ngroups = E / EW;
    const long long ws = (long long)gridDim.x * 4;
    for (long long g = (long long)blockIdx.x * 4 + wv; g < ngroups; g += ws) {
        float4 d[2];
        float4* src = reinterpret_cast<float4*>(dff + g * EW * HW);
        unsigned short p = 0;
        int c = 0;
        if (MODE & 1) {
            d[0] = src[lane];
            if (lane < 8) d[1] = src[64 + lane];
        }
        if (MODE & 6) p = pos[g * EW * A + lane];
        if (MODE & 8) c = cnt[g * EW + (lane >> 5)];
        // a little dependent work
        if (MODE & 1) {
            d[0].x *= scale; d[0].y *= scale; d[0].z *= scale; d[0].w *= scale;
            if (lane < 8) { d[1].x *= scale; d[1].y *= scale; d[1].z *= scale; d[1].w *= scale; }
            src[lane] = d[0];
            if (lane < 8) src[64 + lane] = d[1];
        }
        if (MODE & 2) pos[g * EW * A + lane] = (unsigned short)(p + 1);
        if (MODE & 4) if ((lane & 31) < 16) pos[g * EW * A + lane] = (unsigned short)(p + 1);
        if (MODE & 8) if ((lane & 31) == 0) cnt[g * EW + (lane >> 5)] = c + 1;
    }
}

template <int MODE>
int run(float* dff, unsigned short* pos, int* cnt, long long E, int blocks, const char* name) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; i++) state_copy<MODE><<<blocks, 256>>>(dff, pos, cnt, E, 1.0f);
    CK(hipEventRecord(a));
    const int iters = 200;
    for (int i = 0; i < iters; i++) state_copy<MODE><<<blocks, 256>>>(dff, pos, cnt, E, 1.0f);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = (double)E * (((MODE & 1) ? 2 * HW * 4 : 0) + ((MODE & 6) ? 2 * A * 2 : 0) + ((MODE & 8) ? 8 : 0));
    printf("%-28s blocks=%5d  %8.2f us/launch  %7.1f GB/s\n", name, blocks, ms * 1e3 / iters, bytes / (ms / iters * 1e-3) / 1e9);
    return 0;
}

__global__ void fill_rand(float* p, long long n, unsigned seed) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) { unsigned h = (unsigned)i * 2654435761u ^ seed; h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15; p[i] = (float)(h & 0xFFFFFF) * 1e-6f; }
}
int probe();
int main() {
    {
        const long long E = 65536;
        float* d; unsigned short* ps; int* c;
        CK(hipMalloc(&d, E * HW * 4)); CK(hipMalloc(&ps, E * A * 2)); CK(hipMalloc(&c, E * 4));
        CK(hipMemset(d, 0, E * HW * 4));
        run<1>(d, ps, c, E, 1024, "zeros: dff only");
        fill_rand<<<(E * HW + 255) / 256, 256>>>(d, E * HW, 7);
        CK(hipDeviceSynchronize());
        run<1>(d, ps, c, E, 1024, "random: dff only");
    }
    if (probe()) return 1;
    const long long E = 65536;
    float* dff;
    unsigned short* pos;
    int* cnt;
    CK(hipMalloc(&dff, E * HW * 4));
    CK(hipMalloc(&pos, E * A * 2));
    CK(hipMalloc(&cnt, E * 4));
    CK(hipMemset(dff, 0, E * HW * 4));
    CK(hipMemset(pos, 0, E * A * 2));
    CK(hipMemset(cnt, 0, E * 4));
    for (int blocks : {1024, 2048, 8192}) {
        run<1>(dff, pos, cnt, E, blocks, "dff only");
        run<1 | 2>(dff, pos, cnt, E, blocks, "dff+pos(full)");
        run<1 | 4>(dff, pos, cnt, E, blocks, "dff+pos(partial)");
        run<1 | 2 | 8>(dff, pos, cnt, E, blocks, "dff+pos+cnt");
        run<1 | 4 | 8>(dff, pos, cnt, E, blocks, "dff+pos(partial)+cnt");
    }
    return 0;
}

// ---- latency probe: prefetch next group at the top, spin, stage at the bottom ----
// variant 1: state_copy + an LDS round trip of the data (no prefetch)
__global__ __launch_bounds__(256) void lds_roundtrip(float* dff, long long E) {
    __shared__ float4 stage[4][72];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long ngroups = E / EW;
    const long long ws = (long long)gridDim.x * 4;
    float4* base = reinterpret_cast<float4*>(dff);
    for (long long g = (long long)blockIdx.x * 4 + wv; g < ngroups; g += ws) {
        float4 a0 = base[g * 72 + lane];
        float4 a1 = lane < 8 ? base[g * 72 + 64 + lane] : make_float4(0, 0, 0, 0);
        stage[wv][lane] = a0;
        if (lane < 8) stage[wv][64 + lane] = a1;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        float4 c0 = stage[wv][63 - lane];
        float4 c1 = lane < 8 ? stage[wv][64 + 7 - lane] : make_float4(0, 0, 0, 0);
        base[g * 72 + lane] = c0;
        if (lane < 8) base[g * 72 + 64 + lane] = c1;
    }
}
// variant 2: register prefetch (loop-carried copy)
__global__ __launch_bounds__(256) void reg_prefetch(float* dff, long long E) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long ngroups = E / EW;
    const long long ws = (long long)gridDim.x * 4;
    float4* base = reinterpret_cast<float4*>(dff);
    long long g = (long long)blockIdx.x * 4 + wv;
    float4 c0 = make_float4(0, 0, 0, 0), c1 = c0;
    if (g < ngroups) { c0 = base[g * 72 + lane]; if (lane < 8) c1 = base[g * 72 + 64 + lane]; }
    for (; g < ngroups; g += ws) {
        float4 n0 = make_float4(0, 0, 0, 0), n1 = n0;
        if (g + ws < ngroups) { n0 = base[(g + ws) * 72 + lane]; if (lane < 8) n1 = base[(g + ws) * 72 + 64 + lane]; }
        base[g * 72 + lane] = c0;
        if (lane < 8) base[g * 72 + 64 + lane] = c1;
        c0 = n0; c1 = n1;
    }
}

template <bool STAMP>
__global__ __launch_bounds__(256) void pipelined(float* dff, long long E, int spin, unsigned long long* cyc, int nostore) {
    __shared__ float4 stage[4][72];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long ngroups = E / EW;
    const long long ws = (long long)gridDim.x * 4;
    long long g = (long long)blockIdx.x * 4 + wv;
    float4* base = reinterpret_cast<float4*>(dff);
    if (g < ngroups) {
        stage[wv][lane] = base[g * 72 + lane];
        if (lane < 8) stage[wv][64 + lane] = base[g * 72 + 64 + lane];
    }
    unsigned long long waitc = 0;
    for (; g < ngroups; g += ws) {
        float4 n0 = make_float4(0, 0, 0, 0), n1 = n0;
        const long long gn = g + ws;
        if (gn < ngroups) {
            n0 = base[gn * 72 + lane];
            if (lane < 8) n1 = base[gn * 72 + 64 + lane];
        }
        float4 c0 = stage[wv][lane];
        float4 c1 = lane < 8 ? stage[wv][64 + lane] : make_float4(0, 0, 0, 0);
        float x = c0.x;
        for (int i = 0; i < spin; i++) x = x * 0.999f + 1e-7f;   // dependent ALU chain
        c0.x = x;
        const unsigned long long t0 = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        stage[wv][lane] = n0;               // waits for the prefetch
        if (lane < 8) stage[wv][64 + lane] = n1;
        const unsigned long long t1 = STAMP ? __builtin_amdgcn_s_memtime() : 0;
        waitc += t1 - t0;
        if (!nostore) {
            base[g * 72 + lane] = c0;
            if (lane < 8) base[g * 72 + 64 + lane] = c1;
        } else if (c0.x == 12345.f) {
            base[0] = c0;   // keep the data live
        }
    }
    if (lane == 0) atomicAdd(cyc, waitc);
}

__global__ __launch_bounds__(256) void store_lat(float* dff, long long E, unsigned long long* cyc, int mode) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long ngroups = E / EW;
    const long long ws = (long long)gridDim.x * 4;
    unsigned long long acc = 0;
    float4* base = reinterpret_cast<float4*>(dff);
    for (long long g = (long long)blockIdx.x * 4 + wv; g < ngroups; g += ws) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        if (mode == 0) {
            base[g * 72 + lane] = make_float4(1.f, 2.f, 3.f, (float)g);
        } else {
            float4 v = base[g * 72 + lane];
            if (v.x == 12345.f) base[0] = v;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        acc += t1 - t0;
    }
    if (lane == 0) atomicAdd(cyc, acc);
}

int probe() {
    const long long E = 65536;
    float* dff;
    unsigned long long* cyc;
    CK(hipMalloc(&dff, E * HW * 4));
    CK(hipMemset(dff, 0, E * HW * 4));
    CK(hipMalloc(&cyc, 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int v = 0; v < 2; v++) {
        for (int blocks : {1024, 2048}) {
            for (int i = 0; i < 3; i++) { if (v) reg_prefetch<<<blocks, 256>>>(dff, E); else lds_roundtrip<<<blocks, 256>>>(dff, E); }
            CK(hipEventRecord(a));
            for (int i = 0; i < 20; i++) { if (v) reg_prefetch<<<blocks, 256>>>(dff, E); else lds_roundtrip<<<blocks, 256>>>(dff, E); }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%s blocks=%d: %.2f us/launch\n", v ? "reg_prefetch " : "lds_roundtrip", blocks, ms * 1e3 / 20);
        }
    }
    for (int mode : {0, 1}) {
        for (int blocks : {256, 1024}) {
            CK(hipMemset(cyc, 0, 8));
            store_lat<<<blocks, 256>>>(dff, E, cyc, mode);
            CK(hipDeviceSynchronize());
            unsigned long long c;
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            printf("%s latency (issue -> vmcnt(0)), blocks=%d: %.0f cyc\n", mode ? "load " : "store", blocks,
                   (double)c / (E / EW));
        }
    }
    for (int spin : {0, 200}) {
        for (int blocks : {1024, 2048}) {
          for (int nostore : {0, 1, 2, 3}) {
            CK(hipMemset(cyc, 0, 8));
            pipelined<true><<<blocks, 256>>>(dff, E, spin, cyc, nostore);
            CK(hipMemset(cyc, 0, 8));
            CK(hipEventRecord(a));
            for (int i = 0; i < 20; i++) {
                if (nostore & 2) pipelined<false><<<blocks, 256>>>(dff, E, spin, cyc, nostore & 1);
                else pipelined<true><<<blocks, 256>>>(dff, E, spin, cyc, nostore & 1);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            unsigned long long c;
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            const double waves = blocks * 4.0, groups = E / EW;
            printf("pipelined spin=%5d blocks=%5d nostore=%d  %8.2f us/launch  stage-wait %8.0f cyc/group\n", spin,
                   blocks, nostore, ms * 1e3 / 20, (double)c / 20 / groups);
            (void)waves;
          }
        }
    }
    return 0;
}
