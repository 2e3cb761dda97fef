// device_common.h -- device-side arithmetic shared by the FFM kernels (gfx950).
//
// Everything here reproduces a piece of third-party arithmetic the reference
// relies on, bit for bit:
//   * np_expf      -- NumPy 2.x float32 exp (called at model/ffm_core.py:80)
//   * u53 / MT19937 -- NumPy legacy RandomState and CPython `random`
//                      (model/ffm_core.py:25,84,95,96)
//   * randbelow    -- CPython Random._randbelow_with_getrandbits
// plus the production Philox4x32-10 generator.  Translation units that
// include this are compiled with -ffp-contract=off: every + and * rounds on
// its own, as in NumPy's element-wise loops; fmaf is used only where NumPy's
// own exp uses FMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ffm {

constexpr uint16_t kEmpty = 0xFFFF;     // occupancy: no agent in this cell
constexpr uint16_t kNoReq = 0xFFFF;     // decide: no move request
constexpr uint16_t kPending = 0xFFFE;   // decide (MT pass 1): needs a draw

enum : uint32_t { kPurDecide = 1, kPurFriction = 2, kPurReset = 3 };

// ---- NumPy float32 exp ----------------------------------------------------
__device__ __forceinline__ float np_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return __builtin_inff();
    if (x < -103.97208404541015625f) return 0.0f;
    const float q = __builtin_rintf(x * 1.442695040888963407359924681001892137f);
    float r = __builtin_fmaf(q, -6.93145752e-1f, x);
    r = __builtin_fmaf(q, -1.42860677e-6f, r);
    float num = __builtin_fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    num = __builtin_fmaf(num, r, 5.114512081637298353406e-02f);
    num = __builtin_fmaf(num, r, 2.473615434895520810817e-01f);
    num = __builtin_fmaf(num, r, 7.257664613233124478488e-01f);
    num = __builtin_fmaf(num, r, 9.999999999980870924916e-01f);
    float den = __builtin_fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    den = __builtin_fmaf(den, r, 1.0f);
    return __builtin_ldexpf(num / den, (int)q);   // IEEE divide (correctly rounded build)
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ int bit_length(uint32_t n) { return n ? 32 - __builtin_clz(n) : 0; }

// ---- Philox4x32-10 ----------------------------------------------------------
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
    // Opaque key: keeps the compiler from hoisting the 20-word key schedule out of
    // the step loop into SGPRs (it spills them); 2 s_add per round are cheaper.
    // (the keys are wave-uniform everywhere; readfirstlane pins them to SGPRs where a
    // kernel's register allocation moved them into VGPRs -- a no-op otherwise)
    k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);
    k1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
    asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
    for (int r = 0; r < 10; r++) {
        // one v_mad_u64_u32 per product: ~30% cheaper than mul_lo + mul_hi on gfx950
        const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
        const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        // three-input xor in one v_bitop3_b32 (gfx950; truth table 0x96): the compiler
        // otherwise issues two v_xor_b32 per word
        c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
                       __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// A keyed word stream: counter (t, env, idx, purpose<<28 | sub), 4 words per block.
struct PhiloxStream {
    uint4 ctr;
    uint32_t k0, k1;
    uint4 buf;
    int used;
    __device__ PhiloxStream(uint32_t key0, uint32_t key1, uint32_t t, uint32_t env, uint32_t idx,
                            uint32_t purpose)
        : ctr(make_uint4(t, env, idx, purpose << 28)), k0(key0), k1(key1), buf(), used(4) {}
    __device__ uint32_t next() {
        if (used == 4) {
            buf = philox(ctr, k0, k1);
            ctr.w++;
            used = 0;
        }
        const uint32_t w = used == 0 ? buf.x : used == 1 ? buf.y : used == 2 ? buf.z : buf.w;
        used++;
        return w;
    }
    __device__ double next_u53() {
        const uint32_t a = next();
        const uint32_t b = next();
        return u53(a, b);
    }
    __device__ uint32_t randbelow(uint32_t n) {
        if (n <= 1) return 0;
        const int k = bit_length(n);
        uint32_t r = next() >> (32 - k);
        while (r >= n) r = next() >> (32 - k);
        return r;
    }
};

// ---- MT19937 on a 625-word state (624 words + position) in LDS ---------------
__device__ inline void mt_twist(uint32_t* mt) {
    const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MA = 0x9908b0dfu;
    int kk;
    uint32_t y;
    for (kk = 0; kk < 624 - 397; kk++) {
        y = (mt[kk] & UP) | (mt[kk + 1] & LO);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
    }
    for (; kk < 623; kk++) {
        y = (mt[kk] & UP) | (mt[kk + 1] & LO);
        mt[kk] = mt[kk - 227] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
    }
    y = (mt[623] & UP) | (mt[0] & LO);
    mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
}

__device__ inline uint32_t mt_next(uint32_t* mt) {
    uint32_t pos = mt[624];
    if (pos >= 624) {
        mt_twist(mt);
        pos = 0;
    }
    uint32_t y = mt[pos];
    mt[624] = pos + 1;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ inline double mt_u53(uint32_t* mt) {
    const uint32_t a = mt_next(mt);
    const uint32_t b = mt_next(mt);
    return u53(a, b);
}

__device__ inline uint32_t mt_randbelow(uint32_t* mt, uint32_t n) {
    if (n == 0) return 0;
    const int k = bit_length(n);
    uint32_t r = mt_next(mt) >> (32 - k);
    while (r >= n) r = mt_next(mt) >> (32 - k);
    return r;
}

// ---- neighbourhoods (model/ffm_core.py:28-34, order matters) -----------------
template <int NB>
__device__ __forceinline__ constexpr int nb_dx(int s) {
    return NB == 4 ? (s == 0 ? -1 : s == 1 ? 1 : 0) : (s < 3 ? -1 : s < 5 ? 0 : 1);
}
template <int NB>
__device__ __forceinline__ constexpr int nb_dy(int s) {
    return NB == 4 ? (s == 2 ? -1 : s == 3 ? 1 : 0)
                   : (s == 0 || s == 3 || s == 5 ? -1 : s == 1 || s == 6 ? 0 : 1);
}

}  // namespace ffm
