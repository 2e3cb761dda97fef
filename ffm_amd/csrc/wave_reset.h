// wave_reset.h -- Philox placement of one env by one wavefront (shared by the
// wave, pack and reset kernels).  See DESIGN.md 3.2 "placement".
#pragma once
#include "core_common.h"
#include "kernels.h"

namespace ffm {

__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

// Philox placement of one env, stored straight to its global positions gpos[0..N)
// (unpadded cell indices): all 64 lanes.
// fl = padded free-cell list (LDS).  F <= 128: the (key, j) pairs go to LDS and
// each lane ranks its two by broadcast reads -- few registers, because this
// rarely-taken branch sits inside the step loop and would otherwise set the
// kernel's VGPR peak.  Larger F: threshold the keys into an LDS candidate list
// first (about 2N + 16 survive).
__device__ inline void wave_reset_env(const CoreStepArgs& a, uint32_t genv, unsigned long long* keys, const uint16_t* fl,
                               uint16_t* gpos, int lane) {
    const int PW = a.W + 2;
    const int F = a.F, N = a.N;
    if (F <= 128) {
        // lane holds keys j0 = lane and j1 = lane + 64 and ranks both in one pass over
        // 16-B broadcast reads of the key list (two keys per read; keys is 16-B aligned)
        const int j0 = lane, j1 = lane + 64;
        const unsigned long long k0 =
            j0 < F ? ((unsigned long long)reset_key(a.key0, a.key1, a.t, genv, (uint32_t)j0) << 32) | (unsigned)j0
                   : ~0ull;
        const unsigned long long k1 =
            j1 < F ? ((unsigned long long)reset_key(a.key0, a.key1, a.t, genv, (uint32_t)j1) << 32) | (unsigned)j1
                   : ~0ull;
        if (j0 < F) keys[j0] = k0;
        if (j1 < F) keys[j1] = k1;
        if (lane == 0 && (F & 1)) keys[F] = ~0ull;   // pad to pairs: ~0 is never below a key
        wave_sync();
        int r0 = 0, r1 = 0;
        const ulonglong2* kv = reinterpret_cast<const ulonglong2*>(keys);
#pragma unroll 8
        for (int q = 0; q < (F + 1) / 2; q++) {
            const ulonglong2 p = kv[q];
            r0 += (p.x < k0 ? 1 : 0) + (p.y < k0 ? 1 : 0);
            r1 += (p.x < k1 ? 1 : 0) + (p.y < k1 ? 1 : 0);
        }
        if (j0 < F && r0 < N) gpos[r0] = (uint16_t)unpad(fl[j0], PW);
        if (j1 < F && r1 < N) gpos[r1] = (uint16_t)unpad(fl[j1], PW);
        wave_sync();
        return;
    }
    uint32_t T = reset_threshold(N, F);
    int C = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        C = 0;
        for (int j0 = 0; j0 < F; j0 += 64) {
            const int j = j0 + lane;
            uint32_t k = 0;
            bool cand = false;
            if (j < F) {
                k = reset_key(a.key0, a.key1, a.t, genv, (uint32_t)j);
                cand = k <= T;
            }
            const unsigned long long m = __ballot(cand);
            if (cand) keys[C + lanes_below(m)] = ((unsigned long long)k << 32) | (unsigned)j;
            C += __popcll(m);
        }
        if (C >= N || T == 0xFFFFFFFFu) break;
        T = 0xFFFFFFFFu;
    }
    wave_sync();
    for (int i = lane; i < C; i += 64) {
        const unsigned long long ki = keys[i];
        int rank = 0;
        for (int q = 0; q < C; q++) rank += keys[q] < ki ? 1 : 0;
        if (rank < N) gpos[rank] = (uint16_t)unpad(fl[(int)(ki & 0xFFFFu)], PW);
    }
    wave_sync();
}

}  // namespace ffm
