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
        for (int j = lane; j < F; j += 64)
            keys[j] = ((unsigned long long)reset_key(a.key0, a.key1, a.t, genv, (uint32_t)j) << 32) | (unsigned)j;
        wave_sync();
        for (int j = lane; j < F; j += 64) {
            const unsigned long long kj = keys[j];
            int r = 0;
#pragma unroll 4
            for (int q = 0; q < F; q++) r += keys[q] < kj ? 1 : 0;
            if (r < N) gpos[r] = (uint16_t)unpad(fl[j], PW);
        }
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
