// lane_common.h -- pieces shared by the lane (pair-per-wave) and group (packed agent
// lanes) Philox step kernels: DFF tile geometry, buffer-resource I/O and the
// per-agent decide() of model/ffm_core.py:40-88 (fast pass + exact NumPy fallback).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "core_common.h"

namespace ffm {
namespace {

__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// DFF tile of one env: 4 leading zero floats, H + 2 rows of W floats (a zero row
// above and below the map; no halo columns, so the float4 slots of consecutive lanes
// are consecutive and the 16-B accesses are bank-conflict free), 4 trailing zeros.
// Cell (x, y) at 4 + (x + 1) * W + y.  Left / right neighbours across the map edge
// are read from a zero word instead (the stencil) or belong to blocked cells whose
// score is masked (decide).
__host__ __device__ constexpr int lane_tile_floats(int H, int W) { return 4 + (H + 2) * W + 4; }

// Buffer resources over one env pair's rows of pos / cnt / DFF: a lane whose offset
// is past the pair's bytes reads 0 and its store is dropped by the hardware, so no
// load or store of the loop needs a lane branch, and the number of memory
// instructions after the prefetch is fixed (the loop head then waits for the
// prefetch only, not for the previous group's stores).
constexpr int kOOB = 0x7FFFFFF0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pair_rsrc(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r,
                                           off, 0, 0);
}


// Candidate cells, validity and float32 scores of decide() (model/ffm_core.py:41-80)
// for the agent at padded cell pp; shared by the fast and the exact pass.
// PRE: psff holds f32(-k_S) * SFF already (the product the score takes, staged once per
// workgroup), so kS is not applied again; results are identical.
// DWS: the DFF tile's row stride minus the grid's (the small-env tiles have no halo columns:
// -2; a tile laid out like the grid: 0).
template <int NB, bool PRE = false, int DWS = -2>
__device__ __forceinline__ int lane_scores(int pp, int PW, const uint16_t* gk, const float* psff, const float* dk,
                                           int dd0, float kS, float kD, bool (&v)[NB + 1], float (&xs)[NB + 1],
                                           int& exit_slot) {
    int cell[NB + 1], dcell[NB + 1];
    uint32_t g[NB];
    float sf[NB + 1], df[NB + 1];
#pragma unroll
    for (int s = 0; s < NB; s++) {
        cell[s] = pp + nb_dx<NB>(s) * PW + nb_dy<NB>(s);
        dcell[s] = cell[s] + dd0 + nb_dx<NB>(s) * DWS;   // the tile row is -DWS shorter than the grid row
        g[s] = gk[cell[s]];
    }
    cell[NB] = pp;
    dcell[NB] = pp + dd0;
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        sf[k] = psff[cell[k]];
        df[k] = dk[dcell[k]];
    }
    v[NB] = true;
    int nvalid = 0;
    exit_slot = -1;
#pragma unroll
    for (int s = NB - 1; s >= 0; s--) {
        v[s] = g[s] == 0u || g[s] == 3u;                                 // :52-60
        nvalid += v[s] ? 1 : 0;
        exit_slot = g[s] == 3u ? s : exit_slot;                          // :66-72
    }
    float sc[NB + 1];
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        const float a = PRE ? sf[k] : kS * sf[k];
        const float b = kD * df[k];
        sc[k] = a + b;                                                   // :77
    }
    float mx = -__builtin_inff();
#pragma unroll
    for (int k = 0; k <= NB; k++) mx = (v[k] && sc[k] > mx) ? sc[k] : mx;   // :78
#pragma unroll
    for (int k = 0; k <= NB; k++) xs[k] = v[k] ? sc[k] - mx : -__builtin_inff();
    return nvalid;
}

// decide(), fast pass: returns the slot (0..NB-1 neighbour, NB stay), kNoReq, or
// kPending when u lies within the margin of a cdf boundary.  The fast path compares
// a float32 copy of u (|error| < 2^-24) inside fast_choice's 1e-4 margin; selects
// only, no branch.
//   * An invalid candidate's score is masked to -inf before the max and the exp, so
//     its term is exactly 0 and its cum equals the previous one: the lowest slot with
//     cum >= t - d is then valid, or slot 0 invalid with u <= the margin, which the
//     acceptance test (cum > t + d) sends to the exact pass -- the same decisions as
//     masking every step separately, in 7 instead of 11 VALU per candidate.
//   * KD1 (k_D == 1, the drivers' setting): k_D * DFF is DFF itself (an exact product).
template <int NB, bool PRE = false, bool KD1 = false, int DWS = -2>
__device__ __forceinline__ uint32_t lane_decide(int pp, int PW, const uint16_t* gk, const float* psff,
                                                const float* dk, int dd0, float kS, float kD, uint32_t wx,
                                                bool& to_exit) {
    int cell[NB + 1], dcell[NB + 1];
    uint32_t g[NB];
    float sf[NB + 1], df[NB + 1];
#pragma unroll
    for (int s = 0; s < NB; s++) {
        cell[s] = pp + nb_dx<NB>(s) * PW + nb_dy<NB>(s);
        dcell[s] = cell[s] + dd0 + nb_dx<NB>(s) * DWS;   // the tile row is -DWS shorter than the grid row
        g[s] = gk[cell[s]];
    }
    cell[NB] = pp;
    dcell[NB] = pp + dd0;
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        sf[k] = psff[cell[k]];
        df[k] = dk[dcell[k]];
    }
    bool v[NB + 1];
    v[NB] = true;
    bool anyv = false;     // a valid neighbour (a lane-mask OR, not a per-lane count)
    int exit_slot = -1;
#pragma unroll
    for (int s = NB - 1; s >= 0; s--) {
        v[s] = g[s] == 0u || g[s] == 3u;                                 // :52-60
        anyv = anyv || v[s];
        exit_slot = g[s] == 3u ? s : exit_slot;                          // :66-72
    }
    float scm[NB + 1];
    float mx = -__builtin_inff();
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        const float a = PRE ? sf[k] : kS * sf[k];
        const float b = KD1 ? df[k] : kD * df[k];
        scm[k] = v[k] ? a + b : -__builtin_inff();                       // :77
        mx = __builtin_fmaxf(mx, scm[k]);                                // :78
    }
    float cum[NB + 1];
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        const float x = __builtin_amdgcn_exp2f((scm[k] - mx) * 1.44269504088896341f);
        acc = k == 0 ? x : acc + x;      // exp2 is never -0: 0 + x == x, one add fewer
        cum[k] = acc;
    }
    const float uf = (float)(wx >> 8) * 0x1p-24f;
    const float t = uf * acc;
    const float d = kFastMargin * acc;
    int slot = NB;
    float cs = cum[NB];
#pragma unroll
    for (int k = NB - 1; k >= 0; k--) {
        const bool ge = cum[k] >= t - d;
        slot = ge ? k : slot;
        cs = ge ? cum[k] : cs;
    }
    to_exit = exit_slot >= 0;
    return !anyv ? (uint32_t)kNoReq                                      // :63
           : exit_slot >= 0 ? (uint32_t)exit_slot                        // :66-72, no draw
           : cs > t + d ? (uint32_t)slot : (uint32_t)kPending;
}

// decide(), exact pass (rare): NumPy's float32 exp and add.reduce, float32 divide,
// float64 cumsum, cdf /= cdf[-1], searchsorted(side="right") on the float64 u53.
// Streams over the candidates, re-reading the scores from LDS in each of its passes
// (max, sum, cdf total, search) with one candidate live at a time: this path sets
// the kernel's register peak otherwise.  Neumann only (the 8-lane pairwise sum of
// add.reduce needs every term at once: lane_decide_exact_arr).
template <int NB, bool PRE = false, int DWS = -2>
__device__ __forceinline__ float lane_score1(int k, int pp, int PW, const uint16_t* gk, const float* psff,
                                             const float* dk, int dd0, float kS, float kD, bool& valid) {
    int dx = 0, dy = 0;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        dx = k == s ? nb_dx<NB>(s) : dx;
        dy = k == s ? nb_dy<NB>(s) : dy;
    }
    const int cell = pp + dx * PW + dy;
    const uint32_t g = gk[cell];
    valid = k == NB || g == 0u || g == 3u;
    const float sa = PRE ? psff[cell] : kS * psff[cell];
    const float sb = kD * dk[cell + dd0 + dx * DWS];
    return sa + sb;                                                      // :77
}

template <int NB, bool PRE = false, int DWS = -2>
__device__ __forceinline__ uint32_t lane_decide_exact(int pp, int PW, const uint16_t* gk, const float* psff,
                                                      const float* dk, int dd0, float kS, float kD, double u) {
    float mx = -__builtin_inff();
#pragma unroll 1
    for (int k = 0; k <= NB; k++) {
        bool v;
        const float sc = lane_score1<NB, PRE, DWS>(k, pp, PW, gk, psff, dk, dd0, kS, kD, v);
        mx = (v && sc > mx) ? sc : mx;                                   // :78
    }
    float sum = -0.0f;                                                   // add.reduce, < 8 terms: left fold
#pragma unroll 1
    for (int k = 0; k <= NB; k++) {
        bool v;
        const float sc = lane_score1<NB, PRE, DWS>(k, pp, PW, gk, psff, dk, dd0, kS, kD, v);
        if (v) sum += np_expf(sc - mx);                                  // :80-81
    }
    double last = 0.0;
#pragma unroll 1
    for (int k = 0; k <= NB; k++) {
        bool v;
        const float sc = lane_score1<NB, PRE, DWS>(k, pp, PW, gk, psff, dk, dd0, kS, kD, v);
        if (v) last += (double)(np_expf(sc - mx) / sum);                 // :83, cumsum in choice
    }
    const double inv = 1.0 / last;
    double run = 0.0;
    uint32_t pick = NB;                                                  // cdf[-1] == 1 > u
#pragma unroll 1
    for (int k = 0; k < NB; k++) {
        bool v;
        const float sc = lane_score1<NB, PRE, DWS>(k, pp, PW, gk, psff, dk, dd0, kS, kD, v);
        if (v) {
            run += (double)(np_expf(sc - mx) / sum);
            if (cdf_gt(run, last, inv, u)) {
                pick = (uint32_t)k;
                break;
            }
        }
    }
    return pick;
}

// The same with every term held (Moore: add.reduce pairs 8 terms).
template <int NB, bool PRE = false, int DWS = -2>
__device__ __forceinline__ uint32_t lane_decide_exact_arr(int pp, int PW, const uint16_t* gk, const float* psff,
                                                          const float* dk, int dd0, float kS, float kD, double u) {
    bool v[NB + 1];
    float xs[NB + 1];
    int exit_slot;
    const int nvalid = lane_scores<NB, PRE, DWS>(pp, PW, gk, psff, dk, dd0, kS, kD, v, xs, exit_slot);
    float e[NB + 1];
#pragma unroll
    for (int k = 0; k <= NB; k++) e[k] = v[k] ? np_expf(xs[k]) : 0.0f;   // :80
    const float sum = np_sum<NB, float>(e, v, nvalid + 1);               // :81
    double last = 0.0;
#pragma unroll
    for (int k = 0; k <= NB; k++)
        if (v[k]) last += (double)(e[k] / sum);                          // :83, cumsum in choice
    const double inv = 1.0 / last;
    double run = 0.0;
    uint32_t pick = NB;
    bool found = false;
#pragma unroll
    for (int k = 0; k < NB; k++) {
        if (v[k]) run += (double)(e[k] / sum);
        if (v[k] && !found && cdf_gt(run, last, inv, u)) {
            found = true;
            pick = (uint32_t)k;
        }
    }
    return pick;
}

}  // namespace
}  // namespace ffm
