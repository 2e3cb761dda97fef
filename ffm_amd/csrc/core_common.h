// core_common.h -- per-agent pieces of the ffm_core step shared by the
// wave-per-env and block-per-env kernels (model/ffm_core.py of SoraKurihara/FFM).
//
// Layout convention inside LDS: every per-env grid is PADDED by one cell on
// each side (row stride PW = W + 2), so neighbour offsets are constants and no
// bounds checks are needed.  The halo is "blocked" in the grid and 0 in the
// DFF tile, which is exactly the zero padding of np.pad in update_dff
// (model/ffm_core.py:111).
//
// Grid cell codes: 0 free, 2 blocked (wall or any non-walkable value), 3 exit,
// AGENT_BIT | i = agent i currently there (model/ffm_ac_core.py:120-122 builds
// the same "state map").  A cell is a candidate iff its code is 0 or 3
// (model/ffm_core.py:52-60: walkable AND not occupied by another agent).
#pragma once
#include "device_common.h"

namespace ffm {

template <class GT>
struct GridCodes;
template <>
struct GridCodes<uint8_t> {
    static constexpr uint32_t kAgent = 0x80u, kIdx = 0x7Fu;
};
template <>
struct GridCodes<uint16_t> {
    static constexpr uint32_t kAgent = 0x8000u, kIdx = 0x7FFFu;
};

struct DrawPhilox {
    uint32_t k0, k1, t, env, agent;
    __device__ double get() const {
        const uint4 w = philox(make_uint4(t, env, agent, kPurDecide << 28), k0, k1);
        return u53(w.x, w.y);
    }
};
struct DrawFixed {
    double u;
    __device__ double get() const { return u; }
};
struct DrawPending {
    __device__ double get() const { return -1.0; }
};

// NumPy add.reduce of the candidate exps: left fold below 8 elements, 8-lane
// pairwise at >= 8 (only reachable with the Moore neighbourhood).
template <int NB, class T>
__device__ __forceinline__ T np_sum(const T (&e)[NB + 1], const bool (&v)[NB + 1], int nc) {
    if (NB == 8 && nc >= 8) {
        int q = NB + 1;  // slot of the (at most one) invalid neighbour
#pragma unroll
        for (int s = NB - 1; s >= 0; s--)
            if (!v[s]) q = s;
        T a[8];
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = (j < q) ? e[j] : e[j + 1];
        T res = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        if (nc == 9) res += e[8];
        return res;
    }
    T res = T(-0.0);
#pragma unroll
    for (int s = 0; s <= NB; s++)
        if (v[s]) res += e[s];
    return res;
}

// np.random.choice's comparison fl(cdf_k / cdf_last) > u without a float64
// division in the common case: q = cdf_k * (1/cdf_last) is within a few ulp
// of the correctly rounded quotient, so it decides unless it lands within
// 2^-48 of u; only then is the exact IEEE division evaluated.
__device__ __forceinline__ bool cdf_gt(double ck, double last, double inv_last, double u) {
    const double q = ck * inv_last;
    const double d = q - u;
    if (d > 0x1p-48) return true;
    if (d < -0x1p-48) return false;
    return ck / last > u;
}

// np.random.choice on the exact float64 cdf: cdf /= cdf[-1];
// idx = searchsorted(cdf, u, side="right").
template <int NB>
__device__ __forceinline__ uint32_t exact_pick(const double (&cdf)[NB + 1], double last, const bool (&v)[NB + 1],
                                               double u) {
    const double inv = 1.0 / last;
    uint32_t slot = NB;
    bool found = false;
#pragma unroll
    for (int k = 0; k < NB; k++) {
        if (v[k] && !found && cdf_gt(cdf[k], last, inv, u)) {
            found = true;
            slot = (uint32_t)k;
        }
    }
    return slot;  // the stay slot has cdf == 1 > u
}

// Fast path of the choice.  Probabilities from the hardware exp2 (v_exp_f32)
// and a float32 running sum differ from NumPy's exact pipeline (np.exp f32,
// pairwise sum, f32 divide, f64 cumsum and normalisation) by less than 1e-5
// of the total for every argument that matters (|x| < 30; terms below e^-30
// are < 1e-13 of the total).  A slot is returned only when u is at least
// kFastMargin = 1e-4 (10x that bound) away from every cdf boundary it is
// compared with, so the answer equals the exact one; otherwise -1 and the
// caller runs the exact emulation.  Branch-free (selects only).
#ifndef FFM_FAST_MARGIN
#define FFM_FAST_MARGIN 1e-4f
#endif
constexpr float kFastMargin = FFM_FAST_MARGIN;

template <int NB>
__device__ __forceinline__ int fast_choice(const float (&x)[NB + 1], const bool (&v)[NB + 1], double u) {
    float cum[NB + 1];
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        const float e = __builtin_amdgcn_exp2f(x[k] * 1.44269504088896341f);
        acc += v[k] ? e : 0.0f;
        cum[k] = v[k] ? acc : -1.0f;   // invalid slots never selected
    }
    const float t = (float)u * acc;
    const float d = kFastMargin * acc;
    // The valid cum values are non-decreasing, so the first slot with cum >= t - d
    // is the only candidate: it is the answer when cum > t + d, else u is too
    // close to a boundary (-1).  Selects from the top down: VALU only.
    int slot = NB;
    float cs = cum[NB];
#pragma unroll
    for (int k = NB - 1; k >= 0; k--) {
        const bool ge = cum[k] >= t - d;
        slot = ge ? k : slot;
        cs = ge ? cum[k] : cs;
    }
    return cs > t + d ? slot : -1;
}

// decide() for one agent at padded cell pp: model/ffm_core.py:41-88.
// Returns the chosen slot (neighbour index, NB = stay), kNoReq, or kPending (draw
// needed, MT pass 1); slot_cell() turns a slot into the padded target cell.
// Every slot is evaluated unconditionally (all neighbour cells exist in the
// padded grid), so the LDS loads issue together and no lane diverges except
// into the rare exact path.
// The DFF tile may use a wider row stride than the grid: the tile index of grid
// cell c in row x + dx of the agent is c + dd0 + dx * dws (dd0 = dws = 0 when the
// tile shares the grid's layout).
template <int NB, bool F64, class GT, class Draw>
__device__ __forceinline__ uint32_t decide(int pp, int PW, const GT* grid, const float* sff32,
                                           const double* sff64, const float* dff, int dd0, int dws,
                                           float kS32, float kD32, double kS64, const Draw& draw) {
    int cell[NB + 1];
    int dcell[NB + 1];
    bool v[NB + 1];
    uint32_t g[NB];
#pragma unroll
    for (int s = 0; s < NB; s++) {
        cell[s] = pp + nb_dx<NB>(s) * PW + nb_dy<NB>(s);
        dcell[s] = cell[s] + dd0 + nb_dx<NB>(s) * dws;
        g[s] = grid[cell[s]];
    }
    cell[NB] = pp;                                                   // :64 stay, last
    dcell[NB] = pp + dd0;
    v[NB] = true;
    int nvalid = 0;
    int exit_slot = -1;
#pragma unroll
    for (int s = NB - 1; s >= 0; s--) {
        v[s] = g[s] == 0u || g[s] == 3u;                             // :52-60
        nvalid += v[s] ? 1 : 0;
        exit_slot = g[s] == 3u ? s : exit_slot;                      // :66-72 first exit
    }
    const int nc = nvalid + 1;

    if (!F64) {
        float sc[NB + 1];
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            const float a = kS32 * sff32[cell[k]];
            const float b = kD32 * dff[dcell[k]];
            sc[k] = a + b;                                           // :77
        }
        float mx = -__builtin_inff();
#pragma unroll
        for (int k = 0; k <= NB; k++) mx = (v[k] && sc[k] > mx) ? sc[k] : mx;   // :78
        float xs[NB + 1];
#pragma unroll
        for (int k = 0; k <= NB; k++) xs[k] = v[k] ? sc[k] - mx : -__builtin_inff();   // :80 argument, exact
        const double u = draw.get();                                 // :84
        if (nvalid == 0) return kNoReq;                              // :63
        if (exit_slot >= 0) return (uint32_t)exit_slot;
        if (u < 0.0) return kPending;
        const int fs = fast_choice<NB>(xs, v, u);
        if (fs >= 0) return (uint32_t)fs;
        // u is within the margin of a boundary: the exact NumPy arithmetic decides.
        float e[NB + 1];
#pragma unroll
        for (int k = 0; k <= NB; k++) e[k] = v[k] ? np_expf(xs[k]) : 0.0f;                // :80
        const float sum = np_sum<NB, float>(e, v, nc);                                    // :81
        double cdf[NB + 1];
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            if (v[k]) acc += (double)(e[k] / sum);                   // :83, then cumsum in choice
            cdf[k] = acc;
        }
        return exact_pick<NB>(cdf, acc, v, u);
    } else {
        if (nvalid == 0) return kNoReq;
        if (exit_slot >= 0) return (uint32_t)exit_slot;
        double sc[NB + 1], e[NB + 1];
        double mx = -__builtin_inf();
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            if (!v[k]) { sc[k] = 0.0; continue; }
            const float b = kD32 * dff[dcell[k]];
            sc[k] = kS64 * sff64[cell[k]] + (double)b;
            mx = sc[k] > mx ? sc[k] : mx;
        }
#pragma unroll
        for (int k = 0; k <= NB; k++) e[k] = v[k] ? exp(sc[k] - mx) : 0.0;
        const double sum = np_sum<NB, double>(e, v, nc);
        double cdf[NB + 1];
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            if (v[k]) acc += e[k] / sum;
            cdf[k] = acc;
        }
        const double u = draw.get();                                 // :84
        if (u < 0.0) return kPending;
        return exact_pick<NB>(cdf, acc, v, u);
    }
}

// Padded cell of slot `slot` around pp (kNoReq / kPending pass through).
template <int NB>
__device__ __forceinline__ uint32_t slot_cell(uint32_t slot, int pp, int PW) {
    int off = 0;
#pragma unroll
    for (int s = 0; s < NB; s++) off = slot == (uint32_t)s ? nb_dx<NB>(s) * PW + nb_dy<NB>(s) : off;
    return slot <= (uint32_t)NB ? (uint32_t)(pp + off) : slot;
}

// slot_cell with the padded row stride known at compile time: the four Neumann offsets
// (U, D, L, R: -PW, +PW, -1, +1; stay 0) as 6-bit fields of one constant, read by one
// signed bit-field extract instead of a compare-and-select per direction.
template <int NB, int PW>
__device__ __forceinline__ uint32_t slot_cell_k(uint32_t slot, int pp) {
    if constexpr (NB == 4 && PW <= 31) {
        constexpr uint32_t K = ((uint32_t)(-PW) & 63u) | (((uint32_t)PW & 63u) << 6) | (63u << 12) | (1u << 18);
        const int off = __builtin_amdgcn_sbfe((int)K, slot * 6u, 6u);
        return slot <= 4u ? (uint32_t)(pp + off) : slot;
    } else {
        return slot_cell<NB>(slot, pp, PW);
    }
}

// The requesters of target r (padded): agents adjacent to r whose request is r.
// who[s] = agent index at r - off(s) (or 0xFFFF), is[s] = it requests r.
template <int NB, class GT, class RT = uint16_t>
__device__ __forceinline__ int requesters(int r, int PW, const GT* grid, const RT* sreq,
                                          uint16_t (&who)[NB], bool (&is)[NB]) {
    uint32_t g[NB];
#pragma unroll
    for (int s = 0; s < NB; s++) g[s] = grid[r - nb_dx<NB>(s) * PW - nb_dy<NB>(s)];
    RT q[NB];
#pragma unroll
    for (int s = 0; s < NB; s++) {
        const bool ag = (g[s] & GridCodes<GT>::kAgent) != 0u;
        who[s] = ag ? (uint16_t)(g[s] & GridCodes<GT>::kIdx) : (uint16_t)0xFFFF;
        q[s] = sreq[ag ? (g[s] & GridCodes<GT>::kIdx) : 0u];         // unconditional load
    }
    int m = 0;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        is[s] = who[s] != 0xFFFF && q[s] == (RT)r;
        m += is[s] ? 1 : 0;
    }
    return m;
}

// Direction-coded occupancy grid (u16, wave and pack kernels): 0 free, 2
// blocked, 3 exit; an agent cell holds kAgent | index | slot << 8, where slot is
// the neighbour index its decide chose (NB = stay, kNoDir = no request).
struct DirCodes {
    static constexpr uint32_t kAgent = 0x80u, kIdx = 0x7Fu, kNoDir = 0xFu;
};

// Requesters of target r from a direction-coded grid: the agents on r's
// neighbour cells whose chosen slot points at r -- one LDS round trip.
template <int NB>
__device__ __forceinline__ int requesters_dir(int r, int PW, const uint16_t* grid, uint16_t (&who)[NB],
                                              bool (&is)[NB]) {
    int m = 0;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        const uint32_t c = grid[r - nb_dx<NB>(s) * PW - nb_dy<NB>(s)];
        is[s] = (c & DirCodes::kAgent) != 0u && ((c >> 8) & 0xFu) == (uint32_t)s;
        who[s] = (uint16_t)(c & DirCodes::kIdx);
        m += is[s] ? 1 : 0;
    }
    return m;
}

// Slot (neighbour index) of the k-th smallest requester.
template <int NB>
__device__ __forceinline__ int kth_slot(const uint16_t (&who)[NB], const bool (&is)[NB], int k) {
    int sel = -1;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        int rank = 0;
#pragma unroll
        for (int q = 0; q < NB; q++) rank += (is[q] && who[q] < who[s]) ? 1 : 0;
        if (is[s] && rank == k) sel = s;
    }
    return sel;
}

// Philox-mode friction for a contested target: z, w = words 2, 3
// of the owner's decide block.  Coin: z < 2^31 (exactly 1/2).  Winner rank:
// Lemire multiply-shift of w by m, exact through rejection of the low word below
// 2^32 mod m (probability < m/2^32); a rejected word is replaced from the owner's
// friction stream.  Returns the rank in [0, m) or -1 (nobody moves).
__device__ __forceinline__ int philox_friction(uint32_t z, uint32_t w, uint32_t m, uint32_t k0, uint32_t k1,
                                               uint32_t t, uint32_t genv, uint32_t owner) {
    if (z >= 0x80000000u) return -1;
    const uint32_t thr = (uint32_t)((0x044101000ull >> (4 * m)) & 0xFu);   // 2^32 mod m, m = 2..8
    unsigned long long prod = (unsigned long long)w * m;
    if ((uint32_t)prod < thr) {
        PhiloxStream ps(k0, k1, t, genv, owner, kPurFriction);
        do prod = (unsigned long long)ps.next() * m; while ((uint32_t)prod < thr);
    }
    return (int)(prod >> 32);
}

// Philox-mode placement key of free-list entry j (see DESIGN.md "Placement").
__device__ __forceinline__ uint32_t reset_key(uint32_t k0, uint32_t k1, uint32_t t, uint32_t genv, uint32_t j) {
    return philox(make_uint4(t, genv, j, kPurReset << 28), k0, k1).x;
}

// Candidate threshold: ~2N of F keys fall below it; exact fallback = all.
__device__ __forceinline__ uint32_t reset_threshold(int N, int F) {
    if (N >= F) return 0xFFFFFFFFu;
    const unsigned long long t = ((unsigned long long)(2 * N + 16) << 32) / (unsigned long long)F;
    return t >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t;
}

// n / d by one multiply-high, m = ceil(2^32 / d) (magic_div), exact whenever n * d < 2^32:
// m = (2^32 + r) / d with r < d, so n * m / 2^32 = n / d + n * r / (d * 2^32), and the error
// term n * r / (d * 2^32) < n * d / (d * 2^32) < 1 / d stays below the gap to the next integer.
// (n < 2^17 alone is not enough: d = 65535, n = 131069 gives 2.)  Checked on the host.
__device__ __forceinline__ int mdiv(int n, uint32_t m) { return (int)__umulhi((uint32_t)n, m); }

// unpad with a runtime row width: the quotient by magic_div(PW)
__device__ __forceinline__ int unpad_m(int pp, int PW, uint32_t mPW) {
    const int q = mdiv(pp, mPW);
    return (q - 1) * (PW - 2) + (pp - q * PW - 1);
}

__device__ __forceinline__ int unpad(int pp, int PW) {
    const int x = pp / PW - 1, y = pp - (pp / PW) * PW - 1;
    return x * (PW - 2) + y;
}

// Number of set bits of `m` in lanes below this one (v_mbcnt; no per-lane mask).
__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

}  // namespace ffm
