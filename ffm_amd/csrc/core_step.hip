// core_step.hip -- fused ffm_core step for a batch of independent environments.
//
// One launch advances every env by one FloorFieldModel.step()
// (model/ffm_core.py:36-104 of SoraKurihara/FFM):
//   decide   (:40-88)  lanes = agents; occupancy grid + DFF + SFF + map in LDS
//   resolve  (:90-98)  lanes = agents; the first requester of a target owns it
//   exit     (:100-102) order-preserving ballot/popcount compaction
//   update_dff (:106-117) lanes = cells; 4/8-point stencil over the LDS copy
//
// Work mapping: a workgroup holds K consecutive envs entirely in LDS
// (DFF f32 [K][HW], occupancy u16 [K][HW], positions/requests/next u16 [K][A]),
// so each env's state makes exactly one HBM round trip per step: positions
// (2A B) + count (4 B) + DFF (4HW B), read once and written once.  Map and
// SFF are shared by all envs and stay L2-resident.
//
// Sequential semantics in parallel:
//   * agent order: occupancy is built from the CURRENT positions only, so
//     decisions are independent across agents (the reference also reads only
//     the current positions at :48-60);
//   * dict insertion order of targets (:90): the requesters of a target T are
//     the agents adjacent to T (or T's occupant, for a stay); the requester
//     with the smallest index owns T and resolves it, which is the order the
//     dict would visit it in;
//   * RNG order: Philox draws are keyed by (t, env, agent | owner, purpose),
//     so order is irrelevant; MT mode (reference replay) serialises the draws
//     per env in exactly the reference's order (one lane per env, LDS state).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "kernels.h"

namespace ffm {

// ---------------------------------------------------------------------------
// decide(): candidate test, exit forcing, softmax and choice for one agent.
// Candidates are kept in fixed slots (neighbour order, stay last) with a
// validity mask instead of a compacted list, so every register index is static.
// ---------------------------------------------------------------------------
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

template <int NB>
__device__ __forceinline__ float sum_f32(const float (&e)[NB + 1], const bool (&v)[NB + 1], int nc) {
    // NumPy add.reduce: left fold below 8 elements, 8-lane pairwise at >= 8.
    if (NB == 8 && nc >= 8) {
        int q = NB + 1;  // slot of the (at most one) invalid neighbour
#pragma unroll
        for (int s = NB - 1; s >= 0; s--)
            if (!v[s]) q = s;
        float a[8];
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = (j < q) ? e[j] : e[j + 1];
        float res = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        if (nc == 9) res += e[8];
        return res;
    }
    float res = -0.0f;
#pragma unroll
    for (int s = 0; s <= NB; s++)
        if (v[s]) res += e[s];
    return res;
}

template <int NB>
__device__ __forceinline__ double sum_f64(const double (&e)[NB + 1], const bool (&v)[NB + 1], int nc) {
    if (NB == 8 && nc >= 8) {
        int q = NB + 1;
#pragma unroll
        for (int s = NB - 1; s >= 0; s--)
            if (!v[s]) q = s;
        double a[8];
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = (j < q) ? e[j] : e[j + 1];
        double res = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        if (nc == 9) res += e[8];
        return res;
    }
    double res = -0.0;
#pragma unroll
    for (int s = 0; s <= NB; s++)
        if (v[s]) res += e[s];
    return res;
}

template <int NB, bool F64, class Draw>
__device__ __forceinline__ uint32_t decide(int x, int y, int W, const uint8_t* smap, const float* ssff32,
                                           const double* ssff64, const float* sdff, const uint16_t* socc,
                                           float kS32, float kD32, double kS64, const Draw& draw) {
    int cell[NB + 1];
    bool v[NB + 1];
    int nvalid = 0;
    int exit_cell = -1;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        const int c = (x + nb_dx<NB>(s)) * W + (y + nb_dy<NB>(s));
        cell[s] = c;
        const uint8_t m = smap[c];
        const bool ok = (m == 0 || m == 3) && socc[c] == kEmpty;      // :52-60
        v[s] = ok;
        nvalid += ok ? 1 : 0;
        if (ok && m == 3 && exit_cell < 0) exit_cell = c;           // :66-72
    }
    if (nvalid == 0) return kNoReq;                                  // :63
    if (exit_cell >= 0) return (uint32_t)exit_cell;
    cell[NB] = x * W + y;                                            // :64 stay
    v[NB] = true;
    const int nc = nvalid + 1;

    double cdf[NB + 1];
    double last;
    if (!F64) {
        float s[NB + 1], e[NB + 1];
        float mx = -__builtin_inff();
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            const float a = kS32 * ssff32[cell[k]];
            const float b = kD32 * sdff[cell[k]];
            s[k] = a + b;                                            // :77
            if (v[k]) mx = s[k] > mx ? s[k] : mx;                    // :78
        }
#pragma unroll
        for (int k = 0; k <= NB; k++) e[k] = v[k] ? np_expf(s[k] - mx) : 0.0f;   // :80
        const float sum = sum_f32<NB>(e, v, nc);                                 // :81
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            if (v[k]) acc += (double)(e[k] / sum);                   // :83 + cumsum in choice
            cdf[k] = acc;
        }
        last = acc;
    } else {
        double s[NB + 1], e[NB + 1];
        double mx = -__builtin_inf();
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            const float b = kD32 * sdff[cell[k]];
            s[k] = kS64 * ssff64[cell[k]] + (double)b;
            if (v[k]) mx = s[k] > mx ? s[k] : mx;
        }
#pragma unroll
        for (int k = 0; k <= NB; k++) e[k] = v[k] ? exp(s[k] - mx) : 0.0;
        const double sum = sum_f64<NB>(e, v, nc);
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k <= NB; k++) {
            if (v[k]) acc += e[k] / sum;
            cdf[k] = acc;
        }
        last = acc;
    }
    const double u = draw.get();                                     // :84
    if (u < 0.0) return kPending;
    // np.random.choice: cdf /= cdf[-1]; searchsorted(u, side="right")
    uint32_t target = (uint32_t)cell[NB];
    bool found = false;
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        if (v[k] && !found && cdf[k] / last > u) {
            found = true;
            target = (uint32_t)cell[k];
        }
    }
    return target;
}

// ---------------------------------------------------------------------------
// Requesters of target r: the agents adjacent to r whose request is r.
// Returns m = number of requesters, sets owner (smallest index) and, for
// rank k, the k-th smallest requester in *sel.
// ---------------------------------------------------------------------------
template <int NB>
__device__ __forceinline__ int requesters(int r, int H, int W, const uint16_t* socc, const uint16_t* sreq,
                                          uint16_t (&who)[NB], bool (&is)[NB]) {
    const int rx = r / W, ry = r - (r / W) * W;
    int m = 0;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        const int cx = rx - nb_dx<NB>(s), cy = ry - nb_dy<NB>(s);
        bool ok = false;
        uint16_t j = kEmpty;
        if (cx >= 0 && cx < H && cy >= 0 && cy < W) {
            j = socc[cx * W + cy];
            ok = (j != kEmpty) && sreq[j] == (uint16_t)r;
        }
        who[s] = j;
        is[s] = ok;
        m += ok ? 1 : 0;
    }
    return m;
}

template <int NB>
__device__ __forceinline__ uint16_t kth_requester(const uint16_t (&who)[NB], const bool (&is)[NB], int k) {
    uint16_t sel = kEmpty;
#pragma unroll
    for (int s = 0; s < NB; s++) {
        int rank = 0;
#pragma unroll
        for (int q = 0; q < NB; q++) rank += (is[q] && who[q] < who[s]) ? 1 : 0;
        if (is[s] && rank == k) sel = who[s];
    }
    return sel;
}

// ---------------------------------------------------------------------------
// LDS carve-up, shared by host (size) and device (pointers).
// ---------------------------------------------------------------------------
__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

struct Carve {
    size_t map, sff, dff, occ, pos, req, nxt, misc, mt, u, flag, total;
};

__host__ __device__ inline Carve carve(int HW, int A, int K, bool f64, bool mt) {
    Carve c;
    size_t o = 0;
    c.map = o;  o += align16((size_t)HW);
    c.sff = o;  o += align16((size_t)HW * (f64 ? 8 : 4));
    c.dff = o;  o += align16((size_t)K * HW * 4);
    c.occ = o;  o += align16((size_t)K * HW * 2);
    c.pos = o;  o += align16((size_t)K * A * 2);
    c.req = o;  o += align16((size_t)K * A * 2);
    c.nxt = o;  o += align16((size_t)K * A * 2);
    c.misc = o; o += align16((size_t)(8 * K + 64) * 4);
    c.mt = o;   o += mt ? align16((size_t)K * 2 * 625 * 4) : 0;
    c.u = o;    o += mt ? align16((size_t)K * A * 8) : 0;
    c.flag = o; o += mt ? align16((size_t)K * A * 2) : 0;
    c.total = o;
    return c;
}

size_t core_step_smem_bytes(int HW, int A, int K, bool f64, bool mt) { return carve(HW, A, K, f64, mt).total; }

// ---------------------------------------------------------------------------
// The fused step kernel.
// ---------------------------------------------------------------------------
template <int NB, bool F64, bool MT, int BS>
__global__ __launch_bounds__(BS) void core_step_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int H = a.H, W = a.W, HW = a.HW, A = a.A;
    const long long e0 = (long long)blockIdx.x * a.K;
    const int K = (int)((a.E - e0) < a.K ? (a.E - e0) : a.K);
    const Carve cv = carve(HW, A, a.K, F64, MT);
    uint8_t* smap = smem + cv.map;
    float* ssff32 = reinterpret_cast<float*>(smem + cv.sff);
    double* ssff64 = reinterpret_cast<double*>(smem + cv.sff);
    float* sdff = reinterpret_cast<float*>(smem + cv.dff);
    uint16_t* socc = reinterpret_cast<uint16_t*>(smem + cv.occ);
    uint16_t* spos = reinterpret_cast<uint16_t*>(smem + cv.pos);
    uint16_t* sreq = reinterpret_cast<uint16_t*>(smem + cv.req);
    uint16_t* snxt = reinterpret_cast<uint16_t*>(smem + cv.nxt);
    int* scnt = reinterpret_cast<int*>(smem + cv.misc);        // [K] count at step start
    int* snew = scnt + a.K;                                     // [K] count after exits
    int* sreset = snew + a.K;                                   // [K] reset flag
    int* sseg = sreset + a.K;                                   // [K] segment base of the scan
    int* swsum = sseg + a.K;                                    // [BS/64] wave sums

    const int nitems_a = K * A;
    const int nitems_c = K * HW;

    // ---- load shared inputs and this block's env state ----------------------
    for (int i = tid; i < HW; i += BS) {
        smap[i] = a.map[i];
        if (F64) ssff64[i] = reinterpret_cast<const double*>(a.sff)[i];
        else ssff32[i] = reinterpret_cast<const float*>(a.sff)[i];
    }
    {
        const float* g = a.dff + e0 * HW;
        if ((HW & 3) == 0) {
            const float4* g4 = reinterpret_cast<const float4*>(g);
            float4* s4 = reinterpret_cast<float4*>(sdff);
            for (int i = tid; i < nitems_c / 4; i += BS) s4[i] = g4[i];
        } else {
            for (int i = tid; i < nitems_c; i += BS) sdff[i] = g[i];
        }
        const uint16_t* gp = a.pos + e0 * A;
        for (int i = tid; i < nitems_a; i += BS) spos[i] = gp[i];
        for (int i = tid; i < nitems_c; i += BS) socc[i] = kEmpty;
    }
    if (tid < K) {
        const int c = a.cnt[e0 + tid];
        const bool rs = a.auto_reset && c == 0;
        sreset[tid] = rs ? 1 : 0;
        scnt[tid] = rs ? a.N : c;
    }
    if (MT) {
        uint32_t* smt = reinterpret_cast<uint32_t*>(smem + cv.mt);
        for (int i = tid; i < K * 625; i += BS) {
            const int k = i / 625, w = i - k * 625;
            smt[k * 1250 + w] = a.mt_np[(e0 + k) * 625 + w];
            smt[k * 1250 + 625 + w] = a.mt_py[(e0 + k) * 625 + w];
        }
    }
    __syncthreads();

    // ---- on-device auto-reset (Philox): partial Fisher-Yates over the free list
    if (!MT && a.auto_reset) {
        bool any = false;
        for (int k = 0; k < K; k++) any |= sreset[k] != 0;
        if (any) {
            for (int i = tid; i < K * a.F; i += BS) {
                const int k = i / a.F, j = i - k * a.F;
                if (sreset[k]) socc[k * HW + j] = a.free_list[j];   // scratch: free list copy
            }
            for (int i = tid; i < nitems_c; i += BS)
                if (sreset[i / HW]) sdff[i] = 0.0f;
            __syncthreads();
            if (tid < K && sreset[tid]) {
                uint16_t* sc = socc + tid * HW;
                uint16_t* p = spos + tid * A;
                PhiloxStream ps(a.key0, a.key1, a.t, (uint32_t)(a.env_base + e0 + tid), 0u, kPurReset);
                for (int s = 0; s < a.N; s++) {
                    const uint32_t j = (uint32_t)s + ps.randbelow((uint32_t)(a.F - s));
                    const uint16_t tmp = sc[s];
                    sc[s] = sc[j];
                    sc[j] = tmp;
                    p[s] = sc[s];
                }
            }
            __syncthreads();
            for (int i = tid; i < nitems_c; i += BS)
                if (sreset[i / HW]) socc[i] = kEmpty;
            __syncthreads();
        }
    }

    // ---- occupancy of the current positions -------------------------------
    for (int it = tid; it < nitems_a; it += BS) {
        const int k = it / A, i = it - k * A;
        if (i < scnt[k]) socc[k * HW + spos[it]] = (uint16_t)i;
        snxt[it] = spos[it];
        sreq[it] = kNoReq;
    }
    __syncthreads();

    // ---- decide (model/ffm_core.py:40-88) ----------------------------------
    for (int it = tid; it < nitems_a; it += BS) {
        const int k = it / A, i = it - k * A;
        if (i >= scnt[k]) continue;
        const int p = spos[it];
        const int x = p / W, y = p - (p / W) * W;
        uint32_t r;
        if (MT) {
            r = decide<NB, F64>(x, y, W, smap, ssff32, ssff64, sdff + k * HW, socc + k * HW, a.kS32, a.kD32,
                                a.kS64, DrawPending{});
        } else {
            const DrawPhilox d{a.key0, a.key1, a.t, (uint32_t)(a.env_base + e0 + k), (uint32_t)i};
            r = decide<NB, F64>(x, y, W, smap, ssff32, ssff64, sdff + k * HW, socc + k * HW, a.kS32, a.kD32,
                                a.kS64, d);
        }
        sreq[it] = (uint16_t)r;
    }
    __syncthreads();

    if (MT) {
        // Draws in agent order from the env's NumPy stream, then redo the choice.
        uint32_t* smt = reinterpret_cast<uint32_t*>(smem + cv.mt);
        double* su = reinterpret_cast<double*>(smem + cv.u);
        if (tid < K) {
            uint32_t* mt_np = smt + tid * 1250;
            for (int i = 0; i < scnt[tid]; i++)
                if (sreq[tid * A + i] == kPending) su[tid * A + i] = mt_u53(mt_np);
        }
        __syncthreads();
        for (int it = tid; it < nitems_a; it += BS) {
            const int k = it / A, i = it - k * A;
            if (i >= scnt[k] || sreq[it] != kPending) continue;
            const int p = spos[it];
            const int x = p / W, y = p - (p / W) * W;
            sreq[it] = (uint16_t)decide<NB, F64>(x, y, W, smap, ssff32, ssff64, sdff + k * HW, socc + k * HW,
                                                 a.kS32, a.kD32, a.kS64, DrawFixed{su[it]});
        }
        __syncthreads();
    }

    // ---- resolve (model/ffm_core.py:90-98) ----------------------------------
    if (MT) {
        // pass 1: owners publish their multiplicity; serial draws in owner order.
        uint16_t* sflag = reinterpret_cast<uint16_t*>(smem + cv.flag);
        for (int it = tid; it < nitems_a; it += BS) {
            const int k = it / A, i = it - k * A;
            sflag[it] = 0;
            if (i >= scnt[k]) continue;
            const int r = sreq[it];
            if (r == kNoReq || r == spos[it]) continue;
            uint16_t who[NB];
            bool is[NB];
            const int m = requesters<NB>(r, H, W, socc + k * HW, sreq + k * A, who, is);
            if (m >= 2 && kth_requester<NB>(who, is, 0) == i) sflag[it] = (uint16_t)m;
        }
        __syncthreads();
        uint32_t* smt = reinterpret_cast<uint32_t*>(smem + cv.mt);
        if (tid < K) {
            uint32_t* mt_np = smt + tid * 1250;
            uint32_t* mt_py = mt_np + 625;
            for (int i = 0; i < scnt[tid]; i++) {
                const int m = sflag[tid * A + i];
                if (m >= 2) {
                    const double u = mt_u53(mt_np);                         // np.random.rand()
                    const int kk = u < 0.5 ? (int)mt_randbelow(mt_py, (uint32_t)m) : -1;   // random.choice
                    sflag[tid * A + i] = (uint16_t)(kk >= 0 ? 0x100 | kk : 0x200);
                }
            }
        }
        __syncthreads();
    }
    for (int it = tid; it < nitems_a; it += BS) {
        const int k = it / A, i = it - k * A;
        if (i >= scnt[k]) continue;
        const int r = sreq[it];
        if (r == kNoReq) continue;
        float* dk = sdff + k * HW;
        if (r == spos[it]) {  // stay: the agent's own cell, nobody else can request it
            dk[r] += 1.0f;                                                    // :93
            continue;
        }
        uint16_t who[NB];
        bool is[NB];
        const int m = requesters<NB>(r, H, W, socc + k * HW, sreq + k * A, who, is);
        if (kth_requester<NB>(who, is, 0) != i) continue;   // not the owner
        uint16_t w = kEmpty;
        if (m == 1) {
            w = (uint16_t)i;
        } else if (MT) {
            const int f = reinterpret_cast<uint16_t*>(smem + cv.flag)[it];
            if (f & 0x100) w = kth_requester<NB>(who, is, f & 0xFF);
        } else {
            PhiloxStream ps(a.key0, a.key1, a.t, (uint32_t)(a.env_base + e0 + k), (uint32_t)i, kPurFriction);
            const double u = ps.next_u53();                                   // :95
            if (u < 0.5) w = kth_requester<NB>(who, is, (int)ps.randbelow((uint32_t)m));   // :96
        }
        if (w != kEmpty) {
            snxt[k * A + w] = (uint16_t)r;
            dk[spos[k * A + w]] += 1.0f;                                      // :98
        }
    }
    __syncthreads();

    // ---- exits: order-preserving compaction (model/ffm_core.py:100-102) ---------
    {
        const int lane = tid & 63, wave = tid >> 6;
        int carry = 0;
        for (int base = 0; base < nitems_a; base += BS) {
            const int it = base + tid;
            const int k = it / A, i = it - k * A;
            const bool live = it < nitems_a && i < scnt[k];
            const bool keep = live && smap[snxt[it]] != 3;
            const unsigned long long mask = __ballot(keep);
            const int lp = __popcll(mask & ((1ull << lane) - 1ull));
            if (lane == 0) swsum[wave] = __popcll(mask);
            __syncthreads();
            int wp = 0, tot = 0;
#pragma unroll
            for (int v = 0; v < BS / 64; v++) {
                const int c = swsum[v];
                wp += v < wave ? c : 0;
                tot += c;
            }
            const int excl = carry + wp + lp;
            if (it < nitems_a && i == 0) sseg[k] = excl;
            __syncthreads();
            if (it < nitems_a) {
                const int seg = sseg[k];
                if (keep) spos[k * A + (excl - seg)] = snxt[it];
                if (i == A - 1) snew[k] = excl + (keep ? 1 : 0) - seg;
            }
            carry += tot;
            __syncthreads();
        }
    }

    // ---- write agents back; counters ------------------------------------------
    {
        uint16_t* gp = a.pos + e0 * A;
        for (int i = tid; i < nitems_a; i += BS) gp[i] = spos[i];
        if (tid == 0) {
            unsigned long long steps = 0, exits = 0, resets = 0;
            for (int k = 0; k < K; k++) {
                steps += (unsigned long long)scnt[k];
                exits += (unsigned long long)(scnt[k] - snew[k]);
                resets += (unsigned long long)sreset[k];
            }
            atomicAdd(&a.counters[0], steps);
            atomicAdd(&a.counters[1], exits);
            if (resets) atomicAdd(&a.counters[2], resets);
            if (blockIdx.x == 0) atomicAdd(&a.counters[3], 1ull);
        }
        if (tid < K) {
            a.cnt[e0 + tid] = snew[tid];
            if (sreset[tid] && a.episodes) a.episodes[e0 + tid] += 1;
        }
        if (MT) {
            const uint32_t* smt = reinterpret_cast<const uint32_t*>(smem + cv.mt);
            for (int i = tid; i < K * 625; i += BS) {
                const int k = i / 625, w = i - k * 625;
                a.mt_np[(e0 + k) * 625 + w] = smt[k * 1250 + w];
                a.mt_py[(e0 + k) * 625 + w] = smt[k * 1250 + 625 + w];
            }
        }
    }

    // ---- update_dff (model/ffm_core.py:106-117) --------------------------------
    {
        float* g = a.dff + e0 * HW;
        for (int c = tid; c < nitems_c; c += BS) {
            const int k = c / HW, cell = c - k * HW;
            const int x = cell / W, y = cell - (cell / W) * W;
            const float* dk = sdff + k * HW;
            float acc = a.c0 * dk[cell];                          // :109  B = c0 * D
#pragma unroll
            for (int s = 0; s < NB; s++) {
                const int nx = x + nb_dx<NB>(s), ny = y + nb_dy<NB>(s);
                const float b = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? a.c0 * dk[nx * W + ny] : 0.0f;
                const float t = a.c1 * b;                         // :113
                acc = acc + t;
            }
            g[c] = acc < 1e-4f ? 0.0f : acc;                      // :116-117
        }
    }
}

// ---------------------------------------------------------------------------
// Reset every env: Philox partial Fisher-Yates over the free list (the same
// placement the step kernel's auto-reset performs), counts = N.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void core_reset_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* sc = reinterpret_cast<uint16_t*>(smem);
    const long long e = blockIdx.x;
    for (int j = threadIdx.x; j < a.F; j += 64) sc[j] = a.free_list[j];
    __syncthreads();
    uint16_t* p = a.pos + e * a.A;
    if (threadIdx.x == 0) {
        PhiloxStream ps(a.key0, a.key1, a.t, (uint32_t)(a.env_base + e), 0u, kPurReset);
        for (int s = 0; s < a.N; s++) {
            const uint32_t j = (uint32_t)s + ps.randbelow((uint32_t)(a.F - s));
            const uint16_t tmp = sc[s];
            sc[s] = sc[j];
            sc[j] = tmp;
        }
        a.cnt[e] = a.N;
    }
    __syncthreads();
    for (int s = threadIdx.x; s < a.N; s += 64) p[s] = sc[s];
}

hipError_t launch_core_reset(const CoreStepArgs& a, hipStream_t s) {
    const size_t smem = align16((size_t)(a.F > 0 ? a.F : 1) * 2);
    core_reset_kernel<<<dim3((unsigned)a.E), dim3(64), smem, s>>>(a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Standalone update_dff (FloorFieldModel.update_dff): src -> dst, per cell.
// ---------------------------------------------------------------------------
template <int NB>
__global__ __launch_bounds__(256) void update_dff_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                         long long total, int H, int W, float c0, float c1) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c >= total) return;
    const int HW = H * W;
    const long long e = c / HW;
    const int cell = (int)(c - e * HW);
    const int x = cell / W, y = cell - (cell / W) * W;
    const float* d = src + e * HW;
    float acc = c0 * d[cell];
#pragma unroll
    for (int s = 0; s < NB; s++) {
        const int nx = x + nb_dx<NB>(s), ny = y + nb_dy<NB>(s);
        const float b = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? c0 * d[nx * W + ny] : 0.0f;
        const float t = c1 * b;
        acc = acc + t;
    }
    dst[c] = acc < 1e-4f ? 0.0f : acc;
}

__global__ void np_expf_kernel(const float* __restrict__ x, float* __restrict__ y, long long n) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = np_expf(x[i]);
}

// ---------------------------------------------------------------------------
// Host launchers.
// ---------------------------------------------------------------------------
template <int NB, bool F64, bool MT>
static hipError_t launch_t(const CoreStepArgs& a, int block, hipStream_t s) {
    const long long nblk = (a.E + a.K - 1) / a.K;
    const size_t smem = carve(a.HW, a.A, a.K, F64, MT).total;
    if (block == 512) {
        core_step_kernel<NB, F64, MT, 512><<<dim3((unsigned)nblk), dim3(512), smem, s>>>(a);
    } else {
        core_step_kernel<NB, F64, MT, 256><<<dim3((unsigned)nblk), dim3(256), smem, s>>>(a);
    }
    return hipGetLastError();
}

hipError_t launch_core_step(const CoreStepArgs& a, int nb, bool f64, bool mt, int block, hipStream_t s) {
    if (nb == 4) {
        if (f64) return mt ? launch_t<4, true, true>(a, block, s) : launch_t<4, true, false>(a, block, s);
        return mt ? launch_t<4, false, true>(a, block, s) : launch_t<4, false, false>(a, block, s);
    }
    if (f64) return mt ? launch_t<8, true, true>(a, block, s) : launch_t<8, true, false>(a, block, s);
    return mt ? launch_t<8, false, true>(a, block, s) : launch_t<8, false, false>(a, block, s);
}

hipError_t launch_update_dff(const float* src, float* dst, long long E, int H, int W, int nb, float c0, float c1,
                             hipStream_t s) {
    const long long total = E * H * W;
    const unsigned nblk = (unsigned)((total + 255) / 256);
    if (nblk == 0) return hipSuccess;
    if (nb == 4) update_dff_kernel<4><<<nblk, 256, 0, s>>>(src, dst, total, H, W, c0, c1);
    else update_dff_kernel<8><<<nblk, 256, 0, s>>>(src, dst, total, H, W, c0, c1);
    return hipGetLastError();
}

hipError_t launch_np_expf(const float* x, float* y, long long n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    np_expf_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(x, y, n);
    return hipGetLastError();
}

}  // namespace ffm
