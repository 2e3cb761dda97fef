// core_lane.hip -- the production (Philox) ffm_core step for small envs, one
// wavefront per env pair, written for CDNA4 issue economy.
//
// One launch advances every env by one FloorFieldModel.step()
// (model/ffm_core.py:36-117 of SoraKurihara/FFM).  Same semantics and RNG
// definition as core_wave_kernel<.., MT=false, ..>, and the
// same LDS picture: a padded direction-coded occupancy grid and a zero-halo DFF
// tile per env.  What differs is how the work maps onto the wave:
//
//  * conflicts are settled by every requester for itself.  A moving agent reads
//    the four (eight) codes around its target, which give the number of
//    requesters m, its own rank k among them and the owner o (smallest index);
//    with m > 1 it reads the owner's two friction words and evaluates the
//    owner's draw (philox_friction, keyed by o as before).  It moves iff m == 1
//    or the draw picks rank k.  No owner scatters a winner, so there is no
//    next-position array and no per-target selection loop;
//  * every granted request deposits at the mover's own source cell
//    (model/ffm_core.py:91-98: dff[positions[i]] += 1, and a cell holds one
//    agent), so deposits never collide: one LDS float add each, no read-back;
//  * per-lane state (position, count, DFF slots) lives in registers from the
//    prefetch to the store; LDS holds only what other lanes gather;
//  * the stencil scales on the fly (B = c0 * D per operand, rounded exactly as
//    the reference's separate pass) instead of a scale pass over the tile;
//  * the per-agent code is nearly branch-free: decide evaluates every slot with
//    selects and only the rare exact-arithmetic fallback branches; LDS writes of
//    idle lanes are exec-masked (a shared dummy address would serialise them);
//  * the DFF tile has no halo columns, so consecutive lanes' float4 slots are
//    consecutive in LDS and the 16-B stage / stencil accesses are conflict free.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "core_common.h"
#include "kernels.h"
#include "lane_common.h"
#include "wave_reset.h"

#ifndef FFM_STAMPS
#define FFM_STAMPS 0   // diagnostic builds only: per-phase s_memtime cycle sums per wave
#endif
#if FFM_STAMPS
#define LSTAMP(k)                                                                          \
    do {                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                        \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        st[k] += t_ - tlast;                                                               \
        tlast = t_;                                                                        \
    } while (0)
#else
#define LSTAMP(k) \
    do {          \
    } while (0)
#endif

namespace ffm {

namespace {

struct LaneCarve {
    size_t grid, tile, words, keys, pend, per_wave;
};

// Per-wave LDS: two grids, two tiles, the 64 lanes' friction words, the placement
// keys, and the bitmask of envs this launch emptied (their placement is deferred to
// the end of the launch, where none of the step's registers are live: placing in the
// loop would set the kernel's register peak).  Bit 2 i + s = env s of the wave's
// i-th pair; the host keeps every wave at <= kLaneMaxPairs pairs.
constexpr int kLaneMaxPairs = 64;
constexpr int kLanePendWords = 2 * kLaneMaxPairs / 32;
__host__ __device__ inline LaneCarve lane_carve(int PHW, int TS, int F) {
    LaneCarve c;
    size_t o = 0;
    c.grid = o;  o += a16((size_t)(2 * PHW) * 2);
    c.tile = o;  o += a16((size_t)(2 * TS) * 4);
    c.words = o; o += 64 * 8;
    c.keys = o;  o += a16((size_t)(F > 0 ? F : 1) * 8);
    c.pend = o;  o += kLanePendWords * 4;
    c.per_wave = o;
    return c;
}

__host__ __device__ inline size_t lane_shared_bytes(int PHW, int F) {
    return a16((size_t)PHW) + a16((size_t)PHW * 4) + a16((size_t)(F > 0 ? F : 1) * 2);
}

}  // namespace

#ifndef FFM_LANE_PIPE
#define FFM_LANE_PIPE 0   // 1: the decide draws of the next pair are computed a pair ahead
#endif
#ifndef FFM_LANE_ABLATE
#define FFM_LANE_ABLATE 0   // diagnostic builds only: bit k replaces / skips one piece (tools/ab_core.sh)
#endif
// Minimum waves per SIMD asked of the register allocator.  The 12x12 Neumann build
// (BASELINE config 2) fits 7 (72 VGPRs, SGPR spills to VGPR lanes only, no scratch);
// forcing 7 on the others spills to scratch, so they keep the compiler's choice.
#ifndef FFM_LANE_WAVES
#define FFM_LANE_WAVES 7   // diagnostic builds may lower / raise the 12x12 Neumann occupancy ask
#endif
template <int NB, int HT>
constexpr int lane_waves() { return (NB == 4 && HT == 12) ? FFM_LANE_WAVES : 1; }

template <int NB, int HT, int WT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(lane_waves<NB, HT>(), 8)))
void core_lane_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = HT ? HT : a.H, W = WT ? WT : a.W;
    const int HW = H * W, PW = W + 2, PHW = (H + 2) * PW;
    const int TS = lane_tile_floats(H, W);
    const int A = a.A;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int sub = lane >> 5, al = lane & 31;

    const LaneCarve cv = lane_carve(PHW, TS, a.F);
    uint8_t* pmap = smem;
    float* psff = reinterpret_cast<float*>(smem + a16((size_t)PHW));
    uint16_t* pfree = reinterpret_cast<uint16_t*>(smem + a16((size_t)PHW) + a16((size_t)PHW * 4));
    unsigned char* wbase = smem + lane_shared_bytes(PHW, a.F) + (size_t)wv * cv.per_wave;
    uint16_t* grid = reinterpret_cast<uint16_t*>(wbase + cv.grid);
    float* const tile = reinterpret_cast<float*>(wbase + cv.tile);
    uint2* words = reinterpret_cast<uint2*>(wbase + cv.words);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(wbase + cv.keys);
    uint16_t* gk = grid + sub * PHW;

    // The lane's two float4 DFF slots: cells 4q..4q+3 of the pair (q = lane, lane + 64).
    int tb0 = -1, tb1 = -1;
    {
        const int c0 = 4 * lane, c1 = 4 * (lane + 64);
        if (c0 < 2 * HW) {
            const int s = c0 / HW, cell = c0 - s * HW, x = cell / W, y = cell - x * W;
            tb0 = s * TS + 4 + (x + 1) * W + y;
        }
        if (c1 < 2 * HW) {
            const int s = c1 / HW, cell = c1 - s * HW, x = cell / W, y = cell - x * W;
            tb1 = s * TS + 4 + (x + 1) * W + y;
        }
    }
    // A slot at a row start / end takes its left / right stencil operand from a zero
    // word (tile index 0) instead of the neighbouring row.
    const bool yl0 = tb0 >= 0 && ((tb0 - 4) % TS) % W == 0, yr0 = tb0 >= 0 && ((tb0 - 4) % TS) % W == W - 4;
    const bool yl1 = tb1 >= 0 && ((tb1 - 4) % TS) % W == 0, yr1 = tb1 >= 0 && ((tb1 - 4) % TS) % W == W - 4;
    // Which env each slot's cells belong to (for the reset zeroing): 0, 1 or 2 (none).
    const int zs0 = min((4 * lane) / HW, 2), zs1 = min((4 * (lane + 64)) / HW, 2);

    const int E32 = (int)a.E;                 // host-checked: E * H * W * 4 < 2^31
    const uint32_t ebase = (uint32_t)a.env_base;
    const int ngroups = (E32 + 1) / 2;
    const int wstride = (int)gridDim.x * 4;
    int g = (int)blockIdx.x * 4 + wv;

    // Per-lane byte offsets inside a pair (loop invariant); kOOB = no access.
    const int off_cnt = sub * 4;                       // past the pair's bytes when sub >= nenv
    const int off_d0 = 16 * lane;   // slot 1 is off_d0 + 1024 (the instruction offset)

    // Next pair's state in registers: count, position, the two DFF float4 slots.
    // Buffer loads: out-of-range lanes read 0, no lane branch.
    struct LaneState {
        float4 d0, d1;
        int pos, cnt;
    };
    auto load = [&](int gg, LaneState& st) {
        const int e0 = (gg < 0 ? 0 : gg) * 2;
        const int nenv = gg < 0 ? 0 : min(E32 - e0, 2);
        st.cnt = (int)__builtin_amdgcn_raw_buffer_load_b32(pair_rsrc(a.cnt + e0, nenv * 4), off_cnt, 0, 0);
        st.pos = (int)__builtin_amdgcn_raw_buffer_load_b16(pair_rsrc(a.pos + (long long)e0 * A, nenv * A * 2),
                                                           al < A ? (sub * A + al) * 2 : kOOB, 0, 0);
        const __amdgpu_buffer_rsrc_t rd = pair_rsrc(a.dff + (long long)e0 * HW, nenv * HW * 4);
        st.d0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, off_d0, 0, 0));
        st.d1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, off_d0 + 1024, 0, 0));
    };
    LaneState cur;
    load(g < ngroups ? g : -1, cur);

    for (int i = threadIdx.x; i < PHW; i += 256) {
        pmap[i] = a.pmap[i];
        psff[i] = reinterpret_cast<const float*>(a.psff)[i];
    }
    for (int i = threadIdx.x; i < a.F; i += 256) pfree[i] = a.free_padded[i];
    for (int i = lane; i < 2 * TS; i += 64) tile[i] = 0.0f;
    __syncthreads();
    // Two dropped stores, so that on every path into the loop head the two youngest
    // memory operations are stores (the compiler then waits for the loads with vmcnt(2),
    // not for the previous group's DFF stores).
    buf_st4(pair_rsrc(a.dff, 0), kOOB, make_float4(0.f, 0.f, 0.f, 0.f));
    buf_st4(pair_rsrc(a.dff, 0), kOOB, make_float4(0.f, 0.f, 0.f, 0.f));
    for (int i = lane; i < 2 * PHW; i += 64) grid[i] = pmap[i - (i / PHW) * PHW];
    wave_sync();

    unsigned c_steps = 0, c_exits = 0, c_resets = 0;
    const uint32_t mW = (uint32_t)(((1ull << 32) + (unsigned)W - 1) / (unsigned)W);   // x = c / W for c < 2^16

#if FFM_STAMPS
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
    float* const dk = tile + sub * TS;
    uint32_t* const pend = reinterpret_cast<uint32_t*>(wbase + cv.pend);
    if (lane < kLanePendWords) pend[lane] = 0u;
    const int g_first = g;
#if FFM_LANE_PIPE
    uint4 pbn = philox(make_uint4(a.t, ebase + (uint32_t)(g * 2 + sub), (uint32_t)al, kPurDecide << 28), a.key0, a.key1);
#endif
    for (int iter = 0; g < ngroups; g += wstride, iter++) {
        // ---- stage this pair's DFF (loaded by the previous iteration or the prologue) -----
        if (tb0 >= 0) *reinterpret_cast<float4*>(tile + tb0) = cur.d0;
        if (tb1 >= 0) *reinterpret_cast<float4*>(tile + tb1) = cur.d1;
        const int cnt = cur.cnt;
        const uint32_t cpos = (uint32_t)cur.pos;
        const int e0 = g * 2;
        const int nenv = min(E32 - e0, 2);
        const bool env_ok = sub < nenv;
        const uint32_t genv = ebase + (uint32_t)(e0 + sub);

        // ---- agent cell and occupancy mark ----------------------------------------------
        const bool live = env_ok && al < cnt;
        const int x = (int)__umulhi(cpos, mW);   // exact for cpos < 2^16
        const int y = (int)cpos - x * W;
        const int pp = live ? (x + 1) * PW + y + 1 : PW + 1;       // idle lanes: an in-bounds cell
        const int dd0 = 3 - (x + 1) * 2;                           // tile index = grid index + dd0 - 2/row
        uint16_t* const mine = gk + pp;
        if (live) *mine = (uint16_t)(DirCodes::kAgent | (uint32_t)al | (DirCodes::kNoDir << 8));
        {
            const int c0 = __builtin_amdgcn_readlane(cnt, 0), c1 = __builtin_amdgcn_readlane(cnt, 32);
            c_steps += (unsigned)(c0 + (nenv > 1 ? c1 : 0));
        }
        wave_sync();

        LSTAMP(0);
        // ---- decide (model/ffm_core.py:40-88) -------------------------------------------
#if FFM_LANE_PIPE
        const uint4 pb = pbn;
#else
        const uint4 pb = (FFM_LANE_ABLATE & 1)
                             ? make_uint4(genv * 2654435761u ^ (uint32_t)al * 40503u ^ a.t * 97u,
                                          genv ^ (uint32_t)al * 7919u, a.t * 31u ^ genv, (uint32_t)al ^ a.t)
                             : philox(make_uint4(a.t, genv, (uint32_t)al, kPurDecide << 28), a.key0, a.key1);
#endif
        words[lane] = make_uint2(pb.z, pb.w);   // the friction draw, if this agent owns a contested target
        bool to_exit = false;
        uint32_t slot = (FFM_LANE_ABLATE & 16) ? (uint32_t)NB
                                               : lane_decide<NB>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, pb.x, to_exit);
        slot = live ? slot : kNoReq;
        if (slot == kPending)   // u near a cdf boundary: the exact NumPy arithmetic decides
            slot = NB == 4 ? lane_decide_exact<NB>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, u53(pb.x, pb.y))
                           : lane_decide_exact_arr<NB>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, u53(pb.x, pb.y));
        // the request goes into the agent's own grid cell: direction code in the high byte
        if (live)
            *mine = (uint16_t)(DirCodes::kAgent | (uint32_t)al |
                               ((slot <= (uint32_t)NB ? slot : DirCodes::kNoDir) << 8));
        wave_sync();

        LSTAMP(1);
        // ---- resolve (model/ffm_core.py:90-98), by each requester ------------------------
        const int r = (int)slot_cell<NB>(slot, pp, PW);          // kNoReq passes through
        const bool req = slot <= (uint32_t)NB;
        const bool moving = req && r != pp;
        bool granted = req && !moving;                            // a stay is always granted
        {
            const int rt = moving ? r : pp;                       // in-bounds for every lane
            int m = 0, k = 0, o = 0x7F;
#pragma unroll
            for (int s = 0; s < NB; s++) {
                const uint32_t c = gk[rt - nb_dx<NB>(s) * PW - nb_dy<NB>(s)];
                const bool is = (c & DirCodes::kAgent) != 0u && ((c >> 8) & 0xFu) == (uint32_t)s;
                const int who = (int)(c & DirCodes::kIdx);
                m += is ? 1 : 0;
                k += (is && who < al) ? 1 : 0;
                o = (is && who < o) ? who : o;
            }
            if (moving) {
                if ((FFM_LANE_ABLATE & 8) || m == 1) {
                    granted = true;
                } else {
                    const uint2 f = words[sub * 32 + o];
                    const int kk = philox_friction(f.x, f.y, (uint32_t)m, a.key0, a.key1, a.t, genv, (uint32_t)o);
                    granted = kk == k;                                 // :95-96
                }
            }
        }
        // :91-98 -- the mover's source cell gains 1 (one agent per cell: no collisions)
        if (granted) __hip_atomic_fetch_add(dk + pp + dd0, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const int np = granted ? r : pp;

        LSTAMP(2);
        // ---- exits: order-preserving compaction (model/ffm_core.py:100-102) ---------------
        const bool keep = live && !(granted && to_exit);
        const unsigned long long km = __ballot(keep);
        const unsigned long long segm = sub ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
        const int newidx = lanes_below(km & segm);
        const int newcnt = __popcll(km & segm);
        {
            const int n0 = __popcll(km & 0xFFFFFFFFull), n1 = __popcll(km >> 32);
            const int c0 = __builtin_amdgcn_readlane(cnt, 0), c1 = __builtin_amdgcn_readlane(cnt, 32);
            c_exits += (unsigned)((c0 - n0) + (nenv > 1 ? c1 - n1 : 0));
        }
        if (live) *mine = 0;   // unmark: agents only ever stand on free cells
        const bool rs = a.auto_reset && env_ok && newcnt == 0;
        const unsigned long long rsm = __ballot(rs);
        c_resets += (unsigned)(((rsm & 1ull) ? 1 : 0) + ((rsm >> 32) & 1ull ? 1 : 0));
        wave_sync();

        LSTAMP(3);
        // ---- positions and counts; auto-reset (rare, wave-uniform) -------
        // Before the next group's loads are issued, so that the reset's registers and the
        // prefetched state are never live together.
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)unpad(np, PW), pair_rsrc(a.pos + (long long)e0 * A, nenv * A * 2),
                                              keep ? (sub * A + newidx) * 2 : kOOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)(rs ? a.N : newcnt), pair_rsrc(a.cnt + e0, nenv * 4),
                                              al == 0 ? off_cnt : kOOB, 0, 0);
        if (rsm) {   // wave-uniform, rare
            if (a.episodes && al == 0 && rs) a.episodes[e0 + sub] += 1;
            const uint32_t bits = (uint32_t)((rsm & 1ull) | (((rsm >> 32) & 1ull) << 1)) << ((2 * iter) & 31);
            if (lane == 0) pend[(2 * iter) >> 5] |= bits;
        }

        LSTAMP(4);
        // ---- next group's HBM loads, in flight across the stencil, the stores and the
        // next group's head ------------------------------------------------------------
        LaneState nxt;
        load(g + wstride < ngroups ? g + wstride : -1, nxt);
#if FFM_LANE_PIPE
        // the next pair's decide draws: counter-based, so they need no state of this step
        pbn = philox(make_uint4(a.t, ebase + (uint32_t)((g + wstride) * 2 + sub), (uint32_t)al, kPurDecide << 28),
                     a.key0, a.key1);
#endif

        LSTAMP(5);
        // ---- update_dff (model/ffm_core.py:106-117): B = c0 * D, A = B + sum c1 * B[nb] -----
        auto stencil = [&](int tb, bool yl, bool yr, float4& out) {
            const float* p = tile + tb;
            float b[3][6];   // rows dx = -1..1, columns -1..4 (B values)
#pragma unroll
            for (int dx = -1; dx <= 1; dx++) {
                const float4 u = *reinterpret_cast<const float4*>(p + dx * W);
                b[dx + 1][1] = a.c0 * u.x; b[dx + 1][2] = a.c0 * u.y;
                b[dx + 1][3] = a.c0 * u.z; b[dx + 1][4] = a.c0 * u.w;
                if (NB == 4 && dx != 0) continue;
                b[dx + 1][0] = a.c0 * tile[yl ? 0 : tb + dx * W - 1];   // tile[0] == 0
                b[dx + 1][5] = a.c0 * tile[yr ? 0 : tb + dx * W + 4];
            }
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float acc = b[1][j + 1];
#pragma unroll
                for (int s = 0; s < NB; s++) {
                    const float t = a.c1 * b[1 + nb_dx<NB>(s)][j + 1 + nb_dy<NB>(s)];   // :113
                    acc = acc + t;
                }
                o[j] = acc < 1e-4f ? 0.0f : acc;                                       // :116-117
            }
            out = make_float4(o[0], o[1], o[2], o[3]);
        };
        float4 o0 = make_float4(0.f, 0.f, 0.f, 0.f), o1 = o0;
        if (tb0 >= 0) stencil(tb0, yl0, yr0, o0);
        if (!(FFM_LANE_ABLATE & 2) && tb1 >= 0) stencil(tb1, yl1, yr1, o1);

        LSTAMP(6);
        // ---- DFF stores (an env reset this step starts its next episode with a zero DFF) --
        {
            const __amdgpu_buffer_rsrc_t rd = pair_rsrc(a.dff + (long long)e0 * HW, nenv * HW * 4);
            const bool r0 = (rsm & 1ull) != 0, r1 = (rsm >> 32) != 0;   // wave-uniform
            const bool z0 = zs0 == 0 ? r0 : (zs0 == 1 && r1), z1 = zs1 == 0 ? r0 : (zs1 == 1 && r1);
            o0.x = z0 ? 0.f : o0.x; o0.y = z0 ? 0.f : o0.y; o0.z = z0 ? 0.f : o0.z; o0.w = z0 ? 0.f : o0.w;
            o1.x = z1 ? 0.f : o1.x; o1.y = z1 ? 0.f : o1.y; o1.z = z1 ? 0.f : o1.z; o1.w = z1 ? 0.f : o1.w;
            buf_st4(rd, off_d0, o0);
            buf_st4(rd, off_d0 + 1024, o1);
        }
        wave_sync();
        LSTAMP(7);
        cur = nxt;
    }

    // ---- deferred auto-reset placements ------------------------------
    wave_sync();
    for (int w = 0; w < kLanePendWords; w++) {
        uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend[w]);
        while (m) {
            const int bit = w * 32 + __builtin_ctz(m);
            m &= m - 1u;
            const int e = (g_first + (bit >> 1) * wstride) * 2 + (bit & 1);
            if (!(FFM_LANE_ABLATE & 64)) wave_reset_env(a, ebase + (uint32_t)e, keys, pfree, a.pos + (long long)e * A, lane);
        }
    }

    if (lane == 0) {
#if FFM_STAMPS
        if (a.dbg) {
            for (int k = 0; k < 8; k++) atomicAdd(&a.dbg[k], st[k]);
            atomicAdd(&a.dbg[8], 1ull);
        }
#endif
        unsigned long long* ctr = a.counters + 4 * ((size_t)blockIdx.x * 4 + wv);
        if (c_steps) atomicAdd(&ctr[0], (unsigned long long)c_steps);
        if (c_exits) atomicAdd(&ctr[1], (unsigned long long)c_exits);
        if (c_resets) atomicAdd(&ctr[2], (unsigned long long)c_resets);
        if (blockIdx.x == 0 && wv == 0) atomicAdd(&ctr[3], 1ull);
    }
}

size_t core_lane_smem_bytes(int H, int W, int F, int waves) {
    const int PHW = (H + 2) * (W + 2);
    return lane_shared_bytes(PHW, F) + (size_t)waves * lane_carve(PHW, lane_tile_floats(H, W), F).per_wave;
}

template <int NB, int HT, int WT>
static hipError_t lane_op(const CoreStepArgs& a, int blocks, hipStream_t s, int op, int* occ) {
    const size_t smem = core_lane_smem_bytes(a.H, a.W, a.F, 4);
    if (!op && ((a.E + 1) / 2 + (long long)blocks * 4 - 1) / ((long long)blocks * 4) > kLaneMaxPairs)
        return hipErrorInvalidConfiguration;   // the grid must give every wave <= kLaneMaxPairs pairs
    if (op) {
        *occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, core_lane_kernel<NB, HT, WT>, 256, smem) != hipSuccess)
            *occ = 0;
        return hipSuccess;
    }
    core_lane_kernel<NB, HT, WT><<<dim3((unsigned)blocks), dim3(256), smem, s>>>(a);
    return hipGetLastError();
}

static hipError_t lane_dispatch(const CoreStepArgs& a, int nb, int blocks, hipStream_t s, int op, int* occ) {
    if (a.H == 12 && a.W == 12)
        return nb == 4 ? lane_op<4, 12, 12>(a, blocks, s, op, occ) : lane_op<8, 12, 12>(a, blocks, s, op, occ);
    return nb == 4 ? lane_op<4, 0, 0>(a, blocks, s, op, occ) : lane_op<8, 0, 0>(a, blocks, s, op, occ);
}

hipError_t launch_core_lane(const CoreStepArgs& a, int nb, int blocks, hipStream_t s) {
    return lane_dispatch(a, nb, blocks, s, 0, nullptr);
}

int core_lane_max_pairs_per_wave() { return kLaneMaxPairs; }

int core_lane_blocks_per_cu(const CoreStepArgs& a, int nb) {
    int n = 0;
    (void)lane_dispatch(a, nb, 0, nullptr, 1, &n);
    return n;
}

}  // namespace ffm
