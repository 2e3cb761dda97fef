// core_group.hip -- the production (Philox) ffm_core step for the small-room
// configs (12x12, A <= 32), with the live agents of G envs packed densely into
// the lanes of one wavefront.
//
// One launch advances every env by one FloorFieldModel.step()
// (model/ffm_core.py:36-117 of SoraKurihara/FFM), with the RNG definition and
// the semantics of core_lane_kernel and the same LDS
// picture per env: a padded direction-coded occupancy grid and a zero-halo DFF
// tile.  The lane kernel gives every env a fixed half-wave of 32 agent lanes and
// every pair a second DFF slot that only 8 lanes fill.  On MI355X that kernel is
// instruction-issue bound (occupancy 4..7 waves/SIMD all run within 2 %, and
// the waves' summed active-instruction cycles equal the kernel's wall time),
// and at steady state half its agent lanes are idle (16.9 of 32 agents live per
// env).  Here one wave steps a group of G consecutive envs per iteration:
//
//  * the group's cnt / pos / DFF rows are contiguous in HBM; the DFF streams as
//    ceil(G * HW / 256) float4 slots per lane (G = 8 at 12x12: 4.5 slots, 90 %
//    of the lanes busy, against 56 % in the lane kernel);
//  * the live agents of the G envs are concatenated in env order and packed 64
//    to a chunk: packed index j = 64 c + lane belongs to env s with
//    S[s] <= j < S[s+1] (S = exclusive prefix of the counts, wave-uniform);
//    chunks = ceil(live / 64), about 2.6 per 8 envs at steady state against
//    4 half-empty pair iterations;
//  * every phase (mark, decide, resolve, compaction) loops over the chunks, so
//    every agent of every env has decided before any resolves: the phases are
//    separated exactly as in the lane kernel;
//  * the order-preserving exit compaction (model/ffm_core.py:100-102) works on
//    the packed order: the exclusive kept-prefix of every packed index goes to
//    LDS, an agent's new index is its prefix minus the prefix at its env's
//    start, an env's new count the difference of the prefixes at its bounds;
//  * the owner's friction bit (the top bit of its Philox word z) rides in bit 12
//    of its grid code, so the shared friction words are one dword per agent.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "core_common.h"
#include "kernels.h"
#include "lane_common.h"
#include "wave_reset.h"

namespace ffm {

namespace {

// Deferred auto-reset placements: 8 bits per group iteration (env s of the wave's
// i-th group = bit 8 i + s), so a wave steps at most kGroupMaxIters groups.
constexpr int kGroupMaxIters = 16;
constexpr int kGroupPendWords = 8 * kGroupMaxIters / 32;

struct GroupCarve {
    size_t grid, tile, words, posst, kp, keys, pend, dummy, per_wave;
};

// The staged positions are dead once the agents are marked, so the kept-prefix
// array reuses them; the placement keys are used only after the step loop, so
// they reuse the grids and tiles.
template <int G>
__host__ __device__ inline GroupCarve group_carve(int PHW, int TS, int F) {
    GroupCarve c;
    size_t o = 0;
    c.grid = o;  o += a16((size_t)G * PHW * 2);
    c.tile = o;  o += a16((size_t)G * TS * 4);
    c.keys = 0;
    const size_t keys_end = a16((size_t)(F > 0 ? F : 1) * 8);
    if (o < keys_end) o = keys_end;
    c.words = o; o += (size_t)G * 32 * 4;
    c.posst = o;
    // the compaction writes an entry for every lane of every agent chunk (idle lanes too: no
    // exec-mask branch), so the array spans whole chunks: (G * 32 + 63) / 64 * 64 + 1 entries
    c.kp = o;    o += a16((size_t)(((G * 32 + 63) / 64) * 64 + 1) * 2);
    c.pend = o;  o += kGroupPendWords * 4;
    c.dummy = o; o += 4;   // the target of the idle lanes' LDS writes (no exec-mask branch per write)
    c.per_wave = a16(o);
    return c;
}

// Block-shared: the map (u8), the staged SFF term (f32), the free-cell list (u16) and
// the map widened to the grid's u16 codes (each wave's grids are copied from it).
__host__ __device__ inline size_t group_shared_bytes(int PHW, int F) {
    return a16((size_t)PHW) + a16((size_t)PHW * 4) + a16((size_t)(F > 0 ? F : 1) * 2) + a16((size_t)PHW * 2);
}

// Packed per-chunk state (one VGPR each):
//   cs: pp (bits 0-15) | al (16-20) | s (21-23) | live (24) | x + 1 (25-31)
//   cr: slot (0-3, 15 = no request) | to_exit (4)          -- after decide
//       np (0-15) | keep (16) | kept prefix (17-26)         -- after resolve
__device__ __forceinline__ int cs_pp(uint32_t v) { return (int)(v & 0xFFFFu); }
__device__ __forceinline__ int cs_al(uint32_t v) { return (int)((v >> 16) & 31u); }
__device__ __forceinline__ int cs_s(uint32_t v) { return (int)((v >> 21) & 7u); }
__device__ __forceinline__ bool cs_live(uint32_t v) { return ((v >> 24) & 1u) != 0u; }
__device__ __forceinline__ int cs_xp1(uint32_t v) { return (int)(v >> 25); }

}  // namespace

#ifndef FFM_GROUP_PROBE_VALU
#define FFM_GROUP_PROBE_VALU 0   // diagnostic builds only
#endif
#ifndef FFM_GROUP_PROBE_SALU
#define FFM_GROUP_PROBE_SALU 0
#endif
#ifndef FFM_GROUP_PROBE_DUP
#define FFM_GROUP_PROBE_DUP 0
#endif

#ifndef FFM_GROUP_ABLATE
#define FFM_GROUP_ABLATE 0   // diagnostic builds only
#endif

#ifndef FFM_GROUP_TAIL
#define FFM_GROUP_TAIL 1    // the stencil's partial last slot, one cell per lane
#endif

// Skeleton ladder (diagnostic builds only; results invalid, timing only; profiles/r06/c2/):
//   0: the group loop streams the state in and stores it back unchanged (no prologue, no LDS)
//   1: + the block prologue (map / SFF term / free list staging, tile clears, grid init)
//   2: + the group staged in LDS and the DFF stencil (positions and counts stored back)
//   3: + count prefix, mark, unmark, compaction and stores (every agent stays: no decide,
//        no resolve)
//   4: the product kernel
#ifndef FFM_GROUP_LADDER
#define FFM_GROUP_LADDER 4
#endif

// Where the next group's HBM loads are issued (diagnostic A/B): 0 before the stencil, 1 after
// decide, 2 after mark, 3 right after the staging.
#ifndef FFM_GROUP_PF
#define FFM_GROUP_PF 0
#endif

// Waves that step fewer groups than the most loaded ones start late by s_sleep(N) (64 N
// clocks): their phases leave the others' (diagnostic A/B; 0 = off).
#ifndef FFM_GROUP_STAGGER
#define FFM_GROUP_STAGGER 0
#endif

#ifndef FFM_GROUP_WAVES
#define FFM_GROUP_WAVES 6   // minimum waves per SIMD asked of the register allocator (G = 4 needs 71 VGPRs; the grid holds 6 per SIMD)
#endif

template <int NB, int HT, int WT, int G, bool KD1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FFM_GROUP_WAVES, 8)))
void core_group_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int H = HT, W = WT, HW = H * W, PW = W + 2, PHW = (H + 2) * PW;
    constexpr int TS = lane_tile_floats(H, W);
    constexpr int Q4 = HW / 4;                 // float4s per env
    constexpr int Q = G * Q4;                  // float4s per group
    constexpr int NS = (Q + 63) / 64;          // float4 slots per lane (staging)
    constexpr int NSF = Q / 64;                // full float4 slots
    // a partial last slot of at most 16 float4s is stepped as one cell per lane instead
    // (G = 4 at 12x12: 144 float4s = 2 full slots + 64 cells), so its stencil keeps every
    // lane busy (Neumann only: the Moore stencil keeps the float4 form)
    constexpr bool SCALAR_TAIL = NB == 4 && FFM_GROUP_TAIL && Q % 64 != 0 && (Q % 64) * 4 == 64;
    constexpr int MAXC = (G * 32 + 63) / 64;   // agent chunks per group (A <= 32)
    constexpr int PWORDS = G * 16;             // position dwords per group (A <= 32)
    static_assert(G >= 1 && G <= 8 && HW % 4 == 0 && H + 1 < 128, "group geometry");
    static_assert(MAXC * 64 >= G * 32 && PWORDS * 4 <= (MAXC * 64 + 1) * 2, "kp spans the chunks; posst fits in it");
    const int A = a.A;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));

    const GroupCarve cv = group_carve<G>(PHW, TS, a.F);
    uint8_t* pmap = smem;
    float* psff = reinterpret_cast<float*>(smem + a16((size_t)PHW));
    uint16_t* pfree = reinterpret_cast<uint16_t*>(smem + a16((size_t)PHW) + a16((size_t)PHW * 4));
    uint16_t* pmap16 = reinterpret_cast<uint16_t*>(smem + a16((size_t)PHW) + a16((size_t)PHW * 4) +
                                                   a16((size_t)(a.F > 0 ? a.F : 1) * 2));
    unsigned char* wbase = smem + group_shared_bytes(PHW, a.F) + (size_t)wv * cv.per_wave;
    uint16_t* const grid = reinterpret_cast<uint16_t*>(wbase + cv.grid);
    float* const tile = reinterpret_cast<float*>(wbase + cv.tile);
    uint32_t* const words = reinterpret_cast<uint32_t*>(wbase + cv.words);
    uint32_t* const posst32 = reinterpret_cast<uint32_t*>(wbase + cv.posst);
    const uint16_t* const posst = reinterpret_cast<const uint16_t*>(wbase + cv.posst);
    uint16_t* const kp = reinterpret_cast<uint16_t*>(wbase + cv.kp);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(wbase + cv.keys);
    uint32_t* const pend = reinterpret_cast<uint32_t*>(wbase + cv.pend);
    const int kDummy16 = (int)((cv.dummy - cv.grid) / 2);    // grid index of the dummy word
    const int kDummy32 = (int)((cv.dummy - cv.words) / 4);   // words index of the dummy word

    // The lane's DFF float4 slots: q = 64 k + lane of the group's G * HW cells,
    // env q / Q4, cell 4 (q % Q4) of that env.
    int toff[NS];
    uint32_t yfl = 0, senv = 0;
#pragma unroll
    for (int k = 0; k < NS; k++) {
        const int q = k * 64 + lane;
        const int s = q / Q4, c = 4 * (q - s * Q4), y = c % W;
        toff[k] = q < Q ? s * TS + 4 + W + c : -1;
        yfl |= (q < Q && y == 0 ? 1u : 0u) << (2 * k);
        yfl |= (q < Q && y == W - 4 ? 2u : 0u) << (2 * k);
        senv |= (uint32_t)(q < Q ? s : 15) << (4 * k);
    }

    const long long E = a.E;                   // host-checked: (E + 7) * HW * 4 < 2^31
    const uint32_t ebase = (uint32_t)a.env_base;
    // Whole-array buffer resources, built once.  The engine pads pos / cnt / DFF to whole groups
    // of 8 envs (zeroed), so a partial last group reads zero counts and DFF and its stores land
    // in the padding; every access takes its group's byte base as the scalar offset, and lanes
    // past the group's bytes use kOOB (dropped).
    const int Epad = (int)((E + 7) & ~7LL);
    const __amdgpu_buffer_rsrc_t rC = pair_rsrc(a.cnt, Epad * 4);
    const __amdgpu_buffer_rsrc_t rP = pair_rsrc(a.pos, Epad * A * 2 + 4);   // + the dword of slack
    const __amdgpu_buffer_rsrc_t rD = pair_rsrc(a.dff, Epad * HW * 4);
    const int ngroups = (int)((E + G - 1) / G);
    const int wstride = (int)gridDim.x * 4;
    int g = (int)blockIdx.x * 4 + wv;

    struct GState {
        float4 d[NS];
        uint32_t p0, p1;
        int c;
    };
    // past the last group (the loop's final prefetch) the loads go through empty resources:
    // every lane's access is out of range, no bytes move, and no value is conditionally
    // defined (a `return` there cost 8-14 VGPRs)
    const __amdgpu_buffer_rsrc_t rZ = pair_rsrc(a.dff, 0);
    auto load = [&](int gg, GState& st) {
        const bool ok = gg >= 0;
        const int e0 = ok ? gg * G : 0;
        const __amdgpu_buffer_rsrc_t rc = ok ? rC : rZ, rp = ok ? rP : rZ, rd = ok ? rD : rZ;
        st.c = (int)__builtin_amdgcn_raw_buffer_load_b32(rc, lane < G ? lane * 4 : kOOB, e0 * 4, 0);
        st.p0 = __builtin_amdgcn_raw_buffer_load_b32(rp, lane < PWORDS ? lane * 4 : kOOB, e0 * A * 2, 0);
        st.p1 = PWORDS > 64 ? __builtin_amdgcn_raw_buffer_load_b32(rp, 64 + lane < PWORDS ? 256 + lane * 4 : kOOB,
                                                                 e0 * A * 2, 0)
                            : 0u;
#pragma unroll
        for (int k = 0; k < NS; k++) {
            const int q = k * 64 + lane;
            st.d[k] = __builtin_bit_cast(float4,
                                         __builtin_amdgcn_raw_buffer_load_b128(rd, q < Q ? q * 16 : kOOB, e0 * HW * 4, 0));
        }
    };
    constexpr int LAD = FFM_GROUP_LADDER;
    constexpr int PF = FFM_GROUP_PF;
    if (FFM_GROUP_STAGGER > 0) {
        const int mine = g < ngroups ? (ngroups - 1 - g) / wstride + 1 : 0;
        const int most = (ngroups - 1) / wstride + 1;
        if (mine < most) __builtin_amdgcn_s_sleep(FFM_GROUP_STAGGER);
    }
    GState cur;
    load(g < ngroups ? g : -1, cur);

    if (LAD >= 1) {
    for (int i = threadIdx.x; i < PHW; i += 256) {
        const uint8_t mv = a.pmap[i];
        pmap[i] = mv;
        pmap16[i] = mv;
        psff[i] = a.kS32 * reinterpret_cast<const float*>(a.psff)[i];   // the score's SFF term
    }
    for (int i = threadIdx.x; i < a.F; i += 256) pfree[i] = a.free_padded[i];
    static_assert((G * TS) % 4 == 0 && PHW % 2 == 0, "16-B tile clears, 4-B grid copies");
    for (int i = lane; i < G * TS / 4; i += 64) reinterpret_cast<float4*>(tile)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane < kGroupPendWords) pend[lane] = 0u;
    __syncthreads();
    // every env's grid starts as the map: dword copies of the widened map, no per-cell modulo
#pragma unroll
    for (int s = 0; s < G; s++)
        for (int i = lane; i < PHW / 2; i += 64)
            reinterpret_cast<uint32_t*>(grid)[s * (PHW / 2) + i] = reinterpret_cast<const uint32_t*>(pmap16)[i];
    wave_sync();
    }

    unsigned c_steps = 0, c_exits = 0, c_resets = 0;
    constexpr uint32_t mW = (uint32_t)(((1ull << 32) + (unsigned)W - 1) / (unsigned)W);   // x = c / W, c < 2^16
    const int g_first = g;
    for (int iter = 0; g < ngroups; g += wstride, iter++) {
        const int e0 = g * G;
        const int nenv = (int)min((long long)G, E - e0);
        if (LAD <= 2) {   // ladder rungs 0-2: positions and counts stored back unchanged
            const __amdgpu_buffer_rsrc_t rq = pair_rsrc(a.pos + e0 * A, (nenv * A * 2 + 3) & ~3);
            __builtin_amdgcn_raw_buffer_store_b32(cur.p0, rq, lane < PWORDS ? lane * 4 : kOOB, 0, 0);
            if (PWORDS > 64)
                __builtin_amdgcn_raw_buffer_store_b32(cur.p1, rq, 64 + lane < PWORDS ? 256 + lane * 4 : kOOB, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32((unsigned)cur.c, pair_rsrc(a.cnt + e0, nenv * 4),
                                                  lane < G ? lane * 4 : kOOB, 0, 0);
            c_steps += (unsigned)A * (unsigned)nenv;
        }
        if (LAD <= 1) {   // rungs 0-1: the DFF stored back from registers
            const __amdgpu_buffer_rsrc_t rq = pair_rsrc(a.dff + e0 * HW, nenv * HW * 4);
#pragma unroll
            for (int k = 0; k < NS; k++) {
                const int q = k * 64 + lane;
                buf_st4(rq, q < Q ? q * 16 : kOOB, cur.d[k]);
            }
            GState nx;
            load(g + wstride < ngroups ? g + wstride : -1, nx);
            cur = nx;
            continue;
        }

        GState nxt;
        const int gn = g + wstride < ngroups ? g + wstride : -1;
        // ---- stage the group (prefetched by the previous iteration or the prologue) -------
#pragma unroll
        for (int k = 0; k < NS; k++)
            if (k < NSF || toff[k] >= 0) *reinterpret_cast<float4*>(tile + toff[k]) = cur.d[k];
        if (PF == 3) load(gn, nxt);
        unsigned long long rsm = 0ull;   // envs re-placed at the end of this step
        if (LAD == 2) wave_sync();       // ladder rung 2: the staged tile before the stencil reads it
        if (LAD >= 3) {
        if (lane < PWORDS) posst32[lane] = cur.p0;
        if (PWORDS > 64 && 64 + lane < PWORDS) posst32[64 + lane] = cur.p1;
        int S[G + 1];   // exclusive prefix of the counts (wave-uniform)
        S[0] = 0;
#pragma unroll
        for (int s = 0; s < G; s++) S[s + 1] = S[s] + __builtin_amdgcn_readlane(cur.c, s);
        const int T = S[G];
        c_steps += (unsigned)T;
        wave_sync();

        // ---- packed agents: cell and occupancy mark ------------------------------------
        uint32_t cs[MAXC], cr[MAXC];
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            cs[c] = (uint32_t)(PW + 1) | (1u << 25);   // idle: an in-bounds cell
            cr[c] = 15u;
            if (c * 64 < T) {
                const int j = c * 64 + lane;
                int s = 0, st = 0;
#pragma unroll
                for (int q = 1; q < G; q++) {
                    const bool ge = j >= S[q];
                    s += ge ? 1 : 0;
                    st = ge ? S[q] : st;
                }
                const bool live = j < T;
                const int al = live ? j - st : 0;
                const uint32_t p = posst[live ? s * A + al : 0];
                const int x = (int)__umulhi(p, mW);
                const int y = (int)p - x * W;
                const int pp = live ? (x + 1) * PW + y + 1 : PW + 1;
                grid[live ? s * PHW + pp : kDummy16] = (uint16_t)(DirCodes::kAgent | (uint32_t)al | (DirCodes::kNoDir << 8));
                cs[c] = (uint32_t)pp | ((uint32_t)al << 16) | ((uint32_t)s << 21) | ((live ? 1u : 0u) << 24) |
                        ((uint32_t)(live ? x + 1 : 1) << 25);
            }
        }
        wave_sync();

        if (PF == 2) load(gn, nxt);
        // ---- decide (model/ffm_core.py:40-88) -------------------------------------------
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            if (LAD == 3) cr[c] = DirCodes::kNoDir;   // ladder: every agent stays, no request
            if (LAD >= 4 && c * 64 < T) {
                const uint32_t v = cs[c];
                const int pp = cs_pp(v), al = cs_al(v), s = cs_s(v);
                const bool live = cs_live(v);
                const uint32_t genv = ebase + (uint32_t)e0 + (uint32_t)s;
                const uint4 pb = philox(make_uint4(a.t, genv, (uint32_t)al, kPurDecide << 28), a.key0, a.key1);
                words[live ? s * 32 + al : kDummy32] = pb.w;   // the friction draw, if this agent owns a contested target
                const uint16_t* gk = grid + s * PHW;
                const float* dk = tile + s * TS;
                const int dd0 = 3 - 2 * cs_xp1(v);
                bool to_exit = false;
                uint32_t slot = lane_decide<NB, true, KD1>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, pb.x, to_exit);
                slot = live ? slot : kNoReq;
                if (slot == kPending)   // u near a cdf boundary: the exact NumPy arithmetic decides
                    slot = NB == 4 ? lane_decide_exact<NB, true>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32,
                                                                 u53(pb.x, pb.y))
                                   : lane_decide_exact_arr<NB, true>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32,
                                                               u53(pb.x, pb.y));
                const uint32_t sd = slot <= (uint32_t)NB ? slot : DirCodes::kNoDir;
                grid[live ? s * PHW + pp : kDummy16] =
                    (uint16_t)(DirCodes::kAgent | (uint32_t)al | (sd << 8) | ((pb.z >> 31) << 12));
                cr[c] = sd | ((to_exit ? 1u : 0u) << 4);
#if FFM_GROUP_PROBE_DUP
                if (c == MAXC - 1) {   // diagnostic (timing only): the last chunk's draw and decide again
                    uint32_t salt;
                    asm volatile("v_mov_b32 %0, 0" : "=v"(salt));
                    const uint4 pb2 = philox(make_uint4(a.t, genv, (uint32_t)al + salt, kPurDecide << 28), a.key0,
                                             a.key1);
                    bool te2 = false;
                    const uint32_t slot2 =
                        lane_decide<NB, true, KD1>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, pb2.x, te2);
                    asm volatile("" ::"v"(slot2), "v"(pb2.w), "v"(te2 ? 1u : 0u));
                }
#endif
            }
        }
        wave_sync();

        if (PF == 1) load(gn, nxt);
        // ---- resolve (model/ffm_core.py:90-98), by each requester ------------------------
        unsigned long long km[MAXC];
        int kept = 0;
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            km[c] = 0ull;
            if (c * 64 < T) {
                const uint32_t v = cs[c];
                const int pp = cs_pp(v), al = cs_al(v), s = cs_s(v);
                const bool live = cs_live(v);
                const uint32_t sd = cr[c] & 15u;
                const bool to_exit = (cr[c] & 16u) != 0u;
                const uint32_t slot = sd == DirCodes::kNoDir ? (uint32_t)kNoReq : sd;
                const uint16_t* gk = grid + s * PHW;
                const int r = (int)slot_cell_k<NB, PW>(slot, pp);
                const bool req = slot <= (uint32_t)NB;
                const bool moving = req && r != pp;
                bool granted = req && !moving;   // a stay is always granted
                if (LAD >= 4) {
                    const int rt = moving ? r : pp;
                    int m = 0, k = 0, o = 0x7F;
                    uint32_t zo = 0u;
#pragma unroll
                    for (int d = 0; d < NB; d++) {
                        const uint32_t cc = gk[rt - nb_dx<NB>(d) * PW - nb_dy<NB>(d)];
                        const bool is = (cc & DirCodes::kAgent) != 0u && ((cc >> 8) & 0xFu) == (uint32_t)d;
                        const int who = (int)(cc & DirCodes::kIdx);
                        m += is ? 1 : 0;
                        k += (is && who < al) ? 1 : 0;
                        const bool lower = is && who < o;
                        zo = lower ? (cc >> 12) & 1u : zo;
                        o = lower ? who : o;
                    }
                    granted = moving ? m == 1 : granted;   // an uncontested move is granted
                    if (moving && m > 1) {
                        const uint32_t w = words[s * 32 + o];
                        const uint32_t genv = ebase + (uint32_t)e0 + (uint32_t)s;
                        const int kk = philox_friction(zo << 31, w, (uint32_t)m, a.key0, a.key1, a.t, genv,
                                                       (uint32_t)o);
                        granted = kk == k;   // :95-96
                    }
                }
                // :91-98 -- the mover's source cell gains 1 (one agent per cell: no collisions)
                if (granted)
                    __hip_atomic_fetch_add(tile + s * TS + pp + 3 - 2 * cs_xp1(v), 1.0f, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WAVEFRONT);
                const int np = granted ? r : pp;
                const bool keep = live && !(granted && to_exit);
                km[c] = __ballot(keep);
                const int kpv = kept + lanes_below(km[c]);
                kept += __popcll(km[c]);
                cr[c] = (uint32_t)np | ((keep ? 1u : 0u) << 16) | ((uint32_t)kpv << 17);
            }
        }

        // ---- exits: order-preserving compaction (model/ffm_core.py:100-102) ---------------
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            if (c * 64 < T) {
                const uint32_t v = cs[c];
                kp[c * 64 + lane] = (uint16_t)(cr[c] >> 17);   // idle lanes' entries are never read
                grid[cs_live(v) ? cs_s(v) * PHW + cs_pp(v) : kDummy16] = 0;   // unmark: agents stand on free cells
            }
        }
        if (lane == 0) kp[T] = (uint16_t)kept;
        c_exits += (unsigned)(T - kept);
        wave_sync();
#pragma unroll
        for (int c = 0; c < MAXC; c++) {
            if (c * 64 < T) {
                const uint32_t v = cs[c], w = cr[c];
                const int j = c * 64 + lane;
                const int s = cs_s(v);
                const bool keep = ((w >> 16) & 1u) != 0u;
                const int start = j - cs_al(v);
                const int newidx = (int)(w >> 17) - (int)kp[cs_live(v) ? start : 0];
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)unpad((int)(w & 0xFFFFu), PW), rP,
                                                      keep ? (s * A + newidx) * 2 : kOOB, e0 * A * 2, 0);
            }
        }
        int Sl = T, Sh = T;   // lane s < G: [S[s], S[s+1])
#pragma unroll
        for (int s = 0; s < G; s++) {
            Sl = lane == s ? S[s] : Sl;
            Sh = lane == s ? S[s + 1] : Sh;
        }
        const int nk = (int)kp[Sh] - (int)kp[Sl];
        const bool rs = a.auto_reset && lane < nenv && nk == 0;
        rsm = __ballot(rs);
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)(rs ? a.N : nk), rC, lane < G ? lane * 4 : kOOB, e0 * 4, 0);
        if (rsm) {   // wave-uniform, rare
            c_resets += (unsigned)__popcll(rsm);
            if (a.episodes && rs) a.episodes[e0 + lane] += 1;
            if (lane == 0) pend[iter >> 2] |= (uint32_t)rsm << (8 * (iter & 3));
        }
        }   // LAD >= 3

        // ---- next group's HBM loads, in flight across the stencil, the stores and the
        // next group's head ------------------------------------------------------------
        if (PF == 0 || LAD < 3) load(gn, nxt);

#if FFM_GROUP_PROBE_VALU > 0 || FFM_GROUP_PROBE_SALU > 0
        {   // diagnostic issue probes (timing only): N extra VALU / SALU instructions per group
            uint32_t pv = (uint32_t)lane, ps = (uint32_t)g;
#pragma unroll
            for (int i = 0; i < FFM_GROUP_PROBE_VALU; i++) asm volatile("v_add_u32 %0, %0, 1" : "+v"(pv));
#pragma unroll
            for (int i = 0; i < FFM_GROUP_PROBE_SALU; i++) asm volatile("s_add_u32 %0, %0, 1" : "+s"(ps));
            asm volatile("" ::"v"(pv), "s"(ps));
        }
#endif
        // ---- update_dff (model/ffm_core.py:106-117): B = c0 * D, A = B + sum c1 * B[nb],
        // then the DFF stores (an env reset this step starts its next episode at zero) ----
        if (SCALAR_TAIL) {     // the last, partial float4 slot as one cell per lane (all lanes busy)
            const int q = 4 * 64 * NSF + lane;                 // the group's cell
            const int s = q / HW, c = q - s * HW, y = c % W;
            const float* p = tile + s * TS + 4 + W + c;
            // p[-1] / p[1] lie inside the tile at the map's edges too (the zero rows above and
            // below): read them unconditionally, select the edge's zero (no exec-mask branch)
            const float m0 = p[0], mu = p[-W], md = p[W], pl = p[-1], pr = p[1];
            const float ml = y == 0 ? 0.0f : pl, mr = y == W - 1 ? 0.0f : pr;
            // B = c0 * D per operand, then A = B + sum c1 * B[nb] in neighbour order (:106-117)
            const float b0 = a.c0 * m0, bu = a.c0 * mu, bd = a.c0 * md, bl = a.c0 * ml, br = a.c0 * mr;
            float acc = b0;
            acc = acc + a.c1 * bu;
            acc = acc + a.c1 * bd;
            acc = acc + a.c1 * bl;
            acc = acc + a.c1 * br;
            float o = acc < 1e-4f ? 0.0f : acc;
            if (rsm && ((rsm >> s) & 1ull)) o = 0.0f;   // rsm wave-uniform and rare
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, o), rD, q * 4, e0 * HW * 4, 0);
        }
#pragma unroll
        for (int k = 0; k < (SCALAR_TAIL ? NSF : NS); k++) {
            const int tb = toff[k];
            if (k >= NSF && tb < 0) continue;
            const bool yl = ((yfl >> (2 * k)) & 1u) != 0u, yr = ((yfl >> (2 * k)) & 2u) != 0u;
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
            for (int jj = 0; jj < 4; jj++) {
                float acc = b[1][jj + 1];
#pragma unroll
                for (int d = 0; d < NB; d++) {
                    const float t = a.c1 * b[1 + nb_dx<NB>(d)][jj + 1 + nb_dy<NB>(d)];   // :113
                    acc = acc + t;
                }
                o[jj] = acc < 1e-4f ? 0.0f : acc;                                     // :116-117
            }
            float4 out = make_float4(o[0], o[1], o[2], o[3]);
            if (rsm) {   // wave-uniform, rare: an env re-placed this step starts its next episode at zero
                if ((rsm >> ((senv >> (4 * k)) & 15u)) & 1ull) out = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, out),
                                                   rD, (k * 64 + lane) * 16, e0 * HW * 4, 0);
        }
        wave_sync();
        cur = nxt;
    }

    // ---- deferred auto-reset placements ------------------------------
    wave_sync();
    for (int w = 0; w < (LAD >= 1 ? kGroupPendWords : 0); w++) {   // ladder rung 0: pend never initialised
        uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend[w]);
        while (m) {
            const int bit = w * 32 + __builtin_ctz(m);
            m &= m - 1u;
            const long long e = (long long)(g_first + (bit >> 3) * wstride) * G + (bit & 7);
            wave_reset_env(a, ebase + (uint32_t)e, keys, pfree, a.pos + e * A, lane);
            if (FFM_GROUP_ABLATE & 1)   // diagnostic: the same placement again (identical result)
                wave_reset_env(a, ebase + (uint32_t)e, keys, pfree, a.pos + e * A, lane);
        }
    }

    if (lane == 0) {
        unsigned long long* ctr = a.counters + 4 * ((size_t)blockIdx.x * 4 + wv);
        if (c_steps) atomicAdd(&ctr[0], (unsigned long long)c_steps);
        if (c_exits) atomicAdd(&ctr[1], (unsigned long long)c_exits);
        if (c_resets) atomicAdd(&ctr[2], (unsigned long long)c_resets);
        if (blockIdx.x == 0 && wv == 0) atomicAdd(&ctr[3], 1ull);
    }
}

#ifndef FFM_GROUP_G
#define FFM_GROUP_G 4
#endif
constexpr int kGroupG = FFM_GROUP_G;   // envs per group at large E
#ifndef FFM_GROUP_G_SMALL
#define FFM_GROUP_G_SMALL 2
#endif
constexpr int kGroupGSmall = FFM_GROUP_G_SMALL;   // envs per group when the large-E groups fill under half the waves

size_t core_group_smem_bytes(int H, int W, int F, int waves, int G) {
    const int PHW = (H + 2) * (W + 2);
    const size_t per_wave = G == kGroupGSmall ? group_carve<kGroupGSmall>(PHW, lane_tile_floats(H, W), F).per_wave
                                              : group_carve<kGroupG>(PHW, lane_tile_floats(H, W), F).per_wave;
    return group_shared_bytes(PHW, F) + (size_t)waves * per_wave;
}

bool core_group_supported(int H, int W) { return H == 12 && W == 12; }

int core_group_max_iters() { return kGroupMaxIters; }

// KD1: k_D == 1 (the drivers' setting), where k_D * DFF is DFF itself: a kernel of its own
// rather than a runtime flag, which the register allocator would keep (and spill) all launch.
template <int NB, bool KD1, int G>
static hipError_t group_op(const CoreStepArgs& a, int blocks, hipStream_t s, int op, int* occ) {
    const size_t smem = core_group_smem_bytes(a.H, a.W, a.F, 4, G);
    if (op) {
        *occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, core_group_kernel<NB, 12, 12, G, KD1>, 256, smem) !=
            hipSuccess)
            *occ = 0;
        return hipSuccess;
    }
    const long long groups = (a.E + G - 1) / G;
    if (a.H != 12 || a.W != 12 || a.A > 32 || (groups + (long long)blocks * 4 - 1) / ((long long)blocks * 4) > kGroupMaxIters)
        return hipErrorInvalidConfiguration;   // shapes the kernel and its grid assume
    core_group_kernel<NB, 12, 12, G, KD1><<<dim3((unsigned)blocks), dim3(256), smem, s>>>(a);
    return hipGetLastError();
}

template <int NB>
static hipError_t group_op_kd(const CoreStepArgs& a, int blocks, hipStream_t s, int op, int* occ, int G) {
    if (G == kGroupGSmall)
        return a.kD32 == 1.0f ? group_op<NB, true, kGroupGSmall>(a, blocks, s, op, occ)
                              : group_op<NB, false, kGroupGSmall>(a, blocks, s, op, occ);
    return a.kD32 == 1.0f ? group_op<NB, true, kGroupG>(a, blocks, s, op, occ)
                          : group_op<NB, false, kGroupG>(a, blocks, s, op, occ);
}

hipError_t launch_core_group(const CoreStepArgs& a, int nb, int blocks, hipStream_t s, int G) {
    return nb == 4 ? group_op_kd<4>(a, blocks, s, 0, nullptr, G) : group_op_kd<8>(a, blocks, s, 0, nullptr, G);
}

int core_group_blocks_per_cu(const CoreStepArgs& a, int nb, int G) {
    int n = 0;
    (void)(nb == 4 ? group_op_kd<4>(a, 0, nullptr, 1, &n, G) : group_op_kd<8>(a, 0, nullptr, 1, &n, G));
    return n;
}

// Envs per group for E envs: the large-E size, unless its groups would fill less than half the
// resident waves -- then each wave's one group is the launch's critical path, and halving the
// group (one agent chunk, half the DFF slots) shortens it (E-sweep, profiles/r06/c2: 8,192 envs
// 13.8 -> 12.7 us; from 16,384 envs on G = 4 is faster).  FFM_GROUP_ENVS=2|4 forces it.
int core_group_pick_envs(const CoreStepArgs& a, int nb, long long E, int cus) {
    if (const char* ov = std::getenv("FFM_GROUP_ENVS")) {
        const int v = std::atoi(ov);
        if (v == kGroupGSmall || v == kGroupG) return v;
    }
    const long long waves = (long long)cus * std::max(1, core_group_blocks_per_cu(a, nb, kGroupG)) * 4;
    return 2 * ((E + kGroupG - 1) / kGroupG) <= waves ? kGroupGSmall : kGroupG;
}

}  // namespace ffm
