// core_step.hip -- fused ffm_core step for a batch of independent environments.
//
// One launch advances every env by one FloorFieldModel.step()
// (model/ffm_core.py:36-104 of SoraKurihara/FFM):
//   decide     (:40-88)  lanes = agents; grid (map + occupancy), DFF, SFF in LDS
//   resolve    (:90-98)  lanes = agents; the first requester of a target owns it
//   exit       (:100-102) order-preserving ballot/popcount compaction
//   update_dff (:106-117) lanes = cells; 4/8-point stencil on a zero-halo tile
//
// Two kernels share the per-agent code in core_common.h:
//
//  * core_wave_kernel -- small envs (A <= 64): one WAVE owns one or two envs
//    end to end (lanes 0-31 / 32-63 = the agents of env a / env b), so the
//    whole step needs no workgroup barrier, only in-order LDS within the wave.
//    Waves are persistent (grid-stride over env groups).  Used for BASELINE
//    configs 1, 2 and 4 (12x12, 32 agents).
//  * core_block_kernel -- larger envs (A up to a few thousand, H*W up to
//    ~20k cells): a workgroup owns K >= 1 envs, phases separated by
//    __syncthreads().  Used for config 3 (64x64, 512 agents) and main.py's
//    50x50 / 100-agent room.
//
// Each env's mutable state makes exactly one HBM round trip per step:
// positions (2A B) + count (4 B) + DFF (4HW B) read once and written once.
// Map and SFF are shared by all envs (L2-resident, staged once per block).
//
// Sequential semantics in parallel:
//   * decisions read only the CURRENT positions (the reference builds its
//     occupied set from self.positions, :48-60), so agents decide independently;
//   * dict insertion order of targets (:90): the requesters of target T are
//     the agents adjacent to T (or T's occupant, for a stay); the requester
//     with the smallest index owns T and resolves it, which is the position T
//     has in the dict;
//   * RNG order: Philox draws are keyed by (t, env, agent | owner, purpose),
//     so order does not matter; MT mode (reference replay) serialises the
//     draws of each env on one lane in exactly the reference's order.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "core_common.h"
#include "kernels.h"
#include "lane_common.h"
#include "wave_reset.h"

#ifndef FFM_STAMPS
#define FFM_STAMPS 0   // diagnostic builds only: per-phase s_memtime cycle sums per wave
#endif
#if FFM_STAMPS
#define STAMP(k)                                                                           \
    do {                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        unsigned long long t_;                                                             \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        st[k] += t_ - tlast;                                                               \
        tlast = t_;                                                                        \
    } while (0)
#elif defined(FFM_MARKS)   // diagnostic: phase markers in the ISA (tools/phase_count.py)
#define STAMP(k)                                   \
    do {                                           \
        __builtin_amdgcn_sched_barrier(0);         \
        asm volatile("; @PHASE " #k ::: "memory"); \
        __builtin_amdgcn_sched_barrier(0);         \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif
#ifndef FFM_BLOCK_ABLATE
#define FFM_BLOCK_ABLATE 0   // diagnostic builds only: bit k replaces / skips one phase of the block kernel
#endif

#ifndef FFM_ABLATE
#define FFM_ABLATE 0   // diagnostic builds only (tools/ablate.sh): bit k skips one phase
#endif
#ifndef FFM_WAVES_PER_EU
#define FFM_WAVES_PER_EU 0   // minimum waves/SIMD requested for the wave kernel (0 = compiler's choice)
#endif
#ifndef FFM_PREFETCH_LATE
#define FFM_PREFETCH_LATE 1   // 0: next group's loads at the top; 1: after decide; 2: after resolve
#endif
#ifndef FFM_LDS_PAD
#define FFM_LDS_PAD 0  // diagnostic builds only: extra dynamic LDS per block to pin occupancy
#endif

namespace ffm {

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// ===========================================================================
// Wave kernel: EW envs per wave, AL = 64 / EW agent lanes per env.
// ===========================================================================
struct WaveCarve {
    size_t grid, dff, req, nxt, u, flag, keys, spos, per_wave;
};

// DFF tile of one env: 4 leading zero floats, then rows of DW = W + 4 floats
// (16-B aligned, W % 4 == 0): a zero halo row above and below the map; columns
// W..W+3 of each row are zero and serve as the right halo of that row and the left
// halo of the next (the leading 4 floats are the left halo of the top halo row,
// read by Moore diagonals).  TS floats per env; cell (x, y) at 4 + (x+1)*DW + y.
__host__ __device__ inline int wave_tile_floats(int H, int W) { return 4 + (H + 2) * (W + 4); }

__host__ __device__ inline WaveCarve wave_carve(int PHW, int TS, int AL, int EW, int F, bool mt, bool reset) {
    WaveCarve c;
    size_t o = 0;
    c.grid = o; o += align16((size_t)EW * PHW * 2);        // u16 direction-coded cells
    c.dff = o;  o += align16((size_t)EW * TS * 4);         // f32 tiles, zero halo
    c.req = o;  o += align16((size_t)EW * AL * 2);
    c.nxt = o;  o += align16((size_t)EW * AL * 2);
    c.u = o;    o += align16((size_t)EW * AL * 8);        // MT: f64 draws; Philox: friction words
    c.flag = o; o += mt ? align16((size_t)EW * AL * 2) : 0;
    c.spos = o; o += align16(64 * 2 + 2 * 4);
    c.keys = o; o += reset ? align16((size_t)F * 8) : 0;   // last: the only runtime-sized region
    c.per_wave = o;
    return c;
}

// Block-shared LDS of the wave kernel: padded map codes, padded SFF, padded free-cell list.
__host__ __device__ inline size_t wave_shared_bytes(int PHW) {
    return align16((size_t)PHW) + align16((size_t)PHW * 4) + align16((size_t)PHW * 2);
}

size_t core_wave_smem_bytes(int H, int W, int A, int F, bool mt, bool reset, int waves) {
    const int EW = A <= 32 ? 2 : 1;
    const int PHW = (H + 2) * (W + 2);
    return wave_shared_bytes(PHW) +
           (size_t)waves * wave_carve(PHW, wave_tile_floats(H, W), 64 / EW, EW, F, mt, reset).per_wave;
}

// One env group's HBM state in registers (software pipelining: the next
// group's loads are issued at the top of a group and staged into LDS at its
// bottom, so no register is carried across the loop back edge -- the
// compiler would otherwise wait for the loads at the loop head).
struct WavePrefetch {
    float4 d0, d1;
    int pos;
    int cnt;
};

template <int NB, bool MT, int EW, int HT, int WT>
__global__ __launch_bounds__(256)
#if FFM_WAVES_PER_EU
__attribute__((amdgpu_waves_per_eu(FFM_WAVES_PER_EU)))
#endif
void core_wave_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    using GT = uint16_t;   // DirCodes
    constexpr int AL = 64 / EW;
    const int H = HT ? HT : a.H, W = WT ? WT : a.W;
    const int HW = H * W, PW = W + 2, PHW = (H + 2) * PW;
    const int DW = W + 4, TS = wave_tile_floats(H, W);   // DFF tile row stride / floats per env
    constexpr int kDWS = 2;                    // DW - PW
    const int A = a.A;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform (SGPR)
    const int sub = EW == 2 ? (lane >> 5) : 0;
    const int al = lane - sub * AL;
    const bool do_reset = !MT && a.auto_reset;

    // ---- LDS carve-up: uniform bases, per-lane views ------------------------------
    const WaveCarve cv = wave_carve(PHW, TS, AL, EW, a.F, MT, do_reset);
    uint8_t* pmap = smem;
    float* psff = reinterpret_cast<float*>(smem + align16((size_t)PHW));
    uint16_t* pfree = reinterpret_cast<uint16_t*>(smem + align16((size_t)PHW) + align16((size_t)PHW * 4));
    unsigned char* wbase = smem + wave_shared_bytes(PHW) + (size_t)wv * cv.per_wave;
    GT* grid = reinterpret_cast<GT*>(wbase + cv.grid);
    float* tile = reinterpret_cast<float*>(wbase + cv.dff);
    uint16_t* snxt = reinterpret_cast<uint16_t*>(wbase + cv.nxt);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(wbase + cv.keys);
    uint16_t* spos = reinterpret_cast<uint16_t*>(wbase + cv.spos);
    int* scnt = reinterpret_cast<int*>(wbase + cv.spos + 128);
    GT* gk = grid + sub * PHW;
    float* dk = tile + sub * TS;
    uint16_t* nx = snxt + sub * AL;

    // This lane's two float4 DFF slots (cells 4q..4q+3 of the group, q = lane,
    // lane + 64): 16-B aligned tile offsets, fixed for every group.  W % 4 == 0, so
    // a slot never straddles a row (checked on the host).
    int tb0 = -1, tb1 = -1;
    {
        const int c0 = 4 * lane, c1 = 4 * (lane + 64);
        if (c0 < EW * HW) {
            const int s = c0 / HW, cell = c0 - s * HW, x = cell / W, y = cell - (cell / W) * W;
            tb0 = s * TS + 4 + (x + 1) * DW + y;
        }
        if (c1 < EW * HW) {
            const int s = c1 / HW, cell = c1 - s * HW, x = cell / W, y = cell - (cell / W) * W;
            tb1 = s * TS + 4 + (x + 1) * DW + y;
        }
    }

    const int ngroups = (int)((a.E + EW - 1) / EW);
    const int wstride = (int)gridDim.x * 4;
    int g = (int)blockIdx.x * 4 + wv;   // wave-uniform

    auto prefetch = [&](int gg, WavePrefetch& pf) {
        pf.d0 = pf.d1 = make_float4(0.f, 0.f, 0.f, 0.f);
        pf.pos = 0;
        pf.cnt = 0;
        if (gg < 0) return;
        const long long e0 = (long long)gg * EW;
        const int nenv = (int)((a.E - e0) < EW ? (a.E - e0) : EW);
        const int* cp = a.cnt + e0;
        const uint16_t* pp = a.pos + e0 * A;
        const float4* dp = reinterpret_cast<const float4*>(a.dff + e0 * HW);
        const int n4 = nenv * HW / 4;
        if (sub < nenv) pf.cnt = cp[sub];
        if (sub < nenv && al < A) pf.pos = pp[sub * A + al];
        if (lane < n4) pf.d0 = dp[lane];
        if (lane + 64 < n4) pf.d1 = dp[lane + 64];
    };
    auto stage = [&](const WavePrefetch& pf0) {
        WavePrefetch pf = pf0;
        if (FFM_ABLATE & 512) {   // diagnostic: fixed synthetic state (agents on row 5/6)
            pf.d0 = pf.d1 = make_float4(0.f, 0.f, 0.f, 0.f);
            pf.cnt = a.N;
            pf.pos = (5 + (al >= 10) + (al >= 20)) * W + 1 + (al % 10);
            if (FFM_ABLATE & 1024) asm volatile("" ::"v"(pf0.d0.x), "v"(pf0.d1.x), "v"(pf0.pos), "v"(pf0.cnt));
        }
        if (tb0 >= 0) *reinterpret_cast<float4*>(tile + tb0) = pf.d0;   // ds_write_b128
        if (tb1 >= 0) *reinterpret_cast<float4*>(tile + tb1) = pf.d1;
        spos[lane] = (uint16_t)pf.pos;
        if (al == 0) scnt[sub] = pf.cnt;
    };

    {
        WavePrefetch pf0;
        prefetch(g < ngroups ? g : -1, pf0);
        // Block-shared padded map and SFF; this wave's grids (map codes; agents are
        // marked per step and unmarked after it) and zero-halo DFF tiles.
        for (int i = threadIdx.x; i < PHW; i += 256) {
            pmap[i] = a.pmap[i];
            psff[i] = reinterpret_cast<const float*>(a.psff)[i];
        }
        for (int i = threadIdx.x; i < a.F; i += 256) pfree[i] = a.free_padded[i];
        for (int i = lane; i < EW * TS; i += 64) tile[i] = 0.0f;
        __syncthreads();
        for (int i = lane; i < EW * PHW; i += 64) grid[i] = pmap[i - (i / PHW) * PHW];
        wave_sync();
        stage(pf0);
        wave_sync();
    }

    if (FFM_ABLATE & 4096) return;   // diagnostic: prologue only
    unsigned c_steps = 0, c_exits = 0, c_resets = 0;   // wave-uniform (SGPRs)
#if FFM_STAMPS
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif

    for (; g < ngroups; g += wstride) {
        // Next group's HBM loads: issued after decide (FFM_PREFETCH_LATE), so that the
        // prefetch registers are not live across the decide phase (the VGPR peak).
        WavePrefetch nxtpf;
        auto issue_prefetch = [&]() {
            prefetch(((FFM_ABLATE & 8) || ((FFM_ABLATE & 512) && !(FFM_ABLATE & 1024))) ? -1
                                                                                  : (g + wstride < ngroups ? g + wstride : -1),
                     nxtpf);
        };
        if (!FFM_PREFETCH_LATE) issue_prefetch();

        const long long e0 = (long long)g * EW;
        const int nenv = (int)((a.E - e0) < EW ? (a.E - e0) : EW);
        const bool env_ok = sub < nenv;
        const uint32_t genv = (uint32_t)(a.env_base + e0 + sub);

        const int cnt = scnt[sub];
        int pp = -1, dd0 = 0;   // padded grid cell; DFF tile index = grid index + dd0 (+ 2 per row below)
        if (env_ok && al < A && al < cnt) {
            const int c = spos[lane];
            const int x = c / W, y = c - (c / W) * W;
            pp = (x + 1) * PW + y + 1;
            dd0 = (x + 1) * kDWS + 3;
        }
        // agent-steps of the group: counts at step start of its (1 or 2) envs
        const unsigned gcnt = (unsigned)__builtin_amdgcn_readfirstlane(scnt[0] + (EW == 2 && nenv > 1 ? scnt[1] : 0));
        c_steps += gcnt;
        const bool live = pp >= 0;
        STAMP(0);

        // ---- occupancy marks; default next = stay -----------------------------
        if (live) gk[pp] = (GT)(DirCodes::kAgent | (uint32_t)al | (DirCodes::kNoDir << 8));
        nx[al] = (uint16_t)(live ? pp : 0);
        wave_sync();
        STAMP(1);

        // ---- decide (model/ffm_core.py:40-88) --------------------------------------
        uint32_t slot = kNoReq;
        if (live && !(FFM_ABLATE & 1)) {
            if (MT) {
                slot = decide<NB, false, GT>(pp, PW, gk, psff, nullptr, dk, dd0, kDWS, a.kS32, a.kD32, a.kS64, DrawPending{});
            } else if (FFM_ABLATE & 256) {   // diagnostic: cheap hash instead of Philox
                const uint32_t hsh = (genv * 2654435761u) ^ ((uint32_t)al * 40503u) ^ (a.t * 97u);
                slot = decide<NB, false, GT>(pp, PW, gk, psff, nullptr, dk, dd0, kDWS, a.kS32, a.kD32, a.kS64,
                                             DrawFixed{(double)(hsh >> 8) * (1.0 / 16777216.0)});
            } else {
                const uint4 pb = philox(make_uint4(a.t, genv, (uint32_t)al, kPurDecide << 28), a.key0, a.key1);
                // words 2, 3 feed the friction draw if this agent owns a contested target
                reinterpret_cast<uint2*>(wbase + cv.u)[lane] = make_uint2(pb.z, pb.w);
                slot = decide<NB, false, GT>(pp, PW, gk, psff, nullptr, dk, dd0, kDWS, a.kS32, a.kD32, a.kS64,
                                             DrawFixed{u53(pb.x, pb.y)});
            }
        }
        if (MT) {
            double* su = reinterpret_cast<double*>(wbase + cv.u) + sub * AL;
            const unsigned long long pend = __ballot(slot == kPending);
            if (al == 0 && env_ok) {
                uint32_t* mt_np = a.mt_np + (e0 + sub) * 625;
                unsigned long long mk = (pend >> (sub * AL)) & (AL == 64 ? ~0ull : ((1ull << AL) - 1ull));
                while (mk) {
                    const int i = __builtin_ctzll(mk);
                    mk &= mk - 1ull;
                    su[i] = mt_u53(mt_np);
                }
            }
            wave_sync();
            if (slot == kPending)
                slot = decide<NB, false, GT>(pp, PW, gk, psff, nullptr, dk, dd0, kDWS, a.kS32, a.kD32, a.kS64, DrawFixed{su[al]});
        }
        STAMP(2);
        // The request goes into the agent's own grid cell (resolve reads it there).
        // Other lanes may still be reading this cell for validity: they only test
        // the agent bit, which does not change.
        const uint32_t r = live ? slot_cell<NB>(slot, pp, PW) : kNoReq;
        if (live)   // the high byte of the agent's u16 cell: its chosen slot
            reinterpret_cast<uint8_t*>(gk)[2 * pp + 1] = (uint8_t)(slot <= (uint32_t)NB ? slot : DirCodes::kNoDir);
        wave_sync();
        STAMP(3);

        if (FFM_PREFETCH_LATE == 1) issue_prefetch();

        // ---- resolve (model/ffm_core.py:90-98) ---------------------------------------
        {
            uint16_t who[NB];
            bool is[NB];
            const bool moving = live && r != kNoReq && (int)r != pp;
            int m = 0, s0 = -1;
            bool owner = false;
            if (moving) {
                m = requesters_dir<NB>((int)r, PW, gk, who, is);
                s0 = kth_slot<NB>(who, is, 0);
                owner = s0 >= 0 && who[s0] == al;
            }
            if (MT) {
                uint16_t* fl = reinterpret_cast<uint16_t*>(wbase + cv.flag) + sub * AL;
                const int fr_m = (owner && m >= 2) ? m : 0;
                fl[al] = (uint16_t)fr_m;
                const unsigned long long cont = __ballot(fr_m >= 2);
                wave_sync();
                if (al == 0 && env_ok) {
                    uint32_t* mt_np = a.mt_np + (e0 + sub) * 625;
                    uint32_t* mt_py = a.mt_py + (e0 + sub) * 625;
                    unsigned long long mk = (cont >> (sub * AL)) & (AL == 64 ? ~0ull : ((1ull << AL) - 1ull));
                    while (mk) {
                        const int i = __builtin_ctzll(mk);
                        mk &= mk - 1ull;
                        const double u = mt_u53(mt_np);                                   // np.random.rand()
                        const int kk = u < 0.5 ? (int)mt_randbelow(mt_py, (uint32_t)fl[i]) : -1;   // random.choice
                        fl[i] = (uint16_t)(kk >= 0 ? 0x100 | kk : 0x200);
                    }
                }
                wave_sync();
            }
            if (live && r != kNoReq && !(FFM_ABLATE & 2)) {
                if ((int)r == pp) {
                    dk[pp + dd0] += 1.0f;                                                 // :91-93 (stay)
                } else if (owner) {
                    int ws = -1;
                    if (m == 1) {
                        ws = s0;
                    } else if (MT) {
                        const int f = (reinterpret_cast<uint16_t*>(wbase + cv.flag) + sub * AL)[al];
                        if (f & 0x100) ws = kth_slot<NB>(who, is, f & 0xFF);
                    } else if (FFM_ABLATE & 128) {   // diagnostic: cheap hash instead of Philox
                        const uint32_t hsh = (genv * 2654435761u) ^ ((uint32_t)al * 40503u) ^ a.t;
                        if (hsh & 1) ws = kth_slot<NB>(who, is, (int)((hsh >> 8) % (uint32_t)m));
                    } else {
                        const uint2 f = reinterpret_cast<const uint2*>(wbase + cv.u)[lane];
                        const int kk = philox_friction(f.x, f.y, (uint32_t)m, a.key0, a.key1, a.t, genv, (uint32_t)al);
                        if (kk >= 0) ws = kth_slot<NB>(who, is, kk);                            // :95-96
                    }
                    if (ws >= 0) {
                        int wcell = (int)r;
                        uint16_t wi = 0;
#pragma unroll
                        for (int s = 0; s < NB; s++)
                            if (s == ws) {
                                wcell = (int)r - nb_dx<NB>(s) * PW - nb_dy<NB>(s);
                                wi = who[s];
                            }
                        nx[wi] = (uint16_t)r;
                        dk[wcell + (wcell / PW) * kDWS + 3] += 1.0f;                      // :97-98
                    }
                }
            }
        }
        wave_sync();
        STAMP(4);

        if (FFM_PREFETCH_LATE == 2) issue_prefetch();

        // ---- exits: order-preserving compaction (model/ffm_core.py:100-102) ---------
        const int nxt = live ? (int)nx[al] : 0;
        const bool keep = live && pmap[nxt] != 3;
        const unsigned long long km = __ballot(keep);
        const unsigned long long segm = AL == 64 ? ~0ull : (((1ull << AL) - 1ull) << (sub * AL));
        const int newidx = lanes_below(km & segm);
        const int newcnt = __popcll(km & segm);
        c_exits += gcnt - (unsigned)__popcll(km);
        if (live) gk[pp] = 0;   // unmark: agents only ever stand on free cells

        // An env this step emptied is re-placed at the end of the group (below).
        const bool rs = do_reset && env_ok && newcnt == 0 && !(FFM_ABLATE & 32);
        {
            const unsigned long long rb = __ballot(rs);
            c_resets += (unsigned)((rb & 1ull) + (EW == 2 ? ((rb >> AL) & 1ull) : 0ull));
        }
        STAMP(5);

        // ---- update_dff (model/ffm_core.py:106-117), float4 per lane ------------------
        // Pass 1: B = c0 * D in place (:109; halo stays 0).  Pass 2: per slot, three
        // aligned ds_read_b128 (rows x-1, x, x+1) and the scalars left/right of them.
        float b0[4], b1[4];
        auto scale = [&](int tb, float (&bq)[4]) {
            float4* p = reinterpret_cast<float4*>(tile + tb);
            const float4 q = *p;
            bq[0] = a.c0 * q.x; bq[1] = a.c0 * q.y; bq[2] = a.c0 * q.z; bq[3] = a.c0 * q.w;
            *p = make_float4(bq[0], bq[1], bq[2], bq[3]);
        };
        if (tb0 >= 0) scale(tb0, b0);
        if (tb1 >= 0) scale(tb1, b1);
        wave_sync();
        auto stencil = [&](int tb, const float (&bq)[4], float (&o)[4]) {
            const float* p = tile + tb;
            float v[3][6];   // rows dx = -1..1, columns -1..4 of the slot (B values)
#pragma unroll
            for (int dx = -1; dx <= 1; dx += 2) {
                const float4 q = *reinterpret_cast<const float4*>(p + dx * DW);
                v[dx + 1][1] = q.x; v[dx + 1][2] = q.y; v[dx + 1][3] = q.z; v[dx + 1][4] = q.w;
            }
#pragma unroll
            for (int dx = -1; dx <= 1; dx++) {
                v[dx + 1][0] = p[dx * DW - 1];
                v[dx + 1][5] = p[dx * DW + 4];
            }
            v[1][1] = bq[0]; v[1][2] = bq[1]; v[1][3] = bq[2]; v[1][4] = bq[3];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float acc = bq[j];
#pragma unroll
                for (int k = 0; k < NB; k++) {
                    if (FFM_ABLATE & 4) break;
                    const float t = a.c1 * v[1 + nb_dx<NB>(k)][j + 1 + nb_dy<NB>(k)];     // :113
                    acc = acc + t;
                }
                o[j] = acc < 1e-4f ? 0.0f : acc;                                         // :116-117
            }
        };
        float o0[4], o1[4];
        if (tb0 >= 0) stencil(tb0, b0, o0);
        if (tb1 >= 0) stencil(tb1, b1, o1);
        wave_sync();
        STAMP(6);

        // ---- stage the next group (its loads were issued at the top), then store ------
        const unsigned long long rsm = __ballot(rs);
        stage(nxtpf);
        if (!(FFM_ABLATE & 16)) {
            uint16_t* gp = a.pos + e0 * A;
            int* gc = a.cnt + e0;
            float4* gd = reinterpret_cast<float4*>(a.dff + e0 * HW);
            const int n4 = nenv * HW / 4;
            if (keep) gp[sub * A + newidx] = (uint16_t)unpad(nxt, PW);
            if (al == 0 && env_ok) {
                gc[sub] = rs ? a.N : newcnt;
                if (rs && a.episodes) a.episodes[e0 + sub] += 1;
            }
            // a reset env starts its next episode with a zero DFF
            const int zs0 = (4 * lane) / HW, zs1 = (4 * (lane + 64)) / HW;
            const bool z0 = zs0 < EW && ((rsm >> (zs0 * AL)) & 1ull);
            const bool z1 = zs1 < EW && ((rsm >> (zs1 * AL)) & 1ull);
            if (tb0 >= 0 && lane < n4)
                gd[lane] = z0 ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(o0[0], o0[1], o0[2], o0[3]);
            if (tb1 >= 0 && lane + 64 < n4)
                gd[lane + 64] = z1 ? make_float4(0.f, 0.f, 0.f, 0.f) : make_float4(o1[0], o1[1], o1[2], o1[3]);
        }
        // ---- auto-reset: Philox placement keyed by t, stored straight
        // to the env's positions.  Rare; placed last, where little else is live.
        if (rsm) {   // wave-uniform
#pragma unroll
            for (int s = 0; s < EW; s++)
                if ((rsm >> (s * AL)) & 1ull)
                    wave_reset_env(a, (uint32_t)(a.env_base + e0 + s), keys, pfree, a.pos + (e0 + s) * A, lane);
        }
        wave_sync();
        STAMP(7);
    }

    // ---- counters: one atomic per wave ------------------------------------------------
    if (lane == 0) {
        // Counters live in one 32-B slot per wave: no two waves ever add to the
        // same address (a single contended word saturates near 100 adds/us).
        unsigned long long* slot = a.counters + 4 * ((size_t)blockIdx.x * 4 + wv);
        if (c_steps) atomicAdd(&slot[0], (unsigned long long)c_steps);
        if (c_exits) atomicAdd(&slot[1], (unsigned long long)c_exits);
        if (c_resets) atomicAdd(&slot[2], (unsigned long long)c_resets);
        if (blockIdx.x == 0 && wv == 0) atomicAdd(&slot[3], 1ull);
#if FFM_STAMPS
        if (a.dbg) {
            for (int k = 0; k < 8; k++) atomicAdd(&a.dbg[k], st[k]);
            atomicAdd(&a.dbg[8], 1ull);
        }
#endif
    }
}

// ===========================================================================
// Block kernel: K envs per workgroup of BS threads.
// ===========================================================================
// The map and SFF are read from global memory (L2-resident, shared by every
// block) and the placement keys are capped: LDS per block drops from ~82 KB to
// ~40 KB at config 3 (64x64, 512 agents), 3 blocks per CU instead of 1.
struct BlockCarve {
    size_t grid, dff, pos, req, nxt, misc, u, flag, keys, total;
    size_t lds;     // LDS bytes per block (big: the misc words only; the rest is global scratch)
};

// Placement candidates kept in LDS: the threshold of reset_threshold() passes
// ~2N + 16 keys (N <= A); room for 8 standard deviations more.  More (or fewer
// than N) take the exact recomputing path (probability < 1e-15).
__host__ __device__ inline int block_keys_cap(int A, int F) {
    const int m = 2 * A + 16;
    int r = 1;
    while (r * r < m) r++;
    const int cap = m + 8 * r + 64;
    return cap < F ? cap : F;
}

// big: maps whose state exceeds the LDS (up to 256 x 256): one env per block, the
// grid, DFF tile, cell lists and placement keys in a global scratch region of the
// block (L2-resident while the block runs), padded cells as u32 (> 65,535 of them).
__host__ __device__ inline BlockCarve block_carve(int PHW, int A, int K, int F, bool f64, bool mt, bool reset,
                                                  bool big = false) {
    BlockCarve c;
    size_t o = 0;
    (void)f64;
    const size_t ix = big ? 4 : 2;
    const size_t misc = align16((size_t)(8 * K + 64) * 4);
    // the DFF tile and the misc words live through the whole step; the grid and the agent
    // arrays are dead once the exits are compacted, so the auto-reset's placement keys
    // (used only after that) share their bytes -- 11 KB less LDS at C3, a fourth block per CU
    c.dff = o;  o += align16((size_t)K * PHW * 4);
    c.misc = big ? 0 : o;
    o += big ? 0 : misc;
    const size_t dead = o;
    c.grid = o; o += align16((size_t)K * PHW * 2);
    c.pos = o;  o += align16((size_t)K * A * ix);
    c.req = o;  o += align16((size_t)K * A * ix);
    c.nxt = o;  o += align16((size_t)K * A * ix);
    c.u = o;    o += align16((size_t)K * A * 8);   // MT: the pending draws; Philox: the friction words
    c.flag = o; o += mt ? align16((size_t)K * A * 2) : 0;
    c.keys = dead;
    if (reset) {
        const size_t kb = align16((size_t)block_keys_cap(A, F) * 8);
        if (dead + kb > o) o = dead + kb;
    }
    c.total = o;
    c.lds = big ? misc : o;
    return c;
}

size_t core_block_smem_bytes(int H, int W, int A, int K, int F, bool f64, bool mt, bool reset) {
    return block_carve((H + 2) * (W + 2), A, K, F, f64, mt, reset).total;
}

size_t core_big_scratch_bytes(int H, int W, int A, int F, bool mt) {
    return block_carve((H + 2) * (W + 2), A, 1, F, false, mt, true, true).total;
}

// (env, row, column) of a flat index i = (k * rows + r) * cols + c, advanced by a
// fixed stride without integer division (a runtime divide is ~30 VALU, and the
// cell loops of the block kernel would otherwise run two per cell).
struct Idx3 {
    int k, r, c;
    int dr, dc, rows, cols;
    __device__ Idx3(int i, int stride, int rows_, int cols_) : rows(rows_), cols(cols_) {
        const int per = rows * cols;
        k = i / per;
        const int rem = i - k * per;
        r = rem / cols;
        c = rem - r * cols;
        dr = stride / cols;
        dc = stride - dr * cols;
    }
    __device__ __forceinline__ void advance() {
        c += dc;
        r += dr;
        if (c >= cols) { c -= cols; r++; }
        while (r >= rows) { r -= rows; k++; }
    }
};

// (env, agent) of flat agent slot it = k * A + i, advanced by the block size
// without integer division.
struct AgentIdx {
    int it, k, i, dk, di, A;
    __device__ AgentIdx(int it0, int stride, int A_) : it(it0), A(A_) {
        k = it0 / A;
        i = it0 - k * A;
        dk = stride / A;
        di = stride - dk * A;
    }
    __device__ __forceinline__ void advance() {
        it += dk * A + di;
        i += di;
        k += dk;
        if (i >= A) { i -= A; k++; }
    }
};

// Block-wide exclusive prefix of a 0/1 flag over thread order (+ total).
template <int BS>
__device__ __forceinline__ int block_excl_scan(bool flag, int* swsum, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long mask = __ballot(flag);
    const int lp = lanes_below(mask);
    if (lane == 0) swsum[wave] = __popcll(mask);
    __syncthreads();
    int wp = 0, tot = 0;
#pragma unroll
    for (int v = 0; v < BS / 64; v++) {
        const int c = swsum[v];
        wp += v < wave ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return wp + lp;
}

// Philox placement of env e by the whole workgroup: the N free cells
// with the smallest (key_j, j).  Candidates under a threshold (~2N + 16 of them) are
// kept in `keys` (KC of them) and ranked; more than KC take an exact recomputing path.
template <int BS>
__device__ void block_place_env(const CoreStepArgs& a, long long e, unsigned long long* keys, int KC, int* swsum) {
    const int tid = threadIdx.x;
    const uint32_t genv = (uint32_t)(a.env_base + e);
    uint32_t T = reset_threshold(a.N, a.F);
    int C = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        C = 0;
        for (int j0 = 0; j0 < a.F; j0 += BS) {
            const int j = j0 + tid;
            uint32_t key = 0;
            bool cand = false;
            if (j < a.F) {
                key = reset_key(a.key0, a.key1, a.t, genv, (uint32_t)j);
                cand = key <= T;
            }
            int tot;
            const int ex = block_excl_scan<BS>(cand, swsum, tot);
            if (cand && C + ex < KC) keys[C + ex] = ((unsigned long long)key << 32) | (unsigned)j;
            C += tot;
        }
        if ((C >= a.N && C <= KC) || T == 0xFFFFFFFFu) break;
        if (C > KC) break;       // too many to keep: the recomputing path below
        T = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (C <= KC) {
        for (int i = tid; i < C; i += BS) {
            const unsigned long long ki = keys[i];
            int rank = 0;
#pragma unroll 4
            for (int q = 0; q < C; q++) rank += keys[q] < ki ? 1 : 0;
            if (rank < a.N) a.pos[e * a.A + rank] = a.free_list[(int)(ki & 0xFFFFFFFFu)];
        }
    } else {
        // Exact but slow (keys recomputed per comparison): the candidates exceed KC.
        for (int j = tid; j < a.F; j += BS) {
            const uint32_t kj = reset_key(a.key0, a.key1, a.t, genv, (uint32_t)j);
            if (kj > T) continue;
            const unsigned long long ki = ((unsigned long long)kj << 32) | (unsigned)j;
            int rank = 0;
            for (int q = 0; q < a.F && rank < a.N; q++) {
                const unsigned long long kq =
                    ((unsigned long long)reset_key(a.key0, a.key1, a.t, genv, (uint32_t)q) << 32) | (unsigned)q;
                rank += kq < ki ? 1 : 0;
            }
            if (rank < a.N) a.pos[e * a.A + rank] = a.free_list[j];
        }
    }
    __syncthreads();
}

// Request / target cell of a decide slot: padded cells are u16 (CT) in LDS-sized envs
// and u32 for big maps, whose cell indices reach the u16 sentinels.
template <class CT>
struct ReqCodes {
    static constexpr CT kNone = (CT)~(CT)0, kWait = (CT)(~(CT)0 - 1);
};
template <int NB, class CT>
__device__ __forceinline__ CT req_cell(uint32_t slot, int pp, int PW) {
    return slot <= (uint32_t)NB ? (CT)slot_cell<NB>(slot, pp, PW)
           : slot == kPending ? ReqCodes<CT>::kWait : ReqCodes<CT>::kNone;
}

#ifndef FFM_BLOCK_WAVES
#define FFM_BLOCK_WAVES 8   // Neumann float32: minimum waves per SIMD asked of the register allocator
#endif

// The Neumann float32 kernels fit 8 waves per SIMD (57 VGPRs, 78 SGPRs, no spills) and with
// the placement keys sharing the dead arrays' LDS (block_carve) four 512-lane blocks fit a
// CU: C3 137.3 -> 129.7 us.  Moore and float64 would spill under that bound: theirs stays 1.
template <int NB, bool F64, bool MT, int BS, bool BIG>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(NB == 4 && !F64 ? FFM_BLOCK_WAVES : 1, 8)))
void core_block_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    using GT = uint16_t;
    using CT = typename std::conditional<BIG, uint32_t, uint16_t>::type;
    constexpr CT kNoReqC = ReqCodes<CT>::kNone, kPendingC = ReqCodes<CT>::kWait;
    const int tid = threadIdx.x;
    const int H = a.H, W = a.W, HW = H * W, PW = W + 2, PHW = (H + 2) * PW, A = a.A;
    const long long e0 = (long long)blockIdx.x * a.K;
    const int K = (int)((a.E - e0) < a.K ? (a.E - e0) : a.K);
    const bool do_reset = !MT && a.auto_reset;
    const BlockCarve cv = block_carve(PHW, A, a.K, a.F, F64, MT, do_reset || BIG, BIG);
    // big maps: everything but the misc words in this block's global scratch region
    unsigned char* gbase = BIG ? a.scratch + (size_t)blockIdx.x * a.scratch_stride : smem;
    const uint8_t* pmap = a.pmap;
    const float* psff32 = reinterpret_cast<const float*>(a.psff);
    const double* psff64 = reinterpret_cast<const double*>(a.psff);
    const int KC = block_keys_cap(A, a.F);
    GT* grid = reinterpret_cast<GT*>(gbase + cv.grid);
    float* tile = reinterpret_cast<float*>(gbase + cv.dff);
    CT* spos = reinterpret_cast<CT*>(gbase + cv.pos);
    CT* sreq = reinterpret_cast<CT*>(gbase + cv.req);
    CT* snxt = reinterpret_cast<CT*>(gbase + cv.nxt);
    int* scnt = reinterpret_cast<int*>(smem + cv.misc);   // [K] count at step start
    int* snew = scnt + a.K;                                // [K] count after exits
    int* sreset = snew + a.K;                              // [K] reset flag
    int* sseg = sreset + a.K;                              // [K] scan segment base
    int* swsum = sseg + a.K;                               // [BS/64]
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(gbase + cv.keys);

    const int nA = K * A;
    const int nP = K * PHW;
    const AgentIdx ag0(tid, BS, A);   // this thread's first (env, agent) slot
    const uint32_t mW = a.mW, mPW = a.mPW;   // cell -> row without a divide (host-computed magic numbers)

    // ---- load -------------------------------------------------------------------
    if ((W & 3) == 0) {
        // interior cells as 16-B loads of four cells of a row; the halo ring is zeroed
        // with the grid pass (disjoint cells, one barrier below)
        const int W4 = W >> 2;
        Idx3 iq(tid, BS, H, W4);
        for (int q = tid; q < K * H * W4; q += BS, iq.advance()) {
            const float4 v = *reinterpret_cast<const float4*>(a.dff + ((e0 + iq.k) * H + iq.r) * W + 4 * iq.c);
            float* t = tile + iq.k * PHW + (iq.r + 1) * PW + 4 * iq.c + 1;
            t[0] = v.x; t[1] = v.y; t[2] = v.z; t[3] = v.w;
        }
        // the halo ring of every env's tile: 2 PW + 2 H cells (rows 0 and H + 1, then the
        // side columns), no per-cell row / column arithmetic over the whole grid
        const int ring = 2 * PW + 2 * H;
        for (int k = 0; k < K; k++)
            for (int j = tid; j < ring; j += BS) {
                const int jc = j - 2 * PW;
                const int c = j < PW ? j : j < 2 * PW ? (H + 1) * PW + (j - PW) : (1 + (jc >> 1)) * PW + ((jc & 1) ? W + 1 : 0);
                tile[k * PHW + c] = 0.0f;
            }
        // every env's grid starts as the map: four u8 cells per load, two u16 dwords per store
        // (W % 4 == 0: PW and PHW are even, so each env's grid is dword aligned)
        const uint32_t* m32 = reinterpret_cast<const uint32_t*>(a.pmap);
        const int P4 = PHW >> 2;
        for (int k = 0; k < K; k++) {
            uint32_t* g32 = reinterpret_cast<uint32_t*>(grid + k * PHW);
            for (int i = tid; i < P4; i += BS) {
                const uint32_t m = m32[i];
                g32[2 * i] = (m & 0xFFu) | ((m << 8) & 0xFF0000u);
                g32[2 * i + 1] = ((m >> 16) & 0xFFu) | ((m >> 8) & 0xFF0000u);
            }
            for (int i = 4 * P4 + tid; i < PHW; i += BS) grid[k * PHW + i] = a.pmap[i];
        }
    } else {
        Idx3 ix(tid, BS, H + 2, PW);
        for (int i = tid; i < nP; i += BS, ix.advance()) {
            const int x = ix.r - 1, y = ix.c - 1, pc = ix.r * PW + ix.c;
            const bool in = x >= 0 && x < H && y >= 0 && y < W;
            tile[i] = in ? a.dff[(e0 + ix.k) * HW + x * W + y] : 0.0f;
            grid[i] = a.pmap[pc];
        }
    }
    if (tid < K) {
        scnt[tid] = a.cnt[e0 + tid];
        sreset[tid] = 0;
    }
    __syncthreads();
    for (AgentIdx ag = ag0; ag.it < nA; ag.advance()) {
        const int it = ag.it;
        const int k = ag.k, i = ag.i;
        int pp = 0;
        if (i < scnt[k]) {
            const int c = a.pos[(e0 + k) * A + i];
            const int x = mdiv(c, mW), y = c - x * W;
            pp = (x + 1) * PW + y + 1;
        }
        spos[it] = (CT)pp;
    }
    __syncthreads();

    // ---- occupancy marks --------------------------------------------------------------
    for (AgentIdx ag = ag0; ag.it < nA; ag.advance()) {
        const int it = ag.it;
        const int k = ag.k, i = ag.i;
        if (i < scnt[k]) grid[k * PHW + spos[it]] = (GT)(GridCodes<GT>::kAgent | (uint32_t)i);
        snxt[it] = spos[it];
        sreq[it] = kNoReqC;
    }
    __syncthreads();

    // ---- decide (model/ffm_core.py:40-88) -----------------------------------------------
    for (AgentIdx ag = ag0; ag.it < nA; ag.advance()) {
        const int it = ag.it;
        const int k = ag.k, i = ag.i;
        if (i >= scnt[k]) continue;
        const int pp = spos[it];
        CT r;
        if (MT) {
            r = req_cell<NB, CT>(decide<NB, F64, GT>(pp, PW, grid + k * PHW, psff32, psff64, tile + k * PHW, 0, 0, a.kS32, a.kD32,
                                                     a.kS64, DrawPending{}), pp, PW);
        } else {
            // the agent's draw block; its words z, w are the friction draw if it owns a
            // contested target (the resolve reads them instead of recomputing the block)
            const uint4 pb = (FFM_BLOCK_ABLATE & 1)   // diagnostic: a cheap hash instead of Philox
                                 ? make_uint4((uint32_t)i * 0x9E3779B1u ^ a.t, (uint32_t)k * 0x85EBCA6Bu, (uint32_t)i, 7u)
                                 : philox(make_uint4(a.t, (uint32_t)(a.env_base + e0 + k), (uint32_t)i, kPurDecide << 28),
                                          a.key0, a.key1);
            reinterpret_cast<uint2*>(gbase + cv.u)[it] = make_uint2(pb.z, pb.w);
            if (F64) {
                r = req_cell<NB, CT>(decide<NB, F64, GT>(pp, PW, grid + k * PHW, psff32, psff64, tile + k * PHW, 0, 0,
                                                         a.kS32, a.kD32, a.kS64, DrawFixed{u53(pb.x, pb.y)}), pp, PW);
            } else {
                // the trimmed fast pass of the small-env kernels (float32 u, masked scores, no
                // double conversion; the tile has the grid's layout: DWS = 0), the exact NumPy
                // pass only when u lies within the margin of a cdf boundary (identical results)
                bool to_exit = false;
                uint32_t slot = (FFM_BLOCK_ABLATE & 8) ? (uint32_t)NB   // diagnostic: everyone stays
                                : lane_decide<NB, false, false, 0>(pp, PW, grid + k * PHW, psff32, tile + k * PHW, 0,
                                                                 a.kS32, a.kD32, pb.x, to_exit);
                if (slot == kPending)
                    slot = NB == 4 ? lane_decide_exact<NB, false, 0>(pp, PW, grid + k * PHW, psff32, tile + k * PHW, 0,
                                                                     a.kS32, a.kD32, u53(pb.x, pb.y))
                                   : lane_decide_exact_arr<NB, false, 0>(pp, PW, grid + k * PHW, psff32, tile + k * PHW,
                                                                         0, a.kS32, a.kD32, u53(pb.x, pb.y));
                r = req_cell<NB, CT>(slot, pp, PW);
            }
        }
        sreq[it] = r;
    }
    __syncthreads();

    if (MT) {
        // NumPy stream: one draw per pending agent, in agent order; then redo the choice.
        double* su = reinterpret_cast<double*>(gbase + cv.u);
        if (tid < K) {
            uint32_t* mt_np = a.mt_np + (e0 + tid) * 625;
            for (int i = 0; i < scnt[tid]; i++)
                if (sreq[tid * A + i] == kPendingC) su[tid * A + i] = mt_u53(mt_np);
        }
        __syncthreads();
        for (AgentIdx ag = ag0; ag.it < nA; ag.advance()) {
        const int it = ag.it;
            const int k = ag.k, i = ag.i;
            if (i >= scnt[k] || sreq[it] != kPendingC) continue;
            sreq[it] = req_cell<NB, CT>(decide<NB, F64, GT>(spos[it], PW, grid + k * PHW, psff32, psff64, tile + k * PHW, 0, 0,
                                                            a.kS32, a.kD32, a.kS64, DrawFixed{su[it]}), spos[it], PW);
        }
        __syncthreads();

        // Owners of contested targets, then their draws in owner (= dict) order.
        uint16_t* sflag = reinterpret_cast<uint16_t*>(gbase + cv.flag);
        for (AgentIdx ag = ag0; ag.it < nA; ag.advance()) {
        const int it = ag.it;
            const int k = ag.k, i = ag.i;
            sflag[it] = 0;
            if (i >= scnt[k]) continue;
            const CT r = sreq[it];
            if (r == kNoReqC || r == spos[it]) continue;
            uint16_t who[NB];
            bool is[NB];
            const int m = requesters<NB, GT, CT>((int)r, PW, grid + k * PHW, sreq + k * A, who, is);
            const int s0 = kth_slot<NB>(who, is, 0);
            if (m >= 2 && s0 >= 0 && who[s0] == i) sflag[it] = (uint16_t)m;
        }
        __syncthreads();
        if (tid < K) {
            uint32_t* mt_np = a.mt_np + (e0 + tid) * 625;
            uint32_t* mt_py = a.mt_py + (e0 + tid) * 625;
            for (int i = 0; i < scnt[tid]; i++) {
                const int m = sflag[tid * A + i];
                if (m >= 2) {
                    const double u = mt_u53(mt_np);                                   // np.random.rand()
                    const int kk = u < 0.5 ? (int)mt_randbelow(mt_py, (uint32_t)m) : -1;   // random.choice
                    sflag[tid * A + i] = (uint16_t)(kk >= 0 ? 0x100 | kk : 0x200);
                }
            }
        }
        __syncthreads();
    }

    // ---- resolve (model/ffm_core.py:90-98) ---------------------------------------------------
    for (AgentIdx ag = ag0; ag.it < nA; ag.advance()) {
        const int it = ag.it;
        const int k = ag.k, i = ag.i;
        if (i >= scnt[k]) continue;
        const CT rc = sreq[it];
        if (rc == kNoReqC) continue;
        const int r = (int)rc;
        float* dk = tile + k * PHW;
        const int pp = spos[it];
        if (r == pp) {
            dk[pp] += 1.0f;                                                           // :91-93 (stay)
            continue;
        }
        if (FFM_BLOCK_ABLATE & 2) {   // diagnostic: no requester scan (every mover granted)
            snxt[it] = (CT)r;
            dk[pp] += 1.0f;
            continue;
        }
        uint16_t who[NB];
        bool is[NB];
        const int m = requesters<NB, GT, CT>(r, PW, grid + k * PHW, sreq + k * A, who, is);
        const int s0 = kth_slot<NB>(who, is, 0);
        if (s0 < 0 || who[s0] != i) continue;  // not the owner
        int ws = -1;
        if (m == 1) {
            ws = s0;
        } else if (MT) {
            const int f = reinterpret_cast<uint16_t*>(gbase + cv.flag)[it];
            if (f & 0x100) ws = kth_slot<NB>(who, is, f & 0xFF);
        } else {
            const uint32_t genv = (uint32_t)(a.env_base + e0 + k);
            const uint2 f = reinterpret_cast<const uint2*>(gbase + cv.u)[it];
            const int kk = philox_friction(f.x, f.y, (uint32_t)m, a.key0, a.key1, a.t, genv, (uint32_t)i);
            if (kk >= 0) ws = kth_slot<NB>(who, is, kk);                                // :95-96
        }
        if (ws >= 0) {
            int wcell = r;
            uint16_t wi = 0;
#pragma unroll
            for (int s = 0; s < NB; s++)
                if (s == ws) {
                    wcell = r - nb_dx<NB>(s) * PW - nb_dy<NB>(s);
                    wi = who[s];
                }
            snxt[k * A + wi] = (CT)r;
            dk[wcell] += 1.0f;                                                        // :97-98
        }
    }
    __syncthreads();

    // ---- exits: order-preserving compaction (model/ffm_core.py:100-102) -------------------------
    {
        int carry = 0;
        AgentIdx ex = ag0;
        for (int base = 0; base < nA; base += BS, ex.advance()) {
            const int it = base + tid;
            const int k = ex.k, i = ex.i;
            const bool live = it < nA && i < scnt[k];
            const bool keep = live && pmap[snxt[it]] != 3;
            int tot;
            const int excl = carry + block_excl_scan<BS>(keep, swsum, tot);
            if (it < nA && i == 0) sseg[k] = excl;
            __syncthreads();
            if (it < nA) {
                const int seg = sseg[k];
                if (keep) a.pos[(e0 + k) * A + (excl - seg)] = (uint16_t)unpad_m(snxt[it], PW, mPW);
                if (i == A - 1) snew[k] = excl + (keep ? 1 : 0) - seg;
            }
            carry += tot;
            __syncthreads();
        }
    }

    // ---- auto-reset of envs this step emptied (Philox placement keyed by t) -------------------
    if (do_reset) {
        if (tid < K) sreset[tid] = snew[tid] == 0 ? 1 : 0;
        __syncthreads();
        for (int k = 0; k < K; k++) {
            if (!sreset[k]) continue;   // block-uniform
            block_place_env<BS>(a, e0 + k, keys, KC, swsum);
        }
    }

    // ---- counters ---------------------------------------------------------------------------
    if (tid == 0) {
        unsigned long long steps = 0, exits = 0, resets = 0;
        for (int k = 0; k < K; k++) {
            steps += (unsigned long long)scnt[k];
            exits += (unsigned long long)(scnt[k] - snew[k]);
            resets += (unsigned long long)sreset[k];
        }
        unsigned long long* slot = a.counters + 4 * (size_t)blockIdx.x;   // one slot per block
        atomicAdd(&slot[0], steps);
        atomicAdd(&slot[1], exits);
        if (resets) atomicAdd(&slot[2], resets);
        if (blockIdx.x == 0) atomicAdd(&slot[3], 1ull);
    }
    if (tid < K) {
        a.cnt[e0 + tid] = sreset[tid] ? a.N : snew[tid];
        if (sreset[tid] && a.episodes) a.episodes[e0 + tid] += 1;
    }

    // ---- update_dff (model/ffm_core.py:106-117) --------------------------------------------------
    // B = c0 * D (:109) is formed on the fly from each operand, rounded exactly as the
    // reference's separate pass, so the tile is read once and needs no extra barrier.
    __syncthreads();   // every deposit of the resolve is in the tile
    const float c0 = a.c0, c1 = a.c1;
    if ((W & 3) == 0) {
        // four cells of a row per thread: 16-B DFF stores, shared row operands
        const int W4 = W >> 2;
        Idx3 ix(tid, BS, H, W4);
        for (int q = tid; q < K * H * W4; q += BS, ix.advance()) {
            const int k = ix.k, x = ix.r, y = 4 * ix.c;
            const float* p = tile + k * PHW + (x + 1) * PW + y + 1;
            float b[3][6];   // rows dx = -1..1, columns y-1..y+4
#pragma unroll
            for (int dx = -1; dx <= 1; dx++)
#pragma unroll
                for (int j = -1; j <= 4; j++) b[dx + 1][j + 1] = (NB == 4 && dx != 0 && (j < 0 || j > 3)) ? 0.0f
                                                                  : c0 * p[dx * PW + j];
            float o[4];
            if (FFM_BLOCK_ABLATE & 4) {   // diagnostic: no stencil arithmetic
                o[0] = b[1][1]; o[1] = b[1][2]; o[2] = b[1][3]; o[3] = b[1][4];
            } else
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float acc = b[1][j + 1];
#pragma unroll
                for (int s2 = 0; s2 < NB; s2++) {
                    const float t = c1 * b[1 + nb_dx<NB>(s2)][j + 1 + nb_dy<NB>(s2)];   // :113
                    acc = acc + t;
                }
                o[j] = (acc < 1e-4f || sreset[k]) ? 0.0f : acc;                      // :116-117
            }
            *reinterpret_cast<float4*>(a.dff + (e0 * H + (long long)k * H + x) * W + y) =
                make_float4(o[0], o[1], o[2], o[3]);
        }
    } else {
        Idx3 ix(tid, BS, H, W);
        for (int c = tid; c < K * HW; c += BS, ix.advance()) {
            const int k = ix.k, x = ix.r, y = ix.c;
            const float* p = tile + k * PHW + (x + 1) * PW + y + 1;
            float acc = c0 * *p;
#pragma unroll
            for (int q = 0; q < NB; q++) {
                const float t = c1 * (c0 * p[nb_dx<NB>(q) * PW + nb_dy<NB>(q)]);   // :113
                acc = acc + t;
            }
            // :116-117; an env reset this step starts its next episode with a zero DFF
            a.dff[e0 * HW + c] = (acc < 1e-4f || sreset[k]) ? 0.0f : acc;
        }
    }
}

// ===========================================================================
// Reset every env (Philox placement, counts = N); DFF zeroed by the host.
// ===========================================================================
// mask (device, [E] bytes; ffm_engine_reset_envs): only the envs with a nonzero byte are
// re-placed, their DFF row zeroed and their position row cleared here (the whole-engine reset
// clears every row by memset beforehand).
__global__ __launch_bounds__(64) void core_reset_kernel(CoreStepArgs a, const uint8_t* mask) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    uint16_t* fl = reinterpret_cast<uint16_t*>(smem + align16((size_t)a.F * 8));
    const long long e = blockIdx.x;
    if (mask) {
        if (!mask[e]) return;   // workgroup-uniform
        for (int i = threadIdx.x; i < a.HW; i += 64) a.dff[e * a.HW + i] = 0.0f;
        for (int i = threadIdx.x; i < a.A; i += 64) a.pos[e * a.A + i] = 0xFFFFu;
    }
    for (int i = threadIdx.x; i < a.F; i += 64) fl[i] = a.free_padded[i];
    wave_sync();
    wave_reset_env(a, (uint32_t)(a.env_base + e), keys, fl, a.pos + e * a.A, threadIdx.x);
    if (threadIdx.x == 0) a.cnt[e] = a.N;
}

// Reset every env of a map whose free list does not fit the wave reset's LDS
// (big maps): one workgroup per env, keys in the env block's global scratch.
__global__ __launch_bounds__(1024) void core_block_reset_kernel(CoreStepArgs a, const uint8_t* mask) {
    __shared__ int swsum[16];
    const long long e = blockIdx.x;
    if (mask) {   // as core_reset_kernel
        if (!mask[e]) return;
        for (int i = threadIdx.x; i < a.HW; i += 1024) a.dff[e * a.HW + i] = 0.0f;
        for (int i = threadIdx.x; i < a.A; i += 1024) a.pos[e * a.A + i] = 0xFFFFu;
        __syncthreads();
    }
    const BlockCarve cv = block_carve((a.H + 2) * (a.W + 2), a.A, 1, a.F, false, false, true, true);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(a.scratch + (size_t)e * a.scratch_stride + cv.keys);
    block_place_env<1024>(a, e, keys, block_keys_cap(a.A, a.F), swsum);
    if (threadIdx.x == 0) a.cnt[e] = a.N;
}

// ===========================================================================
// Standalone update_dff (FloorFieldModel.update_dff): src -> dst, per cell.
// ===========================================================================
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

// ===========================================================================
// Host launchers.
// ===========================================================================
template <int NB, bool MT, int EW, int HT, int WT>
static hipError_t launch_wave_t(const CoreStepArgs& a, int blocks, hipStream_t s) {
    const size_t smem = core_wave_smem_bytes(a.H, a.W, a.A, a.F, MT, !MT && a.auto_reset, 4) + FFM_LDS_PAD;
    core_wave_kernel<NB, MT, EW, HT, WT><<<dim3((unsigned)blocks), dim3(256), smem, s>>>(a);
    return hipGetLastError();
}

template <int NB, bool MT, int EW, int HT, int WT>
static int occ_wave_t(const CoreStepArgs& a) {
    const size_t smem = core_wave_smem_bytes(a.H, a.W, a.A, a.F, MT, !MT && a.auto_reset, 4) + FFM_LDS_PAD;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, core_wave_kernel<NB, MT, EW, HT, WT>, 256, smem) != hipSuccess)
        return 0;
    return n;
}

// Dispatch over (NB, MT, EW, dims) for the wave kernel: op 0 = launch, 1 = occupancy.
template <int NB, bool MT, int EW>
static hipError_t wave_dims(const CoreStepArgs& a, int blocks, hipStream_t s, int op, int* occ) {
    if (a.H == 12 && a.W == 12) {
        if (op) { *occ = occ_wave_t<NB, MT, EW, 12, 12>(a); return hipSuccess; }
        return launch_wave_t<NB, MT, EW, 12, 12>(a, blocks, s);
    }
    if (op) { *occ = occ_wave_t<NB, MT, EW, 0, 0>(a); return hipSuccess; }
    return launch_wave_t<NB, MT, EW, 0, 0>(a, blocks, s);
}

static hipError_t wave_dispatch(const CoreStepArgs& a, int nb, bool mt, int blocks, hipStream_t s, int op,
                                int* occ) {
    const bool two = a.A <= 32;
    if (nb == 4) {
        if (mt) return two ? wave_dims<4, true, 2>(a, blocks, s, op, occ) : wave_dims<4, true, 1>(a, blocks, s, op, occ);
        return two ? wave_dims<4, false, 2>(a, blocks, s, op, occ) : wave_dims<4, false, 1>(a, blocks, s, op, occ);
    }
    if (mt) return two ? wave_dims<8, true, 2>(a, blocks, s, op, occ) : wave_dims<8, true, 1>(a, blocks, s, op, occ);
    return two ? wave_dims<8, false, 2>(a, blocks, s, op, occ) : wave_dims<8, false, 1>(a, blocks, s, op, occ);
}

hipError_t launch_core_wave(const CoreStepArgs& a, int nb, bool mt, int blocks, hipStream_t s) {
    return wave_dispatch(a, nb, mt, blocks, s, 0, nullptr);
}

int core_wave_blocks_per_cu(const CoreStepArgs& a, int nb, bool mt) {
    int n = 0;
    (void)wave_dispatch(a, nb, mt, 0, nullptr, 1, &n);
    return n;
}

template <int NB, bool F64, bool MT>
static hipError_t launch_block_t(const CoreStepArgs& a, int block, hipStream_t s) {
    const long long nblk = (a.E + a.K - 1) / a.K;
    if (a.scratch) {   // big maps: K = 1, state in global scratch
        const size_t smem = block_carve((a.H + 2) * (a.W + 2), a.A, 1, a.F, F64, MT, true, true).lds;
        core_block_kernel<NB, F64, MT, 1024, true><<<dim3((unsigned)nblk), dim3(1024), smem, s>>>(a);
        return hipGetLastError();
    }
    const size_t smem = core_block_smem_bytes(a.H, a.W, a.A, a.K, a.F, F64, MT, !MT && a.auto_reset);
    if (block == 512) {
        core_block_kernel<NB, F64, MT, 512, false><<<dim3((unsigned)nblk), dim3(512), smem, s>>>(a);
    } else {
        core_block_kernel<NB, F64, MT, 256, false><<<dim3((unsigned)nblk), dim3(256), smem, s>>>(a);
    }
    return hipGetLastError();
}

hipError_t launch_core_block(const CoreStepArgs& a, int nb, bool f64, bool mt, int block, hipStream_t s) {
    if (nb == 4) {
        if (f64) return mt ? launch_block_t<4, true, true>(a, block, s) : launch_block_t<4, true, false>(a, block, s);
        return mt ? launch_block_t<4, false, true>(a, block, s) : launch_block_t<4, false, false>(a, block, s);
    }
    if (f64) return mt ? launch_block_t<8, true, true>(a, block, s) : launch_block_t<8, true, false>(a, block, s);
    return mt ? launch_block_t<8, false, true>(a, block, s) : launch_block_t<8, false, false>(a, block, s);
}

hipError_t launch_core_block_reset(const CoreStepArgs& a, hipStream_t s, const uint8_t* mask) {
    core_block_reset_kernel<<<dim3((unsigned)a.E), dim3(1024), 0, s>>>(a, mask);
    return hipGetLastError();
}

hipError_t launch_core_reset(const CoreStepArgs& a, hipStream_t s, const uint8_t* mask) {
    const size_t smem = align16((size_t)(a.F > 0 ? a.F : 1) * 8) + align16((size_t)(a.N > 0 ? a.N : 1) * 2) +
                        align16((size_t)(a.F > 0 ? a.F : 1) * 2);
    core_reset_kernel<<<dim3((unsigned)a.E), dim3(64), smem, s>>>(a, mask);
    return hipGetLastError();
}

// ---- trajectory capture (model/ffm_core.py:119-133 run() / main.py:44-54 keep a copy of
// `positions` after every step; the last row of an episode is the empty one) ---------
// One wave per selected env, launched after every step.  An env whose episode counter
// moved during the step was emptied by it (and re-placed by the auto-reset): its row is
// the empty row that ended the logged episode.  An env that was already empty (no
// auto-reset) logs nothing.
__global__ __launch_bounds__(64) void core_capture_init_kernel(CoreStepArgs a, CoreCapture c) {
    const int i = (int)(blockIdx.x * 64 + threadIdx.x);
    if (i >= c.n_sel) return;
    const long long e = c.envs[i];
    c.state[3 * i] = a.episodes[e];
    c.state[3 * i + 1] = 0;
    c.state[3 * i + 2] = a.cnt[e];
}

__global__ __launch_bounds__(64) void core_capture_kernel(CoreStepArgs a, CoreCapture c) {
    const int b = (int)blockIdx.x, lane = (int)threadIdx.x;
    const long long e = c.envs[b];
    int* st = c.state + 3 * b;
    const int k = st[0], steps = st[1] + 1, last = st[2];
    const int know = a.episodes[e], n = a.cnt[e];
    const bool ended = know != k;
    const int rc = ended ? 0 : n;
    const int ph = c.phase ? c.phase[b] : 0;
    const bool log = !(rc == 0 && last == 0) && (k + ph) % c.period == 0;
    if (log) {
        unsigned long long row = 0;
        if (lane == 0) row = atomicAdd(c.n, 1ull);
        row = (unsigned long long)__shfl((long long)row, 0);
        if ((long long)row < c.cap) {
            if (lane == 0) {
                int* m = c.meta + 4 * row;
                m[0] = (int)(a.env_base + e);
                m[1] = k;
                m[2] = steps;
                m[3] = rc;
            }
            for (int j = lane; j < a.A; j += 64)
                c.cells[row * a.A + j] = j < rc ? a.pos[e * a.A + j] : (uint16_t)0xFFFF;
        }
    }
    if (lane == 0) {
        st[0] = know;
        st[1] = ended ? 0 : (rc == 0 && last == 0 ? st[1] : steps);
        st[2] = n;
    }
}

hipError_t launch_core_capture_init(const CoreStepArgs& a, const CoreCapture& c, hipStream_t s) {
    core_capture_init_kernel<<<dim3((unsigned)((c.n_sel + 63) / 64)), dim3(64), 0, s>>>(a, c);
    return hipGetLastError();
}

hipError_t launch_core_capture(const CoreStepArgs& a, const CoreCapture& c, hipStream_t s) {
    core_capture_kernel<<<dim3((unsigned)c.n_sel), dim3(64), 0, s>>>(a, c);
    return hipGetLastError();
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
