// core_pack.hip -- the C2 hot kernel: one step of model/ffm_core.py
// FloorFieldModel.step() (:36-117) for every env, Philox mode, envs packed onto
// wavefront lanes by their live agent count.
//
// Why packing: agents leave as they exit, so an env of capacity A holds ~A/2
// live agents on average (17.8 of 32 at C2).  The wave kernel (core_step.hip)
// gives every env A fixed lanes, so half the lanes of the agent phases idle.
// Here a wave takes a *bundle* of up to NMAX consecutive envs whose live
// agents fit in 64 lanes, packed back to back: lane -> (bundle slot s, agent
// index al).  At C2 that is 0.34 bundles per env instead of 0.5 env pairs.
//
// Per wave: a contiguous range of <= 64 envs (counts at step start read once
// into a VGPR; bundles planned greedily from them, wave-uniform).  Bundle
// state arrives by LDS-DMA (global_load_lds, no VGPRs) into one of two
// buffers, issued during the previous bundle's resolve/stencil.  DFF tiles are
// the global layout verbatim ([s][H][W] floats, unpadded): the stencil masks
// its borders; the occupancy grids are padded ([s][(H+2)(W+2)] u8 codes).
//
// Semantics and RNG streams are identical to core_step.hip,
// so both kernels, and the oracle, agree bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "core_common.h"
#include "kernels.h"
#include "wave_reset.h"

#ifndef FFM_STAMPS
#define FFM_STAMPS 0
#endif
#if FFM_STAMPS   // diagnostic: per-phase s_memtime cycle sums (tools/stamps.py)
#define PSTAMP(k)                                                                  \
    do {                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                         \
        unsigned long long t_;                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                         \
        st[k] += t_ - tlast;                                                       \
        tlast = t_;                                                                \
    } while (0)
#elif !defined(FFM_PACK_MARKS)
#define PSTAMP(k) \
    do {          \
    } while (0)
#else   // diagnostic: phase markers in the ISA (tools/phase_count.py --pack)
#define PSTAMP(k)                                  \
    do {                                           \
        __builtin_amdgcn_sched_barrier(0);         \
        asm volatile("; @PHASE " #k ::: "memory"); \
        __builtin_amdgcn_sched_barrier(0);         \
    } while (0)
#endif

namespace ffm {

typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* gbl_void_t;

__host__ __device__ inline size_t pk_align16(size_t x) { return (x + 15) & ~(size_t)15; }

struct PackCarve {
    size_t dbuf0, dbuf1, pbuf0, pbuf1, grid, req, nxt, fric, keys, per_wave;
};

__host__ __device__ inline PackCarve pack_carve(int HW, int PHW, int A, int F, int nmax, bool reset) {
    PackCarve c;
    size_t o = 0;
    c.dbuf0 = o; o += pk_align16((size_t)nmax * HW * 4);     // DFF of the bundle, global layout
    c.dbuf1 = o; o += pk_align16((size_t)nmax * HW * 4);
    // positions [s][A]: u16 (A even: dword DMA), or one dword per u16 (A odd: the
    // u16 LDS-DMA writes a dword per lane)
    const size_t pbytes = (size_t)nmax * A * ((A & 1) ? 4 : 2);
    c.pbuf0 = o; o += pk_align16(pbytes);
    c.pbuf1 = o; o += pk_align16(pbytes);
    c.grid = o;  o += pk_align16((size_t)nmax * PHW);        // u8 occupancy codes, padded
    c.req = o;   o += 128;                                   // u16 per lane
    c.nxt = o;   o += 128;
    c.fric = o;  o += 512;                                   // uint2 per lane: friction words
    c.keys = o;  o += reset ? pk_align16((size_t)F * 8) : 0; // last: the only runtime-sized region
    c.per_wave = o;
    return c;
}

// Block-shared: padded map codes, padded SFF (f32), padded free-cell list.
__host__ __device__ inline size_t pack_shared_bytes(int PHW, int F) {
    return pk_align16((size_t)PHW) + pk_align16((size_t)PHW * 4) + pk_align16((size_t)F * 2);
}

size_t core_pack_smem_bytes(int H, int W, int A, int F, int nmax, bool reset, int waves) {
    const int PHW = (H + 2) * (W + 2);
    return pack_shared_bytes(PHW, F) + (size_t)waves * pack_carve(H * W, PHW, A, F, nmax, reset).per_wave;
}

// Bundle plan from env j of the wave's range (wave-uniform): n envs whose
// counts (lanes of cntv) sum to <= 64; bo[k] = first lane of slot k (bo[k] =
// total for k >= n).
template <int NMAX>
__device__ __forceinline__ void pack_plan(int j, int R, int cntv, int& n, int (&bo)[NMAX + 1]) {
    n = 0;
    int tot = 0;
    bo[0] = 0;
#pragma unroll
    for (int k = 0; k < NMAX; k++) {
        const int jj = j + k < 63 ? j + k : 63;
        const int c = __builtin_amdgcn_readlane(cntv, jj);
        const bool take = n == k && j + k < R && tot + c <= 64;
        tot += take ? c : 0;
        n += take ? 1 : 0;
        bo[k + 1] = tot;
    }
}

template <int NB, int NMAX, int HT, int WT>
__global__ __launch_bounds__(256) void core_pack_kernel(CoreStepArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    using GT = uint8_t;
    const int H = HT ? HT : a.H, W = WT ? WT : a.W;
    const int HW = H * W, PW = W + 2, PHW = (H + 2) * PW;
    constexpr int kDWS = -2;   // DFF tile row stride (W) minus grid row stride (W + 2)
    const int A = a.A;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool do_reset = a.auto_reset != 0;

    const PackCarve cv = pack_carve(HW, PHW, A, a.F, NMAX, do_reset);
    uint8_t* pmap = smem;
    float* psff = reinterpret_cast<float*>(smem + pk_align16((size_t)PHW));
    uint16_t* pfree = reinterpret_cast<uint16_t*>(smem + pk_align16((size_t)PHW) + pk_align16((size_t)PHW * 4));
    unsigned char* wbase = smem + pack_shared_bytes(PHW, a.F) + (size_t)wv * cv.per_wave;
    GT* grid = reinterpret_cast<GT*>(wbase + cv.grid);
    uint16_t* sreq = reinterpret_cast<uint16_t*>(wbase + cv.req);
    uint16_t* snxt = reinterpret_cast<uint16_t*>(wbase + cv.nxt);
    uint2* sfric = reinterpret_cast<uint2*>(wbase + cv.fric);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(wbase + cv.keys);

    // This wave's env range [r0, r1), at most 64 envs (host sizes the grid).
    const long long nw = (long long)gridDim.x * 4;
    const long long w = (long long)blockIdx.x * 4 + wv;
    const long long r0 = w * a.E / nw, r1 = (w + 1) * a.E / nw;
    const int R = (int)(r1 - r0);
    const int cntv = lane < R ? a.cnt[r0 + lane] : 0;   // counts at step start

    // LDS-DMA of bundle (j, n) into buffer b: DFF as 16-B pieces, positions as
    // dwords (A even) or u16 (A odd); lane-linear, as the global layout is.
    auto dma = [&](int j, int n, int b) {
        unsigned char* db = wbase + (b ? cv.dbuf1 : cv.dbuf0);
        unsigned char* pb = wbase + (b ? cv.pbuf1 : cv.pbuf0);
        const float4* src = reinterpret_cast<const float4*>(a.dff + (r0 + j) * HW);
        const int n4 = n * HW / 4;
        for (int p = 0; p * 64 < n4; p++)
            if (p * 64 + lane < n4)
                __builtin_amdgcn_global_load_lds((gbl_void_t)(src + p * 64 + lane), (lds_void_t)(db + p * 1024), 16, 0, 0);
        const uint16_t* ps = a.pos + (r0 + j) * A;
        if ((A & 1) == 0) {
            const int nw32 = n * A / 2;
            const uint32_t* ps32 = reinterpret_cast<const uint32_t*>(ps);
            for (int p = 0; p * 64 < nw32; p++)
                if (p * 64 + lane < nw32)
                    __builtin_amdgcn_global_load_lds((gbl_void_t)(ps32 + p * 64 + lane), (lds_void_t)(pb + p * 256), 4, 0, 0);
        } else {
            const int nw16 = n * A;
            for (int p = 0; p * 64 < nw16; p++)
                if (p * 64 + lane < nw16)
                    __builtin_amdgcn_global_load_lds((gbl_void_t)(ps + p * 64 + lane), (lds_void_t)(pb + p * 256), 2, 0, 0);
        }
    };

    int n = 0, bo[NMAX + 1];
    pack_plan<NMAX>(0, R, cntv, n, bo);
    if (R > 0) dma(0, n, 0);
    for (int i = threadIdx.x; i < PHW; i += 256) {
        pmap[i] = a.pmap[i];
        psff[i] = reinterpret_cast<const float*>(a.psff)[i];
    }
    for (int i = threadIdx.x; i < a.F; i += 256) pfree[i] = a.free_padded[i];
    __syncthreads();
    for (int i = lane; i < NMAX * PHW; i += 64) grid[i] = pmap[i - (i / PHW) * PHW];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();

    unsigned c_steps = 0, c_exits = 0, c_resets = 0;   // wave-uniform
#if FFM_STAMPS
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tlast = __builtin_amdgcn_s_memtime();
#endif
    int j = 0, b = 0;
    while (j < R) {
        const long long e0 = r0 + j;   // first env of the bundle
        float* db = reinterpret_cast<float*>(wbase + (b ? cv.dbuf1 : cv.dbuf0));
        const uint16_t* pb = reinterpret_cast<const uint16_t*>(wbase + (b ? cv.pbuf1 : cv.pbuf0));
        const int tot = bo[NMAX];

        // lane -> (slot s, agent al); lanes >= tot are idle
        int s = 0;
#pragma unroll
        for (int k = 1; k < NMAX; k++) s += lane >= bo[k] ? 1 : 0;
        int bs = 0;
#pragma unroll
        for (int k = 1; k < NMAX; k++) bs = s == k ? bo[k] : bs;
        const bool live = lane < tot;
        const int al = lane - bs;
        GT* gk = grid + s * PHW;
        float* dk = db + s * HW;
        const uint32_t genv = (uint32_t)(a.env_base + e0 + s);

        int pp = -1, dd0 = 0;
        if (live) {
            const int c = (A & 1) ? (int)(reinterpret_cast<const uint32_t*>(pb)[s * A + al] & 0xFFFFu)
                                  : (int)pb[s * A + al];
            const int x = c / W, y = c - (c / W) * W;
            pp = (x + 1) * PW + y + 1;
            dd0 = c - pp;   // DFF tile index = grid index + dd0 + kDWS per row below
        }
        c_steps += (unsigned)tot;

        // Next bundle: plan, then its LDS-DMA into the other buffer (in flight
        // during this whole bundle; waited before the stores).  LDS-DMA holds no
        // VGPRs, so it can be issued this early.
        const int j2 = j + n;
        int n2 = 0, bo2[NMAX + 1];
        pack_plan<NMAX>(j2, R, cntv, n2, bo2);
        if (j2 < R) dma(j2, n2, b ^ 1);
        PSTAMP(0);

        // ---- occupancy marks; default next = stay -----------------------------------
        if (live) gk[pp] = (GT)(GridCodes<GT>::kAgent | (uint32_t)al);
        sreq[lane] = kNoReq;
        snxt[lane] = (uint16_t)(live ? pp : 0);
        wave_sync();
        PSTAMP(1);

        // ---- decide (model/ffm_core.py:40-88) ------------------------------------------
        uint32_t r = kNoReq;
        if (live) {
            const uint4 pbk = philox(make_uint4(a.t, genv, (uint32_t)al, kPurDecide << 28), a.key0, a.key1);
            sfric[lane] = make_uint2(pbk.z, pbk.w);   // friction words (owner of a contest)
            r = slot_cell<NB>(decide<NB, false, GT>(pp, PW, gk, psff, nullptr, dk, dd0, kDWS, a.kS32, a.kD32, a.kS64,
                                                    DrawFixed{u53(pbk.x, pbk.y)}),
                              pp, PW);
        }
        PSTAMP(2);

        if (live) sreq[lane] = (uint16_t)r;
        wave_sync();
        PSTAMP(3);

        // ---- resolve (model/ffm_core.py:90-98) -----------------------------------------
        uint16_t* rqe = sreq + bs;   // this env's requests / next cells, by agent index
        uint16_t* nxe = snxt + bs;
        {
            uint16_t who[NB];
            bool is[NB];
            const bool moving = live && r != kNoReq && (int)r != pp;
            int m = 0, s0 = -1;
            bool owner = false;
            if (moving) {
                m = requesters<NB, GT>((int)r, PW, gk, rqe, who, is);
                s0 = kth_slot<NB>(who, is, 0);
                owner = s0 >= 0 && who[s0] == al;
            }
            if (live && r != kNoReq) {
                if ((int)r == pp) {
                    dk[pp + dd0] += 1.0f;                                                     // :91-93 (stay)
                } else if (owner) {
                    int ws = -1;
                    if (m == 1) {
                        ws = s0;
                    } else {
                        const uint2 f = sfric[lane];
                        const int kk = philox_friction(f.x, f.y, (uint32_t)m, a.key0, a.key1, a.t, genv, (uint32_t)al);
                        if (kk >= 0) ws = kth_slot<NB>(who, is, kk);                           // :95-96
                    }
                    if (ws >= 0) {
                        int wcell = (int)r;
                        uint16_t wi = 0;
#pragma unroll
                        for (int q = 0; q < NB; q++)
                            if (q == ws) {
                                wcell = (int)r - nb_dx<NB>(q) * PW - nb_dy<NB>(q);
                                wi = who[q];
                            }
                        nxe[wi] = (uint16_t)r;
                        dk[wcell + (wcell / PW) * kDWS + (dd0 - (pp / PW) * kDWS)] += 1.0f;    // :97-98
                    }
                }
            }
        }
        wave_sync();
        PSTAMP(4);

        // ---- exits: order-preserving compaction per env (model/ffm_core.py:100-102) ------
        const int nxt = live ? (int)snxt[lane] : 0;
        const bool keep = live && pmap[nxt] != 3;
        const unsigned long long km = __ballot(keep);
        int kb[NMAX + 1];   // kept lanes below each slot's first lane (wave-uniform)
#pragma unroll
        for (int k = 0; k <= NMAX; k++)
            kb[k] = bo[k] >= 64 ? __popcll(km) : __popcll(km & ((1ull << bo[k]) - 1ull));
        int kbs = 0;
#pragma unroll
        for (int k = 1; k < NMAX; k++) kbs = s == k ? kb[k] : kbs;
        const int newidx = lanes_below(km) - kbs;
        c_exits += (unsigned)(tot - __popcll(km));
        if (live) gk[pp] = 0;   // unmark
        // slots emptied by this step reset at the end of the bundle (wave-uniform mask)
        unsigned rsm = 0;
#pragma unroll
        for (int k = 0; k < NMAX; k++) rsm |= (do_reset && k < n && kb[k + 1] == kb[k]) ? (1u << k) : 0u;
        c_resets += (unsigned)__popc(rsm);
        PSTAMP(5);

        // ---- update_dff (model/ffm_core.py:106-117) over the bundle's n*HW cells --------
        // Pass 1: B = c0 * D in place (:109).  Pass 2: per float4 slot, rows x-1, x,
        // x+1 of B with the map border masked to 0 (np.pad, :111).
        const int n4 = n * HW / 4;
        constexpr int kPass = (NMAX * (HT ? HT * WT : 4096) / 4 + 63) / 64;   // upper bound of passes
        for (int p = 0; p * 64 < n4; p++) {
            const int q = p * 64 + lane;
            if (q < n4) {
                float4* pq = reinterpret_cast<float4*>(db) + q;
                const float4 v = *pq;
                *pq = make_float4(a.c0 * v.x, a.c0 * v.y, a.c0 * v.z, a.c0 * v.w);
            }
        }
        wave_sync();
        float o[kPass > 4 ? 4 : kPass][4];
        const int W4 = W / 4;
#pragma unroll
        for (int p = 0; p < (kPass > 4 ? 4 : kPass); p++) {
            const int q = p * 64 + lane;
            if (q < n4) {
                const int qs = q / (HW / 4), qc = q - qs * (HW / 4);
                const int x = qc / W4, y = (qc - x * W4) * 4;
                const float* pc = db + 4 * q;
                float v[3][6];
#pragma unroll
                for (int dx = -1; dx <= 1; dx++) {
                    const bool rowok = dx == 0 || (dx < 0 ? x > 0 : x < H - 1);
                    const float4 r4 = *reinterpret_cast<const float4*>(pc + (rowok ? dx * W : 0));
                    const float lf = pc[(rowok ? dx * W : 0) - (y > 0 ? 1 : 0)];
                    const float rt = pc[(rowok ? dx * W : 0) + (y + 4 < W ? 4 : 3)];
                    v[dx + 1][0] = rowok && y > 0 ? lf : 0.0f;
                    v[dx + 1][1] = rowok ? r4.x : 0.0f;
                    v[dx + 1][2] = rowok ? r4.y : 0.0f;
                    v[dx + 1][3] = rowok ? r4.z : 0.0f;
                    v[dx + 1][4] = rowok ? r4.w : 0.0f;
                    v[dx + 1][5] = rowok && y + 4 < W ? rt : 0.0f;
                }
                const bool zero = (rsm >> qs) & 1u;   // env reset this step: next episode starts at 0
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    float acc = v[1][jj + 1];
#pragma unroll
                    for (int k = 0; k < NB; k++) {
                        const float t = a.c1 * v[1 + nb_dx<NB>(k)][jj + 1 + nb_dy<NB>(k)];    // :113
                        acc = acc + t;
                    }
                    o[p][jj] = (acc < 1e-4f || zero) ? 0.0f : acc;                          // :116-117
                }
            }
        }
        PSTAMP(6);

        // ---- the next bundle's data has landed: stores ---------------------------------------
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        float4* gd = reinterpret_cast<float4*>(a.dff + e0 * HW);
#pragma unroll
        for (int p = 0; p < (kPass > 4 ? 4 : kPass); p++) {
            const int q = p * 64 + lane;
            if (q < n4) gd[q] = make_float4(o[p][0], o[p][1], o[p][2], o[p][3]);
        }
        if (keep) a.pos[(e0 + s) * A + newidx] = (uint16_t)unpad(nxt, PW);
        if (lane < n) {
            int nc = 0;
#pragma unroll
            for (int k = 0; k < NMAX; k++) nc = lane == k ? kb[k + 1] - kb[k] : nc;
            const bool rl = (rsm >> lane) & 1u;
            a.cnt[e0 + lane] = rl ? a.N : nc;
            if (rl && a.episodes) a.episodes[e0 + lane] += 1;
        }
        // ---- auto-reset, straight to the env's global positions -------------
        if (rsm) {
#pragma unroll
            for (int k = 0; k < NMAX; k++)
                if ((rsm >> k) & 1u)
                    wave_reset_env(a, (uint32_t)(a.env_base + e0 + k), keys, pfree, a.pos + (e0 + k) * A, lane);
        }
        wave_sync();
        PSTAMP(7);

        j = j2;
        n = n2;
#pragma unroll
        for (int k = 0; k <= NMAX; k++) bo[k] = bo2[k];
        b ^= 1;
    }

    if (lane == 0) {
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

// ---- host ---------------------------------------------------------------------------------
template <int NB, int NMAX, int HT, int WT>
static hipError_t pack_op(const CoreStepArgs& a, int blocks, hipStream_t s, int op, int* occ) {
    const size_t smem = core_pack_smem_bytes(a.H, a.W, a.A, a.F, NMAX, a.auto_reset != 0, 4);
    if (op) {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, core_pack_kernel<NB, NMAX, HT, WT>, 256, smem) != hipSuccess)
            v = 0;
        *occ = v;
        return hipSuccess;
    }
    core_pack_kernel<NB, NMAX, HT, WT><<<dim3((unsigned)blocks), dim3(256), smem, s>>>(a);
    return hipGetLastError();
}

static hipError_t pack_dispatch(const CoreStepArgs& a, int nb, int blocks, hipStream_t s, int op, int* occ) {
    if (a.H == 12 && a.W == 12)
        return nb == 4 ? pack_op<4, 4, 12, 12>(a, blocks, s, op, occ) : pack_op<8, 4, 12, 12>(a, blocks, s, op, occ);
    return nb == 4 ? pack_op<4, 4, 0, 0>(a, blocks, s, op, occ) : pack_op<8, 4, 0, 0>(a, blocks, s, op, occ);
}

hipError_t launch_core_pack(const CoreStepArgs& a, int nb, int blocks, hipStream_t s) {
    return pack_dispatch(a, nb, blocks, s, 0, nullptr);
}

int core_pack_blocks_per_cu(const CoreStepArgs& a, int nb) {
    int n = 0;
    (void)pack_dispatch(a, nb, 0, nullptr, 1, &n);
    return n;
}

}  // namespace ffm
