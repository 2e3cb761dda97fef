// core_multi.hip -- K consecutive Philox ffm_core steps per launch for the small
// envs of the lane kernel (A <= 32, W % 4 == 0, H * W <= 256, float32 SFF).
//
// ffm_engine_step(e, n) advances every env by n FloorFieldModel.step() calls
// (model/ffm_core.py:36-117).  The single-step kernels pay, every step, a launch
// (ramp, prologue, tail: about 11 us of the 38 us C2 step) and the
// HBM round trip of the state.  Envs are independent, so nothing forces a global
// barrier between two steps of one env: here a wavefront loads an env pair once,
// steps it K times with the state resident on chip, and stores it once.
//
//  * DFF: the pair's zero-halo tile in LDS; each step's stencil results go back
//    into the tile after every lane has read its operands;
//  * positions: one register per agent lane; the order-preserving exit
//    compaction (model/ffm_core.py:100-102) permutes them through a 64-entry LDS
//    row (kept agent -> its new index);
//  * auto-reset happens inline at the end of the step that
//    emptied the env, with that step's t, straight into the LDS row: the next
//    step of the same env needs the placement;
//  * draws, arithmetic and phase order are those of core_lane_kernel, step for
//    step (t = a.t + k), so K fused steps equal K single-step launches bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "core_common.h"
#include "kernels.h"
#include "lane_common.h"
#include "wave_reset.h"

namespace ffm {

namespace {

struct MultiCarve {
    size_t grid, tile, words, keys, posb, per_wave;
};

__host__ __device__ inline MultiCarve multi_carve(int PHW, int TS, int F) {
    MultiCarve c;
    size_t o = 0;
    c.grid = o;  o += a16((size_t)(2 * PHW) * 2);
    c.tile = o;  o += a16((size_t)(2 * TS) * 4);
    c.words = o; o += 64 * 8;
    c.keys = o;  o += a16((size_t)(F > 0 ? F : 1) * 8);
    c.posb = o;  o += 64 * 2;
    c.per_wave = a16(o);
    return c;
}

__host__ __device__ inline size_t multi_shared_bytes(int PHW, int F) {
    return a16((size_t)PHW) + a16((size_t)PHW * 4) + a16((size_t)(F > 0 ? F : 1) * 2);
}

}  // namespace

#ifndef FFM_MULTI_WAVES
#define FFM_MULTI_WAVES 1   // minimum waves per SIMD asked of the register allocator
#endif

template <int NB, int HT, int WT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FFM_MULTI_WAVES, 8)))
void core_multi_kernel(CoreStepArgs a, int nsteps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = HT ? HT : a.H, W = WT ? WT : a.W;
    const int HW = H * W, PW = W + 2, PHW = (H + 2) * PW;
    const int TS = lane_tile_floats(H, W);
    const int A = a.A;
    const int lane = (int)(threadIdx.x & 63);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int sub = lane >> 5, al = lane & 31;

    const MultiCarve cv = multi_carve(PHW, TS, a.F);
    uint8_t* pmap = smem;
    float* psff = reinterpret_cast<float*>(smem + a16((size_t)PHW));
    uint16_t* pfree = reinterpret_cast<uint16_t*>(smem + a16((size_t)PHW) + a16((size_t)PHW * 4));
    unsigned char* wbase = smem + multi_shared_bytes(PHW, a.F) + (size_t)wv * cv.per_wave;
    uint16_t* grid = reinterpret_cast<uint16_t*>(wbase + cv.grid);
    float* const tile = reinterpret_cast<float*>(wbase + cv.tile);
    uint2* words = reinterpret_cast<uint2*>(wbase + cv.words);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(wbase + cv.keys);
    uint16_t* const posb = reinterpret_cast<uint16_t*>(wbase + cv.posb);
    uint16_t* gk = grid + sub * PHW;
    float* const dk = tile + sub * TS;

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
    const bool yl0 = tb0 >= 0 && ((tb0 - 4) % TS) % W == 0, yr0 = tb0 >= 0 && ((tb0 - 4) % TS) % W == W - 4;
    const bool yl1 = tb1 >= 0 && ((tb1 - 4) % TS) % W == 0, yr1 = tb1 >= 0 && ((tb1 - 4) % TS) % W == W - 4;
    const int zs0 = min((4 * lane) / HW, 2), zs1 = min((4 * (lane + 64)) / HW, 2);

    const int E32 = (int)a.E;   // host-checked: E * H * W * 4 < 2^31
    const uint32_t ebase = (uint32_t)a.env_base;
    const int ngroups = (E32 + 1) / 2;
    const int wstride = (int)gridDim.x * 4;

    for (int i = threadIdx.x; i < PHW; i += 256) {
        pmap[i] = a.pmap[i];
        psff[i] = reinterpret_cast<const float*>(a.psff)[i];
    }
    for (int i = threadIdx.x; i < a.F; i += 256) pfree[i] = a.free_padded[i];
    for (int i = lane; i < 2 * TS; i += 64) tile[i] = 0.0f;
    __syncthreads();
    for (int i = lane; i < 2 * PHW; i += 64) grid[i] = pmap[i - (i / PHW) * PHW];
    wave_sync();

    unsigned long long c_steps = 0, c_exits = 0, c_resets = 0;
    const uint32_t mW = (uint32_t)(((1ull << 32) + (unsigned)W - 1) / (unsigned)W);   // x = c / W for c < 2^16

    for (int g = (int)blockIdx.x * 4 + wv; g < ngroups; g += wstride) {
        const int e0 = g * 2;
        const int nenv = min(E32 - e0, 2);
        const bool env_ok = sub < nenv;
        const uint32_t genv = ebase + (uint32_t)(e0 + sub);
        const __amdgpu_buffer_rsrc_t rc = pair_rsrc(a.cnt + e0, nenv * 4);
        const __amdgpu_buffer_rsrc_t rp = pair_rsrc(a.pos + (long long)e0 * A, nenv * A * 2);
        const __amdgpu_buffer_rsrc_t rd = pair_rsrc(a.dff + (long long)e0 * HW, nenv * HW * 4);
        int cnt = (int)__builtin_amdgcn_raw_buffer_load_b32(rc, sub * 4, 0, 0);
        uint32_t cpos = __builtin_amdgcn_raw_buffer_load_b16(rp, al < A ? (sub * A + al) * 2 : kOOB, 0, 0);
        float4 o0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, 16 * lane, 0, 0));
        float4 o1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, 16 * lane + 1024, 0, 0));
        if (tb0 >= 0) *reinterpret_cast<float4*>(tile + tb0) = o0;
        if (tb1 >= 0) *reinterpret_cast<float4*>(tile + tb1) = o1;
        wave_sync();

        for (int k = 0; k < nsteps; k++) {
            const uint32_t t = a.t + (uint32_t)k;

            // ---- agent cell and occupancy mark ------------------------------------------
            const bool live = env_ok && al < cnt;
            const int x = (int)__umulhi(cpos, mW);
            const int y = (int)cpos - x * W;
            const int pp = live ? (x + 1) * PW + y + 1 : PW + 1;
            const int dd0 = 3 - (x + 1) * 2;
            uint16_t* const mine = gk + pp;
            if (live) *mine = (uint16_t)(DirCodes::kAgent | (uint32_t)al | (DirCodes::kNoDir << 8));
            {
                const int c0 = __builtin_amdgcn_readlane(cnt, 0), c1 = __builtin_amdgcn_readlane(cnt, 32);
                c_steps += (unsigned)(c0 + (nenv > 1 ? c1 : 0));
            }
            wave_sync();

            // ---- decide (model/ffm_core.py:40-88) ---------------------------------------
            const uint4 pb = philox(make_uint4(t, genv, (uint32_t)al, kPurDecide << 28), a.key0, a.key1);
            words[lane] = make_uint2(pb.z, pb.w);
            bool to_exit = false;
            uint32_t slot = lane_decide<NB>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, pb.x, to_exit);
            slot = live ? slot : kNoReq;
            if (slot == kPending)
                slot = NB == 4 ? lane_decide_exact<NB>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, u53(pb.x, pb.y))
                               : lane_decide_exact_arr<NB>(pp, PW, gk, psff, dk, dd0, a.kS32, a.kD32, u53(pb.x, pb.y));
            if (live)
                *mine = (uint16_t)(DirCodes::kAgent | (uint32_t)al |
                                   ((slot <= (uint32_t)NB ? slot : DirCodes::kNoDir) << 8));
            wave_sync();

            // ---- resolve (model/ffm_core.py:90-98), by each requester --------------------
            const int r = (int)slot_cell<NB>(slot, pp, PW);
            const bool req = slot <= (uint32_t)NB;
            const bool moving = req && r != pp;
            bool granted = req && !moving;
            {
                const int rt = moving ? r : pp;
                int m = 0, kr = 0, o = 0x7F;
#pragma unroll
                for (int s = 0; s < NB; s++) {
                    const uint32_t c = gk[rt - nb_dx<NB>(s) * PW - nb_dy<NB>(s)];
                    const bool is = (c & DirCodes::kAgent) != 0u && ((c >> 8) & 0xFu) == (uint32_t)s;
                    const int who = (int)(c & DirCodes::kIdx);
                    m += is ? 1 : 0;
                    kr += (is && who < al) ? 1 : 0;
                    o = (is && who < o) ? who : o;
                }
                if (moving) {
                    if (m == 1) {
                        granted = true;
                    } else {
                        const uint2 f = words[sub * 32 + o];
                        const int kk = philox_friction(f.x, f.y, (uint32_t)m, a.key0, a.key1, t, genv, (uint32_t)o);
                        granted = kk == kr;
                    }
                }
            }
            if (granted) __hip_atomic_fetch_add(dk + pp + dd0, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            const int np = granted ? r : pp;

            // ---- exits: order-preserving compaction (model/ffm_core.py:100-102) -----------
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
            if (live) *mine = 0;
            if (keep) posb[sub * 32 + newidx] = (uint16_t)unpad(np, PW);
            const bool rs = a.auto_reset && env_ok && newcnt == 0;
            const unsigned long long rsm = __ballot(rs);
            if (rsm) {   // wave-uniform, rare: re-place at the end of this step, keyed by its t
                c_resets += (unsigned)(((rsm & 1ull) ? 1 : 0) + ((rsm >> 32) & 1ull ? 1 : 0));
                if (a.episodes && al == 0 && rs) a.episodes[e0 + sub] += 1;
                CoreStepArgs ak = a;
                ak.t = t;
                wave_sync();
                for (int s = 0; s < 2; s++)
                    if ((rsm >> (32 * s)) & 1ull) wave_reset_env(ak, ebase + (uint32_t)(e0 + s), keys, pfree, posb + s * 32, lane);
            }
            cnt = rs ? a.N : newcnt;
            wave_sync();
            cpos = posb[lane];

            // ---- update_dff (model/ffm_core.py:106-117) back into the tile ------------------
            auto stencil = [&](int tb, bool yl, bool yr, float4& out) {
                const float* p = tile + tb;
                float b[3][6];
#pragma unroll
                for (int dx = -1; dx <= 1; dx++) {
                    const float4 u = *reinterpret_cast<const float4*>(p + dx * W);
                    b[dx + 1][1] = a.c0 * u.x; b[dx + 1][2] = a.c0 * u.y;
                    b[dx + 1][3] = a.c0 * u.z; b[dx + 1][4] = a.c0 * u.w;
                    if (NB == 4 && dx != 0) continue;
                    b[dx + 1][0] = a.c0 * tile[yl ? 0 : tb + dx * W - 1];
                    b[dx + 1][5] = a.c0 * tile[yr ? 0 : tb + dx * W + 4];
                }
                float ov[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float acc = b[1][j + 1];
#pragma unroll
                    for (int s = 0; s < NB; s++) {
                        const float tt = a.c1 * b[1 + nb_dx<NB>(s)][j + 1 + nb_dy<NB>(s)];
                        acc = acc + tt;
                    }
                    ov[j] = acc < 1e-4f ? 0.0f : acc;
                }
                out = make_float4(ov[0], ov[1], ov[2], ov[3]);
            };
            o0 = make_float4(0.f, 0.f, 0.f, 0.f);
            o1 = o0;
            if (tb0 >= 0) stencil(tb0, yl0, yr0, o0);
            if (tb1 >= 0) stencil(tb1, yl1, yr1, o1);
            {
                const bool r0 = (rsm & 1ull) != 0, r1 = (rsm >> 32) != 0;
                const bool z0 = zs0 == 0 ? r0 : (zs0 == 1 && r1), z1 = zs1 == 0 ? r0 : (zs1 == 1 && r1);
                if (z0) o0 = make_float4(0.f, 0.f, 0.f, 0.f);
                if (z1) o1 = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            wave_sync();   // every lane has read its stencil operands
            if (tb0 >= 0) *reinterpret_cast<float4*>(tile + tb0) = o0;
            if (tb1 >= 0) *reinterpret_cast<float4*>(tile + tb1) = o1;
            wave_sync();
        }

        // ---- store the pair -------------------------------------------------------------
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)cpos, rp, (env_ok && al < cnt) ? (sub * A + al) * 2 : kOOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)cnt, rc, al == 0 ? sub * 4 : kOOB, 0, 0);
        buf_st4(rd, 16 * lane, o0);
        buf_st4(rd, 16 * lane + 1024, o1);
    }

    if (lane == 0) {
        unsigned long long* ctr = a.counters + 4 * ((size_t)blockIdx.x * 4 + wv);
        if (c_steps) atomicAdd(&ctr[0], c_steps);
        if (c_exits) atomicAdd(&ctr[1], c_exits);
        if (c_resets) atomicAdd(&ctr[2], c_resets);
        if (blockIdx.x == 0 && wv == 0) atomicAdd(&ctr[3], (unsigned long long)nsteps);
    }
}

size_t core_multi_smem_bytes(int H, int W, int F, int waves) {
    const int PHW = (H + 2) * (W + 2);
    return multi_shared_bytes(PHW, F) + (size_t)waves * multi_carve(PHW, lane_tile_floats(H, W), F).per_wave;
}

template <int NB, int HT, int WT>
static hipError_t multi_op(const CoreStepArgs& a, int nsteps, int blocks, hipStream_t s, int op, int* occ) {
    const size_t smem = core_multi_smem_bytes(a.H, a.W, a.F, 4);
    if (op) {
        *occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, core_multi_kernel<NB, HT, WT>, 256, smem) != hipSuccess)
            *occ = 0;
        return hipSuccess;
    }
    if (a.A > 32 || a.N > 32 || a.W % 4 != 0 || a.H * a.W > 256 || nsteps < 1)
        return hipErrorInvalidConfiguration;   // shapes the kernel assumes
    core_multi_kernel<NB, HT, WT><<<dim3((unsigned)blocks), dim3(256), smem, s>>>(a, nsteps);
    return hipGetLastError();
}

static hipError_t multi_dispatch(const CoreStepArgs& a, int nb, int nsteps, int blocks, hipStream_t s, int op, int* occ) {
    if (a.H == 12 && a.W == 12)
        return nb == 4 ? multi_op<4, 12, 12>(a, nsteps, blocks, s, op, occ)
                       : multi_op<8, 12, 12>(a, nsteps, blocks, s, op, occ);
    return nb == 4 ? multi_op<4, 0, 0>(a, nsteps, blocks, s, op, occ) : multi_op<8, 0, 0>(a, nsteps, blocks, s, op, occ);
}

hipError_t launch_core_multi(const CoreStepArgs& a, int nb, int nsteps, int blocks, hipStream_t s) {
    return multi_dispatch(a, nb, nsteps, blocks, s, 0, nullptr);
}

int core_multi_blocks_per_cu(const CoreStepArgs& a, int nb) {
    int n = 0;
    (void)multi_dispatch(a, nb, 1, 0, nullptr, 1, &n);
    return n;
}

}  // namespace ffm
