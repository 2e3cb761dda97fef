// engine.cpp -- C ABI (include/ffm_amd.h) over the HIP kernels.
//
// Owns the device state of E independent environments of one model class and
// drives the fused step kernel.  Mirrors the reference's FloorFieldModel
// (model/ffm_core.py:6-133): construction validates and uploads the map/SFF/
// params (:7-21), reset places agents (:23-26), step advances (:36-104),
// update_dff diffuses (:106-117).
#include "../../include/ffm_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.h"

namespace {
thread_local std::string g_err;
}  // namespace

namespace ffm {
// Shared with learn_engine.cpp: records the calling thread's last error.
int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace ffm

namespace {

int fail(int code, const std::string& msg) { return ffm::set_error(code, msg); }

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(FFM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

}  // namespace

struct ffm_engine {
    ffm_engine_desc d{};
    int HW = 0, F = 0, K = 1, block = 256;
    bool f64 = false, mt = false;
    bool lane = false;      // lane kernel (Philox, A <= 32, W % 4 == 0, H*W <= 256): core_lane.hip
    bool wave = false;      // wave-per-env kernel (A <= 64) vs block-per-env kernel
    int wave_blocks = 0;    // persistent grid of the wave kernel
    int lane_blocks = 0;    // persistent grid of the lane kernel
    bool group = false;     // group kernel (lane conditions at 12x12): core_group.hip
    int group_blocks = 0;   // persistent grid of the group kernel
    int group_g = 4;        // envs per group (core_group_pick_envs)
    bool multi = false;     // multi-step kernel available (lane conditions): core_multi.hip
    int multi_blocks = 0;   // its persistent grid
    int fused = 1;          // steps per launch (ffm_engine_set_fused_steps)
    float kS32 = 0, kD32 = 0, c0 = 0, c1 = 0;
    double kS64 = 0;
    uint32_t t = 0;
    uint8_t* d_map = nullptr;    // padded map codes
    void* d_sff = nullptr;       // padded SFF
    uint16_t* d_free = nullptr;
    uint16_t* d_free_padded = nullptr;
    uint16_t* d_pos = nullptr;
    int32_t* d_cnt = nullptr;
    float* d_dff = nullptr;
    float* d_tmp = nullptr;
    int32_t* d_eps = nullptr;
    unsigned long long* d_ctr = nullptr;   // [ctr_slots][4], summed on read
    size_t ctr_slots = 1;
    uint32_t* d_mt_np = nullptr;
    uint32_t* d_mt_py = nullptr;
    unsigned long long* d_dbg = nullptr;   // diagnostic counters (FFM_STAMPS builds)
    bool big = false;            // block kernel with its state in global scratch (maps beyond LDS)
    bool block_reset = false;    // placement by core_block_reset_kernel (free list beyond the wave reset's LDS)
    unsigned char* d_scratch = nullptr;    // [E][scratch_stride]
    size_t scratch_stride = 0;
    ffm::CoreCapture cap{};      // trajectory capture (n_sel = 0: off)
};

static void free_capture(ffm_engine* e) {
    void* bufs[] = {(void*)e->cap.envs, (void*)e->cap.phase, e->cap.state, e->cap.meta, e->cap.cells, e->cap.n};
    for (void* p : bufs) (void)hipFree(p);
    e->cap = ffm::CoreCapture{};
}

extern "C" {

const char* ffm_last_error(void) { return g_err.c_str(); }
int ffm_abi_version(void) { return FFM_ABI_VERSION; }

static void release(ffm_engine* e) {
    if (!e) return;
    (void)hipFree(e->d_map);
    (void)hipFree(e->d_sff);
    (void)hipFree(e->d_free);
    (void)hipFree(e->d_free_padded);
    (void)hipFree(e->d_pos);
    (void)hipFree(e->d_cnt);
    (void)hipFree(e->d_dff);
    (void)hipFree(e->d_tmp);
    (void)hipFree(e->d_eps);
    (void)hipFree(e->d_ctr);
    (void)hipFree(e->d_mt_np);
    (void)hipFree(e->d_mt_py);
    (void)hipFree(e->d_dbg);
    (void)hipFree(e->d_scratch);
    free_capture(e);
    delete e;
}

int ffm_engine_create(const ffm_engine_desc* desc, ffm_engine** out) {
    if (!desc || !out) return fail(FFM_E_INVALID, "null argument");
    *out = nullptr;
    const ffm_engine_desc& d = *desc;
    if (d.abi_version != FFM_ABI_VERSION) return fail(FFM_E_INVALID, "abi_version mismatch");
    if (d.variant != FFM_VARIANT_CORE) return fail(FFM_E_UNSUPPORTED, "only FFM_VARIANT_CORE is built");
    // Positions are u16 cell indices with 0xFFFF = none; a free cell is never on the
    // border, so up to 65,536 cells (256 x 256) every stored cell is < 0xFFFF.
    if (d.H < 3 || d.W < 3 || (long long)d.H * d.W > 65536)
        return fail(FFM_E_INVALID, "map must be at least 3x3 and at most 65536 cells");
    // the kernels divide padded cell indices (< (H + 2)(W + 2)) by W and W + 2 by multiply-high
    if (!ffm::magic_div_ok((uint64_t)(d.H + 2) * (d.W + 2), (uint32_t)d.W + 2u))
        return fail(FFM_E_INVALID, "map too large for the kernels' magic divisors");
    if (!d.map || !d.sff) return fail(FFM_E_INVALID, "map and sff are required");
    if (d.neighborhood != 4 && d.neighborhood != 8) return fail(FFM_E_INVALID, "neighborhood must be 4 or 8");
    if (d.sff_dtype != FFM_SFF_F32 && d.sff_dtype != FFM_SFF_F64) return fail(FFM_E_INVALID, "sff_dtype");
    if (d.n_envs < 1) return fail(FFM_E_INVALID, "n_envs must be >= 1");
    // the block kernel's grid codes hold a 15-bit agent index
    if (d.agent_capacity < 1 || d.agent_capacity > 32767) return fail(FFM_E_INVALID, "agent_capacity");
    if (d.n_agents < 0 || d.n_agents > d.agent_capacity) return fail(FFM_E_INVALID, "n_agents > agent_capacity");
    if (d.rng_mode != FFM_RNG_PHILOX && d.rng_mode != FFM_RNG_MT) return fail(FFM_E_INVALID, "rng_mode");
    const int H = d.H, W = d.W, HW = H * W;
    // The reference indexes neighbours without bounds checks (model/ffm_core.py:45,52):
    // agents must never stand on the outer ring, so no border cell may be free.
    std::vector<uint16_t> fl;
    for (int i = 0; i < HW; i++) {
        const int x = i / W, y = i % W;
        const bool border = x == 0 || y == 0 || x == H - 1 || y == W - 1;
        if (d.map[i] == 0) {
            if (border) return fail(FFM_E_INVALID, "free cell on the map border (walls must enclose the room)");
            fl.push_back((uint16_t)i);
        }
    }
    if (d.n_agents > (int)fl.size())
        return fail(FFM_E_INVALID, "Cannot take a larger sample than population when 'replace=False'");

    ffm_engine* e = new ffm_engine();
    e->d = d;
    e->d.map = nullptr;
    e->d.sff = nullptr;
    e->HW = HW;
    e->F = (int)fl.size();
    e->f64 = d.sff_dtype == FFM_SFF_F64;
    e->mt = d.rng_mode == FFM_RNG_MT;
    // NumPy weak-scalar promotion (NEP 50): python numbers become float32 next
    // to a float32 array (model/ffm_core.py:77,109,113).
    e->kS32 = (float)(-d.k_S);
    e->kD32 = (float)d.k_D;
    e->kS64 = -d.k_S;
    e->c0 = (float)((1.0 - d.decay) * (1.0 - d.diffuse));
    e->c1 = (float)(d.decay * (1.0 - d.diffuse) / (double)d.neighborhood);

    auto cleanup = [&](int rc) {
        release(e);
        return rc;
    };
    hipError_t he = hipSetDevice(d.device);
    if (he != hipSuccess) return cleanup(fail(FFM_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he)));

    // Kernel choice.  Small envs (A <= 64, float32 SFF): one wave per env or
    // env pair, persistent grid.  Otherwise (or when envs_per_block > 0 forces
    // it): K envs per workgroup, LDS-bounded.
    const int A = d.agent_capacity;
    const bool reset_lds = !e->mt && d.auto_reset;
    const int EW = A <= 32 ? 2 : 1;
    // envs_per_block: 0 = auto (lane kernel, else wave kernel, where they fit; else
    // block kernel), > 0 = block kernel with that many envs per workgroup,
    // -1 = wave kernel, -2 = lane kernel, -3 = group kernel.
    const bool lane_ok = !e->mt && !e->f64 && A <= 32 && W % 4 == 0 && HW <= 256 &&
                         ((long long)d.n_envs + 7) * HW * 4 < (1ll << 31);   // 32-bit buffer offsets (padded envs)
    e->group = (d.envs_per_block == 0 || d.envs_per_block == -3) && lane_ok && ffm::core_group_supported(H, W) &&
               ffm::core_group_smem_bytes(H, W, e->F, 4) <= 64 * 1024;
    e->multi = lane_ok && ffm::core_multi_smem_bytes(H, W, e->F, 4) <= 64 * 1024;
    e->lane = !e->group && (d.envs_per_block == 0 || d.envs_per_block == -2) && lane_ok &&
              ffm::core_lane_smem_bytes(H, W, e->F, 4) <= 64 * 1024;
    e->wave = !e->lane && !e->group && (d.envs_per_block == 0 || d.envs_per_block == -1) && A <= 64 && !e->f64 && W % 4 == 0 && EW * HW <= 512 &&
              ffm::core_wave_smem_bytes(H, W, A, e->F, e->mt, reset_lds, 4) <= 64 * 1024;
    e->block = A > 256 ? 512 : 256;
    if (const char* bs = getenv("FFM_BLOCK_BS"))     // A/B switch: the block kernel's workgroup size
        if (atoi(bs) == 256 || atoi(bs) == 512) e->block = atoi(bs);
    int K = d.envs_per_block > 0 ? d.envs_per_block : std::max(1, 256 / A);
    if (e->mt) K = 1;
    while (K > 1 && ffm::core_block_smem_bytes(H, W, A, K, e->F, e->f64, e->mt, reset_lds) > 64 * 1024) K--;
    e->K = K;
    // Maps whose env state exceeds the LDS, or whose padded cell indices exceed u16:
    // the block kernel keeps grid, DFF tile, cell lists and placement keys in a
    // global scratch region per block (one env per block).
    e->big = !e->wave && !e->lane && !e->group &&
             ((size_t)(H + 2) * (W + 2) > 65535 ||
              ffm::core_block_smem_bytes(H, W, A, K, e->F, e->f64, e->mt, reset_lds) > 64 * 1024);
    if (e->big) e->K = 1;
    // Philox placement of the whole free list in the wave reset's LDS, else by blocks
    auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t wave_reset_lds = al16(8 * (size_t)std::max(1, e->F)) + al16(2 * (size_t)std::max(1, d.n_agents)) +
                                  al16(2 * (size_t)std::max(1, e->F));   // launch_core_reset's carve
    e->block_reset = !e->mt && wave_reset_lds > 64 * 1024;

    const size_t E = (size_t)d.n_envs;
    const int PW = W + 2, PHW = (H + 2) * PW;
    const size_t sff_bytes = (size_t)PHW * (e->f64 ? 8 : 4);
    // Padded copies (one halo cell each side): map codes normalised to
    // 0 free / 2 blocked / 3 exit (only ==0 and ==3 matter, model/ffm_core.py:52-53,66,101).
    std::vector<uint8_t> pmap((size_t)PHW, 2);
    std::vector<double> psff64((size_t)PHW, 0.0);
    std::vector<float> psff32((size_t)PHW, 0.0f);
    for (int x = 0; x < H; x++)
        for (int y = 0; y < W; y++) {
            const int i = x * W + y, p = (x + 1) * PW + y + 1;
            pmap[p] = d.map[i] == 0 ? 0 : d.map[i] == 3 ? 3 : 2;
            if (e->f64) psff64[p] = reinterpret_cast<const double*>(d.sff)[i];
            else psff32[p] = reinterpret_cast<const float*>(d.sff)[i];
        }
#define ALLOC(p, n)                                                                                   \
    do {                                                                                              \
        he = hipMalloc((void**)&(p), (n));                                                            \
        if (he != hipSuccess) return cleanup(fail(FFM_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(he))); \
    } while (0)
    ALLOC(e->d_map, (size_t)PHW);
    ALLOC(e->d_sff, sff_bytes);
    ALLOC(e->d_free, std::max<size_t>(1, fl.size()) * 2);
    ALLOC(e->d_free_padded, std::max<size_t>(1, fl.size()) * 2);
    // pos / cnt / DFF hold whole groups of 8 envs (zeroed padding beyond n_envs): the group kernel
    // reads and writes a partial last group through whole-array buffer resources (core_group.hip)
    const size_t Ep = (E + 7) & ~(size_t)7;
    ALLOC(e->d_pos, Ep * A * 2 + 16);   // + a dword: the lane kernel streams positions as dwords
    ALLOC(e->d_cnt, Ep * 4);
    ALLOC(e->d_dff, Ep * HW * 4);
    ALLOC(e->d_eps, E * 4);
    if (e->big || e->block_reset) {
        e->scratch_stride = (ffm::core_big_scratch_bytes(H, W, A, e->F, e->mt) + 255) & ~(size_t)255;
        ALLOC(e->d_scratch, E * e->scratch_stride);
    }
    // Grids.  Persistent wave and lane kernels: CUs x resident blocks per CU.
    int cus = 0;
    he = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d.device);
    if (he != hipSuccess) return cleanup(fail(FFM_E_HIP, "hipDeviceGetAttribute"));
    {
        ffm::CoreStepArgs a{};
        a.H = H; a.W = W; a.A = A; a.F = e->F; a.auto_reset = reset_lds;
        if (e->wave) {
            const int per_cu = std::max(1, ffm::core_wave_blocks_per_cu(a, d.neighborhood, e->mt));
            const long long groups = (d.n_envs + EW - 1) / EW;
            e->wave_blocks = (int)std::min<long long>((groups + 3) / 4, (long long)cus * per_cu);
            if (const char* ov = std::getenv("FFM_WAVE_BLOCKS")) {   // diagnostic override of the grid
                const long long v = std::atoll(ov);
                if (v > 0) e->wave_blocks = (int)std::min<long long>(v, (groups + 3) / 4);
            }
        }
        if (e->lane) {
            const int per_cu = std::max(1, ffm::core_lane_blocks_per_cu(a, d.neighborhood));
            const long long groups = (d.n_envs + 1) / 2;
            e->lane_blocks = (int)std::max<long long>(1, std::min<long long>((groups + 3) / 4, (long long)cus * per_cu));
            if (const char* ov = std::getenv("FFM_WAVE_BLOCKS")) {   // diagnostic override of the grid
                const long long v = std::atoll(ov);
                if (v > 0) e->lane_blocks = (int)std::min<long long>(v, (groups + 3) / 4);
            }
            // every wave steps at most core_lane_max_pairs_per_wave() pairs (its deferred
            // reset mask); beyond that the grid grows past one resident wave of blocks
            const long long per_wave = ffm::core_lane_max_pairs_per_wave();
            e->lane_blocks = (int)std::max<long long>(e->lane_blocks, (groups + 4 * per_wave - 1) / (4 * per_wave));
        }
        if (e->multi) {
            const int per_cu = std::max(1, ffm::core_multi_blocks_per_cu(a, d.neighborhood));
            const long long pairs = (d.n_envs + 1) / 2;
            e->multi_blocks = (int)std::max<long long>(1, std::min<long long>((pairs + 3) / 4, (long long)cus * per_cu));
        }
        if (e->group) {
            e->group_g = ffm::core_group_pick_envs(a, d.neighborhood, d.n_envs, cus);
            const int per_cu = std::max(1, ffm::core_group_blocks_per_cu(a, d.neighborhood, e->group_g));
            const long long G = e->group_g;
            const long long groups = (d.n_envs + G - 1) / G;
            // at most 6 blocks (6 waves per SIMD) per CU: the group kernel fits 7 (71 VGPRs), but 7
            // waves per SIMD step slower (65,536 envs 36.0 vs 33.0 us, 32,768 envs 23.1 vs 21.6 us),
            // and fewer blocks than 6 per CU are slower too (1,366 blocks 36.5 us; 1,024 blocks at
            // 32,768 envs 23.6 us): profiles/r06/c2/ab_grid_balance*.log, ab_occupancy7.log
            const long long bpc = std::min(per_cu, 6);
            e->group_blocks = (int)std::max<long long>(1, std::min<long long>((groups + 3) / 4, (long long)cus * bpc));
            if (const char* ov = std::getenv("FFM_WAVE_BLOCKS")) {   // diagnostic override of the grid
                const long long v = std::atoll(ov);
                if (v > 0) e->group_blocks = (int)std::min<long long>(v, (groups + 3) / 4);
            }
            // every wave steps at most core_group_max_iters() groups (its deferred-reset mask)
            const long long per_wave = ffm::core_group_max_iters();
            e->group_blocks = (int)std::max<long long>(e->group_blocks, (groups + 4 * per_wave - 1) / (4 * per_wave));
        }
    }
    // One counter slot per wave (wave / lane kernel) or block (block kernel):
    // summed by ffm_engine_get_counters, never contended on the device.
    {
        const long long groups = (d.n_envs + EW - 1) / EW;
        const long long blocks = (d.n_envs + K - 1) / K;
        e->ctr_slots = (size_t)std::max<long long>(std::max<long long>(std::max<long long>(1, blocks),
                                                                       (groups + 3) / 4 * 4),
                                                   (long long)std::max(std::max(e->lane_blocks, e->group_blocks), e->multi_blocks) * 4);
    }
    ALLOC(e->d_ctr, e->ctr_slots * 32);
    ALLOC(e->d_dbg, 16 * 8);
    if (e->mt) {
        ALLOC(e->d_mt_np, E * 625 * 4);
        ALLOC(e->d_mt_py, E * 625 * 4);
    }
#undef ALLOC
    he = hipMemcpy(e->d_map, pmap.data(), PHW, hipMemcpyHostToDevice);
    if (he == hipSuccess)
        he = hipMemcpy(e->d_sff, e->f64 ? (const void*)psff64.data() : (const void*)psff32.data(), sff_bytes,
                       hipMemcpyHostToDevice);
    if (he == hipSuccess && !fl.empty()) he = hipMemcpy(e->d_free, fl.data(), fl.size() * 2, hipMemcpyHostToDevice);
    if (he == hipSuccess && !fl.empty()) {
        std::vector<uint16_t> fp(fl.size());
        for (size_t i = 0; i < fl.size(); i++) fp[i] = (uint16_t)((fl[i] / W + 1) * PW + fl[i] % W + 1);
        he = hipMemcpy(e->d_free_padded, fp.data(), fp.size() * 2, hipMemcpyHostToDevice);
    }
    if (he == hipSuccess) he = hipMemset(e->d_pos, 0xFF, Ep * A * 2);
    if (he == hipSuccess) he = hipMemset(e->d_cnt, 0, Ep * 4);
    if (he == hipSuccess) he = hipMemset(e->d_dff, 0, Ep * HW * 4);
    if (he == hipSuccess) he = hipMemset(e->d_eps, 0, E * 4);
    if (he == hipSuccess) he = hipMemset(e->d_ctr, 0, e->ctr_slots * 32);
    if (he == hipSuccess) he = hipMemset(e->d_dbg, 0, 128);
    if (he == hipSuccess && e->mt) he = hipMemset(e->d_mt_np, 0, E * 625 * 4);
    if (he == hipSuccess && e->mt) he = hipMemset(e->d_mt_py, 0, E * 625 * 4);
    if (he != hipSuccess) return cleanup(fail(FFM_E_HIP, std::string("init: ") + hipGetErrorString(he)));
    *out = e;
    return FFM_OK;
}

int ffm_engine_destroy(ffm_engine* e) {
    if (!e) return FFM_OK;
    (void)hipSetDevice(e->d.device);
    (void)hipDeviceSynchronize();
    release(e);
    return FFM_OK;
}

static ffm::CoreStepArgs make_args(ffm_engine* e) {
    ffm::CoreStepArgs a{};
    a.mW = ffm::magic_div((uint32_t)e->d.W);
    a.mPW = ffm::magic_div((uint32_t)e->d.W + 2u);
    a.H = e->d.H;
    a.W = e->d.W;
    a.HW = e->HW;
    a.A = e->d.agent_capacity;
    a.K = e->K;
    a.E = e->d.n_envs;
    a.env_base = e->d.env_base;
    a.pos = e->d_pos;
    a.cnt = e->d_cnt;
    a.dff = e->d_dff;
    a.episodes = e->d_eps;
    a.counters = e->d_ctr;
    a.pmap = e->d_map;
    a.psff = e->d_sff;
    a.kS32 = e->kS32;
    a.kD32 = e->kD32;
    a.kS64 = e->kS64;
    a.c0 = e->c0;
    a.c1 = e->c1;
    a.key0 = (uint32_t)e->d.seed;
    a.key1 = (uint32_t)(e->d.seed >> 32);
    a.t = e->t;
    a.auto_reset = e->d.auto_reset && !e->mt;
    a.N = e->d.n_agents;
    a.free_list = e->d_free;
    a.free_padded = e->d_free_padded;
    a.F = e->F;
    a.mt_np = e->d_mt_np;
    a.mt_py = e->d_mt_py;
    a.dbg = e->d_dbg;
    a.scratch = e->big ? e->d_scratch : nullptr;
    a.scratch_stride = e->scratch_stride;
    return a;
}

int ffm_engine_step(ffm_engine* e, int32_t n_steps, void* stream) {
    if (!e || n_steps < 0) return fail(FFM_E_INVALID, "bad engine/n_steps");
    hipStream_t s = (hipStream_t)stream;
    if (e->fused > 1 && e->multi && e->cap.n_sel == 0) {
        // k steps per launch, the state of each env pair on chip (core_multi.hip)
        for (int done = 0; done < n_steps;) {
            const int k = std::min(e->fused, n_steps - done);
            ffm::CoreStepArgs a = make_args(e);
            HIP_TRY(ffm::launch_core_multi(a, e->d.neighborhood, k, e->multi_blocks, s));
            e->t += (uint32_t)k;
            done += k;
        }
        return FFM_OK;
    }
    for (int i = 0; i < n_steps; i++) {
        ffm::CoreStepArgs a = make_args(e);
        if (e->group) HIP_TRY(ffm::launch_core_group(a, e->d.neighborhood, e->group_blocks, s, e->group_g));
        else if (e->lane) HIP_TRY(ffm::launch_core_lane(a, e->d.neighborhood, e->lane_blocks, s));
        else if (e->wave) HIP_TRY(ffm::launch_core_wave(a, e->d.neighborhood, e->mt, e->wave_blocks, s));
        else HIP_TRY(ffm::launch_core_block(a, e->d.neighborhood, e->f64, e->mt, e->block, s));
        if (e->cap.n_sel) HIP_TRY(ffm::launch_core_capture(a, e->cap, s));
        e->t++;
    }
    return FFM_OK;
}

int ffm_engine_set_fused_steps(ffm_engine* e, int32_t k) {
    if (!e || k < 1) return fail(FFM_E_INVALID, "fused steps must be >= 1");
    e->fused = k;
    return FFM_OK;
}

int ffm_engine_reset(ffm_engine* e, void* stream) {
    if (!e) return fail(FFM_E_INVALID, "null engine");
    hipStream_t s = (hipStream_t)stream;
    const size_t E = (size_t)e->d.n_envs;
    HIP_TRY(hipMemsetAsync(e->d_dff, 0, E * e->HW * 4, s));
    HIP_TRY(hipMemsetAsync(e->d_cnt, 0, E * 4, s));
    HIP_TRY(hipMemsetAsync(e->d_pos, 0xFF, E * e->d.agent_capacity * 2, s));
    HIP_TRY(hipMemsetAsync(e->d_eps, 0, E * 4, s));   // episodes count from this reset
    if (e->mt) {   // the caller uploads positions drawn from its own MT stream
        if (e->cap.n_sel) HIP_TRY(ffm::launch_core_capture_init(make_args(e), e->cap, s));
        return FFM_OK;
    }
    // Philox placement, same stream as the in-kernel auto-reset (key: current t).
    if (e->block_reset) {
        ffm::CoreStepArgs a = make_args(e);
        a.scratch = e->d_scratch;
        HIP_TRY(ffm::launch_core_block_reset(a, s));
    } else {
        HIP_TRY(ffm::launch_core_reset(make_args(e), s));
    }
    e->t++;
    if (e->cap.n_sel) HIP_TRY(ffm::launch_core_capture_init(make_args(e), e->cap, s));
    return FFM_OK;
}

int ffm_engine_reset_envs(ffm_engine* e, const uint8_t* mask, void* stream) {
    if (!e || !mask) return fail(FFM_E_INVALID, "null engine or mask");
    if (e->mt) return fail(FFM_E_UNSUPPORTED, "reset_envs: MT mode places agents on the host (set_state)");
    hipStream_t s = (hipStream_t)stream;
    // the masked envs only: Philox placement keyed by the current t (as ffm_engine_reset),
    // DFF row zeroed, count = N; the episode counters are left alone (not an episode end)
    if (e->block_reset) {
        ffm::CoreStepArgs a = make_args(e);
        a.scratch = e->d_scratch;
        HIP_TRY(ffm::launch_core_block_reset(a, s, mask));
    } else {
        HIP_TRY(ffm::launch_core_reset(make_args(e), s, mask));
    }
    e->t++;
    return FFM_OK;
}

int ffm_engine_update_dff(ffm_engine* e, void* stream) {
    if (!e) return fail(FFM_E_INVALID, "null engine");
    hipStream_t s = (hipStream_t)stream;
    const size_t n = (size_t)e->d.n_envs * e->HW;
    if (!e->d_tmp) HIP_TRY(hipMalloc((void**)&e->d_tmp, n * 4));
    HIP_TRY(ffm::launch_update_dff(e->d_dff, e->d_tmp, e->d.n_envs, e->d.H, e->d.W, e->d.neighborhood, e->c0,
                                   e->c1, s));
    HIP_TRY(hipMemcpyAsync(e->d_dff, e->d_tmp, n * 4, hipMemcpyDeviceToDevice, s));
    return FFM_OK;
}

static int check_range(ffm_engine* e, int64_t env0, int64_t n) {
    if (!e) return fail(FFM_E_INVALID, "null engine");
    if (env0 < 0 || n < 0 || env0 + n > e->d.n_envs) return fail(FFM_E_INVALID, "env range out of bounds");
    return FFM_OK;
}

int ffm_engine_set_state(ffm_engine* e, int64_t env0, int64_t n, const uint16_t* positions,
                         const int32_t* counts, const float* dff, void* stream) {
    int rc = check_range(e, env0, n);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int A = e->d.agent_capacity;
    if (counts) {
        for (int64_t i = 0; i < n; i++)
            if (counts[i] < 0 || counts[i] > A) return fail(FFM_E_INVALID, "count out of [0, agent_capacity]");
    }
    if (positions && counts) {
        // Positions must be distinct passable, non-exit cells (the reference never
        // holds an agent on an exit: model/ffm_core.py:101-102).
        const int PW = e->d.W + 2, PHW = (e->d.H + 2) * PW;
        std::vector<uint8_t> pmap(PHW);
        HIP_TRY(hipMemcpy(pmap.data(), e->d_map, PHW, hipMemcpyDeviceToHost));
        std::vector<uint8_t> seen(e->HW, 0);
        for (int64_t i = 0; i < n; i++) {
            for (int j = 0; j < counts[i]; j++) {
                const uint16_t c = positions[i * A + j];
                if (c >= e->HW || pmap[(c / e->d.W + 1) * PW + c % e->d.W + 1] != 0)
                    return fail(FFM_E_INVALID, "agent on a non-free cell");
                if (seen[c]) return fail(FFM_E_INVALID, "two agents on one cell");
                seen[c] = 1;
            }
            for (int j = 0; j < counts[i]; j++) seen[positions[i * A + j]] = 0;
        }
    }
    if (positions)
        HIP_TRY(hipMemcpyAsync(e->d_pos + env0 * A, positions, (size_t)n * A * 2, hipMemcpyHostToDevice, s));
    if (counts) HIP_TRY(hipMemcpyAsync(e->d_cnt + env0, counts, (size_t)n * 4, hipMemcpyHostToDevice, s));
    if (dff)
        HIP_TRY(hipMemcpyAsync(e->d_dff + env0 * e->HW, dff, (size_t)n * e->HW * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_engine_get_state(ffm_engine* e, int64_t env0, int64_t n, uint16_t* positions, int32_t* counts,
                         float* dff, void* stream) {
    int rc = check_range(e, env0, n);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int A = e->d.agent_capacity;
    if (positions)
        HIP_TRY(hipMemcpyAsync(positions, e->d_pos + env0 * A, (size_t)n * A * 2, hipMemcpyDeviceToHost, s));
    if (counts) HIP_TRY(hipMemcpyAsync(counts, e->d_cnt + env0, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (dff)
        HIP_TRY(hipMemcpyAsync(dff, e->d_dff + env0 * e->HW, (size_t)n * e->HW * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_engine_set_mt_state(ffm_engine* e, int64_t env, const uint32_t* np_key, int32_t np_pos,
                            const uint32_t* py_key, int32_t py_pos, void* stream) {
    int rc = check_range(e, env, 1);
    if (rc) return rc;
    if (!e->mt) return fail(FFM_E_INVALID, "engine is not in MT mode");
    if (np_pos < 0 || np_pos > 624 || py_pos < 0 || py_pos > 624) return fail(FFM_E_INVALID, "MT position");
    hipStream_t s = (hipStream_t)stream;
    uint32_t buf[1250];
    std::memcpy(buf, np_key, 624 * 4);
    buf[624] = (uint32_t)np_pos;
    std::memcpy(buf + 625, py_key, 624 * 4);
    buf[1249] = (uint32_t)py_pos;
    HIP_TRY(hipMemcpyAsync(e->d_mt_np + env * 625, buf, 625 * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(e->d_mt_py + env * 625, buf + 625, 625 * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_engine_get_mt_state(ffm_engine* e, int64_t env, uint32_t* np_key, int32_t* np_pos, uint32_t* py_key,
                            int32_t* py_pos, void* stream) {
    int rc = check_range(e, env, 1);
    if (rc) return rc;
    if (!e->mt) return fail(FFM_E_INVALID, "engine is not in MT mode");
    hipStream_t s = (hipStream_t)stream;
    uint32_t buf[1250];
    HIP_TRY(hipMemcpyAsync(buf, e->d_mt_np + env * 625, 625 * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(buf + 625, e->d_mt_py + env * 625, 625 * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(np_key, buf, 624 * 4);
    *np_pos = (int32_t)buf[624];
    std::memcpy(py_key, buf + 625, 624 * 4);
    *py_pos = (int32_t)buf[1249];
    return FFM_OK;
}

int ffm_engine_set_trajectory_capture(ffm_engine* e, const int32_t* envs, const int32_t* phases, int32_t n_sel,
                                      int32_t period, int64_t capacity_rows, void* stream) {
    if (!e) return fail(FFM_E_INVALID, "null engine");
    if (n_sel < 0 || (n_sel > 0 && (!envs || period < 1 || capacity_rows < 1)))
        return fail(FFM_E_INVALID, "trajectory capture: envs, period >= 1 and capacity_rows >= 1 are required");
    for (int32_t i = 0; i < n_sel; i++) {
        if (envs[i] < 0 || envs[i] >= e->d.n_envs) return fail(FFM_E_INVALID, "trajectory capture: env out of range");
        if (phases && phases[i] < 0) return fail(FFM_E_INVALID, "trajectory capture: phase must be >= 0");
    }
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipStreamSynchronize(s));        // queued steps may still write the old buffers
    free_capture(e);
    if (n_sel == 0) return FFM_OK;
    ffm::CoreCapture& c = e->cap;
    const size_t A = (size_t)e->d.agent_capacity;
    int* de = nullptr; int* dp = nullptr;
    hipError_t he = hipMalloc((void**)&de, (size_t)n_sel * 4);
    if (he == hipSuccess && phases) he = hipMalloc((void**)&dp, (size_t)n_sel * 4);
    c.envs = de; c.phase = dp;
    if (he == hipSuccess) he = hipMalloc((void**)&c.state, (size_t)n_sel * 12);
    if (he == hipSuccess) he = hipMalloc((void**)&c.meta, (size_t)capacity_rows * 16);
    if (he == hipSuccess) he = hipMalloc((void**)&c.cells, (size_t)capacity_rows * A * 2);
    if (he == hipSuccess) he = hipMalloc((void**)&c.n, 8);
    if (he != hipSuccess) {
        free_capture(e);
        return fail(FFM_E_NOMEM, std::string("trajectory capture: ") + hipGetErrorString(he));
    }
    c.cap = capacity_rows; c.period = period;
    HIP_TRY(hipMemcpyAsync(de, envs, (size_t)n_sel * 4, hipMemcpyHostToDevice, s));
    if (dp) HIP_TRY(hipMemcpyAsync(dp, phases, (size_t)n_sel * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(c.n, 0, 8, s));
    c.n_sel = n_sel;
    HIP_TRY(ffm::launch_core_capture_init(make_args(e), c, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_engine_drain_trajectory(ffm_engine* e, int32_t* meta, uint16_t* cells, int64_t cap, int64_t* n,
                                int64_t* dropped, void* stream) {
    if (!e || !n) return fail(FFM_E_INVALID, "null argument");
    *n = 0;
    if (dropped) *dropped = 0;
    if (e->cap.n_sel == 0) return FFM_OK;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long c = 0;
    HIP_TRY(hipMemcpyAsync(&c, e->cap.n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const long long have = std::min<long long>((long long)c, e->cap.cap);
    if (have > cap) {
        *n = have;
        return fail(FFM_E_INVALID, "drain_trajectory: buffer too small (*n holds the count)");
    }
    const size_t A = (size_t)e->d.agent_capacity;
    if (have > 0 && meta) HIP_TRY(hipMemcpyAsync(meta, e->cap.meta, (size_t)have * 16, hipMemcpyDeviceToHost, s));
    if (have > 0 && cells) HIP_TRY(hipMemcpyAsync(cells, e->cap.cells, (size_t)have * A * 2, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemsetAsync(e->cap.n, 0, 8, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n = have;
    if (dropped) *dropped = (int64_t)c - have;
    return FFM_OK;
}

int ffm_engine_get_counters(ffm_engine* e, uint64_t* counters, void* stream) {
    if (!e || !counters) return fail(FFM_E_INVALID, "null argument");
    hipStream_t s = (hipStream_t)stream;
    std::vector<unsigned long long> c(e->ctr_slots * 4);
    HIP_TRY(hipMemcpyAsync(c.data(), e->d_ctr, e->ctr_slots * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int i = 0; i < 4; i++) counters[i] = 0;
    for (size_t j = 0; j < e->ctr_slots; j++)
        for (int i = 0; i < 4; i++) counters[i] += c[j * 4 + i];
    return FFM_OK;
}

int ffm_engine_device_buffers(ffm_engine* e, ffm_device_buffers* out) {
    if (!e || !out) return fail(FFM_E_INVALID, "null argument");
    out->positions = e->d_pos;
    out->counts = e->d_cnt;
    out->dff = e->d_dff;
    out->episodes = e->d_eps;
    out->counters = reinterpret_cast<uint64_t*>(e->d_ctr);
    out->mt_np = e->d_mt_np;
    out->mt_py = e->d_mt_py;
    out->counter_slots = (int64_t)e->ctr_slots;
    return FFM_OK;
}

int ffm_engine_get_step_index(ffm_engine* e, uint32_t* t) {
    if (!e || !t) return fail(FFM_E_INVALID, "null argument");
    *t = e->t;
    return FFM_OK;
}

int ffm_engine_set_step_index(ffm_engine* e, uint32_t t) {
    if (!e) return fail(FFM_E_INVALID, "null engine");
    e->t = t;
    return FFM_OK;
}

// Diagnostic (not part of the ABI header): read the FFM_STAMPS counters.
int ffm_debug_read(ffm_engine* e, uint64_t* out, int n) {
    if (!e || !out || n < 0 || n > 16) return fail(FFM_E_INVALID, "bad args");
    HIP_TRY(hipMemcpy(out, e->d_dbg, (size_t)n * 8, hipMemcpyDeviceToHost));
    return FFM_OK;
}

int ffm_np_expf_device(const float* x, float* y, int64_t n, void* stream) {
    HIP_TRY(ffm::launch_np_expf(x, y, n, (hipStream_t)stream));
    return FFM_OK;
}

}  // extern "C"
