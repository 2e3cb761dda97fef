// learn_engine.cpp -- C ABI (include/ffm_amd.h, ffm_learner_*) over the
// learning-variant kernels of learn_step.hip.
//
// Mirrors the reference's learning classes: model/ffm_ac_core.py
// FloorFieldModel, model/ffm_unified.py FloorFieldModelUnified and
// model/ffm_actor_only.py FloorFieldModelActorOnly.  One learner holds E envs
// and one V table and one H table shared by all of them (the drivers run one
// env and keep the tables across episodes, e.g.
// run_unified_actor_training.py:270-300).
#include "../../include/ffm_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "learn_kernels.h"

namespace ffm {
int set_error(int code, const std::string& msg);
}

namespace {

int fail(int code, const std::string& msg) { return ffm::set_error(code, msg); }

#define HIP_TRY(expr)                                                                           \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(FFM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

struct DevTable {
    ffm::LearnTable t{};
    int width = 1;
    int accw = 1;      // accumulator words per slot: V 2 (sum of td, visits), H 5
    size_t cap = 0;
};

}  // namespace

struct ffm_learner {
    ffm_engine_desc d{};
    ffm_learn_desc L{};
    bool mt = false, f64 = false, actor = false, post_update = false;
    bool trained = false;              // ffm_trained_core: H read only, no learning
    int HW = 0, F = 0, D = 1;
    float smin = 0, smax = 0;
    uint32_t t = 0;
    int cur = 0;                       // which DFF buffer is current
    uint8_t* d_map = nullptr;
    uint32_t* d_map2 = nullptr;              // 2-bit packed map (learn_step.hip map_at)
    void* d_sff = nullptr;
    uint16_t* d_free_cells = nullptr;
    uint16_t* d_pos = nullptr;
    int32_t* d_cnt = nullptr;
    float* d_dff[2] = {nullptr, nullptr};
    int32_t* d_eps = nullptr;
    int32_t* d_ep_steps = nullptr;
    int32_t* d_done = nullptr;
    int32_t* d_nstart = nullptr;
    int32_t* d_epcap = nullptr;              // ffm_learner_set_episode_caps (nullptr: no quota)
    unsigned long long* d_ctr = nullptr;
    double* d_hstat = nullptr;
    double* d_hpart = nullptr;
    ffm::LearnRec* d_recs = nullptr;
    int32_t* d_overflow = nullptr;
    int32_t* h_overflow = nullptr;     // pinned: d_overflow as of the end of the last ffm_learner_step
    uint32_t* d_mt_np = nullptr;
    uint32_t* d_mt_py = nullptr;
    unsigned char* d_scratch = nullptr;
    uint32_t dense_bx = 0;             // dense tables: x blocks (import validation)
    bool hstat_valid = false;          // d_hstat holds the H statistics of the current table
    long long hx_n = 0;                // ffm_learner_set_h_extra: values outside the table
    int hx_nf = 0;
    double hx_mn = 0.0, hx_mx = 0.0;
    int phase = 0;                     // batched step in phases: 0 idle, 1 local done, 2 V applied
    unsigned long long* d_count = nullptr;   // delta export record counter
    int32_t* d_eplog = nullptr;              // [eplog_cap][4] ended episodes
    unsigned long long* d_eplog_n = nullptr;
    long long eplog_cap = 0;
    int F_all = 0;                           // free cells of the map (placement capacity)
    ffm::TrajCapture traj{};                 // trajectory capture (n_sel = 0: off)
    bool v_chain = false;                    // LearnArgs::v_chain: a batched step ran since the last
                                             // set_state / V import (agents' s are the last step's s')
    // The chain holds only if every exit-forced agent wins its exit: true when no exit cell
    // has two free cells among its neighbours (one possible requester).  Otherwise a loser
    // stays on a cell whose state the reference inserts as V(s) at the next step although
    // its V(s') was never looked up (a terminal transition): make_room's Moore exits.
    bool chain_ok = true;
    int sync_period = 1;                     // tables applied every sync_period-th step
    int since_apply = 0;                     // steps since the last apply
    bool external_sync = false;              // driven by a multi-rank TableSync: no local flush
    // tiled step: ffm_unified, dense tables at block size 1, the raster
    // batch kernel; ffm_learner_step at sync period 1 (the phased multi-rank step keeps
    // the accumulators, which its exchange sums)
    int eps_phase = 0;                       // ffm_learner_set_epsilon_phase
    long long eps_stride = 1;
    bool tiled_ok = false;
    bool tstats_valid = false;               // d_tstats summarises the current H
    int NT = 0;
    ffm::TileRec* d_trecs = nullptr;
    uint16_t* d_tstart = nullptr;
    double* d_tstats = nullptr;
    int* d_tdirty = nullptr;
    int* d_tcand = nullptr;
    // tile-major records and the owner-sharded exchange
    bool tile_major = true;                  // owner exchange available (FFM_TILE_MAJOR=0: off)
    bool single_tm = false;                  // one device: tile-major passes too (FFM_TILE_MAJOR=1; env-major
                                             // is faster there: the pack costs more than the passes save)
    int ow = 1, orank = 0, ths = 0;          // ranks, this rank, header row stride
    uint32_t* d_pe = nullptr;                // [E][NT] records of tile t in envs before e
    uint32_t* d_ttot = nullptr;              // [NT] records of the tiles before t in its ownership chunk
    uint32_t* d_toff = nullptr;              // [NT] + chunk sums and offsets
    uint32_t* d_hdr = nullptr;               // [ow][ths] per destination: its tiles' record offsets
    ffm::TileRec* d_pack = nullptr;          // [E][A] records, grouped by destination, tile-major
    long long* d_xcnt = nullptr;             // [kMaxOwners + 2] records per destination
    ffm::TileRec* d_opack = nullptr;         // [ow][rcap] the owner exchange's fixed-capacity send blocks
    ffm::TileRec* x_opack = nullptr;         // an external send buffer (ffm_learner_set_owner_send_buffer)
    uint32_t* x_vslot = nullptr;             // external output buffers (ffm_learner_set_owner_output_buffers)
    double* x_vval = nullptr;
    unsigned long long* x_vn = nullptr;
    uint32_t* x_hkey = nullptr;
    long long* x_hq = nullptr;
    unsigned long long* x_hn = nullptr;
    long long rcap = 0;                      // records per destination block (set_owner_capacity)
    uint32_t* d_vslot = nullptr;             // owner outputs: vcap V values, hcap H increments
    double* d_vval = nullptr;
    uint32_t* d_hkey = nullptr;
    long long* d_hq = nullptr;
    unsigned long long* d_on = nullptr;      // [2] V / H output counts
    size_t vcap = 0, hcap = 0;
    double* d_tsum = nullptr;                // [ths][5] this rank's tile summaries
    unsigned char* d_bph = nullptr;          // the phase-split batch step's per-env state (learn_batch_phases)
    uint16_t* d_tstartT = nullptr;           // [NT + 1][E] transposed tile offsets (one-device env-major passes)
    const ffm::TileRec* own_recs = nullptr;  // the received records of the current owner step
    const uint32_t* own_hdr = nullptr;
    long long own_src = 0;                   // records between the received blocks (0: rcap)
    DevTable V, H;
};

// FFM_TSTART_T=0: the env-major tile passes read the [E][NT + 1] offsets (A/B).
static bool tstart_t_off() {
    const char* v = getenv("FFM_TSTART_T");
    return v && v[0] == '0';
}

static void free_traj(ffm_learner* l) {
    void* bufs[] = {(void*)l->traj.envs, (void*)l->traj.phase, l->traj.meta, l->traj.cells, l->traj.n};
    for (void* p : bufs) (void)hipFree(p);
    l->traj = ffm::TrajCapture{};
}

static void free_table(DevTable& T) {
    (void)hipFree(T.t.rec);
    (void)hipFree(T.t.acc);
    (void)hipFree(T.t.order);
    (void)hipFree(T.t.n);
    (void)hipFree(T.t.mark);
    (void)hipFree(T.t.present);
}

static void release(ffm_learner* l) {
    if (!l) return;
    void* bufs[] = {l->d_map, l->d_map2, l->d_sff, l->d_free_cells, l->d_pos, l->d_cnt, l->d_dff[0], l->d_dff[1],
                    l->d_eps, l->d_ep_steps, l->d_done, l->d_nstart, l->d_epcap, l->d_ctr, l->d_hstat, l->d_hpart,
                    l->d_recs, l->d_overflow, l->d_mt_np, l->d_mt_py, l->d_scratch, l->d_count,
                    l->d_eplog, l->d_eplog_n, l->d_trecs, l->d_tstart, l->d_tstats, l->d_tdirty, l->d_tcand,
                    l->d_pe, l->d_ttot, l->d_toff, l->d_hdr, l->d_pack, l->d_xcnt, l->d_opack,
                    l->d_vslot, l->d_vval, l->d_hkey, l->d_hq, l->d_on, l->d_tsum, l->d_bph, l->d_tstartT};
    for (void* p : bufs) (void)hipFree(p);
    if (l->h_overflow) (void)hipHostFree(l->h_overflow);
    free_traj(l);
    free_table(l->V);
    free_table(l->H);
    delete l;
}

// dense_by > 0: ffm_unified's rank keys map injectively onto
// ranks * (cap / 256) + bx * dense_by + by (learn_step.hip dense_slot); the capacity is
// the next power of two >= 256 * Bx * By and the table can never fill.
// width: values per record (V 1, H 5; H 9 with the Moore neighbourhood).
static hipError_t alloc_table(DevTable& T, int log2cap, int width, uint32_t dense_by = 0, size_t dense_n = 0) {
    T.width = width;
    T.accw = width == 1 ? 2 : width;
    T.t.accw = (uint32_t)T.accw;
    if (dense_by) {
        log2cap = 8;
        while (((size_t)1 << log2cap) < dense_n) log2cap++;
    }
    T.cap = (size_t)1 << log2cap;
    T.t.mask = (uint32_t)(T.cap - 1);
    T.t.dense_by = dense_by;
    T.t.limit = (uint32_t)(T.cap - T.cap / 8);
    hipError_t e;
    T.t.stride = width == 1 ? 2 : width == 5 ? 8 : 10;   // 16 / 64 / 80 B records (key + values [+ pad])
    if ((e = hipMalloc((void**)&T.t.rec, T.cap * T.t.stride * 8)) != hipSuccess) return e;
    // hashed tables: copies of the accumulators (LearnTable::reps); FFM_ACC_REPS overrides
    // (they spread the adds of hot keys over several memory-side atomic units; a large
    // table has few hot keys per slot, so the copies shrink to keep the accumulators
    // within kAccRepBytes: 4 copies up to 2^22 V slots / 2^21 H slots)
    constexpr size_t kAccRepBytes = (size_t)256 << 20;
    uint32_t reps = dense_by ? 1u : 4u;
    if (!dense_by)
        if (const char* ev = getenv("FFM_ACC_REPS")) {
            const long r = strtol(ev, nullptr, 10);
            if (r >= 1 && r <= 8 && (r & (r - 1)) == 0) reps = (uint32_t)r;   // kMaxAccReps
        }
    while (reps > 1 && T.cap * T.accw * 8 * reps > kAccRepBytes) reps >>= 1;
    T.t.reps = reps;
    T.t.rep_stride = (unsigned long long)(T.cap * T.accw);
    if ((e = hipMalloc((void**)&T.t.acc, T.cap * T.accw * 8 * reps)) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&T.t.order, T.cap * 4)) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&T.t.n, 4)) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&T.t.mark, 4)) != hipSuccess) return e;
    if (dense_by && (e = hipMalloc((void**)&T.t.present, T.cap / 8)) != hipSuccess) return e;
    return hipMemset(T.t.mark, 0, 4);
}

static ffm::LearnArgs make_args(ffm_learner* l) {
    ffm::LearnArgs a{};
    const ffm_engine_desc& d = l->d;
    a.H = d.H; a.W = d.W; a.HW = l->HW; a.A = d.agent_capacity; a.N = d.n_agents; a.F = l->F;
    a.E = d.n_envs; a.env_base = d.env_base;
    a.variant = d.variant; a.mode = l->L.mode; a.bs = d.variant == FFM_VARIANT_ACTOR_ONLY ? 5 : l->L.block_size;
    a.D = l->D;
    a.map = l->d_map;
    a.map2 = l->d_map2;
    a.sff32 = l->f64 ? nullptr : reinterpret_cast<const float*>(l->d_sff);
    a.sff64 = l->f64 ? reinterpret_cast<const double*>(l->d_sff) : nullptr;
    a.smin = l->smin; a.smax = l->smax;
    // NumPy weak-scalar promotion (NEP 50): python numbers become float32 next to
    // a float32 array (model/ffm_unified.py:361-364, 442-445).
    a.kS32 = (float)(-d.k_S); a.kD32 = (float)d.k_D; a.kS64 = -d.k_S; a.nkA = -l->L.k_A;
    a.c0 = (float)((1.0 - d.decay) * (1.0 - d.diffuse));
    a.c1 = (float)(d.decay * (1.0 - d.diffuse) / (double)d.neighborhood);
    a.nb = d.neighborhood;
    a.alpha_v = l->L.alpha_v; a.alpha_h = l->L.alpha_h; a.gamma = l->L.gamma;
    a.exit_reward = l->L.exit_reward; a.step_penalty = l->L.step_penalty;
    a.collision_penalty = l->L.collision_penalty; a.epsilon = l->L.epsilon; a.v_default = l->L.v_default;
    a.pos = l->d_pos; a.cnt = l->d_cnt;
    a.dff_in = l->d_dff[l->cur]; a.dff_out = l->d_dff[l->cur ^ 1];
    a.episodes = l->d_eps; a.ep_steps = l->d_ep_steps; a.done = l->d_done; a.nstart = l->d_nstart;
    a.ep_cap = l->d_epcap;
    a.v_chain = l->v_chain ? 1 : 0;
    a.counters = l->d_ctr;
    a.V = l->V.t; a.Ht = l->H.t;
    a.hstat = l->d_hstat; a.hpart = l->d_hpart; a.recs = l->d_recs; a.overflow = l->d_overflow;
    a.hx_n = l->hx_n; a.hx_nf = l->hx_nf; a.hx_mn = l->hx_mn; a.hx_mx = l->hx_mx;
    a.key0 = (uint32_t)d.seed; a.key1 = (uint32_t)(d.seed >> 32); a.t = l->t;
    a.auto_reset = d.auto_reset && !l->mt; a.max_steps = l->L.max_steps;
    a.mt_np = l->d_mt_np; a.mt_py = l->d_mt_py; a.scratch = l->d_scratch;
    a.free_cells = l->d_free_cells;
    a.eps_start = l->L.eps_start; a.eps_end = l->L.eps_end;
    a.eps_offset = l->L.eps_offset; a.eps_span = l->L.eps_span;
    a.eps_phase = l->eps_phase;
    a.eps_stride = l->eps_stride;
    a.eplog = l->d_eplog; a.eplog_n = l->d_eplog_n; a.eplog_cap = l->eplog_cap;
    auto magic = [](int div) { return div <= 1 ? 0u : (uint32_t)(((1ull << 32) + (unsigned)div - 1) / (unsigned)div); };
    a.mW = magic(d.W);
    a.mBS = magic(a.bs);
    a.trecs = nullptr;       // the accumulator path unless a tiled step sets it
    a.tstart = l->d_tstart;
    a.tstartT = nullptr;     // set by the one-device tiled step after its transpose
    a.tstart_out = nullptr;
    a.bph = l->d_bph;
    a.tstats = l->d_tstats;
    a.tdirty = l->d_tdirty;
    a.tcand = l->d_tcand;
    a.NT = l->NT;
    a.tile_ensure = 0;
    return a;
}

// Overflow without a host sync: a step queued a copy of the device flag into pinned
// memory behind itself; whatever of it has landed is reported (every sync point --
// counters, export, get_state -- reports it exactly through check_overflow).
static int async_overflow(ffm_learner* l) {
    const int32_t ov = l->h_overflow ? __atomic_load_n(l->h_overflow, __ATOMIC_ACQUIRE) : 0;
    if (ov & 1) return fail(FFM_E_NOMEM, "V/H hash table is full (raise log2_v_capacity / log2_h_capacity)");
    if (ov & 4) return fail(FFM_E_INVALID, "asynchronous delta export: record buffer too small (raise its capacity)");
    if (ov & 8) return fail(FFM_E_INVALID, "owner exchange: a count exceeded its buffer capacity (set_owner_capacity)");
    return FFM_OK;
}

static int check_overflow(ffm_learner* l, hipStream_t s) {
    int32_t ov = 0;
    HIP_TRY(hipMemcpyAsync(&ov, l->d_overflow, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ov & 1) return fail(FFM_E_NOMEM, "V/H hash table is full (raise log2_v_capacity / log2_h_capacity)");
    if (ov & 2) return fail(FFM_E_HIP, "placement candidate list out of range (reset)");
    if (ov & 4) return fail(FFM_E_INVALID, "asynchronous delta export: record buffer too small (raise its capacity)");
    if (ov & 8) return fail(FFM_E_INVALID, "owner exchange: a count exceeded its buffer capacity (set_owner_capacity)");
    return FFM_OK;
}

static hipError_t clear_table(ffm_learner* l, DevTable& T, double dflt, hipStream_t s) {
    hipError_t e;
    (void)l;
    if (T.t.present && (e = hipMemsetAsync(T.t.present, 0, T.cap / 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(T.t.acc, 0, T.cap * T.accw * 8 * T.t.reps, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(T.t.n, 0, 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(T.t.mark, 0, 4, s)) != hipSuccess) return e;
    return ffm::launch_learn_clear(T.t, T.width, T.width == 1 ? dflt : 0.0, s);
}

extern "C" {

int ffm_learner_create(const ffm_engine_desc* desc, const ffm_learn_desc* learn, ffm_learner** out) {
    if (!desc || !learn || !out) return fail(FFM_E_INVALID, "null argument");
    *out = nullptr;
    const ffm_engine_desc& d = *desc;
    if (d.abi_version != FFM_ABI_VERSION) return fail(FFM_E_INVALID, "abi_version mismatch");
    if (d.variant != FFM_VARIANT_AC && d.variant != FFM_VARIANT_UNIFIED && d.variant != FFM_VARIANT_ACTOR_ONLY &&
        d.variant != FFM_VARIANT_TRAINED)
        return fail(FFM_E_INVALID, "learner variant must be AC, UNIFIED, ACTOR_ONLY or TRAINED");
    if (d.variant == FFM_VARIANT_UNIFIED && (learn->mode < 0 || learn->mode > 2))
        return fail(FFM_E_INVALID, "learning_mode must be one of ['critic_only', 'actor_only', 'both']");
    // Cells are u16 indices and 0xFFFF marks "none": up to 256 x 256 cells, the
    // last one a wall (the border must be walls anyway).
    if (d.H < 3 || d.W < 3 || (long long)d.H * d.W > 65536)
        return fail(FFM_E_INVALID, "map must be at least 3x3 and at most 65536 cells");
    // cell indices (< H W) are divided by W by multiply-high (LearnArgs::mW)
    if ((uint64_t)d.H * d.W * (uint64_t)d.W > 0x100000000ull)
        return fail(FFM_E_INVALID, "map too large for the kernels' magic divisors");
    if (!d.map || !d.sff) return fail(FFM_E_INVALID, "map and sff are required");
    if ((long long)d.H * d.W == 65536 && (d.map[65535] == 0 || d.map[65535] == 3))
        return fail(FFM_E_UNSUPPORTED, "the last cell of a 65536-cell map must be blocked");
    if (d.neighborhood != 4 && d.neighborhood != 8)
        return fail(FFM_E_INVALID, "neighborhood must be 4 ('neumann') or 8 ('moore')");
    if (d.sff_dtype != FFM_SFF_F32 && d.sff_dtype != FFM_SFF_F64) return fail(FFM_E_INVALID, "sff_dtype");
    if (d.n_envs < 1) return fail(FFM_E_INVALID, "n_envs must be >= 1");
    // batched: LDS grid codes hold 14-bit agent indices (<= 16383 agents); the exact (MT) step
    // keeps int scratch and u16 cells, so the drop-in classes can hold every free cell
    if (d.agent_capacity < 1 || d.agent_capacity > (d.rng_mode == FFM_RNG_MT ? 65535 : 16383))
        return fail(FFM_E_INVALID, "agent_capacity");
    if (d.n_agents < 0 || d.n_agents > d.agent_capacity) return fail(FFM_E_INVALID, "n_agents > agent_capacity");
    if (d.rng_mode != FFM_RNG_PHILOX && d.rng_mode != FFM_RNG_MT) return fail(FFM_E_INVALID, "rng_mode");
    if (learn->block_size < 1 && d.variant != FFM_VARIANT_ACTOR_ONLY) return fail(FFM_E_INVALID, "block_size");
    const int H = d.H, W = d.W, HW = H * W;
    std::vector<uint16_t> fl;
    for (int i = 0; i < HW; i++) {
        if (d.map[i] > 3) return fail(FFM_E_UNSUPPORTED, "learning variants need map values in 0..3 (state keys)");
        const int x = i / W, y = i % W;
        const bool border = x == 0 || y == 0 || x == H - 1 || y == W - 1;
        if (d.map[i] == 0) {
            if (border) return fail(FFM_E_INVALID, "free cell on the map border (walls must enclose the room)");
            fl.push_back((uint16_t)i);
        }
    }
    if (d.n_agents > (int)fl.size())
        return fail(FFM_E_INVALID, "Cannot take a larger sample than population when 'replace=False'");
    bool chain_ok = true;
    for (int i = 0; i < HW && chain_ok; i++) {
        if (d.map[i] != 3) continue;
        const int x = i / W, y = i % W;
        int nfree = 0;
        for (int dx = -1; dx <= 1; dx++)
            for (int dy = -1; dy <= 1; dy++) {
                if ((dx == 0 && dy == 0) || (d.neighborhood == 4 && dx != 0 && dy != 0)) continue;
                const int u = x + dx, v = y + dy;
                if (u >= 0 && u < H && v >= 0 && v < W && d.map[u * W + v] == 0) nfree++;
            }
        chain_ok = nfree <= 1;
    }

    ffm_learner* l = new ffm_learner();
    l->chain_ok = chain_ok;
    l->d = d;
    l->d.map = nullptr;
    l->d.sff = nullptr;
    l->L = *learn;
    if (l->L.log2_v_capacity <= 0) l->L.log2_v_capacity = 21;
    if (l->L.log2_h_capacity <= 0) l->L.log2_h_capacity = 21;
    l->L.log2_v_capacity = std::min(std::max(l->L.log2_v_capacity, 8), 30);
    l->L.log2_h_capacity = std::min(std::max(l->L.log2_h_capacity, 8), 28);
    l->mt = d.rng_mode == FFM_RNG_MT;
    l->f64 = d.sff_dtype == FFM_SFF_F64;
    l->HW = HW;
    l->F = (int)fl.size();
    l->F_all = l->F;
    // ffm_actor_only: one decision per neighbour (4, Moore 8; model/ffm_actor_only.py:214-355)
    l->D = d.variant == FFM_VARIANT_ACTOR_ONLY ? d.neighborhood : 1;
    l->actor = d.variant == FFM_VARIANT_ACTOR_ONLY || (d.variant == FFM_VARIANT_UNIFIED && learn->mode != FFM_LEARN_CRITIC_ONLY);
    l->post_update = d.variant == FFM_VARIANT_UNIFIED && learn->mode == FFM_LEARN_ACTOR_ONLY;
    l->trained = d.variant == FFM_VARIANT_TRAINED;
    if (!l->mt && !ffm::learn_batch_supported(HW, d.agent_capacity, l->D)) {
        release(l);
        return fail(FFM_E_UNSUPPORTED, "env does not fit the batched learner's LDS budget");
    }
    // min / max of the inf->0 float32 SFF (model/ffm_unified.py:74-76, 425-426)
    {
        float mn = INFINITY, mx = -INFINITY;
        for (int i = 0; i < HW; i++) {
            const double raw = l->f64 ? reinterpret_cast<const double*>(d.sff)[i]
                                      : (double)reinterpret_cast<const float*>(d.sff)[i];
            const float v = std::isinf(raw) ? 0.0f : (float)raw;
            mn = std::min(mn, v);
            mx = std::max(mx, v);
        }
        l->smin = mn;
        l->smax = mx;
    }
    auto cleanup = [&](int rc) {
        release(l);
        return rc;
    };
    hipError_t he = hipSetDevice(d.device);
    if (he != hipSuccess) return cleanup(fail(FFM_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he)));
    const size_t E = (size_t)d.n_envs, A = (size_t)d.agent_capacity;
#define ALLOC(p, n)                                                                                   \
    do {                                                                                              \
        he = hipMalloc((void**)&(p), (n));                                                            \
        if (he != hipSuccess) return cleanup(fail(FFM_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(he))); \
    } while (0)
    ALLOC(l->d_map, (size_t)HW);
    ALLOC(l->d_map2, ((size_t)HW + 15) / 16 * 4);
    ALLOC(l->d_sff, (size_t)HW * (l->f64 ? 8 : 4));
    ALLOC(l->d_free_cells, std::max<size_t>(1, fl.size()) * 2);
    ALLOC(l->d_pos, E * A * 2);
    ALLOC(l->d_cnt, E * 4);
    ALLOC(l->d_dff[0], E * HW * 4);
    if (!l->mt) ALLOC(l->d_dff[1], E * HW * 4);
    ALLOC(l->d_eps, E * 4);
    ALLOC(l->d_ep_steps, E * 4);
    ALLOC(l->d_done, E * 4);
    ALLOC(l->d_nstart, E * 4);
    ALLOC(l->d_ctr, E * 32);
    ALLOC(l->d_hstat, 4 * 8);
    ALLOC(l->d_hpart, (size_t)ffm::kHstatBlocks * 4 * 8);
    if (l->post_update && !l->mt) ALLOC(l->d_recs, E * A * sizeof(ffm::LearnRec));
    ALLOC(l->d_overflow, 4);
    if (hipHostMalloc((void**)&l->h_overflow, 4, hipHostMallocDefault) == hipSuccess) *l->h_overflow = 0;
    else l->h_overflow = nullptr;
    ALLOC(l->d_count, 8);
    // an env ends at most one episode per step: 16 steps between drains always fit
    l->eplog_cap = std::max<long long>(16 * (long long)E, 4096);
    ALLOC(l->d_eplog, (size_t)l->eplog_cap * 16);
    ALLOC(l->d_eplog_n, 8);
    if (l->mt) {
        ALLOC(l->d_mt_np, E * 625 * 4);
        ALLOC(l->d_mt_py, E * 625 * 4);
        ALLOC(l->d_scratch, ffm::learn_exact_scratch_bytes(HW, (int)A));
    }
#undef ALLOC
    // ffm_unified / ffm_trained_core: dense tables over 256 rank codes x Bx x By blocks
    // (at most 2^28 slots).
    uint32_t dense_by = 0;
    size_t dense_n = 0;
    if (d.variant == FFM_VARIANT_UNIFIED || d.variant == FFM_VARIANT_TRAINED) {
        const size_t bs = (size_t)learn->block_size;
        const size_t bx = (size_t)(H - 1) / bs + 1, by = (size_t)(W - 1) / bs + 1;
        if (256 * bx * by <= ((size_t)1 << 28)) {
            dense_by = (uint32_t)by;
            dense_n = 256 * bx * by;
        }
    }
    l->dense_bx = dense_by ? (uint32_t)((H - 1) / learn->block_size + 1) : 0;
    l->V.t.alpha = l->L.alpha_v;   // the visit-averaged V update (learn_step.hip v_visits)
    if ((he = alloc_table(l->V, l->L.log2_v_capacity, 1, dense_by, dense_n)) != hipSuccess ||
        (he = alloc_table(l->H, l->actor || l->trained ? l->L.log2_h_capacity : 8, d.neighborhood == 8 ? 9 : 5,
                          l->actor || l->trained ? dense_by : 0, dense_n)) != hipSuccess)
        return cleanup(fail(FFM_E_NOMEM, std::string("hipMalloc (tables): ") + hipGetErrorString(he)));
    {
        const char* ev = getenv("FFM_TILED");
        // (Neumann or Moore: the tile passes take 5- or 9-value H rows; dense slots < 2^24)
        l->tiled_ok = !l->mt && d.variant == FFM_VARIANT_UNIFIED && dense_by && learn->block_size == 1 &&
                      l->V.cap <= ((size_t)1 << 24) && l->H.cap <= ((size_t)1 << 24) &&
                      ffm::learn_batch_raster(HW, d.agent_capacity, l->D) && !(ev && ev[0] == '0') &&
                      (unsigned long long)E * (unsigned long long)A < (1ull << 31);
    }
    if (l->tiled_ok) {
        l->NT = (HW + ffm::kTileCells - 1) / ffm::kTileCells;
        const char* tm = getenv("FFM_TILE_MAJOR");
        l->tile_major = !(tm && tm[0] == '0');
        l->single_tm = tm && tm[0] == '1';
        l->ths = l->NT + 1;
        if (hipMalloc((void**)&l->d_trecs, E * A * sizeof(ffm::TileRec)) != hipSuccess ||
            hipMalloc((void**)&l->d_tstart, E * (size_t)(l->NT + 1) * 2) != hipSuccess ||
            hipMalloc((void**)&l->d_tstartT, E * (size_t)(l->NT + 1) * 2) != hipSuccess ||
            hipMalloc((void**)&l->d_tstats, (size_t)l->NT * 32) != hipSuccess ||
            hipMalloc((void**)&l->d_tdirty, (size_t)l->NT * 4) != hipSuccess ||
            hipMalloc((void**)&l->d_tcand, (size_t)(l->NT + 1) * 4) != hipSuccess ||
            hipMemset(l->d_tdirty, 0, (size_t)l->NT * 4) != hipSuccess ||
            hipMalloc((void**)&l->d_pe, E * (size_t)l->NT * 4) != hipSuccess ||
            hipMalloc((void**)&l->d_ttot, (size_t)l->NT * 4) != hipSuccess ||
            hipMalloc((void**)&l->d_toff, ((size_t)l->NT + 2 * ((size_t)l->NT / ffm::kOwnChunk + 1)) * 4) != hipSuccess ||
            hipMalloc((void**)&l->d_hdr, (size_t)l->ths * 4) != hipSuccess ||
            hipMalloc((void**)&l->d_pack, E * A * sizeof(ffm::TileRec)) != hipSuccess ||
            hipMalloc((void**)&l->d_xcnt, (ffm::kMaxOwners + 2) * 8) != hipSuccess ||
            hipMalloc((void**)&l->d_on, 16) != hipSuccess)
            return cleanup(fail(FFM_E_NOMEM, "hipMalloc (tiled step)"));
        const size_t pb = l->actor ? ffm::learn_batch_phase_bytes((long long)E, HW, (int)A) : 0;
        if (pb && hipMalloc((void**)&l->d_bph, pb) != hipSuccess)
            return cleanup(fail(FFM_E_NOMEM, "hipMalloc (phase-split batch step)"));
    }
    he = hipMemcpy(l->d_map, d.map, HW, hipMemcpyHostToDevice);
    if (he == hipSuccess) {
        std::vector<uint32_t> m2(((size_t)HW + 15) / 16, 0u);
        for (size_t c = 0; c < (size_t)HW; c++) m2[c >> 4] |= (uint32_t)(d.map[c] & 3) << ((c & 15) * 2);
        he = hipMemcpy(l->d_map2, m2.data(), m2.size() * 4, hipMemcpyHostToDevice);
    }
    if (he == hipSuccess) he = hipMemcpy(l->d_sff, d.sff, (size_t)HW * (l->f64 ? 8 : 4), hipMemcpyHostToDevice);
    if (he == hipSuccess && !fl.empty()) he = hipMemcpy(l->d_free_cells, fl.data(), fl.size() * 2, hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemset(l->d_pos, 0xFF, E * A * 2);
    if (he == hipSuccess) he = hipMemset(l->d_cnt, 0, E * 4);
    if (he == hipSuccess) he = hipMemset(l->d_dff[0], 0, E * HW * 4);
    if (he == hipSuccess && l->d_dff[1]) he = hipMemset(l->d_dff[1], 0, E * HW * 4);
    if (he == hipSuccess) he = hipMemset(l->d_eps, 0, E * 4);
    if (he == hipSuccess) he = hipMemset(l->d_ep_steps, 0, E * 4);
    if (he == hipSuccess) he = hipMemset(l->d_done, 0, E * 4);
    if (he == hipSuccess) he = hipMemset(l->d_nstart, 0, E * 4);
    if (he == hipSuccess) he = hipMemset(l->d_ctr, 0, E * 32);
    if (he == hipSuccess) he = hipMemset(l->d_hstat, 0, 32);
    if (he == hipSuccess) he = hipMemset(l->d_overflow, 0, 4);
    if (he == hipSuccess) he = hipMemset(l->d_eplog_n, 0, 8);
    if (he == hipSuccess && l->mt) he = hipMemset(l->d_mt_np, 0, E * 625 * 4);
    if (he == hipSuccess && l->mt) he = hipMemset(l->d_mt_py, 0, E * 625 * 4);
    if (he == hipSuccess) he = clear_table(l, l->V, l->L.v_default, nullptr);
    if (he == hipSuccess) he = clear_table(l, l->H, 0.0, nullptr);
    if (he == hipSuccess) he = hipDeviceSynchronize();
    if (he != hipSuccess) return cleanup(fail(FFM_E_HIP, std::string("init: ") + hipGetErrorString(he)));
    *out = l;
    return FFM_OK;
}

int ffm_learner_destroy(ffm_learner* l) {
    if (!l) return FFM_OK;
    (void)hipSetDevice(l->d.device);
    (void)hipDeviceSynchronize();
    release(l);
    return FFM_OK;
}

int ffm_learner_reset(ffm_learner* l, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    hipStream_t s = (hipStream_t)stream;
    const size_t E = (size_t)l->d.n_envs;
    HIP_TRY(hipMemsetAsync(l->d_dff[l->cur], 0, E * l->HW * 4, s));
    HIP_TRY(hipMemsetAsync(l->d_cnt, 0, E * 4, s));
    HIP_TRY(hipMemsetAsync(l->d_ep_steps, 0, E * 4, s));
    HIP_TRY(hipMemsetAsync(l->d_eps, 0, E * 4, s));        // episodes count from this reset
    HIP_TRY(hipMemsetAsync(l->d_pos, 0xFF, E * l->d.agent_capacity * 2, s));
    if (l->mt) return FFM_OK;
    HIP_TRY(ffm::launch_learn_reset(make_args(l), true, s));
    l->t++;
    return check_overflow(l, s);
}

int ffm_learner_reset_envs(ffm_learner* l, const uint8_t* mask, void* stream) {
    if (!l || !mask) return fail(FFM_E_INVALID, "null learner or mask");
    if (l->mt) return fail(FFM_E_UNSUPPORTED, "reset_envs: MT mode places agents on the host (set_state)");
    if (l->phase != 0) return fail(FFM_E_INVALID, "reset_envs inside a phased step");
    HIP_TRY(ffm::launch_learn_reset_mask(make_args(l), mask, (hipStream_t)stream));
    l->t++;
    return FFM_OK;
}

// The batched step in phases (multi-rank runs exchange the table deltas between
// them, ffm_amd/dist.py TableSync): local -> [exchange V (+H)] -> apply V (+ the
// post-update actor increments) -> [exchange H] -> apply H -> end.
static int phase_local(ffm_learner* l, hipStream_t s) {
    // H statistics of the step-start table: produced by the previous step's H
    // apply, recomputed only after the table was replaced (create / import)
    // (each table's mark -- its size at the step start -- is left by the previous
    // step's apply, or by clear / import)
    if ((l->actor || l->trained) && !l->hstat_valid) {
        HIP_TRY(ffm::launch_learn_hstat(make_args(l), s));
        l->hstat_valid = true;
    }
    HIP_TRY(ffm::launch_learn_batch(make_args(l), s));
    l->v_chain = l->chain_ok;
    l->phase = 1;
    return FFM_OK;
}

// With a sync period K > 1 the increments of K steps accumulate and the tables
// (and the H statistics) change only at every K-th step's apply; the post-update
// actor increments of the other steps use the V of the last apply.
static bool apply_due(const ffm_learner* l) { return l->since_apply + 1 >= l->sync_period; }

static int phase_apply(ffm_learner* l, int32_t which, hipStream_t s) {
    const bool due = apply_due(l);
    if (which == FFM_TABLE_V) {
        if (!l->trained && due) HIP_TRY(ffm::launch_learn_apply(make_args(l), true, false, s));
        if (l->post_update) HIP_TRY(ffm::launch_learn_post(make_args(l), s));
        l->phase = 2;
        return FFM_OK;
    }
    if (due) {
        HIP_TRY(ffm::launch_learn_apply(make_args(l), false, true, s));
        l->hstat_valid = true;
        l->tstats_valid = false;
    }
    l->phase = 3;
    return FFM_OK;
}

static int phase_end(ffm_learner* l, hipStream_t s, bool reset_done = false) {
    l->since_apply = apply_due(l) ? 0 : l->since_apply + 1;
    HIP_TRY(ffm::launch_learn_capture(make_args(l), l->traj, s));   // before the reset re-places
    l->cur ^= 1;
    if (l->d.auto_reset && !reset_done) HIP_TRY(ffm::launch_learn_reset(make_args(l), false, s));
    l->t++;
    l->phase = 0;
    return FFM_OK;
}

// With a sync period K > 1, increments of up to K - 1 steps can be pending between two
// applies.  Reading, replacing or re-periodising the tables at such a point applies them
// first (as if the period ended with the last step) and restarts the period, so an
// export never misses steps and a new period never stretches the current one.
//
// A learner driven by a multi-rank exchange (external_sync) never flushes on its own: its
// pending increments are only this rank's, and applying them alone would leave the ranks'
// tables and apply schedules out of step.  Its exports are read-only (the tables as of
// the last apply) and TableSync.flush() applies the exchanged deltas collectively
// (ffm_learner_flush_begin / _end).
static int apply_pending(ffm_learner* l, hipStream_t s) {
    if (!l->trained) HIP_TRY(ffm::launch_learn_apply(make_args(l), true, false, s));
    if (l->actor) {
        HIP_TRY(ffm::launch_learn_apply(make_args(l), false, true, s));
        l->hstat_valid = true;
        l->tstats_valid = false;
    }
    l->since_apply = 0;
    return FFM_OK;
}

static int flush_pending(ffm_learner* l, hipStream_t s) {
    if (l->mt || l->since_apply == 0 || l->phase != 0 || l->external_sync) return FFM_OK;
    return apply_pending(l, s);
}

int ffm_learner_step(ffm_learner* l, int32_t n_steps, void* stream) {
    if (!l || n_steps < 0) return fail(FFM_E_INVALID, "bad learner/n_steps");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    hipStream_t s = (hipStream_t)stream;
    // Overflow without a host sync: the previous call queued a copy of the flag
    // into pinned memory behind its steps; whatever of it has landed is reported
    // here (every sync point -- counters, export, get_state -- reports it exactly).
    int rc0 = async_overflow(l);
    if (rc0) return rc0;
    for (int i = 0; i < n_steps; i++) {
        if (l->mt) {
            HIP_TRY(ffm::launch_learn_exact(make_args(l), s));
            l->t++;
            continue;
        }
        if (l->tiled_ok && l->sync_period == 1) {
            if (l->ow > 1) return fail(FFM_E_INVALID, "an owner-sharded learner steps through its exchange (TableSync)");
            // tiled: records -> per-tile sums in LDS -> applied (no accumulators, no full-table pass)
            if (l->actor && !l->tstats_valid) {
                HIP_TRY(ffm::launch_learn_tiles(make_args(l), true, s));
                l->tstats_valid = l->hstat_valid = true;
            }
            ffm::LearnArgs a = make_args(l);
            a.trecs = l->d_trecs;
            // env-major passes read the tile offsets transposed, written by the stencil launch
            const bool tt = !l->single_tm && !tstart_t_off();
            if (tt) a.tstart_out = l->d_tstartT;
            HIP_TRY(ffm::launch_learn_batch(a, s));
            l->v_chain = l->chain_ok;
            a.tstart_out = nullptr;
            if (l->single_tm) {      // records reordered tile-major, then the passes
                a.ow = 1;
                a.orank = 0;
                a.ochunk = ffm::kOwnChunk;
                a.ths = l->ths;
                HIP_TRY(ffm::launch_learn_tile_pack(a, l->d_pe, l->d_ttot, l->d_toff, l->d_hdr, l->d_xcnt, l->d_pack, s));
                a.trecs = l->d_pack;
                a.thdr = l->d_hdr;
                a.tR = 1;
                a.NTk = l->NT;
            } else if (tt) {
                a.tstartT = l->d_tstartT;
            }
            bool reset_done = false;
            if (l->actor && !l->single_tm && l->d.auto_reset && l->traj.n_sel <= 0 && !ffm::learn_reset_small(a)) {
                l->cur ^= 1;     // the reset's arguments are those after the step's DFF swap
                const ffm::LearnArgs ra = make_args(l);
                l->cur ^= 1;
                HIP_TRY(ffm::launch_learn_tiles_reset(a, ra, s));
                reset_done = true;
            } else {
                HIP_TRY(ffm::launch_learn_tiles(a, false, s));
            }
            if (int rc = phase_end(l, s, reset_done)) return rc;
            continue;
        }
        int rc = phase_local(l, s);
        bool reset_done = false;
        if (!rc && l->actor && !l->trained && !l->post_update && apply_due(l)) {
            // one device, nothing exchanged between the tables: both applies in one launch,
            // and the ended envs re-placed in it too when no trajectory capture must see
            // them first (the reset's arguments are those after the step's DFF swap)
            ffm::LearnArgs a = make_args(l);
            if (l->d.auto_reset && l->traj.n_sel <= 0 && ffm::learn_reset_small(a) && !a.V.dense_by &&
                !a.Ht.dense_by) {
                l->cur ^= 1;
                const ffm::LearnArgs ra = make_args(l);
                l->cur ^= 1;
                HIP_TRY(ffm::launch_learn_apply_reset(a, ra, s));
                reset_done = true;
            } else {
                HIP_TRY(ffm::launch_learn_apply(a, true, true, s));
            }
            l->hstat_valid = true;
            l->tstats_valid = false;
            l->phase = 3;
        } else {
            if (!rc) rc = phase_apply(l, FFM_TABLE_V, s);
            if (!rc && l->actor) rc = phase_apply(l, FFM_TABLE_H, s);
        }
        if (!rc) rc = phase_end(l, s, reset_done);
        if (rc) return rc;
    }
    if (l->h_overflow && n_steps > 0 && !l->mt)
        HIP_TRY(hipMemcpyAsync(l->h_overflow, l->d_overflow, 4, hipMemcpyDeviceToHost, s));
    return FFM_OK;
}

int ffm_learner_step_local(ffm_learner* l, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->mt) return fail(FFM_E_INVALID, "phased steps are the batched (Philox) step");
    if (l->phase != 0) return fail(FFM_E_INVALID, "step_local: previous step not ended");
    int rc = async_overflow(l);    // the flag copy queued by an earlier step_end
    if (rc) return rc;
    return phase_local(l, (hipStream_t)stream);
}

int ffm_learner_step_apply(ffm_learner* l, int32_t which, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (which == FFM_TABLE_V && l->phase != 1) return fail(FFM_E_INVALID, "step_apply(V) must follow step_local");
    if (which == FFM_TABLE_H && (!l->actor || l->phase != 2))
        return fail(FFM_E_INVALID, "step_apply(H) must follow step_apply(V) (actor variants only)");
    if (which != FFM_TABLE_V && which != FFM_TABLE_H) return fail(FFM_E_INVALID, "which");
    return phase_apply(l, which, (hipStream_t)stream);
}

int ffm_learner_step_end(ffm_learner* l, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->phase != (l->actor ? 3 : 2)) return fail(FFM_E_INVALID, "step_end before the tables were applied");
    int rc = phase_end(l, (hipStream_t)stream);
    // the overflow flag (a full hash table, an undersized delta record buffer) as of this
    // step, copied behind it without a host sync: step_local reports it once it has landed
    if (!rc && l->h_overflow)
        HIP_TRY(hipMemcpyAsync(l->h_overflow, l->d_overflow, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return rc;
}

int ffm_learner_delta_export(ffm_learner* l, int32_t which, uint64_t* d_keys, int64_t* d_acc, int64_t cap,
                             int64_t* n, void* stream) {
    if (!l || !n) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = which == FFM_TABLE_V ? &l->V : (which == FFM_TABLE_H && l->actor ? &l->H : nullptr);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    if (l->phase == 0) return fail(FFM_E_INVALID, "delta_export outside a phased step");
    if (cap > 0 && (!d_keys || !d_acc)) return fail(FFM_E_INVALID, "null record buffers");
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(l->d_count, 0, 8, s));
    HIP_TRY(ffm::launch_learn_delta_export(T->t, T->accw, reinterpret_cast<unsigned long long*>(d_keys),
                                           reinterpret_cast<long long*>(d_acc), cap, l->d_count, s));
    unsigned long long c = 0;
    HIP_TRY(hipMemcpyAsync(&c, l->d_count, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n = (int64_t)c;
    if ((int64_t)c > cap) return fail(FFM_E_INVALID, "delta_export: record buffer too small (*n holds the size)");
    return FFM_OK;
}

int ffm_learner_delta_merge(ffm_learner* l, int32_t which, const uint64_t* d_keys, const int64_t* d_acc, int64_t n,
                            void* stream) {
    if (!l || n < 0) return fail(FFM_E_INVALID, "bad argument");
    DevTable* T = which == FFM_TABLE_V ? &l->V : (which == FFM_TABLE_H && l->actor ? &l->H : nullptr);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    if (l->phase == 0) return fail(FFM_E_INVALID, "delta_merge outside a phased step");
    HIP_TRY(ffm::launch_learn_delta_merge(T->t, T->accw, reinterpret_cast<const unsigned long long*>(d_keys),
                                          reinterpret_cast<const long long*>(d_acc), n, l->d_overflow,
                                          (hipStream_t)stream));
    return FFM_OK;
}

static int check_range(ffm_learner* l, int64_t env0, int64_t n) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (env0 < 0 || n < 0 || env0 + n > l->d.n_envs) return fail(FFM_E_INVALID, "env range out of bounds");
    return FFM_OK;
}

int ffm_learner_set_state(ffm_learner* l, int64_t env0, int64_t n, const uint16_t* positions,
                          const int32_t* counts, const float* dff, void* stream) {
    int rc = check_range(l, env0, n);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int A = l->d.agent_capacity;
    if (counts)
        for (int64_t i = 0; i < n; i++)
            if (counts[i] < 0 || counts[i] > A) return fail(FFM_E_INVALID, "count out of [0, agent_capacity]");
    if (positions && counts) {
        std::vector<uint8_t> map(l->HW);
        HIP_TRY(hipMemcpy(map.data(), l->d_map, l->HW, hipMemcpyDeviceToHost));
        std::vector<uint8_t> seen(l->HW, 0);
        for (int64_t i = 0; i < n; i++) {
            for (int j = 0; j < counts[i]; j++) {
                const uint16_t c = positions[i * A + j];
                if (c >= l->HW || !(map[c] == 0)) return fail(FFM_E_INVALID, "agent on a non-free cell");
                if (seen[c]) return fail(FFM_E_INVALID, "two agents on one cell");
                seen[c] = 1;
            }
            for (int j = 0; j < counts[i]; j++) seen[positions[i * A + j]] = 0;
        }
    }
    if (positions) {
        l->v_chain = false;      // the next step's s are not the last step's s'
        HIP_TRY(hipMemcpyAsync(l->d_pos + env0 * A, positions, (size_t)n * A * 2, hipMemcpyHostToDevice, s));
    }
    if (counts) HIP_TRY(hipMemcpyAsync(l->d_cnt + env0, counts, (size_t)n * 4, hipMemcpyHostToDevice, s));
    if (dff)
        HIP_TRY(hipMemcpyAsync(l->d_dff[l->cur] + env0 * l->HW, dff, (size_t)n * l->HW * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_learner_get_state(ffm_learner* l, int64_t env0, int64_t n, uint16_t* positions, int32_t* counts,
                          float* dff, void* stream) {
    int rc = check_range(l, env0, n);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int A = l->d.agent_capacity;
    if (positions)
        HIP_TRY(hipMemcpyAsync(positions, l->d_pos + env0 * A, (size_t)n * A * 2, hipMemcpyDeviceToHost, s));
    if (counts) HIP_TRY(hipMemcpyAsync(counts, l->d_cnt + env0, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (dff)
        HIP_TRY(hipMemcpyAsync(dff, l->d_dff[l->cur] + env0 * l->HW, (size_t)n * l->HW * 4, hipMemcpyDeviceToHost, s));
    return check_overflow(l, s);
}

int ffm_learner_get_episodes(ffm_learner* l, int64_t env0, int64_t n, int32_t* episodes, int32_t* ep_steps,
                             void* stream) {
    int rc = check_range(l, env0, n);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (episodes) HIP_TRY(hipMemcpyAsync(episodes, l->d_eps + env0, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (ep_steps) HIP_TRY(hipMemcpyAsync(ep_steps, l->d_ep_steps + env0, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_learner_set_mt_state(ffm_learner* l, int64_t env, const uint32_t* np_key, int32_t np_pos,
                             const uint32_t* py_key, int32_t py_pos, void* stream) {
    int rc = check_range(l, env, 1);
    if (rc) return rc;
    if (!l->mt) return fail(FFM_E_INVALID, "learner is not in MT mode");
    if (np_pos < 0 || np_pos > 624 || py_pos < 0 || py_pos > 624) return fail(FFM_E_INVALID, "MT position");
    hipStream_t s = (hipStream_t)stream;
    uint32_t buf[1250];
    std::memcpy(buf, np_key, 624 * 4);
    buf[624] = (uint32_t)np_pos;
    std::memcpy(buf + 625, py_key, 624 * 4);
    buf[1249] = (uint32_t)py_pos;
    HIP_TRY(hipMemcpyAsync(l->d_mt_np + env * 625, buf, 625 * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(l->d_mt_py + env * 625, buf + 625, 625 * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_learner_get_mt_state(ffm_learner* l, int64_t env, uint32_t* np_key, int32_t* np_pos, uint32_t* py_key,
                             int32_t* py_pos, void* stream) {
    int rc = check_range(l, env, 1);
    if (rc) return rc;
    if (!l->mt) return fail(FFM_E_INVALID, "learner is not in MT mode");
    hipStream_t s = (hipStream_t)stream;
    uint32_t buf[1250];
    HIP_TRY(hipMemcpyAsync(buf, l->d_mt_np + env * 625, 625 * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(buf + 625, l->d_mt_py + env * 625, 625 * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(np_key, buf, 624 * 4);
    *np_pos = (int32_t)buf[624];
    std::memcpy(py_key, buf + 625, 624 * 4);
    *py_pos = (int32_t)buf[1249];
    return FFM_OK;
}

int ffm_learner_get_counters(ffm_learner* l, uint64_t* counters, void* stream) {
    if (!l || !counters) return fail(FFM_E_INVALID, "null argument");
    hipStream_t s = (hipStream_t)stream;
    std::vector<unsigned long long> c((size_t)l->d.n_envs * 4);
    HIP_TRY(hipMemcpyAsync(c.data(), l->d_ctr, c.size() * 8, hipMemcpyDeviceToHost, s));
    int rc = check_overflow(l, s);
    if (rc) return rc;
    for (int i = 0; i < 4; i++) counters[i] = 0;
    for (size_t j = 0; j < (size_t)l->d.n_envs; j++)
        for (int i = 0; i < 3; i++) counters[i] += c[j * 4 + i];
    counters[3] = l->d.n_envs ? c[3] : 0;     // steps: every env steps every time
    return FFM_OK;
}

int ffm_learner_set_epsilon(ffm_learner* l, double epsilon) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    l->L.epsilon = std::min(std::max(epsilon, 0.0), 1.0);      // np.clip (model/ffm_unified.py:867)
    return FFM_OK;
}

int ffm_learner_set_h_extra(ffm_learner* l, int64_t n_values, double mn, double mx, int32_t nonfinite) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (!l->trained) return fail(FFM_E_INVALID, "extra H statistics are ffm_trained_core's (FFM_VARIANT_TRAINED)");
    if (n_values < 0) return fail(FFM_E_INVALID, "n_values must be >= 0");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    l->hx_n = n_values;
    l->hx_nf = n_values > 0 && nonfinite ? 1 : 0;
    l->hx_mn = n_values > 0 ? mn : 0.0;
    l->hx_mx = n_values > 0 ? mx : 0.0;
    l->hstat_valid = false;            // the next step recomputes the statistics with them
    return FFM_OK;
}

int ffm_learner_set_v_default(ffm_learner* l, double v_default, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    l->L.v_default = v_default;
    ffm::LearnArgs a = make_args(l);
    HIP_TRY(ffm::launch_learn_fill_default(a, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return FFM_OK;
}

static DevTable* pick(ffm_learner* l, int32_t which) {
    if (which == FFM_TABLE_V) return &l->V;
    if (which == FFM_TABLE_H && (l->actor || l->trained)) return &l->H;
    return nullptr;
}

int ffm_learner_table_size(ffm_learner* l, int32_t which, int64_t* n, void* stream) {
    if (!l || !n) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = pick(l, which);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    uint32_t v = 0;
    HIP_TRY(hipMemcpyAsync(&v, T->t.n, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    *n = (int64_t)v;
    return FFM_OK;
}

int ffm_learner_export_table(ffm_learner* l, int32_t which, uint64_t* keys, double* vals, int64_t cap,
                             int64_t* n, void* stream) {
    if (!l || !n) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = pick(l, which);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_pending(l, s);
    if (!rc) rc = check_overflow(l, s);
    if (rc) return rc;
    uint32_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, T->t.n, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n = cnt;
    if ((int64_t)cnt > cap) return fail(FFM_E_INVALID, "export buffer too small");
    if (cnt == 0) return FFM_OK;
    std::vector<uint32_t> order(cnt);
    const size_t st = T->t.stride;
    std::vector<unsigned long long> rec(T->cap * st);
    HIP_TRY(hipMemcpyAsync(order.data(), T->t.order, (size_t)cnt * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(rec.data(), T->t.rec, T->cap * st * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (uint32_t i = 0; i < cnt; i++) {
        const size_t slot = order[i];
        if (keys) keys[i] = rec[slot * st];
        if (vals) std::memcpy(vals + (size_t)i * T->width, rec.data() + slot * st + 1, 8 * (size_t)T->width);
    }
    return FFM_OK;
}

int ffm_learner_import_table(ffm_learner* l, int32_t which, const uint64_t* keys, const double* vals, int64_t n,
                             void* stream) {
    if (!l || (n > 0 && (!keys || !vals))) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = pick(l, which);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    // hashed tables refuse inserts past 7/8 load; a dense table's slots are injective
    // in the key, so any n <= cap valid keys fit
    if ((size_t)n > (T->t.dense_by ? T->cap : (size_t)T->t.limit))
        return fail(FFM_E_NOMEM, "table capacity too small for import");
    for (int64_t i = 0; i < n; i++) {
        if (keys[i] == ~0ull) return fail(FFM_E_INVALID, "invalid key");
        if (T->t.dense_by) {     // rank keys: 8 bits of ranks, blocks inside the map
            const uint64_t bx = (keys[i] >> 26) & 0x7FFFF, by = (keys[i] >> 45) & 0x7FFFF;
            if ((keys[i] & 0x3FFFF00ull) || bx >= l->dense_bx || by >= T->t.dense_by)
                return fail(FFM_E_INVALID, "key is not a rank state of this map / block size");
        }
    }
    hipStream_t s = (hipStream_t)stream;
    if (l->external_sync && l->since_apply != 0 && !l->mt)
        return fail(FFM_E_INVALID, "import between two applies of a shared learner: TableSync.flush() first");
    if (int rc = flush_pending(l, s)) return rc;
    if (which == FFM_TABLE_H) l->hstat_valid = l->tstats_valid = false;
    if (which == FFM_TABLE_V) l->v_chain = false;   // V(s) no longer known present
    HIP_TRY(clear_table(l, *T, which == FFM_TABLE_V ? l->L.v_default : 0.0, s));
    if (n > 0) {
        unsigned long long* dk = nullptr;
        double* dv = nullptr;
        HIP_TRY(hipMalloc((void**)&dk, (size_t)n * 8));
        hipError_t he = hipMalloc((void**)&dv, (size_t)n * T->width * 8);
        if (he == hipSuccess) he = hipMemcpyAsync(dk, keys, (size_t)n * 8, hipMemcpyHostToDevice, s);
        if (he == hipSuccess) he = hipMemcpyAsync(dv, vals, (size_t)n * T->width * 8, hipMemcpyHostToDevice, s);
        if (he == hipSuccess) he = ffm::launch_learn_import(T->t, T->width, dk, dv, n, l->d_overflow, s);
        if (he == hipSuccess) he = hipStreamSynchronize(s);
        (void)hipFree(dk);
        (void)hipFree(dv);
        if (he != hipSuccess) return fail(FFM_E_HIP, std::string("import: ") + hipGetErrorString(he));
    }
    return check_overflow(l, s);
}

int ffm_learner_set_placement(ffm_learner* l, const uint16_t* cells, int32_t count, int32_t n_agents) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (count < 0 || count > l->F_all || (count > 0 && !cells)) return fail(FFM_E_INVALID, "placement cell count");
    const int navail = count > 0 ? count : l->F_all;
    if (n_agents < 0 || n_agents > navail || n_agents > l->d.agent_capacity)
        return fail(FFM_E_INVALID, "n_agents must be <= the candidate cells and agent_capacity");
    std::vector<uint16_t> fl;
    std::vector<uint8_t> map(l->HW);
    HIP_TRY(hipMemcpy(map.data(), l->d_map, l->HW, hipMemcpyDeviceToHost));
    if (count > 0) {
        std::vector<uint8_t> seen(l->HW, 0);
        for (int i = 0; i < count; i++) {
            if (cells[i] >= l->HW || map[cells[i]] != 0) return fail(FFM_E_INVALID, "placement cell is not free");
            if (seen[cells[i]]) return fail(FFM_E_INVALID, "placement cells repeat");
            seen[cells[i]] = 1;
            fl.push_back(cells[i]);
        }
    } else {
        for (int i = 0; i < l->HW; i++)
            if (map[i] == 0) fl.push_back((uint16_t)i);
    }
    HIP_TRY(hipDeviceSynchronize());
    if (!fl.empty()) HIP_TRY(hipMemcpy(l->d_free_cells, fl.data(), fl.size() * 2, hipMemcpyHostToDevice));
    l->F = (int)fl.size();
    l->d.n_agents = n_agents;
    return FFM_OK;
}

int ffm_learner_set_epsilon_schedule(ffm_learner* l, double eps_start, double eps_end, double eps_offset,
                                     double eps_span) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    l->L.eps_start = eps_start; l->L.eps_end = eps_end;
    l->L.eps_offset = eps_offset; l->L.eps_span = eps_span;
    return FFM_OK;
}

// ---- tiled step across ranks ---------------------------------------
int ffm_learner_tiled_buffers(ffm_learner* l, void** d_recs, int64_t* rec_bytes, uint16_t** d_tstart,
                              int64_t* tstart_count) {
    if (!l || !d_recs || !rec_bytes || !d_tstart || !tstart_count) return fail(FFM_E_INVALID, "null argument");
    if (!l->tiled_ok) return fail(FFM_E_UNSUPPORTED, "not a tiled learner (ffm_unified, block size 1, large map)");
    *d_recs = l->d_trecs;
    *rec_bytes = (int64_t)(l->d.n_envs * l->d.agent_capacity * (int64_t)sizeof(ffm::TileRec));
    *d_tstart = l->d_tstart;
    *tstart_count = (int64_t)l->d.n_envs * (l->NT + 1);
    return FFM_OK;
}

int ffm_learner_step_tiled_local(ffm_learner* l, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (!l->tiled_ok || l->sync_period != 1) return fail(FFM_E_UNSUPPORTED, "tiled step: tiled learner at sync period 1");
    if (l->phase != 0) return fail(FFM_E_INVALID, "step_tiled_local: previous step not ended");
    if (int rc = async_overflow(l)) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (l->actor && !l->tstats_valid) {
        HIP_TRY(ffm::launch_learn_tiles(make_args(l), true, s));
        l->tstats_valid = l->hstat_valid = true;
    }
    ffm::LearnArgs a = make_args(l);
    a.trecs = l->d_trecs;
    HIP_TRY(ffm::launch_learn_batch(a, s));
    l->v_chain = l->chain_ok;
    l->phase = 5;
    return FFM_OK;
}

int ffm_learner_step_tiled_apply(ffm_learner* l, const void* d_recs_all, const uint16_t* d_tstart_all,
                                 int64_t n_envs_all, void* stream) {
    if (!l || !d_recs_all || !d_tstart_all || n_envs_all < 1) return fail(FFM_E_INVALID, "bad argument");
    if ((unsigned long long)n_envs_all * (unsigned long long)l->d.agent_capacity >= (1ull << 32))   // 32-bit record indices
        return fail(FFM_E_INVALID, "tiled step: n_envs_all * agent_capacity >= 2^32");
    if (l->phase != 5) return fail(FFM_E_INVALID, "step_tiled_apply must follow step_tiled_local");
    hipStream_t s = (hipStream_t)stream;
    ffm::LearnArgs a = make_args(l);
    a.trecs = const_cast<ffm::TileRec*>(reinterpret_cast<const ffm::TileRec*>(d_recs_all));
    a.tstart = const_cast<uint16_t*>(d_tstart_all);
    a.E = n_envs_all;
    a.tile_ensure = 1;
    HIP_TRY(ffm::launch_learn_tiles(a, false, s));
    int rc = phase_end(l, s);
    if (!rc && l->h_overflow) HIP_TRY(hipMemcpyAsync(l->h_overflow, l->d_overflow, 4, hipMemcpyDeviceToHost, s));
    return rc;
}

// ---- owner-sharded tiled step ---------------------------------------
int ffm_learner_set_tile_owners(ffm_learner* l, int32_t world, int32_t rank) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (!l->tiled_ok) return fail(FFM_E_UNSUPPORTED, "not a tiled learner (ffm_unified, block size 1, large map)");
    if (world < 1 || world > ffm::kMaxOwners || rank < 0 || rank >= world)
        return fail(FFM_E_INVALID, "tile owners: 1 <= world <= 64, 0 <= rank < world");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    if (!l->tile_major && world > 1) return fail(FFM_E_UNSUPPORTED, "owner sharding needs tile-major records");
    HIP_TRY(hipDeviceSynchronize());
    int mx = 0;
    for (int q = 0; q < world; q++) mx = std::max(mx, ffm::owner_tiles(l->NT, world, ffm::kOwnChunk, q));
    const int ths = mx + 1;
    // the new buffers first: a failed allocation leaves the learner as it was
    uint32_t* hdr = nullptr; double* tsum = nullptr;
    if (hipMalloc((void**)&hdr, (size_t)world * ths * 4) != hipSuccess ||
        hipMalloc((void**)&tsum, (size_t)ths * 5 * 8) != hipSuccess) {
        (void)hipFree(hdr); (void)hipFree(tsum);
        return fail(FFM_E_NOMEM, "hipMalloc (owner exchange)");
    }
    (void)hipFree(l->d_hdr);
    (void)hipFree(l->d_tsum);
    (void)hipFree(l->d_opack);
    l->d_hdr = hdr; l->d_tsum = tsum; l->d_opack = nullptr;
    l->rcap = 0;            // the send blocks depend on world: set_owner_capacity again
    l->ow = world;
    l->orank = rank;
    l->ths = ths;
    HIP_TRY(hipMemset(l->d_hdr, 0, (size_t)world * l->ths * 4));
    return FFM_OK;
}

int ffm_learner_set_owner_capacity(ffm_learner* l, int64_t rec_capacity, int64_t v_capacity, int64_t h_capacity) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (!l->tiled_ok) return fail(FFM_E_UNSUPPORTED, "not a tiled learner (ffm_unified, block size 1, large map)");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    if (rec_capacity < 1 || v_capacity < 1 || h_capacity < 1) return fail(FFM_E_INVALID, "capacities must be >= 1");
    if ((unsigned long long)rec_capacity * (unsigned long long)l->ow >= (1ull << 32) || v_capacity >= (1ll << 31) ||
        h_capacity >= (1ll << 31))
        return fail(FFM_E_INVALID, "owner capacities: world * rec_capacity < 2^32, outputs < 2^31");
    HIP_TRY(hipDeviceSynchronize());        // queued steps may still use the old buffers
    const size_t nrec = (size_t)l->ow * (size_t)rec_capacity;
    ffm::TileRec* pack = nullptr;
    uint32_t* vs = nullptr; double* vv = nullptr; uint32_t* hk = nullptr; long long* hq = nullptr;
    if (hipMalloc((void**)&pack, nrec * sizeof(ffm::TileRec)) != hipSuccess ||
        hipMalloc((void**)&vs, (size_t)v_capacity * 4) != hipSuccess ||
        hipMalloc((void**)&vv, (size_t)v_capacity * 8) != hipSuccess ||
        hipMalloc((void**)&hk, (size_t)h_capacity * 4) != hipSuccess ||
        hipMalloc((void**)&hq, (size_t)h_capacity * 8) != hipSuccess) {
        (void)hipFree(pack); (void)hipFree(vs); (void)hipFree(vv); (void)hipFree(hk); (void)hipFree(hq);
        return fail(FFM_E_NOMEM, "hipMalloc (owner exchange capacity)");
    }
    (void)hipFree(l->d_opack); (void)hipFree(l->d_vslot); (void)hipFree(l->d_vval);
    (void)hipFree(l->d_hkey); (void)hipFree(l->d_hq);
    l->d_opack = pack; l->d_vslot = vs; l->d_vval = vv; l->d_hkey = hk; l->d_hq = hq;
    l->rcap = rec_capacity;
    l->vcap = (size_t)v_capacity;
    l->hcap = (size_t)h_capacity;
    HIP_TRY(hipMemset(l->d_on, 0, 16));
    HIP_TRY(hipMemset(l->d_xcnt, 0, (ffm::kMaxOwners + 2) * 8));
    return FFM_OK;
}

int ffm_learner_set_owner_send_buffer(ffm_learner* l, void* d_buf) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    HIP_TRY(hipDeviceSynchronize());
    l->x_opack = reinterpret_cast<ffm::TileRec*>(d_buf);
    return FFM_OK;
}

int ffm_learner_set_owner_output_buffers(ffm_learner* l, uint32_t* v_slot, double* v_val, int64_t* v_count,
                                         uint32_t* h_key, int64_t* h_q, int64_t* h_count) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    const bool vset = v_slot && v_val && v_count, hset = h_key && h_q && h_count;
    if ((v_slot || v_val || v_count) && !vset) return fail(FFM_E_INVALID, "V outputs: all three buffers or none");
    if ((h_key || h_q || h_count) && !hset) return fail(FFM_E_INVALID, "H outputs: all three buffers or none");
    HIP_TRY(hipDeviceSynchronize());
    l->x_vslot = v_slot; l->x_vval = v_val; l->x_vn = reinterpret_cast<unsigned long long*>(v_count);
    l->x_hkey = h_key; l->x_hq = reinterpret_cast<long long*>(h_q); l->x_hn = reinterpret_cast<unsigned long long*>(h_count);
    return FFM_OK;
}

int ffm_learner_owner_buffers(ffm_learner* l, ffm_owner_buffers* b) {
    if (!l || !b) return fail(FFM_E_INVALID, "null argument");
    if (!l->tiled_ok) return fail(FFM_E_UNSUPPORTED, "not a tiled learner (ffm_unified, block size 1, large map)");
    b->world = l->ow;
    b->rank = l->orank;
    b->send_recs = l->x_opack ? l->x_opack : l->d_opack;
    b->send_rec_capacity = (int64_t)l->rcap;
    b->send_hdr = l->d_hdr;
    b->hdr_stride = l->ths;
    b->counts = reinterpret_cast<int64_t*>(l->d_xcnt);
    b->v_slot = l->d_vslot;
    b->v_val = l->d_vval;
    b->h_key = l->d_hkey;
    b->h_q = reinterpret_cast<int64_t*>(l->d_hq);
    b->out_counts = reinterpret_cast<int64_t*>(l->d_on);
    b->v_capacity = (int64_t)l->vcap;
    b->h_capacity = (int64_t)l->hcap;
    b->tsum = l->d_tsum;
    b->tsum_count = (int64_t)ffm::owner_tiles(l->NT, l->ow, ffm::kOwnChunk, l->orank);
    return FFM_OK;
}

static ffm::LearnArgs owner_args(ffm_learner* l) {
    ffm::LearnArgs a = make_args(l);
    a.ow = l->ow;
    a.orank = l->orank;
    a.ochunk = ffm::kOwnChunk;
    a.ths = l->ths;
    a.NTk = ffm::owner_tiles(l->NT, l->ow, ffm::kOwnChunk, l->orank);
    a.tblk = l->rcap;
    return a;
}

int ffm_learner_step_owner_local(ffm_learner* l, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (!l->tiled_ok || l->sync_period != 1 || !l->tile_major)
        return fail(FFM_E_UNSUPPORTED, "owner step: tiled learner, tile-major records, sync period 1");
    if (!l->d_opack) return fail(FFM_E_INVALID, "owner step: ffm_learner_set_tile_owners and set_owner_capacity first");
    if (l->phase != 0) return fail(FFM_E_INVALID, "step_owner_local: previous step not ended");
    if (int rc = async_overflow(l)) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (l->actor && !l->tstats_valid) {     // every rank: the same tables, the same summaries
        HIP_TRY(ffm::launch_learn_tiles(make_args(l), true, s));
        l->tstats_valid = l->hstat_valid = true;
    }
    ffm::LearnArgs a = owner_args(l);
    a.trecs = l->d_trecs;
    HIP_TRY(ffm::launch_learn_batch(a, s));
    l->v_chain = l->chain_ok;
    HIP_TRY(ffm::launch_learn_tile_pack(a, l->d_pe, l->d_ttot, l->d_toff, l->d_hdr, l->d_xcnt,
                                        l->x_opack ? l->x_opack : l->d_opack, s));
    l->phase = 7;
    return FFM_OK;
}

int ffm_learner_step_owner_v(ffm_learner* l, const void* d_recs, const uint32_t* d_hdrs, int64_t src_stride,
                             void* stream) {
    if (!l || !d_recs || !d_hdrs) return fail(FFM_E_INVALID, "null argument");
    if (src_stride != 0 && src_stride < l->rcap) return fail(FFM_E_INVALID, "src_stride below the block capacity");
    if (l->phase != 7) return fail(FFM_E_INVALID, "step_owner_v must follow step_owner_local");
    hipStream_t s = (hipStream_t)stream;
    l->own_recs = reinterpret_cast<const ffm::TileRec*>(d_recs);
    l->own_hdr = d_hdrs;
    ffm::LearnArgs a = owner_args(l);
    a.trecs = const_cast<ffm::TileRec*>(l->own_recs);
    a.thdr = d_hdrs;
    a.tR = l->ow;
    a.tsrc = src_stride;
    l->own_src = src_stride;
    a.vout_slot = l->x_vslot ? l->x_vslot : l->d_vslot;
    a.vout_val = l->x_vslot ? l->x_vval : l->d_vval;
    a.vout_n = l->x_vslot ? l->x_vn : l->d_on;
    a.vout_cap = (long long)l->vcap;
    HIP_TRY(ffm::launch_learn_tiles_owner_v(a, s));
    l->phase = 8;
    return FFM_OK;
}

int ffm_learner_step_owner_h(ffm_learner* l, const uint32_t* d_v_slot, const double* d_v_val,
                             const int64_t* d_v_counts, int64_t v_stride, void* stream) {
    if (!l || !d_v_counts || (l->ow > 1 && (!d_v_slot || !d_v_val))) return fail(FFM_E_INVALID, "null argument");
    if (v_stride < 0) return fail(FFM_E_INVALID, "v_stride");
    if (l->phase != 8) return fail(FFM_E_INVALID, "step_owner_h must follow step_owner_v");
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(ffm::launch_learn_v_scatter(l->V.t, d_v_slot, d_v_val, v_stride, reinterpret_cast<const long long*>(d_v_counts),
                                        l->ow, l->orank, l->d_overflow, s));
    if (l->actor) {     // the actor's td reads the V every owner updated
        ffm::LearnArgs a = owner_args(l);
        a.trecs = const_cast<ffm::TileRec*>(l->own_recs);
        a.thdr = l->own_hdr;
        a.tR = l->ow;
        a.tsrc = l->own_src;
        a.hout_key = l->x_hkey ? l->x_hkey : l->d_hkey;
        a.hout_q = l->x_hkey ? l->x_hq : l->d_hq;
        a.hout_n = l->x_hkey ? l->x_hn : l->d_on + 1;
        a.hout_cap = (long long)l->hcap;
        HIP_TRY(ffm::launch_learn_tiles_owner_h(a, l->d_tsum, s));
    }
    l->phase = 9;
    return FFM_OK;
}

int ffm_learner_step_owner_end(ffm_learner* l, const uint32_t* d_h_key, const int64_t* d_h_q,
                               const int64_t* d_h_counts, int64_t h_stride, const double* d_tsum_all,
                               int64_t tsum_stride, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->phase != 9) return fail(FFM_E_INVALID, "step_owner_end must follow step_owner_h");
    hipStream_t s = (hipStream_t)stream;
    ffm::LearnArgs a = owner_args(l);
    if (l->actor) {
        if (!d_h_counts || !d_tsum_all || h_stride < 0 || (l->ow > 1 && (!d_h_key || !d_h_q)))
            return fail(FFM_E_INVALID, "null argument");
        HIP_TRY(ffm::launch_learn_h_deltas(l->H.t, d_h_key, reinterpret_cast<const long long*>(d_h_q), h_stride,
                                           reinterpret_cast<const long long*>(d_h_counts), l->ow, l->orank,
                                           l->d_overflow, s));
        HIP_TRY(ffm::launch_learn_tsum_unpack(a, d_tsum_all, tsum_stride, s));
        HIP_TRY(ffm::launch_learn_tile_stats(a, s));     // every rank: the same summaries, the same statistics
    } else {
        HIP_TRY(ffm::launch_learn_mark(a, s));
    }
    l->own_recs = nullptr;
    l->own_hdr = nullptr;
    int rc = phase_end(l, s);
    if (!rc && l->h_overflow) HIP_TRY(hipMemcpyAsync(l->h_overflow, l->d_overflow, 4, hipMemcpyDeviceToHost, s));
    return rc;
}

int ffm_learner_set_epsilon_phase(ffm_learner* l, int32_t period) {
    if (!l || period < 0) return fail(FFM_E_INVALID, "epsilon phase period must be >= 0");
    l->eps_phase = period;
    return FFM_OK;
}

int ffm_learner_set_epsilon_stride(ffm_learner* l, int64_t stride) {
    if (!l || stride < 1) return fail(FFM_E_INVALID, "epsilon stride must be >= 1");
    l->eps_stride = stride;
    return FFM_OK;
}

int ffm_learner_set_episode_caps(ffm_learner* l, const int32_t* caps, int64_t n) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (n != 0 && (n != l->d.n_envs || !caps)) return fail(FFM_E_INVALID, "episode caps: n must be n_envs (or 0)");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    HIP_TRY(hipDeviceSynchronize());        // queued steps may still read the old quotas
    if (n == 0) {
        (void)hipFree(l->d_epcap);
        l->d_epcap = nullptr;
        return FFM_OK;
    }
    if (!l->d_epcap) {
        hipError_t he = hipMalloc((void**)&l->d_epcap, (size_t)n * 4);
        if (he != hipSuccess) {
            l->d_epcap = nullptr;
            return fail(FFM_E_NOMEM, std::string("hipMalloc (episode caps): ") + hipGetErrorString(he));
        }
    }
    HIP_TRY(hipMemcpy(l->d_epcap, caps, (size_t)n * 4, hipMemcpyHostToDevice));
    return FFM_OK;
}

int ffm_learner_drain_episodes(ffm_learner* l, int32_t* records, int64_t cap, int64_t* n, int64_t* dropped,
                               void* stream) {
    if (!l || !n) return fail(FFM_E_INVALID, "null argument");
    hipStream_t s = (hipStream_t)stream;
    unsigned long long c = 0;
    HIP_TRY(hipMemcpyAsync(&c, l->d_eplog_n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const long long have = std::min<long long>((long long)c, l->eplog_cap);
    if (have > cap) {
        *n = have;
        return fail(FFM_E_INVALID, "drain_episodes: buffer too small (*n holds the count)");
    }
    if (have > 0 && records)
        HIP_TRY(hipMemcpyAsync(records, l->d_eplog, (size_t)have * 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemsetAsync(l->d_eplog_n, 0, 8, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n = have;
    if (dropped) *dropped = (int64_t)c - have;
    return FFM_OK;
}

int ffm_learner_delta_export_async(ffm_learner* l, int32_t which, uint64_t* d_keys, int64_t* d_acc, int64_t cap,
                                   int64_t* d_count, void* stream) {
    if (!l || !d_count) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = which == FFM_TABLE_V ? &l->V : (which == FFM_TABLE_H && l->actor ? &l->H : nullptr);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    if (l->phase == 0) return fail(FFM_E_INVALID, "delta_export outside a phased step");
    if (cap > 0 && (!d_keys || !d_acc)) return fail(FFM_E_INVALID, "null record buffers");
    hipStream_t s = (hipStream_t)stream;
    auto* cnt = reinterpret_cast<unsigned long long*>(d_count);
    HIP_TRY(hipMemsetAsync(cnt, 0, 8, s));
    HIP_TRY(ffm::launch_learn_delta_export(T->t, T->accw, reinterpret_cast<unsigned long long*>(d_keys),
                                           reinterpret_cast<long long*>(d_acc), cap, cnt, s));
    HIP_TRY(ffm::launch_learn_delta_check(cnt, cap, l->d_overflow, s));
    return FFM_OK;
}

int ffm_learner_delta_merge_async(ffm_learner* l, int32_t which, const uint64_t* d_keys, const int64_t* d_acc,
                                  const int64_t* d_count, int64_t cap, void* stream) {
    if (!l || !d_count || cap < 0) return fail(FFM_E_INVALID, "bad argument");
    DevTable* T = which == FFM_TABLE_V ? &l->V : (which == FFM_TABLE_H && l->actor ? &l->H : nullptr);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    if (l->phase == 0) return fail(FFM_E_INVALID, "delta_merge outside a phased step");
    HIP_TRY(ffm::launch_learn_delta_merge(T->t, T->accw, reinterpret_cast<const unsigned long long*>(d_keys),
                                          reinterpret_cast<const long long*>(d_acc), cap, l->d_overflow,
                                          (hipStream_t)stream, reinterpret_cast<const long long*>(d_count)));
    return FFM_OK;
}

int ffm_learner_set_sync_period(ffm_learner* l, int32_t period) {
    if (!l || period < 1) return fail(FFM_E_INVALID, "sync period must be >= 1");
    if (l->mt && period != 1) return fail(FFM_E_INVALID, "the exact (MT) step applies every step");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    if (l->since_apply != 0 && l->external_sync)
        return fail(FFM_E_INVALID, "new sync period between two applies of a shared learner: TableSync.flush() first");
    if (l->since_apply != 0) {   // no stream argument: order behind every queued step
        HIP_TRY(hipDeviceSynchronize());
        if (int rc = flush_pending(l, nullptr)) return rc;
        HIP_TRY(hipDeviceSynchronize());
    }
    l->sync_period = period;
    l->since_apply = 0;
    return FFM_OK;
}

int ffm_learner_set_external_sync(ffm_learner* l, int32_t on) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    l->external_sync = on != 0;
    return FFM_OK;
}

// The collective flush of a shared learner (TableSync.flush): begin opens a phase in which
// the pending accumulators can be exchanged (delta export / merge, dense buffers / adopt),
// end applies them (V, then H; the post-update actor increments of the pending steps were
// added at their steps) and restarts the period.  *pending = 0: nothing to apply, no phase
// opened (every rank of a TableSync agrees: the periods advance in lockstep).
int ffm_learner_flush_begin(ffm_learner* l, int32_t* pending) {
    if (!l || !pending) return fail(FFM_E_INVALID, "null argument");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    *pending = (!l->mt && l->since_apply != 0) ? 1 : 0;
    if (*pending) l->phase = 6;
    return FFM_OK;
}

int ffm_learner_flush_end(ffm_learner* l, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->phase != 6) return fail(FFM_E_INVALID, "flush_end must follow flush_begin with pending increments");
    l->phase = 0;
    return apply_pending(l, (hipStream_t)stream);
}

int ffm_learner_apply_due(ffm_learner* l, int32_t* due) {
    if (!l || !due) return fail(FFM_E_INVALID, "null argument");
    *due = apply_due(l) ? 1 : 0;
    return FFM_OK;
}

int ffm_learner_dense_buffers(ffm_learner* l, int32_t which, int64_t** d_acc, int64_t* acc_count,
                              uint32_t** d_present, int64_t* present_words) {
    if (!l || !d_acc || !acc_count || !d_present || !present_words) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = which == FFM_TABLE_V ? &l->V : (which == FFM_TABLE_H && (l->actor || l->trained) ? &l->H : nullptr);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    if (!T->t.dense_by) return fail(FFM_E_UNSUPPORTED, "not a dense (rank-key) table");
    *d_acc = reinterpret_cast<int64_t*>(T->t.acc);
    *acc_count = (int64_t)(T->cap * (size_t)T->accw);
    *d_present = T->t.present;
    *present_words = (int64_t)(T->cap / 32);
    return FFM_OK;
}

int ffm_learner_dense_adopt(ffm_learner* l, int32_t which, const uint32_t* d_union, void* stream) {
    if (!l || !d_union) return fail(FFM_E_INVALID, "null argument");
    DevTable* T = which == FFM_TABLE_V ? &l->V : (which == FFM_TABLE_H && l->actor ? &l->H : nullptr);
    if (!T) return fail(FFM_E_INVALID, "no such table for this variant");
    if (!T->t.dense_by) return fail(FFM_E_UNSUPPORTED, "not a dense (rank-key) table");
    if (l->phase == 0 && !l->tiled_ok) return fail(FFM_E_INVALID, "dense_adopt outside a phased step");
    HIP_TRY(ffm::launch_learn_dense_adopt(T->t, d_union, (hipStream_t)stream));
    return FFM_OK;
}

int ffm_learner_set_trajectory_capture(ffm_learner* l, const int32_t* envs, const int32_t* phases, int32_t n_sel,
                                       int32_t period, int64_t capacity_rows, void* stream) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    if (l->mt) return fail(FFM_E_INVALID, "trajectory capture is the batched step's (MT drop-in: run(return_trajectory=True))");
    if (l->phase != 0) return fail(FFM_E_INVALID, "a phased step is in progress");
    if (n_sel < 0 || (n_sel > 0 && (!envs || period < 1 || capacity_rows < 1)))
        return fail(FFM_E_INVALID, "trajectory capture: envs, period >= 1 and capacity_rows >= 1 are required");
    for (int32_t i = 0; i < n_sel; i++) {
        if (envs[i] < 0 || envs[i] >= l->d.n_envs) return fail(FFM_E_INVALID, "trajectory capture: env out of range");
        if (phases && phases[i] < 0) return fail(FFM_E_INVALID, "trajectory capture: phase must be >= 0");
    }
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipStreamSynchronize(s));        // the previous buffers may still be read by queued steps
    free_traj(l);
    if (n_sel == 0) return FFM_OK;
    ffm::TrajCapture& c = l->traj;
    const size_t A = (size_t)l->d.agent_capacity;
    hipError_t e = hipSuccess;
    int* de = nullptr; int* dp = nullptr;
    if (e == hipSuccess) e = hipMalloc((void**)&de, (size_t)n_sel * 4);
    if (e == hipSuccess && phases) e = hipMalloc((void**)&dp, (size_t)n_sel * 4);
    c.envs = de; c.phase = dp;
    if (e == hipSuccess) e = hipMalloc((void**)&c.meta, (size_t)capacity_rows * 16);
    if (e == hipSuccess) e = hipMalloc((void**)&c.cells, (size_t)capacity_rows * A * 2);
    if (e == hipSuccess) e = hipMalloc((void**)&c.n, 8);
    if (e != hipSuccess) {
        free_traj(l);
        return fail(FFM_E_NOMEM, std::string("trajectory capture: ") + hipGetErrorString(e));
    }
    c.n_sel = n_sel; c.period = period; c.cap = capacity_rows;
    HIP_TRY(hipMemcpyAsync(de, envs, (size_t)n_sel * 4, hipMemcpyHostToDevice, s));
    if (dp) HIP_TRY(hipMemcpyAsync(dp, phases, (size_t)n_sel * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(c.n, 0, 8, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FFM_OK;
}

int ffm_learner_drain_trajectory(ffm_learner* l, int32_t* meta, uint16_t* cells, int64_t cap, int64_t* n,
                                 int64_t* dropped, void* stream) {
    if (!l || !n) return fail(FFM_E_INVALID, "null argument");
    *n = 0;
    if (dropped) *dropped = 0;
    if (l->traj.n_sel == 0) return FFM_OK;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long c = 0;
    HIP_TRY(hipMemcpyAsync(&c, l->traj.n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const long long have = std::min<long long>((long long)c, l->traj.cap);
    if (have > cap) {
        *n = have;
        return fail(FFM_E_INVALID, "drain_trajectory: buffer too small (*n holds the count)");
    }
    const size_t A = (size_t)l->d.agent_capacity;
    if (have > 0 && meta) HIP_TRY(hipMemcpyAsync(meta, l->traj.meta, (size_t)have * 16, hipMemcpyDeviceToHost, s));
    if (have > 0 && cells) HIP_TRY(hipMemcpyAsync(cells, l->traj.cells, (size_t)have * A * 2, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemsetAsync(l->traj.n, 0, 8, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n = have;
    if (dropped) *dropped = (int64_t)c - have;
    return FFM_OK;
}

int ffm_learner_get_step_index(ffm_learner* l, uint32_t* t) {
    if (!l || !t) return fail(FFM_E_INVALID, "null argument");
    *t = l->t;
    return FFM_OK;
}

int ffm_learner_set_step_index(ffm_learner* l, uint32_t t) {
    if (!l) return fail(FFM_E_INVALID, "null learner");
    l->t = t;
    return FFM_OK;
}

}  // extern "C"
