// learn_kernels.h -- host-side launch interface of the learning-variant
// kernels (internal): ffm_ac_core, ffm_unified, ffm_actor_only of
// SoraKurihara/FFM.  See learn_step.hip and DESIGN.md section 9.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ffm {

enum : int { kVarAC = 1, kVarUnified = 2, kVarActorOnly = 3, kVarTrained = 4 };
enum : int { kModeCritic = 0, kModeActor = 1, kModeBoth = 2 };

// Per-agent record kept between the step kernel and the post-update actor
// kernel of ffm_unified's actor_only mode (TD error with the updated V).
struct LearnRec {
    double r;              // reward
    int32_t sv, snv;       // V slots of s and s' (-1 = terminal)
    int32_t hslot;         // H slot of s
    int32_t k;             // chosen action, -1 = none / invalid
};

// Tiled learning step: the large-map batch kernel writes one record
// per agent in cell-raster order instead of adding into the fixed-point accumulators,
// and two tile kernels sum a tile of cells' records in LDS and apply them.  A tile owns
// every slot of its cells (rank-major dense slots: p * (cap / 256) + cell at block 1).
struct TileRec {
    uint32_t svk;               // V / H slot of s (bits 0-26), H(s) inserted by this rank's step (27; owner
                                // exchange: the row is new to every other rank), action k (28-31; 15 = none)
    uint32_t snf;               // V slot of s' (bits 0-26; kTileTerminal = terminal), wexit (27), coll + 1
                                // (28-31: Moore's up to eight requesters of one target)
    double td;                  // ffm_unified both: the TD error with the step-start V (the actor's td);
                                // otherwise the TD target r + gamma V(s') (the V pass subtracts V(s))
};
constexpr int kTileCells = 4;   // cells per tile: a tile's slots are 256 rank patterns x 4 cells
// Tiled tables are dense: cap = the smallest power of two >= 256 * cells <= 2^24, so every slot
// is below 2^24 and the 27-bit fields never hold the terminal marker.
constexpr uint32_t kTileNoAct = 15u, kTileTerminal = 0x07FFFFFFu;
constexpr uint32_t kTileSlot = 0x07FFFFFFu, kTileNewH = 1u << 27;   // svk: slot bits, new-row flag
constexpr int kTileExitBit = 27, kTileCollShift = 28;               // snf: wexit, coll + 1
// Owner outputs: an H increment's key is slot (bits 0-23) | action << 24 (up to 8: Moore's
// stay); bit 31 marks the row's first entry when the row is new this step (receivers insert
// it; q may then be 0).
constexpr uint32_t kHoutSlot = 0x00FFFFFFu, kHoutNew = 1u << 31;
constexpr int kHoutActShift = 24;

struct LearnTable {
    // [cap][stride] 64-bit words, one record per slot: the key (~0 = empty), then
    // its `width` values (empty slots hold the default).  A lookup's probe and the
    // values it then reads share one line: 16 B records for V, 64 B for H.
    unsigned long long* rec;
    uint32_t stride;
    // Batched-step accumulators, accw words per slot.  H (accw = width = 5): the
    // fixed-point (2^-32) sum of alpha_h * td per action.  V (accw = 2): the
    // fixed-point sum of td and the visit count k; the apply moves V by
    // (1 - (1 - alpha)^k) * mean(td), the result of k sequential TD(0) updates
    // towards one target.
    long long* acc;
    uint32_t accw;
    // Hashed tables: `reps` (a power of two) copies of the accumulator array,
    // `rep_stride` words apart; workgroup b adds into copy b % reps.  The 13-cell
    // tables hold a few 10^4 keys, and the popular states take thousands of adds
    // per step: on one copy those adds queue on a few memory-side atomic units.
    // Integer sums do not depend on how they are split, so the apply sums the
    // copies to the same bits.  Dense tables: reps = 1.
    uint32_t reps;
    unsigned long long rep_stride;
    double alpha;               // V: alpha_v (the visit-averaged update); H: unused
    uint32_t* order;            // [cap] slot of the i-th inserted key
    uint32_t* n;                // [1] keys inserted
    uint32_t* mark;             // [1] n at the start of the current batched step (delta export)
    uint32_t mask;              // cap - 1
    // Dense layout (ffm_unified's rank keys): slot = ranks * (cap / 256) + bx * dense_by + by,
    // injective, so no probing and never full.  0 = hashed (13-cell keys).
    uint32_t dense_by;
    uint32_t* present;          // dense: [cap / 32] occupancy bits (lookups hit L2, not the key array)
    uint32_t limit;             // hashed: insertions refused beyond this many keys (7/8 load)
};

// Longest probe sequence a hashed lookup walks before reporting the table full.
constexpr uint32_t kMaxProbe = 4096;

struct LearnArgs {
    int H, W, HW, A, N, F;
    long long E, env_base;
    int variant, mode, bs;      // bs: block size of the state keys
    int D;                      // decisions per agent: 4 for ffm_actor_only, else 1
    int sep_stencil;            // large maps: the DFF stencil runs as its own kernel (set by the launcher)
    const uint8_t* map;         // [HW] raw map values (0 free, 1/2 blocked, 3 exit)
    const uint32_t* map2;       // the same, 2 bits per cell (16 KB at 256x256: stays in L1)
    const float* sff32;         // [HW] raw SFF or nullptr
    const double* sff64;        // [HW] (when sff32 == nullptr)
    float smin, smax;           // min/max of the inf->0 SFF (model/ffm_unified.py:425-426)
    float kS32, kD32;           // f32(-k_S), f32(k_D)
    double kS64, nkA;           // -k_S, -k_A
    float c0, c1;               // DFF coefficients (model/ffm_unified.py:779-798)
    int nb;                     // neighbours: 4 (neumann) or 8 (moore: ffm_ac_core, MT mode only)
    double alpha_v, alpha_h, gamma, exit_reward, step_penalty, collision_penalty, epsilon, v_default;
    uint16_t* pos;              // [E][A]
    int* cnt;                   // [E]
    float* dff_in;              // [E][HW] current DFF (deposits land here)
    float* dff_out;             // [E][HW] next DFF (stencil output)
    int* episodes;              // [E]
    int* ep_steps;              // [E]
    int* done;                  // [E] re-place at the end of this step
    const int* ep_cap;          // [E] episodes env e runs before it stays empty (nullptr: no quota)
    int* nstart;                // [E] live agents at step start
    int v_chain;                // every live agent's V(s) is present: its s was the previous step's s',
                                // inserted then (cleared after set_state / import; an env's first step
                                // after a placement has ep_steps 0)
    unsigned long long* counters;  // [E][4] agent_steps, exits, resets, steps
    LearnTable V, Ht;
    double* hstat;              // [4] has, nonfinite, min, max of H (step start)
    // ffm_trained_core: values of rows held outside the table (ffm_learner_set_h_extra),
    // joined into every H statistics pass
    long long hx_n;
    int hx_nf;
    double hx_mn, hx_mx;
    double* hpart;              // [2 * kHstatBlocks * 4] partials
    LearnRec* recs;             // [E][A]
    TileRec* trecs;             // [E][A] tiled step: per-agent records in raster order (nullptr: off)
    uint16_t* tstart;           // [E][NT + 1] tiled step: agents of env e in cells < kTileCells * t (A <= 16384)
    // the same transposed, [NT + 1][E] (one device, env-major passes): a tile's ranges of
    // all envs are contiguous, so a pass loads them coalesced.  nullptr: read tstart.
    const uint16_t* tstartT;
    uint16_t* tstart_out;       // non-null: the batch step's stencil launch also writes tstartT here
    double* tstats;             // [NT][4] tiled step: per-tile H summary (present, non-finite, min, max)
    int* tdirty;                // [NT] tiled step: bit 0 max, 1 min, 2 non-finite flag only a bound (stale)
    int* tcand;                 // [NT + 1] tiled step: tiles to rescan ([0] = count, then the tiles)
    int NT;                     // tiles: ceil(HW / kTileCells)
    int tile_ensure;            // tile kernels: insert the records' slots (records gathered from other ranks)
    // Tile-major records: the tile passes read trecs through per-range
    // headers instead of the env-major tstart.  Range r (a source rank; one range on one
    // device) is a block of records holding the launch's tiles in order: tile k's records
    // at [thdr[r * ths + k], thdr[r * ths + k + 1]) of the block, thdr[r * ths + NTk] = the
    // block's size; the blocks lie back to back in trecs.  The launch processes NTk tiles:
    // tile k is tile own_tile(k) (ow > 1: the tiles rank orank owns, chunks of ochunk tiles
    // dealt round-robin over ow ranks; ow <= 1: k itself).
    const uint32_t* thdr;       // nullptr: env-major (tstart)
    int tR, ths, NTk;
    long long tblk;             // > 0: range r's block starts at record r * tsrc (fixed-capacity blocks of tblk
                                // records, the sync-free owner exchange; a header offset past tblk is clamped),
    long long tsrc;             // 0: back to back.  tsrc: records between two ranges' blocks (tblk when 0)
    int ow, orank, ochunk;
    // owner mode outputs: the V values the launch's tiles updated (slot, new value) and the
    // H increments (slot | action << 28, fixed-point sum), appended for the other ranks
    uint32_t* vout_slot;
    double* vout_val;
    unsigned long long* vout_n;
    uint32_t* hout_key;
    long long* hout_q;
    unsigned long long* hout_n;
    long long vout_cap, hout_cap;   // output capacities: entries past them are dropped and flagged (overflow 8)
    // Phase-split batch step (learn_batch_phases): per env the 2-bit state
    // maps of the current and next positions, the agents in raster order (cell, agent index)
    // and the decide / resolve outputs per raster rank.  nullptr: the fused batch kernel.
    unsigned char* bph;
    int* overflow;              // [1] table full / reset capacity exceeded
    uint32_t key0, key1, t;
    int auto_reset, max_steps;
    uint32_t* mt_np;            // [E][625] (exact mode)
    uint32_t* mt_py;
    unsigned char* scratch;     // exact mode scratch
    const uint16_t* free_cells;    // [F] placement candidates: x*W+y of the free cells, row-major
                                   // (np.argwhere(map == 0)), or a radius-limited subset of them
    double eps_start, eps_end, eps_offset, eps_span;   // batched epsilon schedule (eps_span > 0)
    int eps_phase;              // > 0: global env g adds (g % eps_phase) * eps_stride to its episode count k
    long long eps_stride;
    uint32_t mW, mBS;           // ceil(2^32 / d) for d = W, bs (0 when d = 1): n / d = mulhi(n, m)
    int* eplog;                 // [eplog_cap][4] ended episodes: global env, index, steps, emptied
    unsigned long long* eplog_n;
    long long eplog_cap;
};

constexpr int kHstatBlocks = 2048;

// Tile ownership across ranks: chunks of kOwnChunk consecutive tiles (one
// 256-cell row at W = 256) dealt round-robin, so the crowded rows near an exit spread over
// every rank.
constexpr int kOwnChunk = 64;
constexpr int kMaxOwners = 64;    // ranks of an owner-sharded exchange (one wave scans the ranges)

// Tiles rank q owns among NT (ow ranks, chunks of C tiles).
inline __host__ __device__ int owner_tiles(int NT, int ow, int C, int q) {
    if (ow <= 1) return NT;
    const int nch = NT / C, rem = NT % C;
    int n = nch > q ? ((nch - 1 - q) / ow + 1) * C : 0;
    if (rem && nch % ow == q) n += rem;
    return n;
}

// Trajectory capture of the batched step (ffm_learner_set_trajectory_capture): the
// selected envs' positions after every step of a captured episode, appended as rows.
struct TrajCapture {
    const int* envs;            // [n_sel] local env indices
    const int* phase;           // [n_sel] episode k is captured iff (k + phase) % period == 0
    int n_sel, period;
    int* meta;                  // [cap][4] global env, episode k, step in the episode (1-based), count
    uint16_t* cells;            // [cap][A] x*W+y, live agents first, 0xFFFF after
    unsigned long long* n;      // rows claimed (past cap: dropped)
    long long cap;
};

size_t learn_exact_scratch_bytes(int HW, int A);
int learn_batch_block_size(int A);
size_t learn_batch_smem_bytes(int HW, int A, int D);
bool learn_batch_supported(int HW, int A, int D);
hipError_t launch_learn_hstat(const LearnArgs& a, hipStream_t s);
hipError_t launch_learn_exact(const LearnArgs& a, hipStream_t s);
hipError_t launch_learn_batch(const LearnArgs& a, hipStream_t s);
hipError_t launch_learn_apply(const LearnArgs& a, bool v, bool h, hipStream_t s);
// hashed V + H applies and the small-map reset (ra: the arguments after the step's DFF swap)
bool learn_reset_small(const LearnArgs& a);
hipError_t launch_learn_apply_reset(const LearnArgs& a, const LearnArgs& ra, hipStream_t s);
hipError_t launch_learn_post(const LearnArgs& a, hipStream_t s);
bool learn_batch_raster(int HW, int A, int D);
// Bytes of LearnArgs::bph for a tiled learner of E envs (0: the shape keeps the fused kernel).
size_t learn_batch_phase_bytes(long long E, int HW, int A);
hipError_t launch_learn_tiles(const LearnArgs& a, bool init_stats, hipStream_t s);
// launch_learn_tiles' env-major actor passes with the re-placement of the ended envs (ra:
// the arguments after the step's DFF swap) fused into the statistics' final launch
hipError_t launch_learn_tiles_reset(const LearnArgs& a, const LearnArgs& ra, hipStream_t s);
// tstart [E][NT + 1] -> out [NT + 1][E] (LearnArgs::tstartT)
hipError_t launch_learn_tstart_transpose(const LearnArgs& a, uint16_t* out, hipStream_t s);
// tile-major records: the column scan, the tile offsets in destination order (per-destination
// headers, hdr row stride ths, and record counts xcnt[ow]) and the scatter of trecs into out.
// pe [E][NT], tpre [NT], toff [NT + 2 * ceil(NT / kOwnChunk)] words.
hipError_t launch_learn_tile_pack(const LearnArgs& a, uint32_t* pe, uint32_t* tpre, uint32_t* toff, uint32_t* hdr,
                                  long long* xcnt, TileRec* out, hipStream_t s);
// owner mode: V table only (critic) or the H passes + statistics inputs, then the exchanges
hipError_t launch_learn_tiles_owner_v(const LearnArgs& a, hipStream_t s);
hipError_t launch_learn_tiles_owner_h(const LearnArgs& a, double* tsum, hipStream_t s);
hipError_t launch_learn_tile_stats(const LearnArgs& a, hipStream_t s);
hipError_t launch_learn_mark(const LearnArgs& a, hipStream_t s);
// The other owners' outputs, [ranks][stride] with the counts on the device (counts[r], capped
// at stride): V values (stored), H increments (applied; a kHoutNew entry inserts its row).
hipError_t launch_learn_v_scatter(const LearnTable& T, const uint32_t* slots, const double* vals, long long stride,
                                  const long long* counts, int ranks, int self, int* overflow, hipStream_t s);
hipError_t launch_learn_h_deltas(const LearnTable& T, const uint32_t* keys, const long long* q, long long stride,
                                 const long long* counts, int ranks, int self, int* overflow, hipStream_t s);
hipError_t launch_learn_tsum_unpack(const LearnArgs& a, const double* tsum, long long stride, hipStream_t s);
hipError_t launch_learn_reset(const LearnArgs& a, int all, hipStream_t s);   // all: 0 ended envs, 1 every env
hipError_t launch_learn_reset_mask(const LearnArgs& a, const uint8_t* mask, hipStream_t s);   // the masked envs
hipError_t launch_learn_fill_default(const LearnArgs& a, hipStream_t s);
hipError_t launch_learn_capture(const LearnArgs& a, const TrajCapture& c, hipStream_t s);
hipError_t launch_learn_clear(const LearnTable& T, int width, double dflt, hipStream_t s);
hipError_t launch_learn_delta_export(const LearnTable& T, int width, unsigned long long* keys, long long* acc,
                                    long long cap, unsigned long long* count, hipStream_t s);
hipError_t launch_learn_delta_merge(const LearnTable& T, int width, const unsigned long long* keys,
                                   const long long* acc, long long n, int* overflow, hipStream_t s,
                                   const long long* dn = nullptr);
hipError_t launch_learn_delta_check(const unsigned long long* count, long long cap, int* overflow, hipStream_t s);
hipError_t launch_learn_dense_adopt(const LearnTable& T, const uint32_t* uni, hipStream_t s);
hipError_t launch_learn_import(const LearnTable& T, int width, const unsigned long long* keys, const double* vals,
                              long long n, int* overflow, hipStream_t s);

}  // namespace ffm
