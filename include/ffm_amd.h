/*
 * ffm_amd.h -- C ABI of the MI355X-native batched floor-field stepper.
 *
 * The reference (SoraKurihara/FFM) has no native boundary: its "plugin" API
 * is the duck-typed model class consumed by the drivers.  Each entry point
 * below is what that class's methods bind to when a binding (ctypes stub in
 * INTEGRATION.md, or ffm_amd/engine.py) replaces the NumPy body:
 *
 *   ffm_engine_create      <- FloorFieldModel.__init__      model/ffm_core.py:7-21
 *   ffm_engine_reset       <- initialize_agents / reset     model/ffm_core.py:23-26
 *                                                           (reset(): model/ffm_ac_core.py:319-325)
 *   ffm_engine_step        <- FloorFieldModel.step          model/ffm_core.py:36-104
 *   ffm_engine_update_dff  <- FloorFieldModel.update_dff    model/ffm_core.py:106-117
 *   ffm_engine_{get,set}_state    <- .positions / .dff attributes (read by
 *                                    main.py:44-46, assigned by run_trained_ffm.py:235-236)
 *   ffm_engine_{get,set}_mt_state <- the process-global np.random / random
 *                                    streams the reference consumes
 *                                    (model/ffm_core.py:25,84,95,96)
 *
 * Conventions: plain pointers and sizes, no torch types.  Host pointers
 * unless the name says "device".  Every function returns 0 on success or a
 * negative FFM_E* code; ffm_last_error() describes the last failure of the
 * calling thread.  One engine per thread at a time (the engine is not
 * re-entrant, like the reference's process-global RNG).  Work is
 * stream-ordered on the hipStream_t passed as `stream` (NULL = null stream);
 * the get/set functions synchronise that stream.
 *
 * Agent positions are cell indices x*W + y stored as uint16 (maps up to
 * 65,536 cells); positions[e][0..count[e]) are the live agents of env e in
 * the reference's order (the row order of FloorFieldModel.positions).
 */
#ifndef FFM_AMD_H
#define FFM_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFM_ABI_VERSION 2

enum {
    FFM_OK = 0,
    FFM_E_INVALID = -1,   /* bad argument / shape / map (ValueError in the reference) */
    FFM_E_HIP = -2,       /* HIP runtime failure */
    FFM_E_NOMEM = -3,
    FFM_E_UNSUPPORTED = -4
};

/* Which model class the engine steps. */
enum {
    FFM_VARIANT_CORE = 0,      /* model/ffm_core.py FloorFieldModel              (ffm_engine_*)  */
    FFM_VARIANT_AC = 1,        /* model/ffm_ac_core.py FloorFieldModel           (ffm_learner_*) */
    FFM_VARIANT_UNIFIED = 2,   /* model/ffm_unified.py FloorFieldModelUnified    (ffm_learner_*) */
    FFM_VARIANT_ACTOR_ONLY = 3, /* model/ffm_actor_only.py FloorFieldModelActorOnly (ffm_learner_*) */
    FFM_VARIANT_TRAINED = 4    /* model/ffm_trained_core.py FloorFieldModel: inference with a trained
                                  H (ffm_learner_*; import the table, nothing is learned) */
};

/* Where the random draws come from. */
enum {
    FFM_RNG_PHILOX = 0,       /* counter-based, keyed (seed, step, env, agent, purpose) */
    FFM_RNG_MT = 1            /* per-env NumPy-legacy + CPython MT19937 streams:
                                 reproduces the reference bit for bit */
};

enum { FFM_SFF_F32 = 0, FFM_SFF_F64 = 1 };

typedef struct {
    int32_t abi_version;      /* = FFM_ABI_VERSION */
    int32_t variant;          /* FFM_VARIANT_* */
    int32_t H, W;             /* map shape; H*W <= 65536 */
    const uint8_t* map;       /* host [H*W]: 0 free, 2 wall, 3 exit (others: blocked) */
    const void* sff;          /* host [H*W] static floor field */
    int32_t sff_dtype;        /* FFM_SFF_F32 / FFM_SFF_F64 (dtype of the .npy, model/ffm_core.py:17) */
    int32_t neighborhood;     /* 4 = "neumann", 8 = "moore" (model/ffm_core.py:28-34) */
    double k_S, k_D, diffuse, decay;   /* params, model/ffm_core.py:8-15 */
    int64_t n_envs;           /* E: independent environments on this device */
    int32_t agent_capacity;   /* A: slots per env (>= n_agents; learners: <= 16383 batched, <= 65535 MT) */
    int32_t n_agents;         /* N placed by reset / auto-reset */
    int32_t rng_mode;         /* FFM_RNG_* */
    int32_t auto_reset;       /* 1: an env emptied by a step is re-placed (Philox, keyed by that
                                 step) and its DFF zeroed at the end of that step */
    uint64_t seed;            /* Philox key */
    int64_t env_base;         /* global id of env 0 (multi-GPU sharding keys RNG by global id) */
    int32_t device;           /* HIP device ordinal */
    int32_t envs_per_block;   /* 0 = auto, > 0 = block kernel with that many envs per workgroup,
                                 -1 = wave kernel (core_step.hip), -2 = lane kernel (core_lane.hip),
                                 -3 = group kernel (core_group.hip; 12x12 only, the auto choice there);
                                 the negative values force a kernel for diagnostics and tests */
} ffm_engine_desc;

typedef struct {
    uint16_t* positions;      /* [E][A] */
    int32_t* counts;          /* [E] */
    float* dff;               /* [E][H*W] */
    int32_t* episodes;        /* [E] completed resets */
    uint64_t* counters;       /* [counter_slots][4]: agent_steps, exits, resets, steps;
                                 one slot per wave/workgroup (uncontended), sum over slots */
    uint32_t* mt_np;          /* [E][625] (MT mode only, else NULL) */
    uint32_t* mt_py;          /* [E][625] */
    int64_t counter_slots;
} ffm_device_buffers;

typedef struct ffm_engine ffm_engine;

const char* ffm_last_error(void);
int ffm_abi_version(void);

int ffm_engine_create(const ffm_engine_desc* desc, ffm_engine** out);
int ffm_engine_destroy(ffm_engine* eng);

/* Place n_agents in every env (Philox mode: keyed by the engine step counter,
 * which then advances), zero the DFF and the per-env episode counters.  MT mode places nothing: the caller
 * draws the placement from its own generator (initialize_agents) and uploads it. */
int ffm_engine_reset(ffm_engine* eng, void* stream);

/* Re-place the envs whose byte in `mask` is nonzero (reset(env_mask); the
 * reference's drivers reset one model per episode: run_unified_actor_training.py:263 ->
 * model/ffm_unified.py:800-812 reset()).  `mask` is a DEVICE pointer to n_envs bytes on the
 * engine's device, read on `stream`.  Philox only: the masked envs get the placement
 * ffm_engine_reset would give them (keyed by the step counter, which then advances), a zero
 * DFF and count n_agents; the other envs are untouched.  Episode counters are not changed
 * (an abandoned episode is not a completed one).  MT mode: FFM_E_UNSUPPORTED. */
int ffm_engine_reset_envs(ffm_engine* eng, const uint8_t* mask, void* stream);

/* Advance every env by n_steps steps (model/ffm_core.py:36-104 each). */
int ffm_engine_step(ffm_engine* eng, int32_t n_steps, void* stream);

/* Steps fused per launch by ffm_engine_step (default 1: one launch per step).
 * k > 1 lets Philox engines of the small-env kernels (A <= 32, W % 4 == 0,
 * H*W <= 256, float32 SFF) step each env pair k times with its state on chip;
 * results equal k single steps bit for bit.  Other engines keep one launch per
 * step.  Returns FFM_E_INVALID for k < 1. */
int ffm_engine_set_fused_steps(ffm_engine* eng, int32_t k);

/* Only the diffusion/decay of the DFF (model/ffm_core.py:106-117). */
int ffm_engine_update_dff(ffm_engine* eng, void* stream);

/* Copy envs [env0, env0+n) in/out.  Any pointer may be NULL to skip it.
 * positions: [n][A] uint16, counts: [n] int32, dff: [n][H*W] float32. */
int ffm_engine_set_state(ffm_engine* eng, int64_t env0, int64_t n, const uint16_t* positions,
                         const int32_t* counts, const float* dff, void* stream);
int ffm_engine_get_state(ffm_engine* eng, int64_t env0, int64_t n, uint16_t* positions,
                         int32_t* counts, float* dff, void* stream);

/* MT mode: per-env generator states, 624 words + position (NumPy
 * get_state()[1:3] / CPython getstate()[1]). */
int ffm_engine_set_mt_state(ffm_engine* eng, int64_t env, const uint32_t* np_key, int32_t np_pos,
                            const uint32_t* py_key, int32_t py_pos, void* stream);
int ffm_engine_get_mt_state(ffm_engine* eng, int64_t env, uint32_t* np_key, int32_t* np_pos,
                            uint32_t* py_key, int32_t* py_pos, void* stream);

/* Trajectory capture of the batched step (replaces the positions log of
 * model/ffm_core.py:119-133 run() and main.py:44-54, which keep a copy of `positions`
 * after every step until the room is empty).  For each selected env (local index) its
 * episode k (0-based, counted from the last ffm_engine_reset; one episode per auto-reset)
 * is captured iff (k + phases[i]) % period == 0 (phases NULL: 0).  After every step of a
 * captured episode one row is appended: meta {global env, k, step in the episode
 * (1-based), count} and the agent_capacity cells (x*W+y, live agents first in the
 * reference's order, 0xFFFF after); an episode's last row is the empty one of the step
 * that emptied the room.  An env that is already empty (auto_reset off) logs nothing.
 * Rows past capacity_rows are dropped and counted.  While capture is on, ffm_engine_step
 * makes one launch per step (fused steps are off).  n_sel = 0 turns capture off. */
int ffm_engine_set_trajectory_capture(ffm_engine* eng, const int32_t* envs, const int32_t* phases, int32_t n_sel,
                                      int32_t period, int64_t capacity_rows, void* stream);
/* Rows captured since the last drain, in no particular order (sort by env, k, step);
 * meta [cap][4] int32, cells [cap][agent_capacity] u16, host pointers. */
int ffm_engine_drain_trajectory(ffm_engine* eng, int32_t* meta, uint16_t* cells, int64_t cap, int64_t* n,
                                int64_t* dropped, void* stream);

/* counters[4] = {agent_steps, exits, resets, steps} accumulated since create. */
int ffm_engine_get_counters(ffm_engine* eng, uint64_t* counters, void* stream);
int ffm_engine_device_buffers(ffm_engine* eng, ffm_device_buffers* out);
/* Step counter (Philox key component); settable for replay. */
int ffm_engine_get_step_index(ffm_engine* eng, uint32_t* t);
int ffm_engine_set_step_index(ffm_engine* eng, uint32_t t);

/* ---- learning variants (ffm_ac_core / ffm_unified / ffm_actor_only) ----
 *
 * A learner owns E envs of one learning model class plus its V (state value)
 * and H (action preference) tables, shared by all E envs.  Reference entry
 * points each function replaces:
 *   ffm_learner_create        <- __init__   model/ffm_ac_core.py:9-38, model/ffm_unified.py:27-129,
 *                                           model/ffm_actor_only.py:21-79
 *   ffm_learner_reset         <- reset()    model/ffm_ac_core.py:319-325, model/ffm_unified.py:800-812
 *   ffm_learner_step          <- step()     model/ffm_ac_core.py:111-236, model/ffm_unified.py:271-606,
 *                                           model/ffm_actor_only.py:149-409
 *   ffm_learner_{export,import}_table <- get_v_table / set_v_table / get_h_table and the
 *                                        pretrained-critic loaders (model/ffm_unified.py:84-110)
 *   ffm_learner_table_size    <- get_v_table_size / get_h_table_size
 *   ffm_learner_set_epsilon   <- set_epsilon (model/ffm_unified.py:859-867)
 *
 * rng_mode FFM_RNG_MT: the reference's semantics bit for bit (per-env NumPy +
 * CPython streams, agents and table updates in the reference's order; envs are
 * stepped one after another).  FFM_RNG_PHILOX: the batched production step
 * (DESIGN.md section 9): all envs in parallel against the tables as they were at
 * the start of the step, increments summed in 2^-32 fixed point, on-device
 * episode ends (emptied or max_steps) with Philox placement.
 * Learning variants take neighborhood 4 ("neumann", every reference driver) or 8
 * ("moore": nine moves and nine-value H rows, model/ffm_unified.py:173-185,
 * model/ffm_actor_only.py:87-93; in both rng modes) and map values in 0..3.  Table keys are packed u64
 * (ffm_amd/learn_keys.py): 2 bits per cell / rank in [0,26), bx in [26,45),
 * by in [45,64).
 */
enum { FFM_LEARN_CRITIC_ONLY = 0, FFM_LEARN_ACTOR_ONLY = 1, FFM_LEARN_BOTH = 2 };
enum { FFM_TABLE_V = 0, FFM_TABLE_H = 1 };

typedef struct {
    int32_t mode;             /* FFM_LEARN_* (ffm_unified learning_mode; ignored otherwise) */
    double k_A;               /* actor logit scale */
    double alpha_v, alpha_h, gamma;
    double exit_reward, step_penalty, collision_penalty;
    double epsilon;           /* eps-greedy (actor modes) */
    double v_default;         /* value a V read inserts: 0.0 (-1.0 after ffm_ac_core.set_v_table) */
    int32_t block_size;       /* state-key block size (ffm_actor_only: always 5) */
    int32_t max_steps;        /* Philox mode: an episode also ends after this many steps (0 = never) */
    int32_t log2_v_capacity;  /* hash-table slots (0 = 21); hashed tables also keep up to 4
                                 copies of their fixed-point accumulators (V 16 B, H 40 B per
                                 slot and copy), fewer when the copies would pass 256 MiB */
    int32_t log2_h_capacity;
    /* Philox mode, eps_span > 0: each env explores with
     * clip(eps_start + (eps_end - eps_start) * (k + eps_offset) / eps_span, 0, 1) after k ended
     * episodes (run_actor_only_training.py:190-196: offset 0, span total episodes - 1;
     * run_unified_actor_training.py:253-259: offset 1, span episodes per configuration). */
    double eps_start, eps_end, eps_offset, eps_span;
} ffm_learn_desc;

typedef struct ffm_learner ffm_learner;

/* FFM_VARIANT_TRAINED: ffm_learner_import_table(FFM_TABLE_H, ...) loads the trained actor
 * (model/ffm_trained_core.py:51-68); steps read it and never change it. */
int ffm_learner_create(const ffm_engine_desc* desc, const ffm_learn_desc* learn, ffm_learner** out);
int ffm_learner_destroy(ffm_learner* l);
/* Philox: place n_agents in every env (keyed by the step counter, which advances),
 * zero the DFF and the per-env episode counters.  MT: zero the DFF and counts only (the caller uploads
 * positions drawn from its own generators, like ffm_engine_reset). */
int ffm_learner_reset(ffm_learner* l, void* stream);
/* reset(env_mask) of the batched learner (model/ffm_unified.py:800-812 per env; the drivers'
 * per-episode reset, run_unified_actor_training.py:263): the envs whose byte in the DEVICE
 * array `mask` (n_envs bytes) is nonzero are re-placed as ffm_learner_reset places them
 * (Philox keyed by the step counter, which then advances; an env past its episode quota
 * stays empty), their DFF zeroed and their episode step count cleared.  Not an episode end:
 * nothing is logged or counted, and the tables are untouched.  Between steps only; MT mode:
 * FFM_E_UNSUPPORTED. */
int ffm_learner_reset_envs(ffm_learner* l, const uint8_t* mask, void* stream);
/* Asynchronous: returns once the steps are queued on `stream`.  A hashed V / H
 * table that passes 7/8 load drops the updates that would insert (the step goes
 * on); that condition (FFM_E_NOMEM) is reported exactly at the next sync point
 * (counters, table export / size, get_state) and, without a sync, by the next
 * ffm_learner_step once the previous call's queued flag copy has landed. */
int ffm_learner_step(ffm_learner* l, int32_t n_steps, void* stream);
int ffm_learner_set_state(ffm_learner* l, int64_t env0, int64_t n, const uint16_t* positions,
                          const int32_t* counts, const float* dff, void* stream);
int ffm_learner_get_state(ffm_learner* l, int64_t env0, int64_t n, uint16_t* positions, int32_t* counts,
                          float* dff, void* stream);
/* episodes[n]: completed episodes per env; ep_steps[n]: steps into the current one. */
int ffm_learner_get_episodes(ffm_learner* l, int64_t env0, int64_t n, int32_t* episodes, int32_t* ep_steps,
                             void* stream);
int ffm_learner_set_mt_state(ffm_learner* l, int64_t env, const uint32_t* np_key, int32_t np_pos,
                             const uint32_t* py_key, int32_t py_pos, void* stream);
int ffm_learner_get_mt_state(ffm_learner* l, int64_t env, uint32_t* np_key, int32_t* np_pos,
                             uint32_t* py_key, int32_t* py_pos, void* stream);
int ffm_learner_get_counters(ffm_learner* l, uint64_t* counters, void* stream);
int ffm_learner_set_epsilon(ffm_learner* l, double epsilon);
int ffm_learner_set_v_default(ffm_learner* l, double v_default, void* stream);
int ffm_learner_table_size(ffm_learner* l, int32_t which, int64_t* n, void* stream);
/* Entries in insertion order (= the reference dict's order in MT mode).
 * vals: [cap][1] (V) or [cap][5] (H).  *n receives the entry count; fails if > cap. */
int ffm_learner_export_table(ffm_learner* l, int32_t which, uint64_t* keys, double* vals, int64_t cap,
                             int64_t* n, void* stream);
/* Replace the table by these entries, inserted in the given order. */
int ffm_learner_import_table(ffm_learner* l, int32_t which, const uint64_t* keys, const double* vals,
                             int64_t n, void* stream);
/* ffm_trained_core (FFM_VARIANT_TRAINED only): values of trained H rows the table cannot
 * hold -- rows whose length is not the move count (model/ffm_trained_core.py:228-249: such
 * a state scores as a missing row, zeros) -- that still join the whole-table min / max of
 * the normalisation (:242-267).  n_values values with these min / max (nonfinite: any of
 * them NaN or inf); n_values = 0 clears.  Kept across import_table. */
int ffm_learner_set_h_extra(ffm_learner* l, int64_t n_values, double min, double max, int32_t nonfinite);
/* The batched (Philox) step in phases, for multi-rank runs whose ranks share
 * the tables (ffm_amd/dist.py TableSync):
 *   step_local -> exchange V (and H unless unified actor_only) -> step_apply(V)
 *   -> [unified actor_only: exchange H] -> step_apply(H) (actor variants) -> step_end.
 * ffm_learner_step == the same phases with no exchange.  A delta record is a
 * key (u64) and its pending accumulators (i64 words: V 2 = the fixed-point sum of td
 * and the visit count, H 5 = the fixed-point alpha_h * td sums per action)
 * for every entry inserted or incremented during this step; a rank merges the
 * other ranks' records (inserting missing keys) before applying, so every rank
 * ends the step with the tables a single device holding all envs would have.
 * Record buffers are DEVICE pointers; export fails with *n = the count needed
 * when cap is too small. */
int ffm_learner_step_local(ffm_learner* l, void* stream);
int ffm_learner_step_apply(ffm_learner* l, int32_t which, void* stream);
int ffm_learner_step_end(ffm_learner* l, void* stream);
int ffm_learner_delta_export(ffm_learner* l, int32_t which, uint64_t* d_keys, int64_t* d_acc, int64_t cap,
                             int64_t* n, void* stream);
int ffm_learner_delta_merge(ffm_learner* l, int32_t which, const uint64_t* d_keys, const int64_t* d_acc,
                            int64_t n, void* stream);
/* The same exchange without host synchronisation (multi-rank steps issue no host
 * sync inside the loop): export writes the record count to the DEVICE int64 d_count
 * (records past cap are dropped; count > cap is reported as FFM_E_INVALID at the next
 * sync point or ffm_learner_step); merge reads min(*d_count, cap) records. */
int ffm_learner_delta_export_async(ffm_learner* l, int32_t which, uint64_t* d_keys, int64_t* d_acc, int64_t cap,
                                   int64_t* d_count, void* stream);
int ffm_learner_delta_merge_async(ffm_learner* l, int32_t which, const uint64_t* d_keys, const int64_t* d_acc,
                                  const int64_t* d_count, int64_t cap, void* stream);
/* The tiled step across ranks (ffm_unified, dense tables at block size 1 on large maps,
 * sync period 1): step_tiled_local runs the step and leaves one 16-B record
 * per agent (raster order) and per-env tile offsets in this learner's DEVICE buffers
 * (tiled_buffers: rec_bytes bytes of records, tstart_count uint16 offsets: agent ranks
 * below agent_capacity <= 16383); the ranks
 * all-gather both, rank-major; step_tiled_apply sums every rank's records per tile of
 * cells into the replicated tables (inserting the slots other ranks created) and ends the
 * step.  Every rank holds, bit for bit, the tables one device stepping all envs would hold.
 * Learners of other kinds return FFM_E_UNSUPPORTED. */
int ffm_learner_tiled_buffers(ffm_learner* l, void** d_recs, int64_t* rec_bytes, uint16_t** d_tstart,
                              int64_t* tstart_count);
int ffm_learner_step_tiled_local(ffm_learner* l, void* stream);
int ffm_learner_step_tiled_apply(ffm_learner* l, const void* d_recs_all, const uint16_t* d_tstart_all,
                                 int64_t n_envs_all, void* stream);
/* The owner-sharded tiled step: the tiles of cells are dealt to the ranks
 * (chunks of 64 tiles round-robin) and each rank sums only its own tiles' records, from all
 * ranks, so the per-rank table work does not grow with the rank count.  Every exchange has a
 * fixed size and the counts travel on the device, so the host queues a whole step without
 * waiting for the GPU (ffm_amd/dist.py TableSync).  Per step:
 *   step_owner_local: the step; the records packed tile-major by destination rank into
 *     fixed-capacity blocks (send_recs: rank q's records at [q * send_rec_capacity, + counts[q]);
 *     send_hdr row q: q's tiles' record offsets within its block, hdr_stride u32 per row);
 *   the ranks all-to-all the record blocks (equal splits) and header rows;
 *   step_owner_v: sums this rank's tiles' V (d_recs: the received blocks, rank-major, each
 *     send_rec_capacity records; d_hdrs: the received header rows) and writes the updated V
 *     values to v_slot / v_val (out_counts[0] of them, at most v_capacity);
 *   the ranks all-gather v_capacity entries and the count;
 *   step_owner_h: stores the other ranks' V values; actor modes sum this rank's tiles' H
 *     (h_key = slot (bits 0-23) | action << 24 (0-8: Moore's stay is 8), bit 31 on the first
 *     entry of a row another rank's step
 *     created; h_q = the fixed-point increment; out_counts[1] entries, at most h_capacity)
 *     and write the tiles' H summaries (tsum, tsum_count rows of 5 doubles);
 *   the ranks all-gather h_capacity entries, the count and the summaries;
 *   step_owner_end: inserts the flagged rows, applies the other ranks' H increments and
 *     summaries, the H statistics, ends the step.
 * Counts are DEVICE int64 arrays ([world], rank-major), as are every buffer; "_all"
 * buffers are rank-major with the given row stride in elements.  A count past its capacity
 * is reported at the next sync point (FFM_E_INVALID), never silently dropped.  Every rank
 * ends each step with the H table (keys and values) and the V values one device stepping
 * all envs would hold, bit for bit; the V slots other ranks inserted join a rank's key set
 * when the presence bitmaps are merged (ffm_learner_dense_buffers + dense_adopt, which a
 * shared learner accepts between steps as well): TableSync does so before every export or
 * size query.  set_owner_capacity sizes the buffers (records per destination, V and H output
 * entries); pointers change only there. */
typedef struct ffm_owner_buffers {
    int32_t world, rank;
    void* send_recs;                 /* 16-B records, world blocks of send_rec_capacity */
    int64_t send_rec_capacity;
    uint32_t* send_hdr;
    int64_t hdr_stride;
    int64_t* counts;                 /* [world] records per destination (device) */
    uint32_t* v_slot;
    double* v_val;
    uint32_t* h_key;
    int64_t* h_q;
    int64_t* out_counts;             /* [2] V values, H increments (device) */
    int64_t v_capacity, h_capacity;
    double* tsum;
    int64_t tsum_count;
} ffm_owner_buffers;
int ffm_learner_set_tile_owners(ffm_learner* l, int32_t world, int32_t rank);
int ffm_learner_set_owner_capacity(ffm_learner* l, int64_t rec_capacity, int64_t v_capacity, int64_t h_capacity);
int ffm_learner_owner_buffers(ffm_learner* l, ffm_owner_buffers* b);
int ffm_learner_step_owner_local(ffm_learner* l, void* stream);
/* src_stride: records between two sources' blocks in d_recs (0 = send_rec_capacity: the
 * all-to-all's receive buffer).  set_owner_send_buffer: pack into a caller's device buffer of
 * world * send_rec_capacity records instead (NULL: the learner's own), e.g. one allocation
 * shared by coupled shards, which then read each other's blocks in place. */
int ffm_learner_set_owner_send_buffer(ffm_learner* l, void* d_buf);
/* The V / H outputs written into caller buffers (v_capacity / h_capacity entries, the counts
 * as int64) instead of the learner's own, e.g. rows of the gathered buffers coupled shards
 * read in place; NULLs restore the learner's own.  owner_buffers keeps describing its own. */
int ffm_learner_set_owner_output_buffers(ffm_learner* l, uint32_t* v_slot, double* v_val, int64_t* v_count,
                                         uint32_t* h_key, int64_t* h_q, int64_t* h_count);
int ffm_learner_step_owner_v(ffm_learner* l, const void* d_recs, const uint32_t* d_hdrs, int64_t src_stride,
                             void* stream);
int ffm_learner_step_owner_h(ffm_learner* l, const uint32_t* d_v_slot, const double* d_v_val,
                             const int64_t* d_v_counts, int64_t v_stride, void* stream);
int ffm_learner_step_owner_end(ffm_learner* l, const uint32_t* d_h_key, const int64_t* d_h_q,
                               const int64_t* d_h_counts, int64_t h_stride, const double* d_tsum_all,
                               int64_t tsum_stride, void* stream);
/* Table sync period K >= 1 (default 1 = the reference's per-step updates): the fixed-point
 * increments of K steps accumulate and V / H (and the actor's H statistics) are applied
 * at every K-th step only; a multi-rank run exchanges deltas at those steps only, so
 * sharded == one device at the same K, bit for bit.  apply_due: 1 if the current (or
 * next) step's step_apply applies.  A table export / import or a new period between two
 * applies first applies the pending increments (the period ends at the last step) and
 * restarts the period. */
int ffm_learner_set_sync_period(ffm_learner* l, int32_t period);
int ffm_learner_apply_due(ffm_learner* l, int32_t* due);
/* A learner whose tables are shared with other ranks (TableSync sets it): an export is
 * read-only (the tables as of the last apply: the pending increments are only this rank's),
 * an import or a new period between two applies fails, and the pending increments are
 * applied collectively: flush_begin (*pending = 1 opens a phase in which the deltas are
 * exchanged as in a step) -> exchange V and H -> flush_end (applies them, restarts the
 * period).  *pending = 0: nothing pending, no phase opened. */
int ffm_learner_set_external_sync(ffm_learner* l, int32_t on);
int ffm_learner_flush_begin(ffm_learner* l, int32_t* pending);
int ffm_learner_flush_end(ffm_learner* l, void* stream);
/* Dense (ffm_unified rank-key) tables: the device fixed-point accumulators (acc_count
 * int64) and presence bitmap (present_words u32), for an all-reduce of the increments;
 * dense_adopt then takes the presence union of all ranks (a DEVICE bitmap): slots other
 * ranks inserted get their keys.  Between step_local and step_apply (or, for a tiled learner,
 * between steps). */
int ffm_learner_dense_buffers(ffm_learner* l, int32_t which, int64_t** d_acc, int64_t* acc_count,
                              uint32_t** d_present, int64_t* present_words);
int ffm_learner_dense_adopt(ffm_learner* l, int32_t which, const uint32_t* d_union, void* stream);
/* Philox placement candidates of later resets: `count` distinct free cells (x*W+y) and the
 * agents to place, <= count (the radius curriculum, model/ffm_unified.py:150-171:
 * actual_N = min(N, cells within the radius)).  count = 0 restores every free cell. */
int ffm_learner_set_placement(ffm_learner* l, const uint16_t* cells, int32_t count, int32_t n_agents);
int ffm_learner_set_epsilon_schedule(ffm_learner* l, double eps_start, double eps_end, double eps_offset,
                                     double eps_span);
/* period > 0: global env g explores as if g % period more episodes had ended (k + g % period
 * in the schedule above), so E >= P envs that each run one episode of a configuration cover a
 * P-episode per-configuration schedule (run_unified_actor_training.py:253-259) between them;
 * 0 = off (the default). */
int ffm_learner_set_epsilon_phase(ffm_learner* l, int32_t period);
/* stride >= 1 (default 1): global env g adds (g % period) * stride instead, so envs that each
 * run `stride` episodes cover a run-wide schedule with episodes numbered env-major (the single
 * linear schedule over all episodes of run_actor_only_training.py:186-196). */
int ffm_learner_set_epsilon_stride(ffm_learner* l, int64_t stride);
/* Per-env episode quota of the auto-reset (the drivers' episode counts,
 * run_actor_only_training.py:186-188 / run_unified_actor_training.py:247-252: the run stops
 * after P episodes): env e is re-placed until it has ended caps[e] episodes since the last
 * ffm_learner_reset, then stays empty (no agents, no table reads or increments) until the
 * next reset; caps[e] <= 0 leaves env e empty from the reset on.  n = n_envs (host array)
 * sets the quotas, n = 0 removes them (every env re-placed forever, the default). */
int ffm_learner_set_episode_caps(ffm_learner* l, const int32_t* caps, int64_t n);
/* Ended episodes since the last drain, in no particular order: records of 4 int32
 * {global env, episode index, steps, 1 = emptied / 0 = truncated at max_steps}
 * (the per-episode rows of run_*_training.py's steps_per_episode.csv).  *dropped counts
 * records lost because the log was full (capacity max(16 E, 4096): an env ends at most one
 * episode per step, so draining every 16 steps never loses one). */
int ffm_learner_drain_episodes(ffm_learner* l, int32_t* records, int64_t cap, int64_t* n, int64_t* dropped,
                               void* stream);
/* Trajectory capture of the batched step (replaces run(max_steps, return_trajectory=True),
 * model/ffm_unified.py:902-931 / model/ffm_actor_only.py, and the driver's every-100th-episode
 * trajectory files, run_actor_only_training.py:199-218).  For each selected env (local index)
 * its episode k (0-based, counted from the last ffm_learner_reset) is captured iff
 * (k + phases[i]) % period == 0 (phases NULL: 0).  After every step of a captured episode one
 * row is appended: meta {global env, k, step in the episode (1-based), count} and the
 * agent_capacity cells (x*W+y, live agents first in the reference's order, 0xFFFF after),
 * i.e. the reference's `positions` after that step.  Rows past capacity_rows are dropped and
 * counted.  n_sel = 0 turns capture off.  Batched (Philox) learners only. */
int ffm_learner_set_trajectory_capture(ffm_learner* l, const int32_t* envs, const int32_t* phases, int32_t n_sel,
                                       int32_t period, int64_t capacity_rows, void* stream);
/* Rows captured since the last drain, in no particular order within a step (sort by
 * env, k, step); meta [cap][4] int32, cells [cap][agent_capacity] u16, host pointers. */
int ffm_learner_drain_trajectory(ffm_learner* l, int32_t* meta, uint16_t* cells, int64_t cap, int64_t* n,
                                 int64_t* dropped, void* stream);
int ffm_learner_get_step_index(ffm_learner* l, uint32_t* t);
int ffm_learner_set_step_index(ffm_learner* l, uint32_t t);

/* ---- numerics probes (used by the parity tests) ---------------------- */
/* y[i] = NumPy-exact float32 exp(x[i]) computed on the device; device pointers. */
int ffm_np_expf_device(const float* x, float* y, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FFM_AMD_H */
