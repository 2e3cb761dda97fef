/*
 * ffm_learn_oracle.h -- CPU restatement of SoraKurihara/FFM's learning
 * variants: model/ffm_ac_core.py, model/ffm_unified.py (critic_only /
 * actor_only / both) and model/ffm_actor_only.py.
 *
 * TEST INFRASTRUCTURE ONLY (like ffm_oracle.h): used by tests/ and by
 * bench.py's cpu_baseline leg, never by the product.
 *
 * Two semantics:
 *  * MT ("exact"): one env, the reference's two global MT19937 streams, the
 *    tables read and written in agent order exactly as the reference's dicts
 *    (Gauss-Seidel).  Pinned by tests/golden/learn_*.npz, recorded from the
 *    reference itself (tests/golden/gen_golden_learn.py).
 *  * FFO_VAR_TRAINED restates model/ffm_trained_core.py: the rank-keyed H table
 *    of a trained actor, read only (missing states score as zeros), float32
 *    policy arithmetic, conflicts always have a winner, no learning.
 *  * Philox ("batched"): every env of a batch steps against
 *    the tables as they were at the start of the step; the TD and actor
 *    increments of all envs are summed in 2^-32 fixed point (order-free, so
 *    deterministic) and applied once per step.  This is the GPU's production
 *    semantics; GPU == this code bit for bit.
 *
 * State keys are packed u64 (ffm_amd/learn_keys.py): 2 bits per cell / rank
 * in [0,26), bx in [26,45), by in [45,64).
 */
#ifndef FFM_LEARN_ORACLE_H
#define FFM_LEARN_ORACLE_H

#include <stdint.h>
#include "ffm_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { FFO_VAR_AC = 1, FFO_VAR_UNIFIED = 2, FFO_VAR_ACTOR_ONLY = 3, FFO_VAR_TRAINED = 4 };
enum { FFO_MODE_CRITIC = 0, FFO_MODE_ACTOR = 1, FFO_MODE_BOTH = 2 };

typedef struct {
    int32_t H, W;
    const uint8_t* map;       /* raw map values 0..3 (state maps use them as-is) */
    const float* sff32;       /* raw SFF (inf on walls) or NULL */
    const double* sff64;      /* used when sff32 == NULL */
    int32_t variant, mode;
    double k_S, k_D, k_A, diffuse, decay;
    double alpha_v, alpha_h, gamma, exit_reward, step_penalty, collision_penalty;
    double epsilon;
    double v_default;         /* value of a V entry created by a read (0.0; -1.0 after set_v_table, ac) */
    int32_t block_size;
    /* batched epsilon schedule (eps_span > 0): an env whose k episodes have ended
     * explores with clip(eps_start + (eps_end - eps_start) * (k + eps_offset) / eps_span)
     * (run_actor_only_training.py:190-196: offset 0, span total-1;
     * run_unified_actor_training.py:253-259: offset 1, span episodes per config) */
    double eps_start, eps_end, eps_offset, eps_span;
    int32_t nb;               /* neighbours: 4 (neumann; 0 means 4) or 8 (moore, ffm_ac_core) */
    int32_t eps_phase;        /* > 0: global env g adds (g % eps_phase) * eps_stride to k (envs spread over the schedule) */
    int64_t eps_stride;       /* 0 means 1 */
} ffo_learn_cfg;

typedef struct ffo_tab ffo_tab;

ffo_tab* ffo_tab_new(int32_t width, int32_t log2_cap);
void ffo_tab_free(ffo_tab* t);
int64_t ffo_tab_size(const ffo_tab* t);
/* entries in insertion order (the reference dict's order in MT mode) */
void ffo_tab_export(const ffo_tab* t, uint64_t* keys, double* vals);
/* insert/overwrite in the given order */
int ffo_tab_import(ffo_tab* t, const uint64_t* keys, const double* vals, int64_t n);

/* Reference-exact step of one env (MT streams).  pos: int32 cells x*W+y. */
int ffo_learn_step_mt(const ffo_learn_cfg* c, ffo_tab* V, ffo_tab* Ht, int32_t* pos, int32_t* n,
                      float* dff, ffo_mt* np_rng, ffo_mt* py_rng);

/* Batched Philox step of E envs (see header comment).  pos [E][A_cap] u16,
 * counts [E], dff [E][H*W], episodes [E], ep_steps [E] (steps in the current
 * episode).  An env is re-placed (N_reset agents, DFF zeroed) at the end of a
 * step that empties it or that reaches max_steps (> 0). */
int ffo_learn_step_philox_batch(const ffo_learn_cfg* c, ffo_tab* V, ffo_tab* Ht, int64_t E,
                                int32_t A_cap, uint16_t* pos, int32_t* counts, float* dff,
                                int32_t* episodes, int32_t* ep_steps, uint64_t seed, uint32_t t,
                                int32_t auto_reset, int32_t N_reset, int32_t max_steps,
                                int64_t env_base, uint64_t* agent_steps, int nthreads);

/* The batched step in phases, for multi-rank runs:
 * local (every env against the current tables, increments pending) ->
 * exchange (delta export / merge per table) -> apply V (+ the post-update
 * actor increments of ffm_unified actor_only) -> exchange H -> apply H -> end
 * (episode ends).  ffo_learn_step_philox_batch = local, apply 0, apply 1, end. */
typedef struct ffo_lbatch ffo_lbatch;
ffo_lbatch* ffo_lbatch_new(const ffo_learn_cfg* c, ffo_tab* V, ffo_tab* Ht, int64_t E, int32_t A_cap);
void ffo_lbatch_free(ffo_lbatch* b);
int ffo_lbatch_local(ffo_lbatch* b, uint16_t* pos, int32_t* counts, float* dff, const int32_t* episodes,
                     uint64_t seed, uint32_t t, int64_t env_base, uint64_t* agent_steps, int nthreads);
/* Placement candidates of the episode ends (default: every free cell). */
void ffo_lbatch_set_placement(ffo_lbatch* b, const uint16_t* cells, int32_t count);
void ffo_lbatch_apply(ffo_lbatch* b, int which);
void ffo_lbatch_post(ffo_lbatch* b);
void ffo_lbatch_flush(ffo_lbatch* b);
/* Episode ends; log (may be NULL) receives one record per ended episode:
 * {global env, index of the episode, its steps, 1 if emptied / 0 if truncated};
 * returns the record count. */
int64_t ffo_lbatch_end(ffo_lbatch* b, uint16_t* pos, int32_t* counts, float* dff, int32_t* episodes,
                       int32_t* ep_steps, uint64_t seed, uint32_t t, int32_t auto_reset, int32_t N_reset,
                       int32_t max_steps, int64_t env_base, int32_t* log);
void ffo_tab_mark(ffo_tab* t);
int64_t ffo_tab_delta_export(const ffo_tab* t, uint64_t* keys, int64_t* acc);
int32_t ffo_tab_accw(const ffo_tab* t);
void ffo_tab_set_alpha(ffo_tab* t, double alpha);
int ffo_tab_delta_merge(ffo_tab* t, const uint64_t* keys, const int64_t* acc, int64_t n, const double* init);
void ffo_tab_apply(ffo_tab* t);
void ffo_tab_set_extra(ffo_tab* t, const double* vals, int64_t n);

/* Deterministic float64 exp (fdlibm's algorithm, +,*,/ only): the f64
 * softmax of the actor modes on CPU and GPU alike. */
double ffo_det_exp(double x);

/* State encoders (exposed for unit tests). sm = state map [H*W]. */
uint64_t ffo_encode_rank(const uint8_t* sm, int H, int W, int x, int y, int bs);
uint64_t ffo_encode_cells13(const uint8_t* sm, int H, int W, int x, int y, int bs, int oob);

#ifdef __cplusplus
}
#endif
#endif
