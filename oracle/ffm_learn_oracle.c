/*
 * ffm_learn_oracle.c -- CPU restatement of the learning variants of
 * SoraKurihara/FFM (model/ffm_ac_core.py, model/ffm_unified.py,
 * model/ffm_actor_only.py).  TEST INFRASTRUCTURE ONLY (see the header).
 *
 * Compiled with -ffp-contract=off: every float operation rounds on its own,
 * as in NumPy's element-wise loops and CPython float arithmetic.
 */
#include "ffm_learn_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EMPTY_KEY (~(uint64_t)0)
#define FX_ONE 4294967296.0            /* 2^32: fixed-point scale of batched increments */

static const int NB[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};   /* U, D, L, R: model/ffm_unified.py:174-175 */
/* Moore order of ffm_ac_core.get_neighbors (model/ffm_ac_core.py:51-60) */
static const int MB[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};
static int cfg_nb(const ffo_learn_cfg* c) { return c->nb == 8 ? 8 : 4; }
static int nbx(int nb, int k) { return nb == 8 ? MB[k][0] : NB[k][0]; }
static int nby(int nb, int k) { return nb == 8 ? MB[k][1] : NB[k][1]; }

/* ======================================================================
 * Hash table with insertion order (a Python dict of packed keys).
 * ====================================================================== */
struct ffo_tab {
    int32_t width;
    int32_t accw;          /* accumulator words per slot: V 2 (sum of td, visits), H = width */
    double alpha;          /* V: alpha_v of the visit-averaged batched update */
    int64_t cap, n;
    int64_t mark;          /* n at the start of the current batched step */
    uint64_t* keys;
    double* vals;
    int64_t* acc;          /* batched fixed-point accumulators */
    int64_t* order;        /* slot of the i-th inserted key */
    /* ffm_trained_core: values of rows whose length is not the move count (a state with
     * such a row scores as missing, yet its values join the table's min / max,
     * model/ffm_trained_core.py:228-267) */
    int64_t xn;
    int xnf;
    double xmn, xmx;
};

static uint64_t mix64(uint64_t z) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}

ffo_tab* ffo_tab_new(int32_t width, int32_t log2_cap) {
    ffo_tab* t = (ffo_tab*)calloc(1, sizeof(ffo_tab));
    t->width = width;
    t->accw = width == 1 ? 2 : width;
    t->cap = (int64_t)1 << log2_cap;
    t->keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)t->cap);
    t->vals = (double*)calloc((size_t)(t->cap * width), sizeof(double));
    t->acc = (int64_t*)calloc((size_t)(t->cap * t->accw), sizeof(int64_t));
    t->order = (int64_t*)malloc(sizeof(int64_t) * (size_t)t->cap);
    for (int64_t i = 0; i < t->cap; i++) t->keys[i] = EMPTY_KEY;
    return t;
}

void ffo_tab_free(ffo_tab* t) {
    if (!t) return;
    free(t->keys); free(t->vals); free(t->acc); free(t->order); free(t);
}

int64_t ffo_tab_size(const ffo_tab* t) { return t->n; }

void ffo_tab_export(const ffo_tab* t, uint64_t* keys, double* vals) {
    for (int64_t i = 0; i < t->n; i++) {
        int64_t s = t->order[i];
        if (keys) keys[i] = t->keys[s];
        if (vals) memcpy(vals + i * t->width, t->vals + s * t->width, sizeof(double) * (size_t)t->width);
    }
}

/* slot of `key`, inserting it with `init` (width values) when absent; -1 when full */
static int64_t tab_get(ffo_tab* t, uint64_t key, const double* init) {
    int64_t h = (int64_t)(mix64(key) & (uint64_t)(t->cap - 1));
    for (;;) {
        if (t->keys[h] == key) return h;
        if (t->keys[h] == EMPTY_KEY) break;
        h = (h + 1) & (t->cap - 1);
    }
    if (t->n * 8 >= t->cap * 7) return -1;
    t->keys[h] = key;
    memcpy(t->vals + h * t->width, init, sizeof(double) * (size_t)t->width);
    t->order[t->n++] = h;
    return h;
}

/* slot of `key` or -1 (no insertion) */
static int64_t tab_find(const ffo_tab* t, uint64_t key) {
    int64_t h = (int64_t)(mix64(key) & (uint64_t)(t->cap - 1));
    for (;;) {
        if (t->keys[h] == key) return h;
        if (t->keys[h] == EMPTY_KEY) return -1;
        h = (h + 1) & (t->cap - 1);
    }
}

static int64_t tab_get_sync(ffo_tab* t, uint64_t key, const double* init, int parallel) {
    int64_t s;
    if (parallel) {
#ifdef _OPENMP
#pragma omp critical(ffo_tab_insert)
#endif
        s = tab_get(t, key, init);
    } else {
        s = tab_get(t, key, init);
    }
    return s;
}

/* ---- delta exchange of the batched step (multi-rank) ---- */
void ffo_tab_mark(ffo_tab* t) { t->mark = t->n; }

/* Entries touched since the mark: inserted after it, or with pending increments.
 * keys [n], acc [n][accw]; returns n. */
int64_t ffo_tab_delta_export(const ffo_tab* t, uint64_t* keys, int64_t* acc) {
    int64_t m = 0;
    const int w = t->accw;
    for (int64_t i = 0; i < t->n; i++) {
        const int64_t s = t->order[i];
        int touched = i >= t->mark;
        for (int k = 0; k < w; k++) touched |= t->acc[s * w + k] != 0;
        if (!touched) continue;
        keys[m] = t->keys[s];
        memcpy(acc + m * w, t->acc + s * w, sizeof(int64_t) * (size_t)w);
        m++;
    }
    return m;
}

int32_t ffo_tab_accw(const ffo_tab* t) { return t->accw; }
void ffo_tab_set_alpha(ffo_tab* t, double alpha) { t->alpha = alpha; }

/* V after k visits of one batched step with summed fixed-point td q: k sequential
 * TD(0) updates towards the mean target, V + (1 - (1 - alpha)^k) * mean(td)
 * (ffm_amd/csrc/learn_step.hip v_visits: the same operation sequence). */
static double ffo_v_visits(double v, int64_t q, int64_t k, double alpha) {
    const double mean = (double)q * (1.0 / FX_ONE) / (double)k;
    double p = 1.0, b = 1.0 - alpha;
    for (int64_t e = k; e; e >>= 1) {
        if (e & 1) p = p * b;
        b = b * b;
    }
    return v + (1.0 - p) * mean;
}

/* Add another rank's records: insert missing keys with `init`, add increments. */
int ffo_tab_delta_merge(ffo_tab* t, const uint64_t* keys, const int64_t* acc, int64_t n, const double* init) {
    for (int64_t r = 0; r < n; r++) {
        const int64_t s = tab_get(t, keys[r], init);
        if (s < 0) return -1;
        for (int k = 0; k < t->accw; k++) t->acc[s * t->accw + k] += acc[r * t->accw + k];
    }
    return 0;
}

/* Applies the pending increments; the next delta export starts from here (the
 * device's apply kernels set their mark the same way). */
void ffo_tab_apply(ffo_tab* t) {
    if (t->width == 1) {   /* V: visit-averaged */
        for (int64_t s = 0; s < t->cap; s++)
            if (t->acc[2 * s + 1]) {
                t->vals[s] = ffo_v_visits(t->vals[s], t->acc[2 * s], t->acc[2 * s + 1], t->alpha);
                t->acc[2 * s] = 0;
                t->acc[2 * s + 1] = 0;
            }
    } else {
        for (int64_t s = 0; s < t->cap * t->width; s++)
            if (t->acc[s]) { t->vals[s] = t->vals[s] + (double)t->acc[s] * (1.0 / FX_ONE); t->acc[s] = 0; }
    }
    t->mark = t->n;
}

int ffo_tab_import(ffo_tab* t, const uint64_t* keys, const double* vals, int64_t n) {
    for (int64_t i = 0; i < n; i++) {
        int64_t s = tab_get(t, keys[i], vals + i * t->width);
        if (s < 0) return -1;
        memcpy(t->vals + s * t->width, vals + i * t->width, sizeof(double) * (size_t)t->width);
    }
    t->mark = t->n;
    return 0;
}

/* ======================================================================
 * Deterministic float64 exp: fdlibm e_exp.c's reduction and rational
 * correction, + - * / only, so CPU and GPU agree bit for bit.
 * ====================================================================== */
double ffo_det_exp(double x) {
    if (x != x) return x;
    if (x > 709.782712893383973096) return INFINITY;
    if (x < -745.13321910194110842) return 0.0;
    const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    double kd = rint(x * invln2);
    double hi = x - kd * ln2HI;
    double lo = kd * ln2LO;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    return ldexp(y, (int)kd);
}

/* ======================================================================
 * State encoders.
 * ====================================================================== */
static uint64_t pack_key(uint64_t cells, int64_t bx, int64_t by) {
    return cells | ((uint64_t)bx << 26) | ((uint64_t)by << 45);
}

/* model/ffm_unified.py:188-269: rank per direction U, D, L, R. */
uint64_t ffo_encode_rank(const uint8_t* sm, int H, int W, int x, int y, int bs) {
    uint64_t cells = 0;
    for (int d = 0; d < 4; d++) {
        const int dx = NB[d][0], dy = NB[d][1];
        int rank = 3;
        const int nx1 = x + dx, ny1 = y + dy;
        if (nx1 >= 0 && nx1 < H && ny1 >= 0 && ny1 < W) {
            const uint8_t v1 = sm[nx1 * W + ny1];
            if (v1 == 2 || v1 == 1) {
                rank = 0;                                           /* :219-220 */
            } else {
                int ax, ay, bx_, by_;
                if (dx != 0) { ax = nx1; ay = ny1 - 1; bx_ = nx1; by_ = ny1 + 1; }
                else { ax = nx1 - 1; ay = ny1; bx_ = nx1 + 1; by_ = ny1; }   /* :224-229 */
                int diag = 0;
                if (ax >= 0 && ax < H && ay >= 0 && ay < W && sm[ax * W + ay] == 1) diag = 1;
                if (!diag && bx_ >= 0 && bx_ < H && by_ >= 0 && by_ < W && sm[bx_ * W + by_] == 1) diag = 1;
                if (diag) {
                    rank = 1;                                       /* :239-240 */
                } else {
                    const int nx2 = x + 2 * dx, ny2 = y + 2 * dy;
                    if (nx2 >= 0 && nx2 < H && ny2 >= 0 && ny2 < W) {
                        const uint8_t v2 = sm[nx2 * W + ny2];
                        if (v2 == 2 || v2 == 1) rank = 2;           /* :245-248 */
                    } else {
                        rank = 2;                                   /* :249-251 */
                    }
                }
            }
        } else {
            rank = 0;                                               /* :252-254 */
        }
        cells |= (uint64_t)rank << (2 * d);
    }
    return pack_key(cells, x / bs, y / bs);                        /* :262 */
}

/* model/ffm_ac_core.py:62-109 (oob = 2, block_size param) and
 * model/ffm_actor_only.py:102-147 (oob = 0, block 5): padded 3x3 row-major,
 * then the cells two ahead U, D, L, R. */
uint64_t ffo_encode_cells13(const uint8_t* sm, int H, int W, int x, int y, int bs, int oob) {
    uint64_t cells = 0;
    int i = 0;
    for (int dx = -1; dx <= 1; dx++)
        for (int dy = -1; dy <= 1; dy++, i++) {
            const int nx = x + dx, ny = y + dy;
            const int v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? sm[nx * W + ny] : oob;
            cells |= (uint64_t)(v & 3) << (2 * i);
        }
    static const int AH[4][2] = {{-2, 0}, {2, 0}, {0, -2}, {0, 2}};
    for (int d = 0; d < 4; d++, i++) {
        const int nx = x + AH[d][0], ny = y + AH[d][1];
        const int v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? sm[nx * W + ny] : oob;
        cells |= (uint64_t)(v & 3) << (2 * i);
    }
    return pack_key(cells, x / bs, y / bs);
}

static uint64_t encode(const ffo_learn_cfg* c, const uint8_t* sm, int x, int y) {
    if (c->variant == FFO_VAR_TRAINED) return ffo_encode_rank(sm, c->H, c->W, x, y, c->block_size);
    if (c->variant == FFO_VAR_UNIFIED) return ffo_encode_rank(sm, c->H, c->W, x, y, c->block_size);
    if (c->variant == FFO_VAR_AC) return ffo_encode_cells13(sm, c->H, c->W, x, y, c->block_size, 2);
    return ffo_encode_cells13(sm, c->H, c->W, x, y, 5, 0);         /* block_size = 5 hard-coded, :143 */
}

/* ======================================================================
 * Random draws.  MT: the reference's np.random (choice, randint) and random
 * (random, choice) streams.  Philox: a stream per decision keyed
 * (t, env, seq, DECIDE) and one per contested target keyed by its owner's
 * seq (t, env, owner, FRICTION).
 * ====================================================================== */
enum { PUR_DECIDE = 1, PUR_FRICTION = 2 };

typedef struct {
    uint32_t ctr[4], key[2], buf[4];
    int used;
} pstream;

static void ps_init(pstream* p, uint64_t seed, uint32_t t, uint64_t genv, uint32_t idx, uint32_t pur) {
    p->key[0] = (uint32_t)seed; p->key[1] = (uint32_t)(seed >> 32);
    p->ctr[0] = t; p->ctr[1] = (uint32_t)genv; p->ctr[2] = idx; p->ctr[3] = pur << 28;
    p->used = 4;
}

static uint32_t ps_next(pstream* p) {
    if (p->used == 4) { ffo_philox(p->ctr, p->key, p->buf); p->ctr[3]++; p->used = 0; }
    return p->buf[p->used++];
}

static double u53w(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

static int bitlen(uint32_t n) { int k = 0; while (n) { k++; n >>= 1; } return k; }

typedef struct {
    int philox;
    ffo_mt *np, *py;
    uint64_t seed;
    uint32_t t;
    uint64_t genv;
    pstream ds;            /* current decision stream (Philox) */
} lrng;

static void dec_begin(lrng* r, uint32_t seq) {
    if (r->philox) ps_init(&r->ds, r->seed, r->t, r->genv, seq, PUR_DECIDE);
}
static double dec_coin(lrng* r) {            /* random.random() (eps-greedy) */
    if (!r->philox) return ffo_mt_u53(r->py);
    uint32_t a = ps_next(&r->ds), b = ps_next(&r->ds);
    return u53w(a, b);
}
static double dec_u53(lrng* r) {             /* np.random.choice(p) */
    if (!r->philox) return ffo_mt_u53(r->np);
    uint32_t a = ps_next(&r->ds), b = ps_next(&r->ds);
    return u53w(a, b);
}
static uint32_t dec_randint(lrng* r, uint32_t n) {   /* np.random.randint(n): masked rejection */
    if (!r->philox) return ffo_np_interval(r->np, n - 1);
    uint32_t max = n - 1;
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (ps_next(&r->ds) & mask)) > max) {}
    return v;
}
static uint32_t conflict_pick(lrng* r, uint32_t owner_seq, uint32_t m) {   /* random.choice(agents) */
    if (!r->philox) return ffo_py_randbelow(r->py, m);
    pstream p;
    ps_init(&p, r->seed, r->t, r->genv, owner_seq, PUR_FRICTION);
    const int k = bitlen(m);
    uint32_t v = ps_next(&p) >> (32 - k);
    while (v >= m) v = ps_next(&p) >> (32 - k);
    return v;
}

/* ======================================================================
 * One env step.
 * ====================================================================== */
typedef struct {
    int has;               /* table non-empty */
    int nonfinite;         /* a NaN or inf in the table: normalisation skipped */
    double mn, mx;
} hstats;

static void h_stats(const ffo_tab* Ht, hstats* s) {
    s->has = Ht->n > 0 || Ht->xn > 0; s->nonfinite = Ht->xnf; s->mn = INFINITY; s->mx = -INFINITY;
    if (Ht->xn > 0) { s->mn = Ht->xmn; s->mx = Ht->xmx; }
    for (int64_t i = 0; i < Ht->n; i++) {
        const double* v = Ht->vals + Ht->order[i] * Ht->width;
        for (int k = 0; k < Ht->width; k++) {
            if (!isfinite(v[k])) s->nonfinite = 1;
            if (v[k] < s->mn) s->mn = v[k];
            if (v[k] > s->mx) s->mx = v[k];
        }
    }
}

/* The values of the rows the table cannot hold (all_h_values' other entries,
 * model/ffm_trained_core.py:242-249): their count, min, max and whether one is NaN/inf. */
void ffo_tab_set_extra(ffo_tab* t, const double* vals, int64_t n) {
    t->xn = n; t->xnf = 0; t->xmn = INFINITY; t->xmx = -INFINITY;
    for (int64_t i = 0; i < n; i++) {
        if (!isfinite(vals[i])) t->xnf = 1;
        if (vals[i] < t->xmn) t->xmn = vals[i];
        if (vals[i] > t->xmx) t->xmx = vals[i];
    }
}

typedef struct {
    const ffo_learn_cfg* c;
    ffo_tab *V, *Ht;
    int jacobi, parallel;
    hstats hs;
    float smin, smax;      /* min/max of the inf->0 SFF (model/ffm_unified.py:74-76, 425-426) */
    lrng rng;
    double eps;            /* this env's epsilon (the global one, or the batched schedule's) */
} lctx;

typedef struct {
    int32_t sv, snv;       /* V slots of s and s' (-1: terminal) */
    int32_t hslot, k;      /* H slot, chosen action (-1: none) */
    int32_t valid;         /* action valid */
    double r;
} lrec;

static double np_max(const double* a, int n) {
    double m = a[0];
    for (int i = 1; i < n; i++) {
        if (a[i] != a[i]) return a[i];
        if (m != m) return m;
        m = a[i] > m ? a[i] : m;
    }
    return m;
}

static int choice_cdf(const double* p, int n, double u) {
    double cdf[9], acc = 0.0;
    for (int k = 0; k < n; k++) { acc += p[k]; cdf[k] = acc; }
    const double last = cdf[n - 1];
    for (int k = 0; k < n; k++)
        if (cdf[k] / last > u) return k;
    return n - 1;
}

/* H row of state s, inserting zeros (model/ffm_unified.py:405-410). */
static int64_t h_row(lctx* L, uint64_t s) {
    static const double zeros[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t before = L->Ht->n;
    int64_t slot = tab_get_sync(L->Ht, s, zeros, L->parallel);
    if (!L->jacobi && L->Ht->n > before) {      /* a zero row joins the min/max (:414-423) */
        L->hs.has = 1;
        if (0.0 < L->hs.mn) L->hs.mn = 0.0;
        if (0.0 > L->hs.mx) L->hs.mx = 0.0;
    }
    return slot;
}

/* Actor policy (model/ffm_unified.py:394-499, model/ffm_actor_only.py:241-340) over the
 * NA = |neighbours| + 1 moves (stay last; Moore: 9, add.reduce pairs 8+ terms).
 * compat = ffm_actor_only's masking (invalid -> -inf -> uniform). */
static int actor_choose(lctx* L, int64_t hslot, const int32_t* coord, const int* valid, const float* dff,
                        int compat, int NA) {
    const ffo_learn_cfg* c = L->c;
    double h[9], score[9], e[9], p[9];
    memcpy(h, L->Ht->vals + hslot * L->Ht->width, sizeof(double) * (size_t)NA);
    if (L->hs.has && !L->hs.nonfinite && L->hs.mx - L->hs.mn > 1e-6) {
        const double smin = (double)L->smin, smax = (double)L->smax;
        for (int k = 0; k < NA; k++) h[k] = ((L->hs.mx - h[k]) / (L->hs.mx - L->hs.mn)) * (smax - smin) + smin;
    }
    const float kD = (float)c->k_D;
    const double nkA = -c->k_A;
    for (int k = 0; k < NA; k++) {
        const float d = kD * dff[coord[k]];
        score[k] = nkA * h[k] + (double)d;
    }
    if (compat)
        for (int k = 0; k < NA; k++)
            if (!valid[k]) score[k] = -INFINITY;                    /* actor_only.py:291 */
    int bad = 0;
    for (int k = 0; k < NA; k++) if (!isfinite(score[k])) bad = 1;
    if (bad)
        for (int k = 0; k < NA; k++) score[k] = valid[k] ? 1.0 : 0.0;
    double mx;
    if (compat) {
        double vs[9]; int nv = 0;
        for (int k = 0; k < NA; k++) if (valid[k]) vs[nv++] = score[k];
        mx = nv ? np_max(vs, nv) : 0.0;
    } else {
        mx = np_max(score, NA);
    }
    for (int k = 0; k < NA; k++) e[k] = valid[k] ? ffo_det_exp(score[k] - mx) : 0.0;
    const double sum = ffo_np_sumd(e, NA);
    int nvalid = 0, vidx[9];
    for (int k = 0; k < NA; k++) if (valid[k]) vidx[nvalid++] = k;
    if (isfinite(sum) && sum > 0) {
        for (int k = 0; k < NA; k++) p[k] = e[k] / sum;
    } else {
        for (int k = 0; k < NA; k++) p[k] = valid[k] ? 1.0 / (double)nvalid : 0.0;
    }
    if (L->eps > 0 && dec_coin(&L->rng) < L->eps) {                  /* :478-495 */
        if (nvalid > 0) return vidx[dec_randint(&L->rng, (uint32_t)nvalid)];
        return NA - 1;
    }
    return choice_cdf(p, NA, dec_u53(&L->rng));
}

/* Critic-only policy of ffm_unified (:353-392): raw SFF over all NA moves. */
static int critic_choose(lctx* L, const int32_t* coord, const int* valid, const float* dff, int NA) {
    const ffo_learn_cfg* c = L->c;
    double p[9];
    int nvalid = 0;
    for (int k = 0; k < NA; k++) nvalid += valid[k];
    if (c->sff32) {
        const float kS = (float)(-c->k_S), kD = (float)c->k_D;
        float s[9], e[9];
        for (int k = 0; k < NA; k++) {
            const float a = kS * c->sff32[coord[k]];
            const float b = kD * dff[coord[k]];
            s[k] = a + b;
        }
        float mx = s[0];
        for (int k = 1; k < NA; k++) {
            if (s[k] != s[k]) { mx = s[k]; break; }
            mx = s[k] > mx ? s[k] : mx;
        }
        for (int k = 0; k < NA; k++) e[k] = valid[k] ? ffo_np_expf(s[k] - mx) : 0.0f;
        const float sum = ffo_np_sumf(e, NA);
        if (isfinite(sum) && sum > 0) {
            for (int k = 0; k < NA; k++) p[k] = (double)(e[k] / sum);
        } else {
            const float u = (float)(1.0 / (double)nvalid);
            for (int k = 0; k < NA; k++) p[k] = valid[k] ? (double)u : 0.0;
        }
    } else {
        const double kS = -c->k_S;
        const float kD = (float)c->k_D;
        double s[9], e[9];
        for (int k = 0; k < NA; k++) {
            const float b = kD * dff[coord[k]];
            s[k] = kS * c->sff64[coord[k]] + (double)b;
        }
        const double mx = np_max(s, NA);
        for (int k = 0; k < NA; k++) e[k] = valid[k] ? ffo_det_exp(s[k] - mx) : 0.0;
        const double sum = ffo_np_sumd(e, NA);
        if (isfinite(sum) && sum > 0) {
            for (int k = 0; k < NA; k++) p[k] = e[k] / sum;
        } else {
            for (int k = 0; k < NA; k++) p[k] = valid[k] ? 1.0 / (double)nvalid : 0.0;
        }
    }
    return choice_cdf(p, NA, dec_u53(&L->rng));
}

/* ffm_trained_core policy (model/ffm_trained_core.py:219-300): H row (float32;
 * zeros when the state is missing, :231-239), min/max normalisation of the whole
 * table in float32 (NEP 50: Python floats are weak next to the f32 array,
 * :242-267), score -k_A*h + k_D*dff in float32, NumPy's float32 exp, the masked
 * sum and divide, uniform fallbacks (:270-296), then np.random.choice. */
static int trained_choose(lctx* L, int64_t hslot, const int32_t* coord, const int* valid, const float* dff,
                          int NA) {
    const ffo_learn_cfg* c = L->c;
    float h[9], score[9], e[9];
    double p[9];
    /* NA = 5 (Neumann) or 9 (Moore, :76-85): the H row has one value per move (:228-236) */
    for (int k = 0; k < NA; k++) h[k] = hslot >= 0 ? (float)L->Ht->vals[hslot * NA + k] : 0.0f;
    if (L->hs.has && !L->hs.nonfinite && L->hs.mx - L->hs.mn > 1e-6) {
        const float hmax = (float)L->hs.mx, den = (float)(L->hs.mx - L->hs.mn);
        const float srange = (float)((double)L->smax - (double)L->smin), smin = L->smin;
        for (int k = 0; k < NA; k++) {
            const float a = hmax - h[k];
            const float b = a / den;
            const float d = b * srange;
            h[k] = d + smin;
        }
    }
    const float nkA = (float)(-c->k_A), kD = (float)c->k_D;
    int bad = 0, nvalid = 0;
    for (int k = 0; k < NA; k++) {
        const float a = nkA * h[k];
        const float b = kD * dff[coord[k]];
        score[k] = a + b;
        if (!isfinite(score[k])) bad = 1;
        nvalid += valid[k];
    }
    if (bad)
        for (int k = 0; k < NA; k++) score[k] = valid[k] ? 1.0f : 0.0f;
    float mx = score[0];
    for (int k = 1; k < NA; k++) mx = score[k] > mx ? score[k] : mx;
    for (int k = 0; k < NA; k++) e[k] = valid[k] ? ffo_np_expf(score[k] - mx) : 0.0f;
    const float sum = ffo_np_sumf(e, NA);                 /* pairwise from 8 terms on */
    if (isfinite(sum) && sum > 0) {
        for (int k = 0; k < NA; k++) p[k] = (double)(e[k] / sum);
    } else {
        const float u = (float)(1.0 / (double)nvalid);
        for (int k = 0; k < NA; k++) p[k] = valid[k] ? (double)u : 0.0;
    }
    return choice_cdf(p, NA, dec_u53(&L->rng));
}

/* ffm_ac_core decide = ffm_core decide (model/ffm_ac_core.py:126-199):
 * free neighbours + stay, exit forcing, SFF/DFF softmax.  -1: no request. */
static int32_t ac_decide(lctx* L, int x, int y, const int32_t* occ, const float* dff, int* will_exit) {
    const ffo_learn_cfg* c = L->c;
    const int W = c->W;
    const int nb = cfg_nb(c);
    int32_t cand[9];
    int nc = 0;
    for (int k = 0; k < nb; k++) {
        const int32_t cell = (x + nbx(nb, k)) * W + (y + nby(nb, k));
        const uint8_t m = c->map[cell];
        if (!(m == 0 || m == 3)) continue;
        if (occ[cell] >= 0) continue;
        cand[nc++] = cell;
    }
    if (nc == 0) return -1;
    cand[nc++] = x * W + y;
    for (int k = 0; k < nc; k++)
        if (c->map[cand[k]] == 3) { *will_exit = 1; return cand[k]; }   /* :166-172 */
    double p[9];
    if (c->sff32) {
        const float kS = (float)(-c->k_S), kD = (float)c->k_D;
        float s[9], e[9];
        for (int k = 0; k < nc; k++) {
            const float a = kS * c->sff32[cand[k]];
            const float b = kD * dff[cand[k]];
            s[k] = a + b;
        }
        float mx = s[0];
        for (int k = 1; k < nc; k++) mx = s[k] > mx ? s[k] : mx;
        for (int k = 0; k < nc; k++) e[k] = ffo_np_expf(s[k] - mx);
        const float sum = ffo_np_sumf(e, nc);
        if (!(isfinite(sum) && sum != 0.0f)) return -1;                  /* :187 */
        for (int k = 0; k < nc; k++) p[k] = (double)(e[k] / sum);
    } else {
        const double kS = -c->k_S;
        const float kD = (float)c->k_D;
        double s[9], e[9];
        for (int k = 0; k < nc; k++) {
            const float b = kD * dff[cand[k]];
            s[k] = kS * c->sff64[cand[k]] + (double)b;
        }
        double mx = s[0];
        for (int k = 1; k < nc; k++) mx = s[k] > mx ? s[k] : mx;
        for (int k = 0; k < nc; k++) e[k] = ffo_det_exp(s[k] - mx);
        const double sum = ffo_np_sumd(e, nc);
        if (!(isfinite(sum) && sum != 0.0)) return -1;
        for (int k = 0; k < nc; k++) p[k] = e[k] / sum;
    }
    return cand[choice_cdf(p, nc, dec_u53(&L->rng))];
}

static void update_dff4(const ffo_learn_cfg* c, float* dff, float* B) {
    /* model/ffm_unified.py:779-798 (same as ffm_core.update_dff, neumann) */
    const int H = c->H, W = c->W, HW = H * W;
    const float c0 = (float)((1.0 - c->decay) * (1.0 - c->diffuse));
    const int nb = cfg_nb(c);
    const float c1 = (float)(c->decay * (1.0 - c->diffuse) / (double)nb);
    for (int i = 0; i < HW; i++) B[i] = c0 * dff[i];
    for (int x = 0; x < H; x++)
        for (int y = 0; y < W; y++) {
            float a = B[x * W + y];
            for (int k = 0; k < nb; k++) {
                const int nx = x + nbx(nb, k), ny = y + nby(nb, k);
                const float v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? B[nx * W + ny] : 0.0f;
                const float t = c1 * v;
                a = a + t;
            }
            dff[x * W + y] = (a < 1e-4f) ? 0.0f : a;
        }
}

static int64_t fx(double v) {
    double q = rint(v * FX_ONE);
    if (q > 4.0e18) q = 4.0e18;
    if (q < -4.0e18) q = -4.0e18;
    return (int64_t)q;
}

/* One step of one env.  Scratch: occ [HW] (-1), sm/smn [HW] u8, B [HW] f32.
 * rec (may be NULL in MT mode) receives the per-agent learning records. */
static int env_step(lctx* L, int32_t* pos, int32_t* n_io, float* dff, int32_t* occ, uint8_t* sm,
                    uint8_t* smn, float* B, lrec* rec) {
    const ffo_learn_cfg* c = L->c;
    const int H = c->H, W = c->W, HW = H * W;
    const int n = *n_io;
    const int nb = cfg_nb(c), NA = nb + 1;      /* moves: the neighbours in order, then stay */
    /* ffm_actor_only's inner-loop quirk: one decision per neighbour (4, Moore 8) */
    const int D = c->variant == FFO_VAR_ACTOR_ONLY ? nb : 1;
    const int hw = L->Ht ? L->Ht->width : 5;
    const int actor = c->variant == FFO_VAR_ACTOR_ONLY ||
                      (c->variant == FFO_VAR_UNIFIED && c->mode != FFO_MODE_CRITIC);
    int32_t* rq_tgt = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n * D + 1));
    int32_t* rq_agent = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n * D + 1));
    int32_t* nxt = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    int32_t* coll = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    int32_t* act = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    int32_t* avalid = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    int32_t* wexit = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n + 1));
    uint64_t* skey = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n + 1));
    double* td = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    int nrq = 0, rc = 0;

    memcpy(sm, c->map, (size_t)HW);
    for (int i = 0; i < n; i++) { sm[pos[i]] = 1; occ[pos[i]] = i; }   /* :284-286 */

    /* ---- decide ---- */
    for (int i = 0; i < n; i++) {
        const int x = pos[i] / W, y = pos[i] % W;
        skey[i] = encode(c, sm, x, y);
        nxt[i] = pos[i];
        coll[i] = -1; act[i] = -1; avalid[i] = 0; wexit[i] = 0;
        if (c->variant == FFO_VAR_AC) {
            dec_begin(&L->rng, (uint32_t)i);
            int32_t T = ac_decide(L, x, y, occ, dff, &wexit[i]);
            if (T >= 0) { rq_tgt[nrq] = T; rq_agent[nrq++] = i; }
            continue;
        }
        int32_t coord[9];
        int valid[9], inb[9];
        for (int k = 0; k < NA; k++) {
            const int nx = k < nb ? x + nbx(nb, k) : x, ny = k < nb ? y + nby(nb, k) : y;
            inb[k] = nx >= 0 && nx < H && ny >= 0 && ny < W;
            coord[k] = inb[k] ? nx * W + ny : pos[i];
            const uint8_t m = inb[k] ? c->map[coord[k]] : 2;
            valid[k] = inb[k] && (m == 0 || m == 3) && (k == nb || occ[coord[k]] < 0);
        }
        valid[nb] = 1;
        if (c->variant == FFO_VAR_TRAINED) {            /* model/ffm_trained_core.py:169-258 */
            dec_begin(&L->rng, (uint32_t)i);
            int ex = -1;
            for (int k = 0; k < nb; k++)
                if (inb[k] && c->map[coord[k]] == 3) { ex = k; break; }
            int k = ex;
            if (ex < 0) k = trained_choose(L, tab_find(L->Ht, skey[i]), coord, valid, dff, NA);
            else wexit[i] = 1;
            rq_tgt[nrq] = coord[k]; rq_agent[nrq++] = i;
            continue;
        }
        if (c->variant == FFO_VAR_UNIFIED) {
            dec_begin(&L->rng, (uint32_t)i);
            int ex = -1;
            for (int k = 0; k < nb; k++)
                if (inb[k] && c->map[coord[k]] == 3) { ex = k; break; }   /* :326-334 */
            int k;
            if (ex >= 0) {
                wexit[i] = 1;
                k = ex;
            } else if (!actor) {
                k = critic_choose(L, coord, valid, dff, NA);
            } else {
                const int64_t hs = h_row(L, skey[i]);
                if (hs < 0) { rc = -1; goto out; }
                k = actor_choose(L, hs, coord, valid, dff, 0, NA);
            }
            rq_tgt[nrq] = coord[k]; rq_agent[nrq++] = i;
            act[i] = k; avalid[i] = valid[k];
        } else {
            /* ffm_actor_only: the exit test and the decision sit inside the
             * neighbour loop (model/ffm_actor_only.py:214-355): up to four
             * decisions and requests per agent, the last one recorded. */
            int ex = -1;
            for (int j = 0; j < nb; j++) {
                if (ex < 0 && inb[j] && c->map[coord[j]] == 3) ex = j;
                int k;
                if (ex >= 0) {
                    wexit[i] = 1;
                    k = ex;
                } else {
                    dec_begin(&L->rng, (uint32_t)(i * D + j));
                    const int64_t hs = h_row(L, skey[i]);
                    if (hs < 0) { rc = -1; goto out; }
                    k = actor_choose(L, hs, coord, valid, dff, 1, NA);
                }
                rq_tgt[nrq] = coord[k]; rq_agent[nrq++] = i;
                act[i] = k; avalid[i] = valid[k];
            }
        }
    }

    /* ---- resolve: targets in first-request order; always a winner ---- */
    {
        char* done = (char*)calloc((size_t)(nrq + 1), 1);
        int32_t* list = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nrq + 1));
        for (int q = 0; q < nrq; q++) {
            if (done[q]) continue;
            const int32_t T = rq_tgt[q];
            int m = 0;
            for (int q2 = q; q2 < nrq; q2++)
                if (rq_tgt[q2] == T) { list[m++] = rq_agent[q2]; done[q2] = 1; }
            /* owner seq for the Philox stream: agent*4 + decision index for
             * ffm_actor_only (every agent makes exactly four requests, so that
             * is q itself), the agent index otherwise */
            const uint32_t owner_seq = (uint32_t)(c->variant == FFO_VAR_ACTOR_ONLY ? q : rq_agent[q]);
            int w;
            if (m == 1) {
                w = list[0];
                coll[w] = 0;
            } else {
                w = list[conflict_pick(&L->rng, owner_seq, (uint32_t)m)];
                for (int z = 0; z < m; z++) coll[list[z]] = m - 1;
            }
            nxt[w] = T;
            dff[pos[w]] += 1.0f;
        }
        free(done);
        free(list);
    }

    /* ---- learning (none for the trained actor) ---- */
    if (c->variant == FFO_VAR_TRAINED) goto exits;
    memcpy(smn, c->map, (size_t)HW);
    for (int i = 0; i < n; i++)
        if (c->map[nxt[i]] != 3) smn[nxt[i]] = 1;                    /* :543-546 */
    {
        const double vdef[1] = {c->v_default};
        for (int i = 0; i < n; i++) {
            double r = c->step_penalty;
            if (wexit[i]) r = r + c->exit_reward;
            if (coll[i] >= 0) r = r + (double)coll[i] * c->collision_penalty;
            int64_t sn = -1;
            double vn = 0.0;
            if (!wexit[i]) {
                const uint64_t k2 = encode(c, smn, nxt[i] / W, nxt[i] % W);
                sn = tab_get_sync(L->V, k2, vdef, L->parallel);
                if (sn < 0) { rc = -1; goto out; }
                vn = L->V->vals[sn];
            }
            const int64_t sv = tab_get_sync(L->V, skey[i], vdef, L->parallel);
            if (sv < 0) { rc = -1; goto out; }
            const double v = L->V->vals[sv];
            const double t = (r + c->gamma * vn) - v;
            td[i] = t;
            if (!L->jacobi) {
                L->V->vals[sv] = v + c->alpha_v * t;                   /* :665 */
            } else {
                __atomic_fetch_add(&L->V->acc[2 * sv], fx(t), __ATOMIC_RELAXED);
                __atomic_fetch_add(&L->V->acc[2 * sv + 1], (int64_t)1, __ATOMIC_RELAXED);
            }
            if (rec) { rec[i].sv = (int32_t)sv; rec[i].snv = (int32_t)sn; rec[i].r = r; }
        }
        const int post_update = c->variant == FFO_VAR_UNIFIED && c->mode == FFO_MODE_ACTOR;
        if (post_update && !L->jacobi) {
            /* _get_td_errors with the updated V (model/ffm_unified.py:568-574) */
            for (int i = 0; i < n; i++) {
                double r = c->step_penalty;
                if (wexit[i]) r = r + c->exit_reward;
                if (coll[i] >= 0) r = r + (double)coll[i] * c->collision_penalty;
                double vn = 0.0;
                if (!wexit[i]) {
                    const uint64_t k2 = encode(c, smn, nxt[i] / W, nxt[i] % W);
                    vn = L->V->vals[tab_get(L->V, k2, vdef)];
                }
                const double v = L->V->vals[tab_get(L->V, skey[i], vdef)];
                td[i] = (r + c->gamma * vn) - v;
            }
        }
        if (actor) {
            static const double zeros[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int i = 0; i < n; i++) {
                if (act[i] < 0) continue;
                const int64_t hs = tab_get_sync(L->Ht, skey[i], zeros, L->parallel);   /* :769-773 */
                if (hs < 0) { rc = -1; goto out; }
                if (rec) { rec[i].hslot = (int32_t)hs; rec[i].k = act[i]; rec[i].valid = avalid[i]; }
                if (!avalid[i]) continue;
                if (!L->jacobi) {
                    L->Ht->vals[hs * hw + act[i]] = L->Ht->vals[hs * hw + act[i]] + c->alpha_h * td[i];
                } else if (!post_update) {
                    __atomic_fetch_add(&L->Ht->acc[hs * hw + act[i]], fx(c->alpha_h * td[i]), __ATOMIC_RELAXED);
                }
            }
        }
    }

    /* ---- exit removal, DFF ---- */
exits:
    for (int i = 0; i < n; i++) occ[pos[i]] = -1;
    {
        int nn = 0;
        for (int i = 0; i < n; i++)
            if (c->map[nxt[i]] != 3) pos[nn++] = nxt[i];
        *n_io = nn;
    }
    update_dff4(c, dff, B);
out:
    free(rq_tgt); free(rq_agent); free(nxt); free(coll); free(act); free(avalid); free(wexit);
    free(skey); free(td);
    return rc;
}

static void sff_minmax(const ffo_learn_cfg* c, float* mn, float* mx) {
    /* np.where(isinf(sff), 0, sff).astype(float32); min / max (model/ffm_unified.py:74-76) */
    float a = INFINITY, b = -INFINITY;
    for (int i = 0; i < c->H * c->W; i++) {
        float v = c->sff32 ? c->sff32[i] : (float)c->sff64[i];
        if (c->sff32 ? isinf(c->sff32[i]) : isinf(c->sff64[i])) v = 0.0f;
        if (v < a) a = v;
        if (v > b) b = v;
    }
    *mn = a; *mx = b;
}

int ffo_learn_step_mt(const ffo_learn_cfg* c, ffo_tab* V, ffo_tab* Ht, int32_t* pos, int32_t* n,
                      float* dff, ffo_mt* np_rng, ffo_mt* py_rng) {
    const int HW = c->H * c->W;
    lctx L;
    memset(&L, 0, sizeof L);
    L.c = c; L.V = V; L.Ht = Ht; L.jacobi = 0; L.parallel = 0;
    L.eps = c->epsilon;
    if (Ht) h_stats(Ht, &L.hs);
    sff_minmax(c, &L.smin, &L.smax);
    L.rng.philox = 0; L.rng.np = np_rng; L.rng.py = py_rng;
    int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * (size_t)HW);
    for (int i = 0; i < HW; i++) occ[i] = -1;
    uint8_t* sm = (uint8_t*)malloc((size_t)HW * 2);
    float* B = (float*)malloc(sizeof(float) * (size_t)HW);
    int rc = env_step(&L, pos, n, dff, occ, sm, sm + HW, B, NULL);
    free(occ); free(sm); free(B);
    return rc;
}

/* ---- the batched step in phases ------------------------------------------------ */
struct ffo_lbatch {
    const ffo_learn_cfg* c;
    ffo_tab *V, *Ht;
    int64_t E;
    int32_t A_cap;
    lrec* recs;
    int32_t* nstart;
    uint16_t* place;       /* placement candidates (NULL: every free cell) */
    int32_t nplace;
};

void ffo_lbatch_set_placement(ffo_lbatch* b, const uint16_t* cells, int32_t count) {
    free(b->place);
    b->place = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(count > 0 ? count : 1));
    memcpy(b->place, cells, sizeof(uint16_t) * (size_t)count);
    b->nplace = count;
}

static double eps_of(const ffo_learn_cfg* c, int32_t k, int64_t genv) {
    if (!(c->eps_span > 0)) return c->epsilon;
    const double ph = c->eps_phase > 0 ? (double)((genv % c->eps_phase) * (c->eps_stride > 0 ? c->eps_stride : 1)) : 0.0;
    double e = c->eps_start + (c->eps_end - c->eps_start) * (((double)k + c->eps_offset + ph) / c->eps_span);
    return e < 0.0 ? 0.0 : e > 1.0 ? 1.0 : e;
}

ffo_lbatch* ffo_lbatch_new(const ffo_learn_cfg* c, ffo_tab* V, ffo_tab* Ht, int64_t E, int32_t A_cap) {
    ffo_lbatch* b = (ffo_lbatch*)calloc(1, sizeof(ffo_lbatch));
    b->c = c; b->V = V; b->Ht = Ht; b->E = E; b->A_cap = A_cap;
    V->alpha = c->alpha_v;   /* the visit-averaged V update of the batched step */
    b->recs = (lrec*)calloc((size_t)(E * A_cap), sizeof(lrec));
    b->nstart = (int32_t*)calloc((size_t)E, sizeof(int32_t));
    return b;
}

void ffo_lbatch_free(ffo_lbatch* b) {
    if (!b) return;
    free(b->recs); free(b->nstart); free(b->place); free(b);
}

/* Every env's step against the tables as they are; increments left pending. */
int ffo_lbatch_local(ffo_lbatch* b, uint16_t* pos, int32_t* counts, float* dff, const int32_t* episodes,
                     uint64_t seed, uint32_t t, int64_t env_base, uint64_t* agent_steps, int nthreads) {
    const ffo_learn_cfg* c = b->c;
    const int HW = c->H * c->W;
    const int64_t E = b->E;
    const int32_t A_cap = b->A_cap;
    const int actor = c->variant == FFO_VAR_ACTOR_ONLY ||
                      (c->variant == FFO_VAR_UNIFIED && c->mode != FFO_MODE_CRITIC);
    hstats hs;
    memset(&hs, 0, sizeof hs);
    if (actor || c->variant == FFO_VAR_TRAINED) h_stats(b->Ht, &hs);
    float smin, smax;
    sff_minmax(c, &smin, &smax);
    memset(b->recs, 0, sizeof(lrec) * (size_t)(E * A_cap));
    uint64_t total = 0;
    int err = 0;
    const int nt = nthreads > 0 ? nthreads : 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nt) reduction(+ : total)
#endif
    {
        int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * (size_t)HW);
        for (int i = 0; i < HW; i++) occ[i] = -1;
        uint8_t* sm = (uint8_t*)malloc((size_t)HW * 2);
        float* B = (float*)malloc(sizeof(float) * (size_t)HW);
        int32_t* p32 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(A_cap + 1));
        lctx L;
        memset(&L, 0, sizeof L);
        L.c = c; L.V = b->V; L.Ht = b->Ht; L.jacobi = 1; L.parallel = nt > 1;
        L.hs = hs; L.smin = smin; L.smax = smax;
        L.rng.philox = 1; L.rng.seed = seed; L.rng.t = t;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t e = 0; e < E; e++) {
            uint16_t* pe = pos + e * (int64_t)A_cap;
            int32_t n = counts[e];
            b->nstart[e] = n;
            total += (uint64_t)n;
            for (int i = 0; i < n; i++) p32[i] = pe[i];
            L.rng.genv = (uint64_t)(env_base + e);
            L.eps = eps_of(c, episodes ? episodes[e] : 0, env_base + e);
            if (env_step(&L, p32, &n, dff + e * (int64_t)HW, occ, sm, sm + HW, B, b->recs + e * (int64_t)A_cap))
                err = 1;
            for (int i = 0; i < n; i++) pe[i] = (uint16_t)p32[i];
            counts[e] = n;
        }
        free(occ); free(sm); free(B); free(p32);
    }
    if (agent_steps) *agent_steps = total;
    return err ? -1 : 0;
}

/* which 0: apply V, then (ffm_unified actor_only) the actor's increments from the
 * TD errors of the updated V (model/ffm_unified.py:559-598); which 1: apply H. */
/* ffm_unified actor_only: the actor increments from the TD errors of the (applied) V. */
void ffo_lbatch_post(ffo_lbatch* b) {
    const ffo_learn_cfg* c = b->c;
    if (!(c->variant == FFO_VAR_UNIFIED && c->mode == FFO_MODE_ACTOR)) return;
    for (int64_t e = 0; e < b->E; e++)
        for (int i = 0; i < b->nstart[e]; i++) {
            const lrec* q = b->recs + e * (int64_t)b->A_cap + i;
            if (!q->valid) continue;
            const double vn = q->snv >= 0 ? b->V->vals[q->snv] : 0.0;
            const double td = (q->r + c->gamma * vn) - b->V->vals[q->sv];
            b->Ht->acc[(int64_t)q->hslot * b->Ht->width + q->k] += fx(c->alpha_h * td);
        }
}

/* The pending increments of V and H applied at once, no post-update pass (the post
 * increments of the pending steps were added at their steps): ffm_learner_flush_end. */
void ffo_lbatch_flush(ffo_lbatch* b) {
    const ffo_learn_cfg* c = b->c;
    ffo_tab_apply(b->V);
    if (c->variant == FFO_VAR_ACTOR_ONLY || (c->variant == FFO_VAR_UNIFIED && c->mode != FFO_MODE_CRITIC))
        ffo_tab_apply(b->Ht);
}

void ffo_lbatch_apply(ffo_lbatch* b, int which) {
    if (which == 1) { ffo_tab_apply(b->Ht); return; }
    ffo_tab_apply(b->V);
    ffo_lbatch_post(b);
}

/* Episode ends: emptied, or truncated at max_steps (run_*_training.py MAX_STEPS). */
int64_t ffo_lbatch_end(ffo_lbatch* b, uint16_t* pos, int32_t* counts, float* dff, int32_t* episodes,
                       int32_t* ep_steps, uint64_t seed, uint32_t t, int32_t auto_reset, int32_t N_reset,
                       int32_t max_steps, int64_t env_base, int32_t* log) {
    int64_t nlog = 0;
    const ffo_learn_cfg* c = b->c;
    const int HW = c->H * c->W;
    ffo_core_cfg cc;
    memset(&cc, 0, sizeof cc);
    cc.H = c->H; cc.W = c->W; cc.map = c->map; cc.nb = 4;
    for (int64_t e = 0; e < b->E; e++) {
        ep_steps[e]++;
        if (auto_reset && (counts[e] == 0 || (max_steps > 0 && ep_steps[e] >= max_steps))) {
            if (log) {
                int32_t* r = log + 4 * nlog;
                r[0] = (int32_t)(env_base + e);
                r[1] = episodes ? episodes[e] : 0;
                r[2] = ep_steps[e];
                r[3] = counts[e] == 0;
            }
            nlog++;
            if (b->place) ffo_reset_philox_list(b->place, b->nplace, N_reset, seed, t, env_base + e,
                                                pos + e * (int64_t)b->A_cap);
            else ffo_reset_philox(&cc, N_reset, seed, t, env_base + e, pos + e * (int64_t)b->A_cap);
            counts[e] = N_reset;
            memset(dff + e * (int64_t)HW, 0, sizeof(float) * (size_t)HW);
            ep_steps[e] = 0;
            if (episodes) episodes[e]++;
        }
    }
    return nlog;
}

int ffo_learn_step_philox_batch(const ffo_learn_cfg* c, ffo_tab* V, ffo_tab* Ht, int64_t E,
                                int32_t A_cap, uint16_t* pos, int32_t* counts, float* dff,
                                int32_t* episodes, int32_t* ep_steps, uint64_t seed, uint32_t t,
                                int32_t auto_reset, int32_t N_reset, int32_t max_steps,
                                int64_t env_base, uint64_t* agent_steps, int nthreads) {
    const int actor = c->variant == FFO_VAR_ACTOR_ONLY ||
                      (c->variant == FFO_VAR_UNIFIED && c->mode != FFO_MODE_CRITIC);
    ffo_lbatch* b = ffo_lbatch_new(c, V, Ht, E, A_cap);
    const int rc = ffo_lbatch_local(b, pos, counts, dff, episodes, seed, t, env_base, agent_steps, nthreads);
    ffo_lbatch_apply(b, 0);
    if (actor) ffo_lbatch_apply(b, 1);
    ffo_lbatch_end(b, pos, counts, dff, episodes, ep_steps, seed, t, auto_reset, N_reset, max_steps, env_base,
                   NULL);
    ffo_lbatch_free(b);
    return rc;
}
