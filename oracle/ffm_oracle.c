/*
 * ffm_oracle.c -- CPU restatement of SoraKurihara/FFM's ffm_core hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ffm_oracle.h).  Compiled with
 * -ffp-contract=off so every float operation rounds exactly like NumPy's
 * element-wise loops; the only fused operations are the explicit fmaf()
 * calls of NumPy's own float32 exp (numpy/_core/src/umath/loops_exponent_log).
 *
 * Citations are file:line in the reference repository (SoraKurihara/FFM).
 */
#include "ffm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================
 * MT19937.  NumPy's legacy RandomState (np.random.seed/choice/rand, used at
 * model/ffm_core.py:25,84,95) and CPython's `random` (random.choice at
 * model/ffm_core.py:96) are both MT19937 with the standard tempering; they
 * differ only in how an integer seed is expanded.
 * ====================================================================== */
void ffo_mt_seed_np(ffo_mt* s, uint32_t seed) {
    /* NumPy legacy seeding of an int: init_genrand(seed & 0xffffffff). */
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->pos = 624;
}

void ffo_mt_seed_py(ffo_mt* s, const uint32_t* key, int nkey) {
    /* CPython random.seed(int): init_by_array(|seed| split in 32-bit words). */
    ffo_mt_seed_np(s, 19650218u);
    int i = 1, j = 0;
    int k = 624 > nkey ? 624 : nkey;
    for (; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { s->mt[0] = s->mt[623]; i = 1; }
        if (j >= nkey) j = 0;
    }
    for (k = 623; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { s->mt[0] = s->mt[623]; i = 1; }
    }
    s->mt[0] = 0x80000000u;
    s->pos = 624;
}

static void mt_twist(ffo_mt* s) {
    const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MA = 0x9908b0dfu;
    int kk;
    uint32_t y;
    for (kk = 0; kk < 624 - 397; kk++) {
        y = (s->mt[kk] & UP) | (s->mt[kk + 1] & LO);
        s->mt[kk] = s->mt[kk + 397] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
    }
    for (; kk < 623; kk++) {
        y = (s->mt[kk] & UP) | (s->mt[kk + 1] & LO);
        s->mt[kk] = s->mt[kk - 227] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
    }
    y = (s->mt[623] & UP) | (s->mt[0] & LO);
    s->mt[623] = s->mt[396] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
    s->pos = 0;
}

uint32_t ffo_mt_next(ffo_mt* s) {
    if (s->pos >= 624) mt_twist(s);
    uint32_t y = s->mt[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static double u53_from_words(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

double ffo_mt_u53(ffo_mt* s) {
    uint32_t a = ffo_mt_next(s);
    uint32_t b = ffo_mt_next(s);
    return u53_from_words(a, b);
}

uint32_t ffo_np_interval(ffo_mt* s, uint32_t max) {
    /* NumPy random_interval(): masked rejection on 32-bit words. */
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (ffo_mt_next(s) & mask)) > max) {}
    return v;
}

void ffo_np_permutation(ffo_mt* s, int64_t n, int64_t* out) {
    /* Legacy RandomState.permutation(n) = shuffle(arange(n)):
     * for i = n-1 .. 1: j = interval(i); swap(out[i], out[j]). */
    for (int64_t i = 0; i < n; i++) out[i] = i;
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = (int64_t)ffo_np_interval(s, (uint32_t)i);
        int64_t t = out[i]; out[i] = out[j]; out[j] = t;
    }
}

static int bit_length(uint32_t n) {
    int k = 0;
    while (n) { k++; n >>= 1; }
    return k;
}

uint32_t ffo_py_randbelow(ffo_mt* s, uint32_t n) {
    /* CPython 3.10 Random._randbelow_with_getrandbits. */
    if (n == 0) return 0;
    int k = bit_length(n);
    uint32_t r = ffo_mt_next(s) >> (32 - k);
    while (r >= n) r = ffo_mt_next(s) >> (32 - k);
    return r;
}

/* ======================================================================
 * NumPy float arithmetic used at model/ffm_core.py:77-83.
 * ====================================================================== */
float ffo_np_expf(float x) {
    /* NumPy 2.x SIMD float32 exp (AVX2/AVX512F path): Cody-Waite reduction
     * by ln2 and a [5/2] rational approximation, then exact 2^q scaling.
     * Not correctly rounded; reproduces np.exp(float32) bit for bit
     * (tests/test_oracle.py checks this against NumPy). */
    if (isnan(x)) return x;
    if (x > 88.72283935546875f) return INFINITY;
    if (x < -103.97208404541015625f) return 0.0f;
    float q = rintf(x * 1.442695040888963407359924681001892137f);
    float r = fmaf(q, -6.93145752e-1f, x);
    r = fmaf(q, -1.42860677e-6f, r);
    float num = fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
    num = fmaf(num, r, 5.114512081637298353406e-02f);
    num = fmaf(num, r, 2.473615434895520810817e-01f);
    num = fmaf(num, r, 7.257664613233124478488e-01f);
    num = fmaf(num, r, 9.999999999980870924916e-01f);
    float den = fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
    den = fmaf(den, r, 1.0f);
    return ldexpf(num / den, (int)q);
}

void ffo_np_expf_array(const float* x, float* y, int64_t n, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t i = 0; i < n; i++) y[i] = ffo_np_expf(x[i]);
    (void)nthreads;
}

/* NumPy add.reduce of a short contiguous vector: pairwise_sum() with eight
 * accumulators once n >= 8, a plain left fold below that. */
float ffo_np_sumf(const float* a, int n) {
    if (n < 8) {
        float res = -0.0f;
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    }
    float r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
}

double ffo_np_sumd(const double* a, int n) {
    if (n < 8) {
        double res = -0.0;
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
}

/* ======================================================================
 * Philox4x32-10 (Salmon et al., SC'11).  Production RNG of this build:
 * counter = (t, env, index, purpose<<28 | sub), key = seed.
 * ====================================================================== */
void ffo_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

enum { PUR_DECIDE = 1, PUR_FRICTION = 2, PUR_RESET = 3 };

typedef struct {
    uint32_t ctr[4];
    uint32_t key[2];
    uint32_t buf[4];
    int used;
} pstream;

static void ps_init(pstream* p, uint64_t seed, uint32_t t, uint64_t genv, uint32_t idx, uint32_t purpose) {
    p->key[0] = (uint32_t)seed;
    p->key[1] = (uint32_t)(seed >> 32);
    p->ctr[0] = t;
    p->ctr[1] = (uint32_t)genv;
    p->ctr[2] = idx;
    p->ctr[3] = purpose << 28;
    p->used = 4;
}

static uint32_t ps_next(pstream* p) {
    if (p->used == 4) {
        ffo_philox(p->ctr, p->key, p->buf);
        p->ctr[3]++;
        p->used = 0;
    }
    return p->buf[p->used++];
}

static double ps_u53(pstream* p) {
    uint32_t a = ps_next(p);
    uint32_t b = ps_next(p);
    return u53_from_words(a, b);
}

/* ======================================================================
 * Draw dispatch: MT mode consumes the two global streams in the reference's
 * order; Philox mode keys every draw by (t, env, agent/owner, purpose).
 * ====================================================================== */
typedef struct {
    int philox;
    ffo_mt* np;
    ffo_mt* py;
    uint64_t seed;
    uint32_t t;
    uint64_t genv;
} rngctx;

static double draw_decide(rngctx* r, int agent) {
    if (!r->philox) return ffo_mt_u53(r->np);          /* np.random.choice, :84 */
    pstream p;
    ps_init(&p, r->seed, r->t, r->genv, (uint32_t)agent, PUR_DECIDE);
    return ps_u53(&p);
}

/* Friction for a contested target whose first requester is `owner`:
 * returns winner rank in [0,m) or -1 for "nobody moves" (:95-98). */
static int draw_friction(rngctx* r, int owner, uint32_t m) {
    if (!r->philox) {
        double u = ffo_mt_u53(r->np);                   /* np.random.rand(), :95 */
        if (u < 0.5) return (int)ffo_py_randbelow(r->py, m);  /* random.choice, :96 */
        return -1;
    }
    /* Philox mode: the owner's decide block B supplies the
     * coin (B.z < 2^31, probability exactly 1/2) and the winner rank by
     * Lemire's multiply-shift on B.w, exact through rejection; a rejected word
     * (probability < m/2^32) is replaced by the owner's friction stream. */
    uint32_t ctr[4] = {r->t, (uint32_t)r->genv, (uint32_t)owner, (uint32_t)PUR_DECIDE << 28};
    uint32_t key[2] = {(uint32_t)r->seed, (uint32_t)(r->seed >> 32)};
    uint32_t b[4];
    ffo_philox(ctr, key, b);
    if (b[2] >= 0x80000000u) return -1;
    if (m <= 1) return 0;
    const uint32_t thr = (uint32_t)(-m) % m;
    uint64_t prod = (uint64_t)b[3] * m;
    if ((uint32_t)prod < thr) {
        pstream p;
        ps_init(&p, r->seed, r->t, r->genv, (uint32_t)owner, PUR_FRICTION);
        do prod = (uint64_t)ps_next(&p) * m; while ((uint32_t)prod < thr);
    }
    return (int)(prod >> 32);
}

/* ======================================================================
 * ffm_core step.
 * ====================================================================== */
static const int NB4[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};          /* :29-30 */
static const int NB8[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1},
                              {0, 1},   {1, -1}, {1, 0},  {1, 1}};       /* :32-34 */

static const int (*nb_table(const ffo_core_cfg* c))[2] { return c->nb == 4 ? NB4 : NB8; }

/* Decide for agent at (x,y): model/ffm_core.py:41-88.
 * occ[cell] >= 0 = index of the agent currently there.
 * Returns target cell or -1 (no request). */
static int32_t decide_core(const ffo_core_cfg* c, int x, int y, const int32_t* occ,
                           const float* dff, rngctx* r, int agent) {
    const int W = c->W;
    const int (*nb)[2] = nb_table(c);
    int32_t cand[9];
    int nc = 0;
    for (int k = 0; k < c->nb; k++) {
        int nx = x + nb[k][0], ny = y + nb[k][1];
        int32_t cell = nx * W + ny;
        uint8_t m = c->map[cell];
        if (!(m == 0 || m == 3)) continue;              /* :52-54 */
        if (occ[cell] >= 0) continue;                   /* :57-60 (other agents) */
        cand[nc++] = cell;
    }
    if (nc == 0) return -1;                             /* :63 */
    cand[nc++] = x * W + y;                             /* :64, stay last */
    for (int k = 0; k < nc; k++)                        /* :66-72 exit forcing */
        if (c->map[cand[k]] == 3) return cand[k];

    double cdf[9];
    if (c->sff32) {
        const float kS = (float)(-c->k_S), kD = (float)c->k_D;
        float s[9], e[9];
        for (int k = 0; k < nc; k++) {
            float a = kS * c->sff32[cand[k]];
            float b = kD * dff[cand[k]];
            s[k] = a + b;                               /* :77 */
        }
        float mx = s[0];
        for (int k = 1; k < nc; k++) mx = s[k] > mx ? s[k] : mx;   /* :78 */
        for (int k = 0; k < nc; k++) e[k] = ffo_np_expf(s[k] - mx); /* :80 */
        float sum = ffo_np_sumf(e, nc);                 /* :81 */
        if (!(isfinite(sum) && sum != 0.0f)) return -1; /* :82 */
        double acc = 0.0;
        for (int k = 0; k < nc; k++) {                  /* :83 + choice's cumsum */
            float p = e[k] / sum;
            acc += (double)p;
            cdf[k] = acc;
        }
    } else {
        /* float64 SFF (the 50x50 data files): f64 score, f64 exp. */
        const double kS = -c->k_S;
        const float kD = (float)c->k_D;
        double s[9], e[9];
        for (int k = 0; k < nc; k++) {
            float b = kD * dff[cand[k]];
            s[k] = kS * c->sff64[cand[k]] + (double)b;
        }
        double mx = s[0];
        for (int k = 1; k < nc; k++) mx = s[k] > mx ? s[k] : mx;
        for (int k = 0; k < nc; k++) e[k] = exp(s[k] - mx);
        double sum = ffo_np_sumd(e, nc);
        if (!(isfinite(sum) && sum != 0.0)) return -1;
        double acc = 0.0;
        for (int k = 0; k < nc; k++) {
            acc += e[k] / sum;
            cdf[k] = acc;
        }
    }
    /* np.random.choice(n, p): cdf /= cdf[-1]; searchsorted(u, 'right'). */
    double last = cdf[nc - 1];
    double u = draw_decide(r, agent);
    for (int k = 0; k < nc; k++)
        if (cdf[k] / last > u) return cand[k];
    return cand[nc - 1];
}

static void update_dff_scratch(const ffo_core_cfg* c, float* dff, float* B) {
    /* model/ffm_core.py:106-117 */
    const int H = c->H, W = c->W, HW = H * W;
    const int (*nb)[2] = nb_table(c);
    const float c0 = (float)((1.0 - c->decay) * (1.0 - c->diffuse));
    const float c1 = (float)(c->decay * (1.0 - c->diffuse) / (double)c->nb);
    const float thr = 1e-4f;
    for (int i = 0; i < HW; i++) B[i] = c0 * dff[i];
    for (int x = 0; x < H; x++)
        for (int y = 0; y < W; y++) {
            float a = B[x * W + y];
            for (int k = 0; k < c->nb; k++) {
                int nx = x + nb[k][0], ny = y + nb[k][1];
                float v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? B[nx * W + ny] : 0.0f;
                float t = c1 * v;
                a = a + t;
            }
            dff[x * W + y] = (a < thr) ? 0.0f : a;
        }
}

void ffo_update_dff(const ffo_core_cfg* c, float* dff) {
    float* B = (float*)malloc(sizeof(float) * (size_t)(c->H * c->W));
    update_dff_scratch(c, dff, B);
    free(B);
}

/* One step of one env; pos in/out, n in/out, occ is scratch [H*W] filled -1,
 * work is scratch of 3*n int32 + H*W float. */
static void core_step(const ffo_core_cfg* c, int32_t* pos, int32_t* n, float* dff,
                      int32_t* occ, int32_t* work, rngctx* r) {
    const int W = c->W;
    const int np_ = *n;
    int32_t* req = work;
    int32_t* nxt = req + np_;
    int32_t* tgt_order = nxt + np_;     /* targets in first-request order */
    float* B = (float*)(tgt_order + np_);
    int ntg = 0;

    for (int i = 0; i < np_; i++) occ[pos[i]] = i;
    for (int i = 0; i < np_; i++) {                     /* :40-88 */
        int x = pos[i] / W, y = pos[i] % W;
        req[i] = decide_core(c, x, y, occ, dff, r, i);
        nxt[i] = pos[i];                                /* :38 */
        if (req[i] >= 0) {
            int seen = 0;
            for (int q = 0; q < i; q++)
                if (req[q] == req[i]) { seen = 1; break; }
            if (!seen) tgt_order[ntg++] = i;            /* dict insertion order */
        }
    }
    for (int g = 0; g < ntg; g++) {                     /* :90-98 */
        int owner = tgt_order[g];
        int32_t T = req[owner];
        int32_t reqs[9];
        uint32_t m = 0;
        for (int q = owner; q < np_; q++)
            if (req[q] == T) reqs[m++] = q;
        if (m == 1) {
            nxt[owner] = T;
            dff[pos[owner]] += 1.0f;                    /* :93 */
        } else {
            int k = draw_friction(r, owner, m);
            if (k >= 0) {
                int w = reqs[k];
                nxt[w] = T;
                dff[pos[w]] += 1.0f;                    /* :98 */
            }
        }
    }
    for (int i = 0; i < np_; i++) occ[pos[i]] = -1;     /* scratch back to empty */
    int nn = 0;                                         /* :101-102 */
    for (int i = 0; i < np_; i++)
        if (c->map[nxt[i]] != 3) pos[nn++] = nxt[i];
    *n = nn;
    update_dff_scratch(c, dff, B);                      /* :104 */
}

int ffo_core_step_mt(const ffo_core_cfg* c, int32_t* pos, int32_t* n, float* dff,
                     ffo_mt* np_rng, ffo_mt* py_rng) {
    const int HW = c->H * c->W;
    int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * (size_t)HW);
    for (int i = 0; i < HW; i++) occ[i] = -1;
    int32_t* work = (int32_t*)malloc(sizeof(int32_t) * (size_t)(3 * (*n) + HW + 1));
    rngctx r = {0, np_rng, py_rng, 0, 0, 0};
    core_step(c, pos, n, dff, occ, work, &r);
    free(work);
    free(occ);
    return 0;
}

int ffo_init_agents_mt(const ffo_core_cfg* c, int32_t N, ffo_mt* np_rng, int32_t* pos_out) {
    const int HW = c->H * c->W;
    int32_t* fl = (int32_t*)malloc(sizeof(int32_t) * (size_t)HW);
    int F = 0;
    for (int i = 0; i < HW; i++)
        if (c->map[i] == 0) fl[F++] = i;                /* np.argwhere row-major */
    if (N > F || N < 0) { free(fl); return -1; }        /* ValueError in choice */
    int64_t* perm = (int64_t*)malloc(sizeof(int64_t) * (size_t)(F > 0 ? F : 1));
    ffo_np_permutation(np_rng, F, perm);
    for (int i = 0; i < N; i++) pos_out[i] = fl[perm[i]];
    free(perm);
    free(fl);
    return 0;
}

/* ======================================================================
 * Philox-mode batch (this build's production semantics).
 * ====================================================================== */
static int free_list(const ffo_core_cfg* c, uint16_t* fl) {
    int F = 0;
    for (int i = 0; i < c->H * c->W; i++)
        if (c->map[i] == 0) fl[F++] = (uint16_t)i;
    return F;
}

static int cmp_u64(const void* a, const void* b) {
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* Philox-mode placement (DESIGN.md "Placement"): free-list entry j gets the
 * key philox(t, env, j, RESET).x; the N entries with the smallest
 * (key, j) pairs, in that order, are the agents 0..N-1.  A uniformly random
 * ordered sample without replacement, like initialize_agents()
 * (model/ffm_core.py:23-26), but computable in parallel. */
static void reset_with_list(const uint16_t* fl, int F, int32_t N, uint64_t seed, uint32_t t,
                            int64_t genv, uint64_t* scratch, uint16_t* pos_out) {
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int j = 0; j < F; j++) {
        const uint32_t ctr[4] = {t, (uint32_t)genv, (uint32_t)j, (uint32_t)PUR_RESET << 28};
        uint32_t o[4];
        ffo_philox(ctr, key, o);
        scratch[j] = ((uint64_t)o[0] << 32) | (uint64_t)j;
    }
    qsort(scratch, (size_t)F, sizeof(uint64_t), cmp_u64);
    for (int s = 0; s < N; s++) pos_out[s] = fl[scratch[s] & 0xFFFFu];
}

void ffo_reset_philox_list(const uint16_t* fl, int32_t F, int32_t N, uint64_t seed, uint32_t t, int64_t genv,
                           uint16_t* pos_out) {
    uint64_t* scratch = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(F > 0 ? F : 1));
    reset_with_list(fl, F, N, seed, t, genv, scratch, pos_out);
    free(scratch);
}

void ffo_reset_philox(const ffo_core_cfg* c, int32_t N, uint64_t seed, uint32_t t,
                      int64_t genv, uint16_t* pos_out) {
    const int HW = c->H * c->W;
    uint16_t* fl = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)HW);
    uint64_t* scratch = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)HW);
    int F = free_list(c, fl);
    reset_with_list(fl, F, N, seed, t, genv, scratch, pos_out);
    free(scratch);
    free(fl);
}

void ffo_core_step_philox_batch(const ffo_core_cfg* c, int64_t E, int32_t A_cap,
                                uint16_t* pos, int32_t* counts, float* dff,
                                int32_t* episodes, uint64_t seed, uint32_t t,
                                int32_t auto_reset, int32_t N_reset, int64_t env_base,
                                uint64_t* agent_steps, int nthreads) {
    const int HW = c->H * c->W;
    uint16_t* fl = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)HW);
    const int F = free_list(c, fl);
    uint64_t total = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total)
#endif
    {
        int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * (size_t)HW);
        int32_t* p32 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(A_cap > 0 ? A_cap : 1));
        uint64_t* scratch = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)HW);
        int32_t* work = (int32_t*)malloc(sizeof(int32_t) * (size_t)(3 * (A_cap > N_reset ? A_cap : N_reset) + HW + 1));
        for (int i = 0; i < HW; i++) occ[i] = -1;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t e = 0; e < E; e++) {
            uint16_t* pe = pos + e * (int64_t)A_cap;
            float* de = dff + e * (int64_t)HW;
            int32_t n = counts[e];
            total += (uint64_t)n;
            for (int i = 0; i < n; i++) p32[i] = pe[i];
            rngctx r = {1, NULL, NULL, seed, t, (uint64_t)(env_base + e)};
            core_step(c, p32, &n, de, occ, work, &r);
            for (int i = 0; i < n; i++) pe[i] = (uint16_t)p32[i];
            /* Auto-reset at the END of the step that empties an env (DESIGN.md
             * "Episodes"): placement keyed by this step's t, DFF zeroed. */
            if (auto_reset && n == 0) {
                reset_with_list(fl, F, N_reset, seed, t, env_base + e, scratch, pe);
                n = N_reset;
                for (int i = 0; i < HW; i++) de[i] = 0.0f;
                if (episodes) episodes[e]++;
            }
            counts[e] = n;
        }
        free(occ);
        free(p32);
        free(scratch);
        free(work);
    }
    free(fl);
    if (agent_steps) *agent_steps = total;
}
