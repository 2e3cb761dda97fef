// learn_step.hip -- the learning variants of SoraKurihara/FFM on CDNA4:
//   model/ffm_ac_core.py       critic (TD(0)) over 13-cell state keys
//   model/ffm_unified.py       critic_only / actor_only / both over rank keys
//   model/ffm_actor_only.py    the config-4 actor (13-cell keys, inner-loop quirk)
//
// Two executions of the same step:
//  * learn_exact_kernel -- the reference's semantics bit for bit: the two
//    MT19937 streams, targets and table updates in the reference's order.  It
//    is inherently sequential (every agent's TD update can change the value the
//    next agent reads), so one lane runs it; it serves the drop-in classes
//    (one env) and the golden replays.
//  * learn_batch_kernel -- the production step: one workgroup per env, agents
//    on lanes, occupancy grid and requests in LDS, Philox draws keyed
//    (t, env, seq), the V / H tables in HBM as open-addressing hash tables
//    shared by all envs.  Every env reads the tables as they were at the start
//    of the step; TD and actor increments are summed in 2^-32 fixed point
//    (integer atomics: order-free, so the result is deterministic) and applied
//    once per step by learn_apply_kernel.
// All translation units are built with -ffp-contract=off.
#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "learn_kernels.h"

namespace ffm {
namespace {

constexpr unsigned long long kEmptyKey = ~0ull;
constexpr double kFxOne = 4294967296.0;
constexpr uint16_t kNone16 = 0xFFFF;

__device__ __forceinline__ unsigned long long& tkey(const LearnTable& T, size_t h) { return T.rec[h * T.stride]; }
__device__ __forceinline__ double* tval(const LearnTable& T, size_t h) {
    return reinterpret_cast<double*>(T.rec + h * T.stride + 1);
}

// A dense record's key and first value in one 16-B load (V: the whole record; H: the key
// and action 0).  The key is stored after the presence bit is set, so a non-empty key
// means the slot is present and its presence word need not be read; an empty key sends
// the caller to dense_ensure (which then finds the bit of a concurrent insert).
__device__ __forceinline__ ulonglong2 trec16(const LearnTable& T, size_t h, int i = 0) {
    return *reinterpret_cast<const ulonglong2*>(T.rec + h * T.stride + 2 * i);
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z ^= z >> 33; z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}

// Deterministic float64 exp (fdlibm e_exp.c reduction + rational correction),
// the same code as oracle/ffm_learn_oracle.c: GPU == CPU bit for bit.
__device__ double det_exp(double x) {
    if (x != x) return x;
    if (x > 709.782712893383973096) return __builtin_inf();
    if (x < -745.13321910194110842) return 0.0;
    const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    const double kd = __builtin_rint(x * invln2);
    const double hi = x - kd * ln2HI;
    const double lo = kd * ln2LO;
    const double r = hi - lo;
    const double t = r * r;
    const double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    return __builtin_ldexp(y, (int)kd);
}

__device__ __forceinline__ long long fx(double v) {
    double q = __builtin_rint(v * kFxOne);
    q = q > 4.0e18 ? 4.0e18 : q;
    q = q < -4.0e18 ? -4.0e18 : q;
    return (long long)q;
}

// V after k visits of one batched step with summed fixed-point td q: k sequential
// TD(0) updates towards the mean target, V + (1 - (1 - alpha)^k) * mean(td)
// (oracle/ffm_learn_oracle.c ffo_v_visits: the same operation sequence).
__device__ __forceinline__ double v_visits(double v, long long q, long long k, double alpha) {
    const double mean = (double)q * (1.0 / kFxOne) / (double)k;
    double p = 1.0, b = 1.0 - alpha;
    for (long long e = k; e; e >>= 1) {
        if (e & 1) p = p * b;
        b = b * b;
    }
    return v + (1.0 - p) * mean;
}

__device__ __forceinline__ void acc_add(long long* p, long long q) {
    atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)q);
}

// Accumulator word `i` of this workgroup's copy (LearnTable::reps).
__device__ __forceinline__ long long* acc_at(const LearnTable& T, size_t i) {
    return T.acc + (size_t)(blockIdx.x & (T.reps - 1u)) * T.rep_stride + i;
}

// Words i .. i + NW - 1 summed over the copies (apply / export passes; `clear` zeroes
// them).  Every copy's load is issued before any store, so the gather is one round
// trip, not one per copy.
constexpr uint32_t kMaxAccReps = 8;
template <int NW>
__device__ __forceinline__ void acc_take(const LearnTable& T, size_t i, long long (&q)[NW], bool clear) {
    long long v[kMaxAccReps][NW];
#pragma unroll
    for (uint32_t r = 0; r < kMaxAccReps; r++)
#pragma unroll
        for (int k = 0; k < NW; k++) v[r][k] = r < T.reps ? T.acc[(size_t)r * T.rep_stride + i + k] : 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        q[k] = 0;
#pragma unroll
        for (uint32_t r = 0; r < kMaxAccReps; r++) q[k] += v[r][k];
    }
    if (clear)
#pragma unroll
        for (uint32_t r = 0; r < kMaxAccReps; r++)
#pragma unroll
            for (int k = 0; k < NW; k++)
                if (r < T.reps && v[r][k] != 0) T.acc[(size_t)r * T.rep_stride + i + k] = 0;
}

// V increment of every lane in the wave: the td sum and the visit count of a slot
// share a line, and an atomic wave-instruction costs one memory-side request per
// distinct line, so lane pairs (l, l ^ 1) put a sum and its count into the same
// instruction: even lanes add their own sum and then the partner's count, odd lanes
// the partner's count and then their own sum (one request per visit, not two).
// Called by every lane of the wave (sv < 0: nothing to add).
__device__ __forceinline__ void v_pair_add(const LearnTable& V, int sv, long long q) {
    const bool odd = (__lane_id() & 1u) != 0u;
    const int psv = __shfl_xor(sv, 1);
    const int s1 = odd ? psv : sv, s2 = odd ? sv : psv;
    if (s1 >= 0) acc_add(acc_at(V, 2 * (size_t)s1 + (odd ? 1 : 0)), odd ? 1 : q);
    if (s2 >= 0) acc_add(acc_at(V, 2 * (size_t)s2 + (odd ? 0 : 1)), odd ? q : 1);
}

// ---- hash tables ------------------------------------------------------------
// Slot of `key`, inserting it when absent (a defaultdict read inserts,
// model/ffm_unified.py:658).  Empty slots already hold the default value, so
// an inserter never has to publish a value.  -1 only when the table is full.
// Dense slot of a rank key, rank-major: the records of one rank pattern lie in
// block order, so agents in neighbouring blocks with the same pattern share lines
// (C5: 2.33 -> 2.17 ms per step against block-major).
__device__ __forceinline__ uint32_t dense_slot(unsigned long long key, const LearnTable& T) {
    const uint32_t bx = (uint32_t)(key >> 26) & 0x7FFFFu, by = (uint32_t)(key >> 45) & 0x7FFFFu;
    return (uint32_t)(key & 0xFFu) * ((T.mask + 1) >> 8) + bx * T.dense_by + by;
}

// Next index of T.order for each calling lane: one atomic per wave on the shared
// counter (inserters of a whole step otherwise serialise on that one word).
__device__ __forceinline__ uint32_t wave_claim(uint32_t* ctr) {
    const unsigned long long m = __ballot(1);
    const int leader = __ffsll((unsigned long long)m) - 1;
    const int lane = (int)__lane_id();
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// Dense tables: the slot is the key and an absent slot already holds the default,
// so a caller may load the values together with the presence word (not after it)
// and insert afterwards.  Presence is one bit of a 2 MB-scale bitmap that stays in
// L2; the key is stored for export only.
__device__ __forceinline__ bool dense_ensure_new(const LearnTable& T, uint32_t h, unsigned long long key) {
    const uint32_t bit = 1u << (h & 31);
    uint32_t* w = T.present + (h >> 5);
    if (*w & bit) return false;                           // stale 0 only costs the atomic
    if (atomicOr(w, bit) & bit) return false;
    tkey(T, h) = key;
    T.order[wave_claim(T.n)] = h;
    return true;                                          // this lane inserted the slot
}
__device__ __forceinline__ void dense_ensure(const LearnTable& T, uint32_t h, unsigned long long key) {
    (void)dense_ensure_new(T, h, key);
}


__device__ int tab_get(const LearnTable& T, unsigned long long key, int* overflow) {
    if (T.dense_by) {
        const uint32_t h = dense_slot(key, T);
        dense_ensure(T, h, key);
        return (int)h;
    }
    uint32_t h = (uint32_t)mix64(key) & T.mask;
    for (uint32_t probe = 0; probe < kMaxProbe; probe++) {
        // A plain load may see a slot empty that another CU has just filled; the CAS
        // below then reports the key actually there.  Keys are never removed during
        // a step, so a non-empty value read is never stale.
        const unsigned long long k = tkey(T, h);
        if (k == key) return (int)h;
        if (k == kEmptyKey) {
            // A hashed table past 7/8 load refuses new keys (probe chains would grow
            // without bound); the host reports FFM_E_NOMEM.
            if (!T.dense_by && __hip_atomic_load(T.n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= T.limit) break;
            const unsigned long long old = atomicCAS(&tkey(T, h), kEmptyKey, key);
            if (old == kEmptyKey) {
                const uint32_t idx = wave_claim(T.n);
                T.order[idx] = h;
                return (int)h;
            }
            if (old == key) return (int)h;
        }
        h = (h + 1) & T.mask;
    }
    atomicOr(overflow, 1);
    return -1;
}

// Home-slot look of a hashed table, free of side effects: the key and the first W values
// of the key's home slot in one round trip (a record is one line).  True when the key sits
// there -- the common case -- and v then holds its values (values never change during a
// step; an empty slot already holds the default).  Otherwise the caller takes tab_get
// (probe, insert), so a lookup costs one dependent round trip instead of two (key, then
// values), and independent lookups issue together.
template <int W>
__device__ __forceinline__ bool tab_peek(const LearnTable& T, unsigned long long key, uint32_t& h, double (&v)[W]) {
    h = (uint32_t)mix64(key) & T.mask;
    const unsigned long long* r = T.rec + (size_t)h * T.stride;
    const unsigned long long k = r[0];
#pragma unroll
    for (int i = 0; i < W; i++) v[i] = __longlong_as_double((long long)r[1 + i]);
    return k == key;
}

// tab_peek, then tab_get when the key is not at its home slot: the slot (-1: table full)
// with the W values loaded.
template <int W>
__device__ __forceinline__ int tab_get_row(const LearnTable& T, unsigned long long key, int* overflow,
                                           double (&v)[W]) {
    uint32_t h;
    if (tab_peek<W>(T, key, h, v)) return (int)h;
    const int s = tab_get(T, key, overflow);
    if (s >= 0) {
        const double* p = tval(T, s);
#pragma unroll
        for (int i = 0; i < W; i++) v[i] = p[i];
    }
    return s;
}

// Slot of `key`, or -1 when absent (read-only tables: ffm_trained_core).
__device__ int tab_find(const LearnTable& T, unsigned long long key) {
    if (T.dense_by) {
        const uint32_t h = dense_slot(key, T);
        return (T.present[h >> 5] >> (h & 31)) & 1u ? (int)h : -1;
    }
    uint32_t h = (uint32_t)mix64(key) & T.mask;
    for (uint32_t probe = 0; probe < kMaxProbe; probe++) {
        const unsigned long long k = tkey(T, h);
        if (k == key) return (int)h;
        if (k == kEmptyKey) return -1;
        h = (h + 1) & T.mask;
    }
    return -1;
}

// ---- state maps and encoders ------------------------------------------------
struct SmArray {                 // exact kernel: explicit state map
    const uint8_t* sm;
    __device__ int operator()(int c) const { return sm[c]; }
};
__device__ __forceinline__ int map2_at(const uint32_t* m2, int c) {
    return (int)((m2[c >> 4] >> ((c & 15) << 1)) & 3u);
}
struct SmGrid {                  // batch kernel, current positions: agent grid in LDS
    const uint32_t* map2;
    const uint16_t* grid;
    __device__ int operator()(int c) const {
        const int g = grid[c], m = map2_at(map2, c);
        return g != kNone16 ? 1 : m;
    }
};
struct SmBits {                  // batch kernel, next positions (exit cells excluded)
    const uint32_t* map2;
    const uint32_t* bits;
    __device__ int operator()(int c) const {
        const uint32_t b = bits[c >> 5];
        const int m = map2_at(map2, c);
        return ((b >> (c & 31)) & 1u) ? 1 : m;
    }
};

// Batch kernel: the LDS grid carries the static map class of every cell (bits 14-15:
// 0 free, 1 / 2 blocked, 3 exit) beside the index of the agent standing there (bits
// 0-13, kGIdx = none; batched learners hold at most 16383 agents), so the state
// encoder, the move candidates and the exit tests read one LDS word per cell instead of
// an LDS word and the global 2-bit map.
constexpr uint16_t kGIdx = 0x3FFF;
struct SmGridC {                 // current positions
    const uint16_t* grid;
    __device__ int operator()(int c) const {
        const uint32_t g = grid[c];
        return (g & kGIdx) != kGIdx ? 1 : (int)(g >> 14);
    }
};
struct SmBitsC {                 // next positions (exit cells excluded)
    const uint16_t* grid;
    const uint32_t* bits;
    __device__ int operator()(int c) const {
        const uint32_t b = bits[c >> 5];
        const int m = (int)(grid[c] >> 14);
        return ((b >> (c & 31)) & 1u) ? 1 : m;
    }
};

// n / d for 0 <= n < 65536 through m = ceil(2^32 / d): (n * m) >> 32 (checked
// exhaustively for every 2 <= d <= 65536; m = 0 encodes d = 1).  One v_mul_hi_u32
// instead of a ~30-instruction integer divide.
__device__ __forceinline__ int fdiv(int n, uint32_t m) {
    return m ? (int)__umulhi((unsigned)n, m) : n;
}

__device__ __forceinline__ unsigned long long pack_key(unsigned long long cells, int bx, int by) {
    return cells | ((unsigned long long)bx << 26) | ((unsigned long long)by << 45);
}

__constant__ int kNBx[4] = {-1, 1, 0, 0};   // U, D, L, R (model/ffm_unified.py:174-175)
__constant__ int kNBy[4] = {0, 0, -1, 1};
// Moore order of ffm_ac_core.get_neighbors (model/ffm_ac_core.py:51-60): row-major.
__constant__ int kMBx[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
__constant__ int kMBy[8] = {-1, 0, 1, -1, 1, -1, 0, 1};

// NumPy's pairwise add.reduce (numpy/_core/src/umath/loops_utils.h.src): n < 8 a
// left fold from -0, else eight running partial sums, combined pairwise, then the tail.
template <class T>
__device__ __forceinline__ T np_sum_n(const T* a, int n) {
    if (n < 8) {
        T res = T(-0.0);
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    }
    T r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
}

// model/ffm_unified.py:188-269.  The rank of direction d from the neighbour n1,
// the two cells beside n1 (diagonals of the agent) and the cell two ahead n2:
// 0 blocked / person / off-map at n1, 1 a person on a diagonal, 2 blocked / person
// / off-map at n2, else 3.  All twelve cells are read first (no load waits on
// another), then ranked.
template <class SM>
__device__ unsigned long long enc_rank(const SM& sm, int H, int W, int x, int y, uint32_t mbs) {
    auto at = [&](int cx, int cy) {          // -1 off the map
        const bool in = cx >= 0 && cx < H && cy >= 0 && cy < W;
        const int v = sm(in ? cx * W + cy : 0);
        return in ? v : -1;
    };
    const int dUL = at(x - 1, y - 1), dUR = at(x - 1, y + 1), dDL = at(x + 1, y - 1), dDR = at(x + 1, y + 1);
    const int n1[4] = {at(x - 1, y), at(x + 1, y), at(x, y - 1), at(x, y + 1)};
    const int n2[4] = {at(x - 2, y), at(x + 2, y), at(x, y - 2), at(x, y + 2)};
    const int da[4] = {dUL, dDL, dUL, dUR}, db[4] = {dUR, dDR, dDL, dDR};
    unsigned long long cells = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        int rank;
        if (n1[d] < 0 || n1[d] == 2 || n1[d] == 1) rank = 0;
        else if (da[d] == 1 || db[d] == 1) rank = 1;
        else if (n2[d] < 0 || n2[d] == 2 || n2[d] == 1) rank = 2;
        else rank = 3;
        cells |= (unsigned long long)rank << (2 * d);
    }
    return pack_key(cells, fdiv(x, mbs), fdiv(y, mbs));
}

// model/ffm_ac_core.py:62-109 (oob 2) and model/ffm_actor_only.py:102-147 (oob 0)
template <class SM>
__device__ unsigned long long enc13(const SM& sm, int H, int W, int x, int y, uint32_t mbs, int oob) {
    unsigned long long cells = 0;
    int i = 0;
#pragma unroll
    for (int dx = -1; dx <= 1; dx++)
#pragma unroll
        for (int dy = -1; dy <= 1; dy++, i++) {
            const int nx = x + dx, ny = y + dy;
            const int v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? sm(nx * W + ny) : oob;
            cells |= (unsigned long long)(v & 3) << (2 * i);
        }
#pragma unroll
    for (int d = 0; d < 4; d++, i++) {
        const int nx = x + 2 * (d == 0 ? -1 : d == 1 ? 1 : 0), ny = y + 2 * (d == 2 ? -1 : d == 3 ? 1 : 0);
        const int v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? sm(nx * W + ny) : oob;
        cells |= (unsigned long long)(v & 3) << (2 * i);
    }
    return pack_key(cells, fdiv(x, mbs), fdiv(y, mbs));
}

template <class SM>
__device__ unsigned long long encode_v(const LearnArgs& a, int variant, const SM& sm, int x, int y) {
    if (variant == kVarUnified || variant == kVarTrained) return enc_rank(sm, a.H, a.W, x, y, a.mBS);
    if (variant == kVarAC) return enc13(sm, a.H, a.W, x, y, a.mBS, 2);
    return enc13(sm, a.H, a.W, x, y, a.mBS, 0);                // block 5 hard-coded, :143 (a.bs = 5)
}
template <class SM>
__device__ unsigned long long encode(const LearnArgs& a, const SM& sm, int x, int y) {
    return encode_v(a, a.variant, sm, x, y);
}

// enc13 from packed state rows (learn_batch_kernel's batch_rows: row x + 2 holds map row x,
// cell y at bits 2 (y + 2), two halo rows / columns of the out-of-map value): the 3 x 3
// block's rows shifted into place, then the four cells two steps away -- the key enc13
// builds cell by cell.
__device__ __forceinline__ unsigned long long enc13_rows(const uint32_t* rw, int x, int y, uint32_t mbs) {
    const uint32_t r0 = rw[x], r1 = rw[x + 1], r2 = rw[x + 2], r3 = rw[x + 3], r4 = rw[x + 4];
    const int s1 = 2 * (y + 1);
    const unsigned long long cells =
        (unsigned long long)((r1 >> s1) & 0x3Fu) | ((unsigned long long)((r2 >> s1) & 0x3Fu) << 6) |
        ((unsigned long long)((r3 >> s1) & 0x3Fu) << 12) | ((unsigned long long)((r0 >> (s1 + 2)) & 3u) << 18) |
        ((unsigned long long)((r4 >> (s1 + 2)) & 3u) << 20) | ((unsigned long long)((r2 >> (s1 - 2)) & 3u) << 22) |
        ((unsigned long long)((r2 >> (s1 + 6)) & 3u) << 24);
    return pack_key(cells, fdiv(x, mbs), fdiv(y, mbs));
}

// ---- random draws -----------------------------------------------------------
__device__ uint32_t mt_interval(uint32_t* mt, uint32_t max) {     // NumPy legacy randint(max + 1)
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (mt_next(mt) & mask)) > max) {}
    return v;
}

struct DrawMT {                  // the reference's global streams
    uint32_t* np;
    uint32_t* py;
    __device__ double coin() { return mt_u53(py); }            // random.random()
    __device__ double u() { return mt_u53(np); }               // np.random.choice(p)
    __device__ uint32_t randint(uint32_t n) { return mt_interval(np, n - 1); }
};

struct DrawPh {                  // one keyed Philox stream per decision
    PhiloxStream ps;
    __device__ DrawPh(const LearnArgs& a, uint32_t genv, uint32_t seq)
        : ps(a.key0, a.key1, a.t, genv, seq, kPurDecide) {}
    __device__ double coin() { return ps.next_u53(); }
    __device__ double u() { return ps.next_u53(); }
    __device__ uint32_t randint(uint32_t n) {
        const uint32_t max = n - 1;
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
        uint32_t v;
        while ((v = (ps.next() & mask)) > max) {}
        return v;
    }
};

__device__ __forceinline__ int choice_cdf(const double* p, int n, double u) {
    double cdf[9], acc = 0.0;   // n <= 9: eight Moore neighbours + stay (ffm_ac_core)
#pragma unroll
    for (int k = 0; k < 9; k++) {
        if (k < n) { acc += p[k]; cdf[k] = acc; }
    }
    const double last = cdf[n - 1];
    for (int k = 0; k < n; k++)
        if (cdf[k] / last > u) return k;
    return n - 1;
}

__device__ __forceinline__ double np_max5(const double* s, int n) {
    double m = s[0];
    for (int k = 1; k < n; k++) {
        if (s[k] != s[k]) return s[k];
        if (m != m) return m;
        m = s[k] > m ? s[k] : m;
    }
    return m;
}

struct HStat {
    int has, nonfinite;
    double mn, mx;
};

// Actor policy: model/ffm_unified.py:394-499 (compat = false) and
// model/ffm_actor_only.py:241-340 (compat = true: invalid -> -inf -> uniform), over the
// NA = |neighbours| + 1 moves (stay last; Moore: 9, and add.reduce pairs 8+ terms).
// The exact (one-lane) kernel's; the batched step uses actor_policy.
template <class R>
__device__ int actor_choose(const LearnArgs& a, const double* hrow, const int* coord, const int* valid,
                            const float* dff, const HStat& hs, bool compat, int NA, R& rng) {
    double h[9], score[9], e[9], p[9];
    for (int k = 0; k < NA; k++) h[k] = hrow[k];
    if (hs.has && !hs.nonfinite && hs.mx - hs.mn > 1e-6) {
        const double smin = (double)a.smin, smax = (double)a.smax;
        for (int k = 0; k < NA; k++) h[k] = ((hs.mx - h[k]) / (hs.mx - hs.mn)) * (smax - smin) + smin;
    }
    bool bad = false;
    for (int k = 0; k < NA; k++) {
        const float d = a.kD32 * dff[coord[k]];
        score[k] = a.nkA * h[k] + (double)d;
        if (compat && !valid[k]) score[k] = -__builtin_inf();
        bad = bad || !__builtin_isfinite(score[k]);
    }
    if (bad)
        for (int k = 0; k < NA; k++) score[k] = valid[k] ? 1.0 : 0.0;
    double mx;
    if (compat) {
        double vs[9];
        int nv = 0;
        for (int k = 0; k < NA; k++)
            if (valid[k]) vs[nv++] = score[k];
        mx = nv ? np_max5(vs, nv) : 0.0;
    } else {
        mx = np_max5(score, NA);
    }
    int nvalid = 0, vidx[9];
    for (int k = 0; k < NA; k++) {
        e[k] = valid[k] ? det_exp(score[k] - mx) : 0.0;
        if (valid[k]) vidx[nvalid++] = k;
    }
    const double sum = np_sum_n(e, NA);
    if (__builtin_isfinite(sum) && sum > 0) {
        for (int k = 0; k < NA; k++) p[k] = e[k] / sum;
    } else {
        for (int k = 0; k < NA; k++) p[k] = valid[k] ? 1.0 / (double)nvalid : 0.0;
    }
    if (a.epsilon > 0 && rng.coin() < a.epsilon) {
        if (nvalid > 0) return vidx[rng.randint((uint32_t)nvalid)];
        return NA - 1;
    }
    return choice_cdf(p, NA, rng.u());
}

// Critic-only policy of ffm_unified (:353-392): raw SFF over all NA moves.
template <class R>
__device__ int critic_choose(const LearnArgs& a, const int* coord, const int* valid, const float* dff, int NA,
                             R& rng) {
    double p[9];
    int nvalid = 0;
    for (int k = 0; k < NA; k++) nvalid += valid[k];
    if (a.sff32) {
        float s[9], e[9];
        for (int k = 0; k < NA; k++) {
            const float x = a.kS32 * a.sff32[coord[k]];
            const float y = a.kD32 * dff[coord[k]];
            s[k] = x + y;
        }
        float mx = s[0];
        for (int k = 1; k < NA; k++) {
            if (s[k] != s[k]) { mx = s[k]; break; }
            mx = s[k] > mx ? s[k] : mx;
        }
        for (int k = 0; k < NA; k++) e[k] = valid[k] ? np_expf(s[k] - mx) : 0.0f;
        const float sum = np_sum_n(e, NA);
        if (__builtin_isfinite(sum) && sum > 0) {
            for (int k = 0; k < NA; k++) p[k] = (double)(e[k] / sum);
        } else {
            const float u = (float)(1.0 / (double)nvalid);
            for (int k = 0; k < NA; k++) p[k] = valid[k] ? (double)u : 0.0;
        }
    } else {
        double s[9], e[9];
        for (int k = 0; k < NA; k++) {
            const float y = a.kD32 * dff[coord[k]];
            s[k] = a.kS64 * a.sff64[coord[k]] + (double)y;
        }
        const double mx = np_max5(s, NA);
        for (int k = 0; k < NA; k++) e[k] = valid[k] ? det_exp(s[k] - mx) : 0.0;
        const double sum = np_sum_n(e, NA);
        if (__builtin_isfinite(sum) && sum > 0) {
            for (int k = 0; k < NA; k++) p[k] = e[k] / sum;
        } else {
            for (int k = 0; k < NA; k++) p[k] = valid[k] ? 1.0 / (double)nvalid : 0.0;
        }
    }
    return choice_cdf(p, NA, rng.u());
}

// ffm_ac_core decide == ffm_core decide (model/ffm_ac_core.py:126-199).
// `occ(cell)`: another agent stands there.  Returns the target or -1.
template <class OCC, class R>
__device__ int ac_decide(const LearnArgs& a, int x, int y, const OCC& occ, const float* dff, int& wexit, R& rng) {
    const int W = a.W;
    int cand[9], nc = 0;
    for (int k = 0; k < a.nb; k++) {
        const int cell = a.nb == 8 ? (x + kMBx[k]) * W + (y + kMBy[k]) : (x + kNBx[k]) * W + (y + kNBy[k]);
        const int m = a.map[cell];
        if (!(m == 0 || m == 3)) continue;
        if (occ(cell)) continue;
        cand[nc++] = cell;
    }
    if (nc == 0) return -1;
    cand[nc++] = x * W + y;
    for (int k = 0; k < nc; k++)
        if (a.map[cand[k]] == 3) { wexit = 1; return cand[k]; }
    double p[9];
    if (a.sff32) {
        float s[9], e[9];
        for (int k = 0; k < nc; k++) {
            const float u = a.kS32 * a.sff32[cand[k]];
            const float v = a.kD32 * dff[cand[k]];
            s[k] = u + v;
        }
        float mx = s[0];
        for (int k = 1; k < nc; k++) mx = s[k] > mx ? s[k] : mx;
        for (int k = 0; k < nc; k++) e[k] = np_expf(s[k] - mx);
        const float sum = np_sum_n(e, nc);
        if (!(__builtin_isfinite(sum) && sum != 0.0f)) return -1;
        for (int k = 0; k < nc; k++) p[k] = (double)(e[k] / sum);
    } else {
        double s[9], e[9];
        for (int k = 0; k < nc; k++) {
            const float v = a.kD32 * dff[cand[k]];
            s[k] = a.kS64 * a.sff64[cand[k]] + (double)v;
        }
        double mx = s[0];
        for (int k = 1; k < nc; k++) mx = s[k] > mx ? s[k] : mx;
        for (int k = 0; k < nc; k++) e[k] = det_exp(s[k] - mx);
        const double sum = np_sum_n(e, nc);
        if (!(__builtin_isfinite(sum) && sum != 0.0)) return -1;
        for (int k = 0; k < nc; k++) p[k] = e[k] / sum;
    }
    return cand[choice_cdf(p, nc, rng.u())];
}

// The five moves of agent (x, y) (neighbours U, D, L, R, then stay) with the
// reference's validity mask (model/ffm_unified.py:296-323).
template <class OCC>
__device__ __forceinline__ void moves5(const LearnArgs& a, int x, int y, const OCC& occ, int* coord, int* valid,
                                       int* inb) {
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const int nx = k < 4 ? x + kNBx[k] : x, ny = k < 4 ? y + kNBy[k] : y;
        inb[k] = nx >= 0 && nx < a.H && ny >= 0 && ny < a.W;
        coord[k] = inb[k] ? nx * a.W + ny : x * a.W + y;
        const int m = inb[k] ? map2_at(a.map2, coord[k]) : 2;
        valid[k] = inb[k] && (m == 0 || m == 3) && (k == 4 || !occ(coord[k]));
    }
    valid[4] = 1;
}

// The moves on the class-carrying grid: the NB neighbours in get_neighbors order
// (Neumann U, D, L, R; Moore row-major, model/ffm_unified.py:173-185), then stay, with
// the validity mask; cls[k] = the candidate's map class (2 off the map).
template <int NB>
__device__ __forceinline__ void moves_grid(const LearnArgs& a, int x, int y, const uint16_t* grid, int* coord,
                                           int* valid, int* inb, int* cls) {
#pragma unroll
    for (int k = 0; k <= NB; k++) {
        const int dx = k == NB ? 0 : NB == 8 ? kMBx[k] : kNBx[k], dy = k == NB ? 0 : NB == 8 ? kMBy[k] : kNBy[k];
        const int nx = x + dx, ny = y + dy;
        inb[k] = nx >= 0 && nx < a.H && ny >= 0 && ny < a.W;
        coord[k] = inb[k] ? nx * a.W + ny : x * a.W + y;
        const uint32_t g = grid[coord[k]];
        cls[k] = inb[k] ? (int)(g >> 14) : 2;
        valid[k] = inb[k] && (cls[k] == 0 || cls[k] == 3) && (k == NB || (g & kGIdx) == kGIdx);
    }
    valid[NB] = 1;
}

// The exact kernel's moves: the a.nb neighbours in get_neighbors order, then stay.
template <class OCC>
__device__ void moves_n(const LearnArgs& a, int x, int y, const OCC& occ, int* coord, int* valid, int* inb) {
    const int nb = a.nb;
    for (int k = 0; k <= nb; k++) {
        const int dx = k == nb ? 0 : (nb == 8 ? kMBx[k] : kNBx[k]), dy = k == nb ? 0 : (nb == 8 ? kMBy[k] : kNBy[k]);
        const int nx = x + dx, ny = y + dy;
        inb[k] = nx >= 0 && nx < a.H && ny >= 0 && ny < a.W;
        coord[k] = inb[k] ? nx * a.W + ny : x * a.W + y;
        const int m = inb[k] ? a.map[coord[k]] : 2;
        valid[k] = inb[k] && (m == 0 || m == 3) && (k == nb || !occ(coord[k]));
    }
    valid[nb] = 1;
}

__device__ void update_dff_seq(const LearnArgs& a, float* dff, float* B) {
    const int H = a.H, W = a.W, HW = a.HW;
    for (int i = 0; i < HW; i++) B[i] = a.c0 * dff[i];
    for (int x = 0; x < H; x++)
        for (int y = 0; y < W; y++) {
            float acc = B[x * W + y];
            for (int k = 0; k < a.nb; k++) {   // model/ffm_ac_core.py:298-317: every neighbour in order
                const int nx = x + (a.nb == 8 ? kMBx[k] : kNBx[k]), ny = y + (a.nb == 8 ? kMBy[k] : kNBy[k]);
                const float v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? B[nx * W + ny] : 0.0f;
                const float t = a.c1 * v;
                acc = acc + t;
            }
            dff[x * W + y] = acc < 1e-4f ? 0.0f : acc;
        }
}

__device__ void h_stats_seq(const LearnArgs& a, HStat& hs) {
    const uint32_t n = *a.Ht.n;
    hs.has = n > 0;
    hs.nonfinite = 0;
    hs.mn = __builtin_inf();
    hs.mx = -__builtin_inf();
    const int w = (int)a.Ht.accw;   // H rows: 5 values, 9 with the Moore neighbourhood
    for (uint32_t i = 0; i < n; i++) {
        const double* v = tval(a.Ht, a.Ht.order[i]);
        for (int k = 0; k < w; k++) {
            if (!__builtin_isfinite(v[k])) hs.nonfinite = 1;
            hs.mn = v[k] < hs.mn ? v[k] : hs.mn;
            hs.mx = v[k] > hs.mx ? v[k] : hs.mx;
        }
    }
    if (a.hx_n > 0) {          // ffm_trained_core rows held outside the table
        hs.has = 1;
        hs.nonfinite |= a.hx_nf;
        hs.mn = a.hx_mn < hs.mn ? a.hx_mn : hs.mn;
        hs.mx = a.hx_mx > hs.mx ? a.hx_mx : hs.mx;
    }
}

// A decision's policy, computed once per agent: the normalised cdf of
// np.random.choice (cdf / cdf[-1], model/ffm_unified.py:497) over the NA moves (the
// neighbours in get_neighbors order, then stay: 5 Neumann, 9 Moore; invalid moves
// carry zero mass) and the valid-move mask for the epsilon branch (:478-495).
// ffm_actor_only repeats the same decision once per neighbour (the inner-loop quirk,
// model/ffm_actor_only.py:214-355): within a batched step the table, DFF and
// statistics it reads are fixed, so only the draws differ.
template <int NA>
struct PolicyN {
    double cn[NA];
    int vmask;            // bit k: move k valid
    int none;             // ffm_ac_core: no request (softmax sum not finite / zero, :187)
};
using Policy = PolicyN<5>;

// NumPy's add.reduce of a fixed-length row (np_sum_n with a constant n: a left fold
// from -0 below eight terms, pairwise from eight on -- Moore's nine moves)
template <int N, class T>
__device__ __forceinline__ T np_sum_fix(const T (&e)[N]) {
    if (N < 8) {
        T res = T(-0.0);
#pragma unroll
        for (int k = 0; k < N; k++) res += e[k];
        return res;
    }
    return np_sum_n(e, N);
}

template <int NA>
__device__ __forceinline__ int kth_set_bit(int mask, int r) {
    int k = NA - 1;
#pragma unroll
    for (int j = NA - 1; j >= 0; j--) {
        const int below = __builtin_popcount(mask & ((1 << j) - 1));
        if (((mask >> j) & 1) && below == r) k = j;
    }
    return k;
}

template <int NA>
__device__ __forceinline__ void finish_cdf(PolicyN<NA>& P, const double* p) {
    double acc = 0.0, cdf[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) { acc += p[k]; cdf[k] = acc; }
#pragma unroll
    for (int k = 0; k < NA; k++) P.cn[k] = cdf[k] / acc;
}

template <int NA, class R>
__device__ __forceinline__ int policy_draw(const PolicyN<NA>& P, double eps, R& rng) {
    if (eps > 0 && rng.coin() < eps)
        return kth_set_bit<NA>(P.vmask, (int)rng.randint((uint32_t)__builtin_popcount(P.vmask)));
    const double u = rng.u();
    int k = NA - 1;
#pragma unroll
    for (int j = NA - 2; j >= 0; j--) k = P.cn[j] > u ? j : k;
    return k;
}

// Actor policy (model/ffm_unified.py:394-476; compat: model/ffm_actor_only.py:257-326,
// invalid moves -inf then uniform), the same arithmetic as actor_choose.
template <int NA>
__device__ __forceinline__ void actor_policy(const LearnArgs& a, const double* hrow, const int* coord,
                                             const int* valid, const float* dff, const HStat& hs, bool compat,
                                             PolicyN<NA>& P) {
    double h[NA], score[NA], e[NA], p[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) h[k] = hrow[k];
    if (hs.has && !hs.nonfinite && hs.mx - hs.mn > 1e-6) {
        const double smin = (double)a.smin, smax = (double)a.smax;
#pragma unroll
        for (int k = 0; k < NA; k++) h[k] = ((hs.mx - h[k]) / (hs.mx - hs.mn)) * (smax - smin) + smin;
    }
    bool bad = false;
    int vm = 0;
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const float d = a.kD32 * dff[coord[k]];
        score[k] = a.nkA * h[k] + (double)d;
        if (compat && !valid[k]) score[k] = -__builtin_inf();
        bad = bad || !__builtin_isfinite(score[k]);
        vm |= valid[k] << k;
    }
    // after the bad-score fallback every score is finite: np.max is a plain max
    double mx = -__builtin_inf();
#pragma unroll
    for (int k = 0; k < NA; k++) {
        if (bad) score[k] = valid[k] ? 1.0 : 0.0;
        const bool in = compat ? valid[k] != 0 : true;
        mx = in && score[k] > mx ? score[k] : mx;
    }
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const double x = det_exp(score[k] - mx);
        e[k] = valid[k] ? x : 0.0;
    }
    const double sum = np_sum_fix(e);
    const int nvalid = __builtin_popcount(vm);
    const bool ok = __builtin_isfinite(sum) && sum > 0;
#pragma unroll
    for (int k = 0; k < NA; k++) p[k] = ok ? e[k] / sum : (valid[k] ? 1.0 / (double)nvalid : 0.0);
    P.vmask = vm;
    P.none = 0;
    finish_cdf(P, p);
}

// ffm_unified critic_only policy (:353-392): SFF/DFF softmax over all NA moves,
// invalid ones masked after the exp.
template <int NA>
__device__ __forceinline__ void critic_policy(const LearnArgs& a, const int* coord, const int* valid,
                                              const float* dff, PolicyN<NA>& P) {
    double p[NA];
    int vm = 0;
#pragma unroll
    for (int k = 0; k < NA; k++) vm |= valid[k] << k;
    const int nvalid = __builtin_popcount(vm);
    if (a.sff32) {
        float s[NA], e[NA];
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float x = a.kS32 * a.sff32[coord[k]];
            const float y = a.kD32 * dff[coord[k]];
            s[k] = x + y;
        }
        float mx = s[0];
        bool nan = s[0] != s[0];
#pragma unroll
        for (int k = 1; k < NA; k++) {
            if (!nan && s[k] != s[k]) { mx = s[k]; nan = true; }
            if (!nan) mx = s[k] > mx ? s[k] : mx;
        }
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float x = np_expf(s[k] - mx);
            e[k] = valid[k] ? x : 0.0f;
        }
        const float sum = np_sum_fix(e);
        const bool ok = __builtin_isfinite(sum) && sum > 0;
        const float u = (float)(1.0 / (double)nvalid);
#pragma unroll
        for (int k = 0; k < NA; k++) p[k] = ok ? (double)(e[k] / sum) : (valid[k] ? (double)u : 0.0);
    } else {
        double s[NA], e[NA];
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float y = a.kD32 * dff[coord[k]];
            s[k] = a.kS64 * a.sff64[coord[k]] + (double)y;
        }
        const double mx = np_max5(s, NA);
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const double x = det_exp(s[k] - mx);
            e[k] = valid[k] ? x : 0.0;
        }
        const double sum = np_sum_fix(e);
        const bool ok = __builtin_isfinite(sum) && sum > 0;
#pragma unroll
        for (int k = 0; k < NA; k++) p[k] = ok ? e[k] / sum : (valid[k] ? 1.0 / (double)nvalid : 0.0);
    }
    P.vmask = vm;
    P.none = 0;
    finish_cdf(P, p);
}

// The free moves' terms in order (the compacted candidate list of ffm_ac_core), summed
// as add.reduce sums that list: a fold below eight terms, pairwise from eight on (Moore:
// eight or nine free moves; the list is formed by selects, not an indexed array).
template <int NA, class T>
__device__ __forceinline__ T np_sum_valid(const T (&e)[NA], const int* valid) {
    int nc = 0;
#pragma unroll
    for (int k = 0; k < NA; k++) nc += valid[k] ? 1 : 0;
    if (NA < 8 || nc < 8) {
        T sum = T(-0.0);
#pragma unroll
        for (int k = 0; k < NA; k++) sum = valid[k] ? sum + e[k] : sum;
        return sum;
    }
    if (nc == NA) return np_sum_n(e, NA);
    // NA = 9, one move blocked at z: the list skips it
    int z = 0;
#pragma unroll
    for (int k = NA - 1; k >= 0; k--) z = valid[k] ? z : k;
    T c[8];
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = j < z ? e[j] : e[j + 1 < NA ? j + 1 : j];
    return ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
}

// ffm_ac_core (= ffm_core) policy (model/ffm_ac_core.py:126-199): softmax over the
// free neighbours + stay.  Slots of blocked / occupied neighbours carry zero mass,
// which leaves every sum, running cdf and draw exactly as over the compacted list.
template <int NA>
__device__ __forceinline__ void ac_policy(const LearnArgs& a, const int* coord, const int* valid,
                                          const float* dff, PolicyN<NA>& P) {
    double p[NA];
    int vm = 0;
#pragma unroll
    for (int k = 0; k < NA; k++) vm |= valid[k] << k;
    bool fin;
    if (a.sff32) {
        float s[NA], e[NA];
        float mx = -__builtin_inff();
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float x = a.kS32 * a.sff32[coord[k]];
            const float y = a.kD32 * dff[coord[k]];
            s[k] = x + y;
            mx = valid[k] && s[k] > mx ? s[k] : mx;
        }
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float x = np_expf(s[k] - mx);
            e[k] = valid[k] ? x : 0.0f;
        }
        const float sum = np_sum_valid(e, valid);
        fin = __builtin_isfinite(sum) && sum != 0.0f;
#pragma unroll
        for (int k = 0; k < NA; k++) p[k] = valid[k] ? (double)(e[k] / sum) : 0.0;
    } else {
        double s[NA], e[NA];
        double mx = -__builtin_inf();
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float y = a.kD32 * dff[coord[k]];
            s[k] = a.kS64 * a.sff64[coord[k]] + (double)y;
            mx = valid[k] && s[k] > mx ? s[k] : mx;
        }
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const double x = det_exp(s[k] - mx);
            e[k] = valid[k] ? x : 0.0;
        }
        const double sum = np_sum_valid(e, valid);
        fin = __builtin_isfinite(sum) && sum != 0.0;
#pragma unroll
        for (int k = 0; k < NA; k++) p[k] = valid[k] ? e[k] / sum : 0.0;
    }
    P.vmask = vm;
    P.none = !fin;
    finish_cdf(P, p);
}

// ffm_trained_core policy (model/ffm_trained_core.py:219-300): the trained H row
// (float32; zeros when the state is missing), the whole-table min/max
// normalisation in float32 (Python floats are weak scalars next to the f32
// array), score -k_A*h + k_D*dff in float32, NumPy's float32 exp, masked sum and
// divide, uniform fallbacks.  Same arithmetic as the oracle's trained_choose.
template <int NA>
__device__ __forceinline__ void trained_policy(const LearnArgs& a, int hslot, const int* coord, const int* valid,
                                               const float* dff, const HStat& hs, PolicyN<NA>& P) {
    float h[NA], score[NA], e[NA];
    double p[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) h[k] = hslot >= 0 ? (float)tval(a.Ht, hslot)[k] : 0.0f;
    if (hs.has && !hs.nonfinite && hs.mx - hs.mn > 1e-6) {
        const float hmax = (float)hs.mx, den = (float)(hs.mx - hs.mn);
        const float srange = (float)((double)a.smax - (double)a.smin), smin = a.smin;
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const float q = (hmax - h[k]) / den;
            const float d = q * srange;
            h[k] = d + smin;
        }
    }
    const float nkA = (float)a.nkA;
    bool bad = false;
    int vm = 0;
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const float x = nkA * h[k];
        const float y = a.kD32 * dff[coord[k]];
        score[k] = x + y;
        bad = bad || !__builtin_isfinite(score[k]);
        vm |= valid[k] << k;
    }
    float mx = -__builtin_inff();
#pragma unroll
    for (int k = 0; k < NA; k++) {
        if (bad) score[k] = valid[k] ? 1.0f : 0.0f;
        mx = score[k] > mx ? score[k] : mx;
    }
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const float x = np_expf(score[k] - mx);
        e[k] = valid[k] ? x : 0.0f;
    }
    const float sum = np_sum_fix(e);
    const bool ok = __builtin_isfinite(sum) && sum > 0;
    const float u = (float)(1.0 / (double)__builtin_popcount(vm));
#pragma unroll
    for (int k = 0; k < NA; k++) p[k] = ok ? (double)(e[k] / sum) : (valid[k] ? (double)u : 0.0);
    P.vmask = vm;
    P.none = 0;
    finish_cdf(P, p);
}

// The same for the Moore neighbourhood (MT step only): nine moves in get_neighbors order
// then stay (:76-85), a nine-value H row (:228-236; zeros when missing), NumPy's pairwise
// add.reduce of the nine terms, np.random.choice over nine (cumsum, cdf /= cdf[-1],
// searchsorted).  Same arithmetic as the oracle's trained_choose(NA = 9).
template <class R>
__device__ int trained_choose_n(const LearnArgs& a, int hslot, const int* coord, const int* valid, const float* dff,
                                const HStat& hs, int NA, R& rng) {
    float h[9], score[9], e[9];
    double p[9];
    for (int k = 0; k < NA; k++) h[k] = hslot >= 0 ? (float)tval(a.Ht, hslot)[k] : 0.0f;
    if (hs.has && !hs.nonfinite && hs.mx - hs.mn > 1e-6) {
        const float hmax = (float)hs.mx, den = (float)(hs.mx - hs.mn);
        const float srange = (float)((double)a.smax - (double)a.smin), smin = a.smin;
        for (int k = 0; k < NA; k++) {
            const float q = (hmax - h[k]) / den;
            const float d = q * srange;
            h[k] = d + smin;
        }
    }
    const float nkA = (float)a.nkA;
    bool bad = false;
    int nvalid = 0;
    for (int k = 0; k < NA; k++) {
        const float x = nkA * h[k];
        const float y = a.kD32 * dff[coord[k]];
        score[k] = x + y;
        bad = bad || !__builtin_isfinite(score[k]);
        nvalid += valid[k];
    }
    if (bad)
        for (int k = 0; k < NA; k++) score[k] = valid[k] ? 1.0f : 0.0f;
    float mx = score[0];
    for (int k = 1; k < NA; k++) mx = score[k] > mx ? score[k] : mx;
    for (int k = 0; k < NA; k++) e[k] = valid[k] ? np_expf(score[k] - mx) : 0.0f;
    const float sum = np_sum_n(e, NA);
    if (__builtin_isfinite(sum) && sum > 0) {
        for (int k = 0; k < NA; k++) p[k] = (double)(e[k] / sum);
    } else {
        const float u = (float)(1.0 / (double)nvalid);
        for (int k = 0; k < NA; k++) p[k] = valid[k] ? (double)u : 0.0;
    }
    return choice_cdf(p, NA, rng.u());
}

struct ExactScratch {
    int *occ, *rq_tgt, *rq_agent, *list, *nxt, *coll, *act, *avalid, *wexit;
    uint8_t *sm, *smn, *done;
    float* B;
    unsigned long long* skey;
    double* td;
};

__host__ __device__ inline size_t exact_carve(unsigned char* base, int HW, int A, ExactScratch* s) {
    size_t o = 0;
    auto take = [&](size_t bytes) {
        unsigned char* p = base ? base + o : nullptr;
        o += (bytes + 15) & ~(size_t)15;
        return p;
    };
    const size_t R = (size_t)A * 8 + 1;   // requests: ffm_actor_only makes one per neighbour (Moore: 8)
    ExactScratch t;
    t.occ = (int*)take((size_t)HW * 4);
    t.rq_tgt = (int*)take(R * 4);
    t.rq_agent = (int*)take(R * 4);
    t.list = (int*)take(R * 4);
    t.nxt = (int*)take((size_t)A * 4 + 4);
    t.coll = (int*)take((size_t)A * 4 + 4);
    t.act = (int*)take((size_t)A * 4 + 4);
    t.avalid = (int*)take((size_t)A * 4 + 4);
    t.wexit = (int*)take((size_t)A * 4 + 4);
    t.sm = (uint8_t*)take((size_t)HW);
    t.smn = (uint8_t*)take((size_t)HW);
    t.done = (uint8_t*)take(R);
    t.B = (float*)take((size_t)HW * 4);
    t.skey = (unsigned long long*)take((size_t)A * 8 + 8);
    t.td = (double*)take((size_t)A * 8 + 8);
    if (s) *s = t;
    return o;
}

// ===========================================================================
// Reference-exact step (one lane, envs in order, MT streams).  Restates
// model/ffm_ac_core.py:111-236, model/ffm_unified.py:271-606 and
// model/ffm_actor_only.py:149-409 statement by statement.
// ===========================================================================
__global__ __launch_bounds__(64) void learn_exact_kernel(LearnArgs a) {
    if (threadIdx.x != 0) return;
    ExactScratch S;
    exact_carve(a.scratch, a.HW, a.A, &S);
    const int W = a.W, HW = a.HW, A = a.A;
    const int D = a.D;
    const bool actor = a.variant == kVarActorOnly || (a.variant == kVarUnified && a.mode != kModeCritic);
    const bool post_update = a.variant == kVarUnified && a.mode == kModeActor;
    const bool trained = a.variant == kVarTrained;
    for (int i = 0; i < HW; i++) S.occ[i] = -1;
    for (long long e = 0; e < a.E; e++) {
        uint16_t* pe = a.pos + e * A;
        float* dff = a.dff_in + e * (long long)HW;
        DrawMT rng{a.mt_np + e * 625, a.mt_py + e * 625};
        const int n = a.cnt[e];
        HStat hs{};
        if (actor || trained) h_stats_seq(a, hs);
        for (int c = 0; c < HW; c++) S.sm[c] = a.map[c];
        for (int i = 0; i < n; i++) { S.sm[pe[i]] = 1; S.occ[pe[i]] = i; }
        auto occ = [&](int c) { return S.occ[c] >= 0; };
        int nrq = 0;
        // ---- decide -------------------------------------------------------
        for (int i = 0; i < n; i++) {
            const int x = pe[i] / W, y = pe[i] % W;
            S.skey[i] = encode(a, SmArray{S.sm}, x, y);
            S.nxt[i] = pe[i];
            S.coll[i] = -1; S.act[i] = -1; S.avalid[i] = 0; S.wexit[i] = 0;
            if (a.variant == kVarAC) {
                const int T = ac_decide(a, x, y, occ, dff, S.wexit[i], rng);
                if (T >= 0) { S.rq_tgt[nrq] = T; S.rq_agent[nrq++] = i; }
                continue;
            }
            int coord[9], valid[9], inb[9];
            const int nb = a.nb, NA = nb + 1;
            moves_n(a, x, y, occ, coord, valid, inb);
            if (trained) {                                    // model/ffm_trained_core.py:169-258
                int k = -1;
                for (int j = 0; j < nb; j++)
                    if (inb[j] && a.map[coord[j]] == 3) { k = j; break; }
                if (k < 0 && nb == 8) {
                    k = trained_choose_n(a, tab_find(a.Ht, S.skey[i]), coord, valid, dff, hs, NA, rng);
                } else if (k < 0) {
                    Policy P;
                    trained_policy(a, tab_find(a.Ht, S.skey[i]), coord, valid, dff, hs, P);
                    const double u = rng.u();
                    k = 4;
                    for (int j = 3; j >= 0; j--) k = P.cn[j] > u ? j : k;
                }
                S.rq_tgt[nrq] = coord[k]; S.rq_agent[nrq++] = i;
                continue;
            }
            if (a.variant == kVarUnified) {
                int ex = -1;
                for (int k = 0; k < nb; k++)
                    if (inb[k] && a.map[coord[k]] == 3) { ex = k; break; }
                int k;
                if (ex >= 0) {
                    S.wexit[i] = 1;
                    k = ex;
                } else if (!actor) {
                    k = critic_choose(a, coord, valid, dff, NA, rng);
                } else {
                    const uint32_t before = *a.Ht.n;
                    const int hsl = tab_get(a.Ht, S.skey[i], a.overflow);
                    if (hsl < 0) return;
                    if (*a.Ht.n > before) {                   // a zero row joins min/max (:414-423)
                        hs.has = 1;
                        hs.mn = 0.0 < hs.mn ? 0.0 : hs.mn;
                        hs.mx = 0.0 > hs.mx ? 0.0 : hs.mx;
                    }
                    k = actor_choose(a, tval(a.Ht, hsl), coord, valid, dff, hs, false, NA, rng);
                }
                S.rq_tgt[nrq] = coord[k]; S.rq_agent[nrq++] = i;
                S.act[i] = k; S.avalid[i] = valid[k];
            } else {
                // ffm_actor_only: exit test and decision inside the neighbour loop (:214-355)
                int ex = -1;
                for (int j = 0; j < nb; j++) {
                    if (ex < 0 && inb[j] && a.map[coord[j]] == 3) ex = j;
                    int k;
                    if (ex >= 0) {
                        S.wexit[i] = 1;
                        k = ex;
                    } else {
                        const uint32_t before = *a.Ht.n;
                        const int hsl = tab_get(a.Ht, S.skey[i], a.overflow);
                        if (hsl < 0) return;
                        if (*a.Ht.n > before) {
                            hs.has = 1;
                            hs.mn = 0.0 < hs.mn ? 0.0 : hs.mn;
                            hs.mx = 0.0 > hs.mx ? 0.0 : hs.mx;
                        }
                        k = actor_choose(a, tval(a.Ht, hsl), coord, valid, dff, hs, true, NA, rng);
                    }
                    S.rq_tgt[nrq] = coord[k]; S.rq_agent[nrq++] = i;
                    S.act[i] = k; S.avalid[i] = valid[k];
                }
            }
        }
        // ---- resolve: dict order, always a winner (random.choice) ---------
        for (int q = 0; q < nrq; q++) S.done[q] = 0;
        for (int q = 0; q < nrq; q++) {
            if (S.done[q]) continue;
            const int T = S.rq_tgt[q];
            int m = 0;
            for (int q2 = q; q2 < nrq; q2++)
                if (S.rq_tgt[q2] == T) { S.list[m++] = S.rq_agent[q2]; S.done[q2] = 1; }
            int w;
            if (m == 1) {
                w = S.list[0];
                S.coll[w] = 0;
            } else {
                w = S.list[mt_randbelow(rng.py, (uint32_t)m)];
                for (int z = 0; z < m; z++) S.coll[S.list[z]] = m - 1;
            }
            S.nxt[w] = T;
            dff[pe[w]] += 1.0f;
        }
        // ---- learning (none for the trained actor) ----------------------------
        if (trained) goto exits;
        for (int c = 0; c < HW; c++) S.smn[c] = a.map[c];
        for (int i = 0; i < n; i++)
            if (a.map[S.nxt[i]] != 3) S.smn[S.nxt[i]] = 1;
        for (int i = 0; i < n; i++) {
            double r = a.step_penalty;
            if (S.wexit[i]) r = r + a.exit_reward;
            if (S.coll[i] >= 0) r = r + (double)S.coll[i] * a.collision_penalty;
            double vn = 0.0;
            if (!S.wexit[i]) {
                const int sn = tab_get(a.V, encode(a, SmArray{S.smn}, S.nxt[i] / W, S.nxt[i] % W), a.overflow);
                if (sn < 0) return;
                vn = tval(a.V, sn)[0];
            }
            const int sv = tab_get(a.V, S.skey[i], a.overflow);
            if (sv < 0) return;
            const double v = tval(a.V, sv)[0];
            const double td = (r + a.gamma * vn) - v;
            S.td[i] = td;
            tval(a.V, sv)[0] = v + a.alpha_v * td;
        }
        if (post_update) {        // _get_td_errors with the updated V (model/ffm_unified.py:568-574)
            for (int i = 0; i < n; i++) {
                double r = a.step_penalty;
                if (S.wexit[i]) r = r + a.exit_reward;
                if (S.coll[i] >= 0) r = r + (double)S.coll[i] * a.collision_penalty;
                double vn = 0.0;
                if (!S.wexit[i])
                    vn = tval(a.V, tab_get(a.V, encode(a, SmArray{S.smn}, S.nxt[i] / W, S.nxt[i] % W), a.overflow))[0];
                const double v = tval(a.V, tab_get(a.V, S.skey[i], a.overflow))[0];
                S.td[i] = (r + a.gamma * vn) - v;
            }
        }
        if (actor) {
            for (int i = 0; i < n; i++) {
                if (S.act[i] < 0) continue;
                const int hsl = tab_get(a.Ht, S.skey[i], a.overflow);    // :769-773
                if (hsl < 0) return;
                if (!S.avalid[i]) continue;
                double* hv = tval(a.Ht, hsl) + S.act[i];
                *hv = *hv + a.alpha_h * S.td[i];
            }
        }
        // ---- exit removal, DFF -------------------------------------------------
    exits:
        for (int i = 0; i < n; i++) S.occ[pe[i]] = -1;
        int nn = 0;
        for (int i = 0; i < n; i++)
            if (a.map[S.nxt[i]] != 3) pe[nn++] = (uint16_t)S.nxt[i];
        a.cnt[e] = nn;
        update_dff_seq(a, dff, S.B);
        unsigned long long* slot = a.counters + 4 * e;
        slot[0] += (unsigned long long)n;
        slot[1] += (unsigned long long)(n - nn);
        slot[3] += 1;
        (void)D;
    }
}

// Diagnostic builds only (tools/learn_ablate.sh): FFM_LABLATE bits drop parts of the
// batched step to time them.  1: table increments, 2: learning phase,
// 4: policy (agents stay; no H lookup), 8: DFF stencil, 16: V visit counts.
#ifndef FFM_SMALL_LPE
#define FFM_SMALL_LPE 32
#endif
#ifndef FFM_SMALL_EPB
#define FFM_SMALL_EPB 8
#endif
#ifndef FFM_RASTER
#define FFM_RASTER 1   // large-map learner: lanes walk the agents in cell-raster order (A/B switch)
#endif
#ifndef FFM_LABLATE
#define FFM_LABLATE 0
#endif
// FFM_LSTAMP (diagnostic builds): thread 0 of blocks 0 and gridDim/2 prints the
// wall-clock ticks (100 MHz) of each phase of the batched step.
#ifndef FFM_LSTAMP
#define FFM_LSTAMP 0
#endif
#if FFM_LSTAMP
#define LSTAMP(k) do { __syncthreads(); ts_[k] = wall_clock64(); } while (0)
#else
#define LSTAMP(k) do {} while (0)
#endif

// ===========================================================================
// Batched step: EPB envs per workgroup, LPE = BS / EPB lanes per env, APT
// agents per lane.  Small rooms (A <= 32) pack two envs onto one wavefront.
// ===========================================================================

// This env's epsilon: the learner's, or the batched schedule's after k ended
// episodes (run_actor_only_training.py:190-196, run_unified_actor_training.py:253-259).
// eps_phase spreads envs over the schedule: env g starts at its ((g % eps_phase) * eps_stride)-th
// episode, so E >= P envs running one episode each cover a per-configuration schedule of P
// episodes, and envs running `stride` episodes each cover a run-wide schedule env-major.
__device__ __forceinline__ double env_epsilon(const LearnArgs& a, int k, long long genv) {
    if (!(a.eps_span > 0)) return a.epsilon;
    const double ph = a.eps_phase > 0 ? (double)((genv % a.eps_phase) * (a.eps_stride > 0 ? a.eps_stride : 1)) : 0.0;
    const double e = a.eps_start + (a.eps_end - a.eps_start) * (((double)k + a.eps_offset + ph) / a.eps_span);
    return e < 0.0 ? 0.0 : e > 1.0 ? 1.0 : e;
}

// Tiled records (TileRec::td) carry the TD target r + gamma V(s') instead of the TD error
// unless the H pass needs the step-start error (ffm_unified both): the V pass reads V(s)
// anyway and subtracts it there (record_td), with the same operands and rounding.
__device__ __forceinline__ bool rec_target(const LearnArgs& a) { return a.mode != kModeBoth; }

// One record per ended episode (ffm_learner_drain_episodes).
__device__ __forceinline__ void log_episode(const LearnArgs& a, long long e) {
    const unsigned long long r = atomicAdd(a.eplog_n, 1ull);
    if ((long long)r >= a.eplog_cap) return;
    int* q = a.eplog + 4 * r;
    q[0] = (int)(a.env_base + e);
    q[1] = a.episodes[e];
    q[2] = a.ep_steps[e];
    q[3] = a.cnt[e] == 0;
}

// Segmented exclusive scan of a flag over each env's LPE lanes.
template <int BS, int LPE>
__device__ __forceinline__ int env_scan_flag(bool f, int* ws, int& total) {
    const unsigned long long m = __ballot(f);
    const int lane = threadIdx.x & 63;
    if (LPE <= 64) {
        const int seg = (lane / LPE) * LPE;
        const unsigned long long sm =
            (LPE == 64 ? m : (m >> seg) & ((1ull << (LPE & 63)) - 1));
        const int l = lane - seg;
        total = __popcll(sm);
        return __popcll(sm & ((1ull << l) - 1));
    }
    const int wv = (threadIdx.x % LPE) >> 6;
    const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (lane == 0) ws[wv] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < LPE / 64; w++) {
        const int c = ws[w];
        off += w < wv ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + pre;
}

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS of one env: occupancy grid, next-state bits, requests, scan words.  (Staging
// the map, SFF and DFF in LDS as well measured slower at config 4, 324 vs 295 us:
// they are L1/L2 hits, and the staging delays every short-lived workgroup.)
struct BatchCarve {
    size_t dff, rows, grid, bits, req, km, flist, fw, ws, total;  // per env
    size_t shared;                                     // per block: EPB env regions
};
// Packed state rows (the 13-cell encoders of ffm_ac_core / ffm_actor_only on maps at most
// 12 wide): per env two arrays of H + 4 words, the current and the next state, row x + 2
// holding map row x's 2-bit states at bits 2 (y + 2) and the out-of-map value in the two
// halo rows / columns on each side, so a key is five word reads and a few shifts.
__host__ __device__ inline int batch_rows(int H, int W, bool DL) { return DL && W <= 12 ? H + 4 : 0; }

// DL: the env's DFF is staged in LDS (small maps): the policy's reads, the
// deposits and the stencil stay on chip; only the stencil's output goes to HBM.
__host__ __device__ inline BatchCarve batch_carve(int HW, int A, int D, int EPB, bool DL = false, int RH = 0) {
    BatchCarve c;
    size_t o = 0;
    c.dff = o; o += DL ? align16((size_t)HW * 4) : 0;
    c.rows = o; o += align16((size_t)RH * 2 * 4);
    c.grid = o; o += align16((size_t)HW * 2);
    c.bits = o; o += align16((size_t)((HW + 31) / 32) * 4);
    c.req = o; o += align16((size_t)A * D * 2);
    c.km = o; o += D == 4 ? align16((size_t)A * 4) : 0;   // ffm_actor_only: request directions per agent
    // ffm_actor_only (D = 4): the contested targets' owners listed for one friction draw each
    // (flist, fcnt), the winners' ranks by owner request (fw)
    c.flist = o; o += D == 4 ? align16((size_t)A * D * 2) + 16 : 0;
    c.fw = o; o += D == 4 ? align16((size_t)A * D) : 0;
    c.ws = o; o += 64;
    c.total = o;
    c.shared = (size_t)EPB * o;
    return c;
}

#ifndef FFM_LBATCH_WAVES
#define FFM_LBATCH_WAVES 1   // minimum waves per SIMD asked of the register allocator
#endif

// VK = 1: the shape of BASELINE config 5 fixed at compile time -- ffm_unified in an actor
// mode, dense V and H, tiled records (learn_batch_uni) -- so the unrolled agent slots carry
// none of the other variants' paths (a fraction of the generic kernel's code: fewer
// instruction-cache misses across 16 waves walking it)
// per-slot state word (sa) of learn_batch_kernel: bit 15 = the decide phase inserted H(s)
constexpr uint32_t kSaNewH = 1u << 15;

// NB = 8: the Moore neighbourhood (model/ffm_unified.py:173-185, model/ffm_actor_only.py:
// 87-93): nine moves, nine-value H rows, requesters of a target on its eight neighbours,
// ffm_actor_only's eight decisions per agent (D = 8), the eight-neighbour stencil.
// The several-envs-per-workgroup ffm_actor_only shapes (D = 4) are asked for 8 waves
// per SIMD (64 VGPRs, 78 SGPRs, a few bytes of spill): 211.7 -> 204.6 us per config-4
// step in A/B; the D = 1 variants lose 0.7 % at 8 (a 100 B spill) and keep the default.
#ifndef FFM_LBATCH_SMALL_WAVES
#define FFM_LBATCH_SMALL_WAVES 8
#endif

// ffm_actor_only's resolve (D = 4, 32 lanes per env): the friction draw of a contested
// target depends only on its owner request and its requester count, so the owners are listed
// and each draw is computed once, by a lane of the list, instead of by every requester of
// every decision (four wave-wide Philox passes, whichever lanes need them).  0 = the per-decision draws.
#ifndef FFM_FRICTION_LIST
#define FFM_FRICTION_LIST 1
#endif

__device__ __forceinline__ void bk_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int BS, int EPB, int APT, int D, bool DL, int VK = 0, int NB = 4>
__global__ __launch_bounds__(BS)
__attribute__((amdgpu_waves_per_eu(EPB > 1 && NB == 4 && D == 4 ? FFM_LBATCH_SMALL_WAVES : FFM_LBATCH_WAVES, 8)))
void learn_batch_kernel(LearnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int LPE = BS / EPB;
    const int H = a.H, W = a.W, HW = a.HW, A = a.A;
    const int RH = batch_rows(H, W, DL);
    const BatchCarve cv = batch_carve(HW, A, D, EPB, DL, RH);
    const int sub = threadIdx.x / LPE, tid = threadIdx.x % LPE;
    unsigned char* base = smem + (size_t)sub * cv.total;
    uint32_t* crow = reinterpret_cast<uint32_t*>(base + cv.rows);   // current state rows (RH > 0)
    uint32_t* nrow = crow + RH;                                     // next state rows
    uint16_t* grid = reinterpret_cast<uint16_t*>(base + cv.grid);
    uint32_t* bits = reinterpret_cast<uint32_t*>(base + cv.bits);
    uint16_t* req = reinterpret_cast<uint16_t*>(base + cv.req);
    // D = 4: bit 4 * k + d set when the agent's decision d moves in direction k (0-3 the
    // neighbours, 4 stay or off the map: its own cell), read by the resolve phase
    uint32_t* km = reinterpret_cast<uint32_t*>(base + cv.km);
    int* ws = reinterpret_cast<int*>(base + cv.ws);
    uint16_t* flist = reinterpret_cast<uint16_t*>(base + cv.flist);   // D = 4: contested owners | m << 8
    int* fcnt = reinterpret_cast<int*>(base + cv.flist + align16((size_t)A * D * 2));
    uint8_t* fw = reinterpret_cast<uint8_t*>(base + cv.fw);             // D = 4: winner rank by owner
    const long long e = (long long)blockIdx.x * EPB + sub;
    const bool live = e < a.E;
    const uint32_t genv = (uint32_t)(a.env_base + e);
    const int n = live ? a.cnt[e] : 0;
    const bool vchain = a.v_chain && live && a.ep_steps[e] > 0;   // every V(s) was inserted as a V(s')
    constexpr bool UNI = VK == 1;
    const int variant = UNI ? (int)kVarUnified : a.variant;
    // the 13-cell encoders read the packed rows (out of the map: 2 for ffm_ac_core, 0 for
    // ffm_actor_only)
    const bool rows = !UNI && RH > 0 && (variant == kVarAC || variant == kVarActorOnly);
    const uint32_t oob = variant == kVarAC ? 2u : 0u;
    const bool actor = UNI || variant == kVarActorOnly || (variant == kVarUnified && a.mode != kModeCritic);
    const bool post_update = variant == kVarUnified && a.mode == kModeActor;
    const bool vdense = UNI || a.V.dense_by, hdense = UNI || a.Ht.dense_by;
    float* dff = DL ? reinterpret_cast<float*>(base + cv.dff) : a.dff_in + (live ? e : 0) * (long long)HW;
#if FFM_LSTAMP
    unsigned long long ts_[8];
#endif
    LSTAMP(0);
    // one env per workgroup: the positions' loads first, independent of the count's (both
    // in flight across the staging below; a slot at or past the count drops its value):
    // C5 762.5 -> 757.9 us; the several-envs shapes load them after the staging (C4 is
    // 1.5 us slower with them first)
    constexpr bool kEarlyPos = EPB == 1;
    uint32_t ppos[APT];
#pragma unroll
    for (int j = 0; j < APT; j++) {
        const int i = tid + j * LPE;
        ppos[j] = kEarlyPos && live && i < A ? (uint32_t)a.pos[e * A + i] : 0u;
    }

    {   // map classes into the grid two cells per dword (one map word covers eight pairs)
        uint32_t* g32 = reinterpret_cast<uint32_t*>(grid);
        for (int c2 = tid; c2 < HW / 2; c2 += LPE) {
            const uint32_t m = a.map2[c2 >> 3] >> ((c2 & 7) << 2);
            g32[c2] = (((m & 3u) << 14) | kGIdx) | ((((m >> 2) & 3u) << 14 | kGIdx) << 16);
        }
        if ((HW & 1) && tid == 0) grid[HW - 1] = (uint16_t)((map2_at(a.map2, HW - 1) << 14) | kGIdx);
    }
    if (DL) {
        const float* src = a.dff_in + (live ? e : 0) * (long long)HW;
        for (int c = tid; c < HW; c += LPE) dff[c] = src[c];
    }
    for (int c = tid; c < (HW + 31) / 32; c += LPE) bits[c] = 0u;
    if (rows)       // static rows: map classes (16 per map2 word), halo = the out-of-map value
        for (int r = tid; r < RH; r += LPE) {
            const uint32_t fill = oob * 0x55555555u;
            uint32_t v = fill;
            const int x = r - 2;
            if (x >= 0 && x < H) {
                const int c0 = x * W, w0 = c0 >> 4, sh = 2 * (c0 & 15);
                const unsigned long long m = (unsigned long long)a.map2[w0] |
                                             ((unsigned long long)(sh + 2 * W > 32 ? a.map2[w0 + 1] : 0u) << 32);
                const uint32_t cls = (uint32_t)(m >> sh) & (uint32_t)((1ull << (2 * W)) - 1);
                const uint32_t mid = (uint32_t)((1ull << (2 * W)) - 1) << 4;
                v = (fill & ~mid) | (cls << 4);
            }
            crow[r] = v;
            nrow[r] = v;
        }
    for (int c = tid; c < A * D; c += LPE) req[c] = kNone16;
    if (D == 4)
        for (int c = tid; c < A; c += LPE) km[c] = 0u;
    if (D == 4 && tid == 0) *fcnt = 0;
    __syncthreads();
    // Lane slot j of this thread is rank r = tid + j * LPE.  By default rank = agent
    // index; RASTER (global-memory DFF, >= one wave per env) instead hands rank r to
    // the r-th occupied cell in raster order, so the 64 agents of a wave stand on a
    // few neighbouring rows: their DFF lines, and the records of equal rank patterns
    // (rank-major dense slots), are shared instead of ~10 distinct lines per agent.
    // The agent index (owner priority, Philox keys, order-preserving compaction)
    // is then read back from the grid.
    constexpr bool RASTER = FFM_RASTER && !DL && LPE >= 64 && EPB == 1;
    // tiled step: records in raster order for the tile kernels, no
    // accumulator adds; set by the host for single-rank ffm_unified steps at block size 1
    const bool TILED = UNI || (RASTER && a.trecs != nullptr);
    // Per-agent state, packed so the APT slots of a lane stay in registers (APT = 8 at
    // C5: unpacked, the kernel spilled to scratch).  pa: cell (bits 0-15) | agent index
    // (16-29).  sa, from decide on: act + 1 (0-2), avalid (3), wexit (4), and from
    // resolve: coll + 1 (5-9), wins (10-13), next cell (16-31).  Moore: act + 1 (0-3),
    // avalid (4), wexit (5), coll + 1 (6-12: up to 72 requests of one target), no wins
    // (the resolve deposits them itself).
    constexpr int NA = NB + 1;
    constexpr int kAB = NB == 8 ? 4 : 3;                      // act + 1 bits
    constexpr uint32_t kSaValid = 1u << kAB, kSaWexit = 2u << kAB;
    constexpr int kCS = kAB + 2, kCB = NB == 8 ? 7 : 5;       // coll + 1 shift, bits
    constexpr uint32_t kSaDecide = (1u << kCS) - 1u;          // act, avalid, wexit
    uint32_t pa[APT], sa[APT];
#define BK_P(j) ((int)(pa[j] & 0xFFFFu))
#define BK_IA(j) ((int)(pa[j] >> 16))
#define BK_ACT(j) ((int)(sa[j] & ((1u << kAB) - 1u)) - 1)
#define BK_AVALID(j) ((int)((sa[j] >> kAB) & 1u))
#define BK_WEXIT(j) ((int)((sa[j] >> (kAB + 1)) & 1u))
#define BK_COLL(j) ((int)((sa[j] >> kCS) & ((1u << kCB) - 1u)) - 1)
#define BK_WINS(j) (NB == 8 ? 0 : (int)((sa[j] >> 10) & 15u))
#define BK_NXT(j) ((int)(sa[j] >> 16))
#define BK_NEWH(j) ((sa[j] & kSaNewH) != 0u)
#pragma unroll
    for (int j = 0; j < APT; j++) {
        const int i = tid + j * LPE;
        const int pj = i < n ? (kEarlyPos ? (int)ppos[j] : (int)a.pos[e * A + i]) : 0;
        pa[j] = (uint32_t)pj | ((uint32_t)i << 16);
        sa[j] = 0u;
        if (i < n) {
            grid[pj] = (uint16_t)((grid[pj] & ~kGIdx) | (uint32_t)i);
            if (RASTER) atomicOr(&bits[pj >> 5], 1u << (pj & 31));   // occupancy, for the raster pass
            if (rows) {     // an agent's free cell (class 0) reads 1
                const int x = fdiv(pj, a.mW);
                atomicOr(&crow[x + 2], 1u << (2 * (pj - x * W + 2)));
            }
        }
    }
    if (RASTER) {
        __syncthreads();
        // the occupied cells in raster order from the occupancy words (held in `bits` until
        // the resolve phase needs it): lane l of wave w owns K consecutive words, a scan of
        // the lanes' counts gives each its first rank, and its set bits are listed in order;
        // the list lives in req (A * D >= n entries) until decide overwrites it.
        constexpr int NW = LPE / 64;
        const int w = tid >> 6, lane = tid & 63;
        const int nwords = (HW + 31) / 32;
        const int wpw = (nwords + NW - 1) / NW, K = (wpw + 63) / 64;
        const int lw0 = w * wpw + lane * K;
        const int lw1 = min(min(lw0 + K, (w + 1) * wpw), nwords);
        int lc = 0;
        for (int q = lw0; q < lw1; q++) lc += __popc(bits[q]);
        int incl = lc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        if (lane == 63) ws[w] = incl;
        __syncthreads();
        int off = incl - lc;
#pragma unroll
        for (int q = 0; q < NW; q++) off += q < w ? ws[q] : 0;
        for (int q = lw0; q < lw1; q++) {
            uint32_t m = bits[q];
            if (a.trecs) {      // tiled step: the raster rank of the first agent of each tile
#pragma unroll
                for (int tt = 0; tt < 32 / kTileCells; tt++) {
                    const int tc = q * 32 + tt * kTileCells;
                    if (tc < HW)
                        a.tstart[e * (a.NT + 1) + tc / kTileCells] =
                            (uint16_t)(off + __popc(m & ((1u << (tt * kTileCells)) - 1u)));
                }
            }
            while (m) {
                const int b = __builtin_ctz(m);
                m &= m - 1u;
                req[off++] = (uint16_t)(q * 32 + b);
            }
        }
        if (a.trecs && tid == 0) a.tstart[e * (a.NT + 1) + a.NT] = (uint16_t)n;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < APT; j++) {
            const int r = tid + j * LPE;
            const int pj = r < n ? req[r] : 0;
            pa[j] = (uint32_t)pj | ((uint32_t)(r < n ? (grid[pj] & kGIdx) : r) << 16);
        }
        __syncthreads();   // the list is read: decide may write req
        for (int c = tid; c < n; c += LPE) req[c] = kNone16;
        for (int c = tid; c < nwords; c += LPE) bits[c] = 0u;   // the next-state bits start empty
        __syncthreads();
    }
    const bool trained = variant == kVarTrained;
    const double eps = live && actor ? env_epsilon(a, a.episodes[e], a.env_base + e) : 0.0;
    HStat hs{};
    if (actor || trained) {
        hs.has = (int)a.hstat[0];
        hs.nonfinite = (int)a.hstat[1];
        hs.mn = a.hstat[2];
        hs.mx = a.hstat[3];
    }
    __syncthreads();
    const SmGridC smc{grid};
    LSTAMP(1);

    // ---- decide --------------------------------------------------------------
    // state keys: kept per slot when a lane walks few agents; with APT >= 4 (1,024-lane
    // workgroups on large maps) the learn phase re-encodes them from the unchanged grid
    // instead (twelve LDS reads), which keeps the slots' state in registers
    constexpr bool KEYS = APT < 4;
    unsigned long long skey[KEYS ? APT : 1];
    int hsl[KEYS ? APT : 1];     // H slot of the decide phase's lookup (-1: none)
#pragma unroll
    for (int j = 0; j < APT; j++) {
        const int i = BK_IA(j);
        sa[j] = 0u;
        if (KEYS) { skey[j] = 0; hsl[j] = -1; }
        if (tid + j * LPE >= n) continue;
        const int x = fdiv(BK_P(j), a.mW), y = BK_P(j) - x * W;
        const unsigned long long sk = rows ? enc13_rows(crow, x, y, a.mBS) : encode_v(a, variant, smc, x, y);
        if (KEYS) skey[j] = sk;
        int coord[NA], valid[NA], inb[NA];
        int cls[NA];
        moves_grid<NB>(a, x, y, grid, coord, valid, inb, cls);
        int ex = -1;                               // first exit among the neighbours
#pragma unroll
        for (int k = NB - 1; k >= 0; k--) ex = inb[k] && cls[k] == 3 ? k : ex;
        PolicyN<NA> P;
        if (FFM_LABLATE & 4) {
            req[i * D] = (uint16_t)BK_P(j);
            sa[j] = (uint32_t)NA | kSaValid;
            continue;
        }
        if (variant == kVarAC) {
            // ffm_core candidates: free neighbours, then stay if any (:126-164)
            int anyv = 0;
#pragma unroll
            for (int k = 0; k < NB; k++) anyv |= valid[k];
            if (anyv == 0) continue;
            int exv = -1;
#pragma unroll
            for (int k = NB - 1; k >= 0; k--) exv = valid[k] && cls[k] == 3 ? k : exv;
            if (exv >= 0) {
                sa[j] |= kSaWexit;
                req[i] = (uint16_t)coord[exv];
                continue;
            }
            ac_policy(a, coord, valid, dff, P);
            if (P.none) continue;
            DrawPh rng(a, genv, (uint32_t)i);
            req[i] = (uint16_t)coord[policy_draw(P, 0.0, rng)];
            continue;
        }
        if (D == 1) {
            int k;
            if (ex >= 0) {
                sa[j] |= kSaWexit;
                k = ex;
            } else {
                if (trained) {
                    trained_policy(a, tab_find(a.Ht, sk), coord, valid, dff, hs, P);
                } else if (!actor) {
                    critic_policy(a, coord, valid, dff, P);
                } else if (hdense) {
                    const int h = (int)dense_slot(sk, a.Ht);
                    if (KEYS) hsl[j] = h;
                    // the record's key with the row (one line): present rows skip the bitmap
                    ulonglong2 r[(NA + 2) / 2];
#pragma unroll
                    for (int q = 0; q < (NA + 2) / 2; q++) r[q] = trec16(a.Ht, h, q);
                    double hr[NA];
#pragma unroll
                    for (int q = 0; q < NA; q++)
                        hr[q] = __longlong_as_double((long long)((q & 1) ? r[(q + 1) / 2].x : r[(q + 1) / 2].y));
                    actor_policy(a, hr, coord, valid, dff, hs, false, P);
                    if (r[0].x == kEmptyKey && dense_ensure_new(a.Ht, (uint32_t)h, sk)) sa[j] |= kSaNewH;
                } else {
                    double hr[NA];
                    const int h = tab_get_row<NA>(a.Ht, sk, a.overflow, hr);
                    if (KEYS) hsl[j] = h;
                    if (h < 0) continue;
                    actor_policy(a, hr, coord, valid, dff, hs, false, P);
                }
                DrawPh rng(a, genv, (uint32_t)i);
                k = policy_draw(P, eps, rng);
            }
            req[i] = (uint16_t)coord[k];
            sa[j] = (sa[j] & ~(kSaValid | ((1u << kAB) - 1u))) | (uint32_t)(k + 1) | ((uint32_t)valid[k] << kAB);
        } else {
            // model/ffm_actor_only.py:214-355: decisions for the neighbours before the
            // first exit, then the exit for the rest; the last one is the agent's action.
            if (ex != 0) {
                double hr[NA];
                const int h = tab_get_row<NA>(a.Ht, sk, a.overflow, hr);
                if (KEYS) hsl[j] = h;
                if (h < 0) continue;
                actor_policy(a, hr, coord, valid, dff, hs, true, P);
            }
            int k = NB;
            uint32_t kmi = 0u;
#pragma unroll
            for (int d = 0; d < D; d++) {
                if (ex >= 0 && d >= ex) {
                    k = ex;
                } else {
                    DrawPh rng(a, genv, (uint32_t)(i * D + d));
                    k = policy_draw(P, eps, rng);
                }
                req[i * D + d] = (uint16_t)coord[k];
                if (D == 4) kmi |= 1u << ((inb[k] ? k : 4) * 4 + d);   // off the map: the agent's own cell
            }
            if (D == 4) km[i] = kmi;
            sa[j] = (uint32_t)(k + 1) | ((uint32_t)valid[k] << kAB) | (ex >= 0 ? kSaWexit : 0u);
        }
    }
    __syncthreads();
    LSTAMP(2);

    // ---- resolve -----------------------------------------------------------------
    // Requesters of a target stand on it or next to it; a target's owner is its
    // smallest request seq (= the reference's dict order); every member draws
    // the winner rank from the owner's stream itself.
    constexpr bool FLIST = FFM_FRICTION_LIST && D == 4 && NB == 4 && LPE <= 64 && 64 % LPE == 0 && LPE * APT * D <= 256;
    if constexpr (FLIST) {
        // 1. every decision's requester count m, owner request and rank among the requests;
        //    the owner of a contested target lists it
        uint32_t dr[APT][D];
#pragma unroll
        for (int j = 0; j < APT; j++) {
            const int i = BK_IA(j);
#pragma unroll
            for (int d = 0; d < D; d++) {
                dr[j][d] = 0xFFFFFFFFu;
                if (tid + j * LPE >= n) continue;
                const int T = req[i * D + d];
                if (T == kNone16) continue;
                const int tx = fdiv(T, a.mW), ty = T - tx * W;
                int m = 0, owner = 0x7FFF, rank = 0;
#pragma unroll
                for (int c5 = 0; c5 < NA; c5++) {
                    const int cx = c5 < NB ? tx + kNBx[c5] : tx, cy = c5 < NB ? ty + kNBy[c5] : ty;
                    if (cx < 0 || cx >= H || cy < 0 || cy >= W) continue;
                    const int b = grid[cx * W + cy] & kGIdx;
                    if (b == (int)kGIdx) continue;
                    // see the per-decision form below: one mask read per requester cell
                    const uint32_t f = (km[b] >> ((c5 < 4 ? (c5 ^ 1) : 4) * 4)) & 15u;
                    if (!f) continue;
                    m += __popc(f);
                    const int sq = b * D + (int)__builtin_ctz(f);
                    owner = sq < owner ? sq : owner;
                    rank += b < i ? __popc(f) : b == i ? __popc(f & ((1u << d) - 1u)) : 0;
                }
                dr[j][d] = (uint32_t)m | ((uint32_t)rank << 8) | ((uint32_t)owner << 16);
                if (m > 1 && owner == i * D + d) flist[atomicAdd(fcnt, 1)] = (uint16_t)(owner | (m << 8));
            }
        }
        bk_wave_sync();   // an env's lanes are one wave (LPE divides 64)
        // 2. one friction draw per listed owner (model/ffm_actor_only.py:360-401)
        const int nf = *fcnt;
        for (int c = 0;; c += LPE) {
            const bool has = c + tid < nf;
            if (!__any(has)) break;
            if (has) {
                const uint32_t en = flist[c + tid];
                PhiloxStream ps(a.key0, a.key1, a.t, genv, en & 0xFFu, kPurFriction);
                fw[en & 0xFFu] = (uint8_t)ps.randbelow(en >> 8);
            }
        }
        bk_wave_sync();
        // 3. every request: won iff its rank is the owner's draw
#pragma unroll
        for (int j = 0; j < APT; j++) {
            int nxj = BK_P(j), clj = -1, wnj = 0;
            int best_owner = -1, best_won_owner = -1;
#pragma unroll
            for (int d = 0; d < D; d++) {
                const uint32_t v = dr[j][d];
                if (v == 0xFFFFFFFFu) continue;
                const int m = (int)(v & 0xFFu), rank = (int)((v >> 8) & 0xFFu), owner = (int)(v >> 16);
                const int w = m > 1 ? (int)fw[owner] : 0;
                if (owner > best_owner) { best_owner = owner; clj = m == 1 ? 0 : m - 1; }
                if (rank == w) {
                    wnj++;
                    if (owner > best_won_owner) { best_won_owner = owner; nxj = req[BK_IA(j) * D + d]; }
                }
            }
            sa[j] = (sa[j] & (kSaDecide | kSaNewH)) | ((uint32_t)(clj + 1) << kCS) | ((uint32_t)wnj << 10) |
                    ((uint32_t)nxj << 16);
        }
    }
#pragma unroll
    for (int j = 0; j < (FLIST ? 0 : APT); j++) {
        const int i = BK_IA(j);
        int nxj = BK_P(j), clj = -1, wnj = 0;
        if (tid + j * LPE < n) {
        int best_owner = -1, best_won_owner = -1;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int T = req[i * D + d];
            if (T == kNone16) continue;
            const int mine = i * D + d;
            const int tx = fdiv(T, a.mW), ty = T - tx * W;
            int m = 0, owner = 0x7FFFFFFF, rank = 0;
#pragma unroll
            for (int c5 = 0; c5 < NA; c5++) {
                const int cx = c5 < NB ? tx + (NB == 8 ? kMBx[c5] : kNBx[c5]) : tx,
                          cy = c5 < NB ? ty + (NB == 8 ? kMBy[c5] : kNBy[c5]) : ty;
                if (cx < 0 || cx >= H || cy < 0 || cy >= W) continue;
                const int b = grid[cx * W + cy] & kGIdx;
                if (b == (int)kGIdx) continue;
                if (D == 4) {
                    // agent b on the cell requests T with the decisions whose direction leads
                    // there: from a neighbour of T the opposite of c5 (U<->D, L<->R), from T itself
                    // a stay (or a move off the map) -- one mask read instead of D request reads
                    const uint32_t f = (km[b] >> ((c5 < 4 ? (c5 ^ 1) : 4) * 4)) & 15u;
                    if (!f) continue;
                    m += __popc(f);
                    const int sq = b * D + (int)__builtin_ctz(f);
                    owner = sq < owner ? sq : owner;
                    rank += b < i ? __popc(f) : b == i ? __popc(f & ((1u << d) - 1u)) : 0;
                    continue;
                }
#pragma unroll
                for (int d2 = 0; d2 < D; d2++) {
                    const int sq = b * D + d2;
                    if (req[sq] != T) continue;
                    m++;
                    owner = sq < owner ? sq : owner;
                    rank += sq < mine ? 1 : 0;
                }
            }
            int w = 0;
            if (m > 1) {
                PhiloxStream ps(a.key0, a.key1, a.t, genv, (uint32_t)owner, kPurFriction);
                w = (int)ps.randbelow((uint32_t)m);
            }
            if (owner > best_owner) { best_owner = owner; clj = m == 1 ? 0 : m - 1; }
            if (rank == w) {
                wnj++;
                if (owner > best_won_owner) { best_won_owner = owner; nxj = T; }
                if (NB == 8) {   // the win's deposit at the agent's own cell (no other lane writes it)
                    float* c = dff + BK_P(j);
                    *c = *c + 1.0f;
                }
            }
        }
        }
        sa[j] = (sa[j] & (kSaDecide | kSaNewH)) | ((uint32_t)(clj + 1) << kCS) |
                (NB == 8 ? 0u : (uint32_t)wnj << 10) | ((uint32_t)nxj << 16);
    }
    // deposits at the winners' own cells (distinct per agent: no races); every
    // agent's next cell joins the next state map unless it is an exit
#pragma unroll
    for (int j = 0; j < APT; j++) {
        if (tid + j * LPE >= n) continue;
        if (BK_WINS(j)) {
            float* c = dff + BK_P(j);
            float v = *c;
            for (int q = 0; q < BK_WINS(j); q++) v = v + 1.0f;
            *c = v;
        }
        if ((grid[BK_NXT(j)] >> 14) != 3) {
            atomicOr(&bits[BK_NXT(j) >> 5], 1u << (BK_NXT(j) & 31));
            if (rows) {
                const int x = fdiv(BK_NXT(j), a.mW);
                atomicOr(&nrow[x + 2], 1u << (2 * (BK_NXT(j) - x * W + 2)));
            }
        }
    }
    __syncthreads();
    LSTAMP(3);

    // ---- learning (TD(0) critic, actor) --------------------------------------------------
    const SmBitsC smn{grid, bits};
#pragma unroll
    for (int j = 0; j < APT; j++) {
        const int i = tid + j * LPE;   // recs in lane-rank order: the post kernel inherits the locality
        int vsl = -1;      // this lane's V slot and fixed-point td, added after the block
        long long vq = 0;
        double tdv = 0.0;  // tiled step: the record's td, s' slot and action
        int snv = -1, kk = (int)kTileNoAct;
        bool newh = BK_NEWH(j);   // this step inserted H(s) here (decide, or an exit-forced agent below)
        do {
            if (i >= n || trained || (FFM_LABLATE & 2)) break;
            unsigned long long skj;
            if (KEYS) {
                skj = skey[j];
            } else {
                const int px = fdiv(BK_P(j), a.mW);
                skj = rows ? enc13_rows(crow, px, BK_P(j) - px * W, a.mBS) : encode_v(a, variant, smc, px, BK_P(j) - px * W);
            }
            double r = a.step_penalty;
            if (BK_WEXIT(j)) r = r + a.exit_reward;
            if (BK_COLL(j) >= 0) r = r + (double)BK_COLL(j) * a.collision_penalty;
            int sn = -1, sv;
            double vn = 0.0, vs = 0.0;
            unsigned long long nk = 0;
            if (!BK_WEXIT(j)) {
                const int nx = fdiv(BK_NXT(j), a.mW), ny = BK_NXT(j) - nx * W;
                nk = rows ? enc13_rows(nrow, nx, ny, a.mBS) : encode_v(a, variant, smn, nx, ny);
            }
            if (vdense) {
                if (!BK_WEXIT(j)) {
                    sn = (int)dense_slot(nk, a.V);
                    const ulonglong2 rn = trec16(a.V, sn);      // key and value: one 16-B record
                    vn = __longlong_as_double((long long)rn.y);
                    if (rn.x == kEmptyKey) dense_ensure(a.V, (uint32_t)sn, nk);
                }
                sv = (int)dense_slot(skj, a.V);
                // s is the previous step's s' (inserted then) unless the episode starts here
                // or the tables / positions were replaced since (LearnArgs::v_chain)
                if (!vchain) dense_ensure(a.V, (uint32_t)sv, skj);
                if (!(TILED && rec_target(a))) vs = tval(a.V, sv)[0];
            } else {
                // both home slots in one round trip; the probing / inserting path only for
                // keys away from home, s' before s as before
                uint32_t hn, hv;
                double pn[1], pv[1];
                const bool okn = tab_peek<1>(a.V, nk, hn, pn);
                const bool okv = tab_peek<1>(a.V, skj, hv, pv);
                if (!BK_WEXIT(j)) {
                    if (okn) {
                        sn = (int)hn;
                        vn = pn[0];
                    } else {
                        sn = tab_get(a.V, nk, a.overflow);
                        vn = sn >= 0 ? tval(a.V, sn)[0] : 0.0;
                    }
                }
                if (okv) {
                    sv = (int)hv;
                    vs = pv[0];
                } else {
                    sv = tab_get(a.V, skj, a.overflow);
                    if (sv >= 0) vs = tval(a.V, sv)[0];
                }
            }
            if (sv < 0) break;
            const double y = r + a.gamma * vn;
            vsl = sv;
            if (TILED && rec_target(a)) {
                tdv = y;           // the V pass subtracts V(s) (record_td): one table read less here
            } else {
                const double td = y - vs;
                vq = fx(td);
                tdv = td;
            }
            snv = sn;
            if (!actor) break;
            if (BK_ACT(j) < 0) break;
            // the decide phase's H slot; without KEYS, dense tables recompute it (the decide
            // phase inserted it unless the agent was exit-forced) and hashed ones probe again
            int hslj = KEYS ? hsl[j] : (hdense && !BK_WEXIT(j) ? (int)dense_slot(skj, a.Ht) : -1);
            if (hslj < 0) {     // dense: slot + insert, no probe (flagged for the owner exchange)
                if (hdense) {
                    hslj = (int)dense_slot(skj, a.Ht);
                    if (dense_ensure_new(a.Ht, (uint32_t)hslj, skj)) newh = true;
                } else {
                    hslj = tab_get(a.Ht, skj, a.overflow);
                }
            }
            if (hslj < 0) break;
            if (TILED) {            // the tile kernels sum the increments (hsl == sv: one dense layout)
                kk = BK_AVALID(j) ? BK_ACT(j) : (int)kTileNoAct;
                break;
            }
            if (post_update) {
                LearnRec rc;
                rc.r = r; rc.sv = sv; rc.snv = sn; rc.hslot = hslj; rc.k = BK_AVALID(j) ? BK_ACT(j) : -1;
                a.recs[e * A + i] = rc;
            } else if (BK_AVALID(j) && !(FFM_LABLATE & 1)) {
                acc_add(acc_at(a.Ht, (size_t)hslj * NA + BK_ACT(j)), fx(a.alpha_h * tdv));
            }
        } while (false);
        if (TILED) {
            if (vsl >= 0) {
                TileRec rc;
                rc.svk = (uint32_t)vsl | (newh ? kTileNewH : 0u) | ((uint32_t)kk << 28);
                rc.snf = (snv >= 0 ? (uint32_t)snv : kTileTerminal) | ((uint32_t)BK_WEXIT(j) << kTileExitBit) |
                         ((uint32_t)(BK_COLL(j) + 1) << kTileCollShift);
                rc.td = tdv;
                a.trecs[e * A + i] = rc;
            }
        } else if (!(FFM_LABLATE & 1)) {
            v_pair_add(a.V, vsl, vq);
        }
    }
    LSTAMP(4);
    // ---- exit removal (order preserving), counters ---------------------------------------
    int base_ = 0;
    if (RASTER) {
        // back to agent order for the order-preserving compaction: next cells by agent
        // index through req (resolve's last read of it is behind the barrier above)
#pragma unroll
        for (int j = 0; j < APT; j++)
            if (tid + j * LPE < n) req[BK_IA(j)] = (grid[BK_NXT(j)] >> 14) != 3 ? (uint16_t)BK_NXT(j) : kNone16;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < APT; j++) {
            const int i = tid + j * LPE;
            const int c = i < n ? req[i] : kNone16;
            const bool keep = c != kNone16;
            int tot;
            const int off = env_scan_flag<BS, LPE>(keep, ws, tot);
            if (keep) a.pos[e * A + base_ + off] = (uint16_t)c;
            base_ += tot;
        }
    } else {
#pragma unroll
        for (int j = 0; j < APT; j++) {
            const int i = tid + j * LPE;
            const bool keep = i < n && (grid[BK_NXT(j)] >> 14) != 3;
            int tot;
            const int off = env_scan_flag<BS, LPE>(keep, ws, tot);
            if (keep) a.pos[e * A + base_ + off] = (uint16_t)BK_NXT(j);
            base_ += tot;
        }
    }
    __syncthreads();     // deposits visible to the whole workgroup before the stencil
    LSTAMP(5);

    // ---- update_dff (model/ffm_unified.py:779-798) into the other buffer ---------------------
    if (live && !a.sep_stencil && !(FFM_LABLATE & 8)) {
        float* out = a.dff_out + e * (long long)HW;
        for (int c = tid; c < HW; c += LPE) {
            const int x = fdiv(c, a.mW), y = c - x * W;
            float acc = a.c0 * dff[c];
#pragma unroll
            for (int k = 0; k < NB; k++) {
                const int nx = x + (NB == 8 ? kMBx[k] : kNBx[k]), ny = y + (NB == 8 ? kMBy[k] : kNBy[k]);
                const float v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? a.c0 * dff[nx * W + ny] : 0.0f;
                const float t = a.c1 * v;
                acc = acc + t;
            }
            out[c] = acc < 1e-4f ? 0.0f : acc;
        }
    }
    LSTAMP(6);
#if FFM_LSTAMP
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
        printf("LSTAMP blk %d init %llu decide %llu resolve %llu learn %llu compact %llu stencil %llu\n", (int)blockIdx.x,
               ts_[1] - ts_[0], ts_[2] - ts_[1], ts_[3] - ts_[2], ts_[4] - ts_[3], ts_[5] - ts_[4], ts_[6] - ts_[5]);

#endif
#undef BK_P
#undef BK_IA
#undef BK_ACT
#undef BK_AVALID
#undef BK_WEXIT
#undef BK_COLL
#undef BK_WINS
#undef BK_NXT
    if (live && tid == 0) {
        a.cnt[e] = base_;
        a.nstart[e] = n;
        const int st = a.ep_steps[e] + 1;
        a.ep_steps[e] = st;
        a.done[e] = a.auto_reset && (base_ == 0 || (a.max_steps > 0 && st >= a.max_steps)) ? 1 : 0;
        unsigned long long* slot = a.counters + 4 * e;
        slot[0] += (unsigned long long)n;
        slot[1] += (unsigned long long)(n - base_);
        slot[3] += 1;
    }
}

// ===========================================================================
// The phase-split batch step: learn_batch_kernel's phases for the
// VK = 1 shape (ffm_unified in an actor mode, dense tables, tiled records, one decision
// per agent, maps of at most 65,536 cells) as four launches.  The fused kernel holds an
// env's 128 KB agent grid in LDS, so one 1,024-lane workgroup per CU walks eight agents
// per lane through dependent table reads; here the table-bound phases (decide: state
// key -> H row -> policy; learn: next-state key -> V rows) run one agent per lane at
// full occupancy from two 2-bit state maps in global memory (L2-resident), and only
// the conflict resolution keeps a per-env LDS workgroup (68 KB: two per CU).
//   prep    (env per workgroup): occupancy bits, the current state map, the agents in
//           raster order (cell, agent index), the tile offsets of the records;
//   decide  (agent per lane, raster order): target, action, validity, exit forcing;
//   resolve (env per workgroup): requesters of each target, friction draw, deposits,
//           the next state map, order-preserving exit removal, counters;
//   learn   (agent per lane): the TD error and the record of learn_batch_kernel.
// Every value is computed by the same expressions in the same order as the fused
// kernel's, so the step is bit-identical to it (and to the oracle).
// ===========================================================================
constexpr int kPhBS = 1024;              // prep / resolve workgroup (one env)
constexpr int kPhLanes = 256;            // decide / learn workgroup (256 consecutive raster ranks)
constexpr int kPhWords = 65536 / 32;     // occupancy words of the largest map

struct PhaseCarve {
    uint32_t* sm;     // [E][mw] current state map: 2 bits per cell, occupied ? 1 : map class
    uint32_t* nm;     // [E][mw] next state map (next cells that are not exits)
    uint16_t* rc;     // [E][A] cell of raster rank r
    uint16_t* ri;     // [E][A] agent index of raster rank r
    uint32_t* dec;    // [E][A] decide: target (0-15), action + 1 (16-18), valid (19), exit-forced (20)
    uint32_t* res;    // [E][A] resolve: next cell (0-15), collisions + 1 (16-20), decide bits 16-20 (21-25)
};

__host__ __device__ inline PhaseCarve phase_carve(unsigned char* b, long long E, int HW, int A) {
    const size_t mw = (size_t)(HW + 15) / 16;
    PhaseCarve c;
    c.sm = reinterpret_cast<uint32_t*>(b);
    c.nm = c.sm + (size_t)E * mw;
    c.rc = reinterpret_cast<uint16_t*>(c.nm + (size_t)E * mw);
    c.ri = c.rc + (size_t)E * A;
    c.dec = reinterpret_cast<uint32_t*>(c.ri + (size_t)E * A);
    c.res = c.dec + (size_t)E * A;
    return c;
}

struct Sm2 {                     // a 2-bit state map in global memory
    const uint32_t* m;
    __device__ int operator()(int c) const { return (int)((m[c >> 4] >> ((c & 15) << 1)) & 3u); }
};

// 16 occupancy bits into a word of 16 2-bit map classes: occupied cells read 1.
__device__ __forceinline__ uint32_t state2(uint32_t m2, uint32_t o16) {
    uint32_t x = o16;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return (m2 & ~(x | (x << 1))) | x;
}

// Raster rank of cell c: the occupied cells before it.
__device__ __forceinline__ int cell_rank(const uint32_t* occ, const uint16_t* pre, int c) {
    return (int)pre[c >> 5] + __popc(occ[c >> 5] & ((1u << (c & 31)) - 1u));
}

// Exclusive block scan of one value per thread (BS threads); ends after a barrier.
template <int BS>
__device__ __forceinline__ int block_exscan(int v, int* ws, int& total) {
    const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < BS / 64; w++) {
        const int c = ws[w];
        off += w < wv ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + incl - v;
}

// Occupancy words -> word prefix (pre) of the raster ranks; ends after a barrier.
__device__ __forceinline__ void occ_prefix(const uint32_t* occ, uint16_t* pre, int nw, int* ws) {
    constexpr int K = kPhWords / kPhBS;
    const int tid = (int)threadIdx.x;
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const int w = tid * K + q;
        cnt += w < nw ? __popc(occ[w]) : 0;
    }
    int tot;
    int off = block_exscan<kPhBS>(cnt, ws, tot);
#pragma unroll
    for (int q = 0; q < K; q++) {
        const int w = tid * K + q;
        if (w < nw) {
            pre[w] = (uint16_t)off;
            off += __popc(occ[w]);
        }
    }
    __syncthreads();
}

// The 2-bit map of occupancy bits occ (16 cells per output word).
__device__ __forceinline__ void write_state_map(const LearnArgs& a, const uint32_t* occ, uint32_t* out) {
    const int mw = (a.HW + 15) >> 4;
    for (int w = (int)threadIdx.x; w < mw; w += kPhBS)
        out[w] = state2(a.map2[w], (occ[w >> 1] >> ((w & 1) * 16)) & 0xFFFFu);
}

__global__ __launch_bounds__(kPhBS) void learn_phase_prep_kernel(LearnArgs a) {
    __shared__ uint32_t occ[kPhWords];
    __shared__ uint16_t pre[kPhWords];
    __shared__ int ws[kPhBS / 64];
    const long long e = blockIdx.x;
    const int tid = (int)threadIdx.x, HW = a.HW, A = a.A;
    const int nw = (HW + 31) >> 5, mw = (HW + 15) >> 4;
    const PhaseCarve pc = phase_carve(a.bph, a.E, HW, A);
    const int n = a.cnt[e];
    const uint16_t* pos = a.pos + e * A;
    for (int w = tid; w < nw; w += kPhBS) occ[w] = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += kPhBS) {
        const int c = pos[i];
        atomicOr(&occ[c >> 5], 1u << (c & 31));
    }
    __syncthreads();
    write_state_map(a, occ, pc.sm + e * mw);
    occ_prefix(occ, pre, nw, ws);
    uint16_t* rc = pc.rc + e * A;
    uint16_t* ri = pc.ri + e * A;
    for (int i = tid; i < n; i += kPhBS) {
        const int c = pos[i];
        const int r = cell_rank(occ, pre, c);
        rc[r] = (uint16_t)c;
        ri[r] = (uint16_t)i;
    }
    // the raster rank of the first agent of every tile (learn_batch_kernel's RASTER pass)
    uint16_t* ts = a.tstart + e * (a.NT + 1);
    for (int t = tid; t <= a.NT; t += kPhBS) {
        const int c = t * kTileCells;
        ts[t] = (uint16_t)(c < HW ? cell_rank(occ, pre, c) : n);
    }
}

// Decide / learn work units: the agents of one env in one row-chunk of kPhUnitTiles tiles
// (ranks from the records' tile offsets), one wave each, kPhWaves envs per workgroup.
// Unit u runs on XCD u % 8 for all envs back to back, so the table rows of its cells
// (slot = pattern * Q + cell) that many envs' agents read stay in that XCD's L2 -- in env
// order they were fetched from HBM once per env (C5: L2 hit rate 0.3).
constexpr int kPhUnitTiles = 64;      // 256 cells: one row at W = 256
constexpr int kPhWaves = kPhLanes / 64;

__device__ __forceinline__ bool phase_unit(const LearnArgs& a, long long& e, int& r0, int& r1) {
    const int NU = (a.NT + kPhUnitTiles - 1) / kPhUnitTiles;
    const unsigned EB = (unsigned)((a.E + kPhWaves - 1) / kPhWaves);
    const unsigned x = blockIdx.x & 7u, k = blockIdx.x >> 3;
    const int u = (int)(x + 8u * (k / EB));
    e = (long long)(k % EB) * kPhWaves + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    if (u >= NU || e >= a.E) return false;
    const int t0 = u * kPhUnitTiles, t1 = t0 + kPhUnitTiles < a.NT ? t0 + kPhUnitTiles : a.NT;
    const uint16_t* ts = a.tstart + e * (a.NT + 1);
    r0 = ts[t0];
    r1 = ts[t1];
    return true;
}

unsigned phase_unit_grid(const LearnArgs& a) {
    const unsigned NU = (unsigned)((a.NT + kPhUnitTiles - 1) / kPhUnitTiles);
    const unsigned EB = (unsigned)((a.E + kPhWaves - 1) / kPhWaves);
    return 8u * ((NU + 7u) / 8u) * EB;
}

__device__ __forceinline__ void phase_decide_one(const LearnArgs& a, long long e, int r);
__device__ __forceinline__ void phase_learn_one(const LearnArgs& a, long long e, int r);

__global__ __launch_bounds__(kPhLanes) void learn_phase_decide_kernel(LearnArgs a) {
    long long e;
    int r0, r1;
    if (!phase_unit(a, e, r0, r1)) return;
    for (int r = r0 + (int)(threadIdx.x & 63); r < r1; r += 64) phase_decide_one(a, e, r);
}

__global__ __launch_bounds__(kPhLanes) void learn_phase_learn_kernel(LearnArgs a) {
    long long e;
    int r0, r1;
    if (!phase_unit(a, e, r0, r1)) return;
    for (int r = r0 + (int)(threadIdx.x & 63); r < r1; r += 64) phase_learn_one(a, e, r);
}

// One agent (raster rank r of env e): learn_batch_kernel's decide phase (D = 1, UNI).
__device__ __forceinline__ void phase_decide_one(const LearnArgs& a, long long e, int r) {
    const int H = a.H, W = a.W, A = a.A;
    const PhaseCarve pc = phase_carve(a.bph, a.E, a.HW, A);
    const Sm2 sm{pc.sm + e * ((a.HW + 15) >> 4)};
    const uint32_t genv = (uint32_t)(a.env_base + e);
    const int c = pc.rc[e * A + r], i = pc.ri[e * A + r];
    const int x = fdiv(c, a.mW), y = c - x * W;
    const unsigned long long sk = enc_rank(sm, H, W, x, y, a.mBS);
    int coord[5], valid[5], inb[5], cls[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {      // moves5_grid on the state map and the class map
        const int nx = k < 4 ? x + kNBx[k] : x, ny = k < 4 ? y + kNBy[k] : y;
        inb[k] = nx >= 0 && nx < H && ny >= 0 && ny < W;
        coord[k] = inb[k] ? nx * W + ny : c;
        cls[k] = inb[k] ? map2_at(a.map2, coord[k]) : 2;
        const bool occupied = sm(coord[k]) == 1 && cls[k] != 1;
        valid[k] = inb[k] && (cls[k] == 0 || cls[k] == 3) && (k == 4 || !occupied);
    }
    valid[4] = 1;
    int ex = -1;
#pragma unroll
    for (int k = 3; k >= 0; k--) ex = inb[k] && cls[k] == 3 ? k : ex;
    int k;
    if (ex >= 0) {
        k = ex;
    } else {
        HStat hs;
        hs.has = (int)a.hstat[0];
        hs.nonfinite = (int)a.hstat[1];
        hs.mn = a.hstat[2];
        hs.mx = a.hstat[3];
        const double eps = env_epsilon(a, a.episodes[e], a.env_base + e);
        const int h = (int)dense_slot(sk, a.Ht);
        Policy P;
        actor_policy(a, tval(a.Ht, h), coord, valid, a.dff_in + e * (long long)a.HW, hs, false, P);
        dense_ensure(a.Ht, (uint32_t)h, sk);
        DrawPh rng(a, genv, (uint32_t)i);
        k = policy_draw(P, eps, rng);
    }
    pc.dec[e * A + r] = (uint32_t)coord[k] | ((uint32_t)(k + 1) << 16) | ((uint32_t)valid[k] << 19) |
                        ((ex >= 0 ? 1u : 0u) << 20);
}

// LDS of the resolve workgroup (dynamic): occupancy and next-cell bits, the word prefix,
// targets and agent indices by rank, next cells by agent index, scan words.
struct PhaseResolveCarve {
    size_t occ, nb, pre, rq, rx, nx, ws, total;
};
__host__ __device__ inline PhaseResolveCarve phase_resolve_carve(int HW, int A) {
    PhaseResolveCarve c;
    const size_t nw = (size_t)(HW + 31) / 32;
    size_t o = 0;
    c.occ = o; o += align16(nw * 4);
    c.nb = o; o += align16(nw * 4);
    c.pre = o; o += align16(nw * 2);
    c.rq = o; o += align16((size_t)A * 2);
    c.rx = o; o += align16((size_t)A * 2);
    c.nx = o; o += align16((size_t)A * 2);
    c.ws = o; o += 64;
    c.total = o;
    return c;
}

__global__ __launch_bounds__(kPhBS) void learn_phase_resolve_kernel(LearnArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const PhaseResolveCarve cv = phase_resolve_carve(a.HW, a.A);
    uint32_t* occ = reinterpret_cast<uint32_t*>(smem + cv.occ);
    uint32_t* nb = reinterpret_cast<uint32_t*>(smem + cv.nb);
    uint16_t* pre = reinterpret_cast<uint16_t*>(smem + cv.pre);
    uint16_t* rq = reinterpret_cast<uint16_t*>(smem + cv.rq);
    uint16_t* rx = reinterpret_cast<uint16_t*>(smem + cv.rx);
    uint16_t* nx = reinterpret_cast<uint16_t*>(smem + cv.nx);
    int* ws = reinterpret_cast<int*>(smem + cv.ws);
    const long long e = blockIdx.x;
    const int tid = (int)threadIdx.x, H = a.H, W = a.W, HW = a.HW, A = a.A;
    const int nw = (HW + 31) >> 5, mw = (HW + 15) >> 4;
    const PhaseCarve pc = phase_carve(a.bph, a.E, HW, A);
    const uint32_t genv = (uint32_t)(a.env_base + e);
    const int n = a.cnt[e];
    const uint16_t* rc = pc.rc + e * A;
    const uint32_t* dec = pc.dec + e * A;
    for (int w = tid; w < nw; w += kPhBS) { occ[w] = 0u; nb[w] = 0u; }
    __syncthreads();
    for (int r = tid; r < n; r += kPhBS) {
        const int c = rc[r];
        atomicOr(&occ[c >> 5], 1u << (c & 31));
        rq[r] = (uint16_t)(dec[r] & 0xFFFFu);
        rx[r] = pc.ri[e * A + r];
    }
    __syncthreads();
    occ_prefix(occ, pre, nw, ws);
    // learn_batch_kernel's resolve (D = 1): the requesters of T stand on it or next to it;
    // its owner is the smallest requesting agent index, whose stream draws the winner rank
    float* dff = a.dff_in + e * (long long)HW;
    for (int r = tid; r < n; r += kPhBS) {
        const int c = rc[r], i = rx[r];
        const uint32_t d = dec[r];
        const int T = (int)(d & 0xFFFFu);
        const int tx = fdiv(T, a.mW), ty = T - tx * W;
        int m = 0, owner = 0x7FFFFFFF, rank = 0;
#pragma unroll
        for (int c5 = 0; c5 < 5; c5++) {
            const int cx = c5 < 4 ? tx + kNBx[c5] : tx, cy = c5 < 4 ? ty + kNBy[c5] : ty;
            if (cx < 0 || cx >= H || cy < 0 || cy >= W) continue;
            const int cc = cx * W + cy;
            if (!((occ[cc >> 5] >> (cc & 31)) & 1u)) continue;
            const int b = cell_rank(occ, pre, cc);
            if (rq[b] != T) continue;
            const int ib = rx[b];
            m++;
            owner = ib < owner ? ib : owner;
            rank += ib < i ? 1 : 0;
        }
        int w = 0;
        if (m > 1) {
            PhiloxStream ps(a.key0, a.key1, a.t, genv, (uint32_t)owner, kPurFriction);
            w = (int)ps.randbelow((uint32_t)m);
        }
        const int clj = m == 1 ? 0 : m - 1;
        const bool won = rank == w;
        const int nxt = won ? T : c;
        if (won) {             // the winner's deposit on its own cell (distinct per agent)
            float v = dff[c];
            v = v + 1.0f;
            dff[c] = v;
        }
        const bool stays = map2_at(a.map2, nxt) != 3;
        if (stays) atomicOr(&nb[nxt >> 5], 1u << (nxt & 31));
        nx[i] = stays ? (uint16_t)nxt : kNone16;
        pc.res[e * A + r] = (uint32_t)nxt | ((uint32_t)(clj + 1) << 16) | (((d >> 16) & 31u) << 21);
    }
    __syncthreads();
    write_state_map(a, nb, pc.nm + e * mw);
    // exit removal in agent order (order preserving)
    int base_ = 0;
    for (int j = 0; j < (A + kPhBS - 1) / kPhBS; j++) {
        const int i = tid + j * kPhBS;
        const int c = i < n ? nx[i] : kNone16;
        const bool keep = c != kNone16;
        int tot;
        const int off = env_scan_flag<kPhBS, kPhBS>(keep, ws, tot);
        if (keep) a.pos[e * A + base_ + off] = (uint16_t)c;
        base_ += tot;
    }
    if (tid == 0) {
        a.cnt[e] = base_;
        a.nstart[e] = n;
        const int st = a.ep_steps[e] + 1;
        a.ep_steps[e] = st;
        a.done[e] = a.auto_reset && (base_ == 0 || (a.max_steps > 0 && st >= a.max_steps)) ? 1 : 0;
        unsigned long long* slot = a.counters + 4 * e;
        slot[0] += (unsigned long long)n;
        slot[1] += (unsigned long long)(n - base_);
        slot[3] += 1;
    }
}

// One agent: learn_batch_kernel's learn phase (TD error, record).
__device__ __forceinline__ void phase_learn_one(const LearnArgs& a, long long e, int r) {
    const int H = a.H, W = a.W, A = a.A;
    const PhaseCarve pc = phase_carve(a.bph, a.E, a.HW, A);
    const size_t mo = (size_t)e * ((a.HW + 15) >> 4);
    const Sm2 smc{pc.sm + mo}, smn{pc.nm + mo};
    const int c = pc.rc[e * A + r];
    const uint32_t rs = pc.res[e * A + r];
    const int nxt = (int)(rs & 0xFFFFu), coll = (int)((rs >> 16) & 31u) - 1;
    const int act = (int)((rs >> 21) & 7u) - 1, avalid = (int)((rs >> 24) & 1u), wexit = (int)((rs >> 25) & 1u);
    const int x = fdiv(c, a.mW);
    const unsigned long long skj = enc_rank(smc, H, W, x, c - x * W, a.mBS);
    double rw = a.step_penalty;
    if (wexit) rw = rw + a.exit_reward;
    if (coll >= 0) rw = rw + (double)coll * a.collision_penalty;
    int sn = -1;
    double vn = 0.0;
    if (!wexit) {
        const int qx = fdiv(nxt, a.mW);
        const unsigned long long nk = enc_rank(smn, H, W, qx, nxt - qx * W, a.mBS);
        sn = (int)dense_slot(nk, a.V);
        vn = tval(a.V, sn)[0];
        dense_ensure(a.V, (uint32_t)sn, nk);
    }
    const int sv = (int)dense_slot(skj, a.V);
    dense_ensure(a.V, (uint32_t)sv, skj);
    const double y = rw + a.gamma * vn;
    const double td = rec_target(a) ? y : y - tval(a.V, sv)[0];
    int kk = (int)kTileNoAct;
    if (act >= 0) {
        if (wexit) {           // exit-forced: decide made no H lookup, the learn step inserts s
            const uint32_t h = dense_slot(skj, a.Ht);
            dense_ensure(a.Ht, h, skj);
        }
        kk = avalid ? act : (int)kTileNoAct;
    }
    TileRec rc;
    rc.svk = (uint32_t)sv | ((uint32_t)kk << 28);
    rc.snf = (sn >= 0 ? (uint32_t)sn : kTileTerminal) | ((uint32_t)wexit << kTileExitBit) |
             ((uint32_t)(coll + 1) << kTileCollShift);
    rc.td = td;
    a.trecs[e * A + r] = rc;
}

// ===========================================================================
// Table upkeep.
// ===========================================================================
// Min / max / non-finite flag of the H values (the actor's global normalisation,
// model/ffm_unified.py:413-426), reduced per block into hpart[block][4].
__device__ __forceinline__ void hstat_block_reduce(double mn, double mx, int nf, uint32_t n, double* hpart,
                                                   unsigned bid = blockIdx.x) {
    __shared__ double smn[4], smx[4];
    __shared__ int snf[4];
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(mn, o), b2 = __shfl_xor(mx, o);
        mn = a2 < mn ? a2 : mn;
        mx = b2 > mx ? b2 : mx;
        nf |= __shfl_xor(nf, o);
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smn[wv] = mn; smx[wv] = mx; snf[wv] = nf; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) {
            mn = smn[w] < mn ? smn[w] : mn;
            mx = smx[w] > mx ? smx[w] : mx;
            nf |= snf[w];
        }
        double* o = hpart + bid * 4;
        o[0] = n > 0 ? 1.0 : 0.0;
        o[1] = (double)nf;
        o[2] = mn;
        o[3] = mx;
    }
}

__global__ __launch_bounds__(256) void learn_hstat_partial(LearnArgs a) {
    const uint32_t n = *a.Ht.n;
    double mn = __builtin_inf(), mx = -__builtin_inf();
    int nf = 0;
    const int w = (int)a.Ht.accw;      // H rows: 5 values, 9 with the Moore neighbourhood
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const double* v = tval(a.Ht, a.Ht.order[i]);
        for (int k = 0; k < w; k++) {
            nf |= !__builtin_isfinite(v[k]);
            mn = v[k] < mn ? v[k] : mn;
            mx = v[k] > mx ? v[k] : mx;
        }
    }
    hstat_block_reduce(mn, mx, nf, n, a.hpart);
}

__global__ __launch_bounds__(64) void learn_hstat_final(LearnArgs a, int nb) {
    double mn = __builtin_inf(), mx = -__builtin_inf();
    int nf = 0;
    for (int b = threadIdx.x; b < nb; b += 64) {
        const double* o = a.hpart + b * 4;
        mn = o[2] < mn ? o[2] : mn;
        mx = o[3] > mx ? o[3] : mx;
        nf |= o[1] != 0.0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(mn, o), b2 = __shfl_xor(mx, o);
        mn = a2 < mn ? a2 : mn;
        mx = b2 > mx ? b2 : mx;
        nf |= __shfl_xor(nf, o);
    }
    if (threadIdx.x == 0) {
        if (a.hx_n > 0) {      // ffm_trained_core rows held outside the table (ffm_learner_set_h_extra)
            mn = a.hx_mn < mn ? a.hx_mn : mn;
            mx = a.hx_mx > mx ? a.hx_mx : mx;
            nf |= a.hx_nf;
        }
        a.hstat[0] = *a.Ht.n > 0 || a.hx_n > 0 ? 1.0 : 0.0;
        a.hstat[1] = nf ? 1.0 : 0.0;
        a.hstat[2] = mn;
        a.hstat[3] = mx;
    }
}

// Apply the step's fixed-point increments once; for H also reduce the statistics
// the next step's actor reads (fusing the separate statistics pass).
// One table's apply as workgroup `bid` of `nblk` (learn_apply_kernel; learn_apply_vh_kernel
// runs V's and H's in one launch).
template <int WIDTH, bool STATS>
__device__ __forceinline__ void apply_hashed(const LearnTable& T, double* hpart, unsigned bid, unsigned nblk) {
    const uint32_t n = *T.n;
    // the next step's delta export reports entries inserted after this point
    if (bid == 0 && threadIdx.x == 0) *T.mark = n;
    double mn = __builtin_inf(), mx = -__builtin_inf();
    int nf = 0;
    for (uint32_t i = bid * 256 + threadIdx.x; i < n; i += nblk * 256) {
        const uint32_t slot = T.order[i];
        double* vp = tval(T, slot);
        if (WIDTH == 1) {   // V: visit-averaged
            long long qk[2];
            acc_take<2>(T, 2 * (size_t)slot, qk, true);
            if (qk[1] != 0) vp[0] = v_visits(vp[0], qk[0], qk[1], T.alpha);
            continue;
        }
        const size_t s = (size_t)slot * WIDTH;
        long long qa[WIDTH];
        acc_take<WIDTH>(T, s, qa, true);
#pragma unroll
        for (int k = 0; k < WIDTH; k++) {
            const long long q = qa[k];
            double v = vp[k];
            if (q != 0) {
                v = v + (double)q * (1.0 / kFxOne);
                vp[k] = v;
            }
            if (STATS) {
                nf |= !__builtin_isfinite(v);
                mn = v < mn ? v : mn;
                mx = v > mx ? v : mx;
            }
        }
    }
    if (STATS) hstat_block_reduce(mn, mx, nf, n, hpart, bid);
}

template <int WIDTH, bool STATS>
__global__ __launch_bounds__(256) void learn_apply_kernel(LearnTable T, double* hpart) {
    apply_hashed<WIDTH, STATS>(T, hpart, blockIdx.x, gridDim.x);
}

// Both hashed tables in one launch (their increments are independent): workgroups
// [0, nbv) apply V, the rest H with the statistics partials -- one dispatch fewer per step.
// Dense tables: the same pass in slot order over the presence bitmap.  Most
// slots of a long run are present, so streaming the records beats gathering
// them through the insertion order; min / max / non-finite do not depend on order.
template <int WIDTH, bool STATS>
__global__ __launch_bounds__(256) void learn_apply_dense_kernel(LearnTable T, double* hpart) {
    const uint32_t n = *T.n;
    if (blockIdx.x == 0 && threadIdx.x == 0) *T.mark = n;
    double mn = __builtin_inf(), mx = -__builtin_inf();
    int nf = 0;
    for (size_t slot = (size_t)blockIdx.x * 256 + threadIdx.x; slot <= T.mask; slot += (size_t)gridDim.x * 256) {
        // the record and accumulators are loaded with the presence word, not after it
        // (an absent slot holds the default and a zero accumulator)
        const bool pres = (T.present[slot >> 5] >> (slot & 31)) & 1u;
        double* vp = tval(T, slot);
        if (WIDTH == 1) {   // V: visit-averaged (an absent slot has no visits)
            const long long q = T.acc[2 * slot], k = T.acc[2 * slot + 1];
            if (k != 0) {
                vp[0] = v_visits(vp[0], q, k, T.alpha);
                T.acc[2 * slot] = 0;
                T.acc[2 * slot + 1] = 0;
            }
            continue;
        }
        const size_t s = slot * WIDTH;
        long long qa[WIDTH];
        double va[WIDTH];
#pragma unroll
        for (int k = 0; k < WIDTH; k++) { qa[k] = T.acc[s + k]; va[k] = vp[k]; }
        if (!pres) continue;
#pragma unroll
        for (int k = 0; k < WIDTH; k++) {
            const long long q = qa[k];
            double v = va[k];
            if (q != 0) {
                v = v + (double)q * (1.0 / kFxOne);
                vp[k] = v;
                T.acc[s + k] = 0;
            }
            if (STATS) {
                nf |= !__builtin_isfinite(v);
                mn = v < mn ? v : mn;
                mx = v > mx ? v : mx;
            }
        }
    }
    if (STATS) hstat_block_reduce(mn, mx, nf, n, hpart);
}

// _get_td_errors with the updated V, then the actor (model/ffm_unified.py:559-598).
// One lane per (env, agent) slot.
__global__ __launch_bounds__(256) void learn_post_kernel(LearnArgs a) {
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    if (g >= a.E * a.A) return;
    const long long e = g / a.A;
    const int i = (int)(g - e * a.A);
    if (i >= a.nstart[e]) return;
    const LearnRec rc = a.recs[g];
    if (rc.k < 0) return;
    const double vn = rc.snv >= 0 ? tval(a.V, rc.snv)[0] : 0.0;
    const double td = (rc.r + a.gamma * vn) - tval(a.V, rc.sv)[0];
    acc_add(acc_at(a.Ht, (size_t)rc.hslot * a.Ht.accw + rc.k), fx(a.alpha_h * td));
}

// ===========================================================================
// Tiled learning step (ffm_unified, dense tables, block size 1).
// Tile t = cells [4 t, 4 t + 4) owns the slots p * Q + c of those cells for every
// rank pattern p (Q = cap / 256), 1,024 slots.  One workgroup per tile reads the
// records of every env's agents on those cells (a contiguous raster range per env,
// learn_batch_kernel's tstart) and sums them in LDS: no atomic leaves the chip, and
// only touched slots are read and written.  The integer sums are those the
// accumulators held, so the tables equal the accumulator path's bit for bit.
// ===========================================================================
// 256 threads per tile, two per env: every env's record range of the tile is split
// between a thread pair.  Small tiles and workgroups keep several tiles resident per CU
// (H pass: 40 KB of LDS), so one tile's dependent loads overlap another's.
constexpr int kTileThreads = 256, kTileWaves = kTileThreads / 64;

__device__ __forceinline__ int tile_idx(uint32_t slot, int qsh, uint32_t Q, int c0) {
    return (int)(slot >> qsh) * kTileCells + (int)((slot & (Q - 1u)) - (uint32_t)c0);
}

// XCD-aware tile order: blocks b and b + 8 share an XCD (dealt round-robin), so block b
// takes tile (b % 8) * per + b / 8 and each XCD walks its own contiguous run of tiles.
// Adjacent tiles share the lines of tstart rows, record ranges and table rows; in one
// L2 those lines are fetched once instead of once per XCD.  Grid: 8 * per blocks.
__device__ __forceinline__ int tile_of_block(int NT) {
    const int per = (NT + 7) >> 3, b = (int)blockIdx.x;
    return (b & 7) * per + (b >> 3);
}

// Owner mode: launch tile k <-> tile t (LearnArgs ow / orank / ochunk).
__device__ __forceinline__ int own_tile(const LearnArgs& a, int k) {
    return a.ow <= 1 ? k : ((k / a.ochunk) * a.ow + a.orank) * a.ochunk + k % a.ochunk;
}
__device__ __forceinline__ int own_local(const LearnArgs& a, int t) {
    return a.ow <= 1 ? t : ((t / a.ochunk) / a.ow) * a.ochunk + t % a.ochunk;
}

// A launch's tiles: block -> (launch tile k, tile t); k >= the launch's tiles: nothing to do.
template <bool TM>
__device__ __forceinline__ void tile_of_launch(const LearnArgs& a, int& k, int& t) {
    k = tile_of_block(TM ? a.NTk : a.NT);
    t = TM ? own_tile(a, k) : k;
}
template <bool TM>
__device__ __forceinline__ int launch_tiles(const LearnArgs& a) { return TM ? a.NTk : a.NT; }

// Tile-major records: the ranges of launch tile k (wave 0, tR <= 64 lanes) -> rs[r] = records
// of the ranges before r (rs[tR] = the tile's total), rb[r] = first record of range r (the
// ranges' blocks lie back to back in trecs).
// Ends with a barrier.
__device__ __forceinline__ int tm_spans(const LearnArgs& a, int k, uint32_t* rs, uint32_t* rb) {
    if (threadIdx.x < 64) {
        const int r = (int)threadIdx.x;
        // range r's block starts after the blocks of the ranges before it (each header ends
        // with its block's record count)
        uint32_t lo = 0, n = 0, blk = 0;
        if (r < a.tR) {
            const uint32_t* h = a.thdr + (size_t)r * a.ths;
            lo = h[k];
            n = h[k + 1] - lo;
            blk = h[a.NTk];
            if (a.tblk > 0) {     // fixed-capacity blocks: range r at r * tblk, offsets past tblk clamped
                const uint32_t cap = (uint32_t)a.tblk, l0 = lo < cap ? lo : cap, l1 = h[k + 1] < cap ? h[k + 1] : cap;
                lo = l0;
                n = l1 - l0;
                blk = 0;
            }
        }
        uint32_t incl = n, bincl = blk;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, o), w = (uint32_t)__shfl_up((int)bincl, o);
            if (r >= o) {
                incl += v;
                bincl += w;
            }
        }
        lo += a.tblk > 0 ? (uint32_t)((long long)r * (a.tsrc > 0 ? a.tsrc : a.tblk)) : bincl - blk;
        if (r < a.tR) {
            rs[r + 1] = incl;
            rb[r] = lo;
        }
        if (r == 0) rs[0] = 0u;
    }
    __syncthreads();
    return (int)rs[a.tR];
}

// Record index of the tile's j-th record (rs / rb of tm_spans).
__device__ __forceinline__ uint32_t tm_index(const LearnArgs& a, const uint32_t* rs, const uint32_t* rb, uint32_t j) {
    int lo = 0, hi = a.tR;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (rs[mid] <= j) lo = mid;
        else hi = mid;
    }
    return rb[lo] + (j - rs[lo]);
}

// Block-aggregated append: every thread of the block calls it (uniformly) with P predicates;
// idx[i] = the output index of item i (-1 where p[i] is false).  One global atomic per block:
// a per-wave append on one counter would queue thousands of requests at one address.
// lw: kTileWaves + 1 words of LDS.  Ends with a barrier (lw reusable).
template <int P>
__device__ __forceinline__ void block_append(unsigned long long* ctr, const bool (&p)[P], int (&idx)[P], int* lw) {
    const int lane = (int)__lane_id(), w = (int)threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long m[P];
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < P; i++) {
        m[i] = __ballot(p[i]);
        cnt += __popcll(m[i]);
    }
    if (lane == 0) lw[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int v = 0; v < kTileWaves; v++) {
            const int c = lw[v];
            lw[v] = tot;
            tot += c;
        }
        lw[kTileWaves] = tot ? (int)atomicAdd(ctr, (unsigned long long)tot) : 0;
    }
    __syncthreads();
    int base = lw[kTileWaves] + lw[w];
#pragma unroll
    for (int i = 0; i < P; i++) {
        idx[i] = p[i] ? base + (int)__popcll(m[i] & lt) : -1;
        base += __popcll(m[i]);
    }
    __syncthreads();
}

// The updated V values of J slots (one per item; p: updated here).
template <int J>
__device__ __forceinline__ void vout_push(const LearnArgs& a, const bool (&p)[J], const uint32_t (&slot)[J],
                                          const double (&v)[J], int* lw) {
    if (!a.vout_n) return;
    int idx[J];
    block_append<J>(a.vout_n, p, idx, lw);
#pragma unroll
    for (int j = 0; j < J; j++)
        if (idx[j] >= 0) {
            if (idx[j] >= a.vout_cap) {       // capacity exceeded: reported at the next sync point
                atomicOr(a.overflow, 8);
                continue;
            }
            a.vout_slot[idx[j]] = slot[j];
            a.vout_val[idx[j]] = v[j];
        }
}

// Block-aggregated append of variable-size runs: n[i] items for run i of this thread;
// base[i] = the output index of the run's first item (runs of one thread's rows lie in
// order, every run contiguous).  Called uniformly by the block; lw: kTileWaves + 1 words.
template <int P>
__device__ __forceinline__ void block_append_runs(unsigned long long* ctr, const int (&n)[P], int (&base)[P], int* lw) {
    const int lane = (int)__lane_id(), w = (int)threadIdx.x >> 6;
    int tot = 0;
#pragma unroll
    for (int i = 0; i < P; i++) tot += n[i];
    int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) lw[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int v = 0; v < kTileWaves; v++) {
            const int c = lw[v];
            lw[v] = t;
            t += c;
        }
        lw[kTileWaves] = t ? (int)atomicAdd(ctr, (unsigned long long)t) : 0;
    }
    __syncthreads();
    int b = lw[kTileWaves] + lw[w] + incl - tot;
#pragma unroll
    for (int i = 0; i < P; i++) {
        base[i] = b;
        b += n[i];
    }
    __syncthreads();
}

// The nonzero H increments of the rows a thread applies go out with a row's increments
// adjacent (a receiver's updates of one row then share its record's line): the caller
// counts each row's nonzero increments (n[j]), hout_reserve gives every row its first
// output index (uniform call, block-aggregated), hout_row writes a row.  q is re-read
// per row by the caller, so no thread holds all its rows' sums at once.
template <int J>
__device__ __forceinline__ void hout_reserve(const LearnArgs& a, const int (&n)[J], int (&base)[J], int* lw) {
    if (!a.hout_n) return;
    block_append_runs<J>(a.hout_n, n, base, lw);
}

// nw: the row is new this step: its first entry carries kHoutNew (receivers insert the row),
// and a new row without increments still sends one (q = 0; hout_count counts it).
// NA: values per H row (5 Neumann, 9 Moore).
template <int NA>
__device__ __forceinline__ int hout_count(const long long (&q)[NA], bool nw) {
    int n = 0;
#pragma unroll
    for (int k = 0; k < NA; k++) n += q[k] != 0 ? 1 : 0;
    return n == 0 && nw ? 1 : n;
}

template <int NA>
__device__ __forceinline__ void hout_row(const LearnArgs& a, int base, uint32_t slot, const long long (&q)[NA],
                                         bool nw) {
    if (!a.hout_n) return;
    const int n = hout_count(q, nw);
    if (n == 0) return;
    if ((long long)base + n > a.hout_cap) {    // capacity exceeded: reported at the next sync point
        atomicOr(a.overflow, 8);
        return;
    }
    uint32_t flag = nw ? kHoutNew : 0u;
    bool any = false;
#pragma unroll
    for (int k = 0; k < NA; k++)
        if (q[k] != 0) {
            a.hout_key[base] = slot | ((uint32_t)k << kHoutActShift) | flag;
            a.hout_q[base] = q[k];
            base++;
            flag = 0u;
            any = true;
        }
    if (!any) {
        a.hout_key[base] = slot | kHoutNew;
        a.hout_q[base] = 0;
    }
}

constexpr int kTileEnvChunk = 2 * kTileThreads;   // envs whose ranges one pass gathers
constexpr int kTileList = 4 * kTileThreads;       // record indices per window

// Tile t's record ranges of envs [e0, e0 + 512): loaded together (two envs per thread),
// and a block scan gives each thread the offset of its records in one flat list and the
// block the total.  Ends with a barrier (wsum read); the caller syncs before reusing wsum.
struct TileRanges {
    int lo[2], n[2], off, total;
};

__device__ __forceinline__ TileRanges tile_ranges(const LearnArgs& a, int t, long long e0, int* wsum) {
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    TileRanges r;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const long long e = e0 + tid + j * kTileThreads;
        r.lo[j] = 0;
        r.n[j] = 0;
        if (e < a.E) {
            if (a.tstartT) {       // tile-major offsets: the block's loads are contiguous
                r.lo[j] = a.tstartT[(long long)t * a.E + e];
                r.n[j] = a.tstartT[(long long)(t + 1) * a.E + e] - r.lo[j];
            } else {
                const uint16_t* ts = a.tstart + e * (a.NT + 1) + t;
                r.lo[j] = ts[0];
                r.n[j] = ts[1] - r.lo[j];
            }
        }
    }
    const int c = r.n[0] + r.n[1];
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    r.off = incl - c;
    r.total = 0;
#pragma unroll
    for (int w = 0; w < kTileWaves; w++) {
        r.off += w < wv ? wsum[w] : 0;
        r.total += wsum[w];
    }
    return r;
}

// Window [b, b + kTileList) of the flat list: the record indices (into trecs).
__device__ __forceinline__ void tile_fill(const LearnArgs& a, long long e0, const TileRanges& r, int b,
                                          uint32_t* list) {
    const int tid = (int)threadIdx.x;
    int o = r.off - b;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const uint32_t g0 = (uint32_t)((e0 + tid + j * kTileThreads) * a.A + r.lo[j]);
        for (int i = 0; i < r.n[j]; i++, o++)
            if (o >= 0 && o < kTileList) list[o] = g0 + (uint32_t)i;
    }
}

// Calls f(g) for every record g of tile t's cells, dealt evenly over the threads: one
// dependent chain (range, record, table reads) per record instead of one per env in turn.
template <bool TM, typename F>
__device__ __forceinline__ void tile_records(const LearnArgs& a, int t, int k, uint32_t* list, int* wsum,
                                             uint32_t* rs, uint32_t* rb, F f) {
    const int tid = (int)threadIdx.x;
    if (TM) {       // tile-major: the tile's records are the ranges' runs
        const int total = tm_spans(a, k, rs, rb);
        for (int b = 0; b < total; b += kTileList) {
            const int m = total - b < kTileList ? total - b : kTileList;
            for (int i = tid; i < m; i += kTileThreads) list[i] = tm_index(a, rs, rb, (uint32_t)(b + i));
            __syncthreads();
            for (int i = tid; i < m; i += kTileThreads) f(list[i]);
            __syncthreads();
        }
        return;
    }
    for (long long e0 = 0; e0 < a.E; e0 += kTileEnvChunk) {
        const TileRanges r = tile_ranges(a, t, e0, wsum);
        for (int b = 0; b < r.total; b += kTileList) {
            tile_fill(a, e0, r, b, list);
            __syncthreads();
            const int m = r.total - b < kTileList ? r.total - b : kTileList;
            for (int i = tid; i < m; i += kTileThreads) f(list[i]);
            __syncthreads();
        }
        __syncthreads();    // wsum is rewritten by the next pass
    }
}

// The fast form of a tile pass: every record of the tile in one window (at most 512 envs,
// at most kTileList records, the common case).  Each thread then holds up to J records
// at once; the first record of a slot (its "owner", elected by an LDS atomic) loads the
// slot's table row together with the others' table reads, and applies it after the
// barrier from registers: range, record, (table reads), apply -- three dependent steps.
// Returns the window's record count, or -1 (the caller takes tile_records; no barrier
// owed).
constexpr int kTileJ = kTileList / kTileThreads;

template <bool TM>
__device__ __forceinline__ int tile_window(const LearnArgs& a, int t, int k, uint32_t* list, int* wsum, uint32_t* rs,
                                           uint32_t* rb) {
    if (TM) {       // tile-major: any number of envs, only the tile's record count matters
        const int total = tm_spans(a, k, rs, rb);
        if (total > kTileList) return -1;
        for (int j = (int)threadIdx.x; j < total; j += kTileThreads) list[j] = tm_index(a, rs, rb, (uint32_t)j);
        __syncthreads();
        return total;
    }
    if (a.E > kTileEnvChunk) return -1;
    const TileRanges r = tile_ranges(a, t, 0, wsum);
    if (r.total > kTileList) {
        __syncthreads();
        return -1;
    }
    tile_fill(a, 0, r, 0, list);
    __syncthreads();
    return r.total;
}

// Tile-major, a tile beyond one window: window b's records, kTileJ per thread, every load in
// flight before the first is used (rs / rb of tm_spans).  Returns the window's record count.
__device__ __forceinline__ int tm_load(const LearnArgs& a, const uint32_t* rs, const uint32_t* rb, int total, int b,
                                       TileRec (&rc)[kTileJ]) {
    const int tid = (int)threadIdx.x;
    const int m = total - b < kTileList ? total - b : kTileList;
#pragma unroll
    for (int j = 0; j < kTileJ; j++)
        if (tid + j * kTileThreads < m) rc[j] = a.trecs[tm_index(a, rs, rb, (uint32_t)(b + tid + j * kTileThreads))];
    return m;
}

// The rank key of a dense slot (inverse of dense_slot): ranks in bits 0-7, bx, by.
__device__ __forceinline__ unsigned long long dense_key(uint32_t slot, int qsh, uint32_t Q, uint32_t by) {
    const uint32_t b = slot & (Q - 1u);
    return (unsigned long long)(slot >> qsh) | ((unsigned long long)(b / by) << 26) |
           ((unsigned long long)(b % by) << 45);
}

// V: visit-averaged TD(0) of every touched state (learn_apply_dense_kernel's update).
#ifndef FFM_TILE_V_WAVES
#define FFM_TILE_V_WAVES 8   // 106 -> 78 SGPRs, occupancy 7 -> 8: config-5 step 767 -> 764 us in A/B
#endif

template <bool TM>
__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(FFM_TILE_V_WAVES, 8)))
void learn_tile_v_kernel(LearnArgs a) {
    constexpr int NS = 256 * kTileCells;
    __shared__ long long qs[NS];
    __shared__ uint32_t ks[NS];
    __shared__ uint32_t list[kTileList];
    __shared__ int wsum[kTileWaves + 1];
    __shared__ uint32_t rs[kMaxOwners + 1], rb[kMaxOwners];
    const int tid = (int)threadIdx.x;
    int k, t;
    tile_of_launch<TM>(a, k, t);
    if (blockIdx.x == 0 && tid == 0) a.tcand[0] = 0;    // the H pass's queue of wide tiles
    if (k >= launch_tiles<TM>(a)) return;
    // (tile_window / tile_records pass a barrier -- tm_spans', tile_ranges' -- before any
    // use of these)
    for (int i = tid; i < NS; i += kTileThreads) { qs[i] = 0; ks[i] = 0u; }
    const uint32_t Q = (a.V.mask + 1u) >> 8;
    const int qsh = __builtin_ctz(Q), c0 = t * kTileCells;
    // the record's td (rec_target: the target, minus V(s) at step start, read before any
    // store of this pass)
    const bool tgt = rec_target(a);
    auto add = [&](const TileRec& rc, uint32_t sv, int idx, double vs) {
        const double td = tgt ? rc.td - vs : rc.td;
        atomicAdd(reinterpret_cast<unsigned long long*>(&qs[idx]), (unsigned long long)fx(td));
        if (a.tile_ensure) {     // another rank's agent: its s and s' join this rank's V
            dense_ensure(a.V, sv, dense_key(sv, qsh, Q, a.V.dense_by));
            const uint32_t sn = rc.snf & kTileSlot;
            if (sn != kTileTerminal) dense_ensure(a.V, sn, dense_key(sn, qsh, Q, a.V.dense_by));
        }
    };
    const int m = tile_window<TM>(a, t, k, list, wsum, rs, rb);
    if (m >= 0) {
        TileRec rc[kTileJ];
#pragma unroll
        for (int j = 0; j < kTileJ; j++)
            if (tid + j * kTileThreads < m) rc[j] = a.trecs[list[tid + j * kTileThreads]];
        bool own[kTileJ];
        double vv[kTileJ];
        int ix[kTileJ];
#pragma unroll
        for (int j = 0; j < kTileJ; j++) {
            own[j] = false;
            if (tid + j * kTileThreads >= m) continue;
            const uint32_t sv = rc[j].svk & kTileSlot;
            ix[j] = tile_idx(sv, qsh, Q, c0);
            own[j] = atomicAdd(&ks[ix[j]], 1u) == 0u;
            const double vs = tgt || own[j] ? tval(a.V, sv)[0] : 0.0;
            if (own[j]) vv[j] = vs;
            add(rc[j], sv, ix[j], vs);
        }
        __syncthreads();
        double nv[kTileJ];
        uint32_t sl[kTileJ];
#pragma unroll
        for (int j = 0; j < kTileJ; j++) {
            nv[j] = 0.0;
            sl[j] = rc[j].svk & kTileSlot;
            if (own[j]) {
                nv[j] = v_visits(vv[j], qs[ix[j]], (long long)ks[ix[j]], a.V.alpha);
                tval(a.V, sl[j])[0] = nv[j];
            }
        }
        if (TM) vout_push<kTileJ>(a, own, sl, nv, wsum);
        return;
    }
    if (TM) {           // tile-major (tile_window left the spans in rs / rb)
        const int total = (int)rs[a.tR];
        for (int b = 0; b < total; b += kTileList) {
            TileRec rc[kTileJ];
            const int mw = tm_load(a, rs, rb, total, b, rc);
#pragma unroll
            for (int j = 0; j < kTileJ; j++) {
                if (tid + j * kTileThreads >= mw) continue;
                const uint32_t sv = rc[j].svk & kTileSlot;
                const int idx = tile_idx(sv, qsh, Q, c0);
                atomicAdd(&ks[idx], 1u);
                add(rc[j], sv, idx, tgt ? tval(a.V, sv)[0] : 0.0);
            }
        }
        __syncthreads();
    } else {
        tile_records<TM>(a, t, k, list, wsum, rs, rb, [&](uint32_t g) {
            const TileRec rc = a.trecs[g];
            const uint32_t sv = rc.svk & kTileSlot;
            const int idx = tile_idx(sv, qsh, Q, c0);
            atomicAdd(&ks[idx], 1u);
            add(rc, sv, idx, tgt ? tval(a.V, sv)[0] : 0.0);
        });
    }
    constexpr int kPer = NS / kTileThreads;
    double vv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {    // the loads first (one latency, not four)
        const int i = tid + j * kTileThreads;
        if (ks[i]) vv[j] = tval(a.V, (size_t)(i / kTileCells) * Q + (size_t)(c0 + i % kTileCells))[0];
    }
    bool up[kPer];
    uint32_t sl[kPer];
    double nv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        const int i = tid + j * kTileThreads;
        const uint32_t kv = ks[i];
        sl[j] = (uint32_t)((size_t)(i / kTileCells) * Q + (size_t)(c0 + i % kTileCells));
        up[j] = kv != 0u;
        nv[j] = 0.0;
        if (kv) {
            nv[j] = v_visits(vv[j], qs[i], (long long)kv, a.V.alpha);
            tval(a.V, sl[j])[0] = nv[j];
        }
    }
    if (TM) vout_push<kPer>(a, up, sl, nv, wsum);
}

// Exact min / max / non-finite of one tile's present H rows (a block-wide scan).
template <int NA>
__device__ void tile_rescan(const LearnArgs& a, int t, double* smn, double* smx, int* sfl) {
    constexpr int NS = 256 * kTileCells;
    const int tid = (int)threadIdx.x, wv = tid >> 6;
    const uint32_t Q = (a.Ht.mask + 1u) >> 8;
    const int c0 = t * kTileCells;
    int nf = 0, any = 0;
    double mn = __builtin_inf(), mx = -__builtin_inf();
    for (int i = tid; i < NS; i += kTileThreads) {
        const size_t slot = (size_t)(i / kTileCells) * Q + (size_t)(c0 + i % kTileCells);
        if (!((a.Ht.present[slot >> 5] >> (slot & 31)) & 1u)) continue;
        any = 1;
        const double* vp = tval(a.Ht, slot);
#pragma unroll
        for (int k = 0; k < NA; k++) {
            const double v = vp[k];
            nf |= !__builtin_isfinite(v);
            mn = v < mn ? v : mn;
            mx = v > mx ? v : mx;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(mn, o), b2 = __shfl_xor(mx, o);
        mn = a2 < mn ? a2 : mn;
        mx = b2 > mx ? b2 : mx;
        nf |= __shfl_xor(nf, o);
        any |= __shfl_xor(any, o);
    }
    __syncthreads();
    if ((tid & 63) == 0) { smn[wv] = mn; smx[wv] = mx; sfl[wv] = nf | (any << 1); }
    __syncthreads();
    if (tid == 0) {
        int f = 0;
        for (int w = 0; w < kTileWaves; w++) {
            mn = smn[w] < mn ? smn[w] : mn;
            mx = smx[w] > mx ? smx[w] : mx;
            f |= sfl[w];
        }
        double* ts = a.tstats + 4 * t;
        ts[0] = (f & 2) ? 1.0 : 0.0;
        ts[1] = (f & 1) ? 1.0 : 0.0;
        ts[2] = mn;
        ts[3] = mx;
        a.tdirty[t] = 0;
    }
}

// H: the actor increments (actor_only: the TD error with the updated V, like
// learn_post_kernel; both: the step's td), applied at once, and the tile's summary of
// the H statistics (present, non-finite, min, max) for the next step.  The summary is
// widened by the touched rows' new values; when a touched value held the tile's min or
// max and moved inward, the old extreme stays as a bound and the tile is marked stale
// (tdirty): learn_tile_cand_kernel rescans only the stale tiles whose bound could
// decide the table's min or max.
//
// Pieces shared by the two forms of the H pass:
struct TileHCtx {
    double omn, omx;                    // the tile's summary at step start
    bool onf;
    int flags;                          // 1 non-finite, 2 max stale, 4 any row, 8 min stale, 16 nf stale
    double mn, mx;                      // over the touched rows' new values
};

// The V values the actor's td reads (actor_only: updated by learn_tile_v_kernel).
__device__ __forceinline__ void tile_h_vpair(const LearnArgs& a, const TileRec& rc, uint32_t sv, double& vn,
                                             double& vs) {
    vn = 0.0;
    vs = 0.0;
    if (a.mode != kModeActor || (rc.svk >> 28) == kTileNoAct) return;
    const uint32_t sn = rc.snf & kTileSlot;
    if (sn != kTileTerminal) vn = tval(a.V, sn)[0];
    vs = tval(a.V, sv)[0];
}

// The fixed-point increment alpha_h * td of one record (an action taken).
__device__ __forceinline__ long long tile_h_q(const LearnArgs& a, const TileRec& rc, double vn, double vs) {
    double td = rc.td;
    if (a.mode == kModeActor) {     // _get_td_errors with the updated V (model/ffm_unified.py:568-574)
        double r0 = a.step_penalty;
        if ((rc.snf >> kTileExitBit) & 1u) r0 = r0 + a.exit_reward;
        const int coll = (int)(rc.snf >> kTileCollShift) - 1;
        if (coll >= 0) r0 = r0 + (double)coll * a.collision_penalty;
        td = (r0 + a.gamma * vn) - vs;
    }
    return fx(a.alpha_h * td);
}

// A touched row: new values, the summary's bounds and staleness.
template <int NA>
__device__ __forceinline__ void tile_h_apply(double* vp, const long long (&q)[NA], const double* oldv, TileHCtx& c) {
    c.flags |= 4;
#pragma unroll
    for (int k = 0; k < NA; k++) {
        const double old = oldv[k];
        double v = old;
        if (q[k] != 0) {
            v = v + (double)q[k] * (1.0 / kFxOne);
            vp[k] = v;
            if (old == c.omx && !(v >= old)) c.flags |= 2;    // the max moved inward (or to NaN)
            if (old == c.omn && !(v <= old)) c.flags |= 8;
            if (!__builtin_isfinite(old)) c.flags |= 16;
        }
        c.flags |= __builtin_isfinite(v) ? 0 : 1;
        c.mn = v < c.mn ? v : c.mn;
        c.mx = v > c.mx ? v : c.mx;
    }
}

__device__ __forceinline__ TileHCtx tile_h_begin(const LearnArgs& a, int t) {
    const double* ts = a.tstats + 4 * t;
    TileHCtx c;
    c.omn = ts[2];
    c.omx = ts[3];
    c.onf = ts[1] != 0.0;
    c.flags = 0;
    c.mn = __builtin_inf();
    c.mx = -__builtin_inf();
    return c;
}

// The block's summary of tile t (ends with a barrier: smn / smx / sfl are free again).
__device__ __forceinline__ void tile_h_end(const LearnArgs& a, int t, TileHCtx& c, double* smn, double* smx,
                                           int* sfl) {
    const int tid = (int)threadIdx.x;
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(c.mn, o), b2 = __shfl_xor(c.mx, o);
        c.mn = a2 < c.mn ? a2 : c.mn;
        c.mx = b2 > c.mx ? b2 : c.mx;
        c.flags |= __shfl_xor(c.flags, o);
    }
    const int wv = tid >> 6;
    if ((tid & 63) == 0) { smn[wv] = c.mn; smx[wv] = c.mx; sfl[wv] = c.flags; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kTileWaves; w++) {
            c.mn = smn[w] < c.mn ? smn[w] : c.mn;
            c.mx = smx[w] > c.mx ? smx[w] : c.mx;
            c.flags |= sfl[w];
        }
        // the old extremes stay as bounds (a value that left them is only inward)
        double* ts = a.tstats + 4 * t;
        ts[0] = (ts[0] != 0.0 || (c.flags & 4)) ? 1.0 : 0.0;
        ts[1] = (c.onf || (c.flags & 1)) ? 1.0 : 0.0;
        ts[2] = c.omn < c.mn ? c.omn : c.mn;
        ts[3] = c.omx > c.mx ? c.omx : c.mx;
        a.tdirty[t] |= ((c.flags & 2) ? 1 : 0) | ((c.flags & 8) ? 2 : 0) | ((c.flags & 16) ? 4 : 0);
    }
    __syncthreads();
}

// The fast form: every record of the tile in one window (tile_window), at most
// kTileList records, so at most kTileList (slot, action) pairs are touched.  The sums
// live in one fixed-point word per touched pair, found through a pair -> index map:
// 23 KB of LDS instead of 40 KB for every pair of the tile, so six workgroups share a
// CU (the LDS limit) instead of three, and their dependent loads overlap.
//   1. per record: the slot's first record is its owner (an LDS bit), the pair's first
//      record takes an index (wave-aggregated counter), V reads in flight;
//   2. (barrier) every record adds its increment into its pair's word;
//   3. (barrier) owners read their rows and apply them.
// A tile whose records need more than one window is queued (tcand, count reset by
// learn_tile_v_kernel) for learn_tile_h_wide_kernel.
// (slot, action) pairs of a tile: 256 * kTileCells rows of NA values
template <int NA>
constexpr int tile_pairs() { return 256 * kTileCells * NA; }

#ifndef FFM_TILE_H_WAVES
#define FFM_TILE_H_WAVES 1
#endif

template <bool TM, int NA>
__global__ __launch_bounds__(kTileThreads) __attribute__((amdgpu_waves_per_eu(FFM_TILE_H_WAVES, 8)))
void learn_tile_h_kernel(LearnArgs a) {
    constexpr int NS = 256 * kTileCells, kTilePairs = tile_pairs<NA>();
    static_assert(kTileList * 4 <= kTilePairs * 2, "the window's list fits the pair map");
    __shared__ long long hq[kTileList];             // per touched (slot, action) pair
    // pair -> index into hq (valid where pbit is set); until the records are loaded, the
    // window's record list (tile_window) -- one region, 19 KB of LDS per workgroup
    __shared__ uint32_t pidl[kTilePairs / 2];
    uint16_t* const pid = reinterpret_cast<uint16_t*>(pidl);
    uint32_t* const list = pidl;
    __shared__ uint32_t pbit[kTilePairs / 32];
    __shared__ uint32_t touched[NS / 32];
    __shared__ uint32_t newb[NS / 32];               // rows another rank's step inserted (kTileNewH)
    __shared__ double smn[kTileWaves], smx[kTileWaves];
    __shared__ int sfl[kTileWaves];
    __shared__ int wsum[kTileWaves + 1];
    __shared__ uint32_t rs[kMaxOwners + 1], rb[kMaxOwners];
    __shared__ int npair;
    const int tid = (int)threadIdx.x, lane = tid & 63;
    int k, t;
    tile_of_launch<TM>(a, k, t);
    if (k >= launch_tiles<TM>(a)) return;
    const uint32_t Q = (a.Ht.mask + 1u) >> 8;
    const int qsh = __builtin_ctz(Q), c0 = t * kTileCells;
    for (int i = tid; i < kTileList; i += kTileThreads) hq[i] = 0;
    for (int i = tid; i < kTilePairs / 32; i += kTileThreads) pbit[i] = 0u;
    if (tid < NS / 32) {
        touched[tid] = 0u;
        newb[tid] = 0u;
    }
    if (tid == 0) npair = 0;
    // (tile_window's barriers order these stores before any use)
    const int m = tile_window<TM>(a, t, k, list, wsum, rs, rb);
    if (m < 0) {
        if (tid == 0) a.tcand[1 + atomicAdd(&a.tcand[0], 1)] = t;
        return;
    }
    TileHCtx c = tile_h_begin(a, t);
    TileRec rc[kTileJ];
#pragma unroll
    for (int j = 0; j < kTileJ; j++)
        if (tid + j * kTileThreads < m) rc[j] = a.trecs[list[tid + j * kTileThreads]];
    __syncthreads();                        // the list is read: its LDS becomes the pair map
    bool own[kTileJ], pown[kTileJ];
    int ix[kTileJ], pr[kTileJ];
    double hv[kTileJ][NA], vn[kTileJ], vs[kTileJ];
#pragma unroll
    for (int j = 0; j < kTileJ; j++) {     // owners' rows and the V reads, all in flight
        own[j] = false;
        pown[j] = false;
        pr[j] = -1;
        if (tid + j * kTileThreads >= m) continue;
        const uint32_t sv = rc[j].svk & kTileSlot;
        ix[j] = tile_idx(sv, qsh, Q, c0);
        const uint32_t bit = 1u << (ix[j] & 31);
        own[j] = !(atomicOr(&touched[ix[j] >> 5], bit) & bit);
        if (rc[j].svk & kTileNewH) atomicOr(&newb[ix[j] >> 5], bit);
        tile_h_vpair(a, rc[j], sv, vn[j], vs[j]);
        if (a.tile_ensure) dense_ensure(a.Ht, sv, dense_key(sv, qsh, Q, a.Ht.dense_by));
        const int act = (int)(rc[j].svk >> 28);
        if (act != (int)kTileNoAct) {
            pr[j] = ix[j] * NA + act;
            const uint32_t pb = 1u << (pr[j] & 31);
            pown[j] = !(atomicOr(&pbit[pr[j] >> 5], pb) & pb);
        }
    }
#pragma unroll
    for (int j = 0; j < kTileJ; j++) {     // pair owners take consecutive indices, one atomic per wave
        const unsigned long long bm = __ballot(pown[j]);
        if (!bm) continue;
        int base = 0;
        if (lane == 0) base = atomicAdd(&npair, __popcll(bm));
        base = __shfl(base, 0);
        if (pown[j]) pid[pr[j]] = (uint16_t)(base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)));
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kTileJ; j++)
        if (pr[j] >= 0)
            atomicAdd(reinterpret_cast<unsigned long long*>(&hq[pid[pr[j]]]),
                      (unsigned long long)tile_h_q(a, rc[j], vn[j], vs[j]));
    __syncthreads();
    // the owners' rows are read only now: with no row held across the sums the pass
    // needs 70 VGPRs instead of 98, and six workgroups share a CU instead of five
#pragma unroll
    for (int j = 0; j < kTileJ; j++) {
        if (!own[j]) continue;
        const double* vp = tval(a.Ht, rc[j].svk & kTileSlot);
#pragma unroll
        for (int k = 0; k < NA; k++) hv[j][k] = vp[k];
    }
    auto row_q = [&](int j, long long (&q)[NA]) {
#pragma unroll
        for (int kk = 0; kk < NA; kk++) {
            const int p = ix[j] * NA + kk;
            q[kk] = ((pbit[p >> 5] >> (p & 31)) & 1u) ? hq[pid[p]] : 0;
        }
    };
    int hn[kTileJ], hb[kTileJ];
    bool nw[kTileJ];
#pragma unroll
    for (int j = 0; j < kTileJ; j++) {     // owner mode: each row's nonzero increments, reserved
        hn[j] = 0;
        nw[j] = false;
        if (!own[j]) continue;
        // a row another rank's step inserted joins this rank's table here, and goes out flagged
        nw[j] = TM && ((newb[ix[j] >> 5] >> (ix[j] & 31)) & 1u);
        if (TM && a.hout_n) {
            long long q[NA];
            row_q(j, q);
            hn[j] = hout_count(q, nw[j]);
        }
    }
    if (TM) hout_reserve<kTileJ>(a, hn, hb, wsum);
#pragma unroll
    for (int j = 0; j < kTileJ; j++) {
        if (!own[j]) continue;
        long long q[NA];
        row_q(j, q);
        const uint32_t sl = rc[j].svk & kTileSlot;
        if (nw[j]) dense_ensure(a.Ht, sl, dense_key(sl, qsh, Q, a.Ht.dense_by));
        tile_h_apply(tval(a.Ht, sl), q, hv[j], c);
        if (TM) hout_row(a, hb[j], sl, q, nw[j]);
    }
    tile_h_end(a, t, c, smn, smx, sfl);
}

// The general form, for the tiles the fast form queued (more than one window of
// records: a crowded tile, or more than 512 envs): every (slot, action) pair of the
// tile has its word (40 KB), records stream through windows, then the touched rows.
template <bool TM, int NA>
__global__ __launch_bounds__(kTileThreads) void learn_tile_h_wide_kernel(LearnArgs a) {
    constexpr int NS = 256 * kTileCells;
    __shared__ long long hq[NS * NA];
    __shared__ uint32_t touched[NS / 32];
    __shared__ uint32_t newb[NS / 32];
    __shared__ double smn[kTileWaves], smx[kTileWaves];
    __shared__ int sfl[kTileWaves];
    __shared__ uint32_t list[kTileList];
    __shared__ int wsum[kTileWaves + 1];
    __shared__ uint32_t rs[kMaxOwners + 1], rb[kMaxOwners];
    const int tid = (int)threadIdx.x;
    const uint32_t Q = (a.Ht.mask + 1u) >> 8;
    const int qsh = __builtin_ctz(Q);
    const int n = a.tcand[0];
    for (int ci = (int)blockIdx.x; ci < n; ci += (int)gridDim.x) {
        const int t = a.tcand[1 + ci], c0 = t * kTileCells, kt = TM ? own_local(a, t) : t;
        for (int i = tid; i < NS * NA; i += kTileThreads) hq[i] = 0;
        for (int i = tid; i < NS / 32; i += kTileThreads) {
            touched[i] = 0u;
            newb[i] = 0u;
        }
        __syncthreads();
        TileHCtx c = tile_h_begin(a, t);
        if (TM) {           // tile-major: windows of kTileJ records per thread, the loads first
            const int total = tm_spans(a, kt, rs, rb);
            for (int b = 0; b < total; b += kTileList) {
                TileRec rc[kTileJ];
                const int mw = tm_load(a, rs, rb, total, b, rc);
                double vn[kTileJ], vs[kTileJ];
#pragma unroll
                for (int j = 0; j < kTileJ; j++)
                    if (tid + j * kTileThreads < mw) tile_h_vpair(a, rc[j], rc[j].svk & kTileSlot, vn[j], vs[j]);
#pragma unroll
                for (int j = 0; j < kTileJ; j++) {
                    if (tid + j * kTileThreads >= mw) continue;
                    const int idx = tile_idx(rc[j].svk & kTileSlot, qsh, Q, c0);
                    atomicOr(&touched[idx >> 5], 1u << (idx & 31));
                    if (rc[j].svk & kTileNewH) atomicOr(&newb[idx >> 5], 1u << (idx & 31));
                    const int act = (int)(rc[j].svk >> 28);
                    if (act == (int)kTileNoAct) continue;
                    atomicAdd(reinterpret_cast<unsigned long long*>(&hq[idx * NA + act]),
                              (unsigned long long)tile_h_q(a, rc[j], vn[j], vs[j]));
                }
            }
            __syncthreads();
        } else {
            tile_records<TM>(a, t, kt, list, wsum, rs, rb, [&](uint32_t g) {
                const TileRec rc = a.trecs[g];
                const uint32_t sv = rc.svk & kTileSlot;
                const int idx = tile_idx(sv, qsh, Q, c0);
                atomicOr(&touched[idx >> 5], 1u << (idx & 31));
                if (a.tile_ensure) dense_ensure(a.Ht, sv, dense_key(sv, qsh, Q, a.Ht.dense_by));
                const int act = (int)(rc.svk >> 28);
                if (act == (int)kTileNoAct) return;
                double vn, vs;
                tile_h_vpair(a, rc, sv, vn, vs);
                atomicAdd(reinterpret_cast<unsigned long long*>(&hq[idx * NA + act]),
                          (unsigned long long)tile_h_q(a, rc, vn, vs));
            });
        }
        // every touched row's loads are issued before the first is used (one latency, not four)
        constexpr int kPer = NS / kTileThreads;
        double hv[kPer][NA];
        bool tch[kPer];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const int i = tid + j * kTileThreads;
            tch[j] = (touched[i >> 5] >> (i & 31)) & 1u;
            if (tch[j]) {
                const double* vp = tval(a.Ht, (size_t)(i / kTileCells) * Q + (size_t)(c0 + i % kTileCells));
#pragma unroll
                for (int k = 0; k < NA; k++) hv[j][k] = vp[k];
            }
        }
        int hn[kPer], hb[kPer];
        bool nw[kPer];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const int i = tid + j * kTileThreads;
            hn[j] = 0;
            nw[j] = TM && tch[j] && ((newb[i >> 5] >> (i & 31)) & 1u);
            if (TM && a.hout_n && tch[j]) {
                long long q[NA];
#pragma unroll
                for (int kk = 0; kk < NA; kk++) q[kk] = hq[i * NA + kk];
                hn[j] = hout_count(q, nw[j]);
            }
        }
        if (TM) hout_reserve<kPer>(a, hn, hb, wsum);
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const int i = tid + j * kTileThreads;
            if (!tch[j]) continue;
            const uint32_t sl = (uint32_t)((size_t)(i / kTileCells) * Q + (size_t)(c0 + i % kTileCells));
            long long q[NA];
#pragma unroll
            for (int kk = 0; kk < NA; kk++) q[kk] = hq[i * NA + kk];
            if (nw[j]) dense_ensure(a.Ht, sl, dense_key(sl, qsh, Q, a.Ht.dense_by));
            tile_h_apply(tval(a.Ht, sl), q, hv[j], c);
            if (TM) hout_row(a, hb[j], sl, q, nw[j]);
        }
        tile_h_end(a, t, c, smn, smx, sfl);
    }
}


// The tiles to rescan: a stale tile matters only if its bound could be the table's
// extreme -- its max bound above every exact tile max (or its min bound below every
// exact min), or a non-finite flag that may be stale.  all: every tile (statistics of
// an imported / cleared table).  hpart[0..2] keeps the exact extremes and the
// non-finite flag of the tiles not rescanned for learn_tile_final_kernel.
constexpr int kCandThreads = 1024, kCandUnroll = 4;

__device__ __forceinline__ void tile_summary(const LearnArgs& a, int t, double4& ts, int& d) {
    const double2* p = reinterpret_cast<const double2*>(a.tstats + 4 * (size_t)t);
    const double2 x = p[0], y = p[1];
    ts = make_double4(x.x, x.y, y.x, y.y);
    d = a.tdirty[t];
}

// The candidates' non-finite word beside the partials (hpart[6..7]): learn_tile_final_kernel
// ORs it into the statistics.
__device__ __forceinline__ int* cand_nf(const LearnArgs& a) { return reinterpret_cast<int*>(a.hpart + 6); }

// The candidate scan on the whole chip (learn_tile_cand_kernel's two passes as two launches):
// per-block min / max over the clean tiles, then every block reduces those partials and lists
// its stale tiles that could still hold the table's extreme.  One workgroup took 21 us at
// C5 (16,384 tiles), mostly its own load latency.
constexpr int kCandPartThreads = 256, kCandPartTiles = 4;   // tiles per thread
constexpr int kCandPartMax = 512;                            // partial blocks (hpart[8 ..))

__global__ __launch_bounds__(kCandPartThreads) void learn_tile_cand_part_kernel(LearnArgs a) {
    __shared__ double smn[kCandPartThreads / 64], smx[kCandPartThreads / 64];
    const int tid = (int)threadIdx.x;
    if (blockIdx.x == 0 && tid == 0) {
        a.tcand[0] = 0;
        cand_nf(a)[0] = 0;
    }
    double cmn = __builtin_inf(), cmx = -__builtin_inf();
    double4 ts[kCandPartTiles];
    int d[kCandPartTiles];
#pragma unroll
    for (int u = 0; u < kCandPartTiles; u++) {
        const int t = ((int)blockIdx.x * kCandPartTiles + u) * kCandPartThreads + tid;
        d[u] = 3;
        if (t < a.NT) tile_summary(a, t, ts[u], d[u]);
    }
#pragma unroll
    for (int u = 0; u < kCandPartTiles; u++) {
        if (d[u] == 3 || ts[u].x == 0.0) continue;
        if (!(d[u] & 1)) cmx = ts[u].w > cmx ? ts[u].w : cmx;
        if (!(d[u] & 2)) cmn = ts[u].z < cmn ? ts[u].z : cmn;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(cmn, o), b2 = __shfl_xor(cmx, o);
        cmn = a2 < cmn ? a2 : cmn;
        cmx = b2 > cmx ? b2 : cmx;
    }
    if ((tid & 63) == 0) { smn[tid >> 6] = cmn; smx[tid >> 6] = cmx; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kCandPartThreads / 64; w++) {
            cmn = smn[w] < cmn ? smn[w] : cmn;
            cmx = smx[w] > cmx ? smx[w] : cmx;
        }
        a.hpart[8 + 2 * blockIdx.x] = cmn;
        a.hpart[9 + 2 * blockIdx.x] = cmx;
    }
}

__global__ __launch_bounds__(kCandPartThreads) void learn_tile_cand_list_kernel(LearnArgs a) {
    __shared__ int sfl[kCandPartThreads / 64];
    const int tid = (int)threadIdx.x, lane = tid & 63;
    // every block reduces the partials (a few hundred words, L2-resident)
    double cmn = __builtin_inf(), cmx = -__builtin_inf();
    for (int b = lane; b < (int)gridDim.x; b += 64) {
        const double x = a.hpart[8 + 2 * b], y = a.hpart[9 + 2 * b];
        cmn = x < cmn ? x : cmn;
        cmx = y > cmx ? y : cmx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(cmn, o), b2 = __shfl_xor(cmx, o);
        cmn = a2 < cmn ? a2 : cmn;
        cmx = b2 > cmx ? b2 : cmx;
    }
    int nf = 0;
#pragma unroll
    for (int u = 0; u < kCandPartTiles; u++) {
        const int t = ((int)blockIdx.x * kCandPartTiles + u) * kCandPartThreads + tid;
        double4 ts;
        int d = -1;
        if (t < a.NT) tile_summary(a, t, ts, d);
        bool c = false;
        if (d >= 0) {
            c = ts.x != 0.0 && (((d & 1) && ts.w >= cmx) || ((d & 2) && ts.z <= cmn) || ((d & 4) && ts.y != 0.0));
            if (!c) nf |= ts.x != 0.0 && ts.y != 0.0;
        }
        const unsigned long long m = __ballot(c);
        if (m) {             // wave-aggregated append
            int base = 0;
            if (lane == 0) base = atomicAdd(&a.tcand[0], __popcll(m));
            base = __shfl(base, 0);
            if (c) a.tcand[1 + base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = t;
        }
    }
    for (int o = 32; o > 0; o >>= 1) nf |= __shfl_xor(nf, o);
    if (lane == 0) sfl[tid >> 6] = nf;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kCandPartThreads / 64; w++) nf |= sfl[w];
        if (nf) atomicOr(cand_nf(a), 1);
        if (blockIdx.x == 0) {
            a.hpart[0] = cmn;
            a.hpart[1] = cmx;
            a.hpart[2] = 0.0;    // the non-finite flags: cand_nf
        }
    }
}

__global__ __launch_bounds__(kCandThreads) void learn_tile_cand_kernel(LearnArgs a, int all) {
    constexpr int NW = kCandThreads / 64;
    __shared__ double smn[NW], smx[NW];
    __shared__ int sfl[NW];
    __shared__ int ncand;
    const int tid = (int)threadIdx.x;
    if (tid == 0) {
        ncand = 0;
        cand_nf(a)[0] = 0;
    }
    double cmn = __builtin_inf(), cmx = -__builtin_inf();   // over exact (clean) tiles
    if (!all) {
        for (int t0 = tid; t0 < a.NT; t0 += kCandUnroll * kCandThreads) {
            double4 ts[kCandUnroll];
            int d[kCandUnroll];
#pragma unroll
            for (int u = 0; u < kCandUnroll; u++) {     // the loads first
                const int t = t0 + u * kCandThreads;
                d[u] = 3;
                if (t < a.NT) tile_summary(a, t, ts[u], d[u]);
            }
#pragma unroll
            for (int u = 0; u < kCandUnroll; u++) {
                if (d[u] == 3 || ts[u].x == 0.0) continue;
                if (!(d[u] & 1)) cmx = ts[u].w > cmx ? ts[u].w : cmx;
                if (!(d[u] & 2)) cmn = ts[u].z < cmn ? ts[u].z : cmn;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(cmn, o), b2 = __shfl_xor(cmx, o);
        cmn = a2 < cmn ? a2 : cmn;
        cmx = b2 > cmx ? b2 : cmx;
    }
    if ((tid & 63) == 0) { smn[tid >> 6] = cmn; smx[tid >> 6] = cmx; }
    __syncthreads();
    for (int w = 0; w < NW; w++) {
        cmn = smn[w] < cmn ? smn[w] : cmn;
        cmx = smx[w] > cmx ? smx[w] : cmx;
    }
    int nf = 0;     // non-finite flags of the tiles not rescanned
    for (int t0 = tid; t0 < a.NT; t0 += kCandUnroll * kCandThreads) {
        double4 ts[kCandUnroll];
        int d[kCandUnroll];
#pragma unroll
        for (int u = 0; u < kCandUnroll; u++) {
            const int t = t0 + u * kCandThreads;
            d[u] = -1;
            if (t < a.NT) {
                if (all) d[u] = 0;
                else tile_summary(a, t, ts[u], d[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < kCandUnroll; u++) {
            if (d[u] < 0) continue;
            const bool c = all || (ts[u].x != 0.0 && (((d[u] & 1) && ts[u].w >= cmx) ||
                                                       ((d[u] & 2) && ts[u].z <= cmn) ||
                                                       ((d[u] & 4) && ts[u].y != 0.0)));
            if (c) a.tcand[1 + atomicAdd(&ncand, 1)] = t0 + u * kCandThreads;
            else nf |= ts[u].x != 0.0 && ts[u].y != 0.0;
        }
    }
    for (int o = 32; o > 0; o >>= 1) nf |= __shfl_xor(nf, o);
    if ((tid & 63) == 0) sfl[tid >> 6] = nf;
    __syncthreads();
    if (tid == 0) {
        for (int w = 0; w < NW; w++) nf |= sfl[w];
        a.tcand[0] = ncand;
        a.hpart[0] = cmn;
        a.hpart[1] = cmx;
        a.hpart[2] = nf ? 1.0 : 0.0;
    }
}

// The candidates of this step's statistics (every tile when `all`) on the whole chip, or
// in one workgroup (FFM_CAND_ONE=1 for A/B).
void launch_tile_cands(const LearnArgs& a, hipStream_t s) {
    const char* v = getenv("FFM_CAND_ONE");
    const unsigned nb = (unsigned)((a.NT + kCandPartThreads * kCandPartTiles - 1) / (kCandPartThreads * kCandPartTiles));
    if ((v && v[0] == '1') || nb > kCandPartMax) {
        learn_tile_cand_kernel<<<dim3(1), dim3(kCandThreads), 0, s>>>(a, 0);
        return;
    }
    learn_tile_cand_part_kernel<<<dim3(nb), dim3(kCandPartThreads), 0, s>>>(a);
    learn_tile_cand_list_kernel<<<dim3(nb), dim3(kCandPartThreads), 0, s>>>(a);
}

template <int NA>
__global__ __launch_bounds__(kTileThreads) void learn_tile_rescan_kernel(LearnArgs a) {
    __shared__ double smn[kTileWaves], smx[kTileWaves];
    __shared__ int sfl[kTileWaves];
    const int n = a.tcand[0];
    for (int c = (int)blockIdx.x; c < n; c += (int)gridDim.x) tile_rescan<NA>(a, a.tcand[1 + c], smn, smx, sfl);
}

// The tiles' summaries -> the statistics the next step's actor reads (hstat): the
// exact extremes of the tiles learn_tile_cand_kernel kept (hpart) and the rescanned
// tiles'.  After learn_tile_rescan_kernel a stale tile's bound is never the extreme.
__device__ __forceinline__ void tile_final(const LearnArgs& a) {
    __shared__ double smn[4], smx[4];
    __shared__ int snf[4];
    double mn = a.hpart[0], mx = a.hpart[1];
    int nf = a.hpart[2] != 0.0 || cand_nf(a)[0] != 0;
    const int n = a.tcand[0];
    for (int c = threadIdx.x; c < n; c += 256) {
        const double* ts = a.tstats + 4 * (size_t)a.tcand[1 + c];
        if (ts[0] == 0.0) continue;
        nf |= ts[1] != 0.0;
        mn = ts[2] < mn ? ts[2] : mn;
        mx = ts[3] > mx ? ts[3] : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double a2 = __shfl_xor(mn, o), b2 = __shfl_xor(mx, o);
        mn = a2 < mn ? a2 : mn;
        mx = b2 > mx ? b2 : mx;
        nf |= __shfl_xor(nf, o);
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smn[wv] = mn; smx[wv] = mx; snf[wv] = nf; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) {
            mn = smn[w] < mn ? smn[w] : mn;
            mx = smx[w] > mx ? smx[w] : mx;
            nf |= snf[w];
        }
        a.hstat[0] = *a.Ht.n > 0 ? 1.0 : 0.0;
        a.hstat[1] = nf ? 1.0 : 0.0;
        a.hstat[2] = mn;
        a.hstat[3] = mx;
        *a.Ht.mark = *a.Ht.n;
        *a.V.mark = *a.V.n;
    }
}

__global__ __launch_bounds__(256) void learn_tile_final_kernel(LearnArgs a) { tile_final(a); }

// ===========================================================================
// Tile-major records.  The batch kernel leaves each env's records in
// raster order with per-env tile offsets (tstart); the pack reorders them tile-major, every
// tile's records of all envs contiguous, grouped by the rank that owns the tile: one
// column scan over the envs, one scan over the tiles, one scatter.  The tile passes then
// read a tile's records as at most one run per source rank -- no per-env ranges, and the
// one-window fast form holds for any number of envs -- and the groups are the
// all-to-all's per-destination blocks.
// ===========================================================================
constexpr int kColTiles = kOwnChunk, kColSplit = 4;   // a colscan block covers one ownership chunk

// pe[e][t] = records of tile t in envs < e, minus tstart[e][t] (mod 2^32: a record's raster
// rank plus it is the record's rank among the tile's records); tpre[t] = records of the tiles before t in its
// chunk of kOwnChunk tiles; csum[c] = records of chunk c.  A block owns one chunk (lanes =
// tiles) and splits the envs in four (waves).
__global__ __launch_bounds__(kColTiles * kColSplit) void learn_tile_colscan_kernel(LearnArgs a, uint32_t* pe,
                                                                                  uint32_t* tpre, uint32_t* csum) {
    __shared__ uint32_t part[kColSplit][kColTiles];
    const int lane = (int)threadIdx.x & 63, q = (int)threadIdx.x >> 6;
    const int t = (int)blockIdx.x * kColTiles + lane;
    const long long per = (a.E + kColSplit - 1) / kColSplit;
    const long long e0 = q * per, e1 = e0 + per < a.E ? e0 + per : a.E;
    const bool ok = t < a.NT;
    const long long S = a.NT + 1;
    const uint16_t* ts = a.tstart + t;
    uint32_t sum = 0;
    if (ok) {
#pragma unroll 8
        for (long long e = e0; e < e1; e++) sum += (uint32_t)(ts[e * S + 1] - ts[e * S]);
    }
    part[q][lane] = sum;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kColSplit; w++) {
        base += w < q ? part[w][lane] : 0u;
        tot += part[w][lane];
    }
    if (q == 0) {     // the chunk's tiles: exclusive prefix over the lanes, and the chunk's sum
        uint32_t incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += v;
        }
        if (ok) tpre[t] = incl - tot;
        if (lane == 63) csum[blockIdx.x] = incl;
    }
    if (!ok) return;
#pragma unroll 8
    for (long long e = e0; e < e1; e++) {
        const uint32_t lo = ts[e * S];
        pe[e * a.NT + t] = base - lo;       // mod 2^32: + the record's raster rank = its place in the tile
        base += (uint32_t)(ts[e * S + 1] - lo);
    }
}

// The chunks in destination order (rank q owns chunks q, q + ow, ...; q = 0 .. ow - 1): toff[t]
// = first record of tile t in the packed buffer, hdr[q][k] = the same relative to q's block
// (hdr[q][NTq] = q's record count), xcnt[q] = q's record count.  One 1024-thread block over
// the chunks (256 at 256x256), then every tile.
constexpr int kOffThreads = 1024;

__global__ __launch_bounds__(kOffThreads) void learn_tile_offsets_kernel(LearnArgs a, const uint32_t* tpre,
                                                                        const uint32_t* csum, uint32_t* coff,
                                                                        uint32_t* toff, uint32_t* hdr,
                                                                        long long* xcnt) {
    __shared__ uint32_t wsum[kOffThreads / 64];
    __shared__ uint32_t seg[kMaxOwners + 1];
    const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int C = kOwnChunk, ow = a.ow <= 1 ? 1 : a.ow;
    const int nch = (a.NT + C - 1) / C;
    const int per = (nch + kOffThreads - 1) / kOffThreads;
    // destination position p -> chunk: rank q's chunks (nq of them) after the ranks before q
    auto chunk_at = [&](int p, int& q) {
        int base = 0;
        for (q = 0; q < ow; q++) {
            const int nq = nch > q ? (nch - 1 - q) / ow + 1 : 0;
            if (p < base + nq) return (p - base) * ow + q;
            base += nq;
        }
        return -1;
    };
    const int p0 = tid * per, p1 = p0 + per < nch ? p0 + per : nch;
    uint32_t sum = 0;
    for (int p = p0; p < p1; p++) {
        int q;
        sum += csum[chunk_at(p, q)];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    if (tid <= ow) seg[tid] = 0xFFFFFFFFu;
    __syncthreads();
    uint32_t off = incl - sum, total = 0;
    for (int v = 0; v < kOffThreads / 64; v++) {
        off += v < w ? wsum[v] : 0u;
        total += wsum[v];
    }
    for (int p = p0; p < p1; p++) {
        int q;
        const int c = chunk_at(p, q);
        coff[c] = off;
        if (c == q) seg[q] = off;          // q's first chunk starts its block
        off += csum[c];
    }
    __syncthreads();
    if (tid == 0) {
        seg[ow] = total;
        for (int q = ow - 1; q >= 0; q--)        // ranks without chunks: an empty block
            if (seg[q] == 0xFFFFFFFFu) seg[q] = seg[q + 1];
    }
    __syncthreads();
    for (int t = tid; t < a.NT; t += kOffThreads) {
        const int c = t / C, q = c % ow, k = (c / ow) * C + t % C;
        const uint32_t o = coff[c] + tpre[t];
        // fixed-capacity blocks (tblk > 0): destination q's block starts at q * tblk
        toff[t] = a.tblk > 0 ? (uint32_t)((long long)q * a.tblk) + (o - seg[q]) : o;
        hdr[(size_t)q * a.ths + k] = o - seg[q];
    }
    if (tid < ow) {
        const int n = owner_tiles(a.NT, ow, C, tid);
        const uint32_t cnt = seg[tid + 1] - seg[tid];
        hdr[(size_t)tid * a.ths + n] = cnt;
        xcnt[tid] = (long long)cnt;
        if (a.tblk > 0 && (long long)cnt > a.tblk) atomicOr(a.overflow, 8);   // reported at the next sync point
    }
}

// Every record to its packed place: tile t of record i of env e is its cell's (the slot of s
// is p * Q + cell); its place is toff[t] + pe[e][t] + i.
// Four records per thread, every load issued before the first store.
constexpr int kScatterJ = 4;

__global__ __launch_bounds__(256) void learn_tile_scatter_kernel(LearnArgs a, const uint32_t* pe,
                                                                 const uint32_t* toff, TileRec* out) {
    const long long e = blockIdx.x;
    const long long S = a.NT + 1;
    const int n = a.tstart[e * S + a.NT];
    const int i0 = (int)blockIdx.y * 256 * kScatterJ + (int)threadIdx.x;
    if (i0 >= n) return;
    const uint32_t Q = (a.V.mask + 1u) >> 8;
    TileRec rc[kScatterJ];
    int t[kScatterJ];
#pragma unroll
    for (int j = 0; j < kScatterJ; j++)
        if (i0 + j * 256 < n) rc[j] = a.trecs[e * a.A + i0 + j * 256];
#pragma unroll
    for (int j = 0; j < kScatterJ; j++) t[j] = (int)(((rc[j].svk & kTileSlot) & (Q - 1u)) / kTileCells);
    uint32_t d[kScatterJ];
#pragma unroll
    for (int j = 0; j < kScatterJ; j++)
        if (i0 + j * 256 < n) d[j] = toff[t[j]] + pe[e * a.NT + t[j]] + (uint32_t)(i0 + j * 256);
    bool in[kScatterJ];
#pragma unroll
    for (int j = 0; j < kScatterJ; j++) {
        in[j] = i0 + j * 256 < n;
        // fixed-capacity blocks: a record past its destination's block is dropped (the
        // offsets kernel flagged the overflow)
        if (a.tblk > 0 && in[j])
            in[j] = d[j] < (uint32_t)((long long)((t[j] / kOwnChunk) % (a.ow <= 1 ? 1 : a.ow) + 1) * a.tblk);
    }
#pragma unroll
    for (int j = 0; j < kScatterJ; j++)
        if (in[j]) out[d[j]] = rc[j];
}

__global__ void learn_mark_kernel(LearnArgs a) {
    *a.V.mark = *a.V.n;
    if (a.Ht.n) *a.Ht.mark = *a.Ht.n;
}

// The other owners' updated V values ([ranks][stride], counts on the device).  Each thread
// takes kApplyJ entries at a time, every load issued before the first store (the entries of
// all owners address distinct slots, so none of a batch's stores feeds another's load).
constexpr int kApplyJ = 4;

__device__ __forceinline__ long long owner_count(const long long* counts, int r, long long stride, int* overflow) {
    long long n = counts[r];
    if (n > stride) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(overflow, 8);
        n = stride;
    }
    return n;
}

__global__ __launch_bounds__(256) void learn_v_scatter_kernel(LearnTable T, const uint32_t* slots,
                                                              const double* vals, long long stride,
                                                              const long long* counts, int ranks, int self,
                                                              int* overflow) {
    const long long nthr = (long long)gridDim.x * 256, t0 = (long long)blockIdx.x * 256 + threadIdx.x;
    for (int r = 0; r < ranks; r++) {
        if (r == self) continue;
        const long long n = owner_count(counts, r, stride, overflow);
        const uint32_t* sl = slots + r * stride;
        const double* vl = vals + r * stride;
        for (long long i0 = t0; i0 < n; i0 += nthr * kApplyJ) {
            uint32_t k[kApplyJ];
            double v[kApplyJ];
#pragma unroll
            for (int j = 0; j < kApplyJ; j++) {
                const long long i = i0 + j * nthr;
                if (i < n) {
                    k[j] = sl[i];
                    v[j] = vl[i];
                }
            }
#pragma unroll
            for (int j = 0; j < kApplyJ; j++)
                if (i0 + j * nthr < n) tval(T, k[j])[0] = v[j];
        }
    }
}

// The other owners' H increments: v + q * 2^-32, the owner's tile_h_apply arithmetic; a
// kHoutNew entry first inserts its row (another rank's step created it).  Batches of
// kApplyJ entries: keys and increments, then the rows' values, then the stores.
__global__ __launch_bounds__(256) void learn_h_deltas_kernel(LearnTable T, const uint32_t* keys, const long long* q,
                                                             long long stride, const long long* counts, int ranks,
                                                             int self, int* overflow) {
    const uint32_t Q = (T.mask + 1u) >> 8;
    const int qsh = __builtin_ctz(Q);
    const long long nthr = (long long)gridDim.x * 256, t0 = (long long)blockIdx.x * 256 + threadIdx.x;
    for (int r = 0; r < ranks; r++) {
        if (r == self) continue;
        const long long n = owner_count(counts, r, stride, overflow);
        const uint32_t* kl = keys + r * stride;
        const long long* ql = q + r * stride;
        for (long long i0 = t0; i0 < n; i0 += nthr * kApplyJ) {
            uint32_t k[kApplyJ];
            long long d[kApplyJ];
            double v[kApplyJ];
            bool live[kApplyJ];
#pragma unroll
            for (int j = 0; j < kApplyJ; j++) {
                const long long i = i0 + j * nthr;
                live[j] = i < n;
                k[j] = 0u;
                d[j] = 0;
                if (live[j]) {
                    k[j] = kl[i];
                    d[j] = ql[i];
                }
            }
#pragma unroll
            for (int j = 0; j < kApplyJ; j++) {
                const uint32_t slot = k[j] & kHoutSlot;
                if (live[j] && (k[j] & kHoutNew)) dense_ensure(T, slot, dense_key(slot, qsh, Q, T.dense_by));
                live[j] = live[j] && d[j] != 0;
                if (live[j]) v[j] = tval(T, slot)[(k[j] >> kHoutActShift) & 15u];
            }
#pragma unroll
            for (int j = 0; j < kApplyJ; j++)
                if (live[j])
                    tval(T, k[j] & kHoutSlot)[(k[j] >> kHoutActShift) & 15u] = v[j] + (double)d[j] * (1.0 / kFxOne);
        }
    }
}

// Owned tiles' H summaries (present, non-finite, min, max, stale bits) for the other ranks.
__global__ __launch_bounds__(256) void learn_tsum_pack_kernel(LearnArgs a, double* tsum) {
    const int k = (int)(blockIdx.x * 256 + threadIdx.x);
    if (k >= a.NTk) return;
    const int t = own_tile(a, k);
#pragma unroll
    for (int i = 0; i < 4; i++) tsum[(size_t)k * 5 + i] = a.tstats[4 * (size_t)t + i];
    tsum[(size_t)k * 5 + 4] = (double)a.tdirty[t];
}

// ... and the other ranks' summaries of their tiles, here (tsum: [ow][stride][5]).
__global__ __launch_bounds__(256) void learn_tsum_unpack_kernel(LearnArgs a, const double* tsum, long long stride) {
    const int t = (int)(blockIdx.x * 256 + threadIdx.x);
    if (t >= a.NT) return;
    const int q = (t / a.ochunk) % a.ow;
    if (q == a.orank) return;
    const int k = ((t / a.ochunk) / a.ow) * a.ochunk + t % a.ochunk;
    const double* src = tsum + ((size_t)q * stride + k) * 5;
#pragma unroll
    for (int i = 0; i < 4; i++) a.tstats[4 * (size_t)t + i] = src[i];
    a.tdirty[t] = (int)src[4];
}

__global__ __launch_bounds__(256) void learn_fill_default_kernel(LearnTable T, double v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i <= T.mask; i += (size_t)gridDim.x * 256)
        if (tkey(T, i) == kEmptyKey) tval(T, i)[0] = v;
}

// Every record empty: key ~0, `width` values `v` (the default), padding zero.
__global__ __launch_bounds__(256) void learn_clear_kernel(LearnTable T, int width, double v) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i <= T.mask; i += (size_t)gridDim.x * 256) {
        unsigned long long* r = T.rec + i * T.stride;
        r[0] = kEmptyKey;
        for (uint32_t k = 1; k < T.stride; k++) r[k] = 0ull;
        double* vp = reinterpret_cast<double*>(r + 1);
        for (int k = 0; k < width; k++) vp[k] = v;
    }
}

// Trajectory capture (model/ffm_unified.py:902-931 run(return_trajectory=True): the
// positions after every step; run_actor_only_training.py:199-218 keeps one every 100th
// episode).  One workgroup per selected env, after the step and before the auto-reset
// re-places an env that ended, so an episode's last row holds its final positions.
__global__ __launch_bounds__(256) void learn_capture_kernel(LearnArgs a, TrajCapture c) {
    __shared__ long long row;
    const int b = blockIdx.x;
    const long long e = c.envs[b];
    const int k = a.episodes[e];
    const int ph = c.phase ? c.phase[b] : 0;
    if ((k + ph) % c.period != 0) return;                 // workgroup-uniform
    // an env that was already empty when the step began has no step to log (auto_reset
    // off: its episode never advances); the step that emptied it is still written
    if (a.cnt[e] == 0 && a.nstart[e] == 0) return;
    if (threadIdx.x == 0) row = (long long)atomicAdd(c.n, 1ull);
    __syncthreads();
    if (row >= c.cap) return;                             // counted as dropped by the drain
    const int n = a.cnt[e];
    if (threadIdx.x == 0) {
        int* m = c.meta + 4 * row;
        m[0] = (int)(a.env_base + e);
        m[1] = k;
        m[2] = a.ep_steps[e];
        m[3] = n;
    }
    for (int i = threadIdx.x; i < a.A; i += 256)
        c.cells[row * a.A + i] = i < n ? a.pos[e * a.A + i] : kNone16;
}

// Philox placement: the N free cells with the smallest
// (key_j, j), in that order.  Candidates (all F, or those under a threshold
// chosen so that N <= expected count << capacity) are bitonic-sorted in LDS.
constexpr int kResetBS = 256;
constexpr int kResetCap = 16384;
constexpr int kResetBin = 256;    // keys of one histogram bin (the exact-threshold fallback)

__device__ __forceinline__ void reset_env(const LearnArgs& a, int all, long long e) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(smem);
    __shared__ int cnt;
    if (all != 1 && !a.done[e]) return;   // all: 0 the step's ended envs, 1 every env, 2 a mask in done
    const int tid = threadIdx.x, F = a.F;
    // episode quota (ffm_learner_set_episode_caps): an env past it stays empty; the episode
    // that reaches it ends with no re-placement (logged and counted like any other)
    if (a.ep_cap && !all && a.episodes[e] >= a.ep_cap[e]) {
        if (tid == 0) a.done[e] = 0;
        return;
    }
    const int N = (a.ep_cap && a.episodes[e] + (all ? 0 : 1) >= a.ep_cap[e]) ? 0 : a.N;
    const uint32_t genv = (uint32_t)(a.env_base + e);
    const bool take_all = F <= kResetCap;
    unsigned long long T = 0xFFFFFFFFull;
    if (!take_all) {
        const unsigned long long want = (unsigned long long)N + (unsigned long long)(kResetCap - N) / 2;
        T = (want << 32) / (unsigned long long)F;
    }
    if (tid == 0) cnt = 0;
    __syncthreads();
    for (int j = tid; j < F; j += kResetBS) {
        const uint32_t k = philox(make_uint4(a.t, genv, (uint32_t)j, kPurReset << 28), a.key0, a.key1).x;
        if (take_all) {
            keys[j] = ((unsigned long long)k << 32) | (unsigned)j;
        } else if ((unsigned long long)k <= T) {
            const int slot = atomicAdd(&cnt, 1);
            if (slot < kResetCap) keys[slot] = ((unsigned long long)k << 32) | (unsigned)j;
        }
    }
    __syncthreads();
    int C = take_all ? F : cnt;
    // fallback: the keys of the threshold bin, and how many of them the placement still takes
    __shared__ unsigned long long sbk[kResetBin];
    __shared__ int sbn;
    int need = 0;
    if (C > kResetCap || C < N) {
        // the sampled threshold kept too few or too many (N close to the capacity): the
        // exact threshold from a histogram of the keys' top 12 bits -- bin b, the first whose
        // cumulative count reaches N.  The keys of the bins below b (fewer than N) are sorted
        // as usual; the N - (their count) smallest keys of bin b follow them, ranked apart
        // (a bin holds ~F / 4096 <= 16 keys on average).  Block-uniform.
        __shared__ int sb, sc;
        uint32_t* hist = reinterpret_cast<uint32_t*>(smem);   // 4,096 bins over the key area
        __syncthreads();
        for (int i = tid; i < 4096; i += kResetBS) hist[i] = 0u;
        __syncthreads();
        for (int j = tid; j < F; j += kResetBS)
            atomicAdd(&hist[philox(make_uint4(a.t, genv, (uint32_t)j, kPurReset << 28), a.key0, a.key1).x >> 20], 1u);
        __syncthreads();
        if (tid < 64) {         // one wave: 64 bins per lane, a lane scan, the crossing lane
            int loc = 0;
            for (int q = 0; q < 64; q++) loc += (int)hist[tid * 64 + q];
            int incl = loc;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(incl, o);
                if (tid >= o) incl += u;
            }
            if (N > 0 && incl >= N && incl - loc < N) {
                int c = incl - loc, q = tid * 64;
                while (c + (int)hist[q] < N) c += (int)hist[q++];
                sb = q;
                sc = c;
            }
            if (N == 0 && tid == 0) { sb = -1; sc = 0; }
        }
        __syncthreads();
        const int bb = sb;
        C = sc;                 // < N: fits the key area
        need = N - C;
        if (tid == 0) { cnt = 0; sbn = 0; }
        __syncthreads();
        for (int j = tid; j < F; j += kResetBS) {
            const uint32_t k = philox(make_uint4(a.t, genv, (uint32_t)j, kPurReset << 28), a.key0, a.key1).x;
            const unsigned long long kj = ((unsigned long long)k << 32) | (unsigned)j;
            if ((int)(k >> 20) < bb) {
                keys[atomicAdd(&cnt, 1)] = kj;
            } else if ((int)(k >> 20) == bb) {
                const int q = atomicAdd(&sbn, 1);
                if (q < kResetBin) sbk[q] = kj;
            }
        }
        __syncthreads();
        if (tid == 0 && sbn > kResetBin) atomicOr(a.overflow, 2);   // a bin of > 256 keys: not seen at F <= 65,536
    }
    int P = 1;
    while (P < C) P <<= 1;
    for (int j = C + tid; j < P; j += kResetBS) keys[j] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = tid; i < P; i += kResetBS) {
                const int l = i ^ jj;
                if (l > i) {
                    const unsigned long long x = keys[i], y = keys[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) { keys[i] = y; keys[l] = x; }
                }
            }
            __syncthreads();
        }
    int NN = N < C ? N : C;
    for (int r = tid; r < NN; r += kResetBS) a.pos[e * a.A + r] = a.free_cells[(int)(keys[r] & 0xFFFFFFFFu)];
    if (need > 0) {             // the threshold bin's smallest keys, ranked among themselves
        const int hb = sbn < kResetBin ? sbn : kResetBin;
        for (int i = tid; i < hb; i += kResetBS) {
            const unsigned long long ki = sbk[i];
            int rank = 0;
            for (int q = 0; q < hb; q++) rank += sbk[q] < ki ? 1 : 0;
            if (rank < need) a.pos[e * a.A + NN + rank] = a.free_cells[(int)(ki & 0xFFFFFFFFu)];
        }
        NN += need < hb ? need : hb;
    }
    float* d = a.dff_in + e * (long long)a.HW;
    for (int c = tid; c < a.HW; c += kResetBS) d[c] = 0.0f;
    if (tid == 0) {
        if (!all) log_episode(a, e);
        a.cnt[e] = NN;
        a.ep_steps[e] = 0;
        a.done[e] = 0;
        if (!all) {
            a.episodes[e] += 1;
            a.counters[4 * e + 2] += 1;
        }
    }
}

__global__ __launch_bounds__(kResetBS) void learn_reset_kernel(LearnArgs a, int all) {
    reset_env(a, all, (long long)blockIdx.x);
}

// The H statistics' final reduction (workgroup 0) and the re-placement of the ended envs
// (workgroup 1 + e; ra: the arguments after the step's DFF swap) in one launch: the two are
// independent, and the step saves a dispatch.
static_assert(kResetBS == 256, "the final reduction's workgroup shape");
__global__ __launch_bounds__(kResetBS) void learn_tile_final_reset_kernel(LearnArgs a, LearnArgs ra) {
    if (blockIdx.x == 0) tile_final(a);
    else reset_env(ra, 0, (long long)blockIdx.x - 1);
}

// ---- delta exchange of the batched step (multi-rank) ----
// Entries touched this step: inserted since the mark, or with pending increments.
template <int WIDTH>
__global__ __launch_bounds__(256) void learn_delta_export_kernel(LearnTable T, unsigned long long* keys,
                                                                 long long* acc, long long cap,
                                                                 unsigned long long* count) {
    const uint32_t n = *T.n, mark = *T.mark;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const size_t s = T.order[i];
        long long q[WIDTH];
        bool touched = i >= mark;
        acc_take<WIDTH>(T, s * WIDTH, q, false);
#pragma unroll
        for (int k = 0; k < WIDTH; k++) touched = touched || q[k] != 0;
        if (!touched) continue;
        const unsigned long long r = atomicAdd(count, 1ull);
        if ((long long)r >= cap) continue;     // the caller checks *count against cap
        keys[r] = tkey(T, s);
#pragma unroll
        for (int k = 0; k < WIDTH; k++) acc[r * WIDTH + k] = q[k];
    }
}

// Another rank's records: insert missing keys (default values), add increments.
// dn: the record count on the device (asynchronous exchange, capped at n); else n.
template <int WIDTH>
__global__ __launch_bounds__(256) void learn_delta_merge_kernel(LearnTable T, const unsigned long long* keys,
                                                                const long long* acc, long long n, int* overflow,
                                                                const long long* dn) {
    if (dn) n = min(n, *dn);
    for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < n; r += (long long)gridDim.x * 256) {
        const int s = tab_get(T, keys[r], overflow);
        if (s < 0) continue;
#pragma unroll
        for (int k = 0; k < WIDTH; k++) {
            const long long q = acc[r * WIDTH + k];
            if (q != 0) acc_add(T.acc + (size_t)s * WIDTH + k, q);   // into copy 0
        }
    }
}

// Asynchronous export: record buffer overflow is flagged for the next sync point.
__global__ void learn_delta_check_kernel(const unsigned long long* count, long long cap, int* overflow) {
    if (threadIdx.x == 0 && (long long)*count > cap) atomicOr(overflow, 4);
}

// Dense tables after an all-reduce of the increments: adopt the presence union of
// every rank (slots another rank inserted get their key and an insertion index).
__global__ __launch_bounds__(256) void learn_dense_adopt_kernel(LearnTable T, const uint32_t* uni) {
    const size_t words = ((size_t)T.mask + 1) / 32;
    for (size_t w = (size_t)blockIdx.x * 256 + threadIdx.x; w < words; w += (size_t)gridDim.x * 256) {
        uint32_t nw = uni[w] & ~T.present[w];
        if (!nw) continue;
        T.present[w] |= nw;
        while (nw) {
            const uint32_t h = (uint32_t)(w * 32) + (uint32_t)__builtin_ctz(nw);
            nw &= nw - 1u;
            const uint32_t sh = (uint32_t)__builtin_ctz((T.mask + 1) >> 8);
            const uint32_t rem = h & ((1u << sh) - 1u), bx = rem / T.dense_by, by = rem - bx * T.dense_by;
            tkey(T, h) = (unsigned long long)(h >> sh) | ((unsigned long long)bx << 26) | ((unsigned long long)by << 45);
            T.order[atomicAdd(T.n, 1u)] = h;
        }
    }
}

// Philox placement for maps with F <= 256 free cells: one wave per 64 envs scans
// their done flags and re-places those envs one after another (every lane
// ranks F/64 keys against all F in LDS), instead of one workgroup per env.
constexpr int kResetSmallF = 256;

// Envs per reset wave: the wave re-places its ended envs one after the other, so the
// launch lasts as long as the wave with the most (C4: ~2 % of 65,536 envs end per step;
// 64 envs per wave left the slowest wave ~6 placements; reset kernel 12.6 -> 10.6 us at 8).
#ifndef FFM_RESET_ENVS
#define FFM_RESET_ENVS 8
#endif
constexpr int kResetSmallEnvs = FFM_RESET_ENVS;

__device__ __forceinline__ void lwave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One wave re-places its ended envs among [e0, e0 + kResetSmallEnvs), keys in its own LDS
// row.  WAVE: the wave shares its workgroup with others (learn_apply_vh_kernel), so it
// synchronises itself only.
template <bool WAVE>
__device__ __forceinline__ void reset_small_wave(const LearnArgs& a, int all, long long e0, unsigned long long* keys) {
    const int lane = (int)(threadIdx.x & 63);
    const long long me = e0 + lane;
    bool want = lane < kResetSmallEnvs && me < a.E && (all == 1 || a.done[me]);
    if (want && a.ep_cap && !all && a.episodes[me] >= a.ep_cap[me]) {   // past its quota: stays empty
        a.done[me] = 0;
        want = false;
    }
    unsigned long long m = __ballot(want);
    const int F = a.F, HW = a.HW;
    while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1ull;
        const long long e = e0 + b;
        const uint32_t genv = (uint32_t)(a.env_base + e);
        const int N = (a.ep_cap && a.episodes[e] + (all ? 0 : 1) >= a.ep_cap[e]) ? 0 : a.N;
        for (int j = lane; j < F; j += 64) {
            const uint32_t k = philox(make_uint4(a.t, genv, (uint32_t)j, kPurReset << 28), a.key0, a.key1).x;
            keys[j] = ((unsigned long long)k << 32) | (unsigned)j;
        }
        if (WAVE) lwave_sync(); else __syncthreads();
        // each lane ranks its (up to four) keys in one pass over 16-B broadcast reads
        if (lane == 0 && (F & 1)) keys[F] = ~0ull;   // pad to pairs: ~0 is never below a key
        if (WAVE) lwave_sync(); else __syncthreads();
        unsigned long long kj[kResetSmallF / 64];
        int rank[kResetSmallF / 64];
#pragma unroll
        for (int q = 0; q < kResetSmallF / 64; q++) {
            kj[q] = lane + 64 * q < F ? keys[lane + 64 * q] : ~0ull;
            rank[q] = 0;
        }
        const ulonglong2* kv = reinterpret_cast<const ulonglong2*>(keys);
        for (int i = 0; i < (F + 1) / 2; i++) {
            const ulonglong2 p = kv[i];
#pragma unroll
            for (int q = 0; q < kResetSmallF / 64; q++) rank[q] += (p.x < kj[q] ? 1 : 0) + (p.y < kj[q] ? 1 : 0);
        }
#pragma unroll
        for (int q = 0; q < kResetSmallF / 64; q++) {
            const int j = lane + 64 * q;
            if (j < F && rank[q] < N) a.pos[e * a.A + rank[q]] = a.free_cells[j];
        }
        float* d = a.dff_in + e * (long long)HW;
        for (int c = lane; c < HW; c += 64) d[c] = 0.0f;
        if (lane == 0) {
            if (!all) log_episode(a, e);
            a.cnt[e] = N;
            a.ep_steps[e] = 0;
            a.done[e] = 0;
            if (!all) {
                a.episodes[e] += 1;
                a.counters[4 * e + 2] += 1;
            }
        }
        if (WAVE) lwave_sync(); else __syncthreads();
    }
}

__global__ __launch_bounds__(64) void learn_reset_small_kernel(LearnArgs a, int all) {
    __shared__ __attribute__((aligned(16))) unsigned long long keys[kResetSmallF + 2];
    reset_small_wave<false>(a, all, (long long)blockIdx.x * kResetSmallEnvs, keys);
}

// nbr > 0: the last nbr workgroups re-place the ended envs as well (ra: the step's
// arguments after the DFF swap; independent of the tables), four waves of
// kResetSmallEnvs envs each -- the reset launch's work without its dispatch.
template <int HWIDTH>
__global__ __launch_bounds__(256) void learn_apply_vh_kernel(LearnTable V, LearnTable Ht, double* hpart, unsigned nbv,
                                                             unsigned nbh, LearnArgs ra) {
    if (blockIdx.x < nbv) {
        apply_hashed<1, false>(V, nullptr, blockIdx.x, nbv);
    } else if (blockIdx.x < nbv + nbh) {
        apply_hashed<HWIDTH, true>(Ht, hpart, blockIdx.x - nbv, nbh);
    } else {
        __shared__ __attribute__((aligned(16))) unsigned long long keys[4][kResetSmallF + 2];
        const unsigned w = threadIdx.x >> 6;
        const long long e0 = ((long long)(blockIdx.x - nbv - nbh) * 4 + w) * kResetSmallEnvs;
        if (e0 < ra.E) reset_small_wave<true>(ra, 0, e0, keys[w]);
    }
}

// Insert keys in the given order (one lane: the insertion order is the dict
// order the reference's get_v_table / get_h_table return) and set their values.
__global__ __launch_bounds__(64) void learn_import_kernel(LearnTable T, int width, const unsigned long long* keys,
                                                          const double* vals, long long n, int* overflow) {
    if (threadIdx.x != 0) return;
    for (long long i = 0; i < n; i++) {
        const int s = tab_get(T, keys[i], overflow);
        if (s < 0) break;
        for (int k = 0; k < width; k++) tval(T, s)[k] = vals[i * width + k];
    }
    *T.mark = *T.n;
}

// update_dff of the batched step as its own launch (large maps): the batch
// kernel's workgroup per env would run it at one CU's bandwidth after its
// latency-bound phases; here every cell of every env is a lane.  Same arithmetic
// as the in-kernel stencil (model/ffm_unified.py:779-798).
// XCD-aware: hardware deals consecutive workgroups round-robin over the 8 XCDs, so
// workgroup b takes logical tile (b % 8) * (B / 8) + b / 8; each XCD then sweeps a
// contiguous run of rows and finds the rows above and below in its own L2.
// tstart [E][NT + 1] -> [NT + 1][E] through a 64 x 64 LDS tile (both sides coalesced);
// tile (bx, by) covers offsets [64 bx, 64 bx + 64) of envs [64 by, 64 by + 64).
__device__ __forceinline__ void tstart_transpose_tile(const uint16_t* in, uint16_t* out, long long E, int NT1,
                                                      int bx, int by) {
    __shared__ uint16_t tl[64][66];
    const int t0 = bx * 64;
    const long long e0 = (long long)by * 64;
    const int lx = (int)threadIdx.x & 63, ly = (int)threadIdx.x >> 6;
    uint16_t v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {     // every load in flight before the first LDS store
        const long long e = e0 + ly + 4 * q;
        const int t = t0 + lx;
        v[q] = e < E && t < NT1 ? in[e * NT1 + t] : (uint16_t)0;
    }
#pragma unroll
    for (int q = 0; q < 16; q++) tl[ly + 4 * q][lx] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int i = ly + 4 * q;
        const int t = t0 + i;
        const long long e = e0 + lx;
        if (t < NT1 && e < E) out[(long long)t * E + e] = tl[lx][i];
    }
}

__global__ __launch_bounds__(256) void learn_tstart_transpose_kernel(const uint16_t* in, uint16_t* out, long long E,
                                                                     int NT1) {
    tstart_transpose_tile(in, out, E, NT1, (int)blockIdx.x, (int)blockIdx.y);
}

__global__ __launch_bounds__(256) void learn_stencil_kernel(LearnArgs a, int tiles_per_env) {
    const unsigned B = gridDim.x, b = blockIdx.x;
    const unsigned lt = (B & 7u) ? b : (b & 7u) * (B >> 3) + (b >> 3);
    const long long e = lt / (unsigned)tiles_per_env;
    const int c = (int)((lt - (unsigned)e * (unsigned)tiles_per_env) * 256 + threadIdx.x);
    if (c >= a.HW) return;
    const int H = a.H, W = a.W;
    const float* dff = a.dff_in + e * (long long)a.HW;
    const int x = fdiv(c, a.mW), y = c - x * W;
    float acc = a.c0 * dff[c];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int nx = x + kNBx[k], ny = y + kNBy[k];
        const float v = (nx >= 0 && nx < H && ny >= 0 && ny < W) ? a.c0 * dff[nx * W + ny] : 0.0f;
        const float t = a.c1 * v;
        acc = acc + t;
    }
    a.dff_out[e * (long long)a.HW + c] = acc < 1e-4f ? 0.0f : acc;
}

// The same stencil four cells of a row per lane (W % 4 == 0): 16-B loads of the
// quad and the quads above and below, scalar loads of its left and right
// neighbours, one 16-B store; per cell the identical operation sequence.
__global__ __launch_bounds__(256) void learn_stencil4_kernel(LearnArgs a, int tiles_per_env) {
    const unsigned B = gridDim.x, b = blockIdx.x;
    const unsigned lt = (B & 7u) ? b : (b & 7u) * (B >> 3) + (b >> 3);
    const long long e = lt / (unsigned)tiles_per_env;
    const int c = 4 * (int)((lt - (unsigned)e * (unsigned)tiles_per_env) * 256 + threadIdx.x);
    if (c >= a.HW) return;
    const int H = a.H, W = a.W;
    const float* dff = a.dff_in + e * (long long)a.HW;
    const int x = fdiv(c, a.mW), y = c - x * W;
    const float c0 = a.c0, c1 = a.c1;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 m = *reinterpret_cast<const float4*>(dff + c);
    const float4 u = x > 0 ? *reinterpret_cast<const float4*>(dff + c - W) : z4;
    const float4 d = x < H - 1 ? *reinterpret_cast<const float4*>(dff + c + W) : z4;
    const float l = y > 0 ? dff[c - 1] : 0.f, r = y + 4 < W ? dff[c + 4] : 0.f;
    const float mv[4] = {m.x, m.y, m.z, m.w}, uv[4] = {u.x, u.y, u.z, u.w}, dv[4] = {d.x, d.y, d.z, d.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        float acc = c0 * mv[k];
        const float nb[4] = {uv[k], dv[k], k > 0 ? mv[k - 1] : l, k < 3 ? mv[k + 1] : r};
        const bool in[4] = {x > 0, x < H - 1, k > 0 || y > 0, k < 3 || y + 4 < W};
#pragma unroll
        for (int q = 0; q < 4; q++) {                    // U, D, L, R as kNBx / kNBy
            const float v = in[q] ? c0 * nb[q] : 0.0f;
            const float t = c1 * v;
            acc = acc + t;
        }
        o[k] = acc < 1e-4f ? 0.0f : acc;
    }
    *reinterpret_cast<float4*>(a.dff_out + e * (long long)a.HW + c) = make_float4(o[0], o[1], o[2], o[3]);
}

// The same stencil for rows of whole waves (W % 256 == 0; C5's 256x256): a wave owns a
// 256-cell row segment over kColRows consecutive rows, four cells per lane, and keeps the
// quads of the rows above, at and below in registers, so each row is loaded once per
// strip (plus one halo row above and below) instead of three times; the left and right
// neighbours come from the adjacent lanes (a scalar load only at a segment's inner
// edges).  A workgroup's four waves take consecutive strips.  Per cell the identical
// operation sequence (U, D, L, R).
#ifndef FFM_COL_ROWS
#define FFM_COL_ROWS 8
#endif
constexpr int kColRows = FFM_COL_ROWS;

// tblocks > 0: the launch's first tblocks workgroups transpose the tile offsets
// (a.tstart -> a.tstart_out, independent of the stencil: one dispatch instead of two);
// tblocks is a multiple of 8, so the stencil's XCD-aware numbering is unchanged.
__global__ __launch_bounds__(256) void learn_stencil_col_kernel(LearnArgs a, int strips, int segs, int tblocks) {
    if ((int)blockIdx.x < tblocks) {
        const int NT1 = a.NT + 1, nbx = (NT1 + 63) / 64, nby = (int)((a.E + 63) / 64);
        const int k = (int)blockIdx.x;
        if (k < nbx * nby) tstart_transpose_tile(a.tstart, a.tstart_out, a.E, NT1, k % nbx, k / nbx);
        return;
    }
    const unsigned B = gridDim.x - (unsigned)tblocks, b = blockIdx.x - (unsigned)tblocks;
    const unsigned lt = (B & 7u) ? b : (b & 7u) * (B >> 3) + (b >> 3);
    const int per_env = strips * segs;
    const long long e = lt / (unsigned)per_env;
    const int r = (int)(lt - (unsigned)e * (unsigned)per_env);
    const int sg = r % segs, st = r / segs;
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const int H = a.H, W = a.W;
    const int x0 = (st * 4 + wv) * kColRows;
    if (x0 >= H) return;
    const int y = sg * 256 + 4 * lane;
    const float* dff = a.dff_in + e * (long long)a.HW;
    float* out = a.dff_out + e * (long long)a.HW;
    const float c0 = a.c0, c1 = a.c1;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 q[kColRows + 2];                 // rows x0 - 1 .. x0 + kColRows
#pragma unroll
    for (int i = 0; i < kColRows + 2; i++) {
        const int x = x0 - 1 + i;
        q[i] = (x >= 0 && x < H) ? *reinterpret_cast<const float4*>(dff + (long long)x * W + y) : z4;
    }
    const bool eL = lane == 0 && y > 0, eR = lane == 63 && y + 4 < W;    // segment edges inside the row
    float le[kColRows], re[kColRows];
#pragma unroll
    for (int i = 0; i < kColRows; i++) {
        const int x = x0 + i;
        le[i] = (eL && x < H) ? dff[(long long)x * W + y - 1] : 0.f;
        re[i] = (eR && x < H) ? dff[(long long)x * W + y + 4] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kColRows; i++) {
        const int x = x0 + i;
        if (x >= H) break;
        const float4 m = q[i + 1], u = q[i], d = q[i + 2];
        float l = __shfl_up(m.w, 1), rr = __shfl_down(m.x, 1);
        l = lane == 0 ? le[i] : l;
        rr = lane == 63 ? re[i] : rr;
        const float mv[4] = {m.x, m.y, m.z, m.w}, uv[4] = {u.x, u.y, u.z, u.w}, dv[4] = {d.x, d.y, d.z, d.w};
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float acc = c0 * mv[k];
            const float nb[4] = {uv[k], dv[k], k > 0 ? mv[k - 1] : l, k < 3 ? mv[k + 1] : rr};
            const bool in[4] = {x > 0, x < H - 1, k > 0 || y > 0, k < 3 || y + 4 < W};
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {             // U, D, L, R as kNBx / kNBy
                const float v = in[qq] ? c0 * nb[qq] : 0.0f;
                const float t = c1 * v;
                acc = acc + t;
            }
            o[k] = acc < 1e-4f ? 0.0f : acc;
        }
        *reinterpret_cast<float4*>(out + (long long)x * W + y) = make_float4(o[0], o[1], o[2], o[3]);
    }
}


constexpr int kSepStencilHW = 16384;

// The DFF stencil of large maps as its own all-cells launch (learn_stencil*_kernel).
void launch_sep_stencil(const LearnArgs& a, hipStream_t s) {
    const int tiles = (a.HW + 255) / 256;
    if (a.W % 256 == 0 && !(FFM_LABLATE & 16)) {
        const int segs = a.W / 256, strips = (a.H + 4 * kColRows - 1) / (4 * kColRows);
        int tb = 0;
        if (a.tstart_out) {
            const int NT1 = a.NT + 1;
            tb = ((NT1 + 63) / 64) * (int)((a.E + 63) / 64);
            tb = (tb + 7) & ~7;
        }
        learn_stencil_col_kernel<<<dim3((unsigned)(strips * segs * a.E + tb)), dim3(256), 0, s>>>(a, strips, segs, tb);
        return;
    }
    if (a.tstart_out) (void)launch_learn_tstart_transpose(a, a.tstart_out, s);
    if (a.W % 4 == 0) {
        const int tiles4 = (a.HW / 4 + 255) / 256;
        learn_stencil4_kernel<<<dim3((unsigned)(tiles4 * a.E)), dim3(256), 0, s>>>(a, tiles4);
    } else {
        learn_stencil_kernel<<<dim3((unsigned)(tiles * a.E)), dim3(256), 0, s>>>(a, tiles);
    }
}

template <int BS, int EPB, int APT, int D, bool DL, int VK = 0, int NB = 4>
hipError_t launch_batch_t(const LearnArgs& a0, hipStream_t s) {
    LearnArgs a = a0;
    // the DFF lives in global memory (not DL) and the map is large: stencil apart (the
    // separate stencil kernels are Neumann's; Moore's stays fused)
    a.sep_stencil = NB == 4 && !DL && a.HW >= kSepStencilHW && (long long)((a.HW + 255) / 256) * a.E < (1ll << 31);
    const size_t smem = batch_carve(a.HW, a.A, D, EPB, DL, batch_rows(a.H, a.W, DL)).shared;
    if (smem > 65536) {
        const hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&learn_batch_kernel<BS, EPB, APT, D, DL, VK, NB>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    const unsigned blocks = (unsigned)((a.E + EPB - 1) / EPB);
    learn_batch_kernel<BS, EPB, APT, D, DL, VK, NB><<<dim3(blocks), dim3(BS), smem, s>>>(a);
    if (a.sep_stencil) launch_sep_stencil(a, s);
    else if (a.tstart_out) (void)launch_learn_tstart_transpose(a, a.tstart_out, s);   // stencil fused: its own launch
    return hipGetLastError();
}

// The phase-split step (learn_phase_*_kernel); the DFF stencil always runs apart.
hipError_t launch_batch_phases(const LearnArgs& a, hipStream_t s) {
    const size_t smem = phase_resolve_carve(a.HW, a.A).total;
    if (smem > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&learn_phase_resolve_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    const unsigned E = (unsigned)a.E;
    const unsigned G = phase_unit_grid(a);
    learn_phase_prep_kernel<<<dim3(E), dim3(kPhBS), 0, s>>>(a);
    learn_phase_decide_kernel<<<dim3(G), dim3(kPhLanes), 0, s>>>(a);
    learn_phase_resolve_kernel<<<dim3(E), dim3(kPhBS), smem, s>>>(a);
    learn_phase_learn_kernel<<<dim3(G), dim3(kPhLanes), 0, s>>>(a);
    launch_sep_stencil(a, s);
    return hipGetLastError();
}

// The kernel's VK = 1 shape: ffm_unified in an actor mode on dense tables with tiled
// records (RASTER holds for every 1024-lane shape).  FFM_BATCH_UNI=0 keeps the generic kernel.
bool learn_batch_uni(const LearnArgs& a) {
    static const bool off = [] { const char* v = getenv("FFM_BATCH_UNI"); return v && v[0] == '0'; }();
    return !off && FFM_RASTER && a.variant == kVarUnified && a.mode != kModeCritic && a.V.dense_by && a.Ht.dense_by &&
           a.trecs != nullptr && !(FFM_LABLATE & 2);
}

// FFM_BATCH_PHASES=1 takes the phase-split step for its shapes (measured
// slower than the fused VK = 1 kernel, so off by default); read at every launch.
bool learn_batch_phases_on() {
    const char* v = getenv("FFM_BATCH_PHASES");
    return v && v[0] == '1';
}

// One agent per lane when A <= 1024; beyond that APT agents per lane of a
// 1024-lane block.  The DFF goes to LDS when it fits beside the rest (DL).
template <int D>
hipError_t launch_batch_d(const LearnArgs& a, hipStream_t s) {
    const int A = a.A, HW = a.HW;
    constexpr size_t kLds = 64 * 1024;
    // 32-lane envs: FFM_SMALL_EPB of them per workgroup (a CU holds a limited
    // number of workgroups; one-wave workgroups would leave most of its wave slots idle)
    // FFM_SMALL_LPE = 16: two agent slots per lane (agents i and i + 16), 16 envs per
    // workgroup: at steady state most envs hold <= 16 live agents, so the second slot's
    // phases are skipped wave-wide and half as many waves carry the same agents
    if (FFM_SMALL_LPE == 16 && A <= 32 && batch_carve(HW, A, D, 16, true).shared <= kLds)
        return launch_batch_t<256, 16, 2, D, true>(a, s);
    if (A <= 32 && batch_carve(HW, A, D, FFM_SMALL_EPB, true).shared <= kLds)
        return launch_batch_t<32 * FFM_SMALL_EPB, FFM_SMALL_EPB, 1, D, true>(a, s);
    if (A <= 32 && batch_carve(HW, A, D, 2).shared <= kLds) return launch_batch_t<64, 2, 1, D, false>(a, s);
    if (A <= 64) {
        if (batch_carve(HW, A, D, 1, true).shared <= kLds) return launch_batch_t<64, 1, 1, D, true>(a, s);
        return launch_batch_t<64, 1, 1, D, false>(a, s);
    }
    if (A <= 256) {
        if (batch_carve(HW, A, D, 1, true).shared <= kLds) return launch_batch_t<256, 1, 1, D, true>(a, s);
        return launch_batch_t<256, 1, 1, D, false>(a, s);
    }
    if (A <= 1024) return launch_batch_t<1024, 1, 1, D, false>(a, s);
    // (owner mode keeps the fused kernel: its records carry the new-row flags)
    if (D == 1 && a.bph && a.ow <= 1 && learn_batch_uni(a) && learn_batch_phases_on()) return launch_batch_phases(a, s);
    if (A <= 2048) return launch_batch_t<1024, 1, 2, D, false>(a, s);
    if (A <= 4096) return launch_batch_t<1024, 1, 4, D, false>(a, s);
    if (A <= 8192) {
        if (D == 1 && learn_batch_uni(a)) return launch_batch_t<1024, 1, 8, 1, false, 1>(a, s);
        return launch_batch_t<1024, 1, 8, D, false>(a, s);
    }
    return launch_batch_t<1024, 1, 16, D, false>(a, s);
}

}  // namespace

size_t learn_exact_scratch_bytes(int HW, int A) { return exact_carve(nullptr, HW, A, nullptr); }

int learn_batch_block_size(int A) { return A <= 64 ? 64 : A <= 256 ? 256 : 1024; }

size_t learn_batch_smem_bytes(int HW, int A, int D) { return batch_carve(HW, A, D, 1).shared; }

size_t learn_batch_phase_bytes(long long E, int HW, int A) {
    if (A <= 1024 || A > 16383 || HW > 65536) return 0;
    return (size_t)E * ((size_t)(HW + 15) / 16 * 8 + (size_t)A * 12);
}

bool learn_batch_supported(int HW, int A, int D) {
    return A <= 16383 && learn_batch_smem_bytes(HW, A, D) <= 160 * 1024;
}

hipError_t launch_learn_hstat(const LearnArgs& a, hipStream_t s) {
    learn_hstat_partial<<<dim3(kHstatBlocks), dim3(256), 0, s>>>(a);
    learn_hstat_final<<<dim3(1), dim3(64), 0, s>>>(a, kHstatBlocks);
    return hipGetLastError();
}

hipError_t launch_learn_exact(const LearnArgs& a, hipStream_t s) {
    learn_exact_kernel<<<dim3(1), dim3(64), 0, s>>>(a);
    return hipGetLastError();
}

// The Moore neighbourhood: one workgroup per env (64, 256 or 1,024 lanes, the DFF in LDS
// when it fits), agents per lane by powers of four beyond 1,024 (fewer shapes to build;
// no reference driver runs Moore, so it gets the general shapes only).
template <int D>
hipError_t launch_batch_moore(const LearnArgs& a, hipStream_t s) {
    const int A = a.A, HW = a.HW;
    constexpr size_t kLds = 64 * 1024;
    if (A <= 64) {
        if (batch_carve(HW, A, D, 1, true).shared <= kLds) return launch_batch_t<64, 1, 1, D, true, 0, 8>(a, s);
        return launch_batch_t<64, 1, 1, D, false, 0, 8>(a, s);
    }
    if (A <= 256) {
        if (batch_carve(HW, A, D, 1, true).shared <= kLds) return launch_batch_t<256, 1, 1, D, true, 0, 8>(a, s);
        return launch_batch_t<256, 1, 1, D, false, 0, 8>(a, s);
    }
    if (A <= 1024) return launch_batch_t<1024, 1, 1, D, false, 0, 8>(a, s);
    if (A <= 4096) return launch_batch_t<1024, 1, 4, D, false, 0, 8>(a, s);
    return launch_batch_t<1024, 1, 16, D, false, 0, 8>(a, s);
}

hipError_t launch_learn_batch(const LearnArgs& a, hipStream_t s) {
    if (a.nb == 8) return a.D == 8 ? launch_batch_moore<8>(a, s) : launch_batch_moore<1>(a, s);
    return a.D == 4 ? launch_batch_d<4>(a, s) : launch_batch_d<1>(a, s);
}

bool learn_reset_small(const LearnArgs& a) { return a.F <= kResetSmallF && a.N <= a.F; }

// Hashed V and H applies and the small-map reset of the ended envs (ra) in one launch.
hipError_t launch_learn_apply_reset(const LearnArgs& a, const LearnArgs& ra, hipStream_t s) {
    const unsigned nb = kHstatBlocks / 4;
    const unsigned nbr = (unsigned)((ra.E + 4 * kResetSmallEnvs - 1) / (4 * kResetSmallEnvs));
    if (a.Ht.accw == 9) learn_apply_vh_kernel<9><<<dim3(512 + nb + nbr), dim3(256), 0, s>>>(a.V, a.Ht, a.hpart, 512u, nb, ra);
    else learn_apply_vh_kernel<5><<<dim3(512 + nb + nbr), dim3(256), 0, s>>>(a.V, a.Ht, a.hpart, 512u, nb, ra);
    learn_hstat_final<<<dim3(1), dim3(64), 0, s>>>(a, (int)nb);
    return hipGetLastError();
}

hipError_t launch_learn_apply(const LearnArgs& a, bool v, bool h, hipStream_t s) {
    if (v && h && !a.V.dense_by && !a.Ht.dense_by) {     // hashed V and H together
        const unsigned nb = kHstatBlocks / 4;
        if (a.Ht.accw == 9) learn_apply_vh_kernel<9><<<dim3(512 + nb), dim3(256), 0, s>>>(a.V, a.Ht, a.hpart, 512u, nb, a);
        else learn_apply_vh_kernel<5><<<dim3(512 + nb), dim3(256), 0, s>>>(a.V, a.Ht, a.hpart, 512u, nb, a);
        learn_hstat_final<<<dim3(1), dim3(64), 0, s>>>(a, (int)nb);
        return hipGetLastError();
    }
    if (v) {
        if (a.V.dense_by) learn_apply_dense_kernel<1, false><<<dim3(2048), dim3(256), 0, s>>>(a.V, nullptr);
        else learn_apply_kernel<1, false><<<dim3(512), dim3(256), 0, s>>>(a.V, nullptr);
    }
    if (h) {     // H increments + the next step's statistics
        // dense: a streaming pass over every slot wants the whole chip; hashed: the
        // insertion-order pass over n entries needs far fewer partials
        const int nb = a.Ht.dense_by ? kHstatBlocks : kHstatBlocks / 4;
        // (H rows: 5 values, 9 with the Moore neighbourhood)
        if (a.Ht.dense_by && a.Ht.accw == 9) learn_apply_dense_kernel<9, true><<<dim3(nb), dim3(256), 0, s>>>(a.Ht, a.hpart);
        else if (a.Ht.dense_by) learn_apply_dense_kernel<5, true><<<dim3(nb), dim3(256), 0, s>>>(a.Ht, a.hpart);
        else if (a.Ht.accw == 9) learn_apply_kernel<9, true><<<dim3(nb), dim3(256), 0, s>>>(a.Ht, a.hpart);
        else learn_apply_kernel<5, true><<<dim3(nb), dim3(256), 0, s>>>(a.Ht, a.hpart);
        learn_hstat_final<<<dim3(1), dim3(64), 0, s>>>(a, nb);
    }
    return hipGetLastError();
}

// Which batch kernel a shape gets (launch_batch_d): does it walk agents in raster order?
bool learn_batch_raster(int HW, int A, int D) {
    constexpr size_t kLds = 64 * 1024;
    if (!FFM_RASTER || A <= 32) return false;       // 32-lane envs: several per workgroup
    if (A <= 64) return false;                       // one wave per env: LPE = 64, but DL or not --
    if (A <= 256) return batch_carve(HW, A, D, 1, true).shared > kLds;
    return true;                                     // 1024-lane workgroups, DFF in global memory
}

// The H passes and the rescan for the table's row width (NA: 5 Neumann, 9 Moore).
template <bool TM, int NA>
static void launch_tile_h_na(const LearnArgs& a, unsigned tgrid, unsigned nresc, hipStream_t s) {
    learn_tile_h_kernel<TM, NA><<<dim3(tgrid), dim3(kTileThreads), 0, s>>>(a);
    learn_tile_h_wide_kernel<TM, NA><<<dim3(nresc), dim3(kTileThreads), 0, s>>>(a);
}
template <bool TM>
static void launch_tile_h(const LearnArgs& a, unsigned tgrid, unsigned nresc, hipStream_t s) {
    if (a.nb == 8) launch_tile_h_na<TM, 9>(a, tgrid, nresc, s);
    else launch_tile_h_na<TM, 5>(a, tgrid, nresc, s);
}
static void launch_tile_rescan(const LearnArgs& a, unsigned nresc, hipStream_t s) {
    if (a.nb == 8) learn_tile_rescan_kernel<9><<<dim3(nresc), dim3(kTileThreads), 0, s>>>(a);
    else learn_tile_rescan_kernel<5><<<dim3(nresc), dim3(kTileThreads), 0, s>>>(a);
}

// One tiled step's table work: V, then (actor modes) H and the statistics.  With
// init_stats, only the per-tile statistics of the current H (no records).
hipError_t launch_learn_tiles(const LearnArgs& a, bool init_stats, hipStream_t s) {
    const bool actor = a.mode != kModeCritic;
    const unsigned nresc = (unsigned)(a.NT < 2048 ? a.NT : 2048);
    if (init_stats) {
        learn_tile_cand_kernel<<<dim3(1), dim3(kCandThreads), 0, s>>>(a, 1);
        launch_tile_rescan(a, nresc, s);
        learn_tile_final_kernel<<<dim3(1), dim3(256), 0, s>>>(a);
        return hipGetLastError();
    }
    const unsigned tgrid = 8u * (unsigned)((a.NT + 7) / 8);
    if (a.thdr) learn_tile_v_kernel<true><<<dim3(tgrid), dim3(kTileThreads), 0, s>>>(a);
    else learn_tile_v_kernel<false><<<dim3(tgrid), dim3(kTileThreads), 0, s>>>(a);
    if (actor) {
        if (a.thdr) launch_tile_h<true>(a, tgrid, nresc, s);
        else launch_tile_h<false>(a, tgrid, nresc, s);
        launch_tile_cands(a, s);
        launch_tile_rescan(a, nresc, s);
        learn_tile_final_kernel<<<dim3(1), dim3(256), 0, s>>>(a);
    }
    return hipGetLastError();
}

hipError_t launch_learn_tstart_transpose(const LearnArgs& a, uint16_t* out, hipStream_t s) {
    const int NT1 = a.NT + 1;
    learn_tstart_transpose_kernel<<<dim3((unsigned)((NT1 + 63) / 64), (unsigned)((a.E + 63) / 64)), dim3(256), 0, s>>>(
        a.tstart, out, a.E, NT1);
    return hipGetLastError();
}

hipError_t launch_learn_tiles_reset(const LearnArgs& a, const LearnArgs& ra, hipStream_t s) {
    const unsigned tgrid = 8u * (unsigned)((a.NT + 7) / 8);
    const unsigned nresc = (unsigned)(a.NT < 2048 ? a.NT : 2048);
    int P = 1;
    while (P < (ra.F < kResetCap ? ra.F : kResetCap)) P <<= 1;
    const size_t smem = (size_t)P * 8;
    if (smem > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&learn_tile_final_reset_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    learn_tile_v_kernel<false><<<dim3(tgrid), dim3(kTileThreads), 0, s>>>(a);
    launch_tile_h<false>(a, tgrid, nresc, s);
    launch_tile_cands(a, s);
    launch_tile_rescan(a, nresc, s);
    learn_tile_final_reset_kernel<<<dim3((unsigned)(1 + ra.E)), dim3(kResetBS), smem, s>>>(a, ra);
    return hipGetLastError();
}

hipError_t launch_learn_tile_pack(const LearnArgs& a, uint32_t* pe, uint32_t* tpre, uint32_t* toff, uint32_t* hdr,
                                  long long* xcnt, TileRec* out, hipStream_t s) {
    if (a.ow > kMaxOwners) return hipErrorInvalidValue;
    // chunk sums and offsets live in toff's tail (NT + 2 * chunks words)
    const int nch = (a.NT + kOwnChunk - 1) / kOwnChunk;
    uint32_t* csum = toff + a.NT;
    uint32_t* coff = csum + nch;
    learn_tile_colscan_kernel<<<dim3((unsigned)nch), dim3(kColTiles * kColSplit), 0, s>>>(a, pe, tpre, csum);
    learn_tile_offsets_kernel<<<dim3(1), dim3(kOffThreads), 0, s>>>(a, tpre, csum, coff, toff, hdr, xcnt);
    learn_tile_scatter_kernel<<<dim3((unsigned)a.E, (unsigned)((a.A + 256 * kScatterJ - 1) / (256 * kScatterJ))),
                                dim3(256), 0, s>>>(a, pe, toff, out);
    return hipGetLastError();
}

// Owner mode: the V pass over the owned tiles (V values out), then the H passes (H
// increments and the owned tiles' summaries out).  The statistics (candidates, rescans,
// final) run on every rank once the summaries are exchanged (launch_learn_tile_stats).
hipError_t launch_learn_tiles_owner_v(const LearnArgs& a, hipStream_t s) {
    const unsigned tgrid = 8u * (unsigned)((a.NTk + 7) / 8);
    if (a.vout_n) (void)hipMemsetAsync(a.vout_n, 0, 8, s);
    if (a.NTk > 0) learn_tile_v_kernel<true><<<dim3(tgrid), dim3(kTileThreads), 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_learn_tiles_owner_h(const LearnArgs& a, double* tsum, hipStream_t s) {
    const unsigned tgrid = 8u * (unsigned)((a.NTk + 7) / 8);
    const unsigned nresc = (unsigned)(a.NTk < 2048 ? (a.NTk > 0 ? a.NTk : 1) : 2048);
    if (a.hout_n) (void)hipMemsetAsync(a.hout_n, 0, 8, s);
    if (a.NTk > 0) {
        launch_tile_h<true>(a, tgrid, nresc, s);
        learn_tsum_pack_kernel<<<dim3((unsigned)((a.NTk + 255) / 256)), dim3(256), 0, s>>>(a, tsum);
    }
    return hipGetLastError();
}

hipError_t launch_learn_tile_stats(const LearnArgs& a, hipStream_t s) {
    const unsigned nresc = (unsigned)(a.NT < 2048 ? a.NT : 2048);
    launch_tile_cands(a, s);
    launch_tile_rescan(a, nresc, s);
    learn_tile_final_kernel<<<dim3(1), dim3(256), 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_learn_mark(const LearnArgs& a, hipStream_t s) {
    learn_mark_kernel<<<dim3(1), dim3(1), 0, s>>>(a);
    return hipGetLastError();
}

// Grid of the apply kernels: their counts live on the device, so the grid covers the
// capacity (grid-stride loops; stride entries per rank at most).
static unsigned owner_grid(long long stride) {
    return (unsigned)std::min<long long>(2048, std::max<long long>(1, (stride + 256 * kApplyJ - 1) / (256 * kApplyJ)));
}

hipError_t launch_learn_v_scatter(const LearnTable& T, const uint32_t* slots, const double* vals, long long stride,
                                  const long long* counts, int ranks, int self, int* overflow, hipStream_t s) {
    if (ranks > 1 && stride > 0)
        learn_v_scatter_kernel<<<dim3(owner_grid(stride)), dim3(256), 0, s>>>(T, slots, vals, stride, counts, ranks, self,
                                                                               overflow);
    return hipGetLastError();
}

hipError_t launch_learn_h_deltas(const LearnTable& T, const uint32_t* keys, const long long* q, long long stride,
                                 const long long* counts, int ranks, int self, int* overflow, hipStream_t s) {
    if (ranks > 1 && stride > 0)
        learn_h_deltas_kernel<<<dim3(owner_grid(stride)), dim3(256), 0, s>>>(T, keys, q, stride, counts, ranks, self,
                                                                              overflow);
    return hipGetLastError();
}

hipError_t launch_learn_tsum_unpack(const LearnArgs& a, const double* tsum, long long stride, hipStream_t s) {
    learn_tsum_unpack_kernel<<<dim3((unsigned)((a.NT + 255) / 256)), dim3(256), 0, s>>>(a, tsum, stride);
    return hipGetLastError();
}

hipError_t launch_learn_post(const LearnArgs& a, hipStream_t s) {
    const long long slots = a.E * a.A;
    learn_post_kernel<<<dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s>>>(a);
    return hipGetLastError();
}

// a reset_envs mask (bytes) into the done flags the reset kernels select by
__global__ __launch_bounds__(256) void learn_mask_done_kernel(const uint8_t* mask, int* done, long long E) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e < E) done[e] = mask[e] ? 1 : 0;
}

hipError_t launch_learn_reset_mask(const LearnArgs& a, const uint8_t* mask, hipStream_t s) {
    learn_mask_done_kernel<<<dim3((unsigned)((a.E + 255) / 256)), dim3(256), 0, s>>>(mask, a.done, a.E);
    const hipError_t e = hipGetLastError();
    return e != hipSuccess ? e : launch_learn_reset(a, 2, s);
}

hipError_t launch_learn_reset(const LearnArgs& a, int all, hipStream_t s) {
    if (a.F <= kResetSmallF && a.N <= a.F) {
        learn_reset_small_kernel<<<dim3((unsigned)((a.E + kResetSmallEnvs - 1) / kResetSmallEnvs)), dim3(64), 0, s>>>(
            a, all);
        return hipGetLastError();
    }
    int P = 1;
    while (P < (a.F < kResetCap ? a.F : kResetCap)) P <<= 1;
    const size_t smem = (size_t)P * 8;
    if (smem > 65536) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&learn_reset_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    learn_reset_kernel<<<dim3((unsigned)a.E), dim3(kResetBS), smem, s>>>(a, all);
    return hipGetLastError();
}

hipError_t launch_learn_delta_export(const LearnTable& T, int width, unsigned long long* keys, long long* acc,
                                    long long cap, unsigned long long* count, hipStream_t s) {
    if (width == 2) learn_delta_export_kernel<2><<<dim3(1024), dim3(256), 0, s>>>(T, keys, acc, cap, count);
    else if (width == 9) learn_delta_export_kernel<9><<<dim3(1024), dim3(256), 0, s>>>(T, keys, acc, cap, count);
    else learn_delta_export_kernel<5><<<dim3(1024), dim3(256), 0, s>>>(T, keys, acc, cap, count);
    return hipGetLastError();
}

hipError_t launch_learn_delta_merge(const LearnTable& T, int width, const unsigned long long* keys,
                                   const long long* acc, long long n, int* overflow, hipStream_t s,
                                   const long long* dn) {
    if (n <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<long long>(4096, (n + 255) / 256);
    if (width == 2) learn_delta_merge_kernel<2><<<dim3(blocks), dim3(256), 0, s>>>(T, keys, acc, n, overflow, dn);
    else if (width == 9) learn_delta_merge_kernel<9><<<dim3(blocks), dim3(256), 0, s>>>(T, keys, acc, n, overflow, dn);
    else learn_delta_merge_kernel<5><<<dim3(blocks), dim3(256), 0, s>>>(T, keys, acc, n, overflow, dn);
    return hipGetLastError();
}

hipError_t launch_learn_delta_check(const unsigned long long* count, long long cap, int* overflow, hipStream_t s) {
    learn_delta_check_kernel<<<dim3(1), dim3(64), 0, s>>>(count, cap, overflow);
    return hipGetLastError();
}

hipError_t launch_learn_dense_adopt(const LearnTable& T, const uint32_t* uni, hipStream_t s) {
    const size_t words = ((size_t)T.mask + 1) / 32;
    const unsigned blocks = (unsigned)std::min<size_t>(2048, (words + 255) / 256);
    learn_dense_adopt_kernel<<<dim3(blocks), dim3(256), 0, s>>>(T, uni);
    return hipGetLastError();
}

hipError_t launch_learn_import(const LearnTable& T, int width, const unsigned long long* keys, const double* vals,
                              long long n, int* overflow, hipStream_t s) {
    learn_import_kernel<<<dim3(1), dim3(64), 0, s>>>(T, width, keys, vals, n, overflow);
    return hipGetLastError();
}

hipError_t launch_learn_clear(const LearnTable& T, int width, double dflt, hipStream_t s) {
    learn_clear_kernel<<<dim3(2048), dim3(256), 0, s>>>(T, width, dflt);
    return hipGetLastError();
}

hipError_t launch_learn_capture(const LearnArgs& a, const TrajCapture& c, hipStream_t s) {
    if (c.n_sel <= 0) return hipSuccess;
    learn_capture_kernel<<<dim3((unsigned)c.n_sel), dim3(256), 0, s>>>(a, c);
    return hipGetLastError();
}

hipError_t launch_learn_fill_default(const LearnArgs& a, hipStream_t s) {
    learn_fill_default_kernel<<<dim3(1024), dim3(256), 0, s>>>(a.V, a.v_default);
    return hipGetLastError();
}

}  // namespace ffm
