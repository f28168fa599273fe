/*
 * oracle_core.c -- CPU restatement of the reference's integer/byte arithmetic on
 * the PinSage sampler path.  TEST INFRASTRUCTURE ONLY: imported by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product.
 *
 * Pinned against tests/golden/*.npz, which were produced by running the real
 * reference (imported with dependency stubs) in the dev container
 * (tests/golden/make_golden.py).
 *
 * Restated here:
 *  - torch's CPU generator: MT19937 (at::mt19937 semantics: lazy twist on the
 *    draw that needs it, `left`/`next` bookkeeping) as consumed by
 *    torch.randint(n, ()) = raw % n, torch.rand(()) = (raw & 0xFFFFFF) * 2^-24
 *    and torch.randperm(n) (Fisher-Yates, one draw per step).
 *  - do_random_walks  (pinsage_model.py:32-53): 3 draws per hop in the order
 *    collection choice, item choice, restart test.
 *  - Tensor.topk(k, 1) on a CPU f64 row (pinsage_model.py:107) = libstdc++
 *    std::partial_sort when k*64 <= n, else std::nth_element(k-1) followed by
 *    std::sort of the first k-1, with comparator
 *    (isnan(a) && !isnan(b)) || a > b  over (value, index) pairs.
 *  - Philox4x32-10 (the product's fast RNG mode) so the fast mode has a
 *    bit-exact CPU twin.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ MT19937 */
#define MT_N 624
#define MT_M 397

typedef struct {
    uint64_t seed;
    int32_t left;
    int32_t seeded;
    uint32_t next;
    uint32_t state[MT_N];
} mt_t;

static inline uint32_t mt_twist1(uint32_t u, uint32_t v) {
    uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
    return (y >> 1) ^ ((v & 1u) ? 0x9908b0dfu : 0u);
}

static void mt_next_state(mt_t *g) {
    uint32_t *s = g->state;
    int i = 0;
    for (; i < MT_N - MT_M; ++i) s[i] = s[i + MT_M] ^ mt_twist1(s[i], s[i + 1]);
    for (; i < MT_N - 1; ++i) s[i] = s[i + MT_M - MT_N] ^ mt_twist1(s[i], s[i + 1]);
    s[MT_N - 1] = s[MT_M - 1] ^ mt_twist1(s[MT_N - 1], s[0]);
    g->left = MT_N;
    g->next = 0;
}

void orc_mt_seed(mt_t *g, uint64_t seed) {
    g->seed = seed;
    g->seeded = 1;
    g->state[0] = (uint32_t)(seed & 0xffffffffu);
    for (int j = 1; j < MT_N; ++j)
        g->state[j] = 1812433253u * (g->state[j - 1] ^ (g->state[j - 1] >> 30)) + (uint32_t)j;
    g->left = 1;
    g->next = 0;
}

static inline uint32_t mt_draw(mt_t *g) {
    if (--g->left == 0) mt_next_state(g);
    uint32_t y = g->state[g->next++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

uint32_t orc_mt_draw(mt_t *g) { return mt_draw(g); }

int orc_mt_size(void) { return (int)sizeof(mt_t); }

/* torch.get_rng_state() layout (CPUGeneratorImplState, 5056 bytes):
 * u64 seed @0, i32 left @8, i32 seeded @12, u64 next @16, u64 state[624] @24. */
void orc_mt_from_torch(mt_t *g, const uint8_t *buf) {
    uint64_t seed, next, st;
    int32_t left, seeded;
    memcpy(&seed, buf + 0, 8);
    memcpy(&left, buf + 8, 4);
    memcpy(&seeded, buf + 12, 4);
    memcpy(&next, buf + 16, 8);
    g->seed = seed;
    g->left = left;
    g->seeded = seeded;
    g->next = (uint32_t)next;
    for (int i = 0; i < MT_N; ++i) {
        memcpy(&st, buf + 24 + 8 * i, 8);
        g->state[i] = (uint32_t)st;
    }
}

void orc_mt_to_torch(const mt_t *g, uint8_t *buf) {
    uint64_t next = g->next, st;
    memcpy(buf + 0, &g->seed, 8);
    memcpy(buf + 8, &g->left, 4);
    memcpy(buf + 12, &g->seeded, 4);
    memcpy(buf + 16, &next, 8);
    for (int i = 0; i < MT_N; ++i) {
        st = g->state[i];
        memcpy(buf + 24 + 8 * i, &st, 8);
    }
}

void orc_mt_draws(mt_t *g, uint32_t *out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) out[i] = mt_draw(g);
}

/* torch.randperm(n) on CPU: forward Fisher-Yates, r[i] <-> r[i + raw % (n-i)]. */
void orc_randperm(mt_t *g, int64_t n, int64_t *out) {
    for (int64_t i = 0; i < n; ++i) out[i] = i;
    for (int64_t i = 0; i < n - 1; ++i) {
        int64_t z = (int64_t)(mt_draw(g) % (uint64_t)(n - i));
        int64_t t = out[i];
        out[i] = out[z + i];
        out[z + i] = t;
    }
}

/* ------------------------------------------------------------------ walk */
/* do_random_walks (pinsage_model.py:32-53) over CSR (indptr i64, indices i32).
 * alpha is compared as float32, as `torch.rand(()) < alpha` does.
 * Returns 0, or -1-(index of the source) when a zero-degree node is met. */
int64_t orc_walk_mt(mt_t *g, const int64_t *indptr, const int32_t *indices,
                    const int64_t *sources, int64_t n_src, int64_t n_hops, float alpha,
                    int64_t *trace) {
    for (int64_t i = 0; i < n_src; ++i) {
        int64_t item = sources[i];
        for (int64_t j = 0; j < n_hops; ++j) {
            int64_t b = indptr[item], d = indptr[item + 1] - b;
            if (d <= 0) return -1 - i;
            int64_t col = indices[b + (int64_t)(mt_draw(g) % (uint64_t)d)];
            b = indptr[col];
            d = indptr[col + 1] - b;
            if (d <= 0) return -1 - i;
            item = indices[b + (int64_t)(mt_draw(g) % (uint64_t)d)];
            trace[i * n_hops + j] = item;
            float u = (float)(mt_draw(g) & 0xFFFFFFu) * 0x1p-24f;
            if (u < alpha) item = sources[i];
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ Philox4x32-10 */
static inline void philox_round(uint32_t c[4], const uint32_t k[2]) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k[0];
    uint32_t n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
}

void orc_philox(uint64_t key, const uint32_t ctr_in[4], uint32_t out[4]) {
    uint32_t c[4] = {ctr_in[0], ctr_in[1], ctr_in[2], ctr_in[3]};
    uint32_t k[2] = {(uint32_t)key, (uint32_t)(key >> 32)};
    for (int r = 0; r < 10; ++r) {
        philox_round(c, k);
        if (r < 9) {
            k[0] += 0x9E3779B9u;
            k[1] += 0xBB67AE85u;
        }
    }
    out[0] = c[0];
    out[1] = c[1];
    out[2] = c[2];
    out[3] = c[3];
}

/* Fast-mode walk: draws for (source position p, hop j) = Philox(key=seed,
 * ctr={j, p_lo, p_hi, offset}); words 0,1,2 play the roles of the 3 MT draws. */
int64_t orc_walk_philox(uint64_t seed, uint32_t offset, const int64_t *indptr,
                        const int32_t *indices, const int64_t *sources, int64_t n_src,
                        int64_t src_base, int64_t n_hops, float alpha, int64_t *trace) {
    for (int64_t i = 0; i < n_src; ++i) {
        int64_t item = sources[i];
        uint64_t p = (uint64_t)(src_base + i);
        for (int64_t j = 0; j < n_hops; ++j) {
            uint32_t ctr[4] = {(uint32_t)j, (uint32_t)p, (uint32_t)(p >> 32), offset}, r[4];
            orc_philox(seed, ctr, r);
            int64_t b = indptr[item], d = indptr[item + 1] - b;
            if (d <= 0) return -1 - i;
            int64_t col = indices[b + (int64_t)(r[0] % (uint64_t)d)];
            b = indptr[col];
            d = indptr[col + 1] - b;
            if (d <= 0) return -1 - i;
            item = indices[b + (int64_t)(r[1] % (uint64_t)d)];
            trace[i * n_hops + j] = item;
            float u = (float)(r[2] & 0xFFFFFFu) * 0x1p-24f;
            if (u < alpha) item = sources[i];
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ libstdc++ top-k */
typedef struct {
    double v;
    int64_t i;
} elem_t;

static inline int cmp_gt(const elem_t *a, const elem_t *b) {
    return (isnan(a->v) && !isnan(b->v)) || (a->v > b->v);
}

static void push_heap(elem_t *f, int64_t hole, int64_t top, elem_t val) {
    int64_t parent = (hole - 1) / 2;
    while (hole > top && cmp_gt(&f[parent], &val)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = val;
}

static void adjust_heap(elem_t *f, int64_t hole, int64_t len, elem_t val) {
    const int64_t top = hole;
    int64_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (cmp_gt(&f[child], &f[child - 1])) child--;
        f[hole] = f[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        f[hole] = f[child - 1];
        hole = child - 1;
    }
    push_heap(f, hole, top, val);
}

static void make_heap(elem_t *f, int64_t len) {
    if (len < 2) return;
    int64_t parent = (len - 2) / 2;
    for (;;) {
        elem_t v = f[parent];
        adjust_heap(f, parent, len, v);
        if (parent == 0) return;
        parent--;
    }
}

static void pop_heap(elem_t *f, int64_t len, elem_t *result) {
    elem_t v = *result;
    *result = f[0];
    adjust_heap(f, 0, len, v);
}

static void heap_select(elem_t *f, int64_t mid, int64_t last) {
    make_heap(f, mid);
    for (int64_t i = mid; i < last; ++i)
        if (cmp_gt(&f[i], &f[0])) pop_heap(f, mid, &f[i]);
}

static void sort_heap(elem_t *f, int64_t len) {
    while (len > 1) {
        --len;
        pop_heap(f, len, &f[len]);
    }
}

static inline void swap_e(elem_t *a, elem_t *b) {
    elem_t t = *a;
    *a = *b;
    *b = t;
}

static void move_median_to_first(elem_t *res, elem_t *a, elem_t *b, elem_t *c) {
    if (cmp_gt(a, b)) {
        if (cmp_gt(b, c)) swap_e(res, b);
        else if (cmp_gt(a, c)) swap_e(res, c);
        else swap_e(res, a);
    } else if (cmp_gt(a, c)) swap_e(res, a);
    else if (cmp_gt(b, c)) swap_e(res, c);
    else swap_e(res, b);
}

static elem_t *unguarded_partition(elem_t *first, elem_t *last, elem_t *pivot) {
    for (;;) {
        while (cmp_gt(first, pivot)) ++first;
        --last;
        while (cmp_gt(pivot, last)) --last;
        if (!(first < last)) return first;
        swap_e(first, last);
        ++first;
    }
}

static elem_t *unguarded_partition_pivot(elem_t *first, elem_t *last) {
    elem_t *mid = first + (last - first) / 2;
    move_median_to_first(first, first + 1, mid, last - 1);
    return unguarded_partition(first + 1, last, first);
}

static void unguarded_linear_insert(elem_t *last) {
    elem_t val = *last;
    elem_t *next = last - 1;
    while (cmp_gt(&val, next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

static void insertion_sort(elem_t *first, elem_t *last) {
    if (first == last) return;
    for (elem_t *i = first + 1; i != last; ++i) {
        if (cmp_gt(i, first)) {
            elem_t val = *i;
            memmove(first + 1, first, (size_t)(i - first) * sizeof(elem_t));
            *first = val;
        } else {
            unguarded_linear_insert(i);
        }
    }
}

static int lg2(int64_t n) { return 63 - __builtin_clzll((unsigned long long)n); }

static void introselect(elem_t *first, elem_t *nth, elem_t *last, int depth) {
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(first, (nth + 1) - first, last - first);
            swap_e(first, nth);
            return;
        }
        --depth;
        elem_t *cut = unguarded_partition_pivot(first, last);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort(first, last);
}

static void introsort_loop(elem_t *first, elem_t *last, int depth) {
    while (last - first > 16) {
        if (depth == 0) {
            heap_select(first, last - first, last - first);
            sort_heap(first, last - first);
            return;
        }
        --depth;
        elem_t *cut = unguarded_partition_pivot(first, last);
        introsort_loop(cut, last, depth);
        last = cut;
    }
}

static void final_insertion_sort(elem_t *first, elem_t *last) {
    if (last - first > 16) {
        insertion_sort(first, first + 16);
        for (elem_t *i = first + 16; i != last; ++i) unguarded_linear_insert(i);
    } else {
        insertion_sort(first, last);
    }
}

static void std_sort(elem_t *first, elem_t *last) {
    if (first == last) return;
    introsort_loop(first, last, lg2(last - first) * 2);
    final_insertion_sort(first, last);
}

/* One row of Tensor.topk(k, dim=1, largest=True, sorted=True) on CPU f64. */
void orc_topk_row(const double *row, int64_t n, int64_t k, double *vals, int64_t *idx,
                  elem_t *scratch) {
    if (k <= 0) return;
    for (int64_t j = 0; j < n; ++j) {
        scratch[j].v = row[j];
        scratch[j].i = j;
    }
    if (k * 64 <= n) {
        heap_select(scratch, k, n);
        sort_heap(scratch, k);
    } else {
        introselect(scratch, scratch + k - 1, scratch + n, lg2(n) * 2);
        std_sort(scratch, scratch + k - 1);
    }
    for (int64_t j = 0; j < k; ++j) {
        vals[j] = scratch[j].v;
        idx[j] = scratch[j].i;
    }
}

void orc_topk(const double *m, int64_t rows, int64_t n, int64_t k, double *vals, int64_t *idx) {
    elem_t *s = (elem_t *)malloc((size_t)n * sizeof(elem_t));
    for (int64_t r = 0; r < rows; ++r) orc_topk_row(m + r * n, n, k, vals + r * k, idx + r * k, s);
    free(s);
}
