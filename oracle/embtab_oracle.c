/*
 * embtab_oracle.c — TEST INFRASTRUCTURE ONLY (see embtab_oracle.h).
 *
 * CPU restatement of darchr/EmbeddingTables.jl's hot path, function by
 * function, in the reference's own evaluation order.  Built with
 * -ffp-contract=off so that every fused multiply-add is the explicit fma()
 * the reference's muladd lowers to, and nothing else is fused.
 */
#define _GNU_SOURCE
#include "embtab_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int orc_elsize(int dtype) {
    switch (dtype) {
        case ORC_F32: return 4;
        case ORC_F16: return 2;
        case ORC_F64: return 8;
        case ORC_I32: return 4;
        case ORC_I64: return 8;
        case ORC_BF16: return 2;
        default: return 0;
    }
}

double orc_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------------- */
/* fp16                                                                       */
/* ------------------------------------------------------------------------- */

uint16_t orc_f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t mag = x & 0x7fffffffu;
    if (mag >= 0x7f800000u) { /* inf or nan */
        if (mag > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((mag >> 13) & 0x3ffu));
        return (uint16_t)(sign | 0x7c00u);
    }
    if (mag >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to inf */
    if (mag < 0x38800000u) {                                   /* subnormal or zero */
        if (mag < 0x33000000u) return (uint16_t)sign;          /* < half of min subnormal */
        uint32_t e = mag >> 23;
        uint32_t m = (mag & 0x7fffffu) | 0x800000u;
        uint32_t shift = 126 - e; /* 14 + (113 - e) - 1 */
        uint32_t r = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1);
        uint32_t half = 1u << (shift - 1);
        if (rem > half || (rem == half && (r & 1))) r++;
        return (uint16_t)(sign | r);
    }
    uint32_t r = mag - 0x38000000u; /* rebias exponent 127 -> 15 */
    uint32_t lsb = (r >> 13) & 1u;
    r += 0xfffu + lsb;
    return (uint16_t)(sign | (r >> 13));
}

float orc_f16_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    uint32_t x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else { /* subnormal: normalise */
            int k = 0;
            while (!(m & 0x400u)) { m <<= 1; k++; }
            m &= 0x3ffu;
            x = sign | ((uint32_t)(113 - k) << 23) | (m << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

uint16_t orc_f32_to_bf16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    if ((x & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((x >> 16) | 0x40u);
    x += 0x7fffu + ((x >> 16) & 1u);
    return (uint16_t)(x >> 16);
}

float orc_bf16_to_f32(uint16_t h) {
    uint32_t x = (uint32_t)h << 16;
    float f;
    memcpy(&f, &x, 4);
    return f;
}

/* Julia Float16 `a + b` = Float16(Float32(a) + Float32(b)). */
static inline uint16_t f16_add(uint16_t a, uint16_t b) {
    return orc_f32_to_f16(orc_f16_to_f32(a) + orc_f16_to_f32(b));
}

/* ------------------------------------------------------------------------- */
/* lookup                                                                     */
/* ------------------------------------------------------------------------- */

/* src/lookup.jl:51-67 (generic) / :70-87 (static): dst[:, j] = A[:, I[j]]. */
void orc_gather(int dtype, const void* table, int64_t ld_table, int32_t dim, const int64_t* idx,
                int64_t n, void* dst, int64_t ld_dst) {
    int es = orc_elsize(dtype);
    const char* t = (const char*)table;
    char* o = (char*)dst;
    for (int64_t j = 0; j < n; j++) {
        int64_t col = idx[j] - 1;
        memcpy(o + (size_t)j * ld_dst * es, t + (size_t)col * ld_table * es, (size_t)dim * es);
    }
}

/* src/lookup.jl:108-132 (lookup_generic!) and :134-165 (lookup_static_inner):
 * first row copied, every later row added, in pool order. */
#define POOLED_BODY(T, ADD)                                                                \
    do {                                                                                   \
        const T* A = (const T*)table;                                                      \
        T* O = (T*)dst;                                                                    \
        for (int64_t j = 0; j < batch; j++) {                                              \
            T* vO = O + (size_t)j * ld_dst;                                                \
            const int64_t* I = idx + (size_t)j * ld_idx;                                   \
            if (pool == 0) {                                                               \
                memset(vO, 0, sizeof(T) * (size_t)dim);                                    \
                continue;                                                                  \
            }                                                                              \
            const T* vA = A + (size_t)(I[0] - 1) * ld_table;                               \
            for (int32_t k = 0; k < dim; k++) vO[k] = vA[k];                               \
            for (int32_t i = 1; i < pool; i++) {                                           \
                vA = A + (size_t)(I[i] - 1) * ld_table;                                    \
                for (int32_t k = 0; k < dim; k++) vO[k] = ADD(vO[k], vA[k]);               \
            }                                                                              \
        }                                                                                  \
    } while (0)

#define ADD_PLAIN(a, b) ((a) + (b))
#define ADD_WRAP_I32(a, b) ((int32_t)((uint32_t)(a) + (uint32_t)(b)))
#define ADD_WRAP_I64(a, b) ((int64_t)((uint64_t)(a) + (uint64_t)(b)))

/* 16-bit tables summed in fp32 (first row converted, later rows added in pool order),
 * one rounding per output element: fp16 with f16_fp32_acc, and bfloat16. */
static void pooled_16_fp32acc(const uint16_t* A, int64_t ld_table, int32_t dim,
                              const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                              uint16_t* O, int64_t ld_dst, float (*to32)(uint16_t),
                              uint16_t (*from32)(float)) {
    float acc[4096];
    for (int64_t j = 0; j < batch; j++) {
        uint16_t* vO = O + (size_t)j * ld_dst;
        const int64_t* I = idx + (size_t)j * ld_idx;
        for (int32_t k0 = 0; k0 < dim; k0 += 4096) {
            int32_t kn = dim - k0 < 4096 ? dim - k0 : 4096;
            for (int32_t k = 0; k < kn; k++) acc[k] = 0.0f;
            for (int32_t i = 0; i < pool; i++) {
                const uint16_t* vA = A + (size_t)(I[i] - 1) * ld_table + k0;
                if (i == 0)
                    for (int32_t k = 0; k < kn; k++) acc[k] = to32(vA[k]);
                else
                    for (int32_t k = 0; k < kn; k++) acc[k] += to32(vA[k]);
            }
            for (int32_t k = 0; k < kn; k++) vO[k0 + k] = from32(acc[k]);
        }
    }
}

void orc_pooled_sum(int dtype, const void* table, int64_t ld_table, int32_t dim,
                    const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch, void* dst,
                    int64_t ld_dst, int f16_fp32_acc) {
    switch (dtype) {
        case ORC_F32: POOLED_BODY(float, ADD_PLAIN); break;
        case ORC_F64: POOLED_BODY(double, ADD_PLAIN); break;
        case ORC_I32: POOLED_BODY(int32_t, ADD_WRAP_I32); break;
        case ORC_I64: POOLED_BODY(int64_t, ADD_WRAP_I64); break;
        case ORC_F16:
            if (f16_fp32_acc)
                pooled_16_fp32acc((const uint16_t*)table, ld_table, dim, idx, pool, ld_idx,
                                  batch, (uint16_t*)dst, ld_dst, orc_f16_to_f32,
                                  orc_f32_to_f16);
            else
                POOLED_BODY(uint16_t, f16_add);
            break;
        case ORC_BF16:
            pooled_16_fp32acc((const uint16_t*)table, ld_table, dim, idx, pool, ld_idx, batch,
                              (uint16_t*)dst, ld_dst, orc_bf16_to_f32, orc_f32_to_bf16);
            break;
        default: break;
    }
}

/* ------------------------------------------------------------------------- */
/* maplookup! (PreallocationStrategy)                                         */
/* ------------------------------------------------------------------------- */

typedef struct {
    int dtype;
    const orc_lookup_desc* descs;
    int32_t ntables;
    int64_t batch;
    char* dst;
    int64_t ld_dst;
    int64_t worksize;
    int64_t len;
    int f16_fp32_acc;
    atomic_long count;
} prealloc_ctx;

static void* prealloc_worker(void* arg) {
    prealloc_ctx* c = (prealloc_ctx*)arg;
    int es = orc_elsize(c->dtype);
    for (;;) {
        /* k = Threads.atomic_add!(count, 1); k > len && break   (src/lookup.jl:347-349) */
        long k = atomic_fetch_add(&c->count, 1);
        if (k > c->len) break;
        /* j, i = _divrem_index(k, divisor)   (src/split.jl:59-65) */
        long j = (k - 1) / c->ntables + 1;
        long i = (k - 1) % c->ntables + 1;
        int64_t start = (j - 1) * c->worksize + 1;
        int64_t stop = j * c->worksize < c->batch ? j * c->worksize : c->batch;
        if (stop < start) continue;
        const orc_lookup_desc* d = &c->descs[i - 1];
        char* v = c->dst + ((size_t)(start - 1) * c->ld_dst + d->dst_row_off) * es;
        const int64_t* I = d->idx + (size_t)(start - 1) * d->ld_idx;
        orc_pooled_sum(c->dtype, d->table, d->ld_table, d->dim, I, d->pool, d->ld_idx,
                       stop - start + 1, v, c->ld_dst, c->f16_fp32_acc);
    }
    return NULL;
}

void orc_maplookup_prealloc(int dtype, const orc_lookup_desc* descs, int32_t ntables,
                            int64_t batch, void* dst, int64_t ld_dst, int nthreads,
                            int worksize_div, int f16_fp32_acc) {
    if (ntables <= 0 || batch <= 0) return;
    if (worksize_div <= 0) worksize_div = 8;
    if (nthreads <= 0) nthreads = 1;
    prealloc_ctx c;
    c.dtype = dtype;
    c.descs = descs;
    c.ntables = ntables;
    c.batch = batch;
    c.dst = (char*)dst;
    c.ld_dst = ld_dst;
    c.worksize = 1 + (batch - 1) / worksize_div; /* cdiv(a, b), src/lookup.jl:301-302 */
    c.len = (int64_t)worksize_div * ntables;
    c.f16_fp32_acc = f16_fp32_acc;
    atomic_init(&c.count, 1);
    if (nthreads == 1) {
        prealloc_worker(&c);
        return;
    }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, prealloc_worker, &c);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
}

/* ------------------------------------------------------------------------- */
/* Indexer (src/utils.jl:88-314)                                              */
/* ------------------------------------------------------------------------- */

/* Insertion-ordered hash map int64 -> (order, count): the Dictionaries.jl
 * Dictionary the reference's SparseIndexer uses (ordering = insertion order). */
typedef struct {
    int64_t* slot_key;
    int64_t* slot_val; /* index into the insertion-ordered arrays, -1 = empty */
    int64_t cap;
    int64_t* keys; /* insertion order */
    int64_t* order;
    int64_t* count;
    int64_t n;
} ordmap;

static void ordmap_init(ordmap* m, int64_t expected) {
    int64_t cap = 16;
    while (cap < 2 * expected + 2) cap <<= 1;
    m->cap = cap;
    m->slot_key = (int64_t*)malloc(sizeof(int64_t) * cap);
    m->slot_val = (int64_t*)malloc(sizeof(int64_t) * cap);
    for (int64_t i = 0; i < cap; i++) m->slot_val[i] = -1;
    m->keys = (int64_t*)malloc(sizeof(int64_t) * (expected + 1));
    m->order = (int64_t*)malloc(sizeof(int64_t) * (expected + 1));
    m->count = (int64_t*)malloc(sizeof(int64_t) * (expected + 1));
    m->n = 0;
}

static void ordmap_free(ordmap* m) {
    free(m->slot_key);
    free(m->slot_val);
    free(m->keys);
    free(m->order);
    free(m->count);
}

static inline uint64_t hash64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* gettoken!: returns the insertion index of key, inserting it if absent. */
static int64_t ordmap_token(ordmap* m, int64_t key, int* found) {
    uint64_t h = hash64((uint64_t)key) & (uint64_t)(m->cap - 1);
    for (;;) {
        int64_t v = m->slot_val[h];
        if (v < 0) {
            m->slot_key[h] = key;
            m->slot_val[h] = m->n;
            m->keys[m->n] = key;
            m->order[m->n] = 0;
            m->count[m->n] = 0;
            *found = 0;
            return m->n++;
        }
        if (m->slot_key[h] == key) {
            *found = 1;
            return v;
        }
        h = (h + 1) & (uint64_t)(m->cap - 1);
    }
}

/* `columns(A)` (src/utils.jl:69-86): occurrence k of a P x B array is (bag j, entry i)
 * with i fastest; its gradient column is j.  A vector index is pool = 1. */
#define FOR_OCCURRENCES(body)                                      \
    for (int64_t j_ = 0; j_ < batch; j_++)                         \
        for (int32_t i_ = 0; i_ < pool; i_++) {                    \
            int64_t a_ = idx[(size_t)j_ * ld_idx + i_];            \
            int64_t bag_ = j_ + 1;                                 \
            body                                                   \
        }

int64_t orc_histogram(const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                      int64_t maxindex, int dense, int64_t* keys, int64_t* order,
                      int64_t* count) {
    int64_t n = (int64_t)pool * batch;
    if (dense) {
        /* unsafe_histogram!(::AbstractArray) src/utils.jl:154-167 */
        int64_t* ord = (int64_t*)calloc((size_t)maxindex + 1, sizeof(int64_t));
        int64_t* cnt = (int64_t*)calloc((size_t)maxindex + 1, sizeof(int64_t));
        int64_t o = 0;
        FOR_OCCURRENCES({
            (void)bag_;
            int64_t thisorder = ord[a_];
            int seen = thisorder != 0;
            thisorder = seen ? thisorder : o + 1;
            o = seen ? o : o + 1;
            ord[a_] = thisorder;
            cnt[a_] += 1;
            if (!seen) keys[thisorder - 1] = a_;
        })
        for (int64_t u = 0; u < o; u++) {
            order[u] = ord[keys[u]];
            count[u] = cnt[keys[u]];
        }
        free(ord);
        free(cnt);
        return o;
    }
    /* unsafe_histogram!(::AbstractDictionary) src/utils.jl:136-152 */
    ordmap m;
    ordmap_init(&m, n);
    int64_t o = 0;
    FOR_OCCURRENCES({
        (void)bag_;
        int found;
        int64_t t = ordmap_token(&m, a_, &found);
        if (found) {
            m.count[t] += 1;
        } else {
            o += 1;
            m.order[t] = o;
            m.count[t] = 1;
        }
    })
    for (int64_t u = 0; u < m.n; u++) {
        keys[u] = m.keys[u];
        order[u] = m.order[u];
        count[u] = m.count[u];
    }
    ordmap_free(&m);
    return o;
}

int64_t orc_index_build(const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                        int64_t maxindex, int dense, int64_t* cum_col, int64_t* cum_off,
                        int64_t* map) {
    int64_t n = (int64_t)pool * batch;
    int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* count = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t nnz = orc_histogram(idx, pool, ld_idx, batch, maxindex, dense, keys, order, count);

    /* prefixsum! src/utils.jl:170-239: cumulative[order] = (key, start), first-seen order */
    int64_t next = 1;
    for (int64_t u = 0; u < nnz; u++) {
        int64_t o = order[u] - 1;
        cum_col[o] = keys[u];
        cum_off[o] = count[u]; /* temporarily the count (dense flavour, loop 1) */
    }
    for (int64_t o = 0; o < nnz; o++) {
        int64_t c = cum_off[o];
        cum_off[o] = next;
        next += c;
    }
    cum_col[nnz] = 0;
    cum_off[nnz] = next;

    /* remap! src/utils.jl:242-272: map[next_offset - count] = dst_col, count -= 1 */
    int64_t* rem = (int64_t*)malloc(sizeof(int64_t) * (nnz + 1));
    for (int64_t o = 0; o < nnz; o++) rem[o] = cum_off[o + 1] - cum_off[o];
    if (dense) {
        int64_t* ordof = (int64_t*)calloc((size_t)maxindex + 1, sizeof(int64_t));
        for (int64_t o = 0; o < nnz; o++) ordof[cum_col[o]] = o;
        FOR_OCCURRENCES({
            int64_t o = ordof[a_];
            map[cum_off[o + 1] - rem[o] - 1] = bag_;
            rem[o] -= 1;
        })
        free(ordof);
    } else {
        ordmap m;
        ordmap_init(&m, nnz);
        for (int64_t o = 0; o < nnz; o++) {
            int found;
            int64_t t = ordmap_token(&m, cum_col[o], &found);
            m.order[t] = o;
        }
        FOR_OCCURRENCES({
            int found;
            int64_t t = ordmap_token(&m, a_, &found);
            int64_t o = m.order[t];
            map[cum_off[o + 1] - rem[o] - 1] = bag_;
            rem[o] -= 1;
        })
        ordmap_free(&m);
    }
    free(rem);
    free(keys);
    free(order);
    free(count);
    return nnz;
}

/* ------------------------------------------------------------------------- */
/* update!                                                                    */
/* ------------------------------------------------------------------------- */

void orc_update_specialized_f32(float* table, int64_t ld_table, int32_t dim, const float* delta,
                                int64_t ld_delta, const int64_t* cum_col, const int64_t* cum_off,
                                int64_t ubegin, int64_t uend, const int64_t* map, float alpha) {
    float acc[4096];
    float nalpha = -alpha; /* alpha = -convert(T, alpha0)  (src/sparseupdate.jl:108) */
    for (int64_t e = ubegin; e < uend; e++) {
        int64_t k = cum_col[e];
        int64_t start = cum_off[e];
        int64_t stop = cum_off[e + 1] - 1;
        float* w = table + (size_t)(k - 1) * ld_table;
        for (int32_t k0 = 0; k0 < dim; k0 += 4096) {
            int32_t kn = dim - k0 < 4096 ? dim - k0 : 4096;
            for (int32_t f = 0; f < kn; f++) acc[f] = 0.0f; /* zero(Tiled) */
            for (int64_t i = start; i <= stop; i++) {
                const float* g = delta + (size_t)(map[i - 1] - 1) * ld_delta + k0;
                for (int32_t f = 0; f < kn; f++) acc[f] += g[f];
            }
            /* store(muladd(alpha, accum, load(dest)))  (src/sparseupdate.jl:122-127) */
            for (int32_t f = 0; f < kn; f++) w[k0 + f] = fmaf(nalpha, acc[f], w[k0 + f]);
        }
    }
}

void orc_update_generic_f32(float* table, int64_t ld_table, int32_t dim, const float* delta,
                            int64_t ld_delta, const int64_t* cum_col, const int64_t* cum_off,
                            int64_t ubegin, int64_t uend, const int64_t* map, double alpha,
                            int alpha_f64) {
    float* scratch = (float*)malloc(sizeof(float) * (size_t)(dim > 0 ? dim : 1));
    float a32 = (float)alpha;
    for (int64_t e = ubegin; e < uend; e++) {
        int64_t k = cum_col[e];
        int64_t start = cum_off[e];
        int64_t stop = cum_off[e + 1] - 1;
        for (int32_t f = 0; f < dim; f++) scratch[f] = 0.0f; /* zero!(scratchspace) */
        for (int64_t i = start; i <= stop; i++) {
            const float* g = delta + (size_t)(map[i - 1] - 1) * ld_delta;
            for (int32_t f = 0; f < dim; f++) scratch[f] += g[f];
        }
        float* w = table + (size_t)(k - 1) * ld_table;
        /* f(x, y) = x - alpha * y  (src/sparseupdate.jl:88) */
        if (alpha_f64)
            for (int32_t f = 0; f < dim; f++)
                w[f] = (float)((double)w[f] - alpha * (double)scratch[f]);
        else
            for (int32_t f = 0; f < dim; f++) w[f] = w[f] - a32 * scratch[f];
    }
    free(scratch);
}

void orc_sgd_f32(const orc_update_desc* d, double eta, int fused, int dense_indexer) {
    int64_t n = (int64_t)d->pool * d->batch;
    if (n <= 0) return;
    int64_t* cum_col = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* cum_off = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* map = (int64_t*)malloc(sizeof(int64_t) * n);
    int64_t U = orc_index_build(d->idx, d->pool, d->ld_idx, d->batch, d->nrows, dense_indexer,
                                cum_col, cum_off, map);
    float eta32 = (float)eta; /* convert(eltype(table), opt.eta)  (src/sparseupdate.jl:173) */
    if (fused)
        orc_update_specialized_f32((float*)d->table, d->ld_table, d->dim,
                                   (const float*)d->delta, d->ld_delta, cum_col, cum_off, 0, U,
                                   map, eta32);
    else
        orc_update_generic_f32((float*)d->table, d->ld_table, d->dim, (const float*)d->delta,
                               d->ld_delta, cum_col, cum_off, 0, U, map, (double)eta32, 0);
    free(cum_col);
    free(cum_off);
    free(map);
}

/* ------------------------------------------------------------------------- */
/* update of Float64 / Float16 / BFloat16 tables                              */
/* ------------------------------------------------------------------------- */
/* The same two reference kernels (src/sparseupdate.jl:57-129) evaluated in the
 * table's element type T, with an accumulator type C: C = T for Float64 and for
 * Float16 (Julia Float16 arithmetic: every add / mul / sub rounded to half), C =
 * Float32 for BFloat16 and for Float16 with acc32 (ET_FLAG_F16_FP32_ACC).  alpha is
 * convert(T, alpha0) (then held in C); the fused path is
 * muladd(-alpha, acc, w) = T(fma32(-alpha, acc, w)) for 16-bit T (SIMD.jl's half
 * muladd is promoted to Float32) and fma for Float64; the generic path is x - alpha*y
 * in C, or in Float64 (alpha_f64, the multi-table path) followed by one conversion
 * (16-bit: Float64 -> Float32 -> bf16 for BFloat16, correctly rounded for Float16).
 * Values travel as doubles that are exact in their type. */

/* Correctly rounded double -> binary16 (ties to even). */
uint16_t orc_f64_to_f16(double v) {
    uint64_t bits;
    memcpy(&bits, &v, 8);
    uint16_t sign = (uint16_t)((bits >> 48) & 0x8000u);
    double m = fabs(v);
    if (isnan(v)) return (uint16_t)(sign | 0x7e00u);
    if (m >= 65520.0) return (uint16_t)(sign | 0x7c00u);
    int e;
    frexp(m, &e); /* m = f * 2^e, f in [0.5, 1) => floor(log2 m) = e - 1 */
    int E = e - 1 < -14 ? -14 : e - 1;
    double k = rint(ldexp(m, 10 - E)); /* exact scaling, RNE to an integer */
    if (k >= 2048.0) {
        k = 1024.0;
        E += 1;
    }
    uint32_t K = (uint32_t)k;
    if (K < 1024) return (uint16_t)(sign | K); /* subnormal (E == -14) or zero */
    return (uint16_t)(sign | ((uint32_t)(E + 15) << 10) | (K - 1024));
}

static inline double ty_load(int dtype, const void* p, size_t i) {
    switch (dtype) {
        case ORC_F32: return ((const float*)p)[i];
        case ORC_F64: return ((const double*)p)[i];
        case ORC_F16: return orc_f16_to_f32(((const uint16_t*)p)[i]);
        case ORC_BF16: return orc_bf16_to_f32(((const uint16_t*)p)[i]);
    }
    return 0.0;
}

/* double (exact in float for 16-bit types) -> T */
static inline void ty_store_f(int dtype, void* p, size_t i, float v) {
    switch (dtype) {
        case ORC_F32: ((float*)p)[i] = v; break;
        case ORC_F16: ((uint16_t*)p)[i] = orc_f32_to_f16(v); break;
        case ORC_BF16: ((uint16_t*)p)[i] = orc_f32_to_bf16(v); break;
    }
}

static inline void ty_store_d(int dtype, void* p, size_t i, double v) {
    switch (dtype) {
        case ORC_F32: ((float*)p)[i] = (float)v; break;
        case ORC_F64: ((double*)p)[i] = v; break;
        case ORC_F16: ((uint16_t*)p)[i] = orc_f64_to_f16(v); break;
        case ORC_BF16: ((uint16_t*)p)[i] = orc_f32_to_bf16((float)v); break;
    }
}

/* accumulator kind: 0 = Float64, 1 = Float32, 2 = Float16 */
static inline int ty_acc(int dtype, int acc32) {
    if (dtype == ORC_F64) return 0;
    if (dtype == ORC_F16 && !acc32) return 2;
    return 1;
}

static inline double acc_add(int ak, double a, double x) {
    if (ak == 0) return a + x;
    if (ak == 1) return (double)((float)a + (float)x);
    return orc_f16_to_f32(orc_f32_to_f16((float)a + (float)x));
}

/* convert(T, alpha0) held in the accumulator type */
double orc_convert_eta(int dtype, double eta) {
    switch (dtype) {
        case ORC_F32: return (float)eta;
        case ORC_F64: return eta;
        case ORC_F16: return orc_f16_to_f32(orc_f64_to_f16(eta));
        case ORC_BF16: return orc_bf16_to_f32(orc_f32_to_bf16((float)eta));
    }
    return eta;
}

void orc_update_typed(int dtype, int acc32, void* table, int64_t ld_table, int32_t dim,
                      const void* delta, int64_t ld_delta, const int64_t* cum_col,
                      const int64_t* cum_off, int64_t ubegin, int64_t uend, const int64_t* map,
                      double alpha, int fused, int alpha_f64) {
    const int ak = ty_acc(dtype, acc32);
    double* acc = (double*)malloc(sizeof(double) * (size_t)(dim > 0 ? dim : 1));
    for (int64_t e = ubegin; e < uend; e++) {
        int64_t k = cum_col[e];
        int64_t start = cum_off[e];
        int64_t stop = cum_off[e + 1] - 1;
        for (int32_t f = 0; f < dim; f++) acc[f] = 0.0;
        for (int64_t i = start; i <= stop; i++) {
            size_t g = (size_t)(map[i - 1] - 1) * ld_delta;
            for (int32_t f = 0; f < dim; f++)
                acc[f] = acc_add(ak, acc[f], ty_load(dtype, delta, g + f));
        }
        size_t w0 = (size_t)(k - 1) * ld_table;
        for (int32_t f = 0; f < dim; f++) {
            double w = ty_load(dtype, table, w0 + f);
            if (fused) {
                if (ak == 0)
                    ty_store_d(dtype, table, w0 + f, fma(-alpha, acc[f], w));
                else
                    ty_store_f(dtype, table, w0 + f,
                               fmaf(-(float)alpha, (float)acc[f], (float)w));
            } else if (alpha_f64) {
                ty_store_d(dtype, table, w0 + f, w - alpha * acc[f]);
            } else if (ak == 0) {
                ty_store_d(dtype, table, w0 + f, w - alpha * acc[f]);
            } else if (ak == 1) {
                ty_store_f(dtype, table, w0 + f, (float)w - (float)alpha * (float)acc[f]);
            } else {
                float t = orc_f16_to_f32(orc_f32_to_f16((float)alpha * (float)acc[f]));
                ty_store_f(dtype, table, w0 + f, (float)w - t);
            }
        }
    }
    free(acc);
}

/* orc_sgd_f32 for any table type (single table, eta converted to T). */
void orc_sgd_typed(const orc_update_desc* d, int dtype, int acc32, double eta, int fused,
                   int dense_indexer) {
    int64_t n = (int64_t)d->pool * d->batch;
    if (n <= 0) return;
    int64_t* cum_col = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* cum_off = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
    int64_t* map = (int64_t*)malloc(sizeof(int64_t) * n);
    int64_t U = orc_index_build(d->idx, d->pool, d->ld_idx, d->batch, d->nrows, dense_indexer,
                                cum_col, cum_off, map);
    orc_update_typed(dtype, acc32, d->table, d->ld_table, d->dim, d->delta, d->ld_delta, cum_col,
                     cum_off, 0, U, map, orc_convert_eta(dtype, eta), fused, 0);
    free(cum_col);
    free(cum_off);
    free(map);
}

typedef struct {
    const orc_update_desc* descs;
    int32_t ntables;
    int dtype, acc32;
    double eta;
    const int32_t* fused;
    int num_splits;
    int64_t** cum_col;
    int64_t** cum_off;
    int64_t** map;
    int64_t* nunique;
    atomic_long next_table; /* phase 1 */
    atomic_long count;      /* phase 2 */
    pthread_barrier_t barrier;
} multi_ctx;

static void* multi_worker(void* arg) {
    multi_ctx* c = (multi_ctx*)arg;
    /* Phase 1: index! every table (src/sparseupdate.jl:210-213) */
    for (;;) {
        long t = atomic_fetch_add(&c->next_table, 1);
        if (t >= c->ntables) break;
        const orc_update_desc* d = &c->descs[t];
        c->nunique[t] = orc_index_build(d->idx, d->pool, d->ld_idx, d->batch, d->nrows, 0,
                                        c->cum_col[t], c->cum_off[t], c->map[t]);
    }
    pthread_barrier_wait(&c->barrier);
    /* Phase 2: atomic queue over num_splits * ntables items (:207-237) */
    long len = (long)c->num_splits * c->ntables;
    for (;;) {
        long k = atomic_fetch_add(&c->count, 1);
        if (k > len) break;
        long i = (k - 1) / c->num_splits + 1; /* table */
        long j = (k - 1) % c->num_splits + 1; /* split */
        const orc_update_desc* d = &c->descs[i - 1];
        /* IndexerView(I, num_splits, j)  (src/utils.jl:325-333) */
        int64_t len_c = c->nunique[i - 1] + 1;
        int64_t split = 1 + (len_c - 1) / c->num_splits;
        int64_t start = (j - 1) * split + 1;
        int64_t stop = j * split + 1 < len_c ? j * split + 1 : len_c;
        int64_t ubegin = start - 1, uend = stop - 1; /* entries start..stop-1, 0-based */
        if (uend <= ubegin) continue;
        if (c->dtype != ORC_F32)
            orc_update_typed(c->dtype, c->acc32, d->table, d->ld_table, d->dim, d->delta,
                             d->ld_delta, c->cum_col[i - 1], c->cum_off[i - 1], ubegin, uend,
                             c->map[i - 1],
                             c->fused[i - 1] ? orc_convert_eta(c->dtype, c->eta) : c->eta,
                             c->fused[i - 1], !c->fused[i - 1]);
        else if (c->fused[i - 1])
            orc_update_specialized_f32((float*)d->table, d->ld_table, d->dim,
                                       (const float*)d->delta, d->ld_delta, c->cum_col[i - 1],
                                       c->cum_off[i - 1], ubegin, uend, c->map[i - 1],
                                       (float)c->eta);
        else
            orc_update_generic_f32((float*)d->table, d->ld_table, d->dim,
                                   (const float*)d->delta, d->ld_delta, c->cum_col[i - 1],
                                   c->cum_off[i - 1], ubegin, uend, c->map[i - 1], c->eta, 1);
    }
    return NULL;
}

void orc_sgd_multi_f32(const orc_update_desc* descs, int32_t ntables, double eta,
                       const int32_t* fused, int num_splits, int nthreads) {
    orc_sgd_multi_typed(descs, ntables, ORC_F32, 0, eta, fused, num_splits, nthreads);
}

void orc_sgd_multi_typed(const orc_update_desc* descs, int32_t ntables, int dtype, int acc32,
                         double eta, const int32_t* fused, int num_splits, int nthreads) {
    if (ntables <= 0) return;
    if (nthreads <= 0) nthreads = 1;
    if (num_splits <= 0) num_splits = 4;
    multi_ctx c;
    c.dtype = dtype;
    c.acc32 = acc32;
    c.descs = descs;
    c.ntables = ntables;
    c.eta = eta;
    c.fused = fused;
    c.num_splits = num_splits;
    c.cum_col = (int64_t**)malloc(sizeof(int64_t*) * ntables);
    c.cum_off = (int64_t**)malloc(sizeof(int64_t*) * ntables);
    c.map = (int64_t**)malloc(sizeof(int64_t*) * ntables);
    c.nunique = (int64_t*)calloc(ntables, sizeof(int64_t));
    for (int t = 0; t < ntables; t++) {
        int64_t n = (int64_t)descs[t].pool * descs[t].batch;
        c.cum_col[t] = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
        c.cum_off[t] = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
        c.map[t] = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    }
    atomic_init(&c.next_table, 0);
    atomic_init(&c.count, 1);
    pthread_barrier_init(&c.barrier, NULL, (unsigned)nthreads);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, multi_worker, &c);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    pthread_barrier_destroy(&c.barrier);
    free(th);
    for (int t = 0; t < ntables; t++) {
        free(c.cum_col[t]);
        free(c.cum_off[t]);
        free(c.map[t]);
    }
    free(c.cum_col);
    free(c.cum_off);
    free(c.map);
    free(c.nunique);
}

/* ------------------------------------------------------------------------- */
/* Synthetic data (bit-identical to the HIP fills)                            */
/* ------------------------------------------------------------------------- */

static inline uint64_t fill_hash(uint64_t seed, uint64_t i) {
    return hash64(seed * 0xD1B54A32D192ED03ull + i);
}

typedef struct {
    int dtype;
    void* dst;
    int64_t n;
    uint64_t seed, offset;
    double lo, hi;
    int64_t* idx;
    int64_t nrows;
    int nthreads, tid;
} fill_ctx;

static void fill_range(const fill_ctx* c, int64_t b, int64_t e) {
    double span = c->hi - c->lo;
    for (int64_t i = b; i < e; i++) {
        uint64_t h = fill_hash(c->seed, c->offset + (uint64_t)i);
        if (c->idx) {
            unsigned __int128 p = (unsigned __int128)h * (unsigned __int128)(uint64_t)c->nrows;
            c->idx[i] = 1 + (int64_t)(uint64_t)(p >> 64);
            continue;
        }
        double u = (double)(h >> 40) * (1.0 / 16777216.0);
        double v = fma(span, u, c->lo);
        switch (c->dtype) {
            case ORC_F32: ((float*)c->dst)[i] = (float)v; break;
            case ORC_F64: ((double*)c->dst)[i] = v; break;
            case ORC_F16: ((uint16_t*)c->dst)[i] = orc_f32_to_f16((float)v); break;
            case ORC_BF16: ((uint16_t*)c->dst)[i] = orc_f32_to_bf16((float)v); break;
            case ORC_I32: ((int32_t*)c->dst)[i] = (int32_t)floor(v); break;
            case ORC_I64: ((int64_t*)c->dst)[i] = (int64_t)floor(v); break;
        }
    }
}

static void* fill_worker(void* arg) {
    fill_ctx* c = (fill_ctx*)arg;
    int64_t per = (c->n + c->nthreads - 1) / c->nthreads;
    int64_t b = per * c->tid, e = b + per < c->n ? b + per : c->n;
    if (b < e) fill_range(c, b, e);
    return NULL;
}

static void fill_run(fill_ctx* base, int nthreads) {
    if (nthreads <= 1 || base->n < (1 << 20)) {
        fill_range(base, 0, base->n);
        return;
    }
    fill_ctx* cs = (fill_ctx*)malloc(sizeof(fill_ctx) * nthreads);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) {
        cs[t] = *base;
        cs[t].nthreads = nthreads;
        cs[t].tid = t;
        pthread_create(&th[t], NULL, fill_worker, &cs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(cs);
    free(th);
}

void orc_fill_uniform(int dtype, void* dst, int64_t n, uint64_t seed, uint64_t offset,
                      double lo, double hi, int nthreads) {
    fill_ctx c = {dtype, dst, n, seed, offset, lo, hi, NULL, 0, 1, 0};
    fill_run(&c, nthreads);
}

void orc_fill_index_uniform(int64_t* idx, int64_t n, int64_t nrows, uint64_t seed,
                            uint64_t offset, int nthreads) {
    fill_ctx c = {ORC_I64, NULL, n, seed, offset, 0, 0, idx, nrows, 1, 0};
    fill_run(&c, nthreads);
}
