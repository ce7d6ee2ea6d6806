/*
 * embtab_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference algorithms of darchr/EmbeddingTables.jl
 * (Julia; no Julia toolchain exists in this image, so the reference itself
 * cannot be run — see DESIGN.md "Oracle").  It is the parity checker for the
 * HIP engine and the multithreaded CPU baseline ("kind": "port") of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product path (embeddingtables.jl_amd/) never does.
 *
 * Pinned by the reference's own known-answer tests (README.md:32-73,
 * README.md:115-159, README.md:191-228, test/misc.jl:33-110), committed as
 * fixtures under tests/golden/.
 *
 * Layout conventions are those of include/embtab.h (column-major, 1-based
 * Int64 indices, leading dimensions in elements).
 */
#ifndef EMBTAB_ORACLE_H
#define EMBTAB_ORACLE_H

#include <stdint.h>

#define ORC_F32 0
#define ORC_F16 1
#define ORC_F64 2
#define ORC_I32 3
#define ORC_I64 4
#define ORC_BF16 5 /* not a reference type: fp32 accumulation, one RNE rounding */

/* Same memory layout as et_lookup_desc / et_update_desc in include/embtab.h. */
typedef struct orc_lookup_desc {
    const void* table;
    int64_t ld_table;
    int64_t nrows;
    int32_t dim;
    int32_t pool;
    const int64_t* idx;
    int64_t ld_idx;
    int64_t dst_row_off;
} orc_lookup_desc;

typedef struct orc_update_desc {
    void* table;
    int64_t ld_table;
    int64_t nrows;
    int32_t dim;
    int32_t pool;
    const void* delta;
    int64_t ld_delta;
    const int64_t* idx;
    int64_t ld_idx;
    int64_t batch;
} orc_update_desc;

int orc_elsize(int dtype);

/* fp16 <-> fp32 (round to nearest even), the conversions Julia's Float16 uses. */
uint16_t orc_f32_to_f16(float f);
float orc_f16_to_f32(uint16_t h);
/* bfloat16 <-> fp32 (round to nearest even; NaN stays a quiet NaN). */
uint16_t orc_f32_to_bf16(float f);
float orc_bf16_to_f32(uint16_t h);

/* src/lookup.jl:51-87: non-reducing lookup (bit copy). */
void orc_gather(int dtype, const void* table, int64_t ld_table, int32_t dim, const int64_t* idx,
                int64_t n, void* dst, int64_t ld_dst);

/* src/lookup.jl:108-165: pooled sum, sequential in pool order from the first row. */
void orc_pooled_sum(int dtype, const void* table, int64_t ld_table, int32_t dim,
                    const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch, void* dst,
                    int64_t ld_dst, int f16_fp32_acc);

/* src/lookup.jl:316-371: Preallocation maplookup! with the atomic work queue of
 * worksize_div * ntables items, (chunk, table) = _divrem_index(k, ntables). */
void orc_maplookup_prealloc(int dtype, const orc_lookup_desc* descs, int32_t ntables,
                            int64_t batch, void* dst, int64_t ld_dst, int nthreads,
                            int worksize_div, int f16_fp32_acc);

/* src/utils.jl:131-167 histogram! over the occurrences of a P x B index array (Dict
 * flavour when dense == 0, dense array flavour otherwise).  Writes the distinct keys in
 * first-seen order and their (order, count); returns the number of distinct keys. */
int64_t orc_histogram(const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                      int64_t maxindex, int dense, int64_t* keys, int64_t* order,
                      int64_t* count);

/* src/utils.jl:306-314 index!: cumulative (U+1 entries, 1-based, first-seen order,
 * terminator (0, n+1)) and map (n entries, gradient column = bag, 1-based).
 * Returns U. */
int64_t orc_index_build(const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                        int64_t maxindex, int dense, int64_t* cum_col, int64_t* cum_off,
                        int64_t* map);

/* src/sparseupdate.jl:97-129 _update_specialized_impl! over cumulative entries
 * [ubegin, uend) (0-based), alpha already converted to Float32:
 *   acc = 0; acc += delta[:, map[k]] ...; w = fma(-alpha, acc, w). */
void orc_update_specialized_f32(float* table, int64_t ld_table, int32_t dim, const float* delta,
                                int64_t ld_delta, const int64_t* cum_col, const int64_t* cum_off,
                                int64_t ubegin, int64_t uend, const int64_t* map, float alpha);

/* src/sparseupdate.jl:57-95 _update_generic_impl!: scratch sum then x - alpha*y,
 * unfused; alpha_f64 != 0 evaluates x - alpha*y in Float64 (the multi-table path
 * passes opt.eta unconverted, src/sparseupdate.jl:232). */
void orc_update_generic_f32(float* table, int64_t ld_table, int32_t dim, const float* delta,
                            int64_t ld_delta, const int64_t* cum_col, const int64_t* cum_off,
                            int64_t ubegin, int64_t uend, const int64_t* map, double alpha,
                            int alpha_f64);

/* src/sparseupdate.jl:160-178 update!(::Descent, table, grad): index! then the
 * specialized (fused != 0) or generic (fused == 0) update with eta converted to Float32. */
void orc_sgd_f32(const orc_update_desc* d, double eta, int fused, int dense_indexer);

/* src/sparseupdate.jl:199-238 multi-table update!: phase 1 indexes every table on
 * `nthreads` threads, phase 2 runs a queue of num_splits * ntables items
 * (table, split) = _divrem_index(k, num_splits) over IndexerView ranges
 * (src/utils.jl:325-333).  fused[t] selects the specialized path per table; the
 * generic path sees eta as Float64. */
void orc_sgd_multi_f32(const orc_update_desc* descs, int32_t ntables, double eta,
                       const int32_t* fused, int num_splits, int nthreads);

/* Float64 / Float16 / BFloat16 tables (acc32: Float16 summed in Float32), see
 * embtab_oracle.c "update of Float64 / Float16 / BFloat16 tables" for the arithmetic. */
uint16_t orc_f64_to_f16(double v);
double orc_convert_eta(int dtype, double eta);
void orc_update_typed(int dtype, int acc32, void* table, int64_t ld_table, int32_t dim,
                      const void* delta, int64_t ld_delta, const int64_t* cum_col,
                      const int64_t* cum_off, int64_t ubegin, int64_t uend, const int64_t* map,
                      double alpha, int fused, int alpha_f64);
void orc_sgd_typed(const orc_update_desc* d, int dtype, int acc32, double eta, int fused,
                   int dense_indexer);
void orc_sgd_multi_typed(const orc_update_desc* descs, int32_t ntables, int dtype, int acc32,
                         double eta, const int32_t* fused, int num_splits, int nthreads);

/* Counter-based synthetic data, identical bits to et_fill_uniform /
 * et_fill_index_uniform of the HIP library. */
void orc_fill_uniform(int dtype, void* dst, int64_t n, uint64_t seed, uint64_t offset,
                      double lo, double hi, int nthreads);
void orc_fill_index_uniform(int64_t* idx, int64_t n, int64_t nrows, uint64_t seed,
                            uint64_t offset, int nthreads);

/* Wall-clock seconds (CLOCK_MONOTONIC), for the CPU baseline. */
double orc_now(void);

#endif
