/*
 * embtab.h — C ABI of libembtab_hip.so, the MI355X (gfx950) embedding-table engine.
 *
 * This is the drop-in boundary for the hot path of darchr/EmbeddingTables.jl:
 * the Julia package's `lookup!`, `maplookup!(::PreallocationStrategy, …)` and
 * `update!(::Descent, …)` methods are re-targeted (by a thin `ccall` layer, see
 * INTEGRATION.md) onto the entry points below.  Every entry point:
 *
 *   - takes plain pointers and sizes only (no torch / no Julia types);
 *   - takes DEVICE pointers for every array argument, except arrays of
 *     descriptors (`et_lookup_desc*`, `et_update_desc*`), which live in HOST
 *     memory and are copied into the kernel argument segment at launch;
 *   - is stream-ordered on the caller's `hipStream_t` (passed as `void*`;
 *     NULL = the legacy default stream) and never synchronises the device,
 *     allocates or frees memory, so it may be captured into a hipGraph;
 *   - returns an `int` status (ET_OK = 0, negative = error).  The message for
 *     the last error of the calling thread is `et_last_error()`.
 *
 * Memory layout (identical to the reference, column-major Julia arrays):
 *   - a table is a D x R matrix whose column `r` (1-based) — one embedding
 *     vector of D contiguous elements — starts at `table + (r-1)*ld_table`
 *     (reference `columnpointer`, src/simple.jl:52-55, src/EmbeddingTables.jl:83-85);
 *   - index arrays are Int64 and 1-BASED, as in Julia; a P x B index matrix
 *     (pool P, batch B) stores bag j's P entries at `idx + j*ld_idx`;
 *   - outputs / gradients are D x B column-major with leading dimension `ld`.
 *   - all leading dimensions are in ELEMENTS, not bytes.
 *
 * Out-of-range indices are undefined behaviour in the reference
 * (`@inbounds`, src/lookup.jl).  Here they never fault the GPU: a bad index
 * contributes a zero row (lookup) or is skipped (update), and is counted in a
 * device-side error word readable with `et_check_errors`.
 */
#ifndef EMBTAB_H
#define EMBTAB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ET_ABI_VERSION 9

/* Status codes. */
#define ET_OK 0
#define ET_ERR_ARG (-1)         /* invalid argument (message in et_last_error) */
#define ET_ERR_HIP (-2)         /* a HIP runtime call failed */
#define ET_ERR_WORKSPACE (-3)   /* workspace missing or too small */
#define ET_ERR_UNSUPPORTED (-4) /* dtype / mode not implemented */

/* Element types of tables, outputs and gradients. */
#define ET_F32 0
#define ET_F16 1
#define ET_F64 2
#define ET_I32 3
#define ET_I64 4
#define ET_BF16 5 /* bfloat16 tables: pooled sums accumulate in fp32 and round once (RNE);
                     not a reference type (Julia's reference never uses BFloat16) */

/* Flags (bitwise OR). */
#define ET_FLAG_NONTEMPORAL 1u   /* non-temporal stores of outputs / updated rows
                                    (reference Val{Nontemporal}, src/sparseupdate.jl:165) */
#define ET_FLAG_F16_FP32_ACC 2u  /* F16 pooled sums (and F16 SGD sums) accumulate in fp32
                                    and round once; default F16 mode rounds to fp16 after
                                    every add like Julia Float16 arithmetic */
#define ET_FLAG_EXACT_UPDATE 4u  /* sparse SGD: never split a hot row's occurrence list, so
                                    every row's gradient is summed serially in occurrence
                                    order (bit-identical to the reference, slower on skew) */
#define ET_FLAG_SGD_UNFUSED 8u   /* sparse SGD: w - eta*acc with two roundings, the
                                    reference's generic path (src/sparseupdate.jl:57-95);
                                    default is fma(-eta, acc, w), its specialized path
                                    (src/sparseupdate.jl:97-129) */
#define ET_FLAG_SGD_F64_ALPHA 16u /* with ET_FLAG_SGD_UNFUSED: evaluate w - eta*acc in
                                    Float64, as the multi-table generic path does with the
                                    unconverted opt.eta (src/sparseupdate.jl:232) */
#define ET_FLAG_SGD_INDEX_ONLY 32u /* sparse SGD, phase 1 of 2: only the index work (keys,
                                    sort, segments, chunk records) into the workspace; reads
                                    idx, never delta or the tables (delta may be NULL) — the
                                    reference's "index all" phase, src/sparseupdate.jl:210-213 */
#define ET_FLAG_SGD_APPLY_ONLY 64u /* sparse SGD, phase 2 of 2: the gradient sums and row
                                    updates from a workspace that an INDEX_ONLY call with the
                                    same descriptors, flags and workspace filled earlier in
                                    stream order ("update all", :216-237); idx is not read
                                    again, so it may be refilled once phase 1 is done */
#define ET_FLAG_SGD_HOT_PASS 128u /* sparse SGD, non-exact Float32 dim-128 tables with pool
                                    <= 32: the longest occurrence lists (up to 120 columns
                                    per table, by a log2 length threshold) are summed
                                    bag-major over 1024-bag windows instead of by per-
                                    occurrence gathers (deterministic; EXPERIMENTAL, slower
                                    today — DESIGN.md §7) */
#define ET_FLAG_EXACT_IF_FAST 256u /* sparse SGD, the bindings' default: since ABI v9 the
                                    same as ET_FLAG_EXACT_UPDATE — the exact mode's serial-
                                    chain path covers every element type and gradient size
                                    up to a batch of 2^27 - 1 bags (ABI v8 resolved it to the
                                    split mode for non-Float32 tables and for batch *
                                    ld_delta >= 2^30).  A batch of 2^27 bags or more is still
                                    exact but sums every column in one chunk (one wave per
                                    column: slow for hot columns) */

/* Occurrences per chunk of the non-exact sparse SGD: a column with more occurrences than
 * this is summed as ordered partial sums of ET_SGD_CHUNK consecutive occurrences (so a
 * column with at most ET_SGD_CHUNK occurrences is always the serial, bit-identical sum).
 * 256 measured 2% faster than 512 and 7% faster than 1024 on BASELINE config 4. */
#define ET_SGD_CHUNK 256

/* Tables per launch carried in the kernel-argument segment; longer lists are
 * split into several launches by the library. */
#define ET_MAX_TABLES_PER_LAUNCH 32

/* ABI version compiled into the library (== ET_ABI_VERSION). */
int et_abi_version(void);

/* Message of the last failed call on this thread ("" if none). */
const char* et_last_error(void);

/* Non-reducing gather: dst[:, j] = table[:, idx[j]] for j in 0..n-1
 * (bit copy for every dtype).
 * Replaces lookup!(dst, A, I::AbstractVector) — reference src/lookup.jl:51-67
 * (lookup_generic!), :70-87 (lookup_static! SVector) and dispatch :90-102. */
int et_gather(int dtype, const void* table, int64_t ld_table, int64_t nrows, int32_t dim,
              const int64_t* idx, int64_t n, void* dst, int64_t ld_dst, uint32_t flags,
              void* stream);

/* Reducing (pooled-sum) lookup: dst[:, j] = sum_{i=0..pool-1} table[:, idx[j*ld_idx + i]],
 * accumulated sequentially in pool order starting from the first row (pool == 0
 * writes zeros).
 * Replaces lookup!(dst, A, I::AbstractMatrix) — reference src/lookup.jl:108-132
 * (lookup_generic!), :134-165 (lookup_static_inner / lookup_static! TiledSIMD) and
 * dispatch :167-182. */
int et_pooled_sum(int dtype, const void* table, int64_t ld_table, int64_t nrows, int32_t dim,
                  const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch, void* dst,
                  int64_t ld_dst, uint32_t flags, void* stream);

/* One table of a fused multi-table lookup. */
typedef struct et_lookup_desc {
    const void* table;   /* device pointer to column 1 of the table */
    int64_t ld_table;    /* elements between consecutive columns (>= dim) */
    int64_t nrows;       /* number of columns R (embeddings) in the table */
    int32_t dim;         /* feature size D */
    int32_t pool;        /* P: indices per bag; 1 for a vector (non-reducing) index */
    const int64_t* idx;  /* device pointer, 1-based Int64, bag j at idx + j*ld_idx */
    int64_t ld_idx;      /* elements between consecutive bags' index lists */
    int64_t dst_row_off; /* first row of this table's block in dst (prependrows + sum of
                            previous tables' dims) */
    int64_t cols_per_page; /* 0: contiguous table.  > 0: a PAGED table (the reference's
                            SplitEmbedding, src/split.jl:3-86): `table` is a device array of
                            page pointers, column r (1-based) lives in page (r-1)/cols_per_page
                            at column (r-1)%cols_per_page, ld_table apart within a page;
                            every page pointer must be 16-byte aligned (hipMalloc gives 256)
                            when ld_table * elsize is a multiple of 16 bytes; otherwise the
                            generic (element-aligned) kernels run.  cols_per_page = 1 is a
                            COLUMN-POINTER table — `table` holds one pointer per column, any
                            layout — the form any `columnpointer`-only table type takes
                            (README.md:288-307); ld_table is then only that alignment switch */
} et_lookup_desc;

/* Fused lookup + concat (PreallocationStrategy):
 * dst[desc[t].dst_row_off + (0:dim_t-1), j] = lookup(table_t, idx_t)[:, j] for every
 * table t and bag j, written in place into the (ld_dst x batch) destination.
 * Rows of dst not covered by any table (the prepended rows) are not touched.
 * `descs` is a HOST array of `ntables` descriptors.
 * Replaces maplookup!(::PreallocationStrategy, dst, tables, I) — reference
 * src/lookup.jl:316-371 (and maplookup :305-314 once dst is allocated). */
int et_maplookup_prealloc(int dtype, const et_lookup_desc* descs, int32_t ntables,
                          int64_t batch, void* dst, int64_t ld_dst, uint32_t flags,
                          void* stream);

/* et_maplookup_prealloc with a caller-owned QUEUE BLOCK (ABI v9): `queue` is
 * ET_LOOKUP_QUEUE_BYTES of 16-byte aligned device memory, ZERO before its first use; the
 * multi-table launch then takes its work items from per-XCD queues in that block (an XCD
 * that finishes its own items takes over another's, ~1% faster on BASELINE config 3) and
 * leaves the block zero again when it completes.  A block may serve any number of calls
 * that are ordered with each other (one stream, a captured and replayed HIP graph), never
 * two calls that may run at the same time.  queue == NULL is et_maplookup_prealloc (the
 * static XCD stripe schedule).  Results are identical either way. */
#define ET_LOOKUP_QUEUE_BYTES 128
int et_maplookup_prealloc_q(int dtype, const et_lookup_desc* descs, int32_t ntables,
                            int64_t batch, void* dst, int64_t ld_dst, uint32_t flags, void* queue,
                            void* stream);

/* PreallocationStrategy{U} with a destination of another floating type than the
 * tables (src/lookup.jl:284-315: `similar(example(x), U, ...)`): every pooled sum is
 * formed in the table type (dtype; ET_FLAG_F16_FP32_ACC as for et_pooled_sum), then
 * converted to dst_dtype on the store.  Float types only (ET_F32/F64/F16/BF16);
 * dst_dtype == dtype is et_maplookup_prealloc. */
int et_maplookup_prealloc_to(int dtype, int dst_dtype, const et_lookup_desc* descs,
                             int32_t ntables, int64_t batch, void* dst, int64_t ld_dst,
                             uint32_t flags, void* stream);

/* One table of a (multi-table) fused sparse-SGD update. */
typedef struct et_update_desc {
    void* table;         /* device pointer, updated in place */
    int64_t ld_table;
    int64_t nrows;
    int32_t dim;
    int32_t pool;        /* indices per bag (1 for a vector index) */
    const void* delta;   /* gradient wrt the lookup output: dim x batch, column j at
                            delta + j*ld_delta (may be a row block of a Preallocation
                            gradient, ld_delta = prependrows + sum(dims)) */
    int64_t ld_delta;
    const int64_t* idx;  /* the indices of the forward lookup (1-based) */
    int64_t ld_idx;
    int64_t batch;
    int64_t cols_per_page; /* 0 or a paged table, as in et_lookup_desc */
} et_update_desc;

/* Bytes of device workspace needed by et_sparse_sgd for these descriptors (any
 * alignment: the library lays its buffers out from the workspace's first 256-byte
 * boundary; the size includes that slack). */
int et_sgd_workspace_size(const et_update_desc* descs, int32_t ntables, int64_t* bytes);

/* Fused sparse SGD (Flux.Descent) over one or many tables:
 *   for every table t and every distinct column r referenced by idx_t:
 *     acc = +0 ; for each occurrence (in occurrence order) of r, in bag j: acc += delta_t[:, j]
 *     table_t[:, r] = muladd(-eta, acc, table_t[:, r])   (default: fused, Float32(eta))
 *                   = table_t[:, r] - eta*acc            (ET_FLAG_SGD_UNFUSED)
 * dtype ET_F32 (the reference's tested type; vector kernels), ET_F64, ET_F16 and
 * ET_BF16 (generic kernels): the table and delta share the element type T, eta is
 * convert(T, eta); Float64 accumulates in double, Float16 in Julia Float16 arithmetic
 * (every op rounded to half) or in fp32 with ET_FLAG_F16_FP32_ACC, BFloat16 in fp32;
 * the fused muladd of 16-bit types is one fp32 fma rounded to T (oracle/embtab_oracle.c
 * states the exact model).  Without ET_FLAG_EXACT_UPDATE, occurrence lists
 * longer than the library's chunk length are summed as per-chunk partial sums
 * combined in chunk order (deterministic, not bit-identical to the serial sum).
 * Replaces update!(::Descent, table, ::SparseEmbeddingUpdate, indexer, Val(NT)) —
 * reference src/sparseupdate.jl:160-178 with index! (src/utils.jl:306-314) and
 * _update_specialized_impl! / _update_generic_impl! (:57-154); for ntables > 1 the
 * multi-table update!(opt, tables, grads, indexers; num_splits) :199-238. */
int et_sparse_sgd(int dtype, const et_update_desc* descs, int32_t ntables, double eta,
                  uint32_t flags, void* workspace, int64_t ws_bytes, void* stream);

/* et_sparse_sgd that also copies every table's indices as its index phase reads them (ABI
 * v8): snaps is a HOST array of ntables (<= ET_MAX_TABLES_PER_LAUNCH) device pointers;
 * snaps[t] != NULL receives table t's pool x batch Int64 indices, contiguous (bag-major),
 * stream-ordered inside the index phase (not written by an APPLY_ONLY call).  The copy the
 * multi-table update!(opt, tables, grads, indexers) keeps for filling indexers[i]
 * (src/sparseupdate.jl:210-213) when the caller may refill the index buffers before reading
 * them: 8 bytes written per occurrence beside the keys instead of a separate read-and-write
 * pass.  16-byte aligned snapshots keep the vectorized key pass. */
int et_sparse_sgd_snap(int dtype, const et_update_desc* descs, int32_t ntables, double eta,
                       uint32_t flags, int64_t* const* snaps, void* workspace, int64_t ws_bytes,
                       void* stream);

/* Update from a prebuilt Indexer (et_index_build layout) over its cumulative entries
 * [ubegin, uend) — the reference's lower-level
 * update!(table, ::SparseEmbeddingUpdate, indexer::AbstractIndexer, alpha, Val(NT)),
 * src/sparseupdate.jl:46-154, where an IndexerView (src/utils.jl:320-338) selects a
 * range of distinct columns.  Every column's gradient is summed serially in `map`
 * order (exact).  `cumulative_*` and `map` are device arrays as written by
 * et_index_build; `eta` is the value the reference passes as `alpha`;
 * `cols_per_page` as in et_lookup_desc (0 = contiguous). */
int et_update_indexed(int dtype, void* table, int64_t ld_table, int64_t cols_per_page,
                      int64_t nrows, int32_t dim, const void* delta, int64_t ld_delta, const int64_t* cumulative_col,
                      const int64_t* cumulative_off, int64_t ubegin, int64_t uend,
                      const int64_t* map, double eta, uint32_t flags, void* stream);

/* Bytes of device workspace needed by et_index_build for n occurrences. */
int et_index_workspace_size(int64_t n, int64_t* bytes);

/* The reference's Indexer on the device: groups the occurrences of a P x B (or
 * vector, pool = 1) index array by column, with the distinct columns in
 * FIRST-SEEN order and each column's occurrences in occurrence order.
 * Outputs (device, int64, 1-based like the reference):
 *   cumulative_col[u], cumulative_off[u] for u < U, and the terminator
 *   cumulative_col[U] = 0, cumulative_off[U] = n + 1;
 *   map[k] = gradient column (bag, 1-based) of the k-th grouped occurrence;
 *   *nunique_dev = U.
 * Arrays must hold n+1 (cumulative) and n (map) entries.
 * Replaces index!(::Indexer, A, maxindex) — reference src/utils.jl:306-314 with
 * histogram! :131-167, prefixsum! :170-239, remap! :242-272. */
int et_index_build(const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                   int64_t nrows, int64_t* cumulative_col, int64_t* cumulative_off,
                   int64_t* map, int64_t* nunique_dev, void* workspace, int64_t ws_bytes,
                   void* stream);

/* Assemble the Preallocation concat from per-rank slabs after an all-gather
 * (table-wise sharding across GPUs, no counterpart in the single-process
 * reference): slab r is a (slab_ld x batch) column-major block at
 * slabs + r*slab_ld*batch whose first rows[r] rows are copied to
 * dst[dst_row_off[r] + (0:rows[r]-1), :].  `rows`, `dst_row_off` are HOST arrays
 * of nranks entries; the rank whose slab already sits in dst can be skipped by
 * giving it rows[r] = 0. */
int et_concat_slabs(int dtype, const void* slabs, int32_t nranks, int64_t slab_ld,
                    int64_t batch, const int32_t* rows, const int64_t* dst_row_off, void* dst,
                    int64_t ld_dst, void* stream);

/* The reverse of et_concat_slabs, for the backward exchange of a sharded step:
 * slab_r[:, f] (row f < rows[r] of rank r's (slab_ld x batch) slab, slabs laid out
 * rank after rank) = src[src_row_off[r] + f, :].  Used to cut a batch-sliced gradient
 * into per-rank slabs before an all-to-all. */
int et_split_slabs(int dtype, const void* src, int64_t ld_src, int64_t batch, int32_t nranks,
                   const int32_t* rows, const int64_t* src_row_off, void* slabs,
                   int64_t slab_ld, void* stream);

/* One-sided exchange for a sharded maplookup (the "fused P2P xGMI writes" item of
 * SURVEY.md §8f rank 3; replaces the all-gather + et_concat_slabs of the concat in
 * src/lookup.jl:316-371 when every rank holds the whole destination): rows
 * col..col+ncols-1 of every bag of src ((ld x batch), this rank's finished
 * columns) are stored into the same rows of each peer destination (same ld;
 * `peers` is a HOST array of npeers device pointers from et_ipc_open).  Publish
 * with a stream-ordered barrier after the launch. */
#define ET_MAX_PEERS 16
int et_push_cols(int dtype, const void* src, int64_t ld, int64_t batch, int64_t col,
                 int64_t ncols, void* const* peers, int32_t npeers, void* stream);

/* IPC mapping of a device buffer for et_push_cols: et_ipc_handle fills `handle`
 * (64 bytes) for the allocation holding `ptr` and the byte offset of ptr in it;
 * another process maps it with et_ipc_open (peer access enabled lazily) and
 * unmaps it with et_ipc_close(ptr, offset). */
int et_ipc_handle(const void* ptr, void* handle, int64_t* offset);
int et_ipc_open(const void* handle, int64_t offset, void** ptr);
int et_ipc_close(void* ptr, int64_t offset);

/* ---------------------------------------------------------------------------------
 * Sharded PreallocationStrategy maplookup over the GPUs of a node (BASELINE config 5;
 * SURVEY.md §8e).  No counterpart exists in the single-process reference: these replace
 * the in-place concat of maplookup!(::PreallocationStrategy, dst, tables, I)
 * (src/lookup.jl:316-371, the row-block views at :334-340) when the tables are spread
 * over ranks — one process per GPU, RCCL over xGMI for the one exchange step.
 * ------------------------------------------------------------------------------- */

/* One piece of a shard plan: features [f0, f0+dim) of table `table` (0-based), owned by
 * `rank`; its rows of the destination start at `col` (prependrows included). */
typedef struct et_shard_piece {
    int32_t rank;
    int32_t table;
    int32_t f0;
    int32_t dim;
    int64_t col;
} et_shard_piece;

#define ET_PLAN_TABLEWISE 0   /* whole tables, contiguous groups balanced by count (26 tables
                                 on 8 GPUs: 4,4,3,3,3,3,3,3); with `sizes`, dealt in
                                 descending size round-robin so the largest land on
                                 distinct ranks */
#define ET_PLAN_FEATUREWISE 1 /* the concatenated feature axis cut into equal contiguous
                                 ranges at `granule`-feature boundaries inside tables, each
                                 range cut into vector-kernel widths (96 -> 64 + 32) */

/* The shard plan: every rank's pieces, rank by rank, each rank's in slab order.  With
 * out == NULL only *npieces is set (the count to allocate).  Host-only; no device. */
int et_shard_plan(int32_t mode, int32_t ntables, const int32_t* dims, const int64_t* sizes,
                  int32_t world, int64_t prependrows, int32_t granule, int32_t elsize,
                  et_shard_piece* out, int32_t cap, int32_t* npieces);

/* RCCL communicator of the ranks (one process per GPU, the current HIP device):
 * rank 0 creates a 128-byte id, the host broadcasts it by any means (MPI, a TCP store,
 * torch.distributed), every rank calls et_comm_init with it.  The comm is a
 * ncclComm_t; any ncclComm_t the host already owns may be passed instead. */
#define ET_COMM_ID_BYTES 128
int et_comm_unique_id(void* id);
int et_comm_init(void** comm, int32_t nranks, const void* id, int32_t rank);
int et_comm_destroy(void* comm);

/* A LOOPBACK communicator: nranks simulated ranks of this one process (comms[r] is rank r),
 * all on the current device, for exercising the world > 1 sharded step without nranks
 * GPUs.  Each rank must be driven by its own host thread with its own stream; every
 * collective of the sharded step (et_sharded_maplookup, et_sharded_piece_grads,
 * et_allgather_concat) is then a host rendezvous of the nranks callers followed by device
 * copies between their buffers, stream-ordered with events as RCCL orders its collectives.
 * Accepted wherever an RCCL comm is (world must equal nranks); a caller that does not
 * arrive within 120 s fails the collective.  Free each handle with et_comm_destroy. */
int et_comm_loopback(void** comms, int32_t nranks);

/* The exchange step on its own: ncclAllGather of every rank's (slab_ld x batch) slab into
 * `gathered` (nranks slabs, rank after rank), then et_concat_slabs(gathered, rows,
 * dst_row_off) into dst.  One contiguous run of destination rows per rank.  comm == NULL
 * (allowed for nranks == 1 only) copies the slab instead of calling RCCL. */
int et_allgather_concat(void* comm, int dtype, const void* slab, int64_t slab_ld, int64_t batch,
                        void* gathered, int32_t nranks, const int32_t* rows,
                        const int64_t* dst_row_off, void* dst, int64_t ld_dst, void* stream);

#define ET_EXCHANGE_ALLGATHER 0 /* every rank ends with the whole (ld_dst x batch) dst */
#define ET_EXCHANGE_ALLTOALL 1  /* DLRM layout: rank r ends with bags [r*B/N, (r+1)*B/N) of
                                   every feature (N times less on the links) */

/* A sharded step: the plan (all ranks' pieces, as from et_shard_plan), this rank, the
 * destination geometry, `chunks` batch chunks pipelined through lookup / exchange /
 * assembly (all-gather only).  comm may be NULL only for world == 1 (the exchange is then
 * a device copy).  Creates one side stream and a few events on the current device;
 * everything else is caller-owned. */
int et_sharded_create(void** handle, void* comm, int32_t world, int32_t rank, int dtype,
                      const et_shard_piece* pieces, int32_t npieces, int64_t prependrows,
                      int64_t ld_dst, int64_t batch, int32_t chunks, int32_t exchange);
/* Slab leading dimension, workspace bytes, and the bags [lo, hi) of dst this rank ends
 * with (0..batch for the all-gather). */
int et_sharded_info(void* handle, int64_t* slab_ld, int64_t* ws_bytes, int64_t* batch_lo,
                    int64_t* batch_hi);
/* One step: `local` holds this rank's pieces in plan order (table = the piece's columns,
 * e.g. a column-slice pointer with the parent's ld_table; dim = the piece's dim; idx for
 * the whole batch; dst_row_off ignored).  Stream-ordered on `stream`; dst is
 * (ld_dst x batch), or (ld_dst x (hi - lo)) for the all-to-all. */
int et_sharded_maplookup(void* handle, const et_lookup_desc* local, int32_t nlocal, void* dst,
                         int64_t ld_dst, void* workspace, int64_t ws_bytes, uint32_t flags,
                         void* stream);
/* Backward of the all-to-all layout (rrule of the sharded maplookup, src/lookup.jl:374-389):
 * from this rank's (ld_delta x (hi - lo)) gradient slice, every rank's feature rows are cut
 * out (et_split_slabs) and exchanged, giving `recv` = (slab_ld x batch): this rank's
 * pieces' gradient rows for every bag, pieces in plan order.  (Under the all-gather layout
 * the gradient is replicated and a piece's gradient is a row block of it.) */
int et_sharded_piece_grads(void* handle, const void* delta, int64_t ld_delta, void* recv,
                           void* workspace, int64_t ws_bytes, void* stream);
int et_sharded_destroy(void* handle);

/* Deterministic synthetic data (the same counter-based hash as oracle/):
 * element i of dst = lo + (hi-lo) * u(seed, offset + i), u in [0,1) with 24 bits. */
int et_fill_uniform(int dtype, void* dst, int64_t n, uint64_t seed, uint64_t offset,
                    double lo, double hi, void* stream);

/* Uniform 1-based indices in 1..nrows (hash of seed, offset + i). */
int et_fill_index_uniform(int64_t* idx, int64_t n, int64_t nrows, uint64_t seed,
                          uint64_t offset, void* stream);

/* Synchronise the device, return (and clear) the number of out-of-range indices
 * seen by any kernel since the last call. */
int et_check_errors(uint64_t* oob_count);

#ifdef __cplusplus
}
#endif

#endif /* EMBTAB_H */
