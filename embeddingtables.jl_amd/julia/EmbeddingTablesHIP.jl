# EmbeddingTablesHIP.jl — the Julia host layer of the MI355X engine.
#
# Plugs libembtab_hip.so (include/embtab.h) into darchr/EmbeddingTables.jl through the
# package's own extension points (README.md:277-307, src/EmbeddingTables.jl:44-156):
# a new `AbstractEmbeddingTable` subtype whose hot methods — `lookup!`,
# `maplookup!(::PreallocationStrategy, …)` and `update!(::Descent, …)` — are `ccall`s
# into the C ABI.  Everything else (lookup, maplookup, rrules, SparseEmbeddingUpdate,
# Flux.Optimise.update!) is the reference's unchanged generic code.
#
# STATUS: written against the C ABI but NOT executed — this image has no Julia
# toolchain (SURVEY.md §8c).  The Python ctypes layer (../embtab/) calls the identical
# symbols with the identical arguments and is what the tests exercise; see
# INTEGRATION.md for the one-to-one mapping.
module EmbeddingTablesHIP

using EmbeddingTables
import EmbeddingTables: lookup!, maplookup!, update!, index!, columnpointer, example, featuresize
using EmbeddingTables: AbstractEmbeddingTable, Static, Dynamic, SparseEmbeddingUpdate,
    PreallocationStrategy, AbstractIndexer, Indexer
import Flux

const libembtab = joinpath(@__DIR__, "..", "embtab", "libembtab_hip.so")
const libhip = "libamdhip64.so"

const ET_F32, ET_F16, ET_F64, ET_I32, ET_I64 = Cint(0), Cint(1), Cint(2), Cint(3), Cint(4)
const ET_FLAG_NONTEMPORAL = UInt32(1)
const ET_FLAG_EXACT_UPDATE = UInt32(4)      # every column summed serially (bit-identical)
const ET_FLAG_EXACT_IF_FAST = UInt32(256)   # the default: exact (ABI v9: every eltype and size)
const ET_FLAG_SGD_UNFUSED = UInt32(8)
const ET_FLAG_SGD_F64_ALPHA = UInt32(16)
const ET_FLAG_SGD_INDEX_ONLY = UInt32(32)   # phase 1 of update!: index all (src/sparseupdate.jl:210-213)
const ET_FLAG_SGD_APPLY_ONLY = UInt32(64)   # phase 2: update all (:216-237)

et_dtype(::Type{Float32}) = ET_F32
et_dtype(::Type{Float16}) = ET_F16
et_dtype(::Type{Float64}) = ET_F64
et_dtype(::Type{Int32}) = ET_I32
et_dtype(::Type{Int64}) = ET_I64

struct EmbtabError <: Exception
    status::Cint
    msg::String
end

function check(rc::Cint)
    if rc != 0
        msg = unsafe_string(ccall((:et_last_error, libembtab), Cstring, ()))
        throw(EmbtabError(rc, msg))
    end
    return nothing
end

# The stream every call is ordered on (NULL = the legacy default stream).
const STREAM = Ref{Ptr{Cvoid}}(C_NULL)
stream() = STREAM[]

#####
##### Device arrays (column-major, like Julia's own)
#####

mutable struct HipArray{T,N} <: AbstractArray{T,N}
    ptr::Ptr{T}
    dims::NTuple{N,Int}
    function HipArray{T,N}(::UndefInitializer, dims::NTuple{N,Int}) where {T,N}
        p = Ref{Ptr{Cvoid}}(C_NULL)
        nbytes = max(prod(dims), 1) * sizeof(T)
        ccall((:hipMalloc, libhip), Cint, (Ptr{Ptr{Cvoid}}, Csize_t), p, nbytes) == 0 ||
            error("hipMalloc failed")
        A = new{T,N}(Ptr{T}(p[]), dims)
        finalizer(a -> ccall((:hipFree, libhip), Cint, (Ptr{Cvoid},), a.ptr), A)
        return A
    end
end
const HipVector{T} = HipArray{T,1}
const HipMatrix{T} = HipArray{T,2}
HipArray{T}(::UndefInitializer, dims::Integer...) where {T} =
    HipArray{T,length(dims)}(undef, Int.(dims))
Base.size(A::HipArray) = A.dims
Base.pointer(A::HipArray) = A.ptr
Base.similar(::HipArray, ::Type{T}, dims::Dims) where {T} = HipArray{T,length(dims)}(undef, dims)
# Leading dimension in elements: HipArrays are dense.
leading(A::HipMatrix) = size(A, 1)
# Device memory is never dereferenced on the host: element access copies.
function Base.getindex(A::HipArray{T}, i::Int) where {T}
    r = Ref{T}()
    ccall((:hipMemcpy, libhip), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint), r,
          A.ptr + (i - 1) * sizeof(T), sizeof(T), 2)
    return r[]
end
function Base.setindex!(A::HipArray{T}, v, i::Int) where {T}
    r = Ref{T}(convert(T, v))
    ccall((:hipMemcpy, libhip), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint),
          A.ptr + (i - 1) * sizeof(T), r, sizeof(T), 1)
    return v
end
Base.IndexStyle(::Type{<:HipArray}) = IndexLinear()
# Host array -> new device array (hipMemcpyHostToDevice).
function upload(A::Array{T,N}) where {T,N}
    D = HipArray{T,N}(undef, size(A))
    ccall((:hipMemcpy, libhip), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint),
          D.ptr, A, sizeof(A), 1) == 0 || error("hipMemcpy failed")
    return D
end
# Device array -> host array (hipMemcpyDeviceToHost, after the stream's work).
function download(A::HipArray{T,N}) where {T,N}
    H = Array{T,N}(undef, size(A))
    ccall((:hipStreamSynchronize, libhip), Cint, (Ptr{Cvoid},), stream())
    ccall((:hipMemcpy, libhip), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint),
          H, A.ptr, sizeof(H), 2) == 0 || error("hipMemcpy failed")
    return H
end

#####
##### The table type (AbstractEmbeddingTable contract, README.md:288-307)
#####

struct HipEmbedding{S,T} <: AbstractEmbeddingTable{S,T}
    data::HipMatrix{T}
end
HipEmbedding(data::HipMatrix{T}) where {T} = HipEmbedding{Dynamic,T}(data)
function HipEmbedding{Static{N}}(data::HipMatrix{T}) where {N,T}
    N isa Int || throw(ArgumentError("Expected the type parameter for `Static{N}` to be an Int."))
    N == size(data, 1) || throw(ArgumentError("Parameter `N` should match the number of rows."))
    return HipEmbedding{Static{N},T}(data)
end

Base.size(A::HipEmbedding) = size(A.data)
Base.getindex(A::HipEmbedding, i::Int) = A.data[i]
Base.setindex!(A::HipEmbedding, v, i::Int) = (A.data[i] = v)
# A DEVICE pointer: valid for the kernels, never for unsafe_load on the host.
columnpointer(A::HipEmbedding{S,T}, i::Integer) where {S,T} =
    A.data.ptr + (i - 1) * leading(A.data) * sizeof(T)
example(A::HipEmbedding) = A.data

# Paged table: the reference's SplitEmbedding (src/split.jl:3-86) with its pages on the
# device.  `pagetable` holds the pages' device addresses; the kernels address column r
# as pages[(r-1) ÷ cps] + ((r-1) % cps) * featuresize (et_lookup_desc.cols_per_page).
struct HipSplitEmbedding{S,T} <: AbstractEmbeddingTable{S,T}
    pages::Vector{HipMatrix{T}}
    pagetable::HipVector{UInt64}
    matrixsize::Tuple{Int,Int}
end
function HipSplitEmbedding(A::Matrix{T}, cols_per_shard = 1) where {T}
    n = size(A, 2)
    pages = [upload(A[:, s:min(s + cols_per_shard - 1, n)]) for s in 1:cols_per_shard:n]
    pt = upload(UInt64[UInt64(p.ptr) for p in pages])
    return HipSplitEmbedding{Static{size(A, 1)},T}(pages, pt, (size(A, 1), cols_per_shard))
end
Base.size(A::HipSplitEmbedding) =
    (A.matrixsize[1], A.matrixsize[2] * (length(A.pages) - 1) + size(last(A.pages), 2))
function columnpointer(A::HipSplitEmbedding{S,T}, i::Integer) where {S,T}
    page, col = divrem(i - 1, A.matrixsize[2])
    return A.pages[page + 1].ptr + col * A.matrixsize[1] * sizeof(T)
end
example(A::HipSplitEmbedding) = first(A.pages)

# (table, ld, cols_per_page) of an et_*_desc: contiguous tables pass cols_per_page = 0.
_device_table(A::HipEmbedding) = (Ptr{Cvoid}(A.data.ptr), leading(A.data), 0)
_device_table(A::HipSplitEmbedding) = (Ptr{Cvoid}(A.pagetable.ptr), A.matrixsize[1],
                                       A.matrixsize[2])
# Any other table type that implements only the plug-in contract (size / columnpointer
# / example, README.md:288-307 — e.g. test/constructors.jl's DummyEmbedding over a
# HipMatrix), with its columns in device memory: wrap it as DeviceColumns(table) (the
# wrapper forwards the contract, so the reference's generic code still sees the user
# type's behaviour; it only routes the hot methods here).  Equally spaced columns give a
# contiguous descriptor; anything else a device array of column pointers, one column per
# "page" (cols_per_page = 1).  With 16-byte aligned pointers and rows the vector kernels
# run; otherwise ld_table is set to a non-16-byte spacing, which selects the
# element-aligned kernels (include/embtab.h).
mutable struct DeviceColumns{S,T,A<:AbstractEmbeddingTable{S,T}} <: AbstractEmbeddingTable{S,T}
    table::A
    desc::Any  # (table pointer, ld, cols_per_page, pointer array or nothing), built once
end
DeviceColumns(A::AbstractEmbeddingTable{S,T}) where {S,T} =
    DeviceColumns{S,T,typeof(A)}(A, nothing)
Base.size(A::DeviceColumns) = size(A.table)
Base.getindex(A::DeviceColumns, i::Int) = A.table[i]
Base.setindex!(A::DeviceColumns, v, i::Int) = (A.table[i] = v)
columnpointer(A::DeviceColumns, i::Integer) = columnpointer(A.table, i)
example(A::DeviceColumns) = example(A.table)
function _device_table(A::DeviceColumns{S,T}) where {S,T}
    if A.desc === nothing
        D, R = size(A)
        p = UInt64[UInt64(columnpointer(A.table, i)) for i in 1:R]
        d = diff(p)
        A.desc = if R == 1 || (all(==(d[1]), d) && d[1] % sizeof(T) == 0 &&
                               d[1] ÷ sizeof(T) >= D)
            (Ptr{Cvoid}(p[1]), R == 1 ? D : Int(d[1] ÷ sizeof(T)), 0, nothing)
        else
            vec = all(x -> x % 16 == 0, p) && (D * sizeof(T)) % 16 == 0
            ld = vec || (D * sizeof(T)) % 16 != 0 ? D : D + 1
            dp = upload(p)  # kept alive by the wrapper
            (Ptr{Cvoid}(dp.ptr), ld, 1, dp)
        end
    end
    return A.desc[1:3]
end
const HipTable{S,T} = Union{HipEmbedding{S,T},HipSplitEmbedding{S,T},DeviceColumns{S,T}}

# Preallocation gradients are row blocks of one big matrix: a view's leading dimension.
_ptr_ld(A::HipMatrix) = (Ptr{Cvoid}(A.ptr), leading(A))
function _ptr_ld(V::SubArray{T,2,<:HipMatrix{T}}) where {T}
    P = parent(V)
    r, c = first.(parentindices(V))
    return Ptr{Cvoid}(P.ptr + ((c - 1) * leading(P) + (r - 1)) * sizeof(T)), leading(P)
end

#####
##### lookup! — src/lookup.jl:42-43, :90-102, :167-182
#####

function lookup!(dst, A::HipEmbedding{S,T}, I::HipVector{Int}) where {S,T}
    p, ld = _ptr_ld(dst)
    check(ccall((:et_gather, libembtab), Cint,
                (Cint, Ptr{Cvoid}, Int64, Int64, Int32, Ptr{Int64}, Int64, Ptr{Cvoid}, Int64,
                 UInt32, Ptr{Cvoid}),
                et_dtype(T), A.data.ptr, leading(A.data), size(A, 2), size(A, 1), I.ptr,
                length(I), p, ld, ET_FLAG_NONTEMPORAL, stream()))
    return dst
end

function lookup!(dst, A::HipEmbedding{S,T}, I::HipMatrix{Int}) where {S,T}
    p, ld = _ptr_ld(dst)
    check(ccall((:et_pooled_sum, libembtab), Cint,
                (Cint, Ptr{Cvoid}, Int64, Int64, Int32, Ptr{Int64}, Int32, Int64, Int64,
                 Ptr{Cvoid}, Int64, UInt32, Ptr{Cvoid}),
                et_dtype(T), A.data.ptr, leading(A.data), size(A, 2), size(A, 1), I.ptr,
                size(I, 1), size(I, 1), size(I, 2), p, ld, ET_FLAG_NONTEMPORAL, stream()))
    return dst
end

#####
##### maplookup!(::PreallocationStrategy) — src/lookup.jl:316-371, ONE launch
#####

struct LookupDesc
    table::Ptr{Cvoid}
    ld_table::Int64
    nrows::Int64
    dim::Int32
    pool::Int32
    idx::Ptr{Int64}
    ld_idx::Int64
    dst_row_off::Int64
    cols_per_page::Int64
end

# A paged or column-pointer table's single-table lookup! goes through the descriptor
# entry point.
function lookup!(dst, A::Union{HipSplitEmbedding{S,T},DeviceColumns{S,T}},
                 I::Union{HipVector{Int},HipMatrix{Int}}) where {S,T}
    p, ld = _ptr_ld(dst)
    tp, ldt, cpp = _device_table(A)
    pool = ndims(I) == 1 ? 1 : size(I, 1)
    desc = [LookupDesc(tp, ldt, size(A, 2), size(A, 1), pool, I.ptr, pool, 0, cpp)]
    check(ccall((:et_maplookup_prealloc, libembtab), Cint,
                (Cint, Ptr{LookupDesc}, Int32, Int64, Ptr{Cvoid}, Int64, UInt32, Ptr{Cvoid}),
                et_dtype(T), desc, 1, size(I, ndims(I)), p, ld, ET_FLAG_NONTEMPORAL, stream()))
    return dst
end

# The per-XCD work queues' block for et_maplookup_prealloc_q (ET_LOOKUP_QUEUE_BYTES, zeroed
# once; every launch leaves it zero): one block serves every call, since every call of this
# layer is ordered on the one stream().
const ET_LOOKUP_QUEUE_BYTES = 128
const QUEUE = Ref{Any}(nothing)
function _queue_block()
    if QUEUE[] === nothing
        q = HipArray{UInt8}(undef, ET_LOOKUP_QUEUE_BYTES)
        # zeroed on stream(), so the first et_maplookup_prealloc_q on that stream (blocking or
        # not) sees a zero block
        ccall((:hipMemsetAsync, libhip), Cint, (Ptr{Cvoid}, Cint, Csize_t, Ptr{Cvoid}), q.ptr, 0,
              ET_LOOKUP_QUEUE_BYTES, stream()) == 0 || error("hipMemsetAsync failed")
        QUEUE[] = q
    end
    return QUEUE[].ptr
end

# dst may have another float eltype U than the tables (PreallocationStrategy{U},
# src/lookup.jl:284-315): then the _to entry converts on the store.
function maplookup!(strategy::PreallocationStrategy, dst::HipMatrix{U},
                    x::Vector{<:HipTable{<:Any,T}}, I0; kw...) where {U,T}
    I = EmbeddingTables.colwrap(I0)
    descs = Vector{LookupDesc}(undef, length(x))
    off = strategy.prependrows
    for (t, (A, i)) in enumerate(zip(x, I))
        pool = ndims(i) == 1 ? 1 : size(i, 1)
        tp, ldt, cpp = _device_table(A)
        descs[t] = LookupDesc(tp, ldt, size(A, 2), size(A, 1), pool, pointer(i), pool, off, cpp)
        off += size(A, 1)
    end
    if U === T
        check(ccall((:et_maplookup_prealloc_q, libembtab), Cint,
                    (Cint, Ptr{LookupDesc}, Int32, Int64, Ptr{Cvoid}, Int64, UInt32, Ptr{Cvoid},
                     Ptr{Cvoid}),
                    et_dtype(T), descs, length(descs), EmbeddingTables._batchsize(I), dst.ptr,
                    leading(dst), ET_FLAG_NONTEMPORAL, _queue_block(), stream()))
    else
        check(ccall((:et_maplookup_prealloc_to, libembtab), Cint,
                    (Cint, Cint, Ptr{LookupDesc}, Int32, Int64, Ptr{Cvoid}, Int64, UInt32,
                     Ptr{Cvoid}),
                    et_dtype(T), et_dtype(U), descs, length(descs), EmbeddingTables._batchsize(I),
                    dst.ptr, leading(dst), ET_FLAG_NONTEMPORAL, stream()))
    end
    return dst
end

#####
##### update! — src/sparseupdate.jl:160-178 (single) and :199-238 (multi-table)
#####

struct UpdateDesc
    table::Ptr{Cvoid}
    ld_table::Int64
    nrows::Int64
    dim::Int32
    pool::Int32
    delta::Ptr{Cvoid}
    ld_delta::Int64
    idx::Ptr{Int64}
    ld_idx::Int64
    batch::Int64
    cols_per_page::Int64
end

const UpdateEltype = Union{Float32,Float64,Float16}  # et_sparse_sgd's table types

function _update_desc(A::HipTable{S,<:UpdateEltype}, g::SparseEmbeddingUpdate) where {S}
    dp, dld = _ptr_ld(g.delta)
    I = g.indices
    pool = ndims(I) == 1 ? 1 : size(I, 1)
    tp, ldt, cpp = _device_table(A)
    return UpdateDesc(tp, ldt, size(A, 2), size(A, 1), pool, dp, dld, pointer(I), pool,
                      size(I, ndims(I)), cpp)
end

# The reference picks its fused `muladd` kernel for Static tables of <= 512 bytes per
# column (src/sparseupdate.jl:131-154), the generic `x - alpha*y` path otherwise.
_fused(::HipTable{Static{N},T}) where {N,T} = N * sizeof(T) <= 512
_fused(::HipTable) = false

# Update workspaces, one per (stream, slot): calls that share one are ordered on their stream,
# so setting STREAM[] to another stream never lets two in-flight calls share a workspace.  At
# most WS_STREAMS streams per slot keep theirs (least recently used first out, after its stream
# drains), so a program cycling through many streams does not hold a workspace per stream.
const WORKSPACES = Dict{Tuple{Ptr{Cvoid},Int},Any}()
const WS_ORDER = Tuple{Ptr{Cvoid},Int}[]
const WS_STREAMS = 4
function _workspace(nbytes, slot::Int = -1)
    k = (stream(), slot)
    ws = get(WORKSPACES, k, nothing)
    if ws === nothing || length(ws) < nbytes
        ws = HipArray{UInt8}(undef, nbytes)
        WORKSPACES[k] = ws
    end
    filter!(!=(k), WS_ORDER)
    push!(WS_ORDER, k)
    same = filter(x -> x[2] == slot, WS_ORDER)
    for x in same[1:end-min(WS_STREAMS, length(same))]
        ccall((:hipStreamSynchronize, libhip), Cint, (Ptr{Cvoid},), x[1]) == 0 ||
            error("hipStreamSynchronize failed")
        delete!(WORKSPACES, x)
        filter!(!=(x), WS_ORDER)
    end
    return ws
end

# One update call; snapshot pointers (C_NULL for none) make it et_sparse_sgd_snap.
function _sparse_sgd(::Type{T}, descs::Vector{UpdateDesc}, eta::Float64, flags::UInt32,
                     snaps::Vector{Ptr{Int64}} = Ptr{Int64}[]) where {T}
    nb = Ref{Int64}(0)
    check(ccall((:et_sgd_workspace_size, libembtab), Cint, (Ptr{UpdateDesc}, Int32, Ref{Int64}),
                descs, length(descs), nb))
    ws = _workspace(nb[])
    if any(p -> p != C_NULL, snaps)
        check(ccall((:et_sparse_sgd_snap, libembtab), Cint,
                    (Cint, Ptr{UpdateDesc}, Int32, Float64, UInt32, Ptr{Ptr{Int64}}, Ptr{Cvoid},
                     Int64, Ptr{Cvoid}),
                    et_dtype(T), descs, length(descs), eta, flags, snaps, ws.ptr, length(ws),
                    stream()))
    else
        check(ccall((:et_sparse_sgd, libembtab), Cint,
                    (Cint, Ptr{UpdateDesc}, Int32, Float64, UInt32, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                    et_dtype(T), descs, length(descs), eta, flags, ws.ptr, length(ws), stream()))
    end
end

# The exact update (every column's gradient summed serially in the reference's order) is
# the default: `nothing` passes ET_FLAG_EXACT_IF_FAST, exact for every eltype and gradient
# size since ABI v9 (the serial-chain path); exact = true is the same, exact = false selects
# the split mode (long columns summed as ordered partial sums: deterministic, not
# bit-identical).
const EXACT = Ref{Union{Nothing,Bool}}(nothing)
_exact_flag(exact) = exact === nothing ? ET_FLAG_EXACT_IF_FAST :
                     exact ? ET_FLAG_EXACT_UPDATE : UInt32(0)

# src/sparseupdate.jl:159-178 indexes into `indexer` first (index!(indexer, update.indices,
# size(table, 2))): a HipIndexer receives a snapshot of the indices from the update's own key
# pass (et_sparse_sgd_snap, built when first read), a host Indexer passed by the caller the
# reference's own index! on a downloaded copy; with none (the default here, where the
# reference's default is a fresh Indexer() nobody can read) nothing is indexed.
function update!(opt::Flux.Descent, table::HipTable{S,T}, grad::SparseEmbeddingUpdate,
                 indexer = nothing, ::Val{Nontemporal} = Val(true),
                 args...; exact::Union{Nothing,Bool} = EXACT[]) where {S,T<:UpdateEltype,Nontemporal}
    flags = (Nontemporal ? ET_FLAG_NONTEMPORAL : UInt32(0)) |
            (_fused(table) ? UInt32(0) : ET_FLAG_SGD_UNFUSED) |
            _exact_flag(exact)
    snap = indexer isa HipIndexer && !isempty(grad.indices) ?
           _snapshot!(indexer, grad.indices, size(table, 2)) : Ptr{Int64}(C_NULL)
    # convert(eltype(table), opt.eta) happens inside the library
    _sparse_sgd(T, [_update_desc(table, grad)], Float64(opt.eta), flags, Ptr{Int64}[snap])
    if indexer isa AbstractIndexer && !(indexer isa HipIndexer)
        EmbeddingTables.index!(indexer, download(grad.indices), size(table, 2))
    end
    return nothing
end

#####
##### The Indexer on the device (et_index_build): the reference's cumulative / map layout
##### (src/utils.jl:280-314) in device arrays, so filling indexers[i] costs no host work
#####

mutable struct HipIndexer <: AbstractIndexer
    cumulative_col::Union{Nothing,HipVector{Int64}}  # (col, offset) pairs in first-seen
    cumulative_off::Union{Nothing,HipVector{Int64}}  # order, then the terminator (0, n+1)
    map::Union{Nothing,HipVector{Int64}}             # gradient column of each occurrence
    nunique_dev::Union{Nothing,HipVector{Int64}}
    workspace::Union{Nothing,HipVector{UInt8}}
    # the index array a multi-table update!'s index phase copied (et_sparse_sgd_snap) and its
    # (pool, batch, maxindex) while not yet indexed: built into the fields above on first read
    snapshot::Union{Nothing,HipVector{Int64}}
    pending::Union{Nothing,NTuple{3,Int}}
end
HipIndexer() = HipIndexer(nothing, nothing, nothing, nothing, nothing, nothing, nothing)

# Reading any Indexer field first indexes a pending snapshot (stream-ordered after the
# update that wrote it), as the Python host's Indexer._defer / _materialise.
const _INDEXER_FIELDS = (:cumulative_col, :cumulative_off, :map, :nunique_dev)
function Base.getproperty(ix::HipIndexer, s::Symbol)
    s in _INDEXER_FIELDS && _materialise!(ix)
    return getfield(ix, s)
end

function _materialise!(ix::HipIndexer)
    p = getfield(ix, :pending)
    p === nothing && return ix
    setfield!(ix, :pending, nothing)
    pool, batch, maxindex = p
    return _index_build!(ix, getfield(ix, :snapshot).ptr, pool, batch, maxindex)
end

# The snapshot buffer a multi-table update! hands to et_sparse_sgd_snap for this Indexer
# (contiguous pool x batch; reused while unread or large enough).
function _snapshot!(ix::HipIndexer, I::Union{HipVector{Int},HipMatrix{Int}}, maxindex)
    pool = ndims(I) == 1 ? 1 : size(I, 1)
    batch = size(I, ndims(I))
    buf = getfield(ix, :snapshot)
    if buf === nothing || length(buf) < pool * batch
        buf = HipArray{Int64}(undef, max(pool * batch, 1))
        setfield!(ix, :snapshot, buf)
    end
    setfield!(ix, :pending, (pool, batch, Int(maxindex)))
    return buf.ptr
end

function _index_build!(ix::HipIndexer, idx::Ptr{Int64}, pool, batch, maxindex)
    n = pool * batch
    if getfield(ix, :map) === nothing || length(getfield(ix, :map)) < max(n, 1)
        setfield!(ix, :cumulative_col, HipArray{Int64}(undef, n + 1))
        setfield!(ix, :cumulative_off, HipArray{Int64}(undef, n + 1))
        setfield!(ix, :map, HipArray{Int64}(undef, max(n, 1)))
        setfield!(ix, :nunique_dev, HipArray{Int64}(undef, 1))
        nb = Ref{Int64}(0)
        check(ccall((:et_index_workspace_size, libembtab), Cint, (Int64, Ref{Int64}), n, nb))
        setfield!(ix, :workspace, HipArray{UInt8}(undef, nb[]))
    end
    ws = getfield(ix, :workspace)
    check(ccall((:et_index_build, libembtab), Cint,
                (Ptr{Int64}, Int32, Int64, Int64, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Int64},
                 Ptr{Int64}, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                idx, pool, pool, batch, maxindex, getfield(ix, :cumulative_col).ptr,
                getfield(ix, :cumulative_off).ptr, getfield(ix, :map).ptr,
                getfield(ix, :nunique_dev).ptr, ws.ptr, length(ws), stream()))
    return ix
end

# index!(indexer, A, maxindex) (src/utils.jl:306-314) on the device, stream-ordered.
function index!(ix::HipIndexer, I::Union{HipVector{Int},HipMatrix{Int}}, maxindex)
    setfield!(ix, :pending, nothing)  # an explicit index! replaces an unread snapshot
    pool = ndims(I) == 1 ? 1 : size(I, 1)
    return _index_build!(ix, pointer(I), pool, size(I, ndims(I)), maxindex)
end
nunique(ix::HipIndexer) = download(ix.nunique_dev)[1]

# update!(table, grad, indexer, alpha, Val(NT)) (src/sparseupdate.jl:46-154) from a
# device Indexer: every column serially in map order (et_update_indexed).
function update!(table::HipTable{S,T}, grad::SparseEmbeddingUpdate, ix::HipIndexer, alpha,
                 ::Val{Nontemporal} = Val(true)) where {S,T<:UpdateEltype,Nontemporal}
    dp, dld = _ptr_ld(grad.delta)
    tp, ldt, cpp = _device_table(table)
    flags = (Nontemporal ? ET_FLAG_NONTEMPORAL : UInt32(0)) |
            (_fused(table) ? UInt32(0) : ET_FLAG_SGD_UNFUSED)
    check(ccall((:et_update_indexed, libembtab), Cint,
                (Cint, Ptr{Cvoid}, Int64, Int64, Int64, Int32, Ptr{Cvoid}, Int64, Ptr{Int64},
                 Ptr{Int64}, Int64, Int64, Ptr{Int64}, Float64, UInt32, Ptr{Cvoid}),
                et_dtype(T), tp, ldt, cpp, size(table, 2), size(table, 1), dp, dld,
                ix.cumulative_col.ptr, ix.cumulative_off.ptr, 0, nunique(ix), ix.map.ptr,
                Float64(alpha), flags, stream()))
    return nothing
end

# src/sparseupdate.jl:199-238: index all tables, telemetry_cb(), update all tables.
# One device pipeline per (path, eltype) group, split at the same boundary
# (ET_FLAG_SGD_INDEX_ONLY, then ET_FLAG_SGD_APPLY_ONLY from the same workspace);
# telemetry_cb (if given) runs once the index phase is enqueued.  indexers[i] is filled in
# the index phase, as the reference's (:210-213):
#  * a HipIndexer receives a SNAPSHOT of grads[i].indices written by the update's own key pass
#    (et_sparse_sgd_snap: 8 bytes per occurrence beside the keys, no separate pass and no
#    second sort), indexed on the device (et_index_build) when it is first read — so a caller
#    that refills the index buffer before reading indexers[i] still gets this update's;
#  * a host Indexer (the reference's own type) is filled by the reference's serial index! on a
#    downloaded copy of the indices (fill_host_indexers = true, the default, as the reference
#    does; false skips it: a PCIe copy of every index array and a host pass over every
#    occurrence per step, 272 MB and 34 M insertions at BASELINE config 4).
# One Indexer object at several positions ends up holding the LAST one's indices, as the
# reference's sequential index! calls leave it, so only its last position is snapshotted.
function update!(opt::Flux.Descent, tables::AbstractVector{<:HipTable},
                 grads::AbstractVector{<:SparseEmbeddingUpdate},
                 indexers::AbstractVector{<:AbstractIndexer}, ::Val{Nontemporal} = Val(true);
                 telemetry_cb = nothing, fill_host_indexers::Bool = true,
                 exact::Union{Nothing,Bool} = EXACT[], kw...) where {Nontemporal}
    nt = (Nontemporal ? ET_FLAG_NONTEMPORAL : UInt32(0)) | _exact_flag(exact)
    lastpos = IdDict{Any,Int}(ix => i for (i, ix) in pairs(indexers))
    snap = [indexers[i] isa HipIndexer && lastpos[indexers[i]] == i && !isempty(grads[i].indices) ?
            _snapshot!(indexers[i], grads[i].indices, size(tables[i], 2)) : Ptr{Int64}(C_NULL)
            for i in eachindex(indexers, grads)]
    calls = []
    for fused in (true, false), T in (Float32, Float64, Float16)
        sel = [i for i in eachindex(tables) if _fused(tables[i]) == fused &&
                                               eltype(tables[i]) === T]
        isempty(sel) && continue
        # the multi-table generic path sees opt.eta as Float64 (src/sparseupdate.jl:232)
        flags = nt | (fused ? UInt32(0) : ET_FLAG_SGD_UNFUSED | ET_FLAG_SGD_F64_ALPHA)
        for chunk in Iterators.partition(sel, 32)
            descs = [_update_desc(tables[i], grads[i]) for i in chunk]
            nb = Ref{Int64}(0)
            check(ccall((:et_sgd_workspace_size, libembtab), Cint,
                        (Ptr{UpdateDesc}, Int32, Ref{Int64}), descs, length(descs), nb))
            ws = _workspace(nb[], length(calls))
            push!(calls, (T, descs, flags, ws, Ptr{Int64}[snap[i] for i in chunk]))
        end
    end
    # phase 1 (or the whole update): the snapshots ride in the key pass
    index_phase(phase) = for (T, descs, flags, ws, snaps) in calls
        check(ccall((:et_sparse_sgd_snap, libembtab), Cint,
                    (Cint, Ptr{UpdateDesc}, Int32, Float64, UInt32, Ptr{Ptr{Int64}}, Ptr{Cvoid},
                     Int64, Ptr{Cvoid}),
                    et_dtype(T), descs, length(descs), Float64(opt.eta), flags | phase, snaps,
                    ws.ptr, length(ws), stream()))
    end
    apply_phase() = for (T, descs, flags, ws, _) in calls
        check(ccall((:et_sparse_sgd, libembtab), Cint,
                    (Cint, Ptr{UpdateDesc}, Int32, Float64, UInt32, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                    et_dtype(T), descs, length(descs), Float64(opt.eta),
                    flags | ET_FLAG_SGD_APPLY_ONLY, ws.ptr, length(ws), stream()))
    end
    # without a callback nothing observes the phase boundary: one call per group (the
    # same device work and order; exact mode's early chains start with the call)
    phased = telemetry_cb !== nothing
    index_phase(phased ? ET_FLAG_SGD_INDEX_ONLY : UInt32(0))
    if fill_host_indexers
        for i in eachindex(indexers, grads)
            indexers[i] isa HipIndexer && continue
            EmbeddingTables.index!(indexers[i], download(grads[i].indices), size(tables[i], 2))
        end
    end
    if phased
        telemetry_cb()
        apply_phase()
    end
    return nothing
end

#####
##### Sharded Preallocation maplookup over the GPUs of a node (BASELINE config 5):
##### one Julia process per GPU, RCCL over xGMI (include/embtab.h, csrc/et_shard.cpp)
#####

struct ShardPiece
    rank::Int32
    table::Int32
    f0::Int32
    dim::Int32
    col::Int64
end

const ET_PLAN_TABLEWISE, ET_PLAN_FEATUREWISE = Int32(0), Int32(1)
const ET_EXCHANGE_ALLGATHER, ET_EXCHANGE_ALLTOALL = Int32(0), Int32(1)

function shard_plan(dims::Vector{Int32}, world; mode = ET_PLAN_TABLEWISE, prependrows = 0,
                    sizes = nothing, granule = 32, elsize = 4)
    n = Ref{Int32}(0)
    sz = sizes === nothing ? C_NULL : Int64.(sizes)
    args() = (mode, Int32(length(dims)), dims, sz, Int32(world), Int64(prependrows),
              Int32(granule), Int32(elsize))
    check(ccall((:et_shard_plan, libembtab), Cint,
                (Int32, Int32, Ptr{Int32}, Ptr{Int64}, Int32, Int64, Int32, Int32,
                 Ptr{ShardPiece}, Int32, Ref{Int32}), args()..., C_NULL, 0, n))
    out = Vector{ShardPiece}(undef, n[])
    check(ccall((:et_shard_plan, libembtab), Cint,
                (Int32, Int32, Ptr{Int32}, Ptr{Int64}, Int32, Int64, Int32, Int32,
                 Ptr{ShardPiece}, Int32, Ref{Int32}), args()..., out, n[], n))
    return out
end

# Rank 0: comm_id(); the host broadcasts the 128 bytes (MPI.Bcast!, a TCP store, ...);
# every rank: comm_init(id, world, rank) on its own GPU.
function comm_id()
    id = Vector{UInt8}(undef, 128)
    check(ccall((:et_comm_unique_id, libembtab), Cint, (Ptr{UInt8},), id))
    return id
end
function comm_init(id::Vector{UInt8}, world, rank)
    c = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:et_comm_init, libembtab), Cint, (Ref{Ptr{Cvoid}}, Int32, Ptr{UInt8}, Int32),
                c, world, id, rank))
    return c[]
end
comm_destroy(comm::Ptr{Cvoid}) =
    check(ccall((:et_comm_destroy, libembtab), Cint, (Ptr{Cvoid},), comm))
# `world` simulated ranks of this process (one Julia task per rank, each on its own
# stream): the world > 1 sharded step without `world` GPUs (et_comm_loopback).
function comm_loopback(world)
    cs = Vector{Ptr{Cvoid}}(undef, world)
    check(ccall((:et_comm_loopback, libembtab), Cint, (Ptr{Ptr{Cvoid}}, Int32), cs, world))
    return cs
end

mutable struct ShardedPreallocation
    handle::Ptr{Cvoid}
    workspace::HipVector{UInt8}
    rank::Int
    batch_range::UnitRange{Int}
end

function ShardedPreallocation(comm, plan::Vector{ShardPiece}, world, rank, ::Type{T},
                              prependrows, ld_dst, batch; chunks = 4,
                              exchange = ET_EXCHANGE_ALLGATHER) where {T}
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:et_sharded_create, libembtab), Cint,
                (Ref{Ptr{Cvoid}}, Ptr{Cvoid}, Int32, Int32, Cint, Ptr{ShardPiece}, Int32, Int64,
                 Int64, Int64, Int32, Int32),
                h, comm, world, rank, et_dtype(T), plan, length(plan), prependrows, ld_dst,
                batch, chunks, exchange))
    ld, ws, lo, hi = Ref{Int64}(0), Ref{Int64}(0), Ref{Int64}(0), Ref{Int64}(0)
    check(ccall((:et_sharded_info, libembtab), Cint,
                (Ptr{Cvoid}, Ref{Int64}, Ref{Int64}, Ref{Int64}, Ref{Int64}), h[], ld, ws, lo, hi))
    S = ShardedPreallocation(h[], HipArray{UInt8}(undef, ws[]), rank, (lo[] + 1):hi[])
    finalizer(s -> ccall((:et_sharded_destroy, libembtab), Cint, (Ptr{Cvoid},), s.handle), S)
    return S
end

# maplookup!(PreallocationStrategy(k), dst, tables, I) with this rank's pieces: `tables`
# and `I` are the tables of this rank's plan entries, in plan order (whole tables for
# the table-wise plan).
function maplookup!(S::ShardedPreallocation, dst::HipMatrix{T}, tables::Vector{<:HipTable},
                    I0) where {T}
    I = EmbeddingTables.colwrap(I0)
    descs = Vector{LookupDesc}(undef, length(tables))
    for (t, (A, i)) in enumerate(zip(tables, I))
        pool = ndims(i) == 1 ? 1 : size(i, 1)
        tp, ldt, cpp = _device_table(A)
        descs[t] = LookupDesc(tp, ldt, size(A, 2), size(A, 1), pool, pointer(i), pool, 0, cpp)
    end
    check(ccall((:et_sharded_maplookup, libembtab), Cint,
                (Ptr{Cvoid}, Ptr{LookupDesc}, Int32, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, UInt32,
                 Ptr{Cvoid}),
                S.handle, descs, length(descs), dst.ptr, leading(dst), S.workspace.ptr,
                length(S.workspace), ET_FLAG_NONTEMPORAL, stream()))
    return dst
end

export HipEmbedding, HipSplitEmbedding, HipArray, HipVector, HipMatrix, EmbtabError,
    DeviceColumns, HipIndexer, ShardedPreallocation, shard_plan, comm_id, comm_init,
    comm_destroy, comm_loopback

end # module
