"""Table abstraction — mirrors the reference's AbstractEmbeddingTable contract.

Reference: src/EmbeddingTables.jl:44-156 (AbstractEmbeddingTable, Static/Dynamic,
featuresize, indexing contexts, columnpointer, example, getindex/setindex!) and
src/simple.jl:1-57 (SimpleEmbedding).

Layout rule used everywhere in this package: a Julia array of size
``(d1, ..., dk)`` (column-major) is the contiguous torch tensor of shape
``(dk, ..., d1)``.  So a ``D x R`` table is a ``(R, D)`` tensor whose row ``r-1``
is Julia column ``r`` (one embedding vector, feature-contiguous), a ``P x B``
index matrix is a ``(B, P)`` tensor and a ``D x B`` output is a ``(B, D)`` tensor.
Indices are 1-based ``int64`` as in Julia.
"""
from __future__ import annotations

import torch


class ArgumentError(ValueError):
    """Julia's ArgumentError (constructor misuse, src/simple.jl:11-26)."""


# --- lookup types (src/EmbeddingTables.jl:60-63) -------------------------------------

class AbstractLookupType:
    pass


class _DynamicType(AbstractLookupType):
    def __repr__(self):
        return "Dynamic"

    def __eq__(self, other):
        return isinstance(other, _DynamicType)

    def __hash__(self):
        return hash("Dynamic")


Dynamic = _DynamicType()


class Static(AbstractLookupType):
    """``Static{N}``: feature size known up front (selects the reference's fused paths)."""

    def __init__(self, N):
        if isinstance(N, bool) or not isinstance(N, int):
            raise ArgumentError(
                f"Expected the type parameter for `Static{{N}}` to be an Int. "
                f"Instead, it's a {type(N).__name__}!")
        self.N = N

    def __repr__(self):
        return f"Static{{{self.N}}}"

    def __eq__(self, other):
        return isinstance(other, Static) and other.N == self.N

    def __hash__(self):
        return hash(("Static", self.N))


# --- indexing contexts (src/EmbeddingTables.jl:74-77) --------------------------------

class IndexingContext:
    pass


class NoContext(IndexingContext):
    pass


class Forward(IndexingContext):
    pass


class Update(IndexingContext):
    pass


# --- tables ---------------------------------------------------------------------------

class AbstractEmbeddingTable:
    """A D x R table of feature-contiguous columns on one GPU.

    Subtypes provide ``size()``, ``columnpointer(col, ctx)`` and ``example()``
    (README.md:288-307) — nothing else is required: the columns may sit anywhere in
    device memory (README.md:305-307: "this does not impose any requirement on the
    layout or ordering of the columns themselves").  ``device_table()`` turns the
    ``columnpointer`` contract into a kernel descriptor once per table:

    * equally spaced columns -> a contiguous descriptor (first column, ``ld`` = the
      spacing in elements);
    * anything else -> a device array of R column pointers, described as a paged table
      with one column per page (``cols_per_page = 1``), the generalisation of the
      SplitEmbedding page table.  16-byte aligned pointers (and a 16-byte multiple row)
      keep the vector kernels; otherwise ``ld`` is set to a non-16-byte spacing, which
      selects the generic (element-aligned) kernels — ``ld`` is never used to address a
      one-column page.

    Subtypes with a uniform layout (SimpleEmbedding, SplitEmbedding) override
    ``device_table``/``ld``; a subtype may also override ``columnpointers()`` to hand
    over all R pointers at once.  The descriptor is cached: call ``invalidate()`` after
    moving a table's columns.
    """

    lookup_type: AbstractLookupType = Dynamic

    def size(self):
        raise NotImplementedError

    def columnpointer(self, i: int, ctx: IndexingContext | None = None) -> int:
        raise ArgumentError(f"Please explicitly define `columnpointer` for {type(self).__name__}")

    def example(self) -> torch.Tensor:
        raise NotImplementedError

    def columnpointers(self):
        """Device addresses of columns 1..R (``columnpointer`` of each, by default)."""
        _, R = self.size()
        return [self.columnpointer(i) for i in range(1, R + 1)]

    def invalidate(self):
        self.__dict__.pop("_desc_cache", None)

    def _describe(self):
        c = self.__dict__.get("_desc_cache")
        if c is not None:
            return c
        import numpy as np

        D, R = self.size()
        es = self.example().element_size()
        if R == 0:
            raise ArgumentError("a table needs at least one column")
        p = np.asarray(self.columnpointers(), dtype=np.int64)
        if len(p) != R:
            raise ArgumentError(f"columnpointers() gave {len(p)} pointers for {R} columns")
        if R == 1:
            c = (int(p[0]), D, 0, None)
        else:
            d = np.diff(p)
            stride = int(d[0])
            if (d == stride).all() and stride > 0 and stride % es == 0 and stride // es >= D:
                c = (int(p[0]), stride // es, 0, None)
            else:
                if (p % es).any():
                    raise ArgumentError("column pointers must be aligned to the element size")
                vec = not (p % 16).any() and (D * es) % 16 == 0
                ld = D if vec or (D * es) % 16 else D + 1
                ptrs = torch.from_numpy(p).to(self.example().device)
                c = (ptrs.data_ptr(), ld, 1, ptrs)  # the tensor keeps the array alive
        self.__dict__["_desc_cache"] = c
        return c

    def device_table(self) -> tuple[int, int]:
        """``(table, cols_per_page)`` for an et_lookup_desc / et_update_desc (see the
        class docstring)."""
        t, _, cpp, _ = self._describe()
        return t, cpp

    @property
    def ld(self) -> int:
        """``ld_table`` of the descriptor (elements between columns)."""
        return self._describe()[1]

    @property
    def dtype(self):
        return self.example().dtype

    @property
    def device(self):
        return self.example().device

    def __len__(self):
        d, r = self.size()
        return d * r

    # AbstractArray getindex / setindex! through columnpointer
    # (src/EmbeddingTables.jl:144-156); device memory, so through a copy.
    def __getitem__(self, ij):
        i, j = ij
        d, r = self.size()
        if not (1 <= i <= d and 1 <= j <= r):
            raise IndexError(f"BoundsError: {ij} outside {self.size()}")
        return self._col(j)[i - 1].item()

    def __setitem__(self, ij, v):
        i, j = ij
        d, r = self.size()
        if not (1 <= i <= d and 1 <= j <= r):
            raise IndexError(f"BoundsError: {ij} outside {self.size()}")
        self._col(j)[i - 1] = v

    def _col(self, j: int) -> torch.Tensor:
        raise NotImplementedError


class SimpleEmbedding(AbstractEmbeddingTable):
    """Thin wrapper over a D x R column-major matrix (src/simple.jl:2-28).

    ``data`` is a CUDA tensor of shape ``(R, D)`` with unit feature stride;
    ``lookup_type`` is ``Dynamic`` (default) or ``Static(N)`` with ``N == D``.
    """

    def __init__(self, data: torch.Tensor, lookup_type: AbstractLookupType = Dynamic):
        if not isinstance(data, torch.Tensor) or data.dim() != 2:
            raise ArgumentError("SimpleEmbedding expects a 2-D (ncols, featuresize) tensor")
        if data.stride(1) != 1 and data.shape[1] > 1:
            raise ArgumentError("features of a column must be contiguous (stride(1) == 1)")
        if isinstance(lookup_type, Static):
            if lookup_type.N != data.shape[1]:
                raise ArgumentError(
                    "Parameter `N` should match the number of rows in the passed Matrix. "
                    f"Instead, `N = {lookup_type.N}` while `size(A,1) = {data.shape[1]}`.")
        elif lookup_type is not Dynamic:
            raise ArgumentError(f"unknown lookup type {lookup_type!r}")
        self.data = data
        self.lookup_type = lookup_type

    def __repr__(self):
        d, r = self.size()
        return f"{d}x{r} SimpleEmbedding{{{self.lookup_type!r}, {self.data.dtype}}}"

    def size(self):
        return (int(self.data.shape[1]), int(self.data.shape[0]))

    @property
    def ld(self) -> int:
        return int(self.data.stride(0)) if self.data.shape[0] > 1 else int(self.data.shape[1])

    def columnpointer(self, i: int, ctx: IndexingContext | None = None) -> int:
        """src/simple.jl:52-55: ``pointer(A) + (i - 1) * N * sizeof(T)`` (device address)."""
        return self.data.data_ptr() + (i - 1) * self.ld * self.data.element_size()

    def example(self) -> torch.Tensor:
        return self.data

    def _col(self, j: int) -> torch.Tensor:
        return self.data[j - 1]

    def zeros(self) -> "SimpleEmbedding":
        """``Base.zeros(::SimpleEmbedding)`` (src/simple.jl:30-34)."""
        return SimpleEmbedding(torch.zeros_like(self.data), self.lookup_type)

    def parent(self) -> torch.Tensor:
        return self.data


class SplitEmbedding(AbstractEmbeddingTable):
    """A table whose columns are stored in separately allocated pages of
    ``cols_per_shard`` columns each (src/split.jl:3-86).

    ``SplitEmbedding(data, cols_per_shard)`` copies a ``(R, D)`` tensor into
    ``ceil(R / cols_per_shard)`` page tensors (the last one may be short), like the
    reference's inner constructor (src/split.jl:11-26); the lookup type is always
    ``Static(D)``.  The kernels address a column through a device array of page
    pointers (``et_lookup_desc.cols_per_page``), so a paged table is looked up and
    updated by the same launches as a contiguous one."""

    def __init__(self, data: torch.Tensor, cols_per_shard: int = 1):
        if not isinstance(data, torch.Tensor) or data.dim() != 2:
            raise ArgumentError("SplitEmbedding expects a 2-D (ncols, featuresize) tensor")
        if int(cols_per_shard) < 1:
            raise ArgumentError("cols_per_shard must be positive")
        cps = int(cols_per_shard)
        R = int(data.shape[0])
        pages = [data[s:min(s + cps, R)].clone(memory_format=torch.contiguous_format)
                 for s in range(0, R, cps)]
        self._init(pages, int(data.shape[1]), cps, data.dtype, data.device)

    @classmethod
    def undef(cls, featuresize: int, ncols: int, cols_per_shard: int = 1,
              dtype=torch.float32, device="cuda", lookup_type: AbstractLookupType | None = None):
        """``SplitEmbedding{S,T}(undef, featuresize, ncols, cols_per_shard)``
        (src/split.jl:29-46); ``lookup_type = Static(N)`` must match ``featuresize``."""
        if isinstance(lookup_type, Static) and lookup_type.N != featuresize:
            raise ArgumentError(f"Static{{{lookup_type.N}}} != featuresize {featuresize}")
        cps = int(cols_per_shard)
        if cps < 1:
            raise ArgumentError("cols_per_shard must be positive")
        self = cls.__new__(cls)
        pages = [torch.empty((min(cps, ncols - s), featuresize), dtype=dtype, device=device)
                 for s in range(0, ncols, cps)]
        self._init(pages, featuresize, cps, dtype, device)
        if lookup_type is not None:
            self.lookup_type = lookup_type
        return self

    def _init(self, pages, D, cps, dtype, device):
        if not pages:
            raise ArgumentError("a SplitEmbedding needs at least one column")
        if any(p.data_ptr() % 16 for p in pages):
            raise ArgumentError("every page must be 16-byte aligned (include/embtab.h)")
        self.pages = pages
        self.matrixsize = (D, cps)
        self.lookup_type = Static(D)
        # the device page table the kernels read: one 8-byte pointer per page
        self.page_table = torch.tensor([p.data_ptr() for p in pages], dtype=torch.int64,
                                       device=device)

    def __repr__(self):
        d, r = self.size()
        return (f"{d}x{r} SplitEmbedding{{{self.lookup_type!r}, {self.dtype}}} "
                f"({len(self.pages)} pages of {self.matrixsize[1]})")

    def size(self):
        D, cps = self.matrixsize
        return (D, cps * (len(self.pages) - 1) + int(self.pages[-1].shape[0]))

    @property
    def ld(self) -> int:
        return self.matrixsize[0]

    @property
    def cols_per_page(self) -> int:
        return self.matrixsize[1]

    def _page_col(self, i: int):
        """``_divrem_index(i, shardsize)`` (src/split.jl:59-65), 0-based page/column."""
        return divmod(i - 1, self.matrixsize[1])

    def columnpointer(self, i: int, ctx: IndexingContext | None = None) -> int:
        """src/split.jl:81-86."""
        p, c = self._page_col(i)
        if not 0 <= p < len(self.pages):
            raise IndexError(f"BoundsError: column {i} outside {self.size()}")
        page = self.pages[p]
        return page.data_ptr() + c * self.ld * page.element_size()

    def device_table(self) -> tuple[int, int]:
        return self.page_table.data_ptr(), self.matrixsize[1]

    def example(self) -> torch.Tensor:
        return self.pages[0]

    def _col(self, j: int) -> torch.Tensor:
        p, c = self._page_col(j)
        return self.pages[p][c]

    def copy_(self, src: torch.Tensor) -> "SplitEmbedding":
        """``table .= base`` for a ``(R, D)`` tensor."""
        cps = self.matrixsize[1]
        for k, page in enumerate(self.pages):
            page.copy_(src[k * cps:k * cps + page.shape[0]])
        return self

    def to_dense(self) -> torch.Tensor:
        """All columns as one ``(R, D)`` tensor (``collect``)."""
        return torch.cat(self.pages, 0)

    def zeros(self) -> "SplitEmbedding":
        z = SplitEmbedding.undef(self.matrixsize[0], self.size()[1], self.matrixsize[1],
                                 self.dtype, self.device)
        for p in z.pages:
            p.zero_()
        return z


def featuresize(x) -> int:
    """src/EmbeddingTables.jl:71-72."""
    if isinstance(x, AbstractEmbeddingTable):
        return x.size()[0]
    return int(x.shape[-1])  # a (B, D) torch output is a D x B Julia matrix


def example(x):
    """src/EmbeddingTables.jl:118: ``example(first(x))`` for a vector of tables."""
    if isinstance(x, (list, tuple)):
        return x[0].example()
    return x.example()


def columnpointer(x, i: int, ctx: IndexingContext | None = None) -> int:
    if isinstance(x, AbstractEmbeddingTable):
        return x.columnpointer(i, ctx)
    # plain (N, D) tensor: pointer(A) + strides(A)[2] * sizeof(T) * (i - 1)
    return x.data_ptr() + (i - 1) * x.stride(0) * x.element_size()


def fused_update_path(table: AbstractEmbeddingTable) -> bool:
    """Which update kernel the reference dispatches to (src/sparseupdate.jl:131-154):
    the specialized fused `muladd` path for ``Static{N}`` tables with
    ``N * sizeof(T) <= MAX_ACCUMULATOR_SIZE / 2 = 512`` bytes, otherwise the
    generic scratch path (``x - alpha * y``)."""
    lt = table.lookup_type
    return isinstance(lt, Static) and lt.N * table.example().element_size() <= 512
