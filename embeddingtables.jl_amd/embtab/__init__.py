"""embtab — the MI355X-native engine behind darchr/EmbeddingTables.jl's hot path.

The public names mirror the reference module's exports
(src/EmbeddingTables.jl:7-18); Julia's bang functions carry a trailing
underscore (``lookup_`` is ``lookup!``).  Every hot operation is one call into
libembtab_hip.so (include/embtab.h); importing this package loads that library
and fails if it has not been built.
"""
from . import _lib
from ._lib import EmbtabError, check_errors
from .tables import (AbstractEmbeddingTable, AbstractLookupType, ArgumentError, Dynamic,
                     Forward, IndexingContext, NoContext, SimpleEmbedding, SplitEmbedding, Static,
                     Update, columnpointer, example, featuresize)
from .lookup import (AbstractExecutionStrategy, DefaultStrategy, NoTangent,
                     PreallocationPlan, PreallocationStrategy, SimpleParallelStrategy, colwrap, destination, lookup,
                     lookup_, maplookup, maplookup_)
from .update import (AbstractIndexer, DenseIndexer, Descent, Indexer, IndexerView, PhasedUpdate,
                     SparseEmbeddingUpdate, SparseIndexer, ensemble_update, gettranslations,
                     index_, optimise_update_, rrule, uncompress, update_)

_lib.load()

__all__ = [
    "AbstractEmbeddingTable", "AbstractLookupType", "ArgumentError", "Dynamic", "Static",
    "IndexingContext", "NoContext", "Forward", "Update", "SimpleEmbedding", "SplitEmbedding",
    "featuresize", "example", "columnpointer", "AbstractExecutionStrategy", "DefaultStrategy",
    "SimpleParallelStrategy", "PreallocationStrategy", "PreallocationPlan", "NoTangent", "colwrap", "destination",
    "lookup", "lookup_", "maplookup", "maplookup_", "SparseEmbeddingUpdate", "uncompress",
    "rrule", "Descent", "AbstractIndexer", "Indexer", "SparseIndexer", "DenseIndexer",
    "IndexerView", "index_", "gettranslations", "update_", "optimise_update_",
    "ensemble_update", "PhasedUpdate", "EmbtabError", "check_errors",
]
