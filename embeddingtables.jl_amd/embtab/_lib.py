"""ctypes binding of libembtab_hip.so — the C ABI declared in include/embtab.h.

The product path calls the HIP library only; there is no CPU fallback.  If the
library is missing the import fails loudly with the command that builds it.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads torch's HIP runtime first, so the library shares it)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ET_LIBRARY: an alternative build of the same library (the profiling builds under tools/).
# An EXPERIMENT build (tools/exp_build.sh, -DET_EXPERIMENTS: it reads ET_* tuning knobs from
# the environment and exports et_debug_chain_timeline) is refused unless the process opts in
# with ET_TOOLS_EXPERIMENT=1, which only the scripts under tools/ set — so no environment can
# swap a knob-reading library under the tests, smoke() or bench.py by accident.
LIB_PATH = os.environ.get("ET_LIBRARY") or os.path.join(_HERE, "libembtab_hip.so")
EXPERIMENT_MARKER = "et_debug_chain_timeline"
EXPERIMENT_BUILD = False  # set by load(): the loaded library is an experiment build

ET_OK = 0
ET_F32, ET_F16, ET_F64, ET_I32, ET_I64, ET_BF16 = 0, 1, 2, 3, 4, 5
ET_FLAG_NONTEMPORAL = 1
ET_FLAG_F16_FP32_ACC = 2
ET_FLAG_EXACT_UPDATE = 4
ET_FLAG_EXACT_IF_FAST = 256
ET_FLAG_SGD_UNFUSED = 8
ET_FLAG_SGD_F64_ALPHA = 16
ET_FLAG_SGD_INDEX_ONLY = 32
ET_FLAG_SGD_APPLY_ONLY = 64
ET_FLAG_SGD_HOT_PASS = 128
ET_MAX_TABLES_PER_LAUNCH = 32
ET_SGD_CHUNK = 256  # include/embtab.h: occurrences per chunk of the non-exact SGD
ET_ABI_VERSION = 9
ET_LOOKUP_QUEUE_BYTES = 128  # include/embtab.h: et_maplookup_prealloc_q queue block
ET_MAX_PEERS = 16
ET_PLAN_TABLEWISE, ET_PLAN_FEATUREWISE = 0, 1
ET_EXCHANGE_ALLGATHER, ET_EXCHANGE_ALLTOALL = 0, 1
ET_COMM_ID_BYTES = 128

TORCH_TO_ET = {
    torch.float32: ET_F32,
    torch.float16: ET_F16,
    torch.float64: ET_F64,
    torch.int32: ET_I32,
    torch.int64: ET_I64,
    torch.bfloat16: ET_BF16,
}

# Every entry point declared in include/embtab.h.
EXPORTS = (
    "et_abi_version",
    "et_last_error",
    "et_gather",
    "et_pooled_sum",
    "et_maplookup_prealloc",
    "et_maplookup_prealloc_q",
    "et_maplookup_prealloc_to",
    "et_sgd_workspace_size",
    "et_sparse_sgd",
    "et_sparse_sgd_snap",
    "et_index_workspace_size",
    "et_index_build",
    "et_update_indexed",
    "et_concat_slabs",
    "et_split_slabs",
    "et_push_cols",
    "et_ipc_handle",
    "et_ipc_open",
    "et_ipc_close",
    "et_shard_plan",
    "et_comm_unique_id",
    "et_comm_init",
    "et_comm_destroy",
    "et_comm_loopback",
    "et_allgather_concat",
    "et_sharded_create",
    "et_sharded_info",
    "et_sharded_maplookup",
    "et_sharded_piece_grads",
    "et_sharded_destroy",
    "et_fill_uniform",
    "et_fill_index_uniform",
    "et_check_errors",
)


class EmbtabError(RuntimeError):
    """A C-ABI call returned a non-zero status."""


class LookupDesc(ctypes.Structure):
    """et_lookup_desc (include/embtab.h)."""

    _fields_ = [
        ("table", ctypes.c_void_p),
        ("ld_table", ctypes.c_int64),
        ("nrows", ctypes.c_int64),
        ("dim", ctypes.c_int32),
        ("pool", ctypes.c_int32),
        ("idx", ctypes.c_void_p),
        ("ld_idx", ctypes.c_int64),
        ("dst_row_off", ctypes.c_int64),
        ("cols_per_page", ctypes.c_int64),
    ]


class ShardPiece(ctypes.Structure):
    """et_shard_piece (include/embtab.h)."""

    _fields_ = [
        ("rank", ctypes.c_int32),
        ("table", ctypes.c_int32),
        ("f0", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("col", ctypes.c_int64),
    ]


class UpdateDesc(ctypes.Structure):
    """et_update_desc (include/embtab.h)."""

    _fields_ = [
        ("table", ctypes.c_void_p),
        ("ld_table", ctypes.c_int64),
        ("nrows", ctypes.c_int64),
        ("dim", ctypes.c_int32),
        ("pool", ctypes.c_int32),
        ("delta", ctypes.c_void_p),
        ("ld_delta", ctypes.c_int64),
        ("idx", ctypes.c_void_p),
        ("ld_idx", ctypes.c_int64),
        ("batch", ctypes.c_int64),
        ("cols_per_page", ctypes.c_int64),
    ]


_lib = None


def load() -> ctypes.CDLL:
    """Load libembtab_hip.so (once) and declare the signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "from the repository root (hipcc --offload-arch=gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    global EXPERIMENT_BUILD
    EXPERIMENT_BUILD = hasattr(L, EXPERIMENT_MARKER)
    if EXPERIMENT_BUILD and os.environ.get("ET_TOOLS_EXPERIMENT") != "1":
        raise ImportError(
            f"{LIB_PATH} is an experiment build of the library (it reads ET_* knobs from the "
            "environment); the package loads it only for the tools under tools/, which set "
            "ET_TOOLS_EXPERIMENT=1")
    vp, i64, i32, u32, u64, dbl, c_int = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double,
                                          ctypes.c_int)
    sig = {
        "et_abi_version": ([], c_int),
        "et_last_error": ([], ctypes.c_char_p),
        "et_gather": ([c_int, vp, i64, i64, i32, vp, i64, vp, i64, u32, vp], c_int),
        "et_pooled_sum": ([c_int, vp, i64, i64, i32, vp, i32, i64, i64, vp, i64, u32, vp], c_int),
        "et_maplookup_prealloc": ([c_int, vp, i32, i64, vp, i64, u32, vp], c_int),
        "et_maplookup_prealloc_q": ([c_int, vp, i32, i64, vp, i64, u32, vp, vp], c_int),
        "et_maplookup_prealloc_to": ([c_int, c_int, vp, i32, i64, vp, i64, u32, vp], c_int),
        "et_sgd_workspace_size": ([vp, i32, vp], c_int),
        "et_sparse_sgd": ([c_int, vp, i32, dbl, u32, vp, i64, vp], c_int),
        "et_sparse_sgd_snap": ([c_int, vp, i32, dbl, u32, vp, vp, i64, vp], c_int),
        "et_index_workspace_size": ([i64, vp], c_int),
        "et_index_build": ([vp, i32, i64, i64, i64, vp, vp, vp, vp, vp, i64, vp], c_int),
        "et_update_indexed": ([c_int, vp, i64, i64, i64, i32, vp, i64, vp, vp, i64, i64, vp, dbl, u32,
                               vp], c_int),
        "et_concat_slabs": ([c_int, vp, i32, i64, i64, vp, vp, vp, i64, vp], c_int),
        "et_split_slabs": ([c_int, vp, i64, i64, i32, vp, vp, vp, i64, vp], c_int),
        "et_push_cols": ([c_int, vp, i64, i64, i64, i64, vp, i32, vp], c_int),
        "et_ipc_handle": ([vp, vp, vp], c_int),
        "et_ipc_open": ([vp, i64, vp], c_int),
        "et_ipc_close": ([vp, i64], c_int),
        "et_shard_plan": ([i32, i32, vp, vp, i32, i64, i32, i32, vp, i32, vp], c_int),
        "et_comm_unique_id": ([vp], c_int),
        "et_comm_init": ([vp, i32, vp, i32], c_int),
        "et_comm_destroy": ([vp], c_int),
        "et_comm_loopback": ([vp, i32], c_int),
        "et_allgather_concat": ([vp, c_int, vp, i64, i64, vp, i32, vp, vp, vp, i64, vp], c_int),
        "et_sharded_create": ([vp, vp, i32, i32, c_int, vp, i32, i64, i64, i64, i32, i32], c_int),
        "et_sharded_info": ([vp, vp, vp, vp, vp], c_int),
        "et_sharded_maplookup": ([vp, vp, i32, vp, i64, vp, i64, u32, vp], c_int),
        "et_sharded_piece_grads": ([vp, vp, i64, vp, vp, i64, vp], c_int),
        "et_sharded_destroy": ([vp], c_int),
        "et_fill_uniform": ([c_int, vp, i64, u64, u64, dbl, dbl, vp], c_int),
        "et_fill_index_uniform": ([vp, i64, i64, u64, u64, vp], c_int),
        "et_check_errors": ([vp], c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if L.et_abi_version() != ET_ABI_VERSION:
        raise ImportError(f"ABI mismatch: library {L.et_abi_version()} != {ET_ABI_VERSION}")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != ET_OK:
        msg = load().et_last_error()
        raise EmbtabError(f"embtab status {rc}: {msg.decode() if msg else ''}")


def stream_handle(device=None) -> int:
    """hipStream_t of torch's current stream (where torch.cuda.Event records)."""
    return torch.cuda.current_stream(device).cuda_stream


def et_dtype(t: torch.Tensor) -> int:
    try:
        return TORCH_TO_ET[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported element type {t.dtype}") from None


def check_errors() -> int:
    """Synchronise; return and clear the device count of out-of-range indices."""
    v = ctypes.c_uint64(0)
    check(load().et_check_errors(ctypes.byref(v)))
    return int(v.value)
