"""The C-ABI library loads, exports exactly what include/embtab.h declares, its
struct layouts match the ctypes mirrors, and argument errors come back as status
codes — all without touching a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "embtab.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(et_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from embtab import _lib

    L = _lib.load()
    decl = declared_functions()
    assert decl, "no declarations parsed"
    assert sorted(_lib.EXPORTS) == decl
    for name in decl:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (et_\w+)", out))
    assert set(decl) <= exported


def test_abi_version_and_last_error():
    from embtab import _lib

    L = _lib.load()
    assert L.et_abi_version() == _lib.ET_ABI_VERSION == 9
    assert isinstance(L.et_last_error(), bytes)


def test_struct_layouts_match_header(tmp_path):
    from embtab import _lib

    prog = tmp_path / "layout.c"
    prog.write_text(r'''
#include <stddef.h>
#include <stdio.h>
#include "embtab.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(et_lookup_desc), offsetof(et_lookup_desc, dim),
         offsetof(et_lookup_desc, idx), offsetof(et_lookup_desc, dst_row_off),
         sizeof(et_update_desc));
  printf("%zu %zu %zu\n", offsetof(et_update_desc, delta), offsetof(et_update_desc, idx),
         offsetof(et_update_desc, batch));
  printf("%zu %zu %zu\n", sizeof(et_shard_piece), offsetof(et_shard_piece, dim),
         offsetof(et_shard_piece, col));
  return 0;
}
''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(prog), "-o", str(exe)],
                   check=True)
    l1, l2, l3 = subprocess.run([str(exe)], capture_output=True, text=True,
                                check=True).stdout.split("\n")[:3]
    L, U = _lib.LookupDesc, _lib.UpdateDesc
    assert list(map(int, l1.split())) == [ctypes.sizeof(L), L.dim.offset, L.idx.offset,
                                          L.dst_row_off.offset, ctypes.sizeof(U)]
    assert list(map(int, l2.split())) == [U.delta.offset, U.idx.offset, U.batch.offset]
    S = _lib.ShardPiece
    assert list(map(int, l3.split())) == [ctypes.sizeof(S), S.dim.offset, S.col.offset]


def test_argument_errors_need_no_gpu():
    from embtab import _lib

    L = _lib.load()
    # ld_dst < dim is rejected before any device work
    rc = L.et_gather(_lib.ET_F32, None, 16, 10, 16, None, 5, None, 8, 0, None)
    assert rc == -1 and b"ld_dst" in L.et_last_error()
    # unknown dtype
    rc = L.et_pooled_sum(99, None, 16, 10, 16, None, 2, 2, 5, None, 16, 0, None)
    assert rc == -4
    # empty work is a no-op success
    assert L.et_gather(_lib.ET_F32, None, 16, 10, 16, None, 0, None, 16, 0, None) == 0
    # update supports F32 only
    assert L.et_sparse_sgd(_lib.ET_I32, None, 0, 0.1, 0, None, 0, None) == -4
    # workspace sizing is host-only arithmetic
    d = (_lib.UpdateDesc * 1)()
    d[0] = _lib.UpdateDesc(1 << 20, 128, 1000, 128, 20, 1 << 20, 128, 1 << 20, 20, 4096)
    nb = ctypes.c_int64(0)
    assert L.et_sgd_workspace_size(ctypes.addressof(d), 1, ctypes.byref(nb)) == 0
    assert nb.value > 20 * 4096 * 16
    assert L.et_index_workspace_size(1000, ctypes.byref(nb)) == 0 and nb.value > 0
    # too many tables for one update call
    big = (_lib.UpdateDesc * 33)()
    assert L.et_sgd_workspace_size(ctypes.addressof(big), 33, ctypes.byref(nb)) == -1


def test_phase_flags_need_no_gpu():
    """ET_FLAG_SGD_INDEX_ONLY / APPLY_ONLY are exclusive; INDEX_ONLY accepts NULL
    gradients (it never reads them) but still validates the index arrays; the workspace
    grows by the hot-column region only for dim-128, pool <= 32 tables."""
    from embtab import _lib

    L = _lib.load()
    d = (_lib.UpdateDesc * 1)()
    d[0] = _lib.UpdateDesc(1 << 20, 128, 1000, 128, 20, 0, 128, 1 << 20, 20, 4096)
    both = _lib.ET_FLAG_SGD_INDEX_ONLY | _lib.ET_FLAG_SGD_APPLY_ONLY
    assert L.et_sparse_sgd(_lib.ET_F32, ctypes.addressof(d), 1, 0.1, both, None, 0, None) == -1
    assert b"INDEX_ONLY" in L.et_last_error()
    # delta NULL: an argument error for a full call, not for the index phase (which then
    # stops at the missing workspace, before any device work)
    assert L.et_sparse_sgd(_lib.ET_F32, ctypes.addressof(d), 1, 0.1, 0, None, 0, None) == -1
    rc = L.et_sparse_sgd(_lib.ET_F32, ctypes.addressof(d), 1, 0.1, _lib.ET_FLAG_SGD_INDEX_ONLY,
                         None, 0, None)
    assert rc == -3 and b"workspace" in L.et_last_error()
    d[0].idx = 0
    rc = L.et_sparse_sgd(_lib.ET_F32, ctypes.addressof(d), 1, 0.1, _lib.ET_FLAG_SGD_INDEX_ONLY,
                         None, 0, None)
    assert rc == -1
    sizes = []
    for dim, pool in ((128, 20), (64, 20), (128, 40)):
        d[0] = _lib.UpdateDesc(1 << 20, dim, 1000, dim, pool, 1 << 20, dim, 1 << 20, pool, 4096)
        nb = ctypes.c_int64(0)
        assert L.et_sgd_workspace_size(ctypes.addressof(d), 1, ctypes.byref(nb)) == 0
        sizes.append(nb.value)
    # the dim-128 pool-20 table carries 120 slots x 4 windows x 512 B of window partials
    assert sizes[0] > 120 * 4 * 512 + 20 * 4096 * 16


def test_shard_plan_is_host_only():
    """et_shard_plan: SURVEY.md §8e's 26-table split, argument errors, count query."""
    from embtab import _lib
    from embtab.sharding import native_plan

    L = _lib.load()
    p = native_plan(_lib.ET_PLAN_TABLEWISE, [128] * 26, 8)
    assert [len(x) for x in p] == [4, 4, 3, 3, 3, 3, 3, 3]
    assert [q.col for x in p for q in x] == [128 * t for t in range(26)]
    f = native_plan(_lib.ET_PLAN_FEATUREWISE, [128] * 26, 8, prependrows=16)
    assert [sum(q.dim for q in x) for x in f] == [416] * 8
    assert all(q.dim in (32, 64, 128) and q.col >= 16 for x in f for q in x)
    dims = (ctypes.c_int32 * 2)(5, 7)
    n = ctypes.c_int32(0)
    assert L.et_shard_plan(0, 2, ctypes.addressof(dims), None, 0, 0, 32, 4, None, 0,
                           ctypes.byref(n)) == -1
    assert L.et_shard_plan(7, 2, ctypes.addressof(dims), None, 2, 0, 32, 4, None, 0,
                           ctypes.byref(n)) == -1
    assert L.et_shard_plan(1, 2, ctypes.addressof(dims), None, 2, 0, 32, 4, None, 0,
                           ctypes.byref(n)) == 0 and n.value == 2
    one = (_lib.ShardPiece * 1)()
    assert L.et_shard_plan(1, 2, ctypes.addressof(dims), None, 2, 0, 32, 4,
                           ctypes.addressof(one), 1, ctypes.byref(n)) == -1
    # a sharded step without a communicator is world 1 only
    h = ctypes.c_void_p()
    assert L.et_sharded_create(ctypes.byref(h), None, 2, 0, _lib.ET_F32, None, 0, 0, 16, 8, 1,
                               0) == -1
    assert b"communicator" in L.et_last_error()
