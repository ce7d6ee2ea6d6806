"""The Julia side of the boundary, checked mechanically (no Julia toolchain here).

EmbeddingTablesHIP.jl is the host layer the north star asks for; it reaches the library
only through `ccall((:et_*, libembtab), Cint, (argument types...), args...)`.  This test
parses every such ccall and the shim's three `struct`s (LookupDesc, UpdateDesc,
ShardPiece) and checks them against include/embtab.h: the symbol is declared, the return
type is `int`, the arity matches, every argument has the C width and class (integer of
the same size, double, pointer) of the declared parameter, and every struct field has the
header's name order and type.  The multi-table update! must do no host-side indexing by
default (the reference's serial index! per table on downloaded indices)."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(REPO, "embeddingtables.jl_amd", "julia", "EmbeddingTablesHIP.jl")
HEADER = os.path.join(REPO, "include", "embtab.h")

# Julia ccall argument types -> C class
JL = {
    "Cint": "i32", "Int32": "i32", "UInt32": "u32", "Int64": "i64", "UInt64": "u64",
    "Float64": "f64", "Cstring": "ptr", "Csize_t": "u64",
}
# C parameter types -> class
C = {
    "int": "i32", "int32_t": "i32", "uint32_t": "u32", "int64_t": "i64", "uint64_t": "u64",
    "double": "f64",
}


def jl_class(t: str) -> str:
    t = t.strip()
    if t.startswith(("Ptr{", "Ref{")):
        return "ptr"
    return JL[t]


def c_class(decl: str) -> str:
    decl = re.sub(r"\bconst\b", "", decl).strip()
    if "*" in decl:
        return "ptr"
    typ = decl.split()[0]
    return C[typ]


def header_functions():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?(\w+)\s*(\**)\s*(et_\w+)\s*\(([^)]*)\)\s*;", src,
                         re.M | re.S):
        ret, star, name, params = m.group(1), m.group(2), m.group(3), m.group(4)
        params = " ".join(params.split())
        args = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
        out[name] = (ret + star, [c_class(a) for a in args])
    return out


def header_structs():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\}\s*\w+;", src, re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = " ".join(line.split())
            if not line:
                continue
            name = re.findall(r"\**(\w+)$", line)[0]
            fields.append((name, c_class(line[: line.rfind(name)] + ("" if "*" not in line else "*"))))
        out[m.group(1)] = fields
    return out


def shim_ccalls():
    src = open(SHIM).read()
    src = re.sub(r"#.*", "", src)
    out = []
    for m in re.finditer(r"ccall\(\(:(et_\w+),\s*libembtab\),\s*(\w+),\s*\(([^()]*)\)", src, re.S):
        name, ret, tup = m.group(1), m.group(2), " ".join(m.group(3).split())
        # split at top-level commas (types carry braces: Ptr{Ptr{Cvoid}})
        parts, depth, cur = [], 0, ""
        for ch in tup:
            if ch == "{":
                depth += 1
            elif ch == "}":
                depth -= 1
            if ch == "," and depth == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += ch
        if cur.strip():
            parts.append(cur)
        out.append((name, ret, [p.strip() for p in parts if p.strip()]))
    return out


def shim_structs():
    src = open(SHIM).read()
    out = {}
    for m in re.finditer(r"^struct (\w+)\n(.*?)^end", src, re.S | re.M):
        fields = re.findall(r"^\s+(\w+)::([\w{}]+)", m.group(2), re.M)
        out[m.group(1)] = fields
    return out


def test_every_ccall_matches_the_header():
    decl = header_functions()
    calls = shim_ccalls()
    assert len(calls) >= 20, "ccall parser found too few calls"
    seen = set()
    for name, ret, args in calls:
        assert name in decl, f"{name} is not declared in include/embtab.h"
        cret, cargs = decl[name]
        if name == "et_last_error":
            assert ret == "Cstring" and cret == "char*"
        else:
            assert ret == "Cint" and cret == "int", (name, ret, cret)
        got = [jl_class(a) for a in args]
        assert len(got) == len(cargs), (name, len(got), len(cargs))
        assert got == cargs, (name, got, cargs)
        seen.add(name)
    # the hot-path entries the shim exists for are all bound
    for must in ("et_gather", "et_pooled_sum", "et_maplookup_prealloc",
                 "et_maplookup_prealloc_to", "et_sgd_workspace_size", "et_sparse_sgd",
                 "et_index_workspace_size", "et_index_build", "et_update_indexed",
                 "et_shard_plan", "et_comm_unique_id", "et_comm_init", "et_comm_destroy",
                 "et_comm_loopback", "et_sharded_create", "et_sharded_info",
                 "et_sharded_maplookup", "et_sharded_destroy"):
        assert must in seen, must


JL_FIELD = {"Ptr{Cvoid}": "ptr", "Ptr{Int64}": "ptr", "Int64": "i64", "Int32": "i32"}


def test_shim_structs_match_the_header():
    hs = header_structs()
    js = shim_structs()
    for jl, c in (("LookupDesc", "et_lookup_desc"), ("UpdateDesc", "et_update_desc"),
                  ("ShardPiece", "et_shard_piece")):
        assert jl in js and c in hs, (jl, c)
        jf = [(n, JL_FIELD[t]) for n, t in js[jl]]
        assert jf == hs[c], (jl, jf, hs[c])


def _multi_table_update_body() -> str:
    src = open(SHIM).read()
    m = re.search(r"function update!\(opt::Flux\.Descent, tables::AbstractVector.*?^end", src,
                  re.S | re.M)
    assert m, "multi-table update! not found"
    return m.group(0)


def test_multi_table_update_snapshots_through_et_sparse_sgd_snap():
    """the multi-table update! fills indexers[i] in its index phase as the
    reference does (src/sparseupdate.jl:210-213) and as the Python host does
    (embtab/update.py: Indexer._defer + et_sparse_sgd_snap): the snapshots ride in the update's
    own key pass, and no second sort (et_index_build / index!) runs on that path — a
    HipIndexer is indexed from its snapshot only when first read."""
    body = _multi_table_update_body()
    decl = header_functions()
    calls = [c for c in shim_ccalls() if c[0] == "et_sparse_sgd_snap"]
    assert calls, "the shim never binds et_sparse_sgd_snap"
    for name, ret, args in calls:  # the header's signature
        assert [jl_class(a) for a in args] == decl[name][1] and ret == "Cint"
    assert re.search(r"ccall\(\(:et_sparse_sgd_snap, libembtab\)", body)
    # the snapshot pointers handed to it are the HipIndexers' (last position of each object)
    assert "_snapshot!(indexers[i], grads[i].indices" in body
    # no second device sort per HipIndexer on this path
    assert "et_index_build" not in body and "index!(indexers[i], grads[i]" not in body
    code = re.sub(r"#.*", "", body)
    assert not re.search(r"(?<![.\w])index!\(", code)
    # the deferred build: reading a HipIndexer field materialises a pending snapshot
    src = open(SHIM).read()
    assert re.search(r"function Base\.getproperty\(ix::HipIndexer", src)
    assert "_materialise!(ix)" in src


def test_multi_table_update_fills_host_indexers_by_default():
    """A host Indexer (the reference's type) is filled by the reference's own index! by
    default, as the reference's index phase fills every indexers[i]; the flag turns it off."""
    body = _multi_table_update_body()
    assert "fill_host_indexers::Bool = true" in body
    host = body.index("EmbeddingTables.index!(")
    assert body.rfind("if fill_host_indexers", 0, host) != -1
    # before the telemetry callback and the apply phase (the reference's phase order)
    assert host < body.index("telemetry_cb()") < body.index("apply_phase()", host)


def test_single_table_update_fills_a_given_indexer():
    """src/sparseupdate.jl:159-178 indexes into the caller's `indexer` before updating: the
    shim's single-table update! snapshots for a HipIndexer (et_sparse_sgd_snap through
    _sparse_sgd) and fills a host Indexer with the reference's index!."""
    src = open(SHIM).read()
    m = re.search(r"function update!\(opt::Flux\.Descent, table::HipTable\{S,T\}.*?^end", src,
                  re.S | re.M)
    assert m, "single-table update! not found"
    body = m.group(0)
    assert "_snapshot!(indexer, grad.indices" in body
    assert "EmbeddingTables.index!(indexer, download(grad.indices)" in body
    m = re.search(r"function _sparse_sgd\(.*?^end", src, re.S | re.M)
    assert m and "ccall((:et_sparse_sgd_snap, libembtab)" in m.group(0)
