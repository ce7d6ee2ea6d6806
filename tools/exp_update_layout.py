import os, sys, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/embeddingtables.jl_amd")
import torch
import bench as bb
import embtab as et
from embtab import _lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
L = _lib.load()
T = len(bb.CRITEO_KAGGLE_ROWS); B = 65536; D = 128
tids = list(range(T))
tables = bb.make_tables(et, L, tids, dev)
gen = torch.Generator(device=dev); gen.manual_seed(4000)
idx = [bb.zipf_indices(bb.CRITEO_KAGGLE_ROWS[t], (B, 20), 1.05, gen, dev) for t in tids]
stream = torch.cuda.current_stream(dev)
delta = torch.empty((B, D * T), dtype=torch.float32, device=dev)
_lib.check(L.et_fill_uniform(_lib.ET_F32, delta.data_ptr(), delta.numel(), 4001, 0, -1.0, 1.0, stream.cuda_stream))
opt = et.Descent(0.1)
res = {}
for name in ["strided", "contig", "strided"]:
    if name == "strided":
        g = [et.SparseEmbeddingUpdate(A.lookup_type, delta[:, k*D:(k+1)*D], i) for k, (A, i) in enumerate(zip(tables, idx))]
    else:
        cd = [delta[:, k*D:(k+1)*D].contiguous() for k in range(T)]
        g = [et.SparseEmbeddingUpdate(A.lookup_type, cd[k], i) for k, (A, i) in enumerate(zip(tables, idx))]
    ix = [et.Indexer() for _ in tables]
    ms = bb._timed(lambda: et.update_(opt, tables, g, ix), 10, 2, stream)
    res[name] = ms
    print(name, ms, flush=True)
tr = bb._timed(lambda: [delta[:, k*D:(k+1)*D].contiguous() for k in range(T)], 10, 2, stream)
print("transpose cost", tr)
