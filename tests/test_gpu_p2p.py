"""The one-sided exchange of a sharded maplookup ("fused P2P
xGMI writes"): et_push_cols against a plain copy, and the whole p2p step on 2 and 3
ranks (one process per rank, all on cuda:0, gloo for the handle exchange and the
barriers) against the oracle's single-process Preallocation result."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import embtab as et  # noqa: F401  (loads the library)
from embtab import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
HERE = os.path.dirname(os.path.abspath(__file__))


def _push(src, col, ncols, peers):
    L = _lib.load()
    arr = (ctypes.c_void_p * len(peers))(*[p.data_ptr() for p in peers])
    _lib.check(L.et_push_cols(_lib.et_dtype(src), src.data_ptr(), src.stride(0), src.shape[0],
                              col, ncols, ctypes.addressof(arr), len(peers),
                              _lib.stream_handle(src.device)))


@pytest.mark.parametrize("dtype,ld,col,ncols", [(torch.float32, 3344, 16, 416),
                                                (torch.float32, 37, 5, 11),
                                                (torch.float16, 3344, 0, 3344),
                                                (torch.float64, 100, 36, 64)])
def test_push_cols_matches_copy(dtype, ld, col, ncols):
    B = 301
    src = torch.randn((B, ld), device=DEV).to(dtype)
    peers = [torch.full((B, ld), 7, dtype=dtype, device=DEV) for _ in range(3)]
    _push(src, col, ncols, peers)
    torch.cuda.synchronize()
    for p in peers:
        assert torch.equal(p[:, col:col + ncols], src[:, col:col + ncols])
        assert bool((p[:, :col] == 7).all()) and bool((p[:, col + ncols:] == 7).all())


def test_push_cols_rejects_bad_arguments():
    L = _lib.load()
    src = torch.zeros((4, 8), device=DEV)
    arr = (ctypes.c_void_p * 1)(src.data_ptr())
    addr = ctypes.addressof(arr)
    assert L.et_push_cols(_lib.ET_F32, src.data_ptr(), 8, 4, 4, 5, addr, 1, None) == -1
    assert L.et_push_cols(_lib.ET_F32, src.data_ptr(), 8, 4, 0, 8, addr, 17, None) == -1
    assert L.et_push_cols(_lib.ET_F32, src.data_ptr(), 8, 4, 0, 8, addr, 0, None) == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_sharded_prealloc(world, tmp_path):
    out = str(tmp_path / "res")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(HERE, "workers", "p2p_rank.py"), out]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = []
    for k in range(world):
        with open(f"{out}.{k}") as f:
            res += json.load(f)
    assert len(res) == world * 3 * 2
    assert all(x["ok"] for x in res), [x for x in res if not x["ok"]]
