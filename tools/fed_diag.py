"""Diagnose the fed chain walk (ET_CHAIN_FED): one 3-row table, integer-valued gradients so
every column sum is exact in fp32 whatever the order; the per-(column, feature) error in
units of the gradient tells which occurrences were lost, doubled or misplaced.
Usage: ET_CHAIN_FED=1 python tools/fed_diag.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "embeddingtables.jl_amd"))
import embtab as et  # noqa: E402

DEV = torch.device("cuda:0")


def run(R, D, B, P, mode, seed=1):
    rng = np.random.default_rng(seed)
    I = rng.choice(np.arange(1, R + 1), size=(B, P), p=np.array([0.7, 0.2, 0.1][:R]) /
                   sum([0.7, 0.2, 0.1][:R])).astype(np.int64)
    h = np.zeros((R, D), np.float32)
    if mode == "ones":
        delta = np.ones((B, D), np.float32)
    elif mode == "bag":
        delta = np.repeat((np.arange(B, dtype=np.float32) + 1)[:, None], D, axis=1)
    else:  # feature-tagged: bag + 1 for feature f's own parity, 0 otherwise
        delta = (np.arange(B, dtype=np.float32)[:, None] + 1) * (np.arange(D)[None, :] % 2 == 0)
        delta = delta.astype(np.float32)
    A = et.SimpleEmbedding(torch.from_numpy(h).to(DEV), et.Static(D))
    g = et.SparseEmbeddingUpdate(A.lookup_type, torch.from_numpy(delta).to(DEV),
                                 torch.from_numpy(I).to(DEV))
    et.update_(et.Descent(1.0), A, g, exact=True)
    torch.cuda.synchronize()
    got = -A.data.cpu().numpy().astype(np.float64)
    want = np.zeros((R, D))
    for c in range(R):
        bags = np.nonzero(I == c + 1)[0]
        want[c] = delta[bags].astype(np.float64).sum(0)
    occ = [(I == c + 1).sum() for c in range(R)]
    print(f"R={R} D={D} B={B} P={P} mode={mode} occ={occ} fed={os.environ.get('ET_CHAIN_FED')}")
    for c in range(R):
        err = got[c] - want[c]
        bad = np.nonzero(err != 0)[0]
        print(f"  col {c}: want[0]={want[c][0]:.0f} got[0]={got[c][0]:.0f} bad features "
              f"{len(bad)}/{D} first {bad[:8].tolist()} err[:8]={err[:8].tolist()}")


if __name__ == "__main__":
    for args in [(3, 128, 300, 20, "ones"), (3, 128, 300, 20, "bag"), (3, 128, 300, 20, "tag"),
                 (3, 64, 3000, 20, "ones"), (3, 128, 20000, 20, "ones")]:
        run(*args)
