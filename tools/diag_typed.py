"""Diagnostic: which columns of a typed exact update differ from the oracle (per column:
occurrences, differing features), run twice for determinism.
Usage: python tools/diag_typed.py KIND R [B] [P] [dim]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "embeddingtables.jl_amd"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)


def main():
    import torch

    import embtab as et
    import oracle as orc
    from embtab.tables import fused_update_path

    kind = sys.argv[1]
    R = int(sys.argv[2])
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    P = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    dim = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(21)
    x = rng.standard_normal((R, dim)).astype(np.float32)
    d = rng.standard_normal((B, dim)).astype(np.float32)
    npdt = {"f64": np.float64, "f16": np.float16, "f16acc": np.float16, "f32": np.float32}
    if kind == "bf16":
        base, delta = orc.f32_to_bf16(x), orc.f32_to_bf16(d)
    else:
        base, delta = x.astype(npdt[kind]), d.astype(npdt[kind])
    gen = torch.Generator(device=dev)
    gen.manual_seed(22)
    u = torch.rand((B, P), generator=gen, device=dev, dtype=torch.float64)
    a1 = -0.05
    z = torch.floor(((float(R) ** a1 - 1.0) * u + 1.0) ** (1.0 / a1)).clamp_(1, R).long()
    I = torch.randperm(R, generator=gen, device=dev)[z - 1] + 1
    Ih = I.cpu().numpy()
    counts = np.bincount(Ih.ravel(), minlength=R + 1)[1:]
    outs = []
    for rep in range(2):
        tdev = torch.from_numpy(base).to(dev)
        ddev = torch.from_numpy(delta).to(dev)
        if kind == "bf16":
            tdev, ddev = tdev.view(torch.bfloat16), ddev.view(torch.bfloat16)
        A = et.SimpleEmbedding(tdev, et.Static(dim))
        g = et.SparseEmbeddingUpdate(A.lookup_type, ddev, I)
        et.update_(et.Descent(0.1), A, g, f16_fp32_acc=kind == "f16acc")
        got = (A.data.view(torch.int16) if kind not in ("f64", "f32") else A.data).cpu().numpy()
        outs.append(got)
    ref = base.copy()
    orc.sgd(ref, delta, Ih, 0.1, fused=fused_update_path(A), bf16=kind == "bf16",
            f16_fp32_acc=kind == "f16acc")
    ref = ref.view(outs[0].dtype)
    print("deterministic:", outs[0].tobytes() == outs[1].tobytes())
    bad = np.nonzero((outs[0] != ref).any(1))[0]
    print("columns differing:", len(bad), "of", R, "touched", int((counts > 0).sum()))
    for c in bad[:20]:
        nf = int((outs[0][c] != ref[c]).sum())
        print(f"col {c} occ {counts[c]} features differing {nf} first {np.nonzero(outs[0][c] != ref[c])[0][:8]}")
    print("occurrence histogram of differing columns:", sorted(counts[bad].tolist())[:40])


if __name__ == "__main__":
    main()
