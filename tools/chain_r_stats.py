"""Distribution of r (adds per chain entry) over the early-chain lists of the config-4 batch
(VERDICT r05 item 3): for each table of at most 128 rows (the early chains), its hottest
columns' entries at the S the plan picks (k_ec_plan's cost rule), the share of masked (no-op)
fmac slots (S - r per entry), and what a per-trip body would issue instead (each 64-entry trip
at the maximum r of its entries, or at the next power of two).  CPU only: the bench's Zipf(1.05)
generator (bench.zipf_indices) on a CPU torch generator — the same distribution as the GPU
batch, not the same draw.
Usage: python tools/chain_r_stats.py [out.txt]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

COST2 = {0: 9, 1: 17, 2: 21, 3: 22, 4: 38}  # chain_entry_cost2(2^k), et_update.hip (round-6 streamed loop)
TRIP = 64


def entries_of(r, S):
    """The column's entries at S: ceil(r / S) per bag with r > 0, all S but the last."""
    out = []
    for x in r[r > 0]:
        k = -(-int(x) // S)
        out.extend([S] * (k - 1) + [int(x) - S * (k - 1)])
    return np.asarray(out, np.int64)


def main():
    import torch

    gen = torch.Generator()
    gen.manual_seed(4000)
    B, P = bench.BATCH, bench.POOL
    lines = []
    tot = {"fmac": 0, "adds": 0, "trip_max": 0, "trip_pow2": 0, "entries": 0}
    for R in bench.CRITEO_KAGGLE_ROWS:
        I = bench.zipf_indices(R, (B, P), 1.05, gen, "cpu").numpy()
        if R > 128:
            continue
        counts = np.bincount(I.ravel(), minlength=R + 1)[1:]
        for c in np.argsort(counts)[::-1][:3]:
            if counts[c] <= 256:  # not a chain (one chunk of the chunk pass)
                continue
            r = (I == c + 1).sum(1)
            E = [int(np.ceil(r[r > 0] / 2 ** k).sum()) for k in range(5)]
            k = min(range(5), key=lambda k: (E[k] * COST2[k], k))
            S = 2 ** k
            e = entries_of(r, S)
            n = len(e)
            pad = -(-n // TRIP) * TRIP
            ep = np.concatenate([e, np.zeros(pad - n, np.int64)]).reshape(-1, TRIP)
            tmax = ep.max(1)
            tpow2 = np.where(tmax <= 1, tmax, 2 ** np.ceil(np.log2(np.maximum(tmax, 1))))
            hist = np.bincount(e, minlength=S + 1)[1:]
            fm = n * S
            lines.append(
                f"R={R:4d} col={c:3d} occ={int(counts[c]):7d} S={S:2d} entries={n:6d} "
                f"mean_r={e.mean():5.2f} masked={(fm - e.sum()) / fm:5.3f} "
                f"trip_max_slots={int(tmax.sum()) * TRIP / fm:5.3f} "
                f"trip_pow2_slots={float(tpow2.sum()) * TRIP / fm:5.3f} r_hist(1..S)={hist.tolist()}")
            tot["fmac"] += fm
            tot["adds"] += int(e.sum())
            tot["trip_max"] += int(tmax.sum()) * TRIP
            tot["trip_pow2"] += int(tpow2.sum()) * TRIP
            tot["entries"] += n
    lines.append(f"all listed: masked share {(tot['fmac'] - tot['adds']) / tot['fmac']:.3f}, "
                 f"per-trip max-r body slots {tot['trip_max'] / tot['fmac']:.3f} of today's, "
                 f"per-trip pow2 body {tot['trip_pow2'] / tot['fmac']:.3f}")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(text + "\n")


if __name__ == "__main__":
    main()
