"""Index algebra of the exact update's quad walk (csrc/et_update.hip, chain_walk_quad),
simulated lane by lane on the CPU: the permuted entry-chunk load, DPP row_newbcast and the
permlane16 / permlane32 swaps (semantics as the CDNA4 ISA states them: permlane16_swap
exchanges the odd 16-lane rows of its first operand with the even rows of its second,
permlane32_swap the upper 32 lanes of the first with the lower 32 of the second) must put
a chain's entries into row 0 in serial order — the order the reference adds them
(src/sparseupdate.jl:110-127).  The GPU tests check the kernel's results bit for bit; this
test pins the lane arithmetic they rely on."""
import numpy as np


def permuted_chunk(entries, c):
    """Lane 16r + k of chunk c holds entry 4k + r (the kernel's poff = 4 * (4k + r))."""
    lane = np.arange(64)
    return entries[c * 64 + 4 * (lane & 15) + (lane >> 4)]


def row_newbcast(v, k):
    """DPP row_newbcast:k — lane k of every 16-lane row broadcast to its row."""
    return np.repeat(v.reshape(4, 16)[:, k], 16)


def permlane16_swap(a, b):
    a, b = a.reshape(4, 16).copy(), b.reshape(4, 16).copy()
    for r in (0, 2):  # odd rows of a <-> even rows of b
        a[r + 1], b[r] = b[r].copy(), a[r + 1].copy()
    return a.reshape(64), b.reshape(64)


def permlane32_swap(a, b):
    a, b = a.copy(), b.copy()
    a[32:], b[:32] = b[:32].copy(), a[32:].copy()
    return a, b


def quad_order(entries, nquads):
    """The sequence of entries row 0 adds, quad by quad, as chain_walk_quad does."""
    order = []
    for q in range(nquads):
        chunk = permuted_chunk(entries, q // 16)
        bag = row_newbcast(chunk, q % 16)  # row r: entry 4q + r
        v = bag.copy()                     # stands for the row's loaded gradient slice
        order.append(v[0])                                  # acc += x     (entry 4q)
        s32 = permlane32_swap(v, v)
        s16 = permlane16_swap(s32[0], s32[0])
        order.append(s16[1][0])                             # entry 4q + 1
        z = s32[1]
        order.append(z[0])                                  # entry 4q + 2
        t16 = permlane16_swap(z, z)
        order.append(t16[1][0])                             # entry 4q + 3
        # every lane of row 0 sees the same entry (the broadcast), so lane 0 stands for it
        assert len(set(bag[:16])) == 1
    return order


def test_quad_walk_adds_entries_in_serial_order():
    rng = np.random.default_rng(7)
    entries = rng.integers(0, 1 << 24, 64 * 6)
    got = quad_order(entries, 16 * 6)
    assert got == list(entries)


def test_row_r_gets_entry_4k_plus_r():
    entries = np.arange(128)
    for k in range(16):
        b = row_newbcast(permuted_chunk(entries, 1), k)
        assert list(b.reshape(4, 16)[:, 0]) == [64 + 4 * k + r for r in range(4)]
