"""A symbolic run of the generated chain loops (tools/gen_chain_asm.py: body_stream, the
streamed loop for S = 8, 16; body_deep, the packed 64-deep loop for S = 1, 2, 4; body, the packed
32-deep loop) — no GPU needed.

The loop's correctness rests on its schedule: which SGPR holds which entry's gradient offset
or lane mask when an instruction reads it, which x register holds which entry's gradient row
when the fmacs read it, and whether every read comes after the wait that retires its load.
This test executes the generated instruction list over several trips on a model of those
registers and counters and checks, for every read:

* a buffer load's soffset SGPR holds the offset of the entry whose row it loads, landed
  (an `s_waitcnt lgkmcnt(0)` after its scalar load: scalar loads return out of order); in the
  packed loops its address VGPR was made from the entry a readlane took from a landed entry
  chunk, and the chunk moves only once landed;
* a mask's SGPR pair holds one entry's mask, landed; the fmacs of entry e read the mask
  made from entry e's pair, at least two instructions after it was written (the DPP
  read-after-VALU-write hazard), and the x register loaded with entry e's row, retired by an
  `s_waitcnt vmcnt(n)` (vector loads retire in order; a load issued while 63 are in flight
  waits for the oldest);
* the fmacs take the entries in order 0, 1, 2, ..., S per entry, every entry of every trip;
* nothing reads an SGPR or VGPR whose load is still in flight or was overwritten."""
import os
import re
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))
import gen_chain_asm as g  # noqa: E402


def _lines(S, DS):
    return _asm(g.body_stream(S, DS))


def _asm(text):
    return [m.group(1).replace("\\n\\t", "").strip() for m in re.finditer(r'"(.*?)"\s*$', text,
                                                                          re.M)
            if "\\n\\t" in m.group(1)]


def _sgprs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return [int(m.group(1))] if m else []


def _run(S, DS, trips, edit=None, text=None):
    L = _asm(text) if text is not None else _lines(S, DS)
    if edit:
        L = edit(L)
    head = L.index("1:")
    end = next(i for i, x in enumerate(L) if x.startswith("s_cbranch_scc1"))
    prologue, body, epilogue = L[:head], L[head + 1:end + 1], L[end + 1:]
    sg = {}          # sgpr -> (kind, entry, landed)
    vg = {}          # vgpr -> (kind, entry, landed, written_at)
    vq = []          # vector loads in flight, oldest first: vgpr numbers (None: prefetch)
    ptr = {"off": 0, "msk": 0, "ent": 0}  # entries the stream / entry pointers have advanced
    PO, PM = f"s[{g.PO}:{g.PO + 1}]", f"s[{g.PM}:{g.PM + 1}]"
    P0 = f"s[{g.P0}:{g.P0 + 1}]"
    vcc = [None]
    consumed = []    # entries whose fmacs ran, one per fmac
    step = [0]

    def land_vector(n_keep):
        while len(vq) > n_keep:
            r = vq.pop(0)
            if r is not None:
                k, e, _, w = vg[r]
                vg[r] = (k, e, True, w)

    def push_vector(r):
        if len(vq) == 63:  # the counter holds 63: this issue waits for the oldest
            land_vector(62)
        vq.append(r)

    def execute(ins):
        step[0] += 1
        op, _, rest = ins.partition(" ")
        args = [a.strip() for a in rest.split(",")] if rest else []
        if op.startswith("s_load_dwordx"):
            n = int(op[len("s_load_dwordx"):])
            dst, base, imm = _sgprs(args[0]), args[1], int(args[2], 0)
            assert len(dst) == n
            if base == PO:
                for k in range(n):
                    sg[dst[k]] = ("off", ptr["off"] + imm // 4 + k, False)
            else:
                assert base == PM, ins
                assert imm % 8 == 0
                for k in range(n):
                    sg[dst[k]] = ("msk", ptr["msk"] + imm // 8 + k // 2, False)
        elif op == "s_waitcnt":
            for part in rest.split():
                m = re.fullmatch(r"(vmcnt|lgkmcnt)\((\d+)\)", part)
                assert m, ins
                if m.group(1) == "lgkmcnt":
                    assert m.group(2) == "0", ins  # scalar loads return out of order
                    for r, v in list(sg.items()):
                        sg[r] = (v[0], v[1], True) + tuple(v[3:]) + tuple(sg[r][3:])
                else:
                    land_vector(int(m.group(2)))
        elif op == "buffer_load_dword":
            v = int(args[0][1:])
            if args[1] == "%[lane4]":  # streamed: the offset is the soffset SGPR
                soff = _sgprs(args[3].split()[0])
                k, e, landed = sg[soff[0]][:3]
                assert k == "off" and landed, (ins, sg[soff[0]])
            else:  # packed: the address VGPR made from the entry
                k, e, landed, _ = vg[int(args[1][1:])]
                assert k == "addr" and landed, (ins, k)
            vg[v] = ("x", e, False, step[0])
            push_vector(v)
        elif op.startswith("global_load"):
            base, *mods = args[2].split()
            if base == P0:  # a chunk of 64 entries (lane l: entry base + l)
                v = int(args[0][1:])
                imm = int(mods[0].split(":")[1]) if mods else 0
                vg[v] = ("chunk", ptr["ent"] + imm // 4, False, step[0])
                push_vector(v)
            else:
                push_vector(None)  # the streams' lines toward L2: sinks nobody reads
        elif op == "v_readlane_b32":
            r, v, lane = int(args[0][1:]), int(args[1][1:]), int(args[2])
            k, base, landed, _ = vg[v]
            assert k == "chunk" and landed, (ins, vg[v])
            sg[r] = ("ent", base + lane, True, step[0])
        elif op == "v_mad_u32_u24":
            r = int(args[1][1:])
            k, e, landed, w = sg[r]
            assert k == "ent", (ins, sg[r])  # a VALU read of a VALU-written SGPR: interlocked
            vg[int(args[0][1:])] = ("addr", e, True, step[0])
        elif op == "v_cmp_gt_u32_e32":
            k, e = sg[int(args[1][1:])][:2]
            assert k == "ent", ins
            vcc[0] = e
        elif op == "v_mov_b32_e32":
            src = vg[int(args[1][1:])]
            assert src[2], (ins, src)  # a chunk still in flight would move garbage
            vg[int(args[0][1:])] = src
        elif op == "v_add_f32_e32":  # S = 1: one add per entry
            kx, ex, landed, _ = vg[int(args[2][1:])]
            assert kx == "x" and landed, (ins, kx, ex, landed)
            consumed.append(ex)
        elif op == "v_cndmask_b32_e64":
            v = int(args[0][1:])
            if args[3] == "vcc":
                vg[v] = ("mask", vcc[0], True, step[0])
            else:
                pair = _sgprs(args[3])
                a, b = sg[pair[0]], sg[pair[1]]
                assert a[0] == "msk" and a[:2] == b[:2] and a[2] and b[2], (ins, a, b)
                vg[v] = ("mask", a[1], True, step[0])
        elif op == "v_fmac_f32_dpp":
            vm, vx = int(args[1][1:]), int(args[2].split()[0][1:])
            km, em, _, wm = vg[vm]
            kx, ex, landed, _ = vg[vx]
            assert km == "mask" and kx == "x" and landed, (ins, vg[vm], vg[vx])
            assert em == ex, (ins, em, ex)
            assert step[0] - wm >= 3, ins  # two instructions between the mask and its DPP read
            consumed.append(ex)
        elif op in ("s_add_u32", "s_addc_u32"):
            if op == "s_add_u32":
                reg = int(args[0][1:])
                if reg == g.P0:
                    ptr["ent"] += int(args[2]) // 4
                if reg == g.PO:
                    ptr["off"] += int(args[2]) // 4
                elif reg == g.PM:
                    ptr["msk"] += int(args[2]) // 8
        elif op == "s_nop":
            step[0] += int(args[0])  # s_nop n: n + 1 wait states
        elif op.startswith(("s_mov", "v_mbcnt", "v_lshlrev", "v_and", "v_or", "s_sub", "s_cmp",
                            "s_cbranch")):
            pass
        else:
            raise AssertionError(f"unmodelled instruction {ins!r}")

    for ins in prologue:
        execute(ins)
    for _ in range(trips):
        for ins in body:
            execute(ins)
    for ins in epilogue:
        execute(ins)
    return consumed


@pytest.mark.parametrize("S", g.STREAM_S)
@pytest.mark.parametrize("DS", [32, 64])
def test_streamed_loop_schedule(S, DS):
    trips = 4
    consumed = _run(S, DS, trips)
    want = [e for e in range(64 * trips) for _ in range(S)]
    assert consumed == want


def test_the_model_catches_a_wrong_ring_slot(monkeypatch):
    """The checker has teeth: an off ring indexed one slot off fails it."""
    real = g.s_off
    monkeypatch.setattr(g, "s_off", lambda j: real(j + 1))
    with pytest.raises(AssertionError):
        _run(16, 32, 2)


def _drop_nth(L, pred, n):
    idx = [i for i, x in enumerate(L) if pred(x)]
    return L[:idx[n]] + L[idx[n] + 1:]


@pytest.mark.parametrize("what", ["lgkmcnt", "vmcnt"])
def test_the_model_catches_a_missing_wait(what):
    """... and a wait dropped from the loop body fails it too."""
    head = lambda L: L.index("1:")  # noqa: E731
    with pytest.raises(AssertionError):
        _run(16, 32, 2, edit=lambda L: L[:head(L)] + _drop_nth(
            L[head(L):], lambda x: x.startswith("s_waitcnt") and what in x, 3))


@pytest.mark.parametrize("S", [1, 2, 4])
def test_packed_deep_loop_schedule(S):
    """The packed 64-deep loop (S = 1, 2, 4 in the shipped library): entries from a chunk VGPR
    by readlane, the address by v_mad, the mask by compare + select."""
    trips = 4
    consumed = _run(S, 0, trips, text=g.body_deep(S))
    assert consumed == [e for e in range(64 * trips) for _ in range(S)]


@pytest.mark.parametrize("S", [1, 8, 16])
def test_packed_loop_schedule(S):
    """The packed 32-deep loop (S = 8, 16 when the streamed loop is off, experiment builds)."""
    trips = 4
    consumed = _run(S, 0, trips, text=g.body(S))
    assert consumed == [e for e in range(64 * trips) for _ in range(S)]
