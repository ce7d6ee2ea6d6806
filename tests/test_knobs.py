"""The shipped library reads no environment variable.

Every tuning knob of the kernels is ET_KNOB(name, default) (csrc/et_common.h): a
compile-time constant in the library the package loads, an environment read only in the
experiment build (-DET_EXPERIMENTS, tools/exp_build.sh).  So no user environment can change
what the shipped library computes or how it schedules it.  Checked three ways, without a
GPU: the built library imports no getenv and carries no knob name; every getenv in the
sources sits inside an `#ifdef ET_EXPERIMENTS` block; and the timing-only knob that gave
wrong results (ET_CHAIN_FAKE) and the non-default chain walks it served are gone."""
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "embeddingtables.jl_amd", "csrc")

# Runtime knobs the shipped library may read (each would need a -m gpu test that sets it in
# a subprocess and compares with the oracle): none.
ALLOWED_RUNTIME_KNOBS: set = set()


def _lib_path():
    from embtab import _lib

    return _lib.LIB_PATH


def test_shipped_library_imports_no_getenv():
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib_path()], capture_output=True,
                         text=True, check=True).stdout
    names = set(re.findall(r"\bU (\w+)", out))
    assert not ({"getenv", "secure_getenv", "__secure_getenv"} & names)


def test_shipped_library_carries_no_knob_names():
    out = subprocess.run(["strings", "-n", "4", _lib_path()], capture_output=True, text=True,
                         check=True).stdout
    knobs = {w for w in re.findall(r"\bET_[A-Z][A-Z0-9_]+\b", out)}
    assert knobs <= ALLOWED_RUNTIME_KNOBS, sorted(knobs - ALLOWED_RUNTIME_KNOBS)


def _getenv_outside_experiments(text: str):
    """Lines calling getenv( that are not inside an #ifdef ET_EXPERIMENTS block (nested
    #if blocks tracked; `#if ...` / `#else` flip as C does)."""
    bad, stack = [], []  # stack of "inside ET_EXPERIMENTS" flags per open #if
    for n, line in enumerate(text.split("\n"), 1):
        s = line.strip()
        if re.match(r"#\s*if(def|ndef)?\b", s):
            stack.append(bool(re.match(r"#\s*ifdef\s+ET_EXPERIMENTS\b", s)) or
                         bool(re.match(r"#\s*if\s+defined\(ET_EXPERIMENTS\)", s)))
        elif re.match(r"#\s*else\b", s) and stack:
            stack[-1] = False
        elif re.match(r"#\s*endif\b", s) and stack:
            stack.pop()
        elif "getenv(" in s and not s.startswith("//") and not any(stack):
            bad.append((n, s))
    return bad


def test_every_getenv_is_in_an_experiment_block():
    found = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".h", ".cpp")):
            text = open(os.path.join(CSRC, f)).read()
            found += [(f, n, s) for n, s in _getenv_outside_experiments(text)]
    assert not found, found


def test_the_parser_sees_a_bare_getenv():
    assert _getenv_outside_experiments('int x = atoi(getenv("ET_X"));')
    assert not _getenv_outside_experiments('#ifdef ET_EXPERIMENTS\nchar* e = getenv("X");\n#endif')
    assert _getenv_outside_experiments('#ifdef ET_EXPERIMENTS\n#else\nchar* e = getenv("X");\n#endif')


def test_wrong_result_knob_and_dead_walks_are_gone():
    src = "".join(open(os.path.join(CSRC, f)).read() for f in os.listdir(CSRC)
                  if f.endswith((".hip", ".h", ".cpp")))
    for gone in ("ET_CHAIN_FAKE", "ET_CHAIN_FED", "ET_CHAIN_RING", "chain_walk_ring",
                 "fed_gather_asm", "k_sgd_chains_fed", "hf_pair"):
        assert gone not in src, gone
