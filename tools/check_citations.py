"""Check every `src/*.jl:N[-M]` / `test/*.jl:N[-M]` / `README.md:N` citation in the
repository against the reference (run where /root/reference is):

  * the cited lines exist;
  * the symbol named next to the citation is in the cited range: the identifiers written
    just before the citation on its line (backticked names first, else plain words) that
    occur anywhere in the cited file must include at least one that occurs in the cited
    lines (+-2 lines of slack) — a citation of `_divrem_index` whose range holds no
    `_divrem_index` is reported.  Lines whose candidates never occur in the file (prose)
    are not judged."""
import os
import re
import sys

REF = os.environ.get("REF", "/root/reference")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"((?:src|test)/\w+\.jl|README\.md):(\d+)(?:-(\d+))?((?:,\s*:?\d+(?:-\d+)?)*)")
SHORT = re.compile(r":?(\d+)(?:-(\d+))?")


_cache = {}


def ref_lines(rel):
    if rel not in _cache:
        try:
            with open(os.path.join(REF, rel), errors="replace") as f:
                _cache[rel] = f.read().split("\n")
        except OSError:
            _cache[rel] = None
    return _cache[rel]


def nlines(rel):
    lines = ref_lines(rel)
    return None if lines is None else len(lines) - (1 if lines and lines[-1] == "" else 0)


IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_!]*")
HEAD = re.compile(r"^(?:@\w+\s+)*(?:function|struct|mutable struct|abstract type)\b")
STOP = {"src", "test", "jl", "the", "and", "of", "in", "to", "for", "at", "is", "a", "an",
        "reference", "Replaces", "replaces", "see", "with", "on", "by", "from", "its", "as",
        "README", "md", "int", "const", "void", "T", "A", "I", "x", "y", "n", "t", "u", "k",
        "be", "or", "per", "each", "one", "this", "that", "it", "not", "no", "are", "was"}


def symbol_ok(rel, a, b, before):
    """None: not judged; True/False: a named symbol is / is not in the cited range."""
    lines = ref_lines(rel)
    if lines is None:
        return None
    # code-like names only (an underscore, a bang, an inner capital, or a call), so that
    # prose before a citation is not judged
    chunk = before[-70:]
    cands = [w for w in IDENT.findall(chunk) if w not in STOP and len(w) > 2 and
             ("_" in w or "!" in w or any(c.isupper() for c in w[1:]) or
              re.search(re.escape(w) + r"\(", chunk))]
    text = "\n".join(lines)
    cands = [w for w in cands if re.search(r"\b" + re.escape(w) + r"(?![A-Za-z0-9_])", text)]
    if not cands:
        return None
    lo, hi = max(1, a - 2), min(len(lines), b + 2)
    rng = "\n".join(lines[lo - 1:hi])
    # the header of the definition enclosing the range counts too (a citation of one phase
    # of `update!` names update!)
    for k in range(a - 1, -1, -1):
        if HEAD.match(lines[k]):
            j = k
            while j < len(lines) and j < k + 12 and ")" not in lines[j]:
                j += 1  # a multi-line signature
            rng += "\n" + "\n".join(lines[k:j + 1])
            break
    return any(re.search(r"(?<![A-Za-z0-9_])" + re.escape(w) + r"(?![A-Za-z0-9_])", rng)
               for w in cands)


def main():
    bad = mism = 0
    for root, dirs, files in os.walk(REPO):
        dirs[:] = [d for d in dirs if d not in (".git", "gpurun_out", "scratch", "__pycache__",
                                                 "profiles")]
        for fn in files:
            if not fn.endswith((".py", ".md", ".h", ".hip", ".cpp", ".c", ".jl", ".sh")):
                continue
            if fn in ("VERDICT.md", "ADVICE.md", "SURVEY.md", "PAPERS.md", "SNIPPETS.md",
                      "BASELINE.md"):
                continue
            path = os.path.join(root, fn)
            for ln, line in enumerate(open(path, errors="replace"), 1):
                for m in PAT.finditer(line):
                    n = nlines(m.group(1))
                    if n is None:
                        continue
                    spans = [(m.group(2), m.group(3))] + SHORT.findall(m.group(4) or "")
                    for k, (a, b) in enumerate(spans):
                        hi = int(b or a)
                        if int(a) < 1 or hi > n or (b and int(b) < int(a)):
                            bad += 1
                            print(f"{os.path.relpath(path, REPO)}:{ln}: {m.group(0)} "
                                  f"({m.group(1)} has {n} lines)")
                        elif k == 0 and symbol_ok(m.group(1), int(a), max(
                                int(y or x) for x, y in spans), line[:m.start()]) is False:
                            mism += 1
                            print(f"{os.path.relpath(path, REPO)}:{ln}: {m.group(0)}: the symbol "
                                  f"named before it is not in those lines")
    print(f"{bad} bad citation(s), {mism} symbol mismatch(es)")
    return 1 if bad or mism else 0


if __name__ == "__main__":
    sys.exit(main())
