"""Check that every `src/*.jl:N[-M]` / `test/*.jl:N[-M]` / `README.md:N` citation in the
repository points at lines that exist in the reference (run where /root/reference is)."""
import os
import re
import sys

REF = os.environ.get("REF", "/root/reference")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"((?:src|test)/\w+\.jl|README\.md):(\d+)(?:-(\d+))?((?:,\s*:?\d+(?:-\d+)?)*)")
SHORT = re.compile(r":?(\d+)(?:-(\d+))?")


def nlines(rel):
    try:
        with open(os.path.join(REF, rel), errors="replace") as f:
            return sum(1 for _ in f)
    except OSError:
        return None


def main():
    bad = 0
    for root, dirs, files in os.walk(REPO):
        dirs[:] = [d for d in dirs if d not in (".git", "gpurun_out", "scratch", "__pycache__",
                                                 "profiles")]
        for fn in files:
            if not fn.endswith((".py", ".md", ".h", ".hip", ".cpp", ".c", ".jl", ".sh")):
                continue
            if fn in ("VERDICT.md", "ADVICE.md", "SURVEY.md", "PAPERS.md", "SNIPPETS.md"):
                continue
            path = os.path.join(root, fn)
            for ln, line in enumerate(open(path, errors="replace"), 1):
                for m in PAT.finditer(line):
                    n = nlines(m.group(1))
                    if n is None:
                        continue
                    spans = [(m.group(2), m.group(3))] + SHORT.findall(m.group(4) or "")
                    for a, b in spans:
                        hi = int(b or a)
                        if int(a) < 1 or hi > n or (b and int(b) < int(a)):
                            bad += 1
                            print(f"{os.path.relpath(path, REPO)}:{ln}: {m.group(0)} "
                                  f"({m.group(1)} has {n} lines)")
    print(f"{bad} bad citation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
