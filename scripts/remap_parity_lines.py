"""Keep docs/PARITY.md `path:line` citations pointing at the same source lines
after edits: maps every cited line of a changed file from the committed
version (git HEAD, or --rev) to the working tree with difflib and rewrites the
citation.  Lines that were deleted are reported for a manual look.

Idempotent: the citations are always mapped from PARITY.md as committed at
--rev (its text must otherwise equal the working copy's, or the script stops),
so running it twice between commits does not shift them twice.

    python scripts/remap_parity_lines.py [--rev HEAD] [--dry-run]
"""
import argparse
import difflib
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = "kafka_inferenceengine_amd"
CITE = re.compile(r"`((?:csrc|engine|inference|input_output|models|ops|parallel|utils)/[\w./]+):([\d,\-]+)")


def repo_path(rel: str) -> str:
    return rel if rel.startswith("csrc/") else f"{PKG}/{rel}"


def line_map(rev: str, path: str):
    try:
        old = subprocess.run(["git", "show", f"{rev}:{path}"], cwd=ROOT, capture_output=True, text=True,
                             check=True).stdout.splitlines()
    except subprocess.CalledProcessError:
        return None
    new = (ROOT / path).read_text().splitlines()
    m = {}
    # compared without indentation: a block moved into (or out of) a branch keeps its lines
    sm = difflib.SequenceMatcher(a=[ln.strip() for ln in old], b=[ln.strip() for ln in new], autojunk=False)
    for a, b, n in sm.get_matching_blocks():
        for k in range(n):
            m[a + k + 1] = b + k + 1
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rev", default="HEAD")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args()
    doc = ROOT / "docs" / "PARITY.md"
    work = doc.read_text()
    try:
        text = subprocess.run(["git", "show", f"{a.rev}:docs/PARITY.md"], cwd=ROOT, capture_output=True, text=True,
                              check=True).stdout
    except subprocess.CalledProcessError:
        text = work
    if CITE.sub("`CITE", text) != CITE.sub("`CITE", work):
        raise SystemExit("docs/PARITY.md has edits beyond citation numbers since " + a.rev +
                         ": commit them first (the citations are mapped from the committed text)")
    maps, lost = {}, []

    def fix(mo):
        rel, spec = mo.group(1), mo.group(2)
        path = repo_path(rel)
        if path not in maps:
            maps[path] = line_map(a.rev, path)
        m = maps[path]
        if m is None:
            return mo.group(0)
        parts = []
        for part in spec.split(","):
            first, dash, last = part.partition("-")
            nf = m.get(int(first))
            nl = m.get(int(last)) if dash else None
            if nf is None or (dash and nl is None):
                lost.append(f"{rel}:{part}")
                parts.append(part)
            else:
                parts.append(f"{nf}-{nl}" if dash else str(nf))
        return f"`{rel}:{','.join(parts)}"

    out = CITE.sub(fix, text)
    changed = sum(1 for x, y in zip(CITE.findall(text), CITE.findall(out)) if x != y)
    print(f"{changed} citations moved; {len(lost)} point at edited lines: {lost[:20]}")
    if not a.dry_run:
        doc.write_text(out)


if __name__ == "__main__":
    main()
