"""Re-pin docs/PARITY.md `path:line` citations that name a symbol.

Most citations read ``name`` (`path:line`): a function, kernel, class or
struct next to the place it is defined.  This tool finds each such pair (the
last backticked identifier before the citation, within the same table cell)
and sets the line to the symbol's definition in the current tree -- the
definition nearest to the old line when the name is defined more than once.
Citations without a nearby symbol, or whose symbol has no definition in the
cited file, are left alone and listed.

    python scripts/pin_parity_symbols.py [--dry-run]
"""
import argparse
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = "kafka_inferenceengine_amd"
CITE = re.compile(r"`((?:csrc|engine|inference|input_output|models|ops|parallel|utils)/[\w./]+):(\d+(?:,\d+)*)`")
IDENT = re.compile(r"`([A-Za-z_][\w.]*)(?:\(\))?`")


def repo_path(rel: str) -> Path:
    return ROOT / (rel if rel.startswith("csrc/") else f"{PKG}/{rel}")


TYPES = re.compile(r"\b(?:void|float|bool|int|double|auto|hipError_t|uint8_t|int64_t|int32_t|uint32_t|KF_HD|static|"
                   r"inline|constexpr|__device__|__global__|__forceinline__|[A-Z]\w*Args|[A-Z]\w+)\b")


def definitions(path: Path, name: str):
    """Line numbers (1-based) where ``name`` is defined in ``path``."""
    name = name.split(".")[-1]
    lines = path.read_text().splitlines()
    n = re.escape(name)
    out = []
    if path.suffix == ".py":
        pat = re.compile(rf"^\s*(?:async\s+)?(?:def|class)\s+{n}\b|^\s*{n}\s*[:=]")
        return [i + 1 for i, ln in enumerate(lines) if pat.search(ln)]
    decl = re.compile(rf"^\s*(?:struct|class|enum)\s+{n}\b|^\s*#define\s+{n}\b|^\s*constexpr\s+[\w:<>]+\s+{n}\b")
    use = re.compile(rf"\b{n}\s*(?:<[^;()]*>)?\s*\(")
    for i, ln in enumerate(lines):
        if ln.lstrip().startswith("//"):
            continue
        if decl.search(ln):
            out.append(i + 1)
            continue
        m = use.search(ln)
        if not m:
            continue
        pre = ln[:m.start()]
        while re.search(r"\([^()]*\)", pre):           # __launch_bounds__(BS, MINW) and the like
            pre = re.sub(r"\([^()]*\)", "", pre)
        if any(t in pre for t in ("=", "return", "->", ".", ",", "(")) or not pre.strip():
            continue
        if TYPES.search(pre) and pre.rstrip()[-1:] not in "(":
            out.append(i + 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args()
    doc = ROOT / "docs" / "PARITY.md"
    text = doc.read_text()
    moved, kept = 0, []
    out_lines = []
    for line in text.splitlines(keepends=True):
        pieces, last = [], 0
        for mo in CITE.finditer(line):
            rel, olds = mo.group(1), [int(v) for v in mo.group(2).split(",")]
            old = olds[0]
            cell_start = line.rfind("|", 0, mo.start()) + 1
            # the symbol: nearest backticked identifier in the citation's cell, else
            # in the row's first cell (the reference component the row maps)
            before = line[cell_start:mo.start()]
            names = [m.group(1) for m in IDENT.finditer(before) if "/" not in m.group(1)]
            if not names and line.lstrip().startswith("|"):
                first = line.split("|")[1]
                names = [m.group(1) for m in IDENT.finditer(first) if "/" not in m.group(1)][:1]
            new = old
            path = repo_path(rel)
            if len(olds) > 1:
                # several lines: one symbol per line, from the row's first cell
                first = line.split("|")[1] if line.lstrip().startswith("|") else ""
                fnames = [m.group(1) for m in IDENT.finditer(first) if "/" not in m.group(1)]
                if len(fnames) == len(olds) and path.is_file():
                    news = []
                    for nm, o in zip(fnames, olds):
                        defs = definitions(path, nm)
                        news.append(min(defs, key=lambda d: abs(d - o)) if defs else o)
                    if news != olds:
                        moved += 1
                    pieces.append(line[last:mo.start()] + f"`{rel}:{','.join(map(str, news))}`")
                else:
                    kept.append(f"{rel}:{mo.group(2)} (several lines)")
                    pieces.append(line[last:mo.end()])
                last = mo.end()
                continue
            if names and path.is_file():
                defs = definitions(path, names[-1])
                if defs:
                    new = min(defs, key=lambda d: abs(d - old))
                else:
                    kept.append(f"{rel}:{old} ({names[-1]}: no definition)")
            else:
                kept.append(f"{rel}:{old} (no symbol)")
            if new != old:
                moved += 1
            pieces.append(line[last:mo.start()] + f"`{rel}:{new}`")
            last = mo.end()
        out_lines.append("".join(pieces) + line[last:])
    print(f"{moved} citations re-pinned; {len(kept)} left as they were")
    for k in kept:
        print("  ", k)
    if not a.dry_run:
        doc.write_text("".join(out_lines))


if __name__ == "__main__":
    main()
