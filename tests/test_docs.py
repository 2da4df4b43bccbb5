"""docs/PARITY.md stays in sync with the tree: every ``path:line`` it cites for this
framework exists and the cited line is not blank (SURVEY.md §2 parity map)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "kafka_inferenceengine_amd"
CITE = re.compile(r"`((?:csrc|engine|inference|input_output|models|ops|parallel|utils)/[\w./]+):([\d,\-]+)")


def _resolve(rel: str) -> Path:
    return ROOT / rel if rel.startswith("csrc/") else PKG / rel


def test_parity_citations_resolve():
    text = (ROOT / "docs" / "PARITY.md").read_text()
    cites = CITE.findall(text)
    assert len(cites) > 60
    for rel, lines in cites:
        path = _resolve(rel)
        assert path.is_file(), rel
        src = path.read_text().splitlines()
        for part in lines.split(","):
            first, _, last = part.partition("-")
            for n in {int(first), int(last or first)}:
                assert 1 <= n <= len(src), f"{rel}:{n} past end ({len(src)} lines)"
                assert src[n - 1].strip(), f"{rel}:{n} is blank"
