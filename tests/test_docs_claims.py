"""Every performance figure in README.md and docs/ names its record (VERDICT r4 "next round" #5).

A figure is a number with the unit us / µs (per step, per kernel, per phase) or samples/s.  Per
block -- a paragraph, or a table together with the paragraph just before it -- each figure must be

* in a block that names a driver record (``BENCH_r0N.json`` / ``GPUTEST_r0N.json`` /
  ``SCALE_r0N.json``) that exists at the repository root, or
* found in a ``profiles/`` file the block names (the number itself, or the same time in ms / s,
  or the same throughput as ms per 64-sample step), or
* in a block marked ``(derived)``: a bound or a sum computed in the text from cited figures.
"""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
DOCS = [ROOT / "README.md"] + sorted((ROOT / "docs").glob("*.md"))
_NUM = r"\d{1,3}(?:[ ,]\d{3})+(?:\.\d+)?|\d+(?:\.\d+)?"
_FIG = re.compile(rf"({_NUM})(?:\s*(?:-|–|to)\s*({_NUM}))?\s*(M\s+)?(µs|us\b|samples/s)")
_REC = re.compile(r"\b(BENCH|GPUTEST|SCALE)_r\d\d\.json")
_PROF = re.compile(r"(?:profiles/)?([\w.\-]+(?:/[\w.\-]+)*\.(?:md|txt|json|jsonl))")


def _blocks(text: str):
    lines = text.splitlines()
    blocks, cur, prev_para = [], [], []
    for ln in lines + [""]:
        if ln.strip():
            cur.append(ln)
            continue
        if cur:
            is_table = all(x.lstrip().startswith("|") for x in cur)
            blocks.append("\n".join((prev_para if is_table else []) + cur))
            prev_para = [] if is_table else cur
            cur = []
    return blocks


def _val(s: str) -> float:
    return float(s.replace(",", "").replace(" ", ""))


def _file_numbers(path: Path):
    # magnitudes: a record's "-48.7" (a delta) backs a text's "48.7 µs"
    return [abs(float(x)) for x in re.findall(r"-?\d+(?:\.\d+)?(?:e-?\d+)?", path.read_text(errors="ignore"))]


def _backed(x: float, unit: str, mega: bool, nums) -> bool:
    tol = lambda a, b: abs(a - b) <= 0.006 * abs(b) + 1e-9  # noqa: E731
    if unit == "samples/s":
        x = x * 1e6 if mega else x
        return any(tol(y, x) or (y > 0 and tol(64e3 / y, x)) or (y > 0 and tol(64e6 / y, x)) for y in nums)
    return any(tol(y, x) or tol(y * 1e3, x) or tol(y * 1e6, x) for y in nums)


def _profile_files(block: str):
    out = []
    for m in _PROF.finditer(block):
        name = m.group(1)
        for cand in (ROOT / "profiles" / name, ROOT / name):
            if cand.is_file() and "profiles" in cand.parts:
                out.append(cand)
                break
        else:  # a bare file name cited after a profiles/ path in the same block
            hits = list((ROOT / "profiles").rglob(Path(name).name))
            out.extend(h for h in hits if h.is_file())
    return out


def unbacked_figures():
    bad = []
    for doc in DOCS:
        for block in _blocks(doc.read_text()):
            figs = list(_FIG.finditer(block))
            if not figs:
                continue
            if "(derived)" in block:
                continue
            recs = [m.group(0) for m in _REC.finditer(block)]
            if any((ROOT / r).is_file() for r in recs):
                continue
            nums = [n for f in _profile_files(block) for n in _file_numbers(f)]
            for f in figs:
                vals = [_val(f.group(1))] + ([_val(f.group(2))] if f.group(2) else [])
                if not all(_backed(v, f.group(4), bool(f.group(3)), nums) for v in vals):
                    bad.append(f"{doc.relative_to(ROOT)}: '{f.group(0)}' in: {block.splitlines()[0][:90]}")
    return bad


def test_every_performance_figure_names_its_record():
    bad = unbacked_figures()
    assert not bad, f"{len(bad)} unbacked figures:\n" + "\n".join(bad[:60])


def test_checker_catches_an_unbacked_figure():
    assert _FIG.search("the step takes 37.5 µs on this box")
    assert not _backed(37.5, "µs", False, [38.0, 0.0391])
    assert _backed(37.5, "µs", False, [0.0375])
    assert _backed(1.62, "samples/s", True, [0.03951])  # 64 samples / 39.51 us


def _status_section(text: str) -> str:
    i = text.index("## Status and limits")
    j = text.find("\n## ", i + 1)
    return text[i:] if j < 0 else text[i:j]


def _bench_us(rec: Path) -> float:
    import json
    d = json.loads(rec.read_text())
    line = d.get("parsed") or d
    return float(line["ms_per_step"]) * 1e3


def test_status_headline_is_a_driver_record():
    """README's status section opens with the driver's record -- its first µs
    figure sits in a bullet naming a ``BENCH_r0N.json`` that exists, and equals that record's
    ms_per_step -- and the latest BENCH record is the one quoted (builder-box ranges are context)."""
    status = _status_section((ROOT / "README.md").read_text())
    m = next(f for f in _FIG.finditer(status) if f.group(4) in ("µs", "us"))
    bullet_start = status.rfind("\n* ", 0, m.start())
    bullet_end = status.find("\n* ", m.end())
    bullet = status[bullet_start: bullet_end if bullet_end > 0 else len(status)]
    recs = [r.group(0) for r in _REC.finditer(bullet) if r.group(0).startswith("BENCH")]
    assert recs, f"first µs figure '{m.group(0)}' cites no BENCH record: {bullet[:200]}"
    rec = ROOT / recs[0]
    assert rec.is_file(), rec
    latest = sorted(ROOT.glob("BENCH_r[0-9][0-9].json"))[-1]
    assert rec.name == latest.name, (rec.name, latest.name)
    assert abs(_val(m.group(1)) - _bench_us(rec)) <= 0.006 * _bench_us(rec), (m.group(0), _bench_us(rec))


def test_perf_model_headline_is_a_driver_record():
    text = (ROOT / "docs" / "perf_model.md").read_text()
    first = next(b for b in _blocks(text) if _FIG.search(b))
    latest = sorted(ROOT.glob("BENCH_r[0-9][0-9].json"))[-1]
    assert latest.name in first, first[:300]
    m = next(f for f in _FIG.finditer(first) if f.group(4) in ("µs", "us"))
    assert abs(_val(m.group(1)) - _bench_us(latest)) <= 0.006 * _bench_us(latest), m.group(0)
