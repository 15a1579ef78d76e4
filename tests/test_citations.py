"""Every `<file>.py:<line>[-<line>]` citation of the reference in this repository must resolve: the
file exists in the reference and the cited lines exist in it.  Line counts come from
tests/golden/reference_line_counts.json (make_line_counts.py, from /root/reference); when the
reference tree itself is present, the cited lines are also checked to be inside it directly.
Continuations in the same line (`file.py:17, :72-73`, `charger.py:88/138`) are checked against the
same file.  Names of this repository's own Python files are not reference citations."""
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SOURCES = ["include", "smart-nanogrid-gym_amd/csrc", "smart-nanogrid-gym_amd/smart_nanogrid_gym", "oracle",
           "tests", "tools", "bench.py", "__graft_entry__.py", "DESIGN.md", "INTEGRATION.md", "README.md"]
EXTS = (".h", ".hip", ".cpp", ".c", ".py", ".md", ".sh")
CITE = re.compile(r"\b([A-Za-z_][A-Za-z0-9_]*\.py):(\d+)(?:-(\d+))?")
CONT = re.compile(r"^(?:\s*(?:,|/|and)\s*:?(\d+)(?:-(\d+))?(?![.\d]))")


def reference_counts():
    with open(os.path.join(ROOT, "tests", "golden", "reference_line_counts.json")) as fp:
        return json.load(fp)


def own_python_names():
    names = set()
    for root, dirs, files in os.walk(ROOT):
        dirs[:] = [d for d in dirs if not d.startswith(".") and d not in ("__pycache__", "gpurun_out")]
        names.update(f for f in files if f.endswith(".py"))
    return names


def source_files():
    for s in SOURCES:
        path = os.path.join(ROOT, s)
        if os.path.isfile(path):
            yield path
        for root, dirs, files in os.walk(path):
            dirs[:] = [d for d in dirs if d not in ("__pycache__", "_build", "golden")]
            for f in files:
                if f.endswith(EXTS):
                    yield os.path.join(root, f)


def citations():
    """(where, file name, first line, last line) for every citation and continuation."""
    out = []
    for path in source_files():
        if path.endswith("test_citations.py"):
            continue
        with open(path, encoding="utf-8", errors="replace") as fp:
            for ln, line in enumerate(fp, 1):
                for m in CITE.finditer(line):
                    name, lo, hi = m.group(1), int(m.group(2)), int(m.group(3) or m.group(2))
                    where = f"{os.path.relpath(path, ROOT)}:{ln}"
                    out.append((where, name, lo, hi))
                    rest = line[m.end():]
                    while True:
                        c = CONT.match(rest)
                        if not c:
                            break
                        out.append((where, name, int(c.group(1)), int(c.group(2) or c.group(1))))
                        rest = rest[c.end():]
    return out


def test_reference_citations_resolve():
    counts = reference_counts()
    by_name = {}
    for rel, n in counts.items():
        by_name.setdefault(os.path.basename(rel), []).append(n)
    own = own_python_names() - set(by_name)
    bad, checked = [], 0
    for where, name, lo, hi in citations():
        if name not in by_name:
            if name in own:
                continue   # this repository's own file
            bad.append(f"{where}: {name} is not a file of the reference")
            continue
        checked += 1
        if not (1 <= lo <= hi <= max(by_name[name])):
            bad.append(f"{where}: {name}:{lo}-{hi} is past the end ({max(by_name[name])} lines)")
    assert checked > 150, checked   # the sources do cite the reference
    assert not bad, "\n".join(bad)


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is only in the build container")
def test_line_counts_fixture_is_current():
    for rel, n in reference_counts().items():
        with open(os.path.join(REF, rel), "rb") as fp:
            assert len(fp.read().splitlines()) == n, rel
