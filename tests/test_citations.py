"""Every `<file>.py:<line>[-<line>]` citation of the reference in this repository must resolve: the
file exists in the reference and the cited lines exist in it.  Line counts come from
tests/golden/reference_line_counts.json (make_line_counts.py, from /root/reference); when the
reference tree itself is present, the cited lines are also checked to be inside it directly.
Continuations in the same line (`file.py:17, :72-73`, `charger.py:88/138`) are checked against the
same file.  Names of this repository's own Python files are not reference citations.

By content (tests/golden/reference_identifiers.json: hashed identifiers per reference line, no text):
when the citing line names identifiers of the cited file (`load_initial_values`, `SmartNanogridEnv`:
an underscore or a lower-upper case change; file/module names and the class a cited range lies in do
not count), one of them must be on the cited lines (within 3 lines before / 1 after, for a citation of
the statement a definition starts).  The citations that describe behaviour on lines the named
identifier is not on are listed with the reason in CONTENT_EXCEPTIONS."""
import hashlib
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


IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")

# (citing file, cited file, first line): why the identifier named beside the citation is not on the lines
CONTENT_EXCEPTIONS = {
    ("include/sng.h", "charging_station.py", 50): "the penalty-mode switch reads the ctor's vehicle_uncharged_penalty_mode "
                                                  "through self.UNCHARGED_PENALTY_MODE",
    ("smart-nanogrid-gym_amd/csrc/sng_api.cpp", "pv_system_manager.py", 17):
        "PVSystem(...)'s parameters at :17 give scaling_pv (the local of :68)",
    ("smart-nanogrid-gym_amd/csrc/sng_api.cpp", "charging_station.py", 200):
        "the generator body; clear_initialisation_variables is cited separately (:138-150)",
    ("smart-nanogrid-gym_amd/csrc/sng_kernels.hip", "charging_station.py", 230):
        "the requested-SoC default 1.0 of the generator; the Requested_SOC key is the dict's",
    ("smart-nanogrid-gym_amd/smart_nanogrid_gym/vec_env.py", "charging_station.py", 164):
        "the dict literal generated_initial_values(_json): the initial_values file it is written to",
    ("smart-nanogrid-gym_amd/smart_nanogrid_gym/vec_env.py", "charging_station.py", 119):
        "load_initial_values does not restore Requested_SOC: the cited lines are where it is missing",
    ("oracle/sng_oracle.c", "pv_system_manager.py", 34): "the window means that build solar_irradiance_2 (:19)",
    ("DESIGN.md", "central_management_system.py", 158): "the negative-demand ValueError; charging_mode is a "
                                                        "separate item of the same table row",
    ("INTEGRATION.md", "evaluator.py", 13): "the evaluator loop drives a SmartNanogridEnv built elsewhere",
    ("INTEGRATION.md", "predictor.py", 14): "the predictor loop drives a SmartNanogridEnv built elsewhere",
    ("INTEGRATION.md", "charging_station.py", 119): "load_initial_values: what generate_new_initial_values=False "
                                                    "reaches; Requested_SOC is what it leaves cleared",
}


def ident_hash(tok):
    return hashlib.sha1(tok.encode()).hexdigest()[:8]


def strong(tok):
    return "_" in tok.strip("_") or re.search(r"[a-z][A-Z]", tok) is not None


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


def citing_lines():
    """(path, line number, text, citation match) for every citation of a reference file."""
    for path in source_files():
        if path.endswith("test_citations.py"):
            continue
        with open(path, encoding="utf-8", errors="replace") as fp:
            for ln, line in enumerate(fp, 1):
                for m in CITE.finditer(line):
                    yield path, ln, line, m


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


def test_reference_citations_hold_their_identifiers():
    with open(os.path.join(ROOT, "tests", "golden", "reference_identifiers.json")) as fp:
        idents = json.load(fp)
    by_name = {}
    for rel in idents:
        by_name.setdefault(os.path.basename(rel), []).append(rel)
    modules = {ident_hash(os.path.basename(rel)[:-3]) for rel in idents}
    bad, checked, used = [], 0, set()
    for path, ln, line, m in citing_lines():
        name, lo, hi = m.group(1), int(m.group(2)), int(m.group(3) or m.group(2))
        if name not in by_name:
            continue
        rels = by_name[name]
        cand = set()
        for tok in {t for t in IDENT.findall(line) if strong(t)}:
            h = ident_hash(tok)
            if h in modules:
                continue
            for rel in rels:
                span = idents[rel]["classes"].get(h)
                if span and span[0] <= lo and hi <= span[1]:
                    continue   # a citation inside the class it names
                if any(h in ids for ids in idents[rel]["lines"]):
                    cand.add(h)
        if not cand:
            continue
        checked += 1
        hit = any(cand & set(idents[rel]["lines"][i]) for rel in rels
                  for i in range(max(0, lo - 4), min(len(idents[rel]["lines"]), hi + 1)))
        key = (os.path.relpath(path, ROOT), name, lo)
        if key in CONTENT_EXCEPTIONS:
            used.add(key)
            continue
        if not hit:
            bad.append(f"{key[0]}:{ln}: {name}:{lo}-{hi} holds none of the identifiers named beside it")
    assert checked >= 80, checked   # the sources do name what they cite
    assert not bad, "\n".join(bad)
    assert used == set(CONTENT_EXCEPTIONS), sorted(set(CONTENT_EXCEPTIONS) - used)   # no stale exceptions


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is only in the build container")
def test_identifiers_fixture_is_current():
    with open(os.path.join(ROOT, "tests", "golden", "reference_identifiers.json")) as fp:
        idents = json.load(fp)
    for rel, d in idents.items():
        with open(os.path.join(REF, rel), encoding="utf-8", errors="replace") as fp:
            lines = fp.read().splitlines()
        assert [sorted({ident_hash(t) for t in IDENT.findall(ln) if strong(t)}) for ln in lines] == d["lines"], rel
