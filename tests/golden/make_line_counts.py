"""Write tests/golden/reference_line_counts.json: the line count of every Python file of the
reference (/root/reference, read-only), so that tests/test_citations.py can check every
`<file>.py:<line>` citation in this repository without the reference tree (it does not exist
on the GPU box).  Only file paths and line counts are stored -- no reference text.

Also tests/golden/reference_identifiers.json, for checking citations by content: per file, per line,
the 8-hex-digit SHA-1 prefixes of the identifiers on it that contain an underscore or a lower-upper
case change (`load_initial_values`, `SmartNanogridEnv`), and the line span of every class by the hash
of its name.  Hashes only: no reference text is stored.

Usage:  python tests/golden/make_line_counts.py
"""
import hashlib
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    counts = {}
    for root, dirs, files in os.walk(REF):
        dirs[:] = [d for d in dirs if not d.startswith(".")]
        for f in sorted(files):
            if f.endswith(".py"):
                path = os.path.join(root, f)
                with open(path, "rb") as fp:
                    counts[os.path.relpath(path, REF)] = len(fp.read().splitlines())
    with open(os.path.join(HERE, "reference_line_counts.json"), "w") as fp:
        json.dump(dict(sorted(counts.items())), fp, indent=1)
    idents = {}
    for rel in sorted(counts):
        with open(os.path.join(REF, rel), encoding="utf-8", errors="replace") as fp:
            lines = fp.read().splitlines()
        per_line = [sorted({ident_hash(t) for t in IDENT.findall(ln) if strong(t)}) for ln in lines]
        classes, cur = {}, None
        for i, ln in enumerate(lines, 1):
            m = re.match(r"class\s+(\w+)", ln)
            if m:
                if cur:
                    classes[ident_hash(cur[0])] = [cur[1], i - 1]
                cur = (m.group(1), i)
        if cur:
            classes[ident_hash(cur[0])] = [cur[1], len(lines)]
        idents[rel] = {"lines": per_line, "classes": classes}
    with open(os.path.join(HERE, "reference_identifiers.json"), "w") as fp:
        json.dump(idents, fp, separators=(",", ":"))
    print(f"{len(counts)} files")


IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")


def strong(tok):
    """An identifier that names something: contains an underscore or a lower-upper case change."""
    return "_" in tok.strip("_") or re.search(r"[a-z][A-Z]", tok) is not None


def ident_hash(tok):
    return hashlib.sha1(tok.encode()).hexdigest()[:8]


if __name__ == "__main__":
    main()
