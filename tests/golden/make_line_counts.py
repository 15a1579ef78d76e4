"""Write tests/golden/reference_line_counts.json: the line count of every Python file of the
reference (/root/reference, read-only), so that tests/test_citations.py can check every
`<file>.py:<line>` citation in this repository without the reference tree (it does not exist
on the GPU box).  Only file paths and line counts are stored -- no reference text.

Usage:  python tests/golden/make_line_counts.py
"""
import json
import os

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
    print(f"{len(counts)} files")


if __name__ == "__main__":
    main()
