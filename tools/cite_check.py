#!/usr/bin/env python3
"""Which tracked files under profiles/ no document cites (measurement hygiene).

A file counts as cited when a backticked token in DESIGN.md, README.md,
BASELINE.md, INTEGRATION.md or profiles/README.md names it: its path under
profiles/ (or the last parts of it), its base name, a directory above it
(`r01/fuzz/`, `prof_r03c/`), or a glob / brace pattern that matches it
(`kernel_stats_config*.csv`, `bench_config{9,10}_fill.json`).

usage: tools/cite_check.py            prints the uncited files, exit 1 if any
Used by tests/test_profiles_cited.py."""
import fnmatch
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "BASELINE.md", "INTEGRATION.md", "profiles/README.md"]


def _braces(tok):
    m = re.search(r"\{([^{}]*,[^{}]*)\}", tok)
    if not m:
        return [tok]
    out = []
    for alt in m.group(1).split(","):
        out += _braces(tok[:m.start()] + alt + tok[m.end():])
    return out


def tokens():
    toks = set()
    for d in DOCS:
        p = os.path.join(ROOT, d)
        if not os.path.exists(p):
            continue
        for t in re.findall(r"`([^`]+)`", open(p).read()):
            for part in t.split():
                part = part.strip(",;:()")
                if part.startswith("profiles/"):
                    part = part[len("profiles/"):]
                if part:
                    toks.update(_braces(part))
    return toks


def tracked():
    r = subprocess.run(["git", "-C", ROOT, "ls-files", "profiles"], capture_output=True, text=True, check=True)
    return [f[len("profiles/"):] for f in r.stdout.split() if f != "profiles/README.md"]


def cited(rel, toks):
    parts = rel.split("/")
    cands = {"/".join(parts[i:]) for i in range(len(parts))}  # r01/final5/x.csv, final5/x.csv, x.csv
    dirs = {"/".join(parts[i:j]) + "/" for j in range(1, len(parts)) for i in range(j)}
    for t in toks:
        if t.rstrip("/") + "/" in dirs:
            return True
        if any(fnmatch.fnmatchcase(c, t) for c in cands):
            return True
    return False


def uncited():
    toks = tokens()
    return [f for f in tracked() if not cited(f, toks)]


if __name__ == "__main__":
    u = uncited()
    print("\n".join(u))
    print(f"{len(u)} uncited of {len(tracked())} tracked files under profiles/", file=sys.stderr)
    sys.exit(1 if u else 0)
