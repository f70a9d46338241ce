#!/usr/bin/env python3
"""Side-build patch (measurement only, tools/side_build.sh): k_seg's whole-line
in-place write-back with plain stores instead of non-temporal ones."""
import sys

p = sys.argv[1]
s = open(p).read()
a = "wr_r, (int)off, 0, 2);  // nt"
assert s.count(a) == 1
open(p, "w").write(s.replace(a, "wr_r, (int)off, 0, 0);  // plain (patched)"))
