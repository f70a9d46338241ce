"""Measurement hygiene: every tracked file under profiles/ is
cited by DESIGN.md, README.md, BASELINE.md, INTEGRATION.md or profiles/README.md
(tools/cite_check.py). Needs the git checkout; skipped without it."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_every_profile_file_is_cited():
    if not shutil.which("git") or not os.path.isdir(os.path.join(ROOT, ".git")):
        pytest.skip("no git checkout")
    if subprocess.run(["git", "-C", ROOT, "rev-parse"], capture_output=True).returncode:
        pytest.skip("not a git work tree")
    import cite_check
    assert cite_check.uncited() == []
