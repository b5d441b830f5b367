"""Lint gate (the reference's only CI is ruff: ``.github/workflows/ruff.yml``).

ruff is not installable here, so ``tools/lint.py`` implements the checks this
codebase relies on (E501, W291, E711/E712, E722, F401, F403, F811, F841,
D100) and this test keeps the tree clean."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_lint_detects_problems(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import lint
    finally:
        sys.path.pop(0)
    bad = tmp_path / "bad.py"
    bad.write_text("import os\n\ndef f():\n    x = 1\n    try:\n        pass\n"
                   "    except:\n        pass\n    return None == 1\n")
    lint.ROOT = tmp_path
    codes = {line.split()[1] for line in lint.lint_file(bad)}
    assert {"F401", "F841", "E722", "E711"} <= codes
