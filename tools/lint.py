#!/usr/bin/env python
"""Self-contained lint pass (the reference's ruff CI, ``.github/workflows/ruff.yml``).

``ruff`` is not installable in this image (no package index), so the
checks the reference's ``ruff.toml`` selects that matter for a codebase of
this shape are implemented here on the standard ``ast``/``tokenize``
modules. ``ruff.toml`` at the repository root carries the same selection for
machines that have ruff.

Checks (ruff codes):
  E501  line longer than 100 characters
  W291  trailing whitespace;  W191 tab indentation
  E711/E712  comparison to None / True / False with ``==``
  E722  bare ``except:``
  F401  module-level import never used (``__init__`` re-exports and names in
        ``__all__`` are exempt; ``# noqa`` on the line silences it)
  F403  ``from x import *``
  F811  a function / class redefined at module level
  F841  local variable assigned and never read (simple names only)
  D100  module without a docstring (package sources only)

Usage: ``python tools/lint.py [paths...]``; exits 1 when anything is found.
"""

from __future__ import annotations

import ast
import io
import sys
import tokenize
from pathlib import Path

MAX_LINE = 100
ROOT = Path(__file__).resolve().parents[1]
DEFAULT_PATHS = ["mpitree_amd", "mpitree", "tests", "bench", "tools", "bench.py",
                 "__graft_entry__.py"]


def _noqa(lines, lineno) -> bool:
    return 0 < lineno <= len(lines) and "noqa" in lines[lineno - 1]


class _Names(ast.NodeVisitor):
    def __init__(self):
        self.loads: set[str] = set()
        self.attr_roots: set[str] = set()

    def visit_Name(self, node):
        if isinstance(node.ctx, (ast.Load, ast.Del)):
            self.loads.add(node.id)

    def visit_Attribute(self, node):
        root = node
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.attr_roots.add(root.id)
        self.generic_visit(node)


def _string_names(tree) -> set[str]:
    """Names mentioned in string annotations / __all__ (count as used)."""
    out = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            for tok in node.value.replace("[", " ").replace("]", " ").replace(",", " ").split():
                out.add(tok.split(".")[0])
    return out


def _check_unused_locals(tree, lines, report):
    for fn in ast.walk(tree):
        if not isinstance(fn, (ast.FunctionDef, ast.AsyncFunctionDef)):
            continue
        stores, loads = {}, set()
        nonlocal_names = set()
        for node in ast.walk(fn):
            if isinstance(node, (ast.Global, ast.Nonlocal)):
                nonlocal_names.update(node.names)
            elif isinstance(node, ast.Name):
                if isinstance(node.ctx, ast.Store):
                    stores.setdefault(node.id, node.lineno)
                else:
                    loads.add(node.id)
            elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)) \
                    and node is not fn:
                for n in ast.walk(node):  # closures read enclosing locals
                    if isinstance(n, ast.Name):
                        loads.add(n.id)
        # only plain ``x = ...`` statements count (tuple unpacking / loop targets are exempt)
        plain = set()
        for node in ast.walk(fn):
            if isinstance(node, (ast.Assign, ast.AnnAssign, ast.AugAssign)):
                targets = node.targets if isinstance(node, ast.Assign) else [node.target]
                for t in targets:
                    if isinstance(t, ast.Name):
                        plain.add(t.id)
        for name, ln in stores.items():
            if (name in plain and name not in loads and name not in nonlocal_names
                    and not name.startswith("_") and not _noqa(lines, ln)):
                report(ln, "F841", f"local variable {name!r} is assigned to but never used")


def lint_file(path: Path) -> list[str]:
    src = path.read_text(encoding="utf-8")
    lines = src.splitlines()
    out: list[str] = []

    def report(ln, code, msg):
        out.append(f"{path.relative_to(ROOT)}:{ln}: {code} {msg}")

    for i, line in enumerate(lines, 1):
        if len(line) > MAX_LINE and not _noqa(lines, i) and "http" not in line:
            report(i, "E501", f"line too long ({len(line)} > {MAX_LINE})")
        if line.rstrip() != line:
            report(i, "W291", "trailing whitespace")
        if line.startswith("\t"):
            report(i, "W191", "indentation contains tabs")
    try:
        tree = ast.parse(src, filename=str(path))
    except SyntaxError as e:
        return out + [f"{path}:{e.lineno}: E999 {e.msg}"]
    if path.parts[-2:-1] and "mpitree_amd" in path.parts and ast.get_docstring(tree) is None \
            and path.name != "__init__.py":
        report(1, "D100", "missing module docstring")
    # comments: tokenize so '# noqa' inside strings does not count
    list(tokenize.generate_tokens(io.StringIO(src).readline))
    names = _Names()
    names.visit(tree)
    used = names.loads | names.attr_roots | _string_names(tree)
    is_init = path.name == "__init__.py"
    seen_defs: dict[str, int] = {}
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and any(a.name == "*" for a in node.names):
                report(node.lineno, "F403", f"'from {node.module} import *' used")
                continue
            if is_init or _noqa(lines, node.lineno) or (
                    isinstance(node, ast.ImportFrom) and node.module == "__future__"):
                continue
            for a in node.names:
                bound = (a.asname or a.name).split(".")[0]
                if bound not in used:
                    report(node.lineno, "F401", f"{a.name!r} imported but unused")
        elif isinstance(node, (ast.FunctionDef, ast.ClassDef, ast.AsyncFunctionDef)):
            if node.name in seen_defs and not node.decorator_list:
                report(node.lineno, "F811", f"redefinition of {node.name!r} from line "
                                            f"{seen_defs[node.name]}")
            seen_defs[node.name] = node.lineno
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            report(node.lineno, "E722", "do not use bare 'except'")
        if isinstance(node, ast.Compare):
            lhs = [node.left] + list(node.comparators[:-1])
            for op, a, b in zip(node.ops, lhs, node.comparators):
                for comp in (a, b):
                    if isinstance(op, (ast.Eq, ast.NotEq)) and isinstance(comp, ast.Constant) \
                            and (comp.value is None or comp.value is True
                                 or comp.value is False):
                        code = "E711" if comp.value is None else "E712"
                        report(node.lineno, code, f"comparison to {comp.value} with ==/!=")
    _check_unused_locals(tree, lines, report)
    return out


def iter_files(paths):
    for p in paths:
        p = (ROOT / p) if not Path(p).is_absolute() else Path(p)
        if p.is_file() and p.suffix == ".py":
            yield p
        elif p.is_dir():
            for f in sorted(p.rglob("*.py")):
                if "__pycache__" not in f.parts:
                    yield f


def main(argv=None) -> int:
    paths = (argv if argv else None) or DEFAULT_PATHS
    problems = []
    for f in iter_files(paths):
        problems += lint_file(f)
    for p in problems:
        print(p)
    return 1 if problems else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
