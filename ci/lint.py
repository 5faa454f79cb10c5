"""Repository lint gate (the role of the reference's ``ci/lint_python.py`` + mypy/flake8 runs;
none of those tools are in this image, so the checks are implemented on the stdlib ``ast``):

* every Python file compiles;
* no unused imports (module-level and function-level; ``__init__`` re-exports, ``__all__``
  entries and ``# noqa`` lines exempt);
* no bare ``except:``; no mutable default arguments;
* package functions carry a return annotation (the mypy-strict surface of the reference's
  ``python/src``; tests and tools exempt);
* lines <= 125 characters (HIP: 130), no tabs, no trailing whitespace, files end with a newline;
* HIP sources: no CUDA / hipify compatibility layers (``__HIP_PLATFORM_*`` switches, cuda headers,
  ``__CUDA_ARCH__``) — gfx950 code only.

    python ci/lint.py [paths...]      # exit status 1 on any finding
"""
from __future__ import annotations

import ast
import os
import re
import sys
from typing import Iterator, List, Set, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "spark_rapids_ml_nai_amd"
PY_DIRS = [PKG, "tests", "tools", "ci"]
PY_FILES = ["bench.py", "__graft_entry__.py"]
HIP_DIR = os.path.join(PKG, "ops", "csrc")
MAX_LINE = 125
MAX_LINE_HIP = 130
_HIP_BANNED = [re.compile(p) for p in (r"__HIP_PLATFORM_(AMD|NVIDIA|HCC|NVCC)__", r"#\s*include\s*[<\"]cuda",
                                       r"__CUDA_ARCH__", r"hipify")]


def _py_files(paths: List[str]) -> Iterator[str]:
    for p in paths:
        full = os.path.join(ROOT, p)
        if os.path.isfile(full):
            yield full
            continue
        for d, dirs, files in os.walk(full):
            dirs[:] = [x for x in dirs if not x.startswith((".", "__pycache__")) and x not in ("lib", "fakespark")]
            for f in sorted(files):
                if f.endswith(".py"):
                    yield os.path.join(d, f)


class _Names(ast.NodeVisitor):
    def __init__(self) -> None:
        self.used: Set[str] = set()

    def visit_Name(self, node: ast.Name) -> None:
        self.used.add(node.id)

    def visit_Attribute(self, node: ast.Attribute) -> None:
        root = node
        while isinstance(root, ast.Attribute):
            root = root.value  # type: ignore[assignment]
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(node)


def _string_names(tree: ast.AST) -> Set[str]:
    """Names referenced from string annotations / __all__ (quoted forward references)."""
    out: Set[str] = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            out.update(re.findall(r"[A-Za-z_][A-Za-z0-9_]*", node.value))
    return out


def check_python(path: str) -> List[Tuple[int, str]]:
    rel = os.path.relpath(path, ROOT)
    src = open(path, encoding="utf-8").read()
    lines = src.split("\n")
    out: List[Tuple[int, str]] = []
    try:
        tree = ast.parse(src, filename=path)
    except SyntaxError as e:
        return [(e.lineno or 0, "syntax error: %s" % e.msg)]
    for i, ln in enumerate(lines, 1):
        if len(ln) > MAX_LINE:
            out.append((i, "line longer than %d characters (%d)" % (MAX_LINE, len(ln))))
        if "\t" in ln:
            out.append((i, "tab character"))
        if ln != ln.rstrip():
            out.append((i, "trailing whitespace"))
    if src and not src.endswith("\n"):
        out.append((len(lines), "no newline at end of file"))
    names = _Names()
    names.visit(tree)
    used = names.used | _string_names(tree)
    is_init = os.path.basename(path) == "__init__.py"
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)) and not is_init:
            if "noqa" in lines[node.lineno - 1]:
                continue
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for a in node.names:
                bound = (a.asname or a.name).split(".")[0]
                if bound != "*" and bound not in used:
                    out.append((node.lineno, "unused import %r" % bound))
        elif isinstance(node, ast.ExceptHandler) and node.type is None:
            out.append((node.lineno, "bare except"))
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for d in node.args.defaults + node.args.kw_defaults:
                if isinstance(d, (ast.List, ast.Dict, ast.Set)):
                    out.append((node.lineno, "mutable default argument in %s()" % node.name))
            if rel.startswith(PKG + os.sep) and node.returns is None and "noqa" not in lines[node.lineno - 1]:
                out.append((node.lineno, "missing return annotation on %s()" % node.name))
    return out


def check_hip() -> List[Tuple[str, int, str]]:
    out = []
    d = os.path.join(ROOT, HIP_DIR)
    for f in sorted(os.listdir(d)):
        if not f.endswith((".hip", ".h")):
            continue
        for i, ln in enumerate(open(os.path.join(d, f), encoding="utf-8"), 1):
            for pat in _HIP_BANNED:
                if pat.search(ln):
                    out.append((os.path.join(HIP_DIR, f), i, "compatibility-layer construct: %s" % pat.pattern))
            if len(ln.rstrip("\n")) > MAX_LINE_HIP:
                out.append((os.path.join(HIP_DIR, f), i, "line longer than %d characters" % MAX_LINE_HIP))
    return out


def main(argv: List[str]) -> int:
    paths = argv or PY_DIRS + PY_FILES
    findings = []
    for f in _py_files(paths):
        for ln, msg in check_python(f):
            findings.append((os.path.relpath(f, ROOT), ln, msg))
    if not argv:
        findings += check_hip()
    for f, ln, msg in findings:
        print("%s:%d: %s" % (f, ln, msg))
    print("lint: %d finding(s)" % len(findings))
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
