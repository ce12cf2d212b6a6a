"""Mechanical lint for the repository (the subset of .clang-format / [tool.ruff] that needs no
external tool, so it runs in CI and in tests/test_lint.py on a bare image):

* every source file: UTF-8, LF line ends, no tabs, no trailing whitespace, final newline,
  at most 100 columns;
* Python: compiles;
* native code (csrc/): MI355X-only — no CUDA headers or macros, no dual-platform guards.

    python tools/lint.py [paths...]      (exit 1 and one line per finding on violations)"""
from __future__ import annotations

import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
DIRS = ["oap_mllib_amd", "csrc", "tests", "tools", "benchmarks", "examples"]
TOP = ["bench.py", "__graft_entry__.py", "setup.py"]
SUFFIXES = {".py", ".cpp", ".h", ".hip", ".sh"}
MAX_COLS = 100
SKIP_PARTS = {"__pycache__", "jni_stub"}  # jni_stub mirrors the JDK's header layout
FORBIDDEN_NATIVE = [
    (re.compile(r"#\s*include\s*<cuda"), "CUDA header"),
    (re.compile(r"__CUDA_ARCH__|__NVCC__"), "CUDA macro"),
    (re.compile(r"__HIP_PLATFORM_(AMD|NVIDIA|NVCC|HCC)__"), "dual-platform guard"),
]


def files(paths: list[str]) -> list[Path]:
    if paths:
        out = []
        for p in paths:
            q = Path(p)
            out += [f for f in q.rglob("*") if f.suffix in SUFFIXES] if q.is_dir() else [q]
        return out
    out = [ROOT / t for t in TOP if (ROOT / t).exists()]
    for d in DIRS:
        out += [f for f in sorted((ROOT / d).rglob("*")) if f.suffix in SUFFIXES and f.is_file()]
    return [f for f in out if not SKIP_PARTS.intersection(f.parts)]


def check(f: Path) -> list[str]:
    errs = []
    raw = f.read_bytes()
    try:
        text = raw.decode("utf-8")
    except UnicodeDecodeError:
        return [f"{f}: not UTF-8"]
    if b"\r\n" in raw:
        errs.append(f"{f}: CRLF line ends")
    if raw and not raw.endswith(b"\n"):
        errs.append(f"{f}: no final newline")
    for i, line in enumerate(text.split("\n"), 1):
        if "\t" in line:
            errs.append(f"{f}:{i}: tab")
        if line != line.rstrip():
            errs.append(f"{f}:{i}: trailing whitespace")
        if len(line) > MAX_COLS and f.suffix != ".sh":  # (shell: long command lines)
            errs.append(f"{f}:{i}: {len(line)} columns (max {MAX_COLS})")
    if f.suffix == ".py":
        try:
            compile(text, str(f), "exec")
        except SyntaxError as e:
            errs.append(f"{f}:{e.lineno}: syntax error: {e.msg}")
    if f.suffix in (".cpp", ".h", ".hip") and "csrc" in f.parts:
        for i, line in enumerate(text.split("\n"), 1):
            for pat, what in FORBIDDEN_NATIVE:
                if pat.search(line):
                    errs.append(f"{f}:{i}: {what}")
    return errs


def main(argv: list[str]) -> int:
    errs = []
    fs = files(argv)
    for f in fs:
        errs += check(f)
    for e in errs:
        print(e)
    print(f"lint: {len(fs)} files, {len(errs)} findings", file=sys.stderr)
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
