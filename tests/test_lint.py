"""Repository lint (tools/lint.py: the mechanical subset of .clang-format / [tool.ruff]) and
packaging metadata (pyproject.toml + setup.py's native build hook)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_lint_clean():
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "lint.py")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout[-4000:]


def test_pyproject_metadata():
    import tomli

    meta = tomli.loads((ROOT / "pyproject.toml").read_text())
    assert meta["build-system"]["build-backend"] == "setuptools.build_meta"
    assert meta["project"]["name"] == "oap-mllib-amd"
    assert "*.so" in meta["tool"]["setuptools"]["package-data"]["oap_mllib_amd"]
    assert meta["tool"]["ruff"]["line-length"] == 100
    setup_py = (ROOT / "setup.py").read_text()
    assert "oap_mllib_amd.build import build" in setup_py and "build_py" in setup_py


def test_ci_workflow_runs_the_suites():
    wf = (ROOT / ".github" / "workflows" / "ci.yml").read_text()
    for needle in ("python -m oap_mllib_amd.build", '-m "not gpu"', "-m gpu", "tools/lint.py"):
        assert needle in wf, needle
