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


def test_native_knobs_have_one_home():
    """SURVEY §5 "Config": the native layer reads the environment in one place only
    (runtime/knobs.cpp), and every OAP_* name the C++/HIP sources mention is a documented entry
    of its knob table."""
    import re

    srcs = [p for p in (ROOT / "csrc").rglob("*") if p.suffix in (".cpp", ".hip", ".h")]
    getenv = [str(p.relative_to(ROOT)) for p in srcs if "getenv(" in p.read_text()]
    assert getenv == ["csrc/runtime/knobs.cpp"], getenv
    table = (ROOT / "csrc/runtime/knobs.cpp").read_text()
    listed = set(re.findall(r'\{"(OAP_[A-Z0-9_]+)"', table))
    used = set()
    for p in srcs:
        if p.name == "knobs.cpp":
            continue
        used |= set(re.findall(r'knob_(?:str|int|float|on)\("(OAP_[A-Z0-9_]+)"\)', p.read_text()))
    assert used and used <= listed, sorted(used - listed)


def test_native_knob_registry_and_config():
    import pytest

    from oap_mllib_amd import _loader
    from oap_mllib_amd.config import resolve

    N = _loader.load()
    names = {k["name"] for k in N.knob_table()}
    assert "OAP_KMEANS_ROW_SCAN" in names and all(k["doc"] for k in N.knob_table())
    assert N.knob_value("OAP_KMEANS_REFINE") == "1"
    N.set_knob("OAP_KMEANS_REFINE", "0")
    assert N.knob_value("OAP_KMEANS_REFINE") == "0"
    N.set_knob("OAP_KMEANS_REFINE", "")
    assert N.knob_value("OAP_KMEANS_REFINE") == "1"
    with pytest.raises(Exception):
        N.set_knob("OAP_NOT_A_KNOB", "1")
    cfg = resolve(environ={"OAP_MLLIB_NATIVE_KNOBS": "OAP_KMEANS_ROW_SCAN=0, OAP_EIG_GRID=64"})
    assert cfg.native_knobs == {"OAP_KMEANS_ROW_SCAN": "0", "OAP_EIG_GRID": "64"}
    cfg = resolve(spark_conf={"spark.oap.mllib.native_knobs": "OAP_ALS_LOWRANK=0"})
    assert cfg.native_knobs == {"OAP_ALS_LOWRANK": "0"}
    import oap_mllib_amd as O

    O.shutdown_world()
    w = O.init_world(O.get_config().replace(device="cpu",
                                            native_knobs={"OAP_EIG_GRID": "32"}))
    assert N.knob_value("OAP_EIG_GRID") == "32"
    O.shutdown_world()
    O.init_world(O.get_config().replace(device="cpu"))
    assert N.knob_value("OAP_EIG_GRID") == "0"
    O.shutdown_world()
    del w
