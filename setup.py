"""setuptools hook: ``pip install .`` / ``pip wheel .`` compile the native engine for gfx950 with
oap_mllib_amd/build.py (hipcc, in-tree) before the package files are collected, so the wheel
carries ``_native*.so`` and ``liboap_mllib.so``.  Metadata lives in pyproject.toml.

The reference packages its native library into the Maven assembly jar
(mllib-dal/pom.xml:349-442, src/assembly/assembly.xml:1-78); here the wheel is that artifact."""
import os
import sys

from setuptools import setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
        from oap_mllib_amd.build import build

        build(verbose=True)
        super().run()


class BinaryDistribution(Distribution):
    def has_ext_modules(self):  # platform wheel: it carries gfx950 code objects
        return True


def _legacy_metadata():
    """setuptools < 61 does not read pyproject.toml's [project] table: pass the same metadata."""
    import setuptools

    major = int(setuptools.__version__.split(".")[0])
    if major >= 61:
        return {}
    from setuptools import find_packages

    return dict(name="oap-mllib-amd", version="0.2.0", python_requires=">=3.9",
                install_requires=["numpy>=1.22"],
                packages=find_packages(include=["oap_mllib_amd", "oap_mllib_amd.*"]),
                package_data={"oap_mllib_amd": ["*.so"]},
                entry_points={"console_scripts": [
                    "oap-mllib-amd-build = oap_mllib_amd.build:main"]})


setup(cmdclass={"build_py": BuildNative}, distclass=BinaryDistribution, **_legacy_metadata())
