"""Native build driver: compiles csrc/ (C++17 + HIP for gfx950) into ``oap_mllib_amd/_native*.so``.

The reference builds ``libMLlibDAL.so`` with a hand-written Makefile invoked from Maven
(mllib-dal/src/main/native/Makefile:15-73, pom.xml:349-368).  Here ``hipcc`` builds every
translation unit in parallel (incremental, header-dependency aware via ``-MMD``) and links one
pybind11 extension module in-tree, so the built ``.so`` travels with the repository snapshot to the
GPU box.  Usage::

    python -m oap_mllib_amd.build [--clean] [--jobs N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "oap_mllib_amd"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> Path:
    return PKG / ("_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def capi_path() -> Path:
    return PKG / "liboap_mllib.so"


def _includes() -> list[str]:
    import pybind11

    inc = [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    jh = os.environ.get("JAVA_HOME")
    if jh:  # JNI shim headers
        inc += [f"-I{jh}/include", f"-I{jh}/include/linux"]
    return inc


def _sources() -> list[Path]:
    srcs = []
    for p in sorted(CSRC.rglob("*")):
        if p.suffix not in (".cpp", ".hip"):
            continue
        if "jni" in p.parts and not os.environ.get("JAVA_HOME"):
            continue  # JNI shim only when a JDK is present
        srcs.append(p)
    return srcs


def _obj(src: Path) -> Path:
    rel = src.relative_to(CSRC)
    return BUILD / (str(rel).replace(os.sep, "__") + ".o")


def _stale(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    ot = obj.stat().st_mtime
    dep = obj.with_suffix(".d")
    if not dep.exists():
        return True
    text = dep.read_text().replace("\\\n", " ")
    parts = text.split(":", 1)[1].split() if ":" in text else []
    for p in parts:
        pp = Path(p)
        if not pp.exists() or pp.stat().st_mtime > ot:
            return True
    return False


def _common_flags(debug: bool) -> list[str]:
    opt = ["-O0", "-g"] if debug else ["-O3"]
    return opt + ["-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
                  "-Wno-unused-variable", "-Wno-unused-but-set-variable",
                  "-Wno-unused-result", "-Wno-unused-command-line-argument",
                  "-fvisibility=hidden"]


def _compile(src: Path, debug: bool) -> tuple[Path, str]:
    obj = _obj(src)
    cmd = [HIPCC] + _common_flags(debug) + _includes()
    if src.suffix == ".hip":
        cmd += ["-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    else:
        cmd += ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        if "linalg" in src.parts:  # host fp64 dense kernels: x86-64-v3 (both hosts have it)
            cmd += ["-mavx2", "-mfma", "-fopenmp-simd"]
    cmd += ["-MMD", "-MF", str(obj.with_suffix(".d")), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(jobs: int | None = None, clean: bool = False, debug: bool = False,
          verbose: bool = True) -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    todo = [s for s in srcs if _stale(s, _obj(s))]
    jobs = jobs or min(8, os.cpu_count() or 4)
    if todo:
        if verbose:
            print(f"[oap build] compiling {len(todo)}/{len(srcs)} units for {ARCH} (jobs={jobs})",
                  flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_compile, s, debug): s for s in todo}
            for f in cf.as_completed(futs):
                obj, warn = f.result()
                if verbose and warn.strip():
                    print(warn, file=sys.stderr)
    out = ext_path()
    objs = [_obj(s) for s in srcs]
    if todo or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + [str(o) for o in objs] + [
            "-o", str(out), "-lrccl", "-ldl", "-lpthread",
            "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[oap build] linked {out.relative_to(ROOT)}", flush=True)
    # liboap_mllib.so: the same native core without the Python bindings, exporting the C ABI
    # (csrc/capi/oap_capi.h) and, when a JDK was found, the JNI shim (csrc/jni/).
    lib = capi_path()
    cobjs = [o for o, s in zip(objs, srcs) if "bindings" not in s.relative_to(CSRC).parts]
    if todo or not lib.exists() or any(o.stat().st_mtime > lib.stat().st_mtime for o in cobjs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + [str(o) for o in cobjs] + [
            "-o", str(lib), "-lrccl", "-ldl", "-lpthread", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[oap build] linked {lib.relative_to(ROOT)}", flush=True)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(jobs=a.jobs, clean=a.clean, debug=a.debug)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
