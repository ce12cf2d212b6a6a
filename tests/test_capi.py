"""The C ABI of liboap_mllib.so (csrc/capi) through ctypes: same results as the pybind11
bindings on the native CPU engine; errors come back as codes + messages, never as aborts."""
import numpy as np
import pytest

from oap_mllib_amd import capi
from oap_mllib_amd.fallback import als_vanilla
from oap_mllib_amd.fallback import kmeans_vanilla as vanilla


def blobs(n, d, k, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-10, 10, size=(k, d))
    return c[rng.integers(0, k, n)] + rng.normal(0, 0.5, size=(n, d)), c


def test_version_and_platform():
    L = capi.load()
    assert L.oap_capi_version() == 1
    assert L.oap_device_count() >= 0
    assert L.oap_check_platform(10_000) == 0  # no such device: not an error, just "no"


def test_kmeans_matches_bindings(native):
    X, c = blobs(5000, 7, 5, 1)
    init = c + 0.1
    with capi.Context(-1) as ctx:
        centers, cost, iters = ctx.kmeans_fit(X, init, max_iter=10, tol=0.0)
        lab, d2 = ctx.kmeans_predict(X, centers)
        kc = ctx.kmeans_init(X, 5, "k-means||", 2, 3)
    g = native.Context(-1)
    t = native.upload_dense(g, X, "f64", 7)
    r = native.kmeans_fit(g, native.LocalComm(False), t, init, 5, 10, 0.0)
    assert np.array_equal(centers, r["centers"]) and iters == r["num_iter"]
    assert cost == pytest.approx(r["cost"], rel=1e-12)
    ref_lab, ref_d = vanilla.find_closest(X, centers)
    assert np.array_equal(lab, ref_lab)
    np.testing.assert_allclose(d2, ref_d, rtol=1e-10)
    assert np.array_equal(kc, native.kmeans_init(g, native.LocalComm(False), t, 5, "k-means||",
                                                 2, 3))


def test_pca_matches_numpy():
    rng = np.random.default_rng(2)
    X = rng.normal(size=(2000, 6)) @ rng.normal(size=(6, 6))
    with capi.Context(-1) as ctx:
        pc, ev = ctx.pca_fit(X, 3)
    w, v = np.linalg.eigh(np.cov(X.T))
    order = np.argsort(w)[::-1]
    np.testing.assert_allclose(ev, w[order][:3] / w.sum(), rtol=1e-8)
    np.testing.assert_allclose(np.abs(pc), np.abs(v[:, order[:3]]), atol=1e-6)


def test_als_matches_oracle():
    rng = np.random.default_rng(4)
    u = rng.integers(0, 40, 900).astype(np.int32) * 3
    i = rng.integers(0, 30, 900).astype(np.int32) + 7
    r = rng.integers(1, 6, 900).astype(np.float32)
    with capi.Context(-1) as ctx:
        out = ctx.als_fit(u, i, r, rank=4, max_iter=3, reg=0.1, alpha=2.0, implicit=True, seed=5)
    ref = als_vanilla.fit(u, i, r, 4, 3, 0.1, True, 2.0, False, 5)
    assert np.array_equal(out["user_ids"], ref.user_ids)
    np.testing.assert_allclose(out["user_factors"], ref.user_factors,
                               atol=1e-4 * np.abs(ref.user_factors).max())


def test_errors_are_codes_not_aborts():
    with capi.Context(-1) as ctx:
        X = np.zeros((10, 3))
        with pytest.raises(capi.NativeError, match="k must be"):
            ctx.pca_fit(X, 7)
        with pytest.raises(capi.NativeError, match="unknown init mode"):
            ctx.kmeans_init(X, 2, "nope")
        with pytest.raises(capi.NativeError, match="GPU context"):
            ctx.join(b"\0" * capi.UNIQUE_ID_BYTES, 2, 0)
    L = capi.load()
    assert L.oap_ctx_create(99, 0.5, 0) is None  # no such device
    assert b"device" in L.oap_last_error()


@pytest.mark.gpu
def test_capi_gpu_kmeans_and_pca():
    X, c = blobs(20000, 16, 6, 3)
    with capi.Context(0) as ctx:
        assert capi.load().oap_check_platform(0) == 1
        centers, cost, iters = ctx.kmeans_fit(X, c + 0.05, max_iter=10, tol=0.0)
        pc, ev = ctx.pca_fit(X, 3)
    with capi.Context(-1) as cpu:
        ref, rcost, _ = cpu.kmeans_fit(X.astype(np.float32).astype(np.float64), c + 0.05,
                                       max_iter=10, tol=0.0)
    assert np.array_equal(centers, ref)
    assert cost == pytest.approx(rcost, rel=1e-5)
    w = np.linalg.eigvalsh(np.cov(X.T))[::-1]
    np.testing.assert_allclose(ev, w[:3] / w.sum(), rtol=1e-4)


def test_jni_shim_type_checks():
    """The JNI shim (csrc/jni, built only with a JDK) type-checks against a stub of the JNI C++
    API — no JVM here, so this is the compile guard for that file."""
    import shutil
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    r = subprocess.run([cxx, "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                        f"-I{root / 'tests/native/jni_stub'}", f"-I{root / 'csrc'}",
                        str(root / "csrc/jni/oap_jni.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


# The reference's JNI surface (mllib-dal/src/main/native/javah/*.h): symbol -> signature.
REFERENCE_JNI = {
    "Java_org_apache_spark_ml_clustering_KMeansDALImpl_cKMeansDALComputeWithInitCenters":
        "(JJIDIIILorg/apache/spark/ml/clustering/KMeansResult;)J",
    "Java_org_apache_spark_ml_feature_PCADALImpl_cPCATrainDAL":
        "(JIIILorg/apache/spark/ml/feature/PCAResult;)J",
    "Java_org_apache_spark_ml_recommendation_ALSDALImpl_cDALImplictALS":
        "(JJIIDDIIILorg/apache/spark/ml/recommendation/ALSResult;)J",
    "Java_org_apache_spark_ml_recommendation_ALSDALImpl_cShuffleData":
        "(Ljava/nio/ByteBuffer;IILorg/apache/spark/ml/recommendation/ALSPartitionInfo;)"
        "Ljava/nio/ByteBuffer;",
    "Java_org_apache_spark_ml_util_OneCCL_00024_c_1init":
        "(IILjava/lang/String;Lorg/apache/spark/ml/util/CCLParam;)I",
    "Java_org_apache_spark_ml_util_OneCCL_00024_c_1cleanup": "()V",
    "Java_org_apache_spark_ml_util_OneCCL_00024_isRoot": "()Z",
    "Java_org_apache_spark_ml_util_OneCCL_00024_rankID": "()I",
    "Java_org_apache_spark_ml_util_OneCCL_00024_setEnv": "(Ljava/lang/String;Ljava/lang/String;Z)I",
    "Java_org_apache_spark_ml_util_OneCCL_00024_c_1getAvailPort": "(Ljava/lang/String;)I",
    "Java_org_apache_spark_ml_util_OneDAL_00024_setNumericTableValue": "(JIID)V",
    "Java_org_apache_spark_ml_util_OneDAL_00024_cAddNumericTable": "(JJ)V",
    "Java_org_apache_spark_ml_util_OneDAL_00024_cSetDoubleBatch": "(JI[DII)V",
    "Java_org_apache_spark_ml_util_OneDAL_00024_cFreeDataMemory": "(J)V",
    "Java_org_apache_spark_ml_util_OneDAL_00024_cCheckPlatformCompatibility": "()Z",
    "Java_org_apache_spark_ml_util_OneDAL_00024_cNewCSRNumericTable": "([F[J[JJJ)J",
}

_JNI_TYPES = {"jint": "I", "jlong": "J", "jdouble": "D", "jboolean": "Z", "void": "V",
              "jstring": "Ljava/lang/String;", "jdoubleArray": "[D", "jfloatArray": "[F",
              "jlongArray": "[J"}


def _erase(sig: str) -> str:
    """JNI signature with every object type (other than String and arrays) as 'L'."""
    import re

    sig = sig.replace("Ljava/lang/String;", "S")
    return re.sub(r"L[^;]+;", "L", sig)


def test_jni_entry_points_match_reference_signatures():
    """Every reference entry point exists in the shim with the reference's parameter list (the
    C parameter types, erased to JNI type letters, equal the javah signature)."""
    import re
    from pathlib import Path

    src = (Path(__file__).resolve().parent.parent / "csrc/jni/oap_jni.cpp").read_text()
    for sym, sig in REFERENCE_JNI.items():
        m = re.search(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+" + sym + r"\s*\(([^)]*)\)", src)
        assert m, f"missing JNI entry point {sym}"
        ret, params = m.group(1), [p.strip() for p in m.group(2).split(",")]
        assert params[0].startswith("JNIEnv*") and params[1].startswith("jobject")
        letters = ""
        for p in params[2:]:
            t = re.sub(r"/\*.*?\*/", "", p).split()[0]
            letters += {"jobject": "L"}.get(t, _JNI_TYPES.get(t, "?")).replace(
                "Ljava/lang/String;", "S")
        want = _erase(sig)
        got = "(" + letters + ")" + {"jobject": "L"}.get(ret, _JNI_TYPES.get(ret, "?")).replace(
            "Ljava/lang/String;", "S")
        assert got == want, (sym, got, want)


def test_jni_shim_runs_against_recording_vm(tmp_path):
    """Compile the shim with a fake, type-checking JNIEnv (field names and Java types of the
    reference's result/param classes) and run every entry point on the CPU engine: K-Means on
    the reference example, PCA, the ratings shuffle + 1-based CSR + implicit ALS, CCL params."""
    import shutil
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    cxx = shutil.which("g++") or shutil.which("clang++")
    lib = root / "oap_mllib_amd" / "liboap_mllib.so"
    if cxx is None or not lib.exists():
        pytest.skip("needs a host C++ compiler and the built liboap_mllib.so")
    exe = tmp_path / "jni_harness"
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-Wall", "-Werror",
                        f"-I{root / 'tests/native/jni_stub'}", f"-I{root / 'csrc'}",
                        str(root / "tests/native/jni_harness.cpp"),
                        str(root / "csrc/jni/oap_jni.cpp"), f"-L{lib.parent}", "-loap_mllib",
                        f"-Wl,-rpath,{lib.parent}", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env={**__import__("os").environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0 and "JNI_HARNESS_OK" in r.stdout, r.stdout + r.stderr


def test_jni_c_init_kvs_two_process_world(tmp_path):
    """The reference's rendezvous contract end to end: two executor processes call
    c_init(2, rank, "127.0.0.1_<port>") (OneCCL.scala:32-46, OneCCL.cpp:47-86); rank 0 serves the
    store at that address, the host collectives run over it (CPU engine), and
    cKMeansDALComputeWithInitCenters returns the single-process centers on both ranks."""
    import shutil
    import socket
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    cxx = shutil.which("g++") or shutil.which("clang++")
    lib = root / "oap_mllib_amd" / "liboap_mllib.so"
    if cxx is None or not lib.exists():
        pytest.skip("needs a host C++ compiler and the built liboap_mllib.so")
    exe = tmp_path / "jni_harness"
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-Wall", "-Werror",
                        f"-I{root / 'tests/native/jni_stub'}", f"-I{root / 'csrc'}",
                        str(root / "tests/native/jni_harness.cpp"),
                        str(root / "csrc/jni/oap_jni.cpp"), f"-L{lib.parent}", "-loap_mllib",
                        f"-Wl,-rpath,{lib.parent}", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    with socket.socket() as s:  # a free port for rank 0's store
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([str(exe), "world2", str(port)], capture_output=True, text=True,
                       timeout=120, env={**__import__("os").environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0 and "JNI_WORLD2_OK" in r.stdout, r.stdout + r.stderr
