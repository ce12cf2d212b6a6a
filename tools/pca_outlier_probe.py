"""Exact-mode PCA statistics with an outlier the row sample misses (scales redone) and a far one
(fp64 fallback): engine flags, bounds and errors against np.cov."""
import numpy as np, sys, os
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import oap_mllib_amd as O
from oap_mllib_amd import _loader
from oap_mllib_amd.models.clustering import upload_table
N = _loader.load()
w = O.init_world(O.get_config().replace(device="gpu", device_id=0))
rng = np.random.default_rng(19)
X = rng.normal(size=(200000, 24)).astype(np.float32)
for o in (0.5, 40.0, 1e4):
    X[1, 7] = o
    t = upload_table(w, X, layout="pca_exact")
    r = N.pca_covariance(w.ctx, w.comm, t, False, exact=True)
    Cr = np.cov(X.astype(np.float64).T, ddof=1)
    err = np.max(np.abs(np.asarray(r["cov"]) - Cr)) / np.max(np.abs(Cr))
    print(o, r["engine"], r["scales_redone"], r["fallback_fp64"], r["int8_rel_bound"],
          r["err_bound"], err, flush=True)
