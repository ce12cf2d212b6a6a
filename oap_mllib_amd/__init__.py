"""oap_mllib_amd — an MI355X-native (gfx950) accelerator for Spark-MLlib K-Means, PCA and ALS.

Same estimator contract as ``org.apache.spark.ml`` (params, defaults, dispatch/fallback rules,
on-disk model format) as the reference OAP MLlib (bobjiang82/oap-mllib), with the oneDAL/oneCCL
JNI backend replaced by hand-written CDNA4 HIP kernels, a C++ runtime and RCCL over xGMI.
"""
from . import _loader  # imports torch first (single HIP runtime per process)
from .config import Config, get_config, set_config
from .linalg import DenseMatrix, DenseVector, Matrices, SparseVector, Vectors
from .models.clustering import KMeans, KMeansModel, KMeansSummary
from .models.feature import PCA, PCAModel
from .models.recommendation import ALS, ALSModel
from .parallel.world import get_world, init_world, shutdown_world

__version__ = "0.1.0"

_loader.require_on_gpu_hosts()

__all__ = ["Config", "get_config", "set_config", "DenseMatrix", "DenseVector", "Matrices",
           "SparseVector", "Vectors", "KMeans", "KMeansModel", "KMeansSummary", "PCA", "PCAModel",
           "ALS", "ALSModel", "get_world",
           "init_world", "shutdown_world", "__version__"]
