"""K-Means on the reference's example data (examples/data/sample_kmeans_data.txt, LIBSVM),
the counterpart of the reference's examples/kmeans (KMeansExample.scala / kmeans-pyspark.py).
Run: python examples/kmeans_example.py [path]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oap_mllib_amd as O  # noqa: E402
from oap_mllib_amd.utils import io  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/examples/data/sample_kmeans_data.txt"
_, X = io.read_libsvm(path)
model = O.KMeans(k=2, seed=1).fit(X)
print("engine:", model.fit_info["engine"])
print("Cluster centers:", model.clusterCenters())
print("Training cost:", model.summary.trainingCost, "iterations:", model.summary.numIter)
