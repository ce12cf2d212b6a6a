"""PCA top-3 on the reference's examples/data/pca_data.csv (PCAExample.scala counterpart).
Run: python examples/pca_example.py [path]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oap_mllib_amd as O  # noqa: E402
from oap_mllib_amd.utils import io  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/examples/data/pca_data.csv"
X = io.read_csv(path)
model = O.PCA(k=3, inputCol="features", outputCol="pcaFeatures").fit(X)
print("engine:", model.fit_info["engine"])
print("Principal components:\n", model.pc.toArray())
print("Explained variance:", model.explainedVariance.toArray())
print(model.transform(X)["pcaFeatures"].tolist())
