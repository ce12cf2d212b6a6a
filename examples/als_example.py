"""Implicit ALS on the reference's examples/data/onedal_als_csr_ratings.txt (ALSExample.scala
counterpart: rank 10, maxIter 5, regParam 0.01, alpha 40, 80/20 split, RMSE).
Run: python examples/als_example.py [path]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oap_mllib_amd as O  # noqa: E402
from oap_mllib_amd.utils import io  # noqa: E402

path = (sys.argv[1] if len(sys.argv) > 1
        else "/root/reference/examples/data/onedal_als_csr_ratings.txt")
r = io.read_ratings(path, "::")
rng = np.random.default_rng(0)
mask = rng.random(len(r["user"])) < 0.8
train = {k: v[mask] for k, v in r.items()}
test = {k: v[~mask] for k, v in r.items()}
als = O.ALS(rank=10, maxIter=5, regParam=0.01, alpha=40.0, implicitPrefs=True,
            coldStartStrategy="drop")
model = als.fit(train)
pred = model.transform(test)
rmse = float(np.sqrt(np.mean((pred["prediction"] - pred["rating"]) ** 2)))
print("engine:", model.fit_info["engine"], "RMSE =", rmse)
print(model.recommendForAllUsers(3).head())
