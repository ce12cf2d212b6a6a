"""RDD-style ``org.apache.spark.mllib`` API (the reference's S2 shadow class)."""
