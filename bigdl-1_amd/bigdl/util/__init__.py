"""pyspark-compatible ``bigdl.util`` namespace (``pyspark/bigdl/util``)."""
