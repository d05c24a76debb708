"""Contributed interop (``pyspark/bigdl/contrib``): the ONNX model loader."""
