"""TensorFlow interop examples (``DL/example/tensorflow``): ``loadandsave`` and ``transferlearning``."""
