"""Keras model import (``pyspark/bigdl/keras``) — see :mod:`bigdl.keras.converter`."""
