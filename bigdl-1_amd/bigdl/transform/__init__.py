"""Data transforms (``DL/transform``)."""
