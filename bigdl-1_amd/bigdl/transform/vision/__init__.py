"""Vision transforms (``DL/transform/vision``)."""
