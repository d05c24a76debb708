__version__ = "0.10.0.hip1"
BIGDL_VERSION = "0.10.0-SNAPSHOT"  # reference version the API/format targets (RES/bigdl-version-info.properties:3)
