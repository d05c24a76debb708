from . import *  # noqa: F401,F403  (pyspark module path PY/dlframes/dl_classifier.py)
