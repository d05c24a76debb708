"""``bigdl.dataset.base`` (``PY/dataset/base.py``): ``maybe_download`` and ``display_table``.

There is no network here: ``maybe_download`` returns the local file when it is present (in
``work_directory``, plain or with its ``.gz`` counterpart) and otherwise raises with the URL the
reference would have fetched, so the user can place the file manually.
"""
from __future__ import annotations

import os


def maybe_download(filename: str, work_directory: str, source_url: str = "") -> str:
    os.makedirs(work_directory, exist_ok=True)
    path = os.path.join(work_directory, filename)
    for cand in (path, path[:-3] if path.endswith(".gz") else path + ".gz"):
        if os.path.exists(cand):
            return cand
    raise FileNotFoundError(f"{path} not found and downloads are disabled; fetch {source_url or filename} "
                            f"into {work_directory}")


def display_table(rows, positions):
    """Print rows as fixed-width columns ending at ``positions``."""
    def fmt(row):
        line = ""
        for i, cell in enumerate(row):
            line += str(cell)
            line = line[:positions[i]]
            line += " " * (positions[i] - len(line))
        return line
    for r in rows:
        print(fmt(r))
