"""Sequence-file generators (``DL/models/utils/ImageNetSeqFileGenerator.scala``,
``COCOSeqFileGenerator.scala``): pack an image folder (one sub-folder per class, sorted → labels
1..N) into Hadoop SequenceFiles of BGR images (``BGRImgToLocalSeqFile`` format), optionally
resized, ``block_size`` images per file.

    python -m bigdl.models.utils.seqfile_generator -f /data/imagenet/train -o /data/seq/train -b 12800 [-r 256]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def image_records(folder: str, resize: int = 0, has_name: bool = True):
    from PIL import Image
    classes = sorted(d for d in os.listdir(folder) if os.path.isdir(os.path.join(folder, d)))
    for label, c in enumerate(classes, start=1):
        for fn in sorted(os.listdir(os.path.join(folder, c))):
            p = os.path.join(folder, c, fn)
            try:
                img = Image.open(p).convert("RGB")
            except OSError:
                continue
            if resize:
                w, h = img.size
                s = resize / min(w, h)
                img = img.resize((max(1, round(w * s)), max(1, round(h * s))), Image.BILINEAR)
            bgr = np.asarray(img)[..., ::-1].copy()
            yield (bgr, label, fn) if has_name else (bgr, label)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="seqfile_generator")
    ap.add_argument("-f", "--folder", required=True)
    ap.add_argument("-o", "--output", required=True)
    ap.add_argument("-b", "--blockSize", type=int, default=12800)
    ap.add_argument("-r", "--resize", type=int, default=0, help="shorter side after resizing (0 = keep)")
    ap.add_argument("--hasName", action="store_true")
    a = ap.parse_args(argv)
    from ...dataset.seqfile import BGRImgToLocalSeqFile
    os.makedirs(a.output, exist_ok=True)
    files = BGRImgToLocalSeqFile(a.blockSize, os.path.join(a.output, "imagenet"), a.hasName)(
        image_records(a.folder, a.resize, a.hasName))
    print(f"wrote {len(files)} sequence files to {a.output}")
    return 0


ImageNetSeqFileGenerator = main

if __name__ == "__main__":
    sys.exit(main())
