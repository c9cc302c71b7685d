"""MIOpen tuning database shipped with the repo.

``torch.backends.cudnn.benchmark = True`` makes MIOpen time every applicable
convolution solver per shape (find mode): on MI355X that picks kernels worth
+12 % on ResNet-50 training, but the search takes ~3.5 minutes. The results
(find-db ``*.ufdb.txt``: solver timings per problem; perf-db ``*.udb.txt``:
tuned solver parameters) are plain text written by our own runs on MI355X;
they live in ``tuning/miopen/`` and are installed as the process's MIOpen
user database, so find mode starts from the recorded choices (no search).
Problems not in the db are searched and appended as usual.
"""
from __future__ import annotations

import glob
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DB_DIR = os.path.join(ROOT, "tuning", "miopen")


def install_tuned_db(rank: int = 0, force: bool = False) -> str | None:
    """Point ``MIOPEN_USER_DB_PATH`` at a private writable copy of the shipped db.

    Must run before the first convolution (MIOpen reads the variable when its
    handle is created). Returns the directory, or ``None`` when the user
    already chose a db path or no db ships.
    """
    if os.environ.get("MIOPEN_USER_DB_PATH") and not force:
        return None
    files = glob.glob(os.path.join(DB_DIR, "*.txt"))
    if not files:
        return None
    dst = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"fluxmpi_miopen_{os.getuid()}", f"rank{rank}")
    os.makedirs(dst, exist_ok=True)
    for f in files:
        shutil.copy2(f, os.path.join(dst, os.path.basename(f)))
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst
