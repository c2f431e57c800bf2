"""Filesystem helpers (the reference's HDFS/Hadoop-FS role, on local or NFS paths).

``IOUtils`` (``[common]/io/IOUtils.java:39-143``): recursive delete, glob listing, free port;
plus ``file:`` URI handling so configuration values like ``file:/tmp/Oryx/data/`` and
``hdfs:///...`` paths (mapped to a local root) work unchanged.
"""

from __future__ import annotations

import fnmatch
import glob
import gzip
import os
import shutil
import socket
import tempfile
from typing import List

__all__ = ["to_local_path", "to_uri", "delete_recursively", "list_files", "choose_free_port",
           "read_text", "write_text", "atomic_write_text", "mkdirs", "rename", "exists",
           "open_text_maybe_gz"]

_HDFS_ROOT = os.environ.get("ORYX_HDFS_ROOT", "/tmp/Oryx/hdfs")


def to_local_path(path: str) -> str:
    """Map ``file:`` and ``hdfs:`` URIs to local filesystem paths."""
    if path is None:
        return None
    p = str(path)
    if p.startswith("file://"):
        p = p[len("file://"):]
    elif p.startswith("file:"):
        p = p[len("file:"):]
    elif p.startswith("hdfs://"):
        rest = p[len("hdfs://"):]
        # hdfs://host:port/path or hdfs:///path
        slash = rest.find("/")
        rest = rest[slash:] if slash >= 0 else "/"
        p = _HDFS_ROOT + rest
    elif p.startswith("hdfs:"):
        p = _HDFS_ROOT + p[len("hdfs:"):]
    return p


def to_uri(path: str) -> str:
    p = os.path.abspath(to_local_path(path))
    return "file:" + p


def mkdirs(path: str) -> None:
    os.makedirs(to_local_path(path), exist_ok=True)


def exists(path: str) -> bool:
    return os.path.exists(to_local_path(path))


def rename(src: str, dst: str) -> None:
    os.replace(to_local_path(src), to_local_path(dst))


def delete_recursively(path: str) -> None:
    p = to_local_path(path)
    if p is None or not os.path.exists(p):
        return
    if os.path.isdir(p) and not os.path.islink(p):
        shutil.rmtree(p, ignore_errors=True)
    else:
        os.remove(p)


def list_files(directory: str, pattern: str = "*") -> List[str]:
    """Files under ``directory`` matching a glob (may contain ``/`` segments), sorted."""
    d = to_local_path(directory)
    if not os.path.isdir(d):
        return []
    return sorted(glob.glob(os.path.join(d, pattern)))


def choose_free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def open_text_maybe_gz(path: str, mode: str = "rt"):
    p = to_local_path(path)
    if p.endswith(".gz"):
        return gzip.open(p, mode, encoding="utf-8")
    return open(p, mode, encoding="utf-8")


def read_text(path: str) -> str:
    with open_text_maybe_gz(path, "rt") as f:
        return f.read()


def write_text(path: str, text: str) -> None:
    p = to_local_path(path)
    os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
    with open(p, "w", encoding="utf-8") as f:
        f.write(text)


def atomic_write_text(path: str, text: str) -> None:
    p = to_local_path(path)
    d = os.path.dirname(p) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp-")
    with os.fdopen(fd, "w", encoding="utf-8") as f:
        f.write(text)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, p)
