"""Resource localization: ``SOURCE[::ALIAS][#archive]`` specs (T/LocalizableResource.java:30-114).

TonY ships each resource through HDFS and lets the NodeManager localize it into
the container's working directory.  On one MI355X node the job's staging dir
plays HDFS's role and each task's working directory is populated directly:
plain files are hard-linked (or copied across filesystems) under their alias,
``#archive`` resources are unpacked into a directory named by the alias, and a
directory source expands to its first-level files (Utils.java:562-584).
"""
from __future__ import annotations

import os
import shutil
from dataclasses import dataclass
from typing import List

from .. import constants as C
from .core import unzip_archive


class ResourceParseError(ValueError):
    pass


@dataclass
class LocalizableResource:
    spec: str
    source: str
    localized_name: str
    is_archive: bool
    is_directory: bool

    @classmethod
    def parse(cls, spec: str) -> "LocalizableResource":
        path = spec
        archive = False
        if spec.lower().endswith(C.ARCHIVE_SUFFIX):
            archive = True
            path = spec[: -len(C.ARCHIVE_SUFFIX)]
        parts = path.split(C.RESOURCE_DIVIDER)
        if len(parts) > 2:
            raise ResourceParseError(f"Failed to parse file: {spec}")
        src = parts[0]
        if src.startswith("file://"):
            src = src[len("file://"):]
        if "://" in src:
            raise ResourceParseError(f"remote resource {src!r}: only local paths exist on a single node")
        if not os.path.exists(src):
            raise FileNotFoundError(src)
        name = parts[1] if len(parts) == 2 else os.path.basename(src.rstrip("/"))
        return cls(spec, os.path.abspath(src), name, archive, os.path.isdir(src))

    def is_local_file(self) -> bool:
        return True

    def expand(self) -> List["LocalizableResource"]:
        """A directory resource stands for its first-level files."""
        if not self.is_directory:
            return [self]
        out = []
        for fn in sorted(os.listdir(self.source)):
            full = os.path.join(self.source, fn)
            if os.path.isfile(full):
                out.append(LocalizableResource(full, full, fn, False, False))
        return out

    def localize(self, workdir: str) -> str:
        """Materialise this resource inside ``workdir``; returns the localized path."""
        if self.is_directory:
            raise ResourceParseError("directory resources must be expanded first")
        dst = os.path.join(workdir, self.localized_name)
        if os.path.lexists(dst):
            if os.path.isdir(dst) and not os.path.islink(dst):
                shutil.rmtree(dst)
            else:
                os.unlink(dst)
        if self.is_archive:
            if not unzip_archive(self.source, dst):
                raise ResourceParseError(f"cannot unpack archive {self.source}")
            return dst
        try:
            os.link(self.source, dst)
        except OSError:
            shutil.copy2(self.source, dst)
        return dst


def localize_all(specs: List[str], workdir: str) -> List[str]:
    out = []
    for spec in specs:
        spec = spec.strip()
        if not spec:
            continue
        for r in LocalizableResource.parse(spec).expand():
            out.append(r.localize(workdir))
    return out
