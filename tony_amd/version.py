"""Build/version information injected into every job's configuration as ``tony.version-info.*``
(T/util/VersionInfo.java:28-149 + gradle/version-info.gradle: version, revision, branch, user,
date, url, checksum).

``write_version_info()`` runs at build time (``__graft_entry__.build`` / ``python -m
tony_amd.version``) and records git metadata plus a checksum of the package sources in
``_version_info.json``; at run time ``version_info()`` reads that file, falling back to live
git queries and finally to "Unknown".
"""
from __future__ import annotations

import datetime
import getpass
import hashlib
import json
import os
import subprocess
from typing import Dict

from . import __version__

_HERE = os.path.dirname(os.path.abspath(__file__))
_INFO_FILE = os.path.join(_HERE, "_version_info.json")
KEYS = ("version", "revision", "branch", "user", "date", "url", "checksum")


def _git(*args: str) -> str:
    try:
        out = subprocess.run(["git", "-C", os.path.dirname(_HERE), *args], capture_output=True, text=True,
                             timeout=10)
        return out.stdout.strip() if out.returncode == 0 else ""
    except (OSError, subprocess.SubprocessError):
        return ""


def source_checksum() -> str:
    h = hashlib.md5()
    for root, dirs, files in sorted(os.walk(_HERE)):
        dirs.sort()
        if "__pycache__" in root:
            continue
        for f in sorted(files):
            if f.endswith((".py", ".hip", ".h", ".cpp", ".xml")):
                with open(os.path.join(root, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()


def compute_version_info() -> Dict[str, str]:
    try:
        user = getpass.getuser()
    except Exception:  # noqa: BLE001
        user = "Unknown"
    return {
        "version": __version__,
        "revision": _git("rev-parse", "HEAD") or "Unknown",
        "branch": _git("rev-parse", "--abbrev-ref", "HEAD") or "Unknown",
        "user": user,
        "date": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%MZ"),
        "url": _git("config", "--get", "remote.origin.url") or "file://" + os.path.dirname(_HERE),
        "checksum": source_checksum(),
    }


def write_version_info() -> Dict[str, str]:
    info = compute_version_info()
    with open(_INFO_FILE, "w") as f:
        json.dump(info, f, indent=1)
    return info


def version_info() -> Dict[str, str]:
    try:
        with open(_INFO_FILE) as f:
            info = json.load(f)
    except (OSError, ValueError):
        info = {}
    if not info:
        info = compute_version_info()
    return {k: str(info.get(k, "Unknown")) for k in KEYS}


def inject(conf) -> None:
    """Set every ``tony.version-info.<key>`` (VersionInfo.injectVersionInfo)."""
    from .conf import keys as K

    for k, v in version_info().items():
        conf.set(K.VERSION_INFO_PREFIX + k, v, "VersionInfo")


if __name__ == "__main__":
    print(json.dumps(write_version_info(), indent=1))
