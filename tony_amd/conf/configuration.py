"""Hadoop-``Configuration``-compatible XML config (the ``tony.xml`` / ``tony-site.xml`` format).

Semantics kept from Hadoop (TonY's layering depends on them):

* resources are applied in the order added; a later resource overrides an
  earlier one unless the earlier property was marked ``<final>true</final>``;
* values ``set()`` programmatically (``--conf k=v``) override every resource,
  whenever that resource is added;
* ``${name}`` references are expanded on read (other properties, then the
  environment as ``${env.NAME}``), up to a fixed depth;
* each value remembers its source (written to ``tony-final.xml``).
"""
from __future__ import annotations

import io
import os
import re
import threading
import xml.etree.ElementTree as ET
from typing import Dict, Iterator, List, Optional, Tuple

_VAR = re.compile(r"\$\{([^}$\s]+)\}")
_MAX_SUBST = 20

DEFAULT_XML = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tony-default.xml")


class ConfigurationError(ValueError):
    pass


def parse_xml_properties(src) -> List[Tuple[str, Optional[str], bool, Optional[str], Optional[str]]]:
    """Parse ``<configuration><property>…`` into (name, value, final, description, source); ``source`` is
    the ``<source>`` element a written ``tony-final.xml`` carries per property (None elsewhere)."""
    if isinstance(src, (bytes, bytearray)):
        root = ET.fromstring(src)
    elif hasattr(src, "read"):
        root = ET.parse(src).getroot()
    else:
        root = ET.parse(str(src)).getroot()
    if root.tag != "configuration":
        raise ConfigurationError(f"bad conf root element <{root.tag}>")
    props = []
    for p in root.iter("property"):
        name = p.findtext("name")
        if name is None:
            continue
        value_el = p.find("value")
        value = None if value_el is None else (value_el.text or "")
        final = (p.findtext("final") or "").strip().lower() == "true"
        src_el = p.findtext("source")
        props.append((name.strip(), value, final, p.findtext("description"),
                      src_el.strip() if src_el and src_el.strip() else None))
    return props


class Configuration:
    def __init__(self, load_defaults: bool = True):
        self._lock = threading.RLock()
        self._resources: List[Tuple[str, list]] = []
        self._overlay: Dict[str, Tuple[str, str]] = {}  # set() values: key -> (value, source)
        self._props: Dict[str, Tuple[Optional[str], str]] = {}
        self._final: set = set()
        self._unset: set = set()
        if load_defaults:
            self.add_resource(DEFAULT_XML, "tony-default.xml")

    # -- loading ------------------------------------------------------------------
    def add_resource(self, src, name: Optional[str] = None) -> "Configuration":
        props = parse_xml_properties(src)
        label = name or (str(src) if not hasattr(src, "read") else "stream")
        with self._lock:
            self._resources.append((label, props))
            self._apply_resource(label, props)
        return self

    def _apply_resource(self, label, props):
        for key, value, final, _, source in props:
            if key in self._final:
                continue  # an earlier resource marked it final
            if value is None:
                continue
            # a re-read tony-final.xml keeps each value's original source (e.g. tony-default.xml)
            self._props[key] = (value, source or label)
            if final:
                self._final.add(key)

    # -- access ---------------------------------------------------------------------
    def _raw(self, key: str) -> Optional[Tuple[str, str]]:
        if key in self._unset:
            return None
        if key in self._overlay:
            return self._overlay[key]
        return self._props.get(key)

    def get_raw(self, key: str) -> Optional[str]:
        with self._lock:
            r = self._raw(key)
        return None if r is None else r[0]

    def _expand(self, value: str) -> str:
        for _ in range(_MAX_SUBST):
            m = _VAR.search(value)
            if not m:
                return value
            name = m.group(1)
            if name.startswith("env."):
                rep = os.environ.get(name[4:])
            else:
                rep = self.get_raw(name)
                if rep is None:
                    rep = os.environ.get(name) if name.isupper() else None
            if rep is None:
                return value  # leave unresolvable references as-is (Hadoop behaviour)
            value = value[:m.start()] + rep + value[m.end():]
        raise ConfigurationError(f"variable substitution depth exceeded for {value!r}")

    def get(self, key: str, default: Optional[str] = None) -> Optional[str]:
        v = self.get_raw(key)
        if v is None:
            return default
        return self._expand(v)

    def __getitem__(self, key):
        v = self.get(key)
        if v is None:
            raise KeyError(key)
        return v

    def __contains__(self, key) -> bool:
        return self.get_raw(key) is not None

    def get_trimmed(self, key: str, default: Optional[str] = None) -> Optional[str]:
        v = self.get(key)
        if v is None:
            return default
        v = v.strip()
        return v if v else default

    def get_int(self, key: str, default: int = 0) -> int:
        v = self.get_trimmed(key)
        if v is None:
            return default
        try:
            return int(v, 16) if v.lower().startswith("0x") else int(v)
        except ValueError as e:
            raise ConfigurationError(f"{key}={v!r} is not an integer") from e

    def get_float(self, key: str, default: float = 0.0) -> float:
        v = self.get_trimmed(key)
        return default if v is None else float(v)

    def get_bool(self, key: str, default: bool = False) -> bool:
        v = self.get_trimmed(key)
        if v is None:
            return default
        lv = v.lower()
        if lv in ("true", "1", "yes"):
            return True
        if lv in ("false", "0", "no"):
            return False
        return default

    def get_strings(self, key: str, default=None) -> List[str]:
        v = self.get(key)
        if v is None:
            return list(default) if default is not None else []
        return [s.strip() for s in v.split(",") if s.strip()]

    def get_source(self, key: str) -> Optional[str]:
        with self._lock:
            r = self._raw(key)
        return None if r is None else r[1]

    def is_final(self, key: str) -> bool:
        return key in self._final

    # -- mutation ---------------------------------------------------------------------
    def set(self, key: str, value, source: str = "programmatically") -> None:
        if value is None:
            raise ConfigurationError(f"null value for {key}")
        with self._lock:
            self._unset.discard(key)
            self._overlay[key] = (str(value), source)

    def set_if_unset(self, key: str, value) -> None:
        if self.get_raw(key) is None:
            self.set(key, value)

    def set_int(self, key: str, value: int) -> None:
        self.set(key, int(value))

    def set_bool(self, key: str, value: bool) -> None:
        self.set(key, "true" if value else "false")

    def set_strings(self, key: str, values) -> None:
        self.set(key, ",".join(values))

    def unset(self, key: str) -> None:
        with self._lock:
            self._overlay.pop(key, None)
            self._unset.add(key)

    # -- iteration / export -----------------------------------------------------------
    def keys(self) -> List[str]:
        with self._lock:
            ks = set(self._props) | set(self._overlay)
            return sorted(k for k in ks if k not in self._unset)

    def items(self) -> Iterator[Tuple[str, str]]:
        for k in self.keys():
            v = self.get(k)
            if v is not None:
                yield k, v

    def get_val_by_regex(self, pattern) -> Dict[str, str]:
        rx = re.compile(pattern) if isinstance(pattern, str) else pattern
        return {k: v for k, v in self.items() if rx.match(k)}

    def copy(self) -> "Configuration":
        c = Configuration(load_defaults=False)
        with self._lock:
            c._resources = list(self._resources)
            c._overlay = dict(self._overlay)
            c._props = dict(self._props)
            c._final = set(self._final)
            c._unset = set(self._unset)
        return c

    def to_xml(self) -> str:
        root = ET.Element("configuration")
        for k in self.keys():
            raw = self._raw(k)
            if raw is None:
                continue
            p = ET.SubElement(root, "property")
            ET.SubElement(p, "name").text = k
            ET.SubElement(p, "value").text = raw[0]
            ET.SubElement(p, "final").text = "true" if k in self._final else "false"
            ET.SubElement(p, "source").text = raw[1]
        ET.indent(root)
        buf = io.StringIO()
        buf.write('<?xml version="1.0" encoding="UTF-8" standalone="no"?>\n')
        buf.write(ET.tostring(root, encoding="unicode"))
        buf.write("\n")
        return buf.getvalue()

    def write_xml(self, path: str) -> None:
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(self.to_xml())
        os.replace(tmp, path)

    @classmethod
    def from_xml(cls, path: str, load_defaults: bool = False) -> "Configuration":
        c = cls(load_defaults=load_defaults)
        c.add_resource(path, os.path.basename(path))
        return c

    def __repr__(self):
        return f"Configuration({len(self.keys())} keys, resources={[r[0] for r in self._resources]})"
