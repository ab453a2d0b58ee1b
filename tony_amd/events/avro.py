"""Minimal Apache Avro object-container-file (OCF) writer/reader, null/deflate codecs.

TonY writes its job history (``.jhist``) as Avro container files
(T/events/EventHandler.java:22-157, schemas in tony-core/src/main/avro/).  No
Avro library is installed here, so this module implements the binary encoding
and the container framing directly from the Avro 1.x specification:

* zig-zag varint ``int``/``long``, little-endian IEEE ``float``/``double``,
  length-prefixed ``bytes``/``string``, enums as int index, unions as
  ``long branch + value``, blocked ``array``/``map`` terminated by a 0 count;
* header = ``Obj\\x01`` + metadata map (``avro.schema``, ``avro.codec``) + 16-byte
  sync marker; then blocks of ``count, size, payload, sync``.

Named types declared anywhere in the schema (or pre-registered) may be
referenced by name or full name, which TonY's ``Event`` schema relies on.
"""
from __future__ import annotations

import io
import json
import os
import struct
import zlib
from typing import Any, BinaryIO, Dict, Iterator, List, Optional

MAGIC = b"Obj\x01"


class AvroError(ValueError):
    pass


# -- primitive codecs ----------------------------------------------------------------
def _write_long(out: BinaryIO, n: int) -> None:
    n = (n << 1) ^ (n >> 63)
    while n & ~0x7F:
        out.write(bytes(((n & 0x7F) | 0x80,)))
        n >>= 7
    out.write(bytes((n,)))


def _read_long(inp: BinaryIO) -> int:
    shift = 0
    acc = 0
    while True:
        b = inp.read(1)
        if not b:
            raise EOFError
        b = b[0]
        acc |= (b & 0x7F) << shift
        if not b & 0x80:
            break
        shift += 7
    return (acc >> 1) ^ -(acc & 1)


def _write_bytes(out, b: bytes):
    _write_long(out, len(b))
    out.write(b)


def _read_bytes(inp) -> bytes:
    n = _read_long(inp)
    b = inp.read(n)
    if len(b) != n:
        raise EOFError
    return b


# -- schema handling -------------------------------------------------------------------
_PRIMS = {"null", "boolean", "int", "long", "float", "double", "bytes", "string"}


class Schema:
    """A parsed schema with a table of named types."""

    def __init__(self, schema, named: Optional[Dict[str, Any]] = None):
        self.named: Dict[str, Any] = dict(named or {})
        self.root = self._register(json.loads(schema) if isinstance(schema, str) else schema, None)

    def _fullname(self, name: str, ns: Optional[str]) -> str:
        return name if "." in name or not ns else f"{ns}.{name}"

    def _register(self, s, ns):
        if isinstance(s, list):
            return [self._register(x, ns) for x in s]
        if isinstance(s, str):
            return s
        t = s.get("type")
        if t in ("record", "error", "enum", "fixed"):
            ns = s.get("namespace", ns)
            full = self._fullname(s["name"], ns)
            s = dict(s)
            s["_full"] = full
            self.named[full] = s
            self.named.setdefault(s["name"], s)
            if t in ("record", "error"):
                s["fields"] = [dict(f, type=self._register(f["type"], ns)) for f in s["fields"]]
            return s
        if t == "array":
            return dict(s, items=self._register(s["items"], ns))
        if t == "map":
            return dict(s, values=self._register(s["values"], ns))
        return s

    def resolve(self, s):
        if isinstance(s, str) and s not in _PRIMS:
            if s not in self.named:
                raise AvroError(f"unknown named type {s!r}")
            return self.named[s]
        if isinstance(s, dict) and s.get("type") in _PRIMS:  # e.g. {"type":"string","avro.java.string":..}
            return s["type"]
        return s

    def to_json(self) -> str:
        def strip(s):
            if isinstance(s, list):
                return [strip(x) for x in s]
            if isinstance(s, dict):
                return {k: strip(v) for k, v in s.items() if k != "_full"}
            return s
        return json.dumps(strip(self.root))


def _type_name(s) -> str:
    if isinstance(s, str):
        return s
    if isinstance(s, dict):
        return s.get("_full") or s.get("name") or s["type"]
    return "union"


def _matches(schema: Schema, s, v) -> bool:
    s = schema.resolve(s)
    if s == "null":
        return v is None
    if s == "boolean":
        return isinstance(v, bool)
    if s in ("int", "long"):
        return isinstance(v, int) and not isinstance(v, bool)
    if s in ("float", "double"):
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    if s == "string":
        return isinstance(v, str)
    if s == "bytes":
        return isinstance(v, (bytes, bytearray))
    if isinstance(s, dict):
        t = s["type"]
        if t in ("record", "error"):
            return isinstance(v, dict) and all(f["name"] in v or "default" in f for f in s["fields"])
        if t == "enum":
            return isinstance(v, str) and v in s["symbols"]
        if t == "array":
            return isinstance(v, (list, tuple))
        if t == "map":
            return isinstance(v, dict)
        if t == "fixed":
            return isinstance(v, (bytes, bytearray)) and len(v) == s["size"]
    return False


def encode(schema: Schema, s, v, out: BinaryIO) -> None:
    s = schema.resolve(s)
    if isinstance(s, list):  # union: value may be given as {"TypeName": value} or bare
        if isinstance(v, dict) and len(v) == 1:
            (k, inner), = v.items()
            for i, b in enumerate(s):
                rb = schema.resolve(b)
                if _type_name(rb) == k or (isinstance(rb, dict) and rb.get("name") == k):
                    _write_long(out, i)
                    encode(schema, b, inner, out)
                    return
        for i, b in enumerate(s):
            if _matches(schema, b, v):
                _write_long(out, i)
                encode(schema, b, v, out)
                return
        raise AvroError(f"value {v!r} matches no branch of union {[_type_name(b) for b in s]}")
    if s == "null":
        return
    if s == "boolean":
        out.write(b"\x01" if v else b"\x00")
    elif s in ("int", "long"):
        _write_long(out, int(v))
    elif s == "float":
        out.write(struct.pack("<f", float(v)))
    elif s == "double":
        out.write(struct.pack("<d", float(v)))
    elif s == "string":
        _write_bytes(out, v.encode("utf-8"))
    elif s == "bytes":
        _write_bytes(out, bytes(v))
    elif isinstance(s, dict):
        t = s["type"]
        if t in ("record", "error"):
            for f in s["fields"]:
                val = v.get(f["name"], f.get("default")) if isinstance(v, dict) else getattr(v, f["name"])
                encode(schema, f["type"], val, out)
        elif t == "enum":
            out_i = s["symbols"].index(v)
            _write_long(out, out_i)
        elif t == "array":
            if v:
                _write_long(out, len(v))
                for item in v:
                    encode(schema, s["items"], item, out)
            _write_long(out, 0)
        elif t == "map":
            if v:
                _write_long(out, len(v))
                for k, item in v.items():
                    _write_bytes(out, k.encode("utf-8"))
                    encode(schema, s["values"], item, out)
            _write_long(out, 0)
        elif t == "fixed":
            out.write(bytes(v))
        else:
            raise AvroError(f"unsupported schema {s}")
    else:
        raise AvroError(f"unsupported schema {s}")


def decode(schema: Schema, s, inp: BinaryIO):
    s = schema.resolve(s)
    if isinstance(s, list):
        i = _read_long(inp)
        return decode(schema, s[i], inp)
    if s == "null":
        return None
    if s == "boolean":
        return inp.read(1) != b"\x00"
    if s in ("int", "long"):
        return _read_long(inp)
    if s == "float":
        return struct.unpack("<f", inp.read(4))[0]
    if s == "double":
        return struct.unpack("<d", inp.read(8))[0]
    if s == "string":
        return _read_bytes(inp).decode("utf-8")
    if s == "bytes":
        return _read_bytes(inp)
    t = s["type"]
    if t in ("record", "error"):
        return {f["name"]: decode(schema, f["type"], inp) for f in s["fields"]}
    if t == "enum":
        return s["symbols"][_read_long(inp)]
    if t in ("array", "map"):
        items: Any = [] if t == "array" else {}
        while True:
            n = _read_long(inp)
            if n == 0:
                break
            if n < 0:
                n = -n
                _read_long(inp)  # block byte size
            for _ in range(n):
                if t == "array":
                    items.append(decode(schema, s["items"], inp))
                else:
                    k = _read_bytes(inp).decode("utf-8")
                    items[k] = decode(schema, s["values"], inp)
        return items
    if t == "fixed":
        return inp.read(s["size"])
    raise AvroError(f"unsupported schema {s}")


# -- container files --------------------------------------------------------------------
class DataFileWriter:
    def __init__(self, fobj: BinaryIO, schema: Schema, codec: str = "null", sync_interval: int = 16 * 1024):
        if codec not in ("null", "deflate"):
            raise AvroError(f"unsupported codec {codec}")
        self.f = fobj
        self.schema = schema
        self.codec = codec
        self.sync = os.urandom(16)
        self.buf = io.BytesIO()
        self.count = 0
        self.sync_interval = sync_interval
        self.f.write(MAGIC)
        meta = {"avro.schema": schema.to_json().encode(), "avro.codec": codec.encode()}
        _write_long(self.f, len(meta))
        for k, v in meta.items():
            _write_bytes(self.f, k.encode())
            _write_bytes(self.f, v)
        _write_long(self.f, 0)
        self.f.write(self.sync)

    def append(self, datum) -> None:
        encode(self.schema, self.schema.root, datum, self.buf)
        self.count += 1
        if self.buf.tell() >= self.sync_interval:
            self.flush()

    def flush(self) -> None:
        if self.count:
            payload = self.buf.getvalue()
            if self.codec == "deflate":
                c = zlib.compressobj(zlib.Z_DEFAULT_COMPRESSION, zlib.DEFLATED, -15)
                payload = c.compress(payload) + c.flush()
            _write_long(self.f, self.count)
            _write_long(self.f, len(payload))
            self.f.write(payload)
            self.f.write(self.sync)
            self.buf = io.BytesIO()
            self.count = 0
        self.f.flush()

    def close(self) -> None:
        self.flush()
        self.f.close()


class DataFileReader:
    def __init__(self, fobj: BinaryIO, named: Optional[Dict[str, Any]] = None):
        self.f = fobj
        if self.f.read(4) != MAGIC:
            raise AvroError("not an Avro object container file")
        meta = {}
        while True:
            n = _read_long(self.f)
            if n == 0:
                break
            if n < 0:
                n = -n
                _read_long(self.f)
            for _ in range(n):
                k = _read_bytes(self.f).decode()
                meta[k] = _read_bytes(self.f)
        self.meta = meta
        self.codec = meta.get("avro.codec", b"null").decode()
        self.schema = Schema(meta["avro.schema"].decode(), named)
        self.sync = self.f.read(16)

    def __iter__(self) -> Iterator[Any]:
        while True:
            try:
                count = _read_long(self.f)
            except EOFError:
                return
            size = _read_long(self.f)
            payload = self.f.read(size)
            if self.codec == "deflate":
                payload = zlib.decompress(payload, -15)
            elif self.codec != "null":
                raise AvroError(f"unsupported codec {self.codec}")
            blk = io.BytesIO(payload)
            for _ in range(count):
                yield decode(self.schema, self.schema.root, blk)
            if self.f.read(16) != self.sync:
                raise AvroError("sync marker mismatch")

    def close(self):
        self.f.close()


def read_all(path: str) -> List[Any]:
    """All records of an OCF file; an empty file (a history file whose writer
    never flushed) yields no records."""
    if os.path.getsize(path) == 0:
        return []
    with open(path, "rb") as f:
        return list(DataFileReader(f))
