"""Yjs output sync (the fork's ``workflows`` map: ``server.py:144-145, 825-832``,
``execution.py:334-345``; SURVEY §2.1 C02, §2.3 "Yjs encoder").

The reference keeps a y_py ``YDoc`` with one ``YMap`` named ``workflows``; after a node runs, each
``prompt["outputs"][key] = [node_id, slot]`` result is ``output_map.set(key, json.dumps(value))`` and
the doc is broadcast as ``encode_state_as_update()`` (its send path is broken: ``ws.send`` does not
exist on aiohttp, ``json.dumps(bytes)`` raises). y_py (Rust yrs) is not available here, so this module
implements the one shape the fork uses — a single-writer ``YMap<string, Any>`` — natively, emitting
the real Yjs **update v1** wire format (lib0 encoding) that ``Y.applyUpdate`` accepts:

  update      = varuint #clients, per client (descending id): varuint #structs, varuint client,
                varuint first clock, structs...; then the delete set
  Item        = info byte (content ref | 0x80 origin | 0x40 right origin | 0x20 parentSub),
                [origin ID], and when there is no origin: parent info 1 + varstring root-type key +
                varstring parentSub; then the content
  ContentAny  = ref 8: varuint count, lib0 ``writeAny`` values (string: tag 119 + varstring, ...)
  ContentDeleted = ref 1: varuint length (a garbage-collected overwritten value)
  delete set  = varuint #clients, per client: varuint client, varuint #ranges, (clock, len)...

``YMap.set`` creates an Item whose origin is the key's previous Item (Yjs ``typeMapSet``) and
deletes that previous Item, exactly the history a y_py writer produces. ``decode_update`` parses the
same format back (used to apply client updates and by the tests); byte-for-byte parity against
y_py itself is unpinned (not importable here) — the tests pin the layout from the format spec.
"""
from __future__ import annotations

import base64
import random
import struct
import threading

REF_DELETED, REF_JSON, REF_BINARY, REF_STRING, REF_ANY = 1, 2, 3, 4, 8
BIT_ORIGIN, BIT_RIGHT_ORIGIN, BIT_PARENT_SUB = 0x80, 0x40, 0x20


# ---------------------------------------------------------------------------------------- lib0
def write_varuint(out: bytearray, n: int):
    n = int(n)
    while n > 0x7F:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)


def write_varint(out: bytearray, n: int):
    neg = n < 0
    n = -n if neg else n
    out.append((0x80 if n > 0x3F else 0) | (0x40 if neg else 0) | (n & 0x3F))
    n >>= 6
    while n > 0:
        out.append((0x80 if n > 0x7F else 0) | (n & 0x7F))
        n >>= 7


def write_varstring(out: bytearray, s: str):
    b = s.encode("utf-8")
    write_varuint(out, len(b))
    out += b


def write_any(out: bytearray, v):
    """lib0 ``encoding.writeAny``."""
    if v is None:
        out.append(126)
    elif v is True:
        out.append(120)
    elif v is False:
        out.append(121)
    elif isinstance(v, int) and -(1 << 31) <= v < (1 << 31):
        out.append(125)
        write_varint(out, v)
    elif isinstance(v, (int, float)):
        f = float(v)
        if struct.unpack(">f", struct.pack(">f", f))[0] == f:
            out.append(124)
            out += struct.pack(">f", f)
        else:
            out.append(123)
            out += struct.pack(">d", f)
    elif isinstance(v, str):
        out.append(119)
        write_varstring(out, v)
    elif isinstance(v, (bytes, bytearray)):
        out.append(116)
        write_varuint(out, len(v))
        out += bytes(v)
    elif isinstance(v, dict):
        out.append(118)
        write_varuint(out, len(v))
        for k, x in v.items():
            write_varstring(out, str(k))
            write_any(out, x)
    elif isinstance(v, (list, tuple)):
        out.append(117)
        write_varuint(out, len(v))
        for x in v:
            write_any(out, x)
    else:
        raise TypeError(f"cannot encode {type(v).__name__} as a Yjs Any value")


class Reader:
    def __init__(self, data: bytes):
        self.d = bytes(data)
        self.p = 0

    def u8(self):
        v = self.d[self.p]
        self.p += 1
        return v

    def varuint(self):
        n, shift = 0, 0
        while True:
            b = self.u8()
            n |= (b & 0x7F) << shift
            shift += 7
            if b < 0x80:
                return n

    def varint(self):
        b = self.u8()
        n = b & 0x3F
        neg = b & 0x40
        shift = 6
        while b & 0x80:
            b = self.u8()
            n |= (b & 0x7F) << shift
            shift += 7
        return -n if neg else n

    def varstring(self):
        n = self.varuint()
        s = self.d[self.p:self.p + n].decode("utf-8")
        self.p += n
        return s

    def any(self):
        t = self.u8()
        if t == 127:
            return None     # undefined
        if t == 126:
            return None
        if t == 125:
            return self.varint()
        if t == 124:
            v = struct.unpack(">f", self.d[self.p:self.p + 4])[0]
            self.p += 4
            return v
        if t == 123:
            v = struct.unpack(">d", self.d[self.p:self.p + 8])[0]
            self.p += 8
            return v
        if t == 122:
            v = struct.unpack(">q", self.d[self.p:self.p + 8])[0]
            self.p += 8
            return v
        if t == 121:
            return False
        if t == 120:
            return True
        if t == 119:
            return self.varstring()
        if t == 118:
            return {self.varstring(): self.any() for _ in range(self.varuint())}
        if t == 117:
            return [self.any() for _ in range(self.varuint())]
        if t == 116:
            n = self.varuint()
            v = self.d[self.p:self.p + n]
            self.p += n
            return v
        raise ValueError(f"unknown lib0 any tag {t}")


# ---------------------------------------------------------------------------------------- doc
class _Item:
    __slots__ = ("client", "clock", "key", "value", "origin", "deleted")

    def __init__(self, client, clock, key, value, origin):
        self.client, self.clock, self.key, self.value, self.origin = client, clock, key, value, origin
        self.deleted = False


class YDoc:
    """One client's document holding root ``YMap``s of single values (the fork's usage)."""

    def __init__(self, client_id: int | None = None):
        self.client_id = int(client_id) if client_id is not None else random.getrandbits(32)
        self.items: list[_Item] = []            # this client's structs, clock order (length 1 each)
        self.maps: dict[str, dict[str, _Item]] = {}
        self._lock = threading.RLock()

    def get_map(self, name: str) -> "YMap":
        self.maps.setdefault(name, {})
        return YMap(self, name)

    # -- encoding
    def state_vector(self) -> dict:
        return {self.client_id: len(self.items)} if self.items else {}

    def encode_state_vector(self) -> bytes:
        out = bytearray()
        sv = self.state_vector()
        write_varuint(out, len(sv))
        for c, clk in sorted(sv.items(), reverse=True):
            write_varuint(out, c)
            write_varuint(out, clk)
        return bytes(out)

    def _root_of(self, item: _Item) -> str:
        for name, m in self.maps.items():
            if any(it is item for it in m.values()):
                return name
        for name, m in self.maps.items():   # deleted items: walk the key's origin chain
            cur = m.get(item.key)
            while cur is not None:
                if cur is item:
                    return name
                cur = self._by_id(cur.origin)
        raise KeyError(item.key)

    def _by_id(self, ident):
        if ident is None:
            return None
        c, clk = ident
        return self.items[clk] if c == self.client_id and clk < len(self.items) else None

    def encode_state_as_update(self, since: int = 0) -> bytes:
        """Yjs update v1 with this client's structs from clock ``since`` (0: the whole state) and the
        full delete set (Yjs always ships the whole delete set)."""
        with self._lock:
            out = bytearray()
            structs = self.items[since:]
            if structs:
                write_varuint(out, 1)
                write_varuint(out, len(structs))
                write_varuint(out, self.client_id)
                write_varuint(out, structs[0].clock)
                for it in structs:
                    self._write_item(out, it)
            else:
                write_varuint(out, 0)
            self._write_delete_set(out)
            return bytes(out)

    def _write_item(self, out, it: _Item):
        ref = REF_DELETED if it.deleted else REF_ANY
        info = ref | BIT_PARENT_SUB | (BIT_ORIGIN if it.origin is not None else 0)
        out.append(info)
        if it.origin is not None:
            write_varuint(out, it.origin[0])
            write_varuint(out, it.origin[1])
        else:
            write_varuint(out, 1)                      # parent is a root type, named by its key
            write_varstring(out, self._root_of(it))
            write_varstring(out, it.key)
        if it.deleted:
            write_varuint(out, 1)                      # ContentDeleted length
        else:
            write_varuint(out, 1)                      # ContentAny: one value
            write_any(out, it.value)

    def _write_delete_set(self, out):
        ranges = []
        for it in self.items:
            if it.deleted:
                if ranges and ranges[-1][0] + ranges[-1][1] == it.clock:
                    ranges[-1][1] += 1
                else:
                    ranges.append([it.clock, 1])
        if not ranges:
            write_varuint(out, 0)
            return
        write_varuint(out, 1)
        write_varuint(out, self.client_id)
        write_varuint(out, len(ranges))
        for clk, n in ranges:
            write_varuint(out, clk)
            write_varuint(out, n)


class YMap:
    def __init__(self, doc: YDoc, name: str):
        self.doc, self.name = doc, name

    def set(self, key: str, value):
        d = self.doc
        with d._lock:
            m = d.maps[self.name]
            left = m.get(key)
            it = _Item(d.client_id, len(d.items), key, value,
                       None if left is None else (left.client, left.clock))
            if left is not None:
                left.deleted = True
            d.items.append(it)
            m[key] = it

    def get(self, key, default=None):
        it = self.doc.maps[self.name].get(key)
        return default if it is None or it.deleted else it.value

    def to_json(self) -> dict:
        return {k: it.value for k, it in self.doc.maps[self.name].items() if not it.deleted}

    def __len__(self):
        return len(self.to_json())


def decode_update(data: bytes) -> dict:
    """Parse a Yjs update v1 holding root-map items -> {"structs": [...], "deletes": {client: [(clock, len)]},
    "maps": {root: {key: value}}} (the state a fresh doc reaches by applying it)."""
    r = Reader(data)
    structs = []
    by_id = {}
    for _ in range(r.varuint()):
        n, client, clock = r.varuint(), r.varuint(), r.varuint()
        for _ in range(n):
            info = r.u8()
            ref = info & 0x1F
            origin = right = None
            if info & BIT_ORIGIN:
                origin = (r.varuint(), r.varuint())
            if info & BIT_RIGHT_ORIGIN:
                right = (r.varuint(), r.varuint())
            root = key = None
            if origin is None and right is None:
                if r.varuint() != 1:
                    raise ValueError("only root-type parents are supported")
                root = r.varstring()
                if info & BIT_PARENT_SUB:
                    key = r.varstring()
            else:
                src = by_id.get(origin or right)
                root, key = (src["root"], src["key"]) if src else (None, None)
            if ref == REF_ANY:
                vals = [r.any() for _ in range(r.varuint())]
                value, length = vals[-1], len(vals)
            elif ref == REF_DELETED:
                value, length = None, r.varuint()
            elif ref == REF_STRING:
                value = r.varstring()
                length = len(value)
            else:
                raise ValueError(f"unsupported content ref {ref}")
            s = {"client": client, "clock": clock, "root": root, "key": key, "value": value, "ref": ref,
                 "origin": origin}
            structs.append(s)
            by_id[(client, clock)] = s
            clock += length
    deletes = {}
    for _ in range(r.varuint()):
        client = r.varuint()
        deletes[client] = [(r.varuint(), r.varuint()) for _ in range(r.varuint())]

    def is_deleted(s):
        return s["ref"] == REF_DELETED or any(c <= s["clock"] < c + n for c, n in deletes.get(s["client"], []))
    maps = {}
    for s in structs:
        if s["root"] is not None and not is_deleted(s):
            maps.setdefault(s["root"], {})[s["key"]] = s["value"]
    return {"structs": structs, "deletes": deletes, "maps": maps}


class OutputMap:
    """The server's ``workflows`` map: ``set`` from the executor, ``encode_update`` for the WS
    ``yjs_update`` event (base64 of the full-state update, as the reference broadcasts the whole state)."""

    NAME = "workflows"

    def __init__(self, server=None, client_id=None):
        self.doc = YDoc(client_id)
        self.map = self.doc.get_map(self.NAME)
        self.server = server

    def set(self, key, value):
        self.map.set(key, value)

    def get(self, key, default=None):
        return self.map.get(key, default)

    def to_json(self):
        return self.map.to_json()

    def encode_state_as_update(self) -> bytes:
        return self.doc.encode_state_as_update()

    def encode_update(self, full=True):
        upd = self.doc.encode_state_as_update()
        return {"encoding": "yjs-update-v1", "map": self.NAME, "update": base64.b64encode(upd).decode("ascii"),
                "state_vector": base64.b64encode(self.doc.encode_state_vector()).decode("ascii")}
