"""Compact-protocol AdjacencyDatabase codec in pure Python — CPU ORACLE, test
infrastructure only (tests/ and scripts/ use it as the checker of the native codec in
openr_amd/csrc/host/AdjDbCodec.cpp; nothing in the product imports it).

What it restates:
* the wire format: fbthrift CompactProtocol (third-party, not vendored in
  /root/reference; pinned at build/deps/github_hashes/facebook/fbthrift-rev.txt =
  f101a1f5ff97b4cea790b205e12b10b9e2a2eb0a). Its published algorithm: a struct is a
  sequence of field headers + values ending in a 0x00 STOP byte; a header is one byte
  ``(id_delta << 4) | type`` when 0 < delta <= 15, else the type byte followed by the
  field id as a zigzag varint i16; booleans are folded into the header type (1 = true,
  2 = false; a bool inside a container is one byte 1/2); i16/i32/i64 are zigzag
  varints; binary/string = varint length + bytes; list/set header = one byte
  ``(size << 4) | elem_type`` when size < 15, else ``0xF0 | elem_type`` + varint size;
  map = varint size, then (if non-zero) one ``(ktype << 4) | vtype`` byte; double = 8
  bytes, float = 4 bytes.
* the schema: openr/if/Lsdb.thrift:24-32 (PerfEvent(s)), :71-129 (Adjacency,
  AdjacencyDatabase) and Network.thrift:55-58 (BinaryAddress); fields are written in
  IDL declaration order (Adjacency: 1, 2, 3, 5, 4, 6, ... — id 4 after id 5 needs the
  long header form).
* the call sites: writeThriftObjStr at openr/link-monitor/LinkMonitor.cpp:620 and
  readThriftObjStr at openr/decision/Decision.cpp:1755-1757 (CompactSerializer,
  Decision.h:399).

Parity status: the reference holds no serialized AdjacencyDatabase fixtures and its
thrift library is not importable here, so byte-level parity with fbthrift is pinned
only by the spec restated above and the hand-derived known-answer vectors in
tests/test_adjdb_codec.py ("parity unpinned" against a live fbthrift).

Values are dicts keyed by the thrift field names; addresses are raw bytes.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

STOP, BOOL_TRUE, BOOL_FALSE, BYTE, I16, I32, I64, DOUBLE, BINARY, LIST, SET, MAP, STRUCT, FLOAT = range(14)


class CompactError(ValueError):
    pass


# ----------------------------------------------------------------------------- writer
class Writer:
    def __init__(self) -> None:
        self.out = bytearray()
        self.last = [0]

    def varint(self, v: int) -> None:
        assert v >= 0
        while v >= 0x80:
            self.out.append((v & 0x7F) | 0x80)
            v >>= 7
        self.out.append(v)

    def zigzag32(self, v: int) -> None:
        self.varint(((v << 1) ^ (v >> 31)) & 0xFFFFFFFF)

    def zigzag64(self, v: int) -> None:
        self.varint(((v << 1) ^ (v >> 63)) & 0xFFFFFFFFFFFFFFFF)

    def binary(self, b: bytes) -> None:
        self.varint(len(b))
        self.out += b

    def header(self, ctype: int, fid: int) -> None:
        delta = fid - self.last[-1]
        if 0 < delta <= 15:
            self.out.append((delta << 4) | ctype)
        else:
            self.out.append(ctype)
            self.zigzag32(fid)
        self.last[-1] = fid

    def begin(self) -> None:
        self.last.append(0)

    def end(self) -> None:
        self.out.append(STOP)
        self.last.pop()

    def list_header(self, etype: int, n: int) -> None:
        if n < 15:
            self.out.append((n << 4) | etype)
        else:
            self.out.append(0xF0 | etype)
            self.varint(n)


def _s(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def write_binary_address(w: Writer, a: Dict[str, Any]) -> None:
    w.begin()
    w.header(BINARY, 1)
    w.binary(_s(a.get("addr", b"")))
    if a.get("ifName") is not None:
        w.header(BINARY, 3)
        w.binary(_s(a["ifName"]))
    w.end()


def write_adjacency(w: Writer, a: Dict[str, Any], extra=None) -> None:
    w.begin()
    w.header(BINARY, 1)
    w.binary(_s(a["otherNodeName"]))
    w.header(BINARY, 2)
    w.binary(_s(a["ifName"]))
    w.header(STRUCT, 3)
    write_binary_address(w, a.get("nextHopV6", {"addr": b""}))
    w.header(STRUCT, 5)
    write_binary_address(w, a.get("nextHopV4", {"addr": b""}))
    w.header(I32, 4)
    w.zigzag32(a.get("metric", 0))
    w.header(I32, 6)
    w.zigzag32(a.get("adjLabel", 0))
    w.header(BOOL_TRUE if a.get("isOverloaded", False) else BOOL_FALSE, 7)
    w.header(I32, 8)
    w.zigzag32(a.get("rtt", 0))
    w.header(I64, 9)
    w.zigzag64(a.get("timestamp", 0))
    w.header(I64, 10)
    w.zigzag64(a.get("weight", 1))
    w.header(BINARY, 11)
    w.binary(_s(a.get("otherIfName", "")))
    if extra:
        extra(w)
    w.end()


def write_adjacency_database(db: Dict[str, Any], extra_db=None, extra_adj=None) -> bytes:
    """writeThriftObjStr(AdjacencyDatabase). ``extra_db`` / ``extra_adj`` append
    unknown fields (callables on the Writer) before STOP, for skip tests."""
    w = Writer()
    w.begin()
    w.header(BINARY, 1)
    w.binary(_s(db["thisNodeName"]))
    w.header(BOOL_TRUE if db.get("isOverloaded", False) else BOOL_FALSE, 2)
    w.header(LIST, 3)
    adjs = db.get("adjacencies", [])
    w.list_header(STRUCT, len(adjs))
    for a in adjs:
        write_adjacency(w, a, extra_adj)
    w.header(I32, 4)
    w.zigzag32(db.get("nodeLabel", 0))
    pe = db.get("perfEvents")
    if pe is not None:
        w.header(STRUCT, 5)
        w.begin()
        w.header(LIST, 1)
        w.list_header(STRUCT, len(pe))
        for e in pe:
            w.begin()
            w.header(BINARY, 1)
            w.binary(_s(e["nodeName"]))
            w.header(BINARY, 2)
            w.binary(_s(e["eventDescr"]))
            w.header(I64, 3)
            w.zigzag64(e.get("unixTs", 0))
            w.end()
        w.end()
    w.header(BINARY, 6)
    w.binary(_s(db.get("area", "")))
    if extra_db:
        extra_db(w)
    w.end()
    return bytes(w.out)


# ----------------------------------------------------------------------------- reader
class Reader:
    def __init__(self, data: bytes) -> None:
        self.d = memoryview(data)
        self.p = 0

    def byte(self) -> int:
        if self.p >= len(self.d):
            raise CompactError("truncated input")
        b = self.d[self.p]
        self.p += 1
        return b

    def varint(self, max_bytes: int) -> int:
        v = 0
        for i in range(max_bytes):
            b = self.byte()
            v |= (b & 0x7F) << (7 * i)
            if not b & 0x80:
                return v
        raise CompactError("varint too long")

    def i16(self) -> int:
        u = self.varint(3) & 0xFFFFFFFF
        return _sext((u >> 1) ^ -(u & 1), 16)

    def i32(self) -> int:
        u = self.varint(5) & 0xFFFFFFFF
        return _sext(((u >> 1) ^ -(u & 1)) & 0xFFFFFFFF, 32)

    def i64(self) -> int:
        u = self.varint(10) & 0xFFFFFFFFFFFFFFFF
        return _sext(((u >> 1) ^ -(u & 1)) & 0xFFFFFFFFFFFFFFFF, 64)

    def binary(self) -> bytes:
        n = self.varint(5)
        if n > len(self.d) - self.p:
            raise CompactError("binary length exceeds input")
        b = bytes(self.d[self.p : self.p + n])
        self.p += n
        return b

    def header(self, last: List[int]) -> Optional[Tuple[int, int]]:
        b = self.byte()
        t = b & 0x0F
        if t == STOP:
            return None
        delta = b >> 4
        fid = last[0] + delta if delta else self.i16()
        last[0] = fid
        return t, fid

    def list_header(self) -> Tuple[int, int]:
        b = self.byte()
        n = b >> 4
        if n == 15:
            n = self.varint(5)
        if n > len(self.d) - self.p:
            raise CompactError("container size exceeds input")
        return b & 0x0F, n

    def skip(self, t: int, in_field: bool, depth: int = 0) -> None:
        if depth > 64:
            raise CompactError("nesting too deep")
        if t in (BOOL_TRUE, BOOL_FALSE):
            if not in_field:
                self.byte()
        elif t == BYTE:
            self.byte()
        elif t in (I16, I32, I64):
            self.varint(10)
        elif t in (DOUBLE, FLOAT):
            n = 8 if t == DOUBLE else 4
            if n > len(self.d) - self.p:
                raise CompactError("truncated input")
            self.p += n
        elif t == BINARY:
            self.binary()
        elif t in (LIST, SET):
            et, n = self.list_header()
            for _ in range(n):
                self.skip(et, False, depth + 1)
        elif t == MAP:
            n = self.varint(5)
            if n:
                if n > len(self.d) - self.p:
                    raise CompactError("container size exceeds input")
                kv = self.byte()
                for _ in range(n):
                    self.skip(kv >> 4, False, depth + 1)
                    self.skip(kv & 0x0F, False, depth + 1)
        elif t == STRUCT:
            last = [0]
            while (h := self.header(last)) is not None:
                self.skip(h[0], True, depth + 1)
        else:
            raise CompactError("unknown compact type")


def _sext(v: int, bits: int) -> int:
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def read_binary_address(r: Reader) -> Dict[str, Any]:
    a: Dict[str, Any] = {"addr": None, "ifName": None}
    last = [0]
    while (h := r.header(last)) is not None:
        t, fid = h
        if fid == 1 and t == BINARY:
            a["addr"] = r.binary()
        elif fid == 3 and t == BINARY:
            a["ifName"] = r.binary().decode(errors="surrogateescape")
        else:
            r.skip(t, True, 1)
    if a["addr"] is None:
        raise CompactError("required field 'addr' of BinaryAddress missing")
    return a


def read_adjacency(r: Reader) -> Dict[str, Any]:
    a: Dict[str, Any] = {"otherNodeName": "", "ifName": "", "nextHopV6": {"addr": b"", "ifName": None},
                         "nextHopV4": {"addr": b"", "ifName": None}, "metric": 0, "adjLabel": 0,
                         "isOverloaded": False, "rtt": 0, "timestamp": 0, "weight": 1, "otherIfName": ""}
    strs = {1: "otherNodeName", 2: "ifName", 11: "otherIfName"}
    i32s = {4: "metric", 6: "adjLabel", 8: "rtt"}
    i64s = {9: "timestamp", 10: "weight"}
    last = [0]
    while (h := r.header(last)) is not None:
        t, fid = h
        if fid in strs and t == BINARY:
            a[strs[fid]] = r.binary().decode(errors="surrogateescape")
        elif fid in (3, 5) and t == STRUCT:
            a["nextHopV6" if fid == 3 else "nextHopV4"] = read_binary_address(r)
        elif fid in i32s and t == I32:
            a[i32s[fid]] = r.i32()
        elif fid in i64s and t == I64:
            a[i64s[fid]] = r.i64()
        elif fid == 7 and t in (BOOL_TRUE, BOOL_FALSE):
            a["isOverloaded"] = t == BOOL_TRUE
        else:
            r.skip(t, True, 1)
    return a


def read_adjacency_database(data: bytes) -> Dict[str, Any]:
    """readThriftObjStr<AdjacencyDatabase> (trailing bytes after STOP ignored)."""
    r = Reader(data)
    db: Dict[str, Any] = {"thisNodeName": "", "isOverloaded": False, "adjacencies": [], "nodeLabel": 0,
                          "perfEvents": None, "area": ""}
    last = [0]
    while (h := r.header(last)) is not None:
        t, fid = h
        if fid == 1 and t == BINARY:
            db["thisNodeName"] = r.binary().decode(errors="surrogateescape")
        elif fid == 2 and t in (BOOL_TRUE, BOOL_FALSE):
            db["isOverloaded"] = t == BOOL_TRUE
        elif fid == 3 and t == LIST:
            et, n = r.list_header()
            if et != STRUCT:
                for _ in range(n):
                    r.skip(et, False, 1)
                continue
            db["adjacencies"] = [read_adjacency(r) for _ in range(n)]
        elif fid == 4 and t == I32:
            db["nodeLabel"] = r.i32()
        elif fid == 5 and t == STRUCT:
            events = []
            l2 = [0]
            while (h2 := r.header(l2)) is not None:
                t2, f2 = h2
                if f2 == 1 and t2 == LIST:
                    et, n = r.list_header()
                    if et != STRUCT:
                        for _ in range(n):
                            r.skip(et, False, 2)
                        continue
                    events = []
                    for _ in range(n):
                        e = {"nodeName": "", "eventDescr": "", "unixTs": 0}
                        l3 = [0]
                        while (h3 := r.header(l3)) is not None:
                            t3, f3 = h3
                            if f3 == 1 and t3 == BINARY:
                                e["nodeName"] = r.binary().decode(errors="surrogateescape")
                            elif f3 == 2 and t3 == BINARY:
                                e["eventDescr"] = r.binary().decode(errors="surrogateescape")
                            elif f3 == 3 and t3 == I64:
                                e["unixTs"] = r.i64()
                            else:
                                r.skip(t3, True, 3)
                        events.append(e)
                else:
                    r.skip(t2, True, 2)
            db["perfEvents"] = events
        elif fid == 6 and t == BINARY:
            db["area"] = r.binary().decode(errors="surrogateescape")
        else:
            r.skip(t, True, 1)
    return db
