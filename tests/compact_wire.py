"""Test infrastructure: an independent pure-Python CompactProtocol encoder /
decoder for the Decision path's structs (openr/if/Lsdb.thrift:70-352,
Network.thrift:54-62), written from the published compact-protocol spec.

It checks the C++ codec in openr_amd/csrc/host/Publication.cpp in both
directions.  No fixture of fbthrift-produced bytes exists in the reference,
so the wire format itself is pinned by the spec and the hand-derived
known-answer bytes in tests/test_publication.py ("parity unpinned" against
fbthrift's own serializer).
"""

from __future__ import annotations

import struct

from openr_amd import thrift as T

STOP, TRUE, FALSE, BYTE, I16, I32, I64, DOUBLE, BINARY, LIST, SET, MAP, STRUCT = range(13)


class W:
    def __init__(self):
        self.b = bytearray()
        self.last = [0]

    def varint(self, v):
        while v >= 0x80:
            self.b.append((v & 0x7F) | 0x80)
            v >>= 7
        self.b.append(v)

    def zz(self, v):
        self.varint(((v << 1) ^ (v >> 63)) & 0xFFFFFFFFFFFFFFFF)

    def bin(self, s):
        if isinstance(s, str):
            s = s.encode()
        self.varint(len(s))
        self.b += s

    def field(self, fid, t):
        d = fid - self.last[-1]
        if 0 < d <= 15:
            self.b.append((d << 4) | t)
        else:
            self.b.append(t)
            self.zz(fid)
        self.last[-1] = fid

    def boolf(self, fid, v):
        self.field(fid, TRUE if v else FALSE)

    def lst(self, n, et):
        if n < 15:
            self.b.append((n << 4) | et)
        else:
            self.b.append(0xF0 | et)
            self.varint(n)

    def begin(self):
        self.last.append(0)

    def end(self):
        self.b.append(STOP)
        self.last.pop()


def _addr(w, a):
    w.begin()
    w.field(1, BINARY)
    w.bin(a.addr)
    if a.ifName is not None:
        w.field(3, BINARY)
        w.bin(a.ifName)
    w.end()


def _junk(w, fid):
    """An unknown field exercising every skip path: a PerfEvents-like struct
    with a list of structs, a map, a double, a set and a bool list."""
    w.field(fid, STRUCT)
    w.begin()
    w.field(1, LIST)
    w.lst(2, STRUCT)
    for i in range(2):
        w.begin()
        w.field(1, BINARY)
        w.bin(f"ev{i}")
        w.field(2, I64)
        w.zz(-(10**12) - i)
        w.end()
    w.field(2, MAP)
    w.varint(2)
    w.b.append((BINARY << 4) | I32)
    for k in ("x", "y"):
        w.bin(k)
        w.zz(-7)
    w.field(3, DOUBLE)
    w.b += struct.pack("<d", 2.5)
    w.field(40, SET)  # long-form id
    w.lst(16, BINARY)
    for i in range(16):
        w.bin(str(i))
    w.field(41, LIST)
    w.lst(3, TRUE)
    w.b += bytes([TRUE, FALSE, TRUE])
    w.end()


def encode_adj_db(db: T.AdjacencyDatabase, junk=False) -> bytes:
    w = W()
    w.field(1, BINARY)
    w.bin(db.thisNodeName)
    w.boolf(2, db.isOverloaded)
    w.field(3, LIST)
    w.lst(len(db.adjacencies), STRUCT)
    for a in db.adjacencies:
        w.begin()
        w.field(1, BINARY)
        w.bin(a.otherNodeName)
        w.field(2, BINARY)
        w.bin(a.ifName)
        w.field(3, STRUCT)
        _addr(w, a.nextHopV6)
        w.field(5, STRUCT)
        _addr(w, a.nextHopV4)
        w.field(4, I32)
        w.zz(a.metric)
        w.field(6, I32)
        w.zz(a.adjLabel)
        w.boolf(7, a.isOverloaded)
        w.field(8, I32)
        w.zz(a.rtt)
        w.field(9, I64)
        w.zz(a.timestamp)
        w.field(10, I64)
        w.zz(a.weight)
        w.field(11, BINARY)
        w.bin(a.otherIfName)
        if junk:
            _junk(w, 30)
        w.end()
    w.field(4, I32)
    w.zz(db.nodeLabel)
    if junk:
        _junk(w, 5)  # perfEvents
    w.field(6, BINARY)
    w.bin(db.area)
    w.b.append(STOP)
    return bytes(w.b)


def encode_prefix_db(db: T.PrefixDatabase, area_stacks=None, junk=False, per_prefix_key=None) -> bytes:
    w = W()
    w.field(1, BINARY)
    w.bin(db.thisNodeName)
    w.field(3, LIST)
    w.lst(len(db.prefixEntries), STRUCT)
    for i, e in enumerate(db.prefixEntries):
        w.begin()
        w.field(1, STRUCT)
        w.begin()
        w.field(1, STRUCT)
        _addr(w, e.prefix.prefixAddress)
        w.field(2, I16)
        w.zz(e.prefix.prefixLength)
        w.end()
        w.field(2, I32)
        w.zz(e.type)
        if e.data is not None:
            w.field(3, BINARY)
            w.bin(e.data)
        w.field(4, I32)
        w.zz(e.forwardingType)
        w.field(7, I32)
        w.zz(e.forwardingAlgorithm)
        if e.ephemeral is not None:
            w.boolf(5, e.ephemeral)
        if e.mv is not None:
            w.field(6, STRUCT)
            w.begin()
            w.field(1, I64)
            w.zz(e.mv.version)
            w.field(2, LIST)
            w.lst(len(e.mv.metrics), STRUCT)
            for me in e.mv.metrics:
                w.begin()
                w.field(1, I64)
                w.zz(me.type)
                w.field(2, I64)
                w.zz(me.priority)
                w.field(3, I32)
                w.zz(me.op)
                w.boolf(4, me.isBestPathTieBreaker)
                w.field(5, LIST)
                w.lst(len(me.metric), I64)
                for m in me.metric:
                    w.zz(m)
                w.end()
            w.end()
        if e.minNexthop is not None:
            w.field(8, I64)
            w.zz(e.minNexthop)
        if e.prependLabel is not None:
            w.field(9, I32)
            w.zz(e.prependLabel)
        if junk:
            _junk(w, 10)  # PrefixMetrics
            w.field(11, SET)  # tags
            w.lst(2, BINARY)
            w.bin("t1")
            w.bin("t2")
        st = area_stacks[i] if area_stacks else []
        w.field(12, LIST)
        w.lst(len(st), BINARY)
        for a in st:
            w.bin(a)
        w.end()
    w.boolf(5, db.deletePrefix)
    if junk:
        _junk(w, 4)  # perfEvents (declared after 5: long-form / backward id)
    if per_prefix_key is not None:
        w.boolf(6, per_prefix_key)
    w.field(7, BINARY)
    w.bin(db.area)
    w.b.append(STOP)
    return bytes(w.b)


# ------------------------------------------------------------------ reader


class R:
    def __init__(self, b):
        self.b, self.i = b, 0

    def byte(self):
        x = self.b[self.i]
        self.i += 1
        return x

    def varint(self):
        r = s = 0
        while True:
            x = self.byte()
            r |= (x & 0x7F) << s
            s += 7
            if not x & 0x80:
                return r

    def zz(self):
        v = self.varint()
        return (v >> 1) ^ -(v & 1)

    def bin(self):
        n = self.varint()
        s = bytes(self.b[self.i : self.i + n])
        self.i += n
        return s

    def fields(self):
        last = 0
        while True:
            x = self.byte()
            if x == STOP:
                return
            t, d = x & 15, x >> 4
            fid = last + d if d else self.zz()
            last = fid
            yield fid, t

    def lst(self):
        x = self.byte()
        n, et = x >> 4, x & 15
        if n == 15:
            n = self.varint()
        return n, et


def _raddr(r):
    a = T.BinaryAddress()
    for fid, t in r.fields():
        if fid == 1:
            a.addr = r.bin()
        elif fid == 3:
            a.ifName = r.bin().decode()
        else:
            raise AssertionError(f"unexpected BinaryAddress field {fid}")
    return a


def decode_adj_db(b: bytes) -> T.AdjacencyDatabase:
    r = R(b)
    db = T.AdjacencyDatabase()
    for fid, t in r.fields():
        if fid == 1:
            db.thisNodeName = r.bin().decode()
        elif fid == 2:
            db.isOverloaded = t == TRUE
        elif fid == 3:
            n, et = r.lst()
            assert et == STRUCT
            for _ in range(n):
                a = T.Adjacency()
                for f2, t2 in r.fields():
                    if f2 == 1:
                        a.otherNodeName = r.bin().decode()
                    elif f2 == 2:
                        a.ifName = r.bin().decode()
                    elif f2 == 3:
                        a.nextHopV6 = _raddr(r)
                    elif f2 == 5:
                        a.nextHopV4 = _raddr(r)
                    elif f2 == 7:
                        a.isOverloaded = t2 == TRUE
                    elif f2 == 11:
                        a.otherIfName = r.bin().decode()
                    else:
                        setattr(a, {4: "metric", 6: "adjLabel", 8: "rtt", 9: "timestamp",
                                    10: "weight"}[f2], r.zz())
                db.adjacencies.append(a)
        elif fid == 4:
            db.nodeLabel = r.zz()
        elif fid == 6:
            db.area = r.bin().decode()
        else:
            raise AssertionError(f"unexpected AdjacencyDatabase field {fid}")
    assert r.i == len(b)
    return db
