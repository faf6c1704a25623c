"""Order-free per-route hashes of a RouteDb (TEST INFRASTRUCTURE).

A RouteDb as the bindings return it ({"unicast": {prefix: entry}, "mpls":
{label: next-hop set}}, the same Python form from the engine and the oracle)
becomes {"unicast": {key: h}, "mpls": {key: h}} with h a 64-bit hash of the
route's canonical form (every set sorted), so that a committed golden can
name the routes that differ, and route deltas (getRouteDelta, Decision.cpp:
47-85) can be checked as "the keys whose hash changed".
"""

from __future__ import annotations

import gzip
import hashlib
import json


def _canon(x):
    if isinstance(x, (frozenset, set)):
        return sorted((_canon(i) for i in x), key=repr)
    if isinstance(x, dict):
        return sorted(([_canon(k), _canon(v)] for k, v in x.items()), key=repr)
    if isinstance(x, (list, tuple)):
        return [_canon(i) for i in x]
    if isinstance(x, bytes):
        return x.hex()
    return x


def route_hash(value) -> str:
    return hashlib.blake2b(repr(_canon(value)).encode(), digest_size=8).hexdigest()


def key_str(key) -> str:
    if isinstance(key, tuple):  # unicast: (address bytes, prefix length)
        return f"{key[0].hex()}/{key[1]}"
    return str(int(key))  # MPLS top label


def route_hashes(db) -> dict:
    return {kind: {key_str(k): route_hash(v) for k, v in db[kind].items()}
            for kind in ("unicast", "mpls")}


def digest(hashes) -> str:
    h = hashlib.sha256()
    for kind in ("unicast", "mpls"):
        for k in sorted(hashes[kind]):
            h.update(f"{kind}|{k}|{hashes[kind][k]}\n".encode())
    return h.hexdigest()


def delta(new, base) -> dict:
    """Routes of `new` that differ from `base` (value = new hash, or None for
    a route `new` no longer has) -- getRouteDelta's updates + deletes."""
    out = {}
    for kind in ("unicast", "mpls"):
        a, b = new[kind], base[kind]
        d = {k: h for k, h in a.items() if b.get(k) != h}
        d.update({k: None for k in b if k not in a})
        out[kind] = d
    return out


def apply_delta(base, d) -> dict:
    out = {}
    for kind in ("unicast", "mpls"):
        m = dict(base[kind])
        for k, h in d[kind].items():
            if h is None:
                m.pop(k, None)
            else:
                m[k] = h
        out[kind] = m
    return out


def compare(got, want, what="") -> None:
    """Raise AssertionError naming the first differing routes."""
    for kind in ("unicast", "mpls"):
        a, b = got[kind], want[kind]
        if a == b:
            continue
        missing = sorted(set(b) - set(a))[:3]
        extra = sorted(set(a) - set(b))[:3]
        wrong = sorted(k for k in set(a) & set(b) if a[k] != b[k])[:3]
        raise AssertionError(
            f"{what} {kind}: {len(a)} routes vs {len(b)} golden; missing {missing}, "
            f"extra {extra}, different {wrong}")


def load(path) -> dict:
    with gzip.open(path, "rt") as f:
        return json.load(f)


def save(path, obj) -> None:
    data = json.dumps(obj, sort_keys=True, separators=(",", ":")).encode()
    with open(path, "wb") as raw, gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as f:
        f.write(data)
