"""SURVEY §8(f) row 4 — the step before the SPF path: CompactProtocol blobs
and Decision::processPublication (openr/decision/Decision.cpp:1631-1763,
updateNodePrefixDatabase :1585-1629; PrefixKey::fromStr
openr/common/Util.cpp:68-88; getNodeNameFromKey :1037-1044).

CPU tests: the C++ codec against the independent Python codec in
tests/compact_wire.py and hand-derived spec bytes (no fbthrift-made fixture
exists in the reference, so the wire format is pinned by the published
compact-protocol spec only), then ingest semantics against the object path.
The GPU test checks that RouteDbs built on byte-ingested state equal the
oracle's on object-ingested state.
"""

import random

import pytest

from openr_amd import thrift as T
from tests import compact_wire as CW
from tests import randomized as RZ


@pytest.fixture(scope="module")
def E():
    import openr_amd._openr_spf as E

    return E


def _rand_adj_db(rng, n_adj=3):
    adjs = []
    for i in range(n_adj):
        a = T.createAdjacency(f"nbr{i}", f"if_{i}", f"if_o{i}", f"fe80::{i + 1:x}", f"10.0.{i}.1",
                              rng.randint(-5, 2**31 - 1), rng.randint(0, 2**20))
        a.isOverloaded = rng.random() < 0.3
        a.rtt = rng.randint(-(2**31), 2**31 - 1)
        a.timestamp = rng.randint(-(2**63), 2**63 - 1)
        a.weight = rng.randint(-(2**40), 2**40)
        if rng.random() < 0.3:
            a.nextHopV6.ifName = f"eth{i}"
        adjs.append(a)
    return T.createAdjDb(f"node-{rng.randrange(1000)}", adjs, rng.randint(0, 2**20),
                         rng.random() < 0.5, rng.choice(["0", "A", "spine"]))


def _rand_prefix_db(rng, n=3):
    entries = []
    for i in range(n):
        e = T.createPrefixEntry(T.toIpPrefix(rng.choice([f"fc00:{i:x}::1/128", f"10.{i}.0.0/16"])))
        e.type = rng.choice([1, 2, 3, 4])
        e.forwardingType = rng.choice([0, 1])
        e.forwardingAlgorithm = rng.choice([0, 1])
        if rng.random() < 0.5:
            e.data = bytes(rng.randrange(256) for _ in range(rng.randrange(20)))
        if rng.random() < 0.5:
            e.ephemeral = rng.random() < 0.5
        if rng.random() < 0.5:
            e.minNexthop = rng.randint(0, 2**40)
        if rng.random() < 0.5:
            e.prependLabel = rng.randint(0, 2**20)
        if rng.random() < 0.5:
            e.mv = T.MetricVector(rng.randint(0, 9), [
                T.MetricEntity(rng.randint(0, 5), rng.randint(0, 5), rng.choice([1, 2, 3]),
                               rng.random() < 0.5, [rng.randint(-(2**50), 2**50) for _ in range(rng.randrange(17))])
                for _ in range(rng.randrange(3))])
        entries.append(e)
    db = T.createPrefixDb(f"node-{rng.randrange(1000)}", entries, rng.choice(["0", "A"]))
    db.deletePrefix = rng.random() < 0.2
    return db


def test_known_answer_bytes(E):
    # AdjacencyDatabase{thisNodeName="a", isOverloaded=false, adjacencies=[],
    # nodeLabel=0, area="0"} by the compact spec, fields in IDL order:
    #   18 01 61   field 1 (delta 1) binary "a"
    #   12         field 2 bool false (in the type nibble)
    #   19 0c      field 3 list, header: size 0, element type struct
    #   15 00      field 4 i32, zigzag(0)
    #   28 01 30   field 6 (delta 2) binary "0"
    #   00         stop
    want = bytes.fromhex("180161121 90c1500280130 00".replace(" ", ""))
    db = T.createAdjDb("a", [], 0, False, "0")
    assert E.compact_encode_adj_db(db) == want
    assert CW.encode_adj_db(db) == want
    assert E.compact_decode_adj_db(want) == db
    # one adjacency: field ids 3 -> 5 -> 4 (IDL order) use the long form for 4;
    # metric -1 zigzags to 01, weight 1 to 02
    a = T.Adjacency(otherNodeName="b", ifName="i", metric=-1)
    b = E.compact_encode_adj_db(T.createAdjDb("a", [a], 0, True, "0"))
    assert b[:3] == bytes.fromhex("180161") and b[3] == 0x11  # overloaded: bool true
    assert b[4:6] == bytes.fromhex("191c")  # list of 1 struct
    # otherNodeName "b", ifName "i", nextHopV6 {addr ""} (field 3), nextHopV4
    # (field 5, delta 2), then metric: field 4 after 5 -> long form 05 08, zz(-1) 01
    inner = bytes.fromhex("180162" "180169" "1c180000" "2c180000" "050801")
    assert b[6 : 6 + len(inner)] == inner
    assert E.compact_decode_adj_db(b).adjacencies[0] == a


@pytest.mark.parametrize("seed", range(25))
def test_adj_db_round_trips(E, seed):
    rng = random.Random(seed)
    db = _rand_adj_db(rng, n_adj=rng.choice([0, 1, 3, 14, 15, 40]))
    cpp = E.compact_encode_adj_db(db)
    assert cpp == CW.encode_adj_db(db)  # same bytes as the spec encoder
    assert CW.decode_adj_db(cpp) == db
    assert E.compact_decode_adj_db(cpp) == db
    # unknown fields (perfEvents, fields of later schema versions) are skipped
    assert E.compact_decode_adj_db(CW.encode_adj_db(db, junk=True)) == db


@pytest.mark.parametrize("seed", range(25))
def test_prefix_db_round_trips(E, seed):
    rng = random.Random(100 + seed)
    db = _rand_prefix_db(rng, n=rng.choice([0, 1, 4, 15, 20]))
    stacks = [[rng.choice(["A", "B", "0"]) for _ in range(rng.randrange(3))] for _ in db.prefixEntries]
    cpp = E.compact_encode_prefix_db(db, stacks)
    assert cpp == CW.encode_prefix_db(db, stacks)
    got, got_stacks, ppk = E.compact_decode_prefix_db(cpp)
    assert got == db and got_stacks == stacks and ppk is None
    got, got_stacks, ppk = E.compact_decode_prefix_db(CW.encode_prefix_db(db, stacks, junk=True,
                                                                          per_prefix_key=True))
    assert got == db and got_stacks == stacks and ppk is True


def test_malformed_blobs_raise(E):
    db = _rand_adj_db(random.Random(1), 5)
    b = E.compact_encode_adj_db(db)
    for cut in (1, 2, len(b) // 2, len(b) - 1):
        with pytest.raises(ValueError):
            E.compact_decode_adj_db(b[:cut])
    with pytest.raises(ValueError):
        E.compact_decode_adj_db(b + b"\x00")  # trailing bytes
    with pytest.raises(ValueError):
        E.compact_decode_adj_db(b"\x18\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\x01")  # bad varint
    with pytest.raises(ValueError):
        E.compact_decode_adj_db(b"\x1d" + b"\x00")  # unknown wire type 13
    with pytest.raises(ValueError):
        E.compact_decode_adj_db(b"\x45\x80\x80\x80\x80\x20\x00")  # nodeLabel = 2^32: not an i32
    # a mismatched type on a known id is skipped like an unknown field
    # (area has no IDL default, Lsdb.thrift:127: "" when absent)
    assert E.compact_decode_adj_db(b"\x15\x80\x80\x80\x80\x20\x00") == T.AdjacencyDatabase(area="")
    with pytest.raises(ValueError):  # unknown field 15 nesting 100 structs deep
        E.compact_decode_adj_db(b"\xfc" + b"\x1c" * 99 + b"\x00" * 100)


def test_prefix_key_parsing(E):
    assert E.parse_prefix_key("prefix:node-1:0:[fc00::1/128]") == (
        "node-1", "0", (T.toIpPrefix("fc00::1/128").prefixAddress.addr, 128))
    # createNetwork masks the host bits
    assert E.parse_prefix_key("prefix:a_b.c:A1:[10.1.2.3/8]")[2] == (bytes([10, 0, 0, 0]), 8)
    assert E.parse_prefix_key("prefix:a:0:[fd00:1:2:3::9/33]")[2] == (
        bytes.fromhex("fd000001") + bytes(12), 33)
    for bad in ("prefix:a:0:[10.0.0.0/33]", "prefix:a:0:[fc00::/129]", "prefix:a:0:[zz::/64]",
                "prefix:a", "prefix:a:0:[10.0.0.0/8", "prefix:a:0:[10.0.0.0/1234]",
                "prefix:a b:0:[10.0.0.0/8]", "prefix:a:0-1:[10.0.0.0/8]", "adj:a",
                "prefix:a:0:[10.0.0.0/8]x"):
        assert E.parse_prefix_key(bad) is None, bad
    assert E.get_node_name_from_key("adj:node-7") == "node-7"
    assert E.get_node_name_from_key("prefix:n:0:[fc00::/64]") == "n"
    assert E.get_node_name_from_key("nodelimiter") == ""


def _publish(E, ing, areas, ps, names, adj_dbs, prefix_dbs, seed):
    """Publish everything in KvStore-like batches (one publication per area,
    keys in random order, split into chunks)."""
    rng = random.Random(seed)
    last = None
    for area, dbs in adj_dbs.items():
        kv = {f"adj:{db.thisNodeName}": E.compact_encode_adj_db(db) for db in dbs}
        kv.update({f"prefix:{p.thisNodeName}": E.compact_encode_prefix_db(p)
                   for p in prefix_dbs if p.area == area})
        keys = list(kv)
        rng.shuffle(keys)
        for i in range(0, len(keys), 17):
            last = ing.processPublication(areas, ps, area, {k: kv[k] for k in keys[i:i + 17]})
    return last


def _canon(link):
    area, ends = link.toString().split(" - ", 1)
    return (area, tuple(sorted(ends.split(" <---> "))),
            tuple(sorted((link.getMetricFromNode(x), link.getOverloadFromNode(x))
                         for x in (link.firstNodeName(), link.secondNodeName()))))


@pytest.mark.parametrize("seed", range(3))
def test_publication_ingest_matches_object_path(E, seed):
    names, adj_dbs, prefix_dbs = RZ.random_network(900 + seed, n_nodes=25, n_links=60, areas=("A", "B"))
    oa, op = RZ.load(E, adj_dbs, prefix_dbs, 0)
    ba, bp = E.AreaLinkStates(), E.PrefixState()
    ing = E.PublicationIngest(names[0])
    pend = _publish(E, ing, ba, bp, names, adj_dbs, prefix_dbs, seed)
    assert pend["needsFullRebuild"] and pend["needsRouteUpdate"]
    assert bp.prefixes() == op.prefixes()
    assert sorted(ba.areas()) == sorted(oa.areas())
    for area in oa.areas():
        for n in names:
            assert ba[area].hasNode(n) == oa[area].hasNode(n)
            assert ba[area].isNodeOverloaded(n) == oa[area].isNodeOverloaded(n)
            # a Link keeps the side that completed it first (ingest order)
            assert sorted(map(_canon, ba[area].linksFromNode(n))) == sorted(
                map(_canon, oa[area].linksFromNode(n)))
        assert ba[area].numLinks() == oa[area].numLinks()


def test_publication_semantics(E):
    E.reset_counters()
    areas, ps = E.AreaLinkStates(), E.PrefixState()
    ing = E.PublicationIngest("me")
    a1 = T.createAdjacency("n2", "if12", "if21", "fe80::1", "10.0.0.1", 10, 50001)
    a2 = T.createAdjacency("n1", "if21", "if12", "fe80::2", "10.0.0.2", 10, 50002)
    kv = {"adj:n1": E.compact_encode_adj_db(T.createAdjDb("n1", [a1], 1, False, "X")),
          "adj:n2": E.compact_encode_adj_db(T.createAdjDb("n2", [a2], 2, False, "X"))}
    p = ing.processPublication(areas, ps, "A", kv)
    assert p["needsFullRebuild"] and p["count"] == 2
    assert areas.areas() == ["A"] and areas["A"].numLinks() == 1  # area from the publication
    assert E.get_counters()["decision.adj_db_update"] == 2
    # TTL refresh (no value) and an empty publication change nothing
    ing.resetPending()
    p = ing.processPublication(areas, ps, "A", {"adj:n1": None})
    assert p["count"] == 0 and not p["needsRouteUpdate"]
    # a corrupt blob is logged / counted and the other keys still apply
    pe = T.createPrefixEntry(T.toIpPrefix("fc00::1/128"))
    p = ing.processPublication(areas, ps, "A", {
        "adj:n1": b"\x18\x05ab", "prefix:n1": E.compact_encode_prefix_db(T.createPrefixDb("n1", [pe], "A"))})
    assert E.get_counters()["decision.publication_decode_errors"] == 1
    key = (pe.prefix.prefixAddress.addr, 128)
    assert p["updatedPrefixes"] == {key}
    # per-prefix key for another prefix merges with the full db; per-prefix wins
    pe2 = T.createPrefixEntry(T.toIpPrefix("fc00::2/128"))
    ing.resetPending()
    p = ing.processPublication(areas, ps, "A", {
        "prefix:n1:A:[fc00::2/128]": E.compact_encode_prefix_db(T.createPrefixDb("n1", [pe2], "A"))})
    assert set(ps.prefixes()) == {key, (pe2.prefix.prefixAddress.addr, 128)}
    # expiring the per-prefix key withdraws only that prefix
    p = ing.processPublication(areas, ps, "A", {}, ["prefix:n1:A:[fc00::2/128]"])
    assert set(ps.prefixes()) == {key}
    # self-originated re-distribution (area_stack[0] is one of my areas) is ignored
    pe3 = T.createPrefixEntry(T.toIpPrefix("fc00::3/128"))
    ing.processPublication(areas, ps, "A", {
        "prefix:me:A:[fc00::3/128]": E.compact_encode_prefix_db(T.createPrefixDb("me", [pe3], "A"), [["A"]])})
    assert set(ps.prefixes()) == {key}
    ing.processPublication(areas, ps, "A", {
        "prefix:me:A:[fc00::3/128]": E.compact_encode_prefix_db(T.createPrefixDb("me", [pe3], "A"), [["Z"]])})
    assert set(ps.prefixes()) == {key, (pe3.prefix.prefixAddress.addr, 128)}
    # expired adj key deletes the node's adjacencies
    ing.resetPending()
    p = ing.processPublication(areas, ps, "A", {}, ["adj:n2"])
    assert p["needsFullRebuild"] and areas["A"].numLinks() == 0
    # key / payload node mismatch is a reference CHECK (fatal): raised, not swallowed
    with pytest.raises(RuntimeError):
        ing.processPublication(areas, ps, "A", {"adj:n9": kv["adj:n1"]})


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(2))
def test_route_db_after_byte_ingest_gpu(gpu_ready, seed):
    import openr_amd._openr_spf as E
    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    names, adj_dbs, prefix_dbs = RZ.random_network(950 + seed, n_nodes=30, n_links=70)
    ba, bp = E.AreaLinkStates(), E.PrefixState()
    ing = E.PublicationIngest(names[0])
    # A LinkSet's iteration order (and with it KSP2's choice among parallel
    # links) depends on the order links were created, in the reference too.
    # So publish one key per publication, in the order RZ.load feeds the
    # oracle, rather than in a multi-key publication's hash order.
    rng = random.Random(seed)
    for area, dbs in adj_dbs.items():
        order = list(dbs)
        rng.shuffle(order)
        for db in order:
            ing.processPublication(ba, bp, area, {f"adj:{db.thisNodeName}": E.compact_encode_adj_db(db)})
    for p in prefix_dbs:
        ing.processPublication(ba, bp, p.area, {f"prefix:{p.thisNodeName}": E.compact_encode_prefix_db(p)})
    oa, op = RZ.load(O, adj_dbs, prefix_dbs, seed)
    es = E.SpfSolver(names[0], True, True)
    os_ = O.SpfSolver(names[0], True, True)
    for node in names:
        a, b = es.buildRouteDb(node, ba, bp), os_.buildRouteDb(node, oa, op)
        if a != b:
            diff = {kind: sorted(k for k in set(a[kind]) | set(b[kind]) if a[kind].get(k) != b[kind].get(k))
                    for kind in a}
            pytest.fail(f"{node}: differing keys {diff}; first: "
                        f"{[(a[k].get(x), b[k].get(x)) for k, v in diff.items() for x in v[:1]]}")


@pytest.mark.gpu
def test_ordered_fib_holds_after_byte_ingest_gpu(gpu_ready):
    """enable_ordered_fib_programming: processPublication derives holdUp /
    holdDown TTLs from hop counts of the current LinkState (Decision.cpp:
    1670-1680).  The oracle gets the same TTLs from its own hop queries; the
    hold state and every RouteDb must match while the holds drain."""
    import openr_amd._openr_spf as E
    from oracle import build as obuild

    obuild.build()
    from oracle import _oracle_ref as O

    names, adj_dbs, prefix_dbs = RZ.random_network(977, n_nodes=24, n_links=50, parallel_prob=0.0)
    me = names[0]
    ba, bp = E.AreaLinkStates(), E.PrefixState()
    ing = E.PublicationIngest(me, True)
    rng = random.Random(3)
    order = list(adj_dbs["0"])
    rng.shuffle(order)
    oa = O.AreaLinkStates()
    ols = oa.add("0")
    for db in order:
        up = down = 0
        h = ols.getHopsFromAToB(me, db.thisNodeName)
        if h is not None:
            up = h
            down = ols.getMaxHopsToNode(db.thisNodeName) - h
        ols.updateAdjacencyDatabase(db, up, down)
        ing.processPublication(ba, bp, "0", {f"adj:{db.thisNodeName}": E.compact_encode_adj_db(db)})
    op = O.PrefixState()
    for p in prefix_dbs:
        op.updatePrefixDatabase(p)
        ing.processPublication(ba, bp, p.area, {f"prefix:{p.thisNodeName}": E.compact_encode_prefix_db(p)})
    # churn: raise one link's metric on both ends -> holds
    def ttls(db):
        h = ols.getHopsFromAToB(me, db.thisNodeName)
        return (h, ols.getMaxHopsToNode(db.thisNodeName) - h) if h is not None else (0, 0)

    # a reachable node whose hold-down TTL is positive: a metric increase
    # ("bringing down") is then held for that many decrements
    victim = next(db for db in order if db.adjacencies and ttls(db)[1] > 0)
    victim.adjacencies[0].metric += 7
    up, down = ttls(victim)
    ols.updateAdjacencyDatabase(victim, up, down)
    assert ols.hasHolds()
    ing.processPublication(ba, bp, "0", {f"adj:{victim.thisNodeName}": E.compact_encode_adj_db(victim)})
    es = E.SpfSolver(me, True, False)
    os_ = O.SpfSolver(me, True, False)
    for _ in range(8):
        assert ba["0"].hasHolds() == ols.hasHolds()
        for node in names[:6]:
            assert es.buildRouteDb(node, ba, bp) == os_.buildRouteDb(node, oa, op), node
        if not ols.hasHolds():
            break
        ba["0"].decrementHolds()
        ols.decrementHolds()
