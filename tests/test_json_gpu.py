"""GPU: the Maelstrom Deps JSON (Json.DEPS_ADAPTER, accord-maelstrom/.../Json.java:316-398) parsed and written on device
(acc_deps_from_json / acc_deps_to_json): canonical documents round-trip byte for byte, unsorted documents with
duplicates come back as the Builder result, the parsed keys carry Datum.compareTo order (hash first); every datum kind
(LONG, HASH, STRING with escapes, DOUBLE through Double.parseDouble / Double.toString) against the test-side model
(tests/json_cases.py: a restatement of Gson's writer, Double.toString by exact rationals)."""
import struct
import numpy as np
import pytest

import json_cases as JC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def test_json_round_trip_canonical(ctx):
    from accord_amd.deps import deps_from_json, deps_to_json
    rng = np.random.default_rng(1)
    docs = [JC.write_deps(*JC.random_doc(rng, canonical=True)) for _ in range(300)]
    docs.append(b'{"keyDeps":[],"rangeDeps":[]}')
    r = deps_from_json(ctx, docs, with_view=True)
    out = deps_to_json(ctx, r["view"])
    assert out == docs


def test_json_builder_semantics(ctx):
    from accord_amd.deps import deps_from_json, deps_to_json
    rng = np.random.default_rng(2)
    raw = [JC.random_doc(rng) for _ in range(200)]
    docs = [JC.write_deps(*x) for x in raw]
    # whitespace, field order and a missing field are accepted like Gson's JsonReader
    docs.append(b' { "rangeDeps" : [ ] , "keyDeps" : [ [ 5 , [ 1 , 65538 , "n2" ] ] , [ 3 , [ 1 , 65538 , null ] ] ] } ')
    raw.append(([((JC.LONG, False, 5), (1, 65538, 2)), ((JC.LONG, False, 3), (1, 65538, 0))], []))
    docs.append(b'{}')
    raw.append(([], []))
    r = deps_from_json(ctx, docs, with_view=True)
    out = deps_to_json(ctx, r["view"])
    for i, (ke, re_) in enumerate(raw):
        assert out[i] == JC.write_deps(*JC.build(ke, re_)), i
    # dictionary = the batch's distinct datums in Datum.compareTo order
    seen = {JC.datum_order(d) for ke, re_ in raw for d, _ in ke} | \
           {JC.datum_order(x) for ke, re_ in raw for (a, b), _ in re_ for x in (a, b)}
    assert len(r["dict_kind"]) == len(seen)
    got = [JC.datum_order(dict_datum(r, i)) for i in range(len(r["dict_kind"]))]
    assert got == sorted(seen)
    assert [int(h) for h in r["dict_hash"]] == [g[0] for g in got]


def dict_datum(r, i):
    """(kind, null, value) of dictionary rank i of a deps_from_json result"""
    k, nl, v = int(r["dict_kind"][i]), bool(r["dict_null"][i]), int(r["dict_value"][i])
    if nl:
        return (k, True, 0)
    if k == JC.LONG:
        return (k, False, v - (1 << 64) if v >= 1 << 63 else v)
    if k == JC.HASH:
        return (k, False, int(np.int32(np.uint32(v & 0xFFFFFFFF))))
    if k == JC.DOUBLE:
        return (k, False, struct.unpack(">d", struct.pack(">Q", v))[0])
    n = int(r["dict_len"][i])
    return (k, False, bytes(r["dict_str"][v:v + n]).decode("ascii"))


@pytest.mark.parametrize("p_string,p_double", [(0.6, 0.0), (0.0, 0.6), (0.3, 0.3)])
def test_json_strings_and_doubles(ctx, p_string, p_double):
    """Canonical documents with STRING (escapes incl. Gson's HTML-safe ones) and DOUBLE datums round-trip byte for byte;
    unsorted ones come back as the Builder result; the dictionary is in Datum.compareTo order with the reference's
    hashes (String.hashCode / Double.hashCode through CRC32)."""
    from accord_amd.deps import deps_from_json, deps_to_json
    rng = np.random.default_rng(int(p_string * 10 + p_double * 100))
    canon = [JC.write_deps(*JC.random_doc(rng, canonical=True, p_string=p_string, p_double=p_double)) for _ in range(150)]
    r = deps_from_json(ctx, canon, with_view=True)
    assert deps_to_json(ctx, r["view"]) == canon
    raw = [JC.random_doc(rng, p_string=p_string, p_double=p_double) for _ in range(150)]
    r = deps_from_json(ctx, [JC.write_deps(*x) for x in raw], with_view=True)
    out = deps_to_json(ctx, r["view"])
    for i, (ke, re_) in enumerate(raw):
        assert out[i] == JC.write_deps(*JC.build(ke, re_)), i
    got = [JC.datum_order(dict_datum(r, i)) for i in range(len(r["dict_kind"]))]
    assert got == sorted(got) and len(set(got)) == len(got)
    assert [int(h) for h in r["dict_hash"]] == [g[0] for g in got]


def test_json_number_forms(ctx):
    """Numbers as Datum.read takes them (JsonReader.nextLong, else nextDouble): integral literals in any form are LONG
    ("1.0", "1e2", "-0"), Long overflow goes through the double ("9223372036854775808" -> DOUBLE 9.223372036854776E18,
    Java's (long) d == d quirk at 2^63 keeps "9.223372036854775807E18" a LONG), others DOUBLE exactly rounded
    (Double.parseDouble); escaped strings are unescaped."""
    from accord_amd.deps import deps_from_json, deps_to_json
    lits = [b"1.0", b"1e2", b"-0", b"-0.0", b"9223372036854775807", b"9223372036854775808", b"9.223372036854775807E18",
            b"0.1", b"1.5", b"-2.5e-3", b"123456789012345678e-20", b"4.9E-324", b"2.2250738585072014E-308",
            b"1.7976931348623157E308", b"17976931348623157e292", b"0.30000000000000004", b"\"a\\u003cb\\n\\\"c\""]
    docs = [b'{"keyDeps":[[' + x + b',[1,2,"n1"]]],"rangeDeps":[]}' for x in lits]
    r = deps_from_json(ctx, docs, with_view=True)
    out = deps_to_json(ctx, r["view"])
    def java(x: bytes):
        t = x.decode()
        if t.startswith('"'):
            return JC.gson_string(__import__("json").loads(t))
        if all(c.isdigit() or c == "-" for c in t):
            v = int(t)
            if -(1 << 63) <= v < (1 << 63) and t != "-0":
                return str(v)
        d = float(t)
        ll = max(-(1 << 63), min((1 << 63) - 1, int(d))) if abs(d) < float("inf") else 0
        if float(ll) == d:
            return str(ll)
        return JC.java_double_to_string(d)
    for x, o in zip(lits, out):
        assert o == ('{"keyDeps":[[' + java(x) + ',[1,2,"n1"]]],"rangeDeps":[]}').encode(), (x, o)


def test_json_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException, deps_from_json
    bad = [b'{"keyDeps":[[1,[1,2,"n1"]]', b'{"keyDeps":[["s\xc3\xa9",[1,2,"n1"]]]}', b'{"keyDeps":[[1e400,[1,2,"n1"]]]}',
           b'{"keyDeps":[[1,null]]}', b'{"keyDeps":[[1,[1,2,"x1"]]]}', b'{"keyDeps":[[1,[1,2,"n99999999999"]]]}',
           b'{"keyDeps":[[01,[1,2,"n1"]]]}']
    for doc in bad:
        with pytest.raises(IllegalArgumentException):
            deps_from_json(ctx, [doc])
    with pytest.raises(IllegalStateException):
        deps_from_json(ctx, [b'{"other":[]}'])
    # document offsets outside the byte buffer are rejected before any document is parsed
    import ctypes as C
    from accord_amd import _lib as L
    blob = np.frombuffer(b'{"keyDeps":[],"rangeDeps":[]}', np.uint8).copy()
    for offs in ([0, 40], [5, 30], [0, 20, 10]):
        off = np.array(offs, np.uint64)
        ji = L.JsonIn(L.ACC_MEM_HOST, len(offs) - 1, blob.ctypes.data, off.ctypes.data)
        rc = ctx._lib.acc_deps_from_json(ctx.handle, C.byref(ji), C.byref(L.JsonDepsView()))
        assert rc == L.ACC_E_ARG, offs
    # the context stays usable
    r = deps_from_json(ctx, [b'{"keyDeps":[[7,[1,2,"n1"]]],"rangeDeps":[]}'])
    assert int(r["key"]["key_off"][-1]) == 1
