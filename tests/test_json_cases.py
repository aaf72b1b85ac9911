"""CPU: the test-side JSON writer reproduces the reference's byte forms (Datum.write, Json.writeTimestamp, toString(Id))
and Datum.hash; no GPU."""
import json

import json_cases as JC


def test_writer_forms():
    doc = JC.write_deps([((JC.LONG, False, -7), (32768, 327682, 1)), ((JC.HASH, False, -3), (1, 2, 0)),
                         ((JC.HASH, True, 0), (1, 2, -4)), ((JC.LONG, True, 0), ((1 << 64) - 1, 2, 3))],
                        [(((JC.LONG, False, 1), (JC.LONG, False, 9)), (1, 2, 5))])
    assert doc == (b'{"keyDeps":[[-7,[32768,327682,"n1"]],[["HASH",true,-3],[1,2,null]],[["HASH",false],[1,2,"c-4"]],'
                   b'[["LONG"],[-1,2,"n3"]]],"rangeDeps":[[1,9,[1,2,"n5"]]]}')
    json.loads(doc)


def test_datum_hash_and_order():
    # hash(null) = Integer.MAX_VALUE sorts null datums last; a Hash datum's hash is itself
    assert JC.datum_hash(JC.LONG, True, 0) == 0x7FFFFFFF
    assert JC.datum_hash(JC.HASH, False, -5) == -5
    assert JC.datum_order((JC.HASH, False, 0x7FFFFFFF)) < JC.datum_order((JC.HASH, True, 0))
    vals = [JC.datum_hash(JC.LONG, False, v) for v in range(1000)]
    assert len(set(vals)) == 1000 and sorted(vals) != vals   # hash order, not value order


def test_java_double_to_string():
    # Double.toString (JDK >= 19: shortest digits that round-trip; sci form outside [1e-3, 1e7))
    cases = [(0.0, "0.0"), (-0.0, "-0.0")] + list({1.0: "1.0", 0.1: "0.1", 1e7: "1.0E7", 9999999.0: "9999999.0", 0.001: "0.001",
             0.0009: "9.0E-4", 5e-324: "4.9E-324", 2e23: "2.0E23", 1e22: "1.0E22", 12345678.9: "1.23456789E7",
             1.7976931348623157e308: "1.7976931348623157E308", 2.2250738585072014e-308: "2.2250738585072014E-308",
             0.30000000000000004: "0.30000000000000004", -2.5e-3: "-0.0025", 100.0: "100.0", 123.456: "123.456"}.items())
    for x, want in cases:
        assert JC.java_double_to_string(x) == want, (x, JC.java_double_to_string(x))
    import numpy as np
    rng = np.random.default_rng(5)
    for _ in range(2000):
        x = JC.random_double(rng)
        s = JC.java_double_to_string(x)
        assert float(s) == x            # round trips
        m = s.lstrip("-").split("E")[0].replace(".", "").strip("0")
        assert len(m) <= 17


def test_gson_string():
    # JsonWriter.string with htmlSafe: <, >, &, =, ' as \u00XX; quote, backslash, control chars escaped
    assert JC.gson_string('a<b"\\\n') == '"a\\u003cb\\"\\\\\\n"'
    assert JC.gson_string("x>y&z='w'") == '"x\\u003ey\\u0026z\\u003d\\u0027w\\u0027"'
    assert JC.gson_string("\t\x01/") == '"\\t\\u0001/"'
    import json
    for t in ["", "abc", "a\"b", "q\\\n\r\b\f", "<>&='"]:
        assert json.loads(JC.gson_string(t)) == t
