"""Number formatting of the summary hosts against ECMAScript JSON.stringify.

Map values, prop values and computed annotate-adjust numbers reach the summaries as JSON text. The
reference writes them with JSON.stringify (serializer.ts:120-123 over ECMAScript Number::toString,
ECMA-262 §6.1.6.1.20): decimal form for 1e-7 <= |x| < 1e21, exponents without zero padding, -0 as 0,
and NaN / Infinity as null. The Python host (streams.js_number) must write the same bytes as the
image's Node (the JS host) and as libfmt's C++ formatter (fmt_internal_js_number).
"""
import ctypes
import json
import os
import random
import shutil
import struct
import subprocess

import pytest

from fluidframework_amd.streams import js_json, js_number

NODE = shutil.which("node")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

EDGES = [1e-5, 1.5e-5, 1e-7, 2.5e-8, 1e21, 1e20, 9.999999999999999e20, 5e-324, -0.0, 0.0, 0.1 + 0.2, 123.456,
         1.7976931348623157e308, 1e-6, 1.234e-6, 9.99e-7, 100.0, -2.5, 0.5, 2.0 ** 53, 2.0 ** 53 + 2, -1e-7, 1e300,
         2.2250738585072014e-308, 4.9406564584124654e-324, 123456789012345680000.0, 0.1, 1 / 3, 7.0, -7e22]


def _values():
    rng = random.Random(1234)
    vals = list(EDGES)
    for _ in range(1500):  # random finite doubles, every exponent
        bits = rng.getrandbits(64)
        x = struct.unpack("<d", struct.pack("<Q", bits))[0]
        if x == x and abs(x) != float("inf"):
            vals.append(x)
    for _ in range(1500):  # short decimals around the 1e-7 and 1e21 switch points
        vals.append(round(rng.uniform(-1, 1), rng.randint(0, 12)) * 10.0 ** rng.randint(-12, 24))
    return vals


def _node_strings(vals, tmp_path):
    f = tmp_path / "bits.json"
    f.write_text(json.dumps([struct.pack("<d", v).hex() for v in vals]))
    js = ("const hex=JSON.parse(require('fs').readFileSync(process.argv[1],'utf8'));"
          "console.log(JSON.stringify(hex.map(h=>JSON.stringify(Buffer.from(h,'hex').readDoubleLE(0)))));")
    r = subprocess.run([NODE, "-e", js, str(f)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.skipif(NODE is None, reason="node is not installed")
def test_python_number_format_equals_json_stringify(tmp_path):
    vals = _values()
    want = _node_strings(vals, tmp_path)
    got = [js_number(v) for v in vals]
    bad = [(v, g, w) for v, g, w in zip(vals, got, want) if g != w]
    assert not bad, bad[:10]


def test_python_number_format_edge_values():
    assert [js_number(x) for x in (1e-5, 1.5e-5, 1e-7, 1e21, 5e-324, -0.0, 0.1 + 0.2)] == [
        "0.00001", "0.000015", "1e-7", "1e+21", "5e-324", "0", "0.30000000000000004"]
    assert js_number(float("inf")) == "null" and js_number(float("nan")) == "null"
    # JSON.parse reads every number as a double
    assert js_json(12345678901234567890) == "12345678901234567000"
    assert js_json(json.loads('{"a":1.0e-5,"b":[2.50,-0.0]}')) == '{"a":0.00001,"b":[2.5,0]}'


def test_cpp_number_format_equals_python():
    lib = ctypes.CDLL(os.path.join(REPO, "fluidframework_amd", "libfmt.so"))
    fn = lib.fmt_internal_js_number
    fn.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    buf = ctypes.create_string_buffer(64)
    vals = _values() + [float("inf"), float("-inf"), float("nan")]
    bad = []
    for v in vals:
        n = fn(v, buf, 64)
        got = buf.raw[:n].decode()
        if got != js_number(v):
            bad.append((v, got, js_number(v)))
    assert not bad, bad[:10]
