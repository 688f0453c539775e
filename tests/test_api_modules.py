"""hola_amd.ops (Python API over the native core) and hola_amd.models (the contract as data)."""
import pytest

from hola_amd import ops
from hola_amd.models import FALLBACK_GREETING, ROUTES, swagger_spec


def test_ops_roundtrip():
    assert ops.java_format("Hola de %s", "h") == "Hola de h"
    with pytest.raises(ops.JavaFormatError) as e:
        ops.java_format("%d", "h")
    assert e.value.exception == "IllegalFormatConversionException"
    assert ops.parse_properties("hello=Hola de %s\\n")["hello"] == "Hola de %s\n"
    with pytest.raises(ValueError):
        ops.parse_properties("k=\\uZZZZ")
    assert ops.accepts("text/*", "text/plain") and not ops.accepts("application/json", "text/plain")
    assert ops.b3_extract({"X-B3-Sampled": "0"}) == "not_sampled"
    assert ops.decode_string_list('["a", null]') == ["a", None]
    assert ops.resolve([("Env", 300, {"hello": "x %s"}), ("File", 0, {"hello": "y %s"})], "hello", "d") == \
        ("x %s", "Env")


def test_contract_matches_running_server(hola):
    s = hola(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none"], env={"HOSTNAME": "h"})
    for r in ROUTES:
        if r.path == "/hystrix.stream":
            continue
        st, h, _ = s.get(r.path)
        assert st == 200, r.path
        assert h["content-type"].split(";")[0] == r.produces, r.path
        assert ("access-control-allow-origin" in h) == r.cors, r.path
    assert s.get("/api/hola-chaining")[2].decode().endswith(f'"{FALLBACK_GREETING}"]')
    documented = {"/api" + p for p in swagger_spec()["paths"]}
    assert documented <= {r.path for r in ROUTES}
