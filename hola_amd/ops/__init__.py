"""Python API over the native core operations (the exact C++ code the server runs, via the
in-tree pybind11 module ``hola_amd._native``).

    >>> from hola_amd import ops
    >>> ops.java_format("Hola de %s", "h")
    'Hola de h'
    >>> ops.parse_properties("hello=Hola de %s\\\\n")["hello"]
    'Hola de %s\\n'
"""
from __future__ import annotations

from hola_amd.native import load_native


class JavaFormatError(ValueError):
    """A java.util.Formatter exception (e.g. IllegalFormatConversionException)."""

    def __init__(self, exception: str, detail: str):
        super().__init__(f"{exception}: {detail}")
        self.exception = exception
        self.detail = detail


def parse_properties(text: str | bytes) -> dict[str, str]:
    """java.util.Properties.load semantics; raises ValueError on a malformed \\uXXXX escape."""
    data = text.encode() if isinstance(text, str) else text
    r = load_native().parse_properties(data)
    if not r["ok"]:
        raise ValueError(r["error"])
    return {k.decode(): v.decode() for k, v in r["map"].items()}


def java_format(fmt: str, *args: str) -> str:
    """String.format with String arguments; raises JavaFormatError like the JVM would."""
    r = load_native().java_format(fmt, list(args))
    if isinstance(r, tuple):
        raise JavaFormatError(*r)
    return r.decode()


def accepts(accept: str, media_type: str) -> bool:
    """Does an Accept header admit `media_type` (e.g. "text/plain")? (JAX-RS 406 check)"""
    t, _, st = media_type.partition("/")
    return load_native().accepts(accept, t, st)


def b3_extract(headers: dict[str, str]) -> dict | str:
    """Brave-3 server-side B3 extraction from request headers (case-insensitive keys).
    Returns the span context dict, or "none" / "not_sampled"."""
    h = {k.lower(): v for k, v in headers.items()}
    return load_native().b3_extract(trace_id=h.get("x-b3-traceid", ""), span_id=h.get("x-b3-spanid", ""),
                                     parent_id=h.get("x-b3-parentspanid", ""), sampled=h.get("x-b3-sampled", ""),
                                     flags=h.get("x-b3-flags", ""), single=h.get("b3", ""))


def decode_string_list(body: str | bytes) -> list[str | None]:
    """Jackson-style List<String> binding of a JSON document; raises ValueError."""
    data = body.encode() if isinstance(body, str) else body
    r = load_native().decode_string_list(data)
    if isinstance(r, tuple):
        raise ValueError(r[1])
    return [None if x is None else x.decode() for x in r]


def resolve(sources: list[tuple[str, int, dict[str, str]]], key: str, default: str) -> tuple[str, str]:
    """DeltaSpike-style ordinal resolution; returns (value, source name)."""
    value, source, _, _ = load_native().resolve(sources, key, default)
    return value, source
