"""`String.format(translation, hostname)` (HolaResource.java:65) via the native formatter.

Expected values/exception names are those of java.util.Formatter (Java 8) for a single
java.lang.String argument.
"""
import pytest


def fmt(native, f, *args):
    return native.java_format(f, list(args))


@pytest.mark.parametrize("f,expected", [
    ("Hola de %s", b"Hola de h"),
    ("%s", b"h"),
    ("no placeholder", b"no placeholder"),
    ("%S", b"H"),
    ("[%5s]", b"[    h]"),
    ("[%-5s]", b"[h    ]"),
    ("[%.0s]", b"[]"),
    ("%1$s %1$s", b"h h"),
    ("%s %<s", b"h h"),
    ("100%%", b"100%"),
    ("a%nb", b"a\nb"),
    ("%b", b"true"),
    ("%B", b"TRUE"),
    ("[%3%]", b"[  %]"),
])
def test_conversions(native, f, expected):
    assert fmt(native, f, "h") == expected


def test_hashcode_conversion(native):
    # Integer.toHexString("h".hashCode()) == "68"; "hola".hashCode() == 3208380 == 0x30f4bc
    assert fmt(native, "%h", "h") == b"68"
    assert fmt(native, "%h", "hola") == b"30f4bc"
    assert native.java_string_hash("hola") == 3208380
    for s in ("señor", "😀x", "a" * 40):
        assert native.java_string_hash(s) == java_hash(s)


def java_hash(s: str) -> int:
    h = 0
    for unit in s.encode("utf-16-be").hex(" ", 2).split():
        h = (31 * h + int(unit, 16)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def test_precision_and_width_count_utf16_units(native):
    assert fmt(native, "[%3s]", "é") == "[  é]".encode()
    assert fmt(native, "[%.1s]", "éa") == "[é]".encode()
    assert fmt(native, "%S", "señor") == "SEÑOR".encode()


@pytest.mark.parametrize("f,exc", [
    ("%d", "IllegalFormatConversionException"),
    ("%x", "IllegalFormatConversionException"),
    ("%f", "IllegalFormatConversionException"),
    ("%c", "IllegalFormatConversionException"),
    ("%tH", "IllegalFormatConversionException"),
    ("%s %s", "MissingFormatArgumentException"),
    ("%2$s", "MissingFormatArgumentException"),
    ("%<s", "MissingFormatArgumentException"),
    ("%q", "UnknownFormatConversionException"),
    ("trailing %", "UnknownFormatConversionException"),
    ("%-s", "MissingFormatWidthException"),
    ("%#s", "FormatFlagsConversionMismatchException"),
    ("%+s", "FormatFlagsConversionMismatchException"),
    ("%5n", "IllegalFormatWidthException"),
    ("%.2%", "IllegalFormatPrecisionException"),
    ("%--5s", "DuplicateFormatFlagsException"),
    ("%99999999999s", "IllegalFormatWidthException"),  # past Integer.MAX_VALUE: MIN_VALUE
    ("%.3000000000s", "IllegalFormatPrecisionException"),
    ("%100000000s", "OutOfMemoryError"),  # the JVM's -Xmx512m heap; bounded here (32 Mi units)
    ("%20000000s%1$20000000s", "OutOfMemoryError"),
])
def test_exceptions(native, f, exc):
    r = fmt(native, f, "h")
    assert isinstance(r, tuple) and r[0] == exc


def test_width_overflow_detail_and_large_but_bounded_widths(native):
    assert fmt(native, "%99999999999s", "h") == ("IllegalFormatWidthException", "-2147483648")
    out = fmt(native, "%1000000s", "h")
    assert isinstance(out, bytes) and len(out) == 1000000 and out.endswith(b" h")


def test_format_error_is_500(hola, tmp_path):
    conf = tmp_path / "t.properties"
    conf.write_text("hello=Hola %d\n")
    s = hola(args=[f"-Dconf={conf}"])
    st, h, body = s.get("/api/hola")
    assert st == 500 and b"Internal Server Error" in body
    assert "access-control-allow-origin" not in h  # filters do not run for unhandled exceptions
    assert s.get("/api/health")[0] == 200
