"""java.util.Properties.load grammar (Configuration.java:29) via the native parser.

Expected values follow the Java 8 Properties/LineReader rules (the reference JVM); no JVM is
available here, so each case states the rule it pins.
"""
from pathlib import Path

from hypothesis import given, settings, strategies as st

ROOT = Path(__file__).resolve().parent.parent


def parse(native, text):
    r = native.parse_properties(text.encode() if isinstance(text, str) else text)
    return r["ok"], {k.decode(): v.decode() for k, v in r["map"].items()}


def test_translation_properties_trailing_newline(native):
    ok, m = parse(native, (ROOT / "translation.properties").read_bytes())
    assert ok
    assert m["hello"] == "Hola de %s mediante el archivo de configuraciones\n"


def test_separators(native):
    ok, m = parse(native, "a=1\nb:2\nc 3\nd = 4\ne : 5\nf\t6\ng =: 7\nh\n i\n")
    assert m == {"a": "1", "b": "2", "c": "3", "d": "4", "e": "5", "f": "6", "g": ": 7", "h": "", "i": ""}


def test_comments_and_blank_lines(native):
    ok, m = parse(native, "# c\n! also\n\n   \n  # indented comment\nk=v # not a comment\n")
    assert m == {"k": "v # not a comment"}


def test_comment_line_is_not_continued(native):
    ok, m = parse(native, "# comment \\\nk=v\n")
    assert m == {"k": "v"}


def test_continuation(native):
    ok, m = parse(native, "k = a \\\n    b\\\n\tc\nx=1\n")
    assert m == {"k": "a bc", "x": "1"}


def test_even_backslashes_do_not_continue(native):
    ok, m = parse(native, "k=a\\\\\nx=1\n")
    assert m == {"k": "a\\", "x": "1"}


def test_continuation_then_empty_line(native):
    ok, m = parse(native, "k=a\\\n\nx=1\n")
    assert m == {"k": "a", "x": "1"}


def test_escapes(native):
    ok, m = parse(native, r"k=\t\n\r\f\\\=\:\ \q" + "\n")
    assert m["k"] == "\t\n\r\f\\=: q"


def test_escaped_separator_in_key(native):
    ok, m = parse(native, "a\\=b=c\nd\\ e f\n")
    assert m == {"a=b": "c", "d e": "f"}


def test_unicode_escapes(native):
    ok, m = parse(native, "k=\\u00e9t\\u00E9 \\ud83d\\ude00\n")
    assert m["k"] == "été 😀"


def test_malformed_unicode_fails_whole_file(native):
    # Properties.load throws IllegalArgumentException; Configuration.java:34-36 swallows it
    # and returns an empty map.
    r = native.parse_properties(b"a=1\nk=\\u12G4\n")
    assert not r["ok"] and r["map"] == {} and "Malformed" in r["error"]


def test_crlf_and_cr_line_endings(native):
    ok, m = parse(native, "a=1\r\nb=2\rc=3\r\nd=x\\\r\n  y\r\n")
    assert m == {"a": "1", "b": "2", "c": "3", "d": "xy"}


def test_last_duplicate_wins(native):
    ok, m = parse(native, "k=1\nk=2\n")
    assert m == {"k": "2"}


def test_no_trailing_newline_and_trailing_backslash_at_eof(native):
    ok, m = parse(native, "k=v\\")
    assert m == {"k": "v"}


def test_utf8_passthrough(native):
    ok, m = parse(native, "saludo=¡Hola, señor %s!\n")
    assert m["saludo"] == "¡Hola, señor %s!"


_key = st.text(alphabet=st.characters(min_codepoint=0x21, max_codepoint=0x7e, blacklist_characters="\\#!=: "),
               min_size=1, max_size=12)
_val = st.text(alphabet=st.characters(min_codepoint=0x20, max_codepoint=0x7e, blacklist_characters="\\"), max_size=30)


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(_key, _val, max_size=8))
def test_roundtrip_simple_pairs(native, d):
    text = "".join(f"{k}={v}\n" for k, v in d.items())
    ok, m = parse(native, text)
    assert ok
    assert m == {k: v.lstrip(" ") for k, v in d.items()}


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=300))
def test_fuzz_never_crashes(native, data):
    r = native.parse_properties(data)
    assert isinstance(r["ok"], bool)
