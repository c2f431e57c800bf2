"""Text codecs: RFC-4180 delimited text with backslash escapes, PMML space-delimited lists, JSON.

Behavioral equivalent of ``TextUtils`` (``[common]/text/TextUtils.java:56-187``): commons-csv
``RFC4180.withEscape('\\\\')`` parsing/printing semantics (MINIMAL quoting), the PMML variant
that escapes quotes as ``\\"`` and drops empty tokens, and JSON array helpers.  Also
``MLFunctions.PARSE_FN`` (``[app-common]/common/fn/MLFunctions.java:39-53``): a line that
starts with ``[`` and ends with ``]`` is a JSON array, anything else CSV.
"""

from __future__ import annotations

import json
import math
from typing import Any, Iterable, List, Optional

import numpy as np

__all__ = ["parse_delimited", "parse_pmml_delimited", "join_delimited", "join_pmml_delimited",
           "join_pmml_delimited_numbers", "parse_json_array", "join_json", "read_json",
           "parse_input_line", "java_float_str", "java_double_str", "format_number"]

_ESC_MAP = {"r": "\r", "n": "\n", "t": "\t", "b": "\b", "f": "\f"}


def _read_escape(s: str, i: int, delim: str):
    """Character after a backslash at s[i-1]; returns (text, new_index)."""
    if i >= len(s):
        return "\\", i
    c = s[i]
    if c in _ESC_MAP:
        return _ESC_MAP[c], i + 1
    if c in ("\\", '"', delim, "\r", "\n", "\t", "\b", "\f"):
        return c, i + 1
    # commons-csv drops the escape for non-meta chars only when they are meta; keep both
    return "\\" + c, i + 1


def parse_delimited(line: str, delimiter: str = ",") -> List[str]:
    """Parse one record; an empty line yields ``[""]`` like the reference."""
    if line == "":
        return [""]
    if '"' not in line and "\\" not in line:
        return line.split(delimiter)      # no quoting or escapes: plain split is exact
    out: List[str] = []
    i, n = 0, len(line)
    while True:
        buf = []
        if i < n and line[i] == '"':
            i += 1
            while i < n:
                c = line[i]
                if c == "\\":
                    t, i = _read_escape(line, i + 1, delimiter)
                    buf.append(t)
                elif c == '"':
                    if i + 1 < n and line[i + 1] == '"':
                        buf.append('"')
                        i += 2
                    else:
                        i += 1
                        break
                else:
                    buf.append(c)
                    i += 1
            # skip anything up to the next delimiter (lenient)
            while i < n and line[i] != delimiter:
                buf.append(line[i])
                i += 1
        else:
            while i < n and line[i] != delimiter:
                c = line[i]
                if c == "\\":
                    t, i = _read_escape(line, i + 1, delimiter)
                    buf.append(t)
                else:
                    buf.append(c)
                    i += 1
        out.append("".join(buf))
        if i >= n:
            return out
        i += 1  # delimiter
        if i >= n:
            out.append("")
            return out


def parse_pmml_delimited(s: str) -> List[str]:
    """Space-delimited PMML content; empty tokens (from runs of spaces) are dropped."""
    return [t for t in parse_delimited(s, " ") if t != ""]


def _needs_quote(value: str, delimiter: str, first: bool) -> bool:
    if value == "":
        return first
    c = value[0]
    o = ord(c)
    if first and (o < 0x20 or 0x21 < o < 0x23 or 0x2B < o < 0x2D or o > 0x7E):
        return True
    if o <= ord("#"):
        return True
    for ch in value:
        if ch in ("\n", "\r", '"', delimiter):
            return True
    return ord(value[-1]) <= 0x20


def _to_text(v: Any) -> str:
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return java_double_str(v)
    return str(v)


def _join_plain(elements, delimiter: str) -> Optional[str]:
    """``delimiter.join(elements)`` when that is already the quoted form, i.e. no element
    needs quoting or escaping (checked over the joined bytes, vectorised: the ID lists of a
    model's PMML hold 1e5-1e7 plain IDs); None otherwise."""
    if not isinstance(elements, (list, tuple)) or len(elements) < 64 or len(delimiter) != 1:
        return None
    try:
        joined = delimiter.join(elements)
    except TypeError:
        return None
    if _needs_quote(elements[0], delimiter, True) or "\\" in elements[0]:
        return None
    raw = np.frombuffer(joined.encode("utf-8"), dtype=np.uint8)
    if any(c in joined for c in ('"', "\\", "\n", "\r")):
        return None
    d = np.flatnonzero(raw == ord(delimiter))
    if len(d) != len(elements) - 1:
        return None                      # an element contains the delimiter
    firsts = raw[d + 1] if len(d) and d[-1] + 1 < len(raw) else None
    if firsts is None or len(firsts) != len(d):
        return None                      # empty last element
    lasts = raw[np.r_[d, len(raw)] - 1]
    if (firsts <= ord("#")).any() or (lasts <= 0x20).any():
        return None
    return joined


def join_delimited(elements: Iterable[Any], delimiter: str = ",") -> str:
    fast = _join_plain(elements, delimiter)
    if fast is not None:
        return fast
    parts = []
    for idx, e in enumerate(elements):
        s = _to_text(e)
        if _needs_quote(s, delimiter, idx == 0):
            s = '"' + s.replace('"', '""') + '"'
        else:
            s = s.replace("\\", "\\\\")
        parts.append(s)
    return delimiter.join(parts)


def join_pmml_delimited(elements: Iterable[Any]) -> str:
    return join_delimited(elements, " ").replace('""', '\\"')


def join_pmml_delimited_numbers(elements: Iterable[Any]) -> str:
    return " ".join(_to_text(e) for e in elements)


def parse_json_array(s: str) -> List[str]:
    arr = json.loads(s)
    if not isinstance(arr, list):
        raise ValueError("not a JSON array: %r" % s)
    return [x if isinstance(x, str) else json.dumps(x) if isinstance(x, (list, dict)) else
            _to_text(x) for x in arr]


def join_json(elements: Iterable[Any]) -> str:
    return json.dumps(list(elements), separators=(",", ":"))


def read_json(s: str):
    return json.loads(s)


def parse_input_line(line: str) -> List[str]:
    """``MLFunctions.PARSE_FN``: JSON array if bracketed, else CSV."""
    if line.startswith("[") and line.endswith("]"):
        return parse_json_array(line)
    return parse_delimited(line, ",")


# ---------------------------------------------------------------- Java number formatting

def _java_repr(x: float, shortest: str) -> str:
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    ax = abs(x)
    if 1e-3 <= ax < 1e7:
        if "e" in shortest or "E" in shortest:
            shortest = "%.17f" % x
            shortest = shortest.rstrip("0")
        if "." not in shortest:
            shortest += ".0"
        if shortest.endswith("."):
            shortest += "0"
        return shortest
    # scientific: d.dddE[-]n
    mant, _, exp = ("%r" % float(shortest)).partition("e")
    if not exp:
        # repr gave a plain number (e.g. 12345678.0); convert
        digits = shortest.replace("-", "").replace(".", "").lstrip("0")
        e = int(math.floor(math.log10(ax)))
        mant = digits[0] + "." + (digits[1:].rstrip("0") or "0")
        if x < 0:
            mant = "-" + mant
        return "%sE%d" % (mant, e)
    if "." not in mant:
        mant += ".0"
    return "%sE%d" % (mant, int(exp))


def java_double_str(x: float) -> str:
    """``Double.toString`` formatting (shortest repr, Java's sci-notation thresholds)."""
    return _java_repr(float(x), repr(float(x)))


def java_float_str(x: float) -> str:
    """``Float.toString``: shortest decimal that round-trips through float32."""
    import numpy as np
    f = np.float32(x)
    if math.isnan(f) or math.isinf(f):
        return _java_repr(float(f), "")
    s = np.format_float_positional(f, unique=True, trim="0") if 1e-3 <= abs(f) < 1e7 else \
        np.format_float_scientific(f, unique=True, trim="0")
    if "e" in s:
        mant, exp = s.split("e")
        if "." not in mant:
            mant += ".0"
        if mant.endswith("."):
            mant += "0"
        return "%sE%d" % (mant, int(exp))
    if s.endswith("."):
        s += "0"
    if "." not in s:
        s += ".0"
    return s


def format_number(x) -> str:
    if isinstance(x, (int,)) and not isinstance(x, bool):
        return str(x)
    return java_double_str(float(x))
