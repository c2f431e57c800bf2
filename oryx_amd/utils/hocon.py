"""A self-contained HOCON parser and resolver.

The reference configures every layer with Typesafe Config HOCON files
(``framework/oryx-common/src/main/resources/reference.conf:14-274``,
``app/oryx-app-common/src/main/resources/reference.conf:16-150``,
``app/conf/*.conf``).  No HOCON library is installed in this image, so this module
implements the subset of the spec those files (and users' deployment files) rely on:

* objects with ``=``, ``:`` or ``{`` separators, ``+=`` appends, dotted path keys,
  quoted keys, comma- or newline-separated fields, duplicate-key object merging;
* arrays, JSON-style quoted strings, triple-quoted strings, unquoted strings,
  numbers, booleans, ``null``;
* ``#`` and ``//`` comments;
* substitutions ``${path}`` / ``${?path}`` (with environment-variable fallback)
  and value concatenation (``${hdfs-base}"/data/"``);
* ``include "file"`` of a relative or absolute path.

Parsing yields a tree of :class:`dict` / :class:`list` / scalars with unresolved
:class:`Subst` / :class:`Concat` nodes; :func:`merge` layers trees (later wins,
objects merge deeply) and :func:`resolve` substitutes against the merged root.
"""

from __future__ import annotations

import json
import os
import re
from typing import Any, List, Optional

__all__ = ["HoconError", "Subst", "Concat", "parse", "merge", "resolve", "render",
           "split_path", "join_path"]


class HoconError(ValueError):
    pass


class Subst:
    """An unresolved ``${path}`` (``optional`` for ``${?path}``)."""

    __slots__ = ("path", "optional")

    def __init__(self, path: str, optional: bool):
        self.path = path
        self.optional = optional

    def __repr__(self):
        return "${%s%s}" % ("?" if self.optional else "", self.path)


class Concat:
    """Value concatenation of several pieces (strings, substitutions, arrays or objects)."""

    __slots__ = ("parts",)

    def __init__(self, parts: List[Any]):
        self.parts = parts

    def __repr__(self):
        return "Concat(%r)" % (self.parts,)


class _Append:
    """``key += value``: appended to whatever the key resolves to."""

    __slots__ = ("path", "value")

    def __init__(self, path: str, value: Any):
        self.path = path
        self.value = value


class _MergedObj:
    """An object overlaid on a value that is not known to be an object until resolution."""

    __slots__ = ("base", "overlay")

    def __init__(self, base: Any, overlay: dict):
        self.base = base
        self.overlay = overlay


# ---------------------------------------------------------------- tokenizer

_FORBIDDEN_UNQUOTED = set('$"{}[]:=,+#`^?!@*&\\')
_WS = " \t\r﻿ "

_T_PUNCT = "punct"      # { } [ ] , : = +=
_T_NL = "nl"
_T_STR = "str"          # quoted string
_T_UNQ = "unq"          # unquoted text
_T_WS = "ws"            # whitespace run between value tokens (kept for concatenation)
_T_SUBST = "subst"
_T_EOF = "eof"


def _tokenize(text: str) -> List[tuple]:
    toks = []
    i, n = 0, len(text)
    while i < n:
        c = text[i]
        if c in _WS:
            j = i
            while j < n and text[j] in _WS:
                j += 1
            toks.append((_T_WS, text[i:j]))
            i = j
        elif c == "\n":
            toks.append((_T_NL, "\n"))
            i += 1
        elif c == "#" or text.startswith("//", i):
            while i < n and text[i] != "\n":
                i += 1
        elif text.startswith("+=", i):
            toks.append((_T_PUNCT, "+="))
            i += 2
        elif c in "{}[],:=":
            toks.append((_T_PUNCT, c))
            i += 1
        elif text.startswith('"""', i):
            j = text.find('"""', i + 3)
            if j < 0:
                raise HoconError("unterminated triple-quoted string")
            while j + 3 < n and text[j + 3] == '"':   # extra quotes belong to the string
                j += 1
            toks.append((_T_STR, text[i + 3:j]))
            i = j + 3
        elif c == '"':
            j = i + 1
            while j < n and text[j] != '"':
                if text[j] == "\\":
                    j += 1
                if j < n and text[j] == "\n":
                    raise HoconError("newline in quoted string")
                j += 1
            if j >= n:
                raise HoconError("unterminated quoted string")
            toks.append((_T_STR, json.loads(text[i:j + 1])))
            i = j + 1
        elif text.startswith("${", i):
            j = text.find("}", i)
            if j < 0:
                raise HoconError("unterminated substitution")
            body = text[i + 2:j].strip()
            optional = body.startswith("?")
            if optional:
                body = body[1:].strip()
            toks.append((_T_SUBST, Subst(_normalize_subst_path(body), optional)))
            i = j + 1
        else:
            j = i
            while j < n:
                ch = text[j]
                if ch in _FORBIDDEN_UNQUOTED or ch in _WS or ch == "\n" or text.startswith("//", j):
                    break
                j += 1
            if j == i:
                raise HoconError("unexpected character %r at offset %d" % (c, i))
            toks.append((_T_UNQ, text[i:j]))
            i = j
    toks.append((_T_EOF, None))
    return toks


def _normalize_subst_path(body: str) -> str:
    # ${"a.b".c} style quoting: keep quoted segments intact
    return join_path(split_path(body))


def split_path(path: str) -> List[str]:
    """Split a HOCON path expression into keys (quoted segments may contain dots)."""
    keys, cur, i, n = [], [], 0, len(path)
    quoted_any = False
    while i < n:
        c = path[i]
        if c == '"':
            j = i + 1
            while j < n and path[j] != '"':
                if path[j] == "\\":
                    j += 1
                j += 1
            cur.append(json.loads(path[i:j + 1]))
            quoted_any = True
            i = j + 1
        elif c == ".":
            keys.append("".join(cur))
            cur, quoted_any = [], False
            i += 1
        else:
            cur.append(c)
            i += 1
    if cur or quoted_any or path.endswith("."):
        keys.append("".join(cur))
    return [k.strip() if not k.startswith(" ") else k for k in keys]


def join_path(keys: List[str]) -> str:
    out = []
    for k in keys:
        if k == "" or any(ch in k for ch in '."$ {}[]:=,+#') :
            out.append(json.dumps(k))
        else:
            out.append(k)
    return ".".join(out)


# ---------------------------------------------------------------- parser

class _Parser:
    def __init__(self, text: str, base_dir: Optional[str]):
        self.toks = _tokenize(text)
        self.pos = 0
        self.base_dir = base_dir

    def peek(self, skip_ws=True, skip_nl=False):
        p = self.pos
        while True:
            t = self.toks[p]
            if (skip_ws and t[0] == _T_WS) or (skip_nl and t[0] == _T_NL):
                p += 1
                continue
            return t

    def next(self, skip_ws=True, skip_nl=False):
        while True:
            t = self.toks[self.pos]
            self.pos += 1
            if (skip_ws and t[0] == _T_WS) or (skip_nl and t[0] == _T_NL):
                continue
            return t

    def skip(self, nl=True):
        while self.toks[self.pos][0] in ((_T_WS, _T_NL) if nl else (_T_WS,)):
            self.pos += 1

    def parse_root(self) -> dict:
        self.skip()
        t = self.peek()
        if t == (_T_PUNCT, "{"):
            self.next()
            obj = self.parse_object_body(closing="}")
            self.skip()
            if self.peek()[0] != _T_EOF:
                raise HoconError("trailing content after root object")
            return obj
        if t == (_T_PUNCT, "["):
            raise HoconError("root must be an object")
        return self.parse_object_body(closing=None)

    def parse_key(self) -> List[str]:
        keys: List[str] = []
        cur: List[str] = []
        seen = False
        while True:
            t = self.toks[self.pos]
            if t[0] == _T_STR:
                cur.append(t[1])
                seen = True
                self.pos += 1
            elif t[0] == _T_UNQ:
                parts = t[1].split(".")
                for idx, part in enumerate(parts):
                    if idx > 0:
                        keys.append("".join(cur))
                        cur = []
                    cur.append(part)
                seen = True
                self.pos += 1
            elif t[0] == _T_WS:
                # whitespace inside a key is only allowed between quoted/unquoted pieces
                nt = self.toks[self.pos + 1]
                if nt[0] in (_T_STR, _T_UNQ) and seen:
                    cur.append(t[1])
                    self.pos += 1
                else:
                    self.pos += 1
                    break
            else:
                break
        if not seen:
            raise HoconError("expected key, got %r" % (t,))
        keys.append("".join(cur))
        return keys

    def parse_object_body(self, closing: Optional[str]) -> dict:
        obj: dict = {}
        while True:
            self.skip()
            t = self.peek()
            if closing and t == (_T_PUNCT, closing):
                self.next()
                return obj
            if t[0] == _T_EOF:
                if closing:
                    raise HoconError("unterminated object")
                return obj
            if t == (_T_PUNCT, ","):
                self.next()
                continue
            if t[0] == _T_UNQ and t[1] == "include":
                self.next()
                inc = self.next()
                if inc[0] == _T_UNQ and inc[1] in ("file", "required", "classpath", "url") :
                    # include file("x") / required(file("x")) forms
                    raise HoconError("only 'include \"path\"' form is supported")
                if inc[0] != _T_STR:
                    raise HoconError("include expects a quoted path")
                path = inc[1]
                if self.base_dir and not os.path.isabs(path):
                    path = os.path.join(self.base_dir, path)
                if os.path.exists(path):
                    with open(path, "r", encoding="utf-8") as f:
                        sub = parse(f.read(), base_dir=os.path.dirname(path))
                    obj.update(merge(obj, sub))
                continue
            keys = self.parse_key()
            self.skip(nl=False)
            t = self.peek()
            append = False
            if t == (_T_PUNCT, "=") or t == (_T_PUNCT, ":"):
                self.next()
            elif t == (_T_PUNCT, "+="):
                self.next()
                append = True
            elif t == (_T_PUNCT, "{"):
                pass
            else:
                raise HoconError("expected '=', ':' or '{' after key %s, got %r" % (keys, t))
            self.skip(nl=False)
            value = self.parse_value()
            if append:
                value = _Append(join_path(keys), value)
            for k in reversed(keys[1:]):
                value = {k: value}
            key = keys[0]
            if key in obj:
                obj[key] = _merge_values(obj[key], value)
            else:
                obj[key] = value
            # field separator: comma, newline, or closing brace
            self.skip(nl=False)
            t = self.peek()
            if t == (_T_PUNCT, ","):
                self.next()
            elif t[0] in (_T_NL, _T_EOF) or (closing and t == (_T_PUNCT, closing)):
                pass
            else:
                raise HoconError("expected separator after field %s, got %r" % (keys, t))

    def parse_array(self) -> list:
        arr = []
        while True:
            self.skip()
            t = self.peek()
            if t == (_T_PUNCT, "]"):
                self.next()
                return arr
            if t == (_T_PUNCT, ","):
                self.next()
                continue
            if t[0] == _T_EOF:
                raise HoconError("unterminated array")
            arr.append(self.parse_value())

    def parse_value(self):
        parts = []
        while True:
            t = self.toks[self.pos]
            if t[0] == _T_WS:
                if parts:
                    nt = self.toks[self.pos + 1]
                    if nt[0] in (_T_STR, _T_UNQ, _T_SUBST) or nt in ((_T_PUNCT, "{"), (_T_PUNCT, "[")):
                        parts.append(_WsPiece(t[1]))
                self.pos += 1
                continue
            if t == (_T_PUNCT, "{"):
                self.pos += 1
                parts.append(self.parse_object_body(closing="}"))
            elif t == (_T_PUNCT, "["):
                self.pos += 1
                parts.append(self.parse_array())
            elif t[0] == _T_STR:
                self.pos += 1
                parts.append(_Quoted(t[1]))
            elif t[0] == _T_UNQ:
                self.pos += 1
                parts.append(t[1])
            elif t[0] == _T_SUBST:
                self.pos += 1
                parts.append(t[1])
            else:
                break
        if not parts:
            raise HoconError("expected a value, got %r" % (self.toks[self.pos],))
        return _simplify(parts)


class _Quoted(str):
    """A string that came from a quoted token (never coerced to a number/bool/null)."""


class _WsPiece(str):
    """Whitespace between concatenated pieces."""


def _scalar(tok: str):
    if isinstance(tok, _Quoted):
        return str(tok)
    if tok == "true":
        return True
    if tok == "false":
        return False
    if tok == "null":
        return None
    if re.fullmatch(r"-?\d+", tok):
        return int(tok)
    if re.fullmatch(r"-?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?", tok):
        return float(tok)
    return tok


def _simplify(parts: list):
    # drop trailing whitespace
    while parts and isinstance(parts[-1], _WsPiece):
        parts.pop()
    if len(parts) == 1:
        p = parts[0]
        if isinstance(p, str):
            return _scalar(p)
        return p
    if all(isinstance(p, str) for p in parts):
        return "".join(str(p) for p in parts)
    return Concat([str(p) if isinstance(p, str) else p for p in parts])


def _merge_values(old, new):
    if isinstance(new, dict):
        if isinstance(old, dict):
            out = dict(old)
            for k, v in new.items():
                out[k] = _merge_values(out[k], v) if k in out else v
            return out
        if isinstance(old, (Subst, Concat, _MergedObj)):
            return _MergedObj(old, new)
        return new
    if isinstance(new, _Append):
        return Concat([old, new.value]) if not isinstance(old, _Append) else new
    if isinstance(new, (Subst, Concat)) and _refers_to_self(new):
        return _SelfRef(old, new)
    return new


class _SelfRef:
    """A value that refers to the previous value of the same key (``a = ${a} x``)."""

    __slots__ = ("prev", "value")

    def __init__(self, prev, value):
        self.prev = prev
        self.value = value


def _refers_to_self(_v) -> bool:
    # Determined lazily during resolution; merging keeps the previous value around so a
    # self-referential substitution can see it.
    return True


def parse(text: str, base_dir: Optional[str] = None) -> dict:
    """Parse HOCON text into an unresolved tree."""
    return _Parser(text, base_dir).parse_root()


def merge(base: dict, overlay: dict) -> dict:
    """Deep-merge ``overlay`` on top of ``base`` (overlay wins)."""
    return _merge_values(base, overlay)


# ---------------------------------------------------------------- resolution

_MISSING = object()


class _Resolver:
    def __init__(self, root):
        self.root = root
        self.resolving = set()
        self.cache = {}

    def lookup(self, keys: List[str], node=_MISSING, depth=0):
        cur = self.root if node is _MISSING else node
        path_so_far = []
        for k in keys:
            cur = self.resolve_node(cur, tuple(path_so_far))
            if not isinstance(cur, dict) or k not in cur:
                return _MISSING
            cur = cur[k]
            path_so_far.append(k)
        return self.resolve_node(cur, tuple(keys))

    def resolve_node(self, node, path: tuple):
        if isinstance(node, (Subst, Concat, _MergedObj, _SelfRef, _Append)):
            key = (id(node), path)
            if key in self.cache:
                return self.cache[key]
            if key in self.resolving:
                raise HoconError("cycle resolving substitution at %s" % join_path(list(path)))
            self.resolving.add(key)
            try:
                val = self._resolve(node, path)
            finally:
                self.resolving.discard(key)
            self.cache[key] = val
            return val
        return node

    def _subst(self, s: Subst, path: tuple, prev=_MISSING):
        keys = split_path(s.path)
        if prev is not _MISSING and tuple(keys) == path:
            return self.full(prev, path)
        v = self.lookup(keys)
        if v is _MISSING or (v is None and not s.optional and False):
            env = os.environ.get(s.path)
            if env is not None:
                return env
            if s.optional:
                return _MISSING
            raise HoconError("could not resolve substitution ${%s}" % s.path)
        return self.full(v, tuple(keys))

    def _resolve(self, node, path: tuple, prev=_MISSING):
        if isinstance(node, _SelfRef):
            return self._resolve_value(node.value, path, node.prev)
        if isinstance(node, _Append):
            base = self.lookup(split_path(node.path))
            val = self.full(node.value, path)
            if base is _MISSING:
                return [val]
            return list(base) + [val]
        return self._resolve_value(node, path, prev)

    def _resolve_value(self, node, path, prev=_MISSING):
        if isinstance(node, Subst):
            return self._subst(node, path, prev)
        if isinstance(node, _MergedObj):
            base = self._resolve_value(node.base, path, prev) if isinstance(
                node.base, (Subst, Concat, _MergedObj)) else node.base
            if base is _MISSING:
                base = {}
            if isinstance(base, dict):
                return _merge_values(base, node.overlay)
            return node.overlay
        if isinstance(node, Concat):
            pieces = []
            for p in node.parts:
                if isinstance(p, Subst):
                    v = self._subst(p, path, prev)
                    if v is _MISSING:
                        continue
                    pieces.append(v)
                elif isinstance(p, (Concat, _MergedObj)):
                    pieces.append(self._resolve_value(p, path, prev))
                elif isinstance(p, _SelfRef):
                    pieces.append(self._resolve(p, path))
                else:
                    pieces.append(self.full(p, path) if isinstance(p, (dict, list)) else p)
            non_ws = [p for p in pieces if not (isinstance(p, str) and p.strip() == "")]
            if non_ws and all(isinstance(p, list) for p in non_ws):
                out = []
                for p in non_ws:
                    out.extend(p)
                return out
            if non_ws and all(isinstance(p, dict) for p in non_ws):
                out = {}
                for p in non_ws:
                    out = _merge_values(out, p)
                return out
            if not pieces:
                return _MISSING
            if len(pieces) == 1 and not isinstance(pieces[0], str):
                return pieces[0]
            return "".join(_render_scalar_for_concat(p) for p in pieces)
        return node

    def full(self, node, path: tuple):
        """Resolve a node and everything beneath it."""
        node = self.resolve_node(node, path)
        if isinstance(node, dict):
            out = {}
            for k, v in node.items():
                rv = self.full(v, path + (k,))
                if rv is not _MISSING:
                    out[k] = rv
            return out
        if isinstance(node, list):
            out = []
            for idx, v in enumerate(node):
                rv = self.full(v, path + (str(idx),))
                if rv is not _MISSING:
                    out.append(rv)
            return out
        return node


def _render_scalar_for_concat(v) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer() and abs(v) < 1e16:
        return repr(v)
    if isinstance(v, (dict, list)):
        raise HoconError("cannot concatenate an object/array with a string")
    return str(v)


def resolve(tree: dict) -> dict:
    """Resolve every substitution in a merged tree; returns plain dict/list/scalars."""
    r = _Resolver(tree)
    # the root itself may have self references; resolve field by field against the root
    out = r.full(tree, ())
    # second pass so that substitutions pointing at objects that contained substitutions
    # see fully resolved values
    return out


# ---------------------------------------------------------------- rendering

def _render_key(k: str) -> str:
    if re.fullmatch(r"[A-Za-z0-9_\-]+", k):
        return k
    return json.dumps(k)


def render(value, indent: int = 0, concise: bool = False) -> str:
    """Render a resolved tree as HOCON (JSON-compatible when ``concise``)."""
    if concise:
        return json.dumps(value, separators=(",", ":"), allow_nan=False)
    pad = "    " * indent
    if isinstance(value, dict):
        if not value:
            return "{}"
        lines = ["{"]
        for k in sorted(value):
            lines.append("%s    %s=%s" % (pad, _render_key(k), render(value[k], indent + 1)))
        lines.append(pad + "}")
        return "\n".join(lines)
    if isinstance(value, list):
        return "[" + ",".join(render(v, indent + 1) for v in value) + "]"
    if isinstance(value, str):
        return json.dumps(value)
    if value is None:
        return "null"
    if value is True:
        return "true"
    if value is False:
        return "false"
    return repr(value) if isinstance(value, float) else str(value)
