"""Configuration: HOCON files layered on packaged defaults.

Equivalent of the reference's ``ConfigUtils`` (``[common]/settings/ConfigUtils.java:37-154``)
and ``ConfigToProperties`` (``[common]/settings/ConfigToProperties.java:33-58``):

* :func:`get_default` -- packaged ``reference.conf`` + the file named by ``$ORYX_CONF`` or the
  ``config.file`` system-property-style env var ``ORYX_CONFIG_FILE``;
* :func:`overlay_on` -- key=value overlay (tests);
* :func:`serialize` / :func:`deserialize` -- ship the ``oryx`` subtree between processes;
* :func:`pretty_print` -- with password redaction;
* :func:`to_properties` -- flatten to ``key=value`` lines for the shell launcher.
"""

from __future__ import annotations

import os
import re
import threading
from typing import Any, Dict, Iterable, List, Mapping, Optional

from . import hocon

__all__ = ["Config", "ConfigError", "get_default", "load_file", "parse_string", "overlay_on",
           "serialize", "deserialize", "pretty_print", "to_properties", "get_optional_string",
           "get_optional_string_list", "set_path"]

_REF_CONF = os.path.join(os.path.dirname(os.path.dirname(__file__)), "conf", "reference.conf")
_REDACT = re.compile(r"(\w*password\w*\s*[=:]\s*).+", re.IGNORECASE)


class ConfigError(KeyError):
    pass


_MISSING = object()


class Config:
    """An immutable, resolved configuration tree with typed getters (Typesafe-Config-like)."""

    def __init__(self, root: Mapping[str, Any]):
        self._root = dict(root)

    # -- structure
    @property
    def root(self) -> Dict[str, Any]:
        return self._root

    def _get(self, path: str):
        cur: Any = self._root
        for k in hocon.split_path(path):
            if not isinstance(cur, dict) or k not in cur:
                return _MISSING
            cur = cur[k]
        return cur

    def has_path(self, path: str) -> bool:
        v = self._get(path)
        return v is not _MISSING and v is not None

    def has_path_or_null(self, path: str) -> bool:
        return self._get(path) is not _MISSING

    def is_null(self, path: str) -> bool:
        return self._get(path) is None

    def _req(self, path: str):
        v = self._get(path)
        if v is _MISSING:
            raise ConfigError("No configuration setting found for key '%s'" % path)
        if v is None:
            raise ConfigError("Configuration key '%s' is set to null" % path)
        return v

    def get(self, path: str, default=None):
        v = self._get(path)
        return default if v is _MISSING else v

    def get_value(self, path: str):
        return self._req(path)

    def get_string(self, path: str) -> str:
        v = self._req(path)
        if isinstance(v, (dict, list)):
            raise ConfigError("'%s' is not a string" % path)
        return hocon._render_scalar_for_concat(v) if not isinstance(v, str) else v

    def get_int(self, path: str) -> int:
        v = self._req(path)
        if isinstance(v, bool):
            raise ConfigError("'%s' is a boolean" % path)
        if isinstance(v, str):
            v = float(v) if re.fullmatch(r"\s*-?[\d.]+([eE][+-]?\d+)?\s*", v) else _bad(path, v)
        if isinstance(v, float):
            if not v.is_integer():
                raise ConfigError("'%s' is not an integer: %r" % (path, v))
            v = int(v)
        return int(v)

    get_long = get_int

    def get_double(self, path: str) -> float:
        v = self._req(path)
        if isinstance(v, bool):
            raise ConfigError("'%s' is a boolean" % path)
        try:
            return float(v)
        except (TypeError, ValueError):
            raise ConfigError("'%s' is not a number: %r" % (path, v))

    def get_bool(self, path: str) -> bool:
        v = self._req(path)
        if isinstance(v, bool):
            return v
        if isinstance(v, str) and v.lower() in ("true", "yes", "on"):
            return True
        if isinstance(v, str) and v.lower() in ("false", "no", "off"):
            return False
        raise ConfigError("'%s' is not a boolean: %r" % (path, v))

    def get_list(self, path: str) -> list:
        v = self._req(path)
        if not isinstance(v, list):
            raise ConfigError("'%s' is not a list" % path)
        return list(v)

    def get_string_list(self, path: str) -> List[str]:
        v = self._req(path)
        if isinstance(v, str):
            # Typesafe accepts a comma-separated string for numerically-indexed objects only;
            # be lenient, as the reference's confs sometimes pass a single string
            return [s.strip() for s in v.split(",") if s.strip()]
        if not isinstance(v, list):
            raise ConfigError("'%s' is not a list" % path)
        return [x if isinstance(x, str) else hocon._render_scalar_for_concat(x) for x in v]

    def get_double_list(self, path: str) -> List[float]:
        return [float(x) for x in self.get_list(path)]

    def get_config(self, path: str) -> "Config":
        v = self._req(path)
        if not isinstance(v, dict):
            raise ConfigError("'%s' is not an object" % path)
        return Config(v)

    def with_fallback(self, other: "Config") -> "Config":
        return Config(hocon.merge(other._root, self._root))

    def with_value(self, path: str, value) -> "Config":
        root = _deep_copy(self._root)
        keys = hocon.split_path(path)
        cur = root
        for k in keys[:-1]:
            nxt = cur.get(k)
            if not isinstance(nxt, dict):
                nxt = {}
                cur[k] = nxt
            cur = nxt
        cur[keys[-1]] = value
        return Config(root)

    def with_only_key(self, key: str) -> "Config":
        return Config({key: self._root[key]} if key in self._root else {})

    def entries(self, prefix: str = "") -> Iterable[tuple]:
        """Flattened (path, leaf) pairs; lists are leaves."""
        def walk(node, path):
            if isinstance(node, dict):
                for k in sorted(node):
                    yield from walk(node[k], path + [k])
            else:
                yield hocon.join_path(path), node
        yield from walk(self._root, hocon.split_path(prefix) if prefix else [])

    def __repr__(self):
        return "Config(%s)" % hocon.render(self._root, concise=True)

    def __eq__(self, other):
        return isinstance(other, Config) and self._root == other._root


def _bad(path, v):
    raise ConfigError("'%s' is not a number: %r" % (path, v))


def _deep_copy(node):
    if isinstance(node, dict):
        return {k: _deep_copy(v) for k, v in node.items()}
    if isinstance(node, list):
        return [_deep_copy(v) for v in node]
    return node


_default_lock = threading.Lock()
_default_cache: Dict[Optional[str], Config] = {}


def _reference_tree() -> dict:
    with open(_REF_CONF, "r", encoding="utf-8") as f:
        return hocon.parse(f.read(), base_dir=os.path.dirname(_REF_CONF))


def parse_string(text: str, fallback_defaults: bool = True) -> Config:
    """Parse (and resolve) a HOCON string, layered over the packaged defaults."""
    tree = hocon.parse(text)
    if fallback_defaults:
        tree = hocon.merge(_reference_tree(), tree)
    return Config(hocon.resolve(tree))


def load_file(path: str, fallback_defaults: bool = True) -> Config:
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    tree = hocon.parse(text, base_dir=os.path.dirname(os.path.abspath(path)))
    if fallback_defaults:
        tree = hocon.merge(_reference_tree(), tree)
    return Config(hocon.resolve(tree))


def get_default() -> Config:
    """Defaults merged with the user's file (``$ORYX_CONFIG_FILE``), resolved once."""
    user = os.environ.get("ORYX_CONFIG_FILE") or os.environ.get("ORYX_CONF")
    with _default_lock:
        if user not in _default_cache:
            _default_cache[user] = load_file(user) if user else Config(
                hocon.resolve(_reference_tree()))
        return _default_cache[user]


def _overlay_value(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        return "null"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_overlay_value(x) for x in v) + "]"
    if isinstance(v, dict):
        return hocon.render(v, concise=True)
    s = str(v)
    # plain strings with characters HOCON forbids unquoted (e.g. "log:/tmp/x") are quoted
    # for convenience; HOCON syntax the caller wrote on purpose ([..], {..}, "..") is kept
    if isinstance(v, str) and s and s[0] not in '[{"' and \
            any(ch in s for ch in ':=,#`^?!@*&\\'):
        return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'
    return s


def overlay_on(overlay: Mapping[str, Any], underlying: Config) -> Config:
    """``ConfigUtils.overlayOn``: each ``k=v`` is parsed as HOCON text and wins over ``underlying``.

    As in the reference, string values must carry their own quotes when they contain HOCON
    special characters; Python lists/dicts/bools/None are rendered for convenience.
    """
    text = "".join("%s=%s\n" % (k, _overlay_value(v)) for k, v in overlay.items())
    tree = hocon.parse(text)
    merged = hocon.merge(underlying.root, tree)
    return Config(hocon.resolve(merged))


def set_path(overlay: Dict[str, Any], key: str, path: str) -> None:
    """``ConfigUtils.set``: put a quoted ``file:`` URI for a local path into an overlay map."""
    real = os.path.realpath(path) if os.path.exists(path) else os.path.abspath(path)
    if os.path.isdir(real) and not real.endswith("/"):
        real += "/"
    overlay[key] = '"file:%s"' % real


def get_optional_string(config: Config, key: str) -> Optional[str]:
    return config.get_string(key) if config.has_path(key) else None


def get_optional_string_list(config: Config, key: str) -> Optional[List[str]]:
    return config.get_string_list(key) if config.has_path(key) else None


def get_optional_double(config: Config, key: str) -> Optional[float]:
    return config.get_double(key) if config.has_path(key) else None


def get_optional_int(config: Config, key: str) -> Optional[int]:
    return config.get_int(key) if config.has_path(key) else None


def get_optional_bool(config: Config, key: str) -> Optional[bool]:
    return config.get_bool(key) if config.has_path(key) else None


def serialize(config: Config) -> str:
    """Concise rendering of only the ``oryx`` subtree (``ConfigUtils.serialize``)."""
    return hocon.render(config.with_only_key("oryx").root, concise=True)


def deserialize(serialized: str) -> Config:
    """Inverse of :func:`serialize`, with defaults as fallback."""
    tree = hocon.parse(serialized)
    return Config(hocon.resolve(hocon.merge(_reference_tree(), tree)))


def pretty_print(config: Config) -> str:
    return redact(hocon.render(config.with_only_key("oryx").root))


def redact(s: str) -> str:
    return _REDACT.sub(lambda m: m.group(1) + "*****", s)


def to_properties(config: Config, prefix: str = "oryx") -> str:
    """``ConfigToProperties``: flatten to sorted ``key=value`` lines (lists comma-joined)."""
    lines = []
    sub = config.get_config(prefix) if prefix else config
    for path, v in sub.entries():
        full = (prefix + "." + path) if prefix else path
        if isinstance(v, list):
            v = ",".join(hocon._render_scalar_for_concat(x) for x in v)
        elif v is None:
            continue
        else:
            v = hocon._render_scalar_for_concat(v)
        lines.append("%s=%s" % (full, v))
    return "\n".join(lines)


def main(argv=None) -> int:  # pragma: no cover - CLI helper
    import sys
    print(to_properties(get_default()))
    return 0
