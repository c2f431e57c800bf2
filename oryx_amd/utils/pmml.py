"""PMML 4.2.1 documents: skeleton, extensions, arrays, read/write.

Equivalent of ``PMMLUtils`` (``[common]/pmml/PMMLUtils.java:41-133``) and the generic parts of
``AppPMMLUtils`` (``[app-common]/pmml/AppPMMLUtils.java:59-285``): a skeleton document with an
``Application name="Oryx"`` header and timestamp, ``Extension`` name/value and space-delimited
content, REAL ``Array`` elements, and ``MODEL`` / ``MODEL-REF`` update-message decoding.

Documents are plain :mod:`xml.etree.ElementTree` trees in the PMML 4.2 namespace; app code
builds model elements (ClusteringModel, TreeModel, MiningModel, DataDictionary, ...) with the
helpers here.  Not a hot path.
"""

from __future__ import annotations

import datetime as _dt
import io
import os
import xml.etree.ElementTree as ET
from typing import Iterable, List, Optional

import numpy as np

from . import text as _text
from . import ioutils

__all__ = ["VERSION", "NS", "PMMLDoc", "build_skeleton_pmml", "read", "write", "to_string",
           "from_string", "read_pmml_from_update_key_message", "q", "sub", "to_array",
           "parse_array"]

VERSION = "4.2.1"
NS = "http://www.dmg.org/PMML-4_2"
ET.register_namespace("", NS)


def q(tag: str) -> str:
    """Namespace-qualified tag."""
    return "{%s}%s" % (NS, tag)


def sub(parent: ET.Element, tag: str, attrib: Optional[dict] = None, text: Optional[str] = None
        ) -> ET.Element:
    e = ET.SubElement(parent, q(tag), {k: _attr(v) for k, v in (attrib or {}).items()
                                        if v is not None})
    if text is not None:
        e.text = text
    return e


def _attr(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return _text.java_double_str(v)
    return str(v)


# Element order inside <PMML> required by the schema
_PMML_CHILD_ORDER = ["Header", "MiningBuildTask", "DataDictionary", "TransformationDictionary"]


class PMMLDoc:
    """A PMML document with convenience accessors."""

    def __init__(self, root: ET.Element):
        self.root = root

    # -- header
    @property
    def header(self) -> ET.Element:
        return self.root.find(q("Header"))

    @property
    def version(self) -> str:
        return self.root.get("version")

    # -- extensions (kept right after Header, as JPMML writes them first)
    def extensions(self) -> List[ET.Element]:
        return self.root.findall(q("Extension"))

    def get_extension_value(self, name: str) -> Optional[str]:
        for e in self.extensions():
            if e.get("name") == name:
                return e.get("value")
        return None

    def get_extension_content(self, name: str) -> Optional[List[str]]:
        for e in self.extensions():
            if e.get("name") == name:
                content = (e.text or "").strip()
                return _text.parse_pmml_delimited(content) if content else []
        return None

    def _insert_extension(self, ext: ET.Element) -> None:
        children = list(self.root)
        idx = 0
        for i, c in enumerate(children):
            if c.tag in (q("Extension"),):
                idx = i + 1
        self.root.insert(idx, ext)

    def add_extension(self, name: str, value) -> None:
        ext = ET.Element(q("Extension"), {"name": name, "value": _attr(value)})
        self._insert_extension(ext)

    def add_extension_content(self, name: str, content: Iterable) -> None:
        content = list(content)
        if not content:
            return
        ext = ET.Element(q("Extension"), {"name": name})
        ext.text = _text.join_pmml_delimited(content)
        self._insert_extension(ext)

    # -- models
    def models(self) -> List[ET.Element]:
        names = ("ClusteringModel", "TreeModel", "MiningModel", "RegressionModel",
                 "NaiveBayesModel", "GeneralRegressionModel")
        return [c for c in self.root if c.tag in tuple(q(n) for n in names)]

    def add(self, element: ET.Element) -> ET.Element:
        """Append a top-level child in schema order (DataDictionary before models)."""
        tag = element.tag.split("}")[-1]
        if tag in _PMML_CHILD_ORDER:
            rank = _PMML_CHILD_ORDER.index(tag)
            insert_at = len(self.root)
            for i, c in enumerate(self.root):
                ctag = c.tag.split("}")[-1]
                if ctag in _PMML_CHILD_ORDER and _PMML_CHILD_ORDER.index(ctag) > rank:
                    insert_at = i
                    break
                if ctag not in _PMML_CHILD_ORDER and ctag != "Extension":
                    insert_at = i
                    break
            self.root.insert(insert_at, element)
        else:
            self.root.append(element)
        return element

    def find(self, tag: str) -> Optional[ET.Element]:
        return self.root.find(q(tag))

    def to_string(self) -> str:
        return to_string(self)

    def __repr__(self):
        return "PMMLDoc(%s)" % self.to_string()[:200]


def _timestamp() -> str:
    now = _dt.datetime.now().astimezone()
    s = now.strftime("%Y-%m-%dT%H:%M:%S%z")
    return s


def build_skeleton_pmml() -> PMMLDoc:
    root = ET.Element(q("PMML"), {"version": VERSION})
    header = sub(root, "Header")
    sub(header, "Application", {"name": "Oryx"})
    sub(header, "Timestamp", text=_timestamp())
    return PMMLDoc(root)


def to_string(doc: PMMLDoc) -> str:
    buf = io.BytesIO()
    tree = ET.ElementTree(doc.root)
    ET.indent(tree, space="    ")
    tree.write(buf, encoding="UTF-8", xml_declaration=True)
    return buf.getvalue().decode("utf-8")


def from_string(s: str) -> PMMLDoc:
    root = ET.fromstring(s.encode("utf-8") if isinstance(s, str) else s)
    if root.tag != q("PMML"):
        # accept other PMML 4.x namespaces by rewriting the namespace
        if root.tag.endswith("PMML"):
            for e in root.iter():
                if "}" in e.tag:
                    e.tag = q(e.tag.split("}", 1)[1])
        else:
            raise ValueError("not a PMML document")
    return PMMLDoc(root)


def write(doc: PMMLDoc, path: str) -> None:
    ioutils.write_text(path, to_string(doc))


def read(path: str) -> PMMLDoc:
    return from_string(ioutils.read_text(path))


def read_pmml_from_update_key_message(key: str, message: str) -> PMMLDoc:
    """``MODEL``: inline PMML; ``MODEL-REF``: a path (``file:`` URI or plain) to read."""
    if key == "MODEL":
        return from_string(message)
    if key == "MODEL-REF":
        return from_string(ioutils.read_text(message))
    raise ValueError("Unknown key " + key)


def to_array(values, as_int: bool = False) -> ET.Element:
    vals = list(values)
    arr = ET.Element(q("Array"), {"type": "int" if as_int else "real", "n": str(len(vals))})
    if as_int:
        arr.text = _text.join_pmml_delimited_numbers([int(v) for v in vals])
        return arr
    a = np.asarray(vals, dtype=np.float64)
    # Double.toString is Python's shortest repr wherever Java writes plain decimals (0 and
    # 1e-3 <= |x| < 1e7); only the other values need the Java formatting one by one
    plain = (a == 0) | ((np.abs(a) >= 1e-3) & (np.abs(a) < 1e7))
    fl = a.tolist()
    if bool(plain.all()):
        arr.text = " ".join(map(repr, fl))
    else:
        arr.text = " ".join(repr(x) if p else _text.java_double_str(x)
                            for x, p in zip(fl, plain.tolist()))
    return arr


def parse_array(arr: ET.Element) -> List[float]:
    return [float(t) for t in _text.parse_pmml_delimited(arr.text or "")]
