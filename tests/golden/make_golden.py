#!/usr/bin/env python3
"""Extract the reference's known-answer data into JSON fixtures.

Run here (where /root/reference exists) to regenerate tests/golden/*.json:

    python tests/golden/make_golden.py

It reads the reference's Go test files as TEXT and writes DATA only (inputs
and expected outputs); no reference source is copied.  Each record carries the
file:line it came from.  The GPU box never runs this script.

Sources:
  * hc/huffmantable.go:9-267     -> huffman_table.json (256 {len, val})
  * hc/huffman_test.go:12-28     -> huffman_vectors.json (text <-> hex)
  * hc/io_test.go:76-87          -> string_vectors.json (7-bit prefix literals)
  * hc/io_test.go:11-21, 62-67   -> int_vectors.json (prefix integers, overflows)
  * io/bitio_test.go:25-45       -> bitio_vectors.json (writer op sequence)
  * hc/testcases_test.go, hc/qpack_test.go
                                 -> embedded_literals.json: every quoted string
    of those files whose Huffman encoding (by the oracle) occurs, behind a
    matching H-bit/length prefix octet, inside a hex vector of the same file.
    The reference's expected bytes therefore pin these pairs.
  * frame_test.go:16-50, 62-77   -> varint_vectors.json (HTTP/3 draft varints:
    shortest and longer encodings, the write overflow, the frame header read)
  * hc/statictable.go            -> static_tables.json (HPACK 1-61, QPACK 0-98 entries)
  * hc/testcases_test.go:46-435  -> header_cases.json (header lists with their
    HPACK block, QPACK encoder-stream updates and header block, and the
    dynamic tables after each; decoded in order as hc/hpack_test.go:76-98 and
    hc/qpack_test.go:591-647 do)
  * errors.log:7-241             -> netbsd_qif.json (the one surviving QIF
    header set, used as corpus text for config 3 and the 'hdr' distribution)
"""
from __future__ import annotations

import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("MHQ_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import oracle  # noqa: E402


def _read(rel):
    with open(os.path.join(REF, rel), encoding="utf-8") as f:
        return f.read().split("\n")


def _lineno_of(lines, needle, start=0):
    for i in range(start, len(lines)):
        if needle in lines[i]:
            return i + 1
    return None


def table():
    lines = _read("hc/huffmantable.go")
    out = []
    for i, ln in enumerate(lines):
        m = re.match(r"^\s*\{(\d+),\s*(0x[0-9a-fA-F]+)\},", ln)
        if m:
            out.append({"sym": len(out), "len": int(m.group(1)), "val": int(m.group(2), 16),
                        "src": f"hc/huffmantable.go:{i + 1}"})
    assert len(out) == 256, len(out)
    return out


def huffman_vectors():
    lines = _read("hc/huffman_test.go")
    text = "\n".join(lines)
    body = text[text.index("var tests"): text.index("func TestHuffmanCompress")]
    out = []
    # {"text", "hex" [+ "hex" ...]},
    for m in re.finditer(r'\{\s*"((?:[^"\\]|\\.)*)",\s*((?:"[0-9a-f]*"\s*\+?\s*)+)\}', body):
        hexs = "".join(re.findall(r'"([0-9a-f]*)"', m.group(2)))
        line = _lineno_of(lines, '"' + m.group(1) + '"')
        out.append({"text": m.group(1), "hex": hexs, "src": f"hc/huffman_test.go:{line}"})
    return out


def string_vectors():
    lines = _read("hc/io_test.go")
    out = []
    start = _lineno_of(lines, "var encodedStrings")
    for i in range(start, len(lines)):
        m = re.match(r'^\s*\{"((?:[^"\\]|\\.)*)",\s*"([0-9a-f]+)"\},', lines[i])
        if m:
            out.append({"text": m.group(1), "hex": m.group(2), "prefix": 7, "src": f"hc/io_test.go:{i + 1}"})
        if lines[i].strip() == "}":
            break
    return out


def int_vectors():
    """encodedIntegers (hc/io_test.go:11-21) and the overflowing encodings of
    TestIntegerOverflow (hc/io_test.go:62-67, read with prefix 8)."""
    lines = _read("hc/io_test.go")
    ok, bad = [], []
    for i, ln in enumerate(lines):
        m = re.match(r'^\s*\{(.+?),\s*"([0-9a-f]+)",\s*(\d+)\},', ln)
        if m:
            expr = m.group(1).strip()
            if expr == "^uint64(0)":
                v = (1 << 64) - 1
            elif expr.startswith("1 << "):
                v = 1 << int(expr[5:])
            else:
                v = int(expr)
            ok.append({"value": str(v), "hex": m.group(2), "prefix": int(m.group(3)), "src": f"hc/io_test.go:{i + 1}"})
        m = re.match(r'^\s*"(ff[0-9a-f]+)",\s*$', ln)
        if m:
            bad.append({"hex": m.group(1), "prefix": 8, "src": f"hc/io_test.go:{i + 1}"})
    assert len(ok) == 9 and len(bad) == 2, (len(ok), len(bad))
    return {"ints": ok, "overflow": bad}


def varint_vectors():
    lines = _read("frame_test.go")
    out = {"shortest": [], "longer": [], "src": "frame_test.go"}
    cur = None
    for i, ln in enumerate(lines):
        if "var varints = " in ln:
            cur = out["shortest"]
        elif "var longerVarints = " in ln:
            cur = out["longer"]
        m = re.match(r"^\s*\{(.+?),\s*\[\]byte\{([^}]*)\}\},", ln)
        if m and cur is not None:
            expr = m.group(1).strip().replace(" ", "")
            if expr.startswith("1<<") and expr.endswith("-1"):
                v = (1 << int(expr[3:-2])) - 1
            elif expr.startswith("1<<"):
                v = 1 << int(expr[3:])
            else:
                v = int(expr)
            b = bytes(int(x, 0) for x in m.group(2).replace(" ", "").split(","))
            cur.append({"value": str(v), "hex": b.hex(), "src": f"frame_test.go:{i + 1}"})
    assert len(out["shortest"]) == 9 and len(out["longer"]) == 7, (len(out["shortest"]), len(out["longer"]))
    out["too_large"] = {"value": str(1 << 63), "src": "frame_test.go:62-67"}
    out["frame"] = {"hex": "010700", "type": 7, "payload": "00", "src": "frame_test.go:69-80"}
    return out


def static_tables():
    lines = _read("hc/statictable.go")
    out, cur = {}, None
    for i, ln in enumerate(lines):
        if "hpackStaticTable = " in ln:
            cur = out.setdefault("hpack", [])
        elif "qpackStaticTable = " in ln:
            cur = out.setdefault("qpack", [])
        m = re.match(r'^\s*\{(\d+), "([^"]*)", "([^"]*)"\},', ln)
        if m and cur is not None:
            cur.append({"index": int(m.group(1)), "name": m.group(2), "value": m.group(3),
                        "src": f"hc/statictable.go:{i + 1}"})
    assert len(out["hpack"]) == 61 and out["hpack"][0]["index"] == 1, len(out["hpack"])
    assert [e["index"] for e in out["qpack"]] == list(range(len(out["qpack"])))
    return out


class _GoLit:
    """A small reader of the Go composite literals in hc/testcases_test.go
    (strings with '+' concatenation, bools, ints, nil, keyed and unkeyed
    elements, type prefixes such as []hc.HeaderField or &[]dynamicTableEntry)."""

    TOK = re.compile(r'\s+|//[^\n]*|("(?:[^"\\]|\\.)*")|([A-Za-z_][A-Za-z0-9_.]*)|(\d+)|(.)')

    def __init__(self, text):
        self.toks = []
        for m in self.TOK.finditer(text):
            if m.group(1):
                self.toks.append(("s", json.loads(m.group(1))))
            elif m.group(2):
                self.toks.append(("id", m.group(2)))
            elif m.group(3):
                self.toks.append(("n", int(m.group(3))))
            elif m.group(4):
                self.toks.append(("p", m.group(4)))
        self.i = 0

    def peek(self, k=0):
        return self.toks[self.i + k] if self.i + k < len(self.toks) else (None, None)

    def take(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def value(self):
        kind, v = self.peek()
        if kind == "s":
            out = self.take()[1]
            while self.peek() == ("p", "+"):
                self.take()
                out += self.take()[1]
            return out
        if kind == "n":
            return self.take()[1]
        if kind == "id" and v in ("true", "false", "nil"):
            self.take()
            return {"true": True, "false": False, "nil": None}[v]
        while self.peek() != ("p", "{"):  # type prefix
            self.take()
        return self.composite()

    def composite(self):
        assert self.take() == ("p", "{")
        keyed, items = {}, []
        while self.peek() != ("p", "}"):
            if self.peek()[0] == "id" and self.peek(1) == ("p", ":"):
                key = self.take()[1]
                self.take()
                keyed[key] = self.value()
            else:
                items.append(self.value())
            if self.peek() == ("p", ","):
                self.take()
        self.take()
        return keyed if keyed else items


def header_cases():
    text = "\n".join(_read("hc/testcases_test.go"))
    start = text.index("var testCases = []testCase")
    line0 = text[:start].count("\n") + 1
    lit = _GoLit(text[start + len("var testCases = []testCase"):])
    cases = lit.composite()
    out = []
    for c in cases:
        heads = [{"name": h["Name"], "value": h["Value"], "sensitive": bool(h.get("Sensitive", False))}
                 for h in c["headers"]]
        qt = c["qpackTable"]
        out.append({
            "reset": c["resetTable"], "headers": heads, "huffman": c["huffman"],
            "hpack": c["hpack"], "hpack_table": [list(e) for e in (c["hpackTable"] or [])],
            "qpack_updates": c["qpackUpdates"], "qpack_header": c["qpackHeader"],
            "qpack_base": qt.get("base", 0),
            "qpack_table": None if qt.get("entries") is None else [list(e) for e in qt["entries"]],
        })
    assert out and out[0]["reset"], len(out)
    return {"src": f"hc/testcases_test.go:{line0}", "cases": out}


def bitio_vectors():
    # io/bitio_test.go:25-45 (TestWriter): the op sequence and the expected
    # buffer after each assertion, transcribed as data.
    lines = _read("io/bitio_test.go")
    src = lambda needle: f"io/bitio_test.go:{_lineno_of(lines, needle)}"  # noqa: E731
    return {
        "ops": [
            {"op": "bit", "v": 0, "expect": "", "src": src("writer.WriteBit(0)")},
            {"op": "bit", "v": 1, "expect": "", "src": src("writer.WriteBit(1)")},
            {"op": "bits", "v": 1, "n": 7, "expect": "40", "src": src("writer.WriteBits(1, 7)")},
            {"op": "pad", "v": 0x55, "expect": "40aa", "src": src("writer.Pad(0x55)")},
            {"op": "bits", "v": 1, "n": 64, "expect": "40aa0000000000000001", "src": src("writer.WriteBits(1, 64)")},
            {"op": "bits", "v": 1, "n": 3, "expect": None, "src": src("writer.WriteBits(1, 3)")},
            {"op": "bits", "v": (1 << 64) - 1, "n": 64, "expect": None, "src": src("writer.WriteBits(^uint64(0), 64)")},
            {"op": "pad", "v": 0x03, "expect": "40aa00000000000000013fffffffffffffffe0", "src": src("writer.Pad(0x03)")},
        ],
        "errors": [
            {"op": "bits", "v": 1, "n": 65, "src": src("WriteBits(1, 65)")},
            {"op": "bits", "v": 2, "n": 1, "src": src("WriteBits(2, 1)")},
        ],
    }


def embedded_literals():
    out = {}
    for rel in ("hc/testcases_test.go", "hc/qpack_test.go"):
        lines = _read(rel)
        quoted = set()
        hexes = []  # (hex, line)
        for i, ln in enumerate(lines):
            for q in re.findall(r'"((?:[^"\\]|\\.)*)"', ln):
                if q and re.fullmatch(r"[0-9a-f]+", q) and len(q) % 2 == 0 and len(q) >= 4:
                    hexes.append((q, i + 1))
                if q:
                    quoted.add(q)
        for s in sorted(quoted):
            raw = s.encode()
            enc = oracle.encode(raw)
            if not enc:
                continue
            eh = enc.hex()
            for hx, line in hexes:
                pos = hx.find(eh)
                while pos != -1:
                    if pos % 2 == 0 and pos >= 2:
                        b = int(hx[pos - 2: pos], 16)
                        for p in (7, 5, 3):
                            if (b >> p) & 1 and len(enc) < (1 << p) - 1 and (b & ((1 << p) - 1)) == len(enc):
                                key = (s, eh)
                                out.setdefault(key, {"text": s, "hex": eh, "prefix": p,
                                                     "src": f"{rel}:{line}"})
                    pos = hx.find(eh, pos + 1)
    return sorted(out.values(), key=lambda r: (r["src"], r["text"]))


def netbsd_qif():
    lines = _read("errors.log")
    fields = []
    # errors.log:7-241 is the first copy of netbsd.qif in diff form ('+' lines)
    for i in range(6, 241):
        ln = lines[i]
        assert ln.startswith("+"), (i + 1, ln)
        body = ln[1:]
        if body == "":
            fields.append(None)  # header-block separator
            continue
        name, _, value = body.partition("\t")
        fields.append([name, value])
    return {"src": "errors.log:7-241", "fields": fields}


def main():
    data = {
        "huffman_table.json": table(),
        "huffman_vectors.json": huffman_vectors(),
        "string_vectors.json": string_vectors(),
        "bitio_vectors.json": bitio_vectors(),
        "int_vectors.json": int_vectors(),
        "varint_vectors.json": varint_vectors(),
        "static_tables.json": static_tables(),
        "header_cases.json": header_cases(),
        "embedded_literals.json": embedded_literals(),
        "netbsd_qif.json": netbsd_qif(),
    }
    for name, obj in data.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1)
            f.write("\n")
        n = len(obj) if isinstance(obj, list) else len(obj.get("fields", obj.get("ops", [])))
        print(f"{name}: {n} records")
    # the static tables are also product data (minhq_amd/headers.py loads them)
    with open(os.path.join(REPO, "minhq_amd", "static_tables.json"), "w") as f:
        json.dump(data["static_tables.json"], f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
