"""Document text extraction (the doc-ingestor's Apache Tika step).

Reference: ``tika.parser.from_file(path, serverEndpoint='http://localhost:9998/tika')``,
result ``content.strip()``, ``None`` on any exception (doc-ingestor/processing.py:10-19).

Native extractors (no JVM, no network):
  * plain text: UTF-8 (BOM/UTF-16 aware), latin-1 fallback;
  * DOCX: the ``word/document.xml`` part of the OOXML zip, paragraphs -> lines;
  * PDF: page tree -> content streams (raw or FlateDecode, objects inside /ObjStm object
    streams too), text-showing operators ``Tj``/``TJ``/``'``/``"`` decoded per font
    through its /ToUnicode CMap (1- or 2-byte codes: Type0 / Identity-H fonts) or WinAnsi,
    literal and hex strings, TJ kerning gaps as spaces; text-positioning operators
    (``Td``/``TD``/``T*``/``ET``/``Tm``) become line breaks.  Parity with Tika is
    unpinned (no Tika offline): tests pin the decoding on generated fixtures;
  * HTML: tags stripped.
If ``TIKA_URL`` is set the file is PUT to that Tika server instead, as in the reference.
"""
from __future__ import annotations

import io
import bisect
import re
import zipfile
import zlib
from pathlib import Path
from xml.etree import ElementTree as ET


def _decode_text(data: bytes) -> str:
    if data.startswith(b"\xef\xbb\xbf"):
        return data[3:].decode("utf-8", errors="replace")
    if data.startswith((b"\xff\xfe", b"\xfe\xff")):
        return data.decode("utf-16", errors="replace")
    try:
        return data.decode("utf-8")
    except UnicodeDecodeError:
        return data.decode("latin-1")


def extract_docx(data: bytes) -> str:
    ns = "{http://schemas.openxmlformats.org/wordprocessingml/2006/main}"
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        root = ET.fromstring(z.read("word/document.xml"))
    lines = []
    for p in root.iter(ns + "p"):
        parts = []
        for node in p.iter():
            if node.tag == ns + "t" and node.text:
                parts.append(node.text)
            elif node.tag == ns + "tab":
                parts.append("\t")
            elif node.tag == ns + "br":
                parts.append("\n")
        lines.append("".join(parts))
    return "\n".join(lines)


# ---------------------------------------------------------------- PDF
# Object-level reader: indirect objects (plain and inside /ObjStm object streams), page
# tree with inherited /Resources, per-font decoding -- a /ToUnicode CMap (bfchar /
# bfrange, 1- or 2-byte codes from its codespacerange: the Type0 / Identity-H fonts of
# most generated PDFs), else WinAnsi (cp1252) for simple fonts -- literal and hex
# strings, TJ arrays with kerning gaps as spaces.  Files it cannot parse that way fall
# back to scanning every content stream with latin-1 decoding (the round-1 behaviour).
#
# Uploads are untrusted, so the reader is bounded: objects are found by one
# linear scan of "N G obj" headers paired with the next "endobj" (no backtracking regex over
# the body); streams are kept compressed and inflated lazily, only the ones text
# extraction touches (page contents, ToUnicode CMaps, object streams), each capped at
# MAX_STREAM_BYTES of output and the document at MAX_INFLATE_BYTES in all, so a small
# deflate bomb or a file of images costs nothing.
_OBJ_HEAD = re.compile(rb"(?<![0-9])(\d+)\s+(\d+)\s+obj\b")
_ENDOBJ = re.compile(rb"\bendobj")
_STREAM_KW = re.compile(rb"(?<![A-Za-z])stream\r?\n")
_REF = re.compile(rb"(\d+)\s+(\d+)\s+R")
MAX_STREAM_BYTES = 16 << 20
MAX_INFLATE_BYTES = 128 << 20
MAX_OBJECTS = 200_000
_ESC = {b"n": b"\n", b"r": b"\r", b"t": b"\t", b"b": b"\b", b"f": b"\f", b"(": b"(", b")": b")", b"\\": b"\\"}


def _pdf_string(buf: bytes, i: int) -> tuple[bytes, int]:
    """Parse a literal string starting at buf[i] == '(' -> (bytes, index after ')')."""
    out = bytearray()
    depth = 0
    i += 1
    while i < len(buf):
        c = buf[i:i + 1]
        if c == b"\\":
            nxt = buf[i + 1:i + 2]
            if nxt in _ESC:
                out += _ESC[nxt]
                i += 2
            elif nxt.isdigit():
                j = i + 1
                while j < len(buf) and j < i + 4 and buf[j:j + 1].isdigit():
                    j += 1
                out.append(int(buf[i + 1:j], 8) & 0xFF)
                i = j
            else:
                i += 2
            continue
        if c == b"(":
            depth += 1
        elif c == b")":
            if depth == 0:
                return bytes(out), i + 1
            depth -= 1
        out += c
        i += 1
    return bytes(out), i


def _hex_string(buf: bytes, i: int) -> tuple[bytes, int]:
    """<4a6f> -> bytes (odd digit count padded with 0), index after '>'."""
    j = buf.find(b">", i)
    j = len(buf) if j < 0 else j
    h = re.sub(rb"\s", b"", buf[i + 1:j])
    if len(h) % 2:
        h += b"0"
    try:
        return bytes.fromhex(h.decode("ascii")), j + 1
    except ValueError:
        return b"", j + 1


def _inflate(body: bytes, cap: int) -> bytes | None:
    d = zlib.decompressobj()
    try:
        out = d.decompress(body, cap)
    except zlib.error:
        return None
    return out


def _decompress(head: bytes, body: bytes, cap: int = MAX_STREAM_BYTES) -> bytes | None:
    if b"/FlateDecode" in head or b"/Fl " in head or head.rstrip().endswith(b"/Fl"):
        return _inflate(body, cap)
    if b"/Filter" in head:
        return None          # images / unsupported filters
    return body[:cap]


def _split_stream(body: bytes) -> tuple[bytes, bytes | None]:
    """(dictionary part, raw stream bytes or None) of one object's body."""
    sm = _STREAM_KW.search(body)
    if not sm:
        return body, None
    end = body.rfind(b"endstream")
    if end < sm.end():
        return body, None
    raw = body[sm.end():end]
    if raw.endswith(b"\r\n"):
        raw = raw[:-2]
    elif raw.endswith((b"\n", b"\r")):
        raw = raw[:-1]
    return body[:sm.start()], raw


class _Objects(dict):
    """num -> (dictionary, decoded stream | None); streams inflate on first access."""

    def __init__(self, pdf: "_Pdf"):
        super().__init__()
        self._pdf = pdf

    def __getitem__(self, num):
        head, raw = super().__getitem__(num)
        return head, self._pdf._stream(num, head, raw)

    def get(self, num, default=None):
        return self[num] if num in self else default

    def heads(self):
        """(num, dictionary) of every object, without inflating anything."""
        return ((k, dict.__getitem__(self, k)[0]) for k in sorted(self.keys()))


class _Pdf:
    def __init__(self, data: bytes):
        self.objs = _Objects(self)
        self._inflated: dict[int, bytes | None] = {}
        self._budget = MAX_INFLATE_BYTES
        heads = []
        for m in _OBJ_HEAD.finditer(data):
            heads.append((m.start(), m.end(), int(m.group(1))))
            if len(heads) >= MAX_OBJECTS:
                break
        ends = [m.start() for m in _ENDOBJ.finditer(data)]
        for k, (_, hend, num) in enumerate(heads):
            nxt = heads[k + 1][0] if k + 1 < len(heads) else len(data)
            j = bisect.bisect_left(ends, hend)
            stop = ends[j] if j < len(ends) and ends[j] < nxt else nxt
            dict.__setitem__(self.objs, num, _split_stream(data[hend:stop]))
        for num, head in list(self.objs.heads()):   # compressed object streams
            if b"/ObjStm" not in head:
                continue
            stream = self.objs[num][1]
            if not stream:
                continue
            try:
                n = int(re.search(rb"/N\s+(\d+)", head).group(1))
                first = int(re.search(rb"/First\s+(\d+)", head).group(1))
                nums = [int(x) for x in stream[:first].split()]
            except (AttributeError, ValueError):
                continue
            offs = [(nums[2 * k], first + nums[2 * k + 1]) for k in range(min(n, len(nums) // 2))]
            for k, (on, off) in enumerate(offs):
                end = offs[k + 1][1] if k + 1 < len(offs) else len(stream)
                if on not in self.objs:
                    dict.__setitem__(self.objs, on, (stream[off:end], None))

    def _stream(self, num: int, head: bytes, raw: bytes | None) -> bytes | None:
        if raw is None:
            return None
        if num in self._inflated:
            return self._inflated[num]
        out = _decompress(head, raw, min(MAX_STREAM_BYTES, max(0, self._budget)))
        self._budget -= len(out or b"")
        self._inflated[num] = out
        return out

    def get(self, ref: bytes | int | None):
        if ref is None:
            return None
        if isinstance(ref, bytes):
            m = _REF.match(ref.strip())
            if not m:
                return None
            ref = int(m.group(1))
        return self.objs.get(ref)

    @staticmethod
    def entry(head: bytes, key: bytes) -> bytes | None:
        """Raw value of /key in a dictionary: a reference, a name, an array or a << dict >>."""
        m = re.search(rb"/" + key + rb"(?![A-Za-z])\s*", head)
        if not m:
            return None
        i = m.end()
        if head[i:i + 2] == b"<<":
            depth, j = 0, i
            while j < len(head):
                if head[j:j + 2] == b"<<":
                    depth += 1
                    j += 2
                    continue
                if head[j:j + 2] == b">>":
                    depth -= 1
                    j += 2
                    if depth == 0:
                        return head[i:j]
                    continue
                j += 1
            return head[i:]
        if head[i:i + 1] == b"[":
            j = head.find(b"]", i)
            return head[i:j + 1]
        r = _REF.match(head, i)
        if r:
            return r.group(0)
        t = re.match(rb"/?[^\s/<>\[\]()]+", head[i:])
        return t.group(0) if t else None

    def resolve_dict(self, v: bytes | None) -> bytes:
        if v is None:
            return b""
        if v.startswith(b"<<"):
            return v
        o = self.get(v)
        return o[0] if o else b""


def _parse_cmap(data: bytes) -> tuple[dict, int]:
    """ToUnicode CMap -> ({code: text}, code byte width)."""
    width = 1
    m = re.search(rb"begincodespacerange\s*<([0-9A-Fa-f]+)>", data)
    if m:
        width = max(1, len(m.group(1)) // 2)

    def uni(h: bytes) -> str:
        b = bytes.fromhex(h.decode("ascii"))
        return b.decode("utf-16-be", errors="replace")

    out: dict[int, str] = {}
    for blk in re.finditer(rb"beginbfchar(.*?)endbfchar", data, re.S):
        for a, b in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]*)>", blk.group(1)):
            out[int(a, 16)] = uni(b)
    for blk in re.finditer(rb"beginbfrange(.*?)endbfrange", data, re.S):
        body = blk.group(1)
        for m in re.finditer(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]+)>\s*(<[0-9A-Fa-f]+>|\[[^\]]*\])", body):
            lo, hi, dst = int(m.group(1), 16), int(m.group(2), 16), m.group(3)
            if dst.startswith(b"["):
                for k, h in enumerate(re.findall(rb"<([0-9A-Fa-f]+)>", dst)):
                    out[lo + k] = uni(h)
            else:
                base = bytes.fromhex(dst[1:-1].decode("ascii"))
                for c in range(lo, min(hi, lo + 65535) + 1):
                    last = int.from_bytes(base[-2:], "big") + (c - lo)
                    out[c] = (base[:-2] + last.to_bytes(2, "big")).decode("utf-16-be", errors="replace")
    return out, width


class _Font:
    def __init__(self, pdf: _Pdf, head: bytes):
        self.cmap, self.width = {}, 1
        tu = _Pdf.entry(head, b"ToUnicode")
        o = pdf.get(tu) if tu else None
        if o and o[1]:
            self.cmap, self.width = _parse_cmap(o[1])
        elif b"/Type0" in head:
            self.width = 2

    def decode(self, s: bytes) -> str:
        if self.cmap:
            w = self.width
            return "".join(self.cmap.get(int.from_bytes(s[k:k + w], "big"), "") for k in range(0, len(s) - w + 1, w))
        if self.width == 2:
            return ""          # CID font without a ToUnicode map: no recoverable text
        return s.decode("cp1252", errors="replace")


# content-stream lexing: whitespace / comment runs and runs of bytes that start no token are
# skipped in one regex step each, so a hostile stream (16 MB of NULs, say) costs C-speed
# scanning, not one Python iteration per byte; MAX_CONTENT_TOKENS bounds the token loop
_CS_SKIP = re.compile(rb"(?:[ \t\r\n\f\x00]+|%[^\n]*)+")
_CS_JUNK = re.compile(rb"[^ \t\r\n\f\x00%(<\[/\-0-9.A-Za-z'\"*>{}]+")
_CS_TOK = re.compile(rb"/[^\s/<>\[\]()]+|-?\d*\.?\d+|[A-Za-z'\"*]+|<<|>>|\{|\}")
_CS_NUM = re.compile(rb"-?\d*\.?\d+")
MAX_CONTENT_TOKENS = 4_000_000


def _content_text(content: bytes, fonts: dict) -> str:
    parts: list[str] = []
    font = None
    i, n = 0, len(content)
    operands: list = []
    budget = MAX_CONTENT_TOKENS
    while i < n and budget > 0:
        budget -= 1
        m = _CS_SKIP.match(content, i)
        if m:
            i = m.end()
            continue
        m = _CS_JUNK.match(content, i)
        if m:
            i = m.end()
            continue
        c = content[i:i + 1]
        if c == b"(":
            s, i = _pdf_string(content, i)
            operands.append(s)
            continue
        if c == b"<" and content[i:i + 2] != b"<<":
            s, i = _hex_string(content, i)
            operands.append(s)
            continue
        if c == b"[":
            # TJ array: strings and kerning numbers
            j, arr = i + 1, []
            while j < n and content[j:j + 1] != b"]" and budget > 0:
                budget -= 1
                m = _CS_SKIP.match(content, j) or _CS_JUNK.match(content, j)
                if m:
                    j = m.end()
                    continue
                cj = content[j:j + 1]
                if cj == b"(":
                    s, j = _pdf_string(content, j)
                    arr.append(s)
                elif cj == b"<":
                    s, j = _hex_string(content, j)
                    arr.append(s)
                else:
                    m = _CS_NUM.match(content, j)
                    if m:
                        arr.append(float(m.group(0)))
                        j += len(m.group(0))
                    else:
                        j += 1
            operands.append(arr)
            i = j + 1
            continue
        m = _CS_TOK.match(content, i)
        if not m:
            i += 1
            continue
        tok = m.group(0)
        i += len(tok)
        if tok[:1] == b"/" or re.match(rb"-?\d*\.?\d+$", tok) or tok in (b"<<", b">>", b"{", b"}"):
            operands.append(tok)
            continue
        op = tok
        dec = (font.decode if font is not None else (lambda b: b.decode("cp1252", errors="replace")))
        if op == b"Tf" and len(operands) >= 2 and isinstance(operands[-2], bytes) and operands[-2][:1] == b"/":
            font = fonts.get(operands[-2][1:])
        elif op in (b"Tj", b"'", b'"') and operands and isinstance(operands[-1], bytes):
            if op != b"Tj":
                parts.append("\n")
            parts.append(dec(operands[-1]))
        elif op == b"TJ" and operands and isinstance(operands[-1], list):
            for e in operands[-1]:
                if isinstance(e, float):
                    if e < -200:
                        parts.append(" ")
                else:
                    parts.append(dec(e))
        elif op in (b"T*", b"Td", b"TD", b"ET", b"Tm"):
            if parts and not parts[-1].endswith("\n"):
                parts.append("\n")
        operands = []
    return "".join(parts)


def _page_fonts(pdf: _Pdf, page_head: bytes, cache: dict) -> dict:
    head, seen = page_head, 0
    res = _Pdf.entry(head, b"Resources")
    while res is None and seen < 32:           # inherited from the page tree
        parent = pdf.get(_Pdf.entry(head, b"Parent"))
        if parent is None:
            break
        head, seen = parent[0], seen + 1
        res = _Pdf.entry(head, b"Resources")
    fonts = {}
    fd = pdf.resolve_dict(_Pdf.entry(pdf.resolve_dict(res), b"Font"))
    for name, ref in re.findall(rb"/([^\s/<>\[\]()]+)\s+(\d+\s+\d+\s+R)", fd):
        key = int(_REF.match(ref).group(1))
        if key not in cache:
            o = pdf.get(key)
            cache[key] = _Font(pdf, o[0]) if o else None
        if cache[key] is not None:
            fonts[name] = cache[key]
    return fonts


def extract_pdf(data: bytes) -> str:
    pdf = _Pdf(data)
    pages = [(num, head) for num, head in pdf.objs.heads() if re.search(rb"/Type\s*/Page(?![s\w])", head)]
    texts, cache = [], {}
    for _, head in pages:
        fonts = _page_fonts(pdf, head, cache)
        cont = _Pdf.entry(head, b"Contents")
        refs = _REF.findall(cont) if cont else []
        body = b"\n".join((pdf.get(int(r[0])) or (b"", None))[1] or b"" for r in refs)
        if body:
            texts.append(_content_text(body, fonts).strip("\n"))
    out = "\n".join(t for t in texts if t.strip())
    if out.strip():
        return out
    # no page tree recovered: every text-bearing stream, latin-1 strings (a linear scan of
    # "stream" keywords, each dictionary taken from the 4 KB before it; same inflate budget)
    budget = MAX_INFLATE_BYTES
    for m in _STREAM_KW.finditer(data):
        end = data.find(b"endstream", m.end())
        if end < 0 or budget <= 0:
            break
        d0 = data.rfind(b"<<", max(0, m.start() - 4096), m.start())
        head = data[d0:m.start()] if d0 >= 0 else b""
        body = _decompress(head, data[m.end():end].rstrip(b"\r\n"), min(MAX_STREAM_BYTES, budget))
        budget -= len(body or b"")
        if body and b"BT" in body:
            texts.append(_content_text(body, {}))
    return "\n".join(t for t in texts if t.strip())


def extract_html(data: bytes) -> str:
    s = _decode_text(data)
    s = re.sub(r"(?is)<(script|style).*?</\1>", " ", s)
    s = re.sub(r"(?i)<br\s*/?>|</p>|</div>|</li>", "\n", s)
    s = re.sub(r"<[^>]+>", " ", s)
    return re.sub(r"[ \t]+", " ", s)


def extract_bytes(data: bytes, filename: str = "") -> str:
    name = filename.lower()
    if data.startswith(b"%PDF") or name.endswith(".pdf"):
        return extract_pdf(data)
    if data.startswith(b"PK") and (name.endswith(".docx") or b"word/" in data[:2000]):
        return extract_docx(data)
    if name.endswith((".html", ".htm")) or data.lstrip()[:15].lower().startswith((b"<!doctype html", b"<html")):
        return extract_html(data)
    return _decode_text(data)


def _extract_tika(path: str, url: str) -> str:
    import httpx

    with open(path, "rb") as f:
        r = httpx.put(url, content=f.read(), headers={"Accept": "text/plain"}, timeout=60.0)
    r.raise_for_status()
    return r.text


def extract_text_from_file(path: str, tika_url: str | None = None) -> str | None:
    """Reference-compatible: stripped text, or None on any failure."""
    try:
        if tika_url:
            return (_extract_tika(path, tika_url) or "").strip()
        data = Path(path).read_bytes()
        return (extract_bytes(data, Path(path).name) or "").strip()
    except Exception as e:  # noqa: BLE001 - reference swallows and logs
        print(f"[extraction] failed on {path}: {e}")
        return None


# ---------------------------------------------------------------- test/demo writers
def make_pdf(text: str, compress: bool = True) -> bytes:
    """Minimal single-page PDF with one text line per input line (used by tests)."""
    def esc(s: str) -> str:
        return s.replace("\\", "\\\\").replace("(", "\\(").replace(")", "\\)")

    ops = ["BT", "/F1 11 Tf", "50 780 Td"]
    for k, line in enumerate(text.split("\n")):
        if k:
            ops.append("0 -14 Td")
        ops.append(f"({esc(line)}) Tj")
    ops.append("ET")
    content = "\n".join(ops).encode("latin-1", errors="replace")
    if compress:
        content = zlib.compress(content)
        head = f"<< /Length {len(content)} /Filter /FlateDecode >>".encode()
    else:
        head = f"<< /Length {len(content)} >>".encode()
    objs = [b"<< /Type /Catalog /Pages 2 0 R >>",
            b"<< /Type /Pages /Kids [3 0 R] /Count 1 >>",
            b"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 842] /Contents 4 0 R "
            b"/Resources << /Font << /F1 5 0 R >> >> >>",
            head + b"\nstream\n" + content + b"\nendstream",
            b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica >>"]
    out = bytearray(b"%PDF-1.4\n")
    offsets = []
    for i, o in enumerate(objs, 1):
        offsets.append(len(out))
        out += f"{i} 0 obj\n".encode() + o + b"\nendobj\n"
    xref = len(out)
    out += f"xref\n0 {len(objs) + 1}\n0000000000 65535 f \n".encode()
    for off in offsets:
        out += f"{off:010d} 00000 n \n".encode()
    out += f"trailer\n<< /Size {len(objs) + 1} /Root 1 0 R >>\nstartxref\n{xref}\n%%EOF\n".encode()
    return bytes(out)


def make_docx(text: str) -> bytes:
    from xml.sax.saxutils import escape

    body = "".join(f"<w:p><w:r><w:t xml:space=\"preserve\">{escape(line)}</w:t></w:r></w:p>"
                   for line in text.split("\n"))
    doc = ('<?xml version="1.0" encoding="UTF-8" standalone="yes"?>'
           '<w:document xmlns:w="http://schemas.openxmlformats.org/wordprocessingml/2006/main">'
           f"<w:body>{body}</w:body></w:document>")
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr("[Content_Types].xml", '<?xml version="1.0"?><Types xmlns="http://schemas.openxmlformats.org/package/2006/content-types"/>')
        z.writestr("word/document.xml", doc)
    return buf.getvalue()
