"""Document text extraction (the doc-ingestor's Apache Tika step).

Reference: ``tika.parser.from_file(path, serverEndpoint='http://localhost:9998/tika')``,
result ``content.strip()``, ``None`` on any exception (doc-ingestor/processing.py:10-19).

Native extractors (no JVM, no network):
  * plain text: UTF-8 (BOM/UTF-16 aware), latin-1 fallback;
  * DOCX: the ``word/document.xml`` part of the OOXML zip, paragraphs -> lines;
  * PDF: content streams (raw or FlateDecode) scanned for the text-showing operators
    ``Tj``, ``TJ``, ``'`` and ``"`` with PDF string escapes; text-positioning operators
    (``Td``/``TD``/``T*``/``ET``) become line breaks;
  * HTML: tags stripped.
If ``TIKA_URL`` is set the file is PUT to that Tika server instead, as in the reference.
"""
from __future__ import annotations

import io
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


_PDF_STREAM = re.compile(rb"<<(.*?)>>\s*stream\r?\n(.*?)\r?\nendstream", re.S)
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


def _pdf_content_text(content: bytes) -> str:
    parts: list[str] = []
    i = 0
    pending: list[bytes] = []
    n = len(content)
    while i < n:
        c = content[i:i + 1]
        if c == b"(":
            s, i = _pdf_string(content, i)
            pending.append(s)
            continue
        if c == b"%":  # comment
            j = content.find(b"\n", i)
            i = n if j < 0 else j
            continue
        m = re.match(rb"(Tj|TJ|'|\"|T\*|Td|TD|ET|Tm)\b", content[i:i + 3]) if c.isalpha() or c in b"'\"" else None
        if m:
            op = m.group(1)
            if op in (b"Tj", b"TJ", b"'", b'"'):
                if op in (b"'", b'"'):
                    parts.append("\n")
                parts.append(b"".join(pending).decode("latin-1"))
                pending = []
            elif op in (b"T*", b"Td", b"TD", b"ET", b"Tm"):
                if parts and not parts[-1].endswith("\n"):
                    parts.append("\n")
            i += len(op)
            continue
        i += 1
    return "".join(parts)


def extract_pdf(data: bytes) -> str:
    texts = []
    for m in _PDF_STREAM.finditer(data):
        head, body = m.group(1), m.group(2)
        if b"/FlateDecode" in head:
            try:
                body = zlib.decompress(body)
            except zlib.error:
                continue
        elif b"/Filter" in head:
            continue  # image / unsupported filter
        if b"BT" in body:
            texts.append(_pdf_content_text(body))
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
