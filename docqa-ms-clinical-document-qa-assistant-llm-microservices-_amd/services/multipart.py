"""Minimal RFC 7578 multipart/form-data parser.

FastAPI's ``File``/``Form`` parameters need ``python-multipart``, which is not installed
here, so the doc-ingestor parses the body itself; the wire contract of
``POST /ingest/`` (``file`` + ``doc_type`` form fields, doc-ingestor/main.py:19-24) is
unchanged for clients such as the UI's ``requests.post(..., files=..., data=...)``
(clinical-ui/app.py:41-49).
"""
from __future__ import annotations

import re
from dataclasses import dataclass


@dataclass
class FilePart:
    filename: str
    content_type: str
    data: bytes


_DISP = re.compile(r'(\w+)\*?="?([^";]*)"?')


def _boundary(content_type: str) -> bytes:
    m = re.search(r'boundary="?([^";]+)"?', content_type or "")
    if not m:
        raise ValueError("multipart boundary missing")
    return m.group(1).encode("latin-1")


def parse_multipart(body: bytes, content_type: str) -> dict:
    """-> {field_name: str | FilePart}.  Raises ValueError on malformed input."""
    if not (content_type or "").lower().startswith("multipart/form-data"):
        raise ValueError("expected multipart/form-data")
    delim = b"--" + _boundary(content_type)
    fields: dict = {}
    parts = body.split(delim)
    for part in parts[1:]:
        if part.startswith(b"--"):
            break
        if part.startswith(b"\r\n"):
            part = part[2:]
        head, sep, data = part.partition(b"\r\n\r\n")
        if not sep:
            continue
        if data.endswith(b"\r\n"):
            data = data[:-2]
        headers = {}
        for line in head.decode("utf-8", errors="replace").split("\r\n"):
            k, _, v = line.partition(":")
            headers[k.strip().lower()] = v.strip()
        disp = headers.get("content-disposition", "")
        params = {k.lower(): v for k, v in _DISP.findall(disp)}
        name = params.get("name")
        if name is None:
            continue
        if "filename" in params:
            fields[name] = FilePart(params["filename"], headers.get("content-type", "application/octet-stream"), data)
        else:
            fields[name] = data.decode("utf-8", errors="replace")
    return fields


def encode_multipart(fields: dict, boundary: str = "docqa-boundary-7d1f") -> tuple[bytes, str]:
    """Inverse helper (tests/clients): fields values are str or FilePart."""
    out = bytearray()
    for name, v in fields.items():
        out += f"--{boundary}\r\n".encode()
        if isinstance(v, FilePart):
            out += (f'Content-Disposition: form-data; name="{name}"; filename="{v.filename}"\r\n'
                    f"Content-Type: {v.content_type}\r\n\r\n").encode()
            out += v.data
        else:
            out += f'Content-Disposition: form-data; name="{name}"\r\n\r\n'.encode() + str(v).encode()
        out += b"\r\n"
    out += f"--{boundary}--\r\n".encode()
    return bytes(out), f"multipart/form-data; boundary={boundary}"
