"""PDF text extraction (text/extraction.py, the doc-ingestor's Tika step): fonts with a
/ToUnicode CMap and 2-byte Identity-H codes (how most generated clinical PDFs embed
text), font objects inside a compressed /ObjStm, inherited page resources, TJ kerning
gaps, WinAnsi accents, hex strings.  Tika itself is not available offline: parity with it
is unpinned; these fixtures pin the decoding rules."""
import zlib

from docqa_amd.text.extraction import extract_bytes, extract_pdf, make_pdf


def _assemble(objs: dict[int, bytes]) -> bytes:
    out = bytearray(b"%PDF-1.5\n")
    offs = {}
    for n in sorted(objs):
        offs[n] = len(out)
        out += f"{n} 0 obj\n".encode() + objs[n] + b"\nendobj\n"
    xref = len(out)
    out += f"xref\n0 {max(objs) + 1}\n".encode()
    out += f"trailer\n<< /Size {max(objs) + 1} /Root 1 0 R >>\nstartxref\n{xref}\n%%EOF\n".encode()
    return bytes(out)


def _stream(data: bytes, extra: bytes = b"", compress=True) -> bytes:
    if compress:
        data = zlib.compress(data)
        return b"<< /Length %d /Filter /FlateDecode %s>>\nstream\n" % (len(data), extra) + data + b"\nendstream"
    return b"<< /Length %d %s>>\nstream\n" % (len(data), extra) + data + b"\nendstream"


CMAP = b"""/CIDInit /ProcSet findresource begin 12 dict begin begincmap
/CMapName /Adobe-Identity-UCS def
1 begincodespacerange <0000> <FFFF> endcodespacerange
3 beginbfchar
<0001> <0050>
<0002> <00E9>
<0010> <0020>
endbfchar
1 beginbfrange
<0003> <0006> <0061>
endbfrange
1 beginbfrange
<0020> <0021> [<0044> <006F>]
endbfrange
endcmap CMapName currentdict /CMap defineresource pop end end"""


def test_type0_tounicode_in_object_stream():
    # text: "Pé ab" / "Do" with a kerning gap, via 2-byte codes
    content = (b"BT /F1 12 Tf 72 720 Td <0001000200100003> Tj 0 -14 Td "
               b"[<0020> -300 <00210004>] TJ ET")
    # objects 5 (Type0 font) and 6 (descendant) live in an object stream
    f5 = b"<< /Type /Font /Subtype /Type0 /BaseFont /ABCDEE+Calibri /Encoding /Identity-H " \
         b"/DescendantFonts [6 0 R] /ToUnicode 7 0 R >>"
    f6 = b"<< /Type /Font /Subtype /CIDFontType2 /BaseFont /ABCDEE+Calibri >>"
    hdr = b"5 0 6 %d " % (len(f5) + 1)
    objstm = hdr + f5 + b" " + f6
    objs = {
        1: b"<< /Type /Catalog /Pages 2 0 R >>",
        2: b"<< /Type /Pages /Kids [3 0 R] /Count 1 /Resources << /Font << /F1 5 0 R >> >> >>",
        3: b"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 792] /Contents [4 0 R] >>",
        4: _stream(content),
        7: _stream(CMAP),
        8: _stream(objstm, b"/Type /ObjStm /N 2 /First %d " % len(hdr)),
    }
    text = extract_pdf(_assemble(objs))
    lines = [l for l in text.split("\n") if l]
    assert lines == ["Pé a", "D ob"], text


def test_winansi_literal_and_hex_strings():
    content = b"BT /F1 11 Tf 50 780 Td (Patient \\351valu\\351) Tj T* <4f4b> Tj ET"
    objs = {
        1: b"<< /Type /Catalog /Pages 2 0 R >>",
        2: b"<< /Type /Pages /Kids [3 0 R] /Count 1 >>",
        3: b"<< /Type /Page /Parent 2 0 R /Contents 4 0 R /Resources << /Font << /F1 5 0 R >> >> >>",
        4: _stream(content, compress=False),
        5: b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica /Encoding /WinAnsiEncoding >>",
    }
    assert extract_pdf(_assemble(objs)).split("\n") == ["Patient évalué", "OK"]


def test_generated_pdf_roundtrip_and_multipage_order():
    txt = "Compte-rendu du 12/03/2021\nTraitement : warfarine (5 mg)"
    assert extract_bytes(make_pdf(txt), "note.pdf").strip() == txt
    page = lambda t: _stream(b"BT /F1 10 Tf 10 10 Td (" + t + b") Tj ET")
    objs = {1: b"<< /Type /Catalog /Pages 2 0 R >>",
            2: b"<< /Type /Pages /Kids [3 0 R 5 0 R] /Count 2 /Resources << /Font << /F1 7 0 R >> >> >>",
            3: b"<< /Type /Page /Parent 2 0 R /Contents 4 0 R >>", 4: page(b"page one"),
            5: b"<< /Type /Page /Parent 2 0 R /Contents 6 0 R >>", 6: page(b"page two"),
            7: b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica >>"}
    assert extract_pdf(_assemble(objs)).split("\n") == ["page one", "page two"]


def test_untrusted_pdf_is_bounded():
    """a deflate bomb is capped, image streams are never inflated, and a file of
    'N 0 obj' markers with no endobj parses in linear time."""
    import time
    import zlib

    from docqa_amd.text import extraction as ex

    bomb = zlib.compress(b"\0" * (256 << 20), 9)             # 256 MB of zeros in ~250 KB
    pdf = (b"%PDF-1.4\n1 0 obj\n<< /Type /Page /Contents 2 0 R >>\nendobj\n"
           + b"2 0 obj\n<< /Length " + str(len(bomb)).encode() + b" /Filter /FlateDecode >>\nstream\n" + bomb +
           b"\nendstream\nendobj\n3 0 obj\n<< /Subtype /Image /Filter /FlateDecode >>\nstream\n" + bomb +
           b"\nendstream\nendobj\n%%EOF")
    t = time.perf_counter()
    p = ex._Pdf(pdf)
    assert 3 not in p._inflated                             # the image is never touched
    body = p.objs[2][1]
    assert body is not None and len(body) <= ex.MAX_STREAM_BYTES
    ex.extract_pdf(pdf)
    assert time.perf_counter() - t < 20
    spam = b"%PDF-1.4\n" + b"1 0 obj << /A 1 >> " * 200_000    # no endobj anywhere
    t = time.perf_counter()
    ex.extract_pdf(spam)
    assert time.perf_counter() - t < 10
