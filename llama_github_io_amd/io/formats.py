"""Native readers for the spreadsheet and row-container formats H2O ingests that have no library in this
image (openpyxl / xlrd / fastavro are absent):

* XLSX — Office Open XML: ``xl/sharedStrings.xml`` + the first worksheet's ``<sheetData>``
  (reference parses spreadsheets with ``water/parser/XlsParser.java``; XLSX arrives through the same
  ParseSetup path).
* XLS — BIFF8 inside an OLE2 compound document (``water/parser/XlsParser.java``: BOF / SST (+CONTINUE)
  / LABELSST / LABEL / NUMBER / RK / MULRK / BOOLERR / FORMULA cached results of the first sheet).
* Avro — object container files, ``null`` and ``deflate`` codecs, records of primitive / enum / fixed /
  nullable-union fields (``h2o-parsers/h2o-avro-parser/.../AvroParser.java``).

Every reader returns a grid (list of rows; Avro's first row is the field names) of ``float`` / ``str`` /
``None`` cells; ``to_frame`` types the columns the way the CSV path does (numeric, enum, string).
"""
from __future__ import annotations

import io
import json
import math
import re
import struct
import zipfile
import zlib
from xml.etree import ElementTree as ET


# ================================================================================================ XLSX
_NS = "{http://schemas.openxmlformats.org/spreadsheetml/2006/main}"


def _col_index(ref: str) -> int:
    n = 0
    for ch in ref:
        if ch.isalpha():
            n = n * 26 + (ord(ch.upper()) - 64)
        else:
            break
    return n - 1


def read_xlsx(buf: bytes):
    z = zipfile.ZipFile(io.BytesIO(buf))
    shared = []
    if "xl/sharedStrings.xml" in z.namelist():
        root = ET.fromstring(z.read("xl/sharedStrings.xml"))
        for si in root.iter(_NS + "si"):
            shared.append("".join(t.text or "" for t in si.iter(_NS + "t")))
    sheets = sorted(n for n in z.namelist() if re.match(r"xl/worksheets/sheet\d+\.xml$", n))
    if not sheets:
        raise ValueError("XLSX has no worksheet")
    first = min(sheets, key=lambda n: int(re.findall(r"\d+", n.rsplit("/", 1)[1])[0]))
    root = ET.fromstring(z.read(first))
    rows = {}
    for r in root.iter(_NS + "row"):
        ri = int(r.get("r")) - 1
        cells = {}
        for c in r.iter(_NS + "c"):
            ci = _col_index(c.get("r", "A"))
            t = c.get("t", "n")
            v = c.find(_NS + "v")
            if t == "inlineStr":
                is_ = c.find(_NS + "is")
                val = "".join(x.text or "" for x in is_.iter(_NS + "t")) if is_ is not None else None
            elif v is None or v.text is None:
                val = None
            elif t == "s":
                val = shared[int(v.text)]
            elif t == "str":
                val = v.text
            elif t == "b":
                val = float(v.text)
            elif t == "e":
                val = None
            else:
                val = float(v.text)
            cells[ci] = val
        rows[ri] = cells
    return _grid(rows)


def _grid(rows: dict):
    if not rows:
        return []
    nr = max(rows) + 1
    nc = max((max(c) + 1 for c in rows.values() if c), default=0)
    return [[rows.get(i, {}).get(j) for j in range(nc)] for i in range(nr)]


# ================================================================================================ OLE2 / XLS
_OLE_SIG = b"\xd0\xcf\x11\xe0\xa1\xb1\x1a\xe1"


def _ole_stream(buf: bytes, names=("Workbook", "Book")) -> bytes:
    if buf[:8] != _OLE_SIG:
        raise ValueError("not an OLE2 compound document")
    sec = 1 << struct.unpack_from("<H", buf, 30)[0]
    msec = 1 << struct.unpack_from("<H", buf, 32)[0]
    n_fat, dir0 = struct.unpack_from("<II", buf, 44)
    cutoff, minifat0, n_minifat, difat0, n_difat = struct.unpack_from("<IIIII", buf, 56)

    def sector(i):
        o = 512 + i * sec
        return buf[o:o + sec]

    fat_secs = list(struct.unpack_from("<109I", buf, 76))
    d = difat0
    for _ in range(n_difat):
        ent = struct.unpack(f"<{sec // 4}I", sector(d))
        fat_secs += ent[:-1]
        d = ent[-1]
    fat_secs = [s for s in fat_secs[:n_fat]]
    fat = []
    for s in fat_secs:
        fat += struct.unpack(f"<{sec // 4}I", sector(s))

    def chain(start, table, getter):
        out, s, guard = [], start, 0
        while s < 0xFFFFFFFA and guard < len(table) + 1:
            out.append(getter(s))
            s = table[s]
            guard += 1
        return b"".join(out)

    dir_bytes = chain(dir0, fat, sector)
    entries = []
    for o in range(0, len(dir_bytes), 128):
        e = dir_bytes[o:o + 128]
        nl = struct.unpack_from("<H", e, 64)[0]
        name = e[:max(0, nl - 2)].decode("utf-16-le", "replace")
        typ = e[66]
        start, size = struct.unpack_from("<II", e, 116)
        entries.append((name, typ, start, size))
    root = next((e for e in entries if e[1] == 5), None)
    for name, typ, start, size in entries:
        if typ == 2 and name in names:
            if size >= cutoff or root is None:
                return chain(start, fat, sector)[:size]
            minifat = []
            if n_minifat:
                mf = chain(minifat0, fat, sector)
                minifat = list(struct.unpack(f"<{len(mf) // 4}I", mf))
            ministream = chain(root[2], fat, sector)
            return chain(start, minifat, lambda i: ministream[i * msec:(i + 1) * msec])[:size]
    raise ValueError("no Workbook stream in the OLE2 document")


def _rk(v: int) -> float:
    if v & 2:
        x = float(v >> 2 if v < (1 << 31) else (v >> 2) - (1 << 30))
    else:
        x = struct.unpack("<d", struct.pack("<Q", (v & 0xFFFFFFFC) << 32))[0]
    return x / 100.0 if v & 1 else x


class _SST:
    """Shared strings across SST + CONTINUE records (a string may resume in the next record with a fresh
    compression-flags byte)."""

    def __init__(self, chunks):
        self.chunks = chunks
        self.ci, self.pos = 0, 0

    def _need(self, n):
        if self.pos + n > len(self.chunks[self.ci]):
            self.ci += 1
            self.pos = 0

    def u8(self):
        self._need(1)
        v = self.chunks[self.ci][self.pos]
        self.pos += 1
        return v

    def u16(self):
        self._need(2)
        v = struct.unpack_from("<H", self.chunks[self.ci], self.pos)[0]
        self.pos += 2
        return v

    def u32(self):
        self._need(4)
        v = struct.unpack_from("<I", self.chunks[self.ci], self.pos)[0]
        self.pos += 4
        return v

    def skip(self, n):
        while n > 0:
            avail = len(self.chunks[self.ci]) - self.pos
            if avail <= 0:
                self.ci += 1
                self.pos = 0
                continue
            k = min(avail, n)
            self.pos += k
            n -= k

    def string(self):
        nch = self.u16()
        flags = self.u8()
        rich = self.u16() if flags & 0x08 else 0
        ext = self.u32() if flags & 0x04 else 0
        out = []
        wide = flags & 0x01
        left = nch
        while left > 0:
            buf = self.chunks[self.ci]
            if self.pos >= len(buf):            # continues in the next CONTINUE record: new flags byte
                self.ci += 1
                self.pos = 0
                wide = self.chunks[self.ci][0] & 0x01
                self.pos = 1
                buf = self.chunks[self.ci]
            w = 2 if wide else 1
            k = min(left, (len(buf) - self.pos) // w)
            raw = buf[self.pos:self.pos + k * w]
            out.append(raw.decode("utf-16-le" if wide else "latin-1"))
            self.pos += k * w
            left -= k
        self.skip(4 * rich + ext)
        return "".join(out)


def read_xls(buf: bytes):
    wb = _ole_stream(buf)
    recs = []
    o = 0
    while o + 4 <= len(wb):
        typ, ln = struct.unpack_from("<HH", wb, o)
        recs.append((typ, o, wb[o + 4:o + 4 + ln]))
        o += 4 + ln
    sst, sheet_off = [], []
    for i, (typ, off, data) in enumerate(recs):
        if typ == 0x0085:                      # BOUNDSHEET: stream offset of the sheet's BOF
            sheet_off.append(struct.unpack_from("<I", data, 0)[0])
        elif typ == 0x00FC:                    # SST (+ CONTINUE)
            chunks = [data[8:]]
            j = i + 1
            while j < len(recs) and recs[j][0] == 0x003C:
                chunks.append(recs[j][2])
                j += 1
            total = struct.unpack_from("<I", data, 4)[0]
            r = _SST(chunks)
            sst = [r.string() for _ in range(total)]
    start = min(sheet_off) if sheet_off else None
    rows = {}
    in_sheet = start is None
    depth = 0
    pending = None
    for typ, off, data in recs:
        if not in_sheet:
            if off == start:
                in_sheet = True
            else:
                continue
        if typ == 0x0809:
            depth += 1
            continue
        if typ == 0x000A:
            depth -= 1
            if depth <= 0 and start is not None:
                break
            continue

        def put(r, c, v):
            rows.setdefault(r, {})[c] = v
        if typ == 0x00FD:
            r, c, _, k = struct.unpack_from("<HHHI", data)
            put(r, c, sst[k] if k < len(sst) else None)
        elif typ == 0x0203:
            r, c, _, v = struct.unpack_from("<HHHd", data)
            put(r, c, v)
        elif typ == 0x027E:
            r, c, _, v = struct.unpack_from("<HHHI", data)
            put(r, c, _rk(v))
        elif typ == 0x00BD:
            r, c0 = struct.unpack_from("<HH", data)
            n = (len(data) - 6) // 6
            for k in range(n):
                _, v = struct.unpack_from("<HI", data, 4 + 6 * k)
                put(r, c0 + k, _rk(v))
        elif typ == 0x0204:
            r, c, _, n, flags = struct.unpack_from("<HHHHB", data)
            raw = data[9:]
            put(r, c, raw[:2 * n].decode("utf-16-le") if flags & 1 else raw[:n].decode("latin-1"))
        elif typ == 0x0205:
            r, c, _, v, is_err = struct.unpack_from("<HHHBB", data)
            put(r, c, None if is_err else float(v))
        elif typ == 0x0006:
            r, c, _ = struct.unpack_from("<HHH", data)
            res = data[6:14]
            if res[6:8] == b"\xff\xff":
                if res[0] == 0:
                    pending = (r, c)           # string result follows in a STRING record
                elif res[0] == 1:
                    put(r, c, float(res[2]))
                else:
                    put(r, c, None)
            else:
                put(r, c, struct.unpack("<d", res)[0])
        elif typ == 0x0207 and pending is not None:
            n, flags = struct.unpack_from("<HB", data)
            raw = data[3:]
            put(pending[0], pending[1], raw[:2 * n].decode("utf-16-le") if flags & 1 else raw[:n].decode("latin-1"))
            pending = None
    return _grid(rows)


# ================================================================================================ Avro
def _zz(b: io.BytesIO) -> int:
    shift, acc = 0, 0
    while True:
        x = b.read(1)
        if not x:
            raise EOFError
        x = x[0]
        acc |= (x & 0x7F) << shift
        if not x & 0x80:
            break
        shift += 7
    return (acc >> 1) ^ -(acc & 1)


def _avro_value(schema, b: io.BytesIO, names: dict):
    if isinstance(schema, str):
        if schema in names:
            return _avro_value(names[schema], b, names)
        if schema == "null":
            return None
        if schema == "boolean":
            return float(b.read(1)[0])
        if schema in ("int", "long"):
            return float(_zz(b))
        if schema == "float":
            return struct.unpack("<f", b.read(4))[0]
        if schema == "double":
            return struct.unpack("<d", b.read(8))[0]
        if schema in ("bytes", "string"):
            n = _zz(b)
            raw = b.read(n)
            return raw.decode("utf-8", "replace")
        raise ValueError(f"unsupported Avro type {schema}")
    if isinstance(schema, list):                       # union
        return _avro_value(schema[_zz(b)], b, names)
    t = schema["type"]
    if t == "enum":
        names.setdefault(schema.get("name", ""), schema)
        return schema["symbols"][_zz(b)]
    if t == "fixed":
        names.setdefault(schema.get("name", ""), schema)
        return b.read(schema["size"]).hex()
    if t == "record":
        names.setdefault(schema.get("name", ""), schema)
        return [_avro_value(f["type"], b, names) for f in schema["fields"]]
    if t in ("array", "map"):
        raise ValueError("Avro arrays/maps are not flat columns (the reference parser rejects them too)")
    return _avro_value(t, b, names)


def read_avro(buf: bytes):
    b = io.BytesIO(buf)
    if b.read(4) != b"Obj\x01":
        raise ValueError("not an Avro object container file")
    meta = {}
    while True:
        n = _zz(b)
        if n == 0:
            break
        if n < 0:
            _zz(b)
            n = -n
        for _ in range(n):
            k = b.read(_zz(b)).decode()
            meta[k] = b.read(_zz(b))
    sync = b.read(16)
    schema = json.loads(meta["avro.schema"])
    codec = meta.get("avro.codec", b"null").decode()
    if schema.get("type") != "record":
        raise ValueError("top-level Avro schema must be a record")
    names = [f["name"] for f in schema["fields"]]
    rows = []
    while True:
        try:
            count = _zz(b)
        except EOFError:
            break
        size = _zz(b)
        block = b.read(size)
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        elif codec == "snappy":
            # Avro's snappy codec: a raw snappy block followed by the big-endian CRC-32 of the uncompressed bytes
            raw = snappy_decompress(block[:-4])
            if zlib.crc32(raw) & 0xFFFFFFFF != int.from_bytes(block[-4:], "big"):
                raise ValueError("Avro snappy block CRC mismatch")
            block = raw
        elif codec != "null":
            raise NotImplementedError(f"Avro codec {codec} is not supported (null, deflate, snappy)")
        bb = io.BytesIO(block)
        nm = {}
        for _ in range(count):
            rows.append(_avro_value(schema, bb, nm))
        if b.read(16) != sync:
            raise ValueError("Avro sync marker mismatch")
    return [names] + rows


def snappy_decompress(buf: bytes) -> bytes:
    """Raw snappy format (the framing-free block format): a varint of the uncompressed length, then literal and
    back-reference (copy) elements. Decoded in pure Python: Avro blocks are small."""
    n, shift, i = 0, 0, 0
    while True:
        c = buf[i]
        i += 1
        n |= (c & 0x7F) << shift
        if c < 0x80:
            break
        shift += 7
    out = bytearray()
    L = len(buf)
    while i < L:
        tag = buf[i]
        i += 1
        t = tag & 3
        if t == 0:                                   # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[i:i + nb], "little")
                i += nb
            ln += 1
            out += buf[i:i + ln]
            i += ln
            continue
        if t == 1:                                   # copy, 1-byte offset
            ln = 4 + ((tag >> 2) & 7)
            off = ((tag >> 5) << 8) | buf[i]
            i += 1
        elif t == 2:                                 # copy, 2-byte offset
            ln = 1 + (tag >> 2)
            off = int.from_bytes(buf[i:i + 2], "little")
            i += 2
        else:                                        # copy, 4-byte offset
            ln = 1 + (tag >> 2)
            off = int.from_bytes(buf[i:i + 4], "little")
            i += 4
        if off <= 0 or off > len(out):
            raise ValueError("corrupt snappy data (bad copy offset)")
        st = len(out) - off
        if off >= ln:
            out += out[st:st + ln]
        else:                                        # overlapping copy: byte by byte
            for k in range(ln):
                out.append(out[st + k])
    if len(out) != n:
        raise ValueError(f"corrupt snappy data (length {len(out)} != {n})")
    return bytes(out)


# ================================================================================================ frame
def to_frame(grid, header: int = 0, column_types=None):
    """Rows of cells -> H2OFrame: the first row is the header when it is all text (header=0 guesses),
    columns typed like the CSV path (numbers -> real/int, text -> enum/string, dates -> time)."""
    import pandas as pd
    from ..frame import H2OFrame
    if not grid:
        return H2OFrame(pd.DataFrame())
    first = grid[0]
    has_header = header == 1 or (header == 0 and all(isinstance(v, str) for v in first if v is not None)
                                 and any(isinstance(v, str) for v in first)
                                 and any(not isinstance(v, str) for r in grid[1:] for v in r if v is not None))
    names = [str(v) if v is not None else f"C{i + 1}" for i, v in enumerate(first)] if has_header else \
        [f"C{i + 1}" for i in range(len(first))]
    body = grid[1:] if has_header else grid
    cols = {}
    for j, n in enumerate(names):
        vals = [r[j] if j < len(r) else None for r in body]
        if any(isinstance(v, str) for v in vals):
            cols[n] = pd.Series([None if v is None else (v if isinstance(v, str) else _num_str(v)) for v in vals],
                                dtype=object)
        else:
            cols[n] = pd.Series([math.nan if v is None else float(v) for v in vals], dtype="float64")
    return H2OFrame(pd.DataFrame(cols), column_types=column_types)


def _num_str(v: float) -> str:
    return str(int(v)) if float(v).is_integer() else repr(float(v))
