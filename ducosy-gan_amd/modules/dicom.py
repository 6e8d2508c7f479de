"""Minimal DICOM Part-10 reader/writer for the slices DuCoSy-GAN consumes and produces.

The reference reads and writes DICOM through pydicom (modules/dataset.py:3, 82-83, 111;
modules/preprocess.py:70; generate.py:64-128), which is not installed in this image.  This
module covers what those call sites use, for uncompressed little-endian files:

  * dcmread(path, stop_before_pixels=False) -> Dataset
  * Dataset attributes by keyword (Rows, Columns, RescaleSlope, RescaleIntercept,
    InstanceNumber, SliceLocation, PixelRepresentation, SeriesDescription, WindowCenter, ...),
    ``get(keyword, default)``, ``pixel_array`` (int16/uint16 [Rows, Columns]),
    ``PixelData`` assignment, ``add_new(tag, VR, value)``, ``file_meta.TransferSyntaxUID``,
    ``save_as(path)`` and ``copy.deepcopy``.
  * Implicit and explicit VR little endian; sequences and other elements it does not
    interpret are carried through verbatim (defined or undefined length).  Compressed
    (encapsulated) pixel data raises NotImplementedError.

It is host-side file I/O, outside the compute path.
"""
from __future__ import annotations

import copy
import struct
from typing import Dict, Optional, Tuple

import numpy as np

IMPLICIT_VR_LE = "1.2.840.10008.1.2"
EXPLICIT_VR_LE = "1.2.840.10008.1.2.1"
CT_IMAGE_STORAGE = "1.2.840.10008.5.1.4.1.1.2"

# keyword -> (tag, VR) for the attributes the reference touches (plus what a valid file needs)
KEYWORDS: Dict[str, Tuple[int, str]] = {
    "FileMetaInformationGroupLength": (0x00020000, "UL"),
    "FileMetaInformationVersion": (0x00020001, "OB"),
    "MediaStorageSOPClassUID": (0x00020002, "UI"),
    "MediaStorageSOPInstanceUID": (0x00020003, "UI"),
    "TransferSyntaxUID": (0x00020010, "UI"),
    "ImplementationClassUID": (0x00020012, "UI"),
    "SOPClassUID": (0x00080016, "UI"),
    "SOPInstanceUID": (0x00080018, "UI"),
    "Modality": (0x00080060, "CS"),
    "SeriesDescription": (0x0008103E, "LO"),
    "PatientID": (0x00100020, "LO"),
    "InstanceNumber": (0x00200013, "IS"),
    "SliceLocation": (0x00201041, "DS"),
    "SamplesPerPixel": (0x00280002, "US"),
    "PhotometricInterpretation": (0x00280004, "CS"),
    "Rows": (0x00280010, "US"),
    "Columns": (0x00280011, "US"),
    "BitsAllocated": (0x00280100, "US"),
    "BitsStored": (0x00280101, "US"),
    "HighBit": (0x00280102, "US"),
    "PixelRepresentation": (0x00280103, "US"),
    "SmallestImagePixelValue": (0x00280106, "SS"),
    "LargestImagePixelValue": (0x00280107, "SS"),
    "WindowCenter": (0x00281050, "DS"),
    "WindowWidth": (0x00281051, "DS"),
    "RescaleIntercept": (0x00281052, "DS"),
    "RescaleSlope": (0x00281053, "DS"),
    "PixelData": (0x7FE00010, "OW"),
}
_TAG_VR = {t: vr for t, vr in KEYWORDS.values()}
_TAG_KW = {t: k for k, (t, _) in KEYWORDS.items()}
_LONG_VRS = {"OB", "OD", "OF", "OL", "OV", "OW", "SQ", "UC", "UN", "UR", "UT", "SV", "UV"}
_UNDEFINED = 0xFFFFFFFF
_ITEM, _ITEM_END, _SEQ_END = 0xFFFEE000, 0xFFFEE00D, 0xFFFEE0DD


class Element:
    __slots__ = ("tag", "vr", "raw", "undefined")

    def __init__(self, tag: int, vr: str, raw: bytes, undefined: bool = False):
        self.tag, self.vr, self.raw, self.undefined = tag, vr, raw, undefined

    @property
    def value(self):
        return _decode(self.vr, self.raw)


def _decode(vr: str, raw: bytes):
    if vr in ("US", "SS", "UL", "SL", "FL", "FD"):
        fmt = {"US": "H", "SS": "h", "UL": "I", "SL": "i", "FL": "f", "FD": "d"}[vr]
        n = len(raw) // struct.calcsize(fmt)
        vals = struct.unpack("<" + fmt * n, raw[:n * struct.calcsize(fmt)])
        return vals[0] if n == 1 else list(vals)
    if vr in ("DS", "IS"):
        parts = [p.strip() for p in raw.decode("ascii", "replace").strip("\x00 ").split("\\") if p.strip()]
        conv = float if vr == "DS" else int
        vals = [conv(float(p)) if vr == "IS" else conv(p) for p in parts]
        return vals[0] if len(vals) == 1 else vals
    if vr in ("OB", "OW", "OF", "OD", "UN", "SQ"):
        return raw
    return raw.decode("latin-1").rstrip("\x00 ")


def _encode(vr: str, value) -> bytes:
    if isinstance(value, (bytes, bytearray)):
        raw = bytes(value)
    elif vr in ("US", "SS", "UL", "SL", "FL", "FD"):
        fmt = {"US": "H", "SS": "h", "UL": "I", "SL": "i", "FL": "f", "FD": "d"}[vr]
        vals = value if isinstance(value, (list, tuple)) else [value]
        raw = struct.pack("<" + fmt * len(vals), *[int(v) if fmt in "HhIi" else float(v) for v in vals])
    elif vr == "DS":
        vals = value if isinstance(value, (list, tuple)) else [value]
        raw = "\\".join(_ds(v) for v in vals).encode("ascii")
    elif vr == "IS":
        vals = value if isinstance(value, (list, tuple)) else [value]
        raw = "\\".join(str(int(v)) for v in vals).encode("ascii")
    else:
        raw = str(value).encode("latin-1")
    if len(raw) % 2:
        raw += b"\x00" if vr in ("UI", "OB") else b" "
    return raw


def _ds(v) -> str:
    s = repr(float(v)) if not float(v).is_integer() else str(int(v))
    return s if len(s) <= 16 else f"{float(v):.10g}"


def _skip_undefined(buf: bytes, pos: int, explicit: bool) -> int:
    """End offset (after the sequence delimiter) of an undefined-length value starting at pos."""
    while pos + 8 <= len(buf):
        g, e, ln = struct.unpack_from("<HHI", buf, pos)
        tag = (g << 16) | e
        pos += 8
        if tag == _SEQ_END:
            return pos
        if tag != _ITEM:
            raise ValueError(f"malformed sequence at offset {pos - 8}")
        if ln != _UNDEFINED:
            pos += ln
            continue
        while True:  # undefined-length item: nested elements up to the item delimiter
            g, e = struct.unpack_from("<HH", buf, pos)
            if (g << 16) | e == _ITEM_END:
                pos += 8
                break
            _, _, _, pos = _read_element(buf, pos, explicit)
    raise ValueError("unterminated sequence")


def _read_element(buf: bytes, pos: int, explicit: bool):
    g, e = struct.unpack_from("<HH", buf, pos)
    tag = (g << 16) | e
    if explicit:
        vr = buf[pos + 4:pos + 6].decode("ascii", "replace")
        if vr in _LONG_VRS:
            (ln,) = struct.unpack_from("<I", buf, pos + 8)
            pos += 12
        else:
            (ln,) = struct.unpack_from("<H", buf, pos + 6)
            pos += 8
    else:
        vr = _TAG_VR.get(tag, "UN")
        (ln,) = struct.unpack_from("<I", buf, pos + 4)
        pos += 8
    if ln == _UNDEFINED:
        end = _skip_undefined(buf, pos, explicit)
        return Element(tag, vr if explicit or vr != "UN" else "SQ", buf[pos:end], True), tag, vr, end
    return Element(tag, vr, buf[pos:pos + ln]), tag, vr, pos + ln


class FileMeta:
    def __init__(self, elements: Dict[int, Element]):
        object.__setattr__(self, "_el", elements)

    def __getattr__(self, name):
        tag = KEYWORDS.get(name, (None,))[0]
        if tag is None or tag not in self._el:
            raise AttributeError(name)
        return self._el[tag].value

    def __setattr__(self, name, value):
        tag, vr = KEYWORDS[name]
        self._el[tag] = Element(tag, vr, _encode(vr, value))


class Dataset:
    """Top-level data elements (tag -> Element) plus the file meta group."""

    def __init__(self, elements=None, meta=None, explicit=True):
        object.__setattr__(self, "_el", dict(elements or {}))
        object.__setattr__(self, "_meta", dict(meta or {}))
        object.__setattr__(self, "_explicit", explicit)

    @property
    def file_meta(self) -> FileMeta:
        return FileMeta(self._meta)

    def __contains__(self, name):
        return KEYWORDS.get(name, (None,))[0] in self._el

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        tag = KEYWORDS.get(name, (None,))[0]
        if tag is None or tag not in self._el:
            raise AttributeError(f"DICOM dataset has no attribute {name!r}")
        return self._el[tag].value

    def __setattr__(self, name, value):
        if name not in KEYWORDS:
            raise AttributeError(f"unknown DICOM keyword {name!r}")
        tag, vr = KEYWORDS[name]
        if name in ("SmallestImagePixelValue", "LargestImagePixelValue"):
            vr = "US" if int(self._el_value(0x00280103, 1)) == 0 else "SS"
        self._el[tag] = Element(tag, vr, _encode(vr, value))

    def _el_value(self, tag, default=None):
        return self._el[tag].value if tag in self._el else default

    def get(self, name, default=None):
        try:
            return getattr(self, name)
        except AttributeError:
            return default

    def add_new(self, tag, vr, value):
        t = (tag[0] << 16) | tag[1] if isinstance(tag, tuple) else int(tag)
        self._el[t] = Element(t, vr, _encode(vr, value))

    def __deepcopy__(self, memo):
        return Dataset({t: copy.copy(e) for t, e in self._el.items()}, {t: copy.copy(e) for t, e in self._meta.items()},
                       self._explicit)

    @property
    def pixel_array(self) -> np.ndarray:
        el = self._el.get(0x7FE00010)
        if el is None:
            raise AttributeError("no PixelData")
        if el.undefined:
            raise NotImplementedError("compressed (encapsulated) pixel data is not supported")
        rows, cols = int(self.Rows), int(self.Columns)
        bits = int(self._el_value(0x00280100, 16))
        spp = int(self._el_value(0x00280002, 1))
        if spp != 1 or bits not in (8, 16):
            raise NotImplementedError(f"pixel format: {spp} samples, {bits} bits")
        signed = int(self._el_value(0x00280103, 0)) == 1
        dt = {(8, False): np.uint8, (8, True): np.int8, (16, False): np.uint16, (16, True): np.int16}[(bits, signed)]
        return np.frombuffer(el.raw, dtype=np.dtype(dt).newbyteorder("<"), count=rows * cols).reshape(rows, cols)

    def save_as(self, path: str):
        ts = _decode("UI", self._meta[0x00020010].raw) if 0x00020010 in self._meta else EXPLICIT_VR_LE
        if ts not in (IMPLICIT_VR_LE, EXPLICIT_VR_LE):
            raise NotImplementedError(f"transfer syntax {ts}")
        explicit = ts == EXPLICIT_VR_LE
        meta = dict(self._meta)
        meta.setdefault(0x00020001, Element(0x00020001, "OB", b"\x00\x01"))
        meta[0x00020010] = Element(0x00020010, "UI", _encode("UI", ts))
        body = b"".join(_write_element(e, True) for t, e in sorted(meta.items()) if t != 0x00020000)
        out = [b"\x00" * 128, b"DICM", _write_element(Element(0x00020000, "UL", struct.pack("<I", len(body))), True), body]
        out += [_write_element(e, explicit) for _, e in sorted(self._el.items())]
        with open(path, "wb") as f:
            f.write(b"".join(out))


def _write_element(e: Element, explicit: bool) -> bytes:
    g, el = e.tag >> 16, e.tag & 0xFFFF
    ln = _UNDEFINED if e.undefined else len(e.raw)
    if not explicit:
        return struct.pack("<HHI", g, el, ln) + e.raw
    vr = e.vr if len(e.vr) == 2 else "UN"
    if vr in _LONG_VRS:
        return struct.pack("<HH", g, el) + vr.encode() + b"\x00\x00" + struct.pack("<I", ln) + e.raw
    if ln > 0xFFFF:
        return struct.pack("<HH", g, el) + b"UN\x00\x00" + struct.pack("<I", ln) + e.raw
    return struct.pack("<HH", g, el) + vr.encode() + struct.pack("<H", ln) + e.raw


def dcmread(path: str, stop_before_pixels: bool = False) -> Dataset:
    with open(path, "rb") as f:
        buf = f.read()
    pos = 0
    meta: Dict[int, Element] = {}
    if len(buf) >= 132 and buf[128:132] == b"DICM":
        pos = 132
        while pos + 8 <= len(buf) and struct.unpack_from("<H", buf, pos)[0] == 0x0002:
            el, tag, _, pos = _read_element(buf, pos, True)
            meta[tag] = el
    ts = _decode("UI", meta[0x00020010].raw) if 0x00020010 in meta else IMPLICIT_VR_LE
    if ts not in (IMPLICIT_VR_LE, EXPLICIT_VR_LE):
        # encapsulated (compressed) syntaxes are explicit VR LE in the dataset encoding
        if ts.startswith("1.2.840.10008.1.2.4") or ts.startswith("1.2.840.10008.1.2.5"):
            explicit = True
        else:
            raise NotImplementedError(f"transfer syntax {ts}")
    else:
        explicit = ts == EXPLICIT_VR_LE
    elements: Dict[int, Element] = {}
    while pos + 8 <= len(buf):
        g = struct.unpack_from("<H", buf, pos)[0]
        if stop_before_pixels and g >= 0x7FE0:
            break
        el, tag, _, pos = _read_element(buf, pos, explicit)
        elements[tag] = el
    return Dataset(elements, meta, explicit)


def new_ct_slice(pixels: np.ndarray, slope: float = 1.0, intercept: float = -1024.0, instance: int = 1,
                 slice_location: Optional[float] = None, uid_suffix: str = "1") -> Dataset:
    """A minimal CT image dataset (explicit VR LE) holding int16/uint16 stored pixels."""
    pixels = np.ascontiguousarray(pixels)
    if pixels.dtype not in (np.int16, np.uint16):
        raise ValueError("pixels must be int16 or uint16")
    ds = Dataset(meta={})
    uid = f"1.2.826.0.1.3680043.10.999.{uid_suffix}"
    m = ds.file_meta
    m.MediaStorageSOPClassUID = CT_IMAGE_STORAGE
    m.MediaStorageSOPInstanceUID = uid
    m.TransferSyntaxUID = EXPLICIT_VR_LE
    m.ImplementationClassUID = "1.2.826.0.1.3680043.10.999"
    ds.SOPClassUID = CT_IMAGE_STORAGE
    ds.SOPInstanceUID = uid
    ds.Modality = "CT"
    ds.InstanceNumber = instance
    if slice_location is not None:
        ds.SliceLocation = slice_location
    ds.SamplesPerPixel = 1
    ds.PhotometricInterpretation = "MONOCHROME2"
    ds.Rows, ds.Columns = int(pixels.shape[0]), int(pixels.shape[1])
    ds.BitsAllocated, ds.BitsStored, ds.HighBit = 16, 16, 15
    ds.PixelRepresentation = 1 if pixels.dtype == np.int16 else 0
    ds.RescaleSlope, ds.RescaleIntercept = slope, intercept
    ds.PixelData = pixels.astype(pixels.dtype.newbyteorder("<")).tobytes()
    return ds
