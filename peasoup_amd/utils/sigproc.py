"""Pure-Python SIGPROC filterbank / time-series I/O (numpy).

Independent of the native reader (csrc/src/sigproc.cpp) so tests can
cross-check the two.  Semantics follow include/data_types/header.hpp:171-403:
length-prefixed keys (1..79 bytes), 26 known keys, ``source_name`` /
``rawdatafile`` followed by a string value, nsamples derived from the file
size when absent.  Sub-byte samples are packed LSB-first.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

_DOUBLE = {"az_start", "za_start", "src_raj", "src_dej", "tstart", "tsamp", "period", "fch1", "foff", "refdm"}
_INT = {"nchans", "telescope_id", "machine_id", "data_type", "ibeam", "nbeams", "nbits", "barycentric",
        "pulsarcentric", "nbins", "nsamples", "nifs", "npuls"}
_STRING = {"source_name", "rawdatafile"}
_CHAR = {"signed"}

HEADER_DEFAULTS = {
    "source_name": "", "rawdatafile": "", "az_start": 0.0, "za_start": 0.0, "src_raj": 0.0, "src_dej": 0.0,
    "tstart": 0.0, "tsamp": 0.0, "period": 0.0, "fch1": 0.0, "foff": 0.0, "nchans": 0, "telescope_id": 0,
    "machine_id": 0, "data_type": 0, "ibeam": 0, "nbeams": 0, "nbits": 0, "barycentric": 0, "pulsarcentric": 0,
    "nbins": 0, "nsamples": 0, "nifs": 0, "npuls": 0, "refdm": 0.0, "signed": 0,
}


def _read_str(buf: bytes, off: int):
    (n,) = struct.unpack_from("<i", buf, off)
    if n <= 0 or n >= 80:
        raise ValueError(f"bad SIGPROC key length {n} at offset {off}")
    return buf[off + 4: off + 4 + n].decode("latin-1"), off + 4 + n


def parse_header(buf: bytes, file_size: Optional[int] = None) -> Dict:
    key, off = _read_str(buf, 0)
    if key != "HEADER_START":
        raise ValueError("not a SIGPROC file (no HEADER_START)")
    hdr = dict(HEADER_DEFAULTS)
    present = []
    while True:
        key, off = _read_str(buf, off)
        if key == "HEADER_END":
            break
        if key in _STRING:
            val, off = _read_str(buf, off)
            hdr[key] = val
        elif key in _DOUBLE:
            (hdr[key],) = struct.unpack_from("<d", buf, off)
            off += 8
        elif key in _INT:
            (hdr[key],) = struct.unpack_from("<i", buf, off)
            off += 4
        elif key in _CHAR:
            hdr[key] = buf[off]
            off += 1
        else:
            raise ValueError(f"unknown SIGPROC key {key!r}")
        present.append(key)
    hdr["size"] = off
    hdr["_present"] = present
    if hdr["nsamples"] == 0 and file_size is not None and hdr["nchans"] and hdr["nbits"]:
        hdr["nsamples"] = (file_size - off) // hdr["nchans"] * 8 // hdr["nbits"]
    return hdr


def read_header(path: str) -> Dict:
    import os

    with open(path, "rb") as f:
        buf = f.read(65536)
    return parse_header(buf, os.path.getsize(path))


def _w_str(s: str) -> bytes:
    b = s.encode("latin-1")
    return struct.pack("<i", len(b)) + b


def header_bytes(hdr: Dict) -> bytes:
    out = [_w_str("HEADER_START")]
    order = ["telescope_id", "machine_id", "data_type", "rawdatafile", "source_name", "barycentric",
             "pulsarcentric", "az_start", "za_start", "src_raj", "src_dej", "tstart", "tsamp", "nbits",
             "nsamples", "fch1", "foff", "nchans", "nifs", "ibeam", "nbeams", "refdm", "period", "nbins", "npuls",
             "signed"]
    must = {"data_type", "tsamp", "nbits", "fch1", "foff", "nchans", "nifs"}
    for k in order:
        v = hdr.get(k, HEADER_DEFAULTS[k])
        if k not in must and not v:
            continue
        if k in _STRING:
            out.append(_w_str(k) + _w_str(str(v)))
        elif k in _DOUBLE:
            out.append(_w_str(k) + struct.pack("<d", float(v)))
        elif k in _INT:
            if k == "data_type" and not v:
                v = 1
            if k == "nifs" and not v:
                v = 1
            out.append(_w_str(k) + struct.pack("<i", int(v)))
        else:
            out.append(_w_str(k) + struct.pack("<B", int(v)))
    out.append(_w_str("HEADER_END"))
    return b"".join(out)


def pack_samples(values: np.ndarray, nbits: int) -> np.ndarray:
    """[nsamps, nchans] integer values -> packed SIGPROC bytes (LSB-first)."""
    v = np.asarray(values, dtype=np.uint8)
    if nbits == 8:
        return v.reshape(-1).copy()
    per = 8 // nbits
    nsamps, nchans = v.shape
    assert nchans % per == 0
    v = (v & ((1 << nbits) - 1)).reshape(nsamps, nchans // per, per).astype(np.uint16)
    out = np.zeros((nsamps, nchans // per), dtype=np.uint16)
    for q in range(per):
        out |= v[:, :, q] << (q * nbits)
    return out.astype(np.uint8).reshape(-1)


def unpack_samples(packed: np.ndarray, nsamps: int, nchans: int, nbits: int) -> np.ndarray:
    """Packed SIGPROC bytes -> [nsamps, nchans] uint8 values."""
    b = np.asarray(packed, dtype=np.uint8)[: nsamps * nchans * nbits // 8]
    if nbits == 8:
        return b.reshape(nsamps, nchans)
    per = 8 // nbits
    b = b.reshape(nsamps, nchans // per)
    out = np.empty((nsamps, nchans // per, per), dtype=np.uint8)
    mask = (1 << nbits) - 1
    for q in range(per):
        out[:, :, q] = (b >> (q * nbits)) & mask
    return out.reshape(nsamps, nchans)


@dataclass
class FilterbankData:
    header: Dict
    data: np.ndarray = field(repr=False)  # [nsamps, nchans] uint8 values

    @property
    def nsamps(self) -> int:
        return self.data.shape[0]

    @property
    def nchans(self) -> int:
        return self.data.shape[1]


def read_filterbank(path: str) -> FilterbankData:
    hdr = read_header(path)
    nbytes = hdr["nsamples"] * hdr["nchans"] * hdr["nbits"] // 8
    raw = np.fromfile(path, dtype=np.uint8, count=nbytes, offset=hdr["size"])
    return FilterbankData(hdr, unpack_samples(raw, hdr["nsamples"], hdr["nchans"], hdr["nbits"]))


def write_filterbank(path: str, header: Dict, values: np.ndarray) -> None:
    hdr = dict(header)
    hdr["nchans"] = int(values.shape[1])
    # Write nsamples explicitly: the reader's size-derived count
    # ((bytes/nchans)*8/nbits, header.hpp:396-401) truncates for sub-byte data.
    hdr["nsamples"] = int(values.shape[0])
    with open(path, "wb") as f:
        f.write(header_bytes(hdr))
        f.write(pack_samples(values, int(hdr["nbits"])).tobytes())


def read_tim(path: str):
    hdr = read_header(path)
    dtype = {32: np.float32, 8: np.uint8}[hdr["nbits"]]
    data = np.fromfile(path, dtype=dtype, count=hdr["nsamples"], offset=hdr["size"]).astype(np.float32)
    return hdr, data


def write_tim(path: str, header: Dict, data: np.ndarray) -> None:
    hdr = dict(header)
    hdr.update(nbits=32, nchans=1, nsamples=len(data), data_type=2)
    with open(path, "wb") as f:
        f.write(header_bytes(hdr))
        f.write(np.asarray(data, dtype=np.float32).tobytes())
