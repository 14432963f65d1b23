"""PSRDADA files: the 4096-byte ASCII header (parsed natively by
``_C.read_dada_header`` with the reference's DadaHeader semantics,
include/data_types/header.hpp:52-161) and complex 8-bit voltage payloads.

The reference's ``DadaFile::extract_channel`` (data_types/dada.hpp) is not in
the repository (accmap does not build), so its payload layout
is not pinned.  Here the payload is taken as the common PSRDADA order for
8-bit complex voltages: time-major, then antenna, channel, polarisation,
(re, im) -- ``[nsamples][nant][nchan][npol][2]`` int8.  Parity unpinned.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

HEADER_SIZE = 4096


def read_header(path: str) -> dict:
    from .. import _C

    return dict(_C.read_dada_header(path))


def write(path: str, header: Dict[str, object], payload: np.ndarray) -> None:
    """Write a DADA file: ``KEY value`` lines padded to 4096 bytes, then the payload."""
    lines = [f"{k} {v}" for k, v in header.items()]
    text = ("\n".join(lines) + "\n").encode()
    if len(text) > HEADER_SIZE:
        raise ValueError("DADA header longer than 4096 bytes")
    with open(path, "wb") as f:
        f.write(text + b"\0" * (HEADER_SIZE - len(text)))
        f.write(np.ascontiguousarray(payload).tobytes())


def read_payload(path: str, hdr: Optional[dict] = None) -> np.ndarray:
    """Memory-mapped int8 payload shaped ``[nsamples, nant, nchan, npol, 2]``."""
    hdr = hdr or read_header(path)
    nant, nchan, npol = int(hdr["nant"]), int(hdr["nchan"]), int(hdr["npol"])
    per = nant * nchan * npol * 2
    n = (os.path.getsize(path) - HEADER_SIZE) // per
    return np.memmap(path, dtype=np.int8, mode="r", offset=HEADER_SIZE, shape=(n, nant, nchan, npol, 2))


def extract_channel(path: str, channel: int, size: int, offset: int = 0, pol: int = 0,
                    hdr: Optional[dict] = None) -> np.ndarray:
    """``int8 [nant, 2*size]`` interleaved (re, im) streams of one channel and
    polarisation for every antenna, starting ``offset`` samples in -- the
    input of the correlator's DelayFinder (models/correlator.py)."""
    data = read_payload(path, hdr)
    seg = data[offset:offset + size, :, channel, pol, :]  # [size, nant, 2]
    if seg.shape[0] < size:
        raise ValueError("not enough samples in the DADA file")
    return np.ascontiguousarray(np.transpose(seg, (1, 0, 2)).reshape(seg.shape[1], 2 * size))
