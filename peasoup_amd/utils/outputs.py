"""Python 3 readers for peasoup outputs (overview.xml, candidates.peasoup).

Parity with tools/peasoup_tools.py:14-412 (Python 2: OverviewFile,
CandidateFileParser, PeasoupOutput) -- rewritten on the standard library
(xml.etree) + numpy; lxml and sigpyproc are not required.
"""
from __future__ import annotations

import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

POD_DTYPE = np.dtype([("dm", "<f4"), ("dm_idx", "<i4"), ("acc", "<f4"), ("nh", "<i4"), ("snr", "<f4"),
                      ("freq", "<f4")])
assert POD_DTYPE.itemsize == 24


def radec_to_str(val: float) -> str:
    """hhmmss.ss-style float -> 'hh:mm:ss.ssss' (peasoup_tools.radec_to_str)."""
    sign = -1 if val < 0 else 1
    frac, integral = np.modf(abs(val))
    xx = (integral - (integral % 10000)) / 10000
    yy = ((integral - (integral % 100)) / 100) - xx * 100
    zz = integral - 100 * yy - 10000 * xx + frac
    return "%02d:%02d:%s" % (sign * xx, yy, "%07.4f" % zz)


class OverviewFile:
    """Parsed overview.xml.  Tolerates an invalid <username> (the reference
    tool strips it on a parse error)."""

    fields = [("period", float), ("opt_period", float), ("dm", float), ("acc", float), ("nh", int), ("snr", float),
              ("folded_snr", float), ("is_adjacent", int), ("is_physical", int), ("ddm_count_ratio", float),
              ("ddm_snr_ratio", float), ("nassoc", int), ("byte_offset", int)]

    def __init__(self, path: str):
        self.path = path
        text = open(path, "r", encoding="latin-1").read()
        try:
            self.root = ET.fromstring(text)
        except ET.ParseError:
            a = text.find("<username>") + len("<username>")
            b = text.find("</username>")
            self.root = ET.fromstring(text[:a] + "pulsar" + text[b:])
        self._cands = self.root.find("candidates").findall("candidate")

    def section(self, name: str) -> Dict[str, str]:
        el = self.root.find(name)
        return {c.tag: (c.text or "") for c in el} if el is not None else {}

    @property
    def dm_list(self) -> List[float]:
        return [float(t.text) for t in self.root.find("dedispersion_trials").findall("trial")]

    @property
    def acc_list(self) -> List[float]:
        return [float(t.text) for t in self.root.find("acceleration_trials").findall("trial")]

    @property
    def execution_times(self) -> Dict[str, float]:
        return {k: float(v) for k, v in self.section("execution_times").items()}

    def __len__(self) -> int:
        return len(self._cands)

    def get_candidate(self, idx: int) -> Dict:
        c = self._cands[idx]
        d = {"cand_num": int(c.attrib["id"])}
        for tag, typ in self.fields:
            el = c.find(tag)
            d[tag] = typ(float(el.text)) if typ is int else typ(el.text)
        return d

    @property
    def header(self) -> Dict[str, str]:
        """The <header_parameters> section (tag -> text)."""
        return self.section("header_parameters")

    def get_candidate_data(self, idx: int) -> "CandidateFileParser":
        """Parser of the candidate file that holds record ``idx`` (the
        reference opens ``candidates.peasoup`` in the working directory,
        peasoup_tools.py:149-151; here the one beside this overview file).
        Read record ``idx`` with ``.cand_from_offset(get_candidate(idx)["byte_offset"])``."""
        import os

        self.get_candidate(idx)  # (IndexError for a missing candidate, as the reference)
        return CandidateFileParser(os.path.join(os.path.dirname(os.path.abspath(self.path)), "candidates.peasoup"))

    def make_predictor(self, idx: int) -> str:
        """Ephemeris-style predictor of candidate ``idx`` (SOURCE, PERIOD, DM,
        ACC, RA, DEC), peasoup_tools.py:153-164.  The reference reads the
        candidate fields as float32 before formatting; so does this."""
        c = self._cands[idx]
        f32 = lambda tag: float(np.float32(c.find(tag).text))  # noqa: E731
        hdr = self.header
        return "\n".join(("SOURCE: %s" % hdr.get("source_name", ""),
                          "PERIOD: %.15f" % f32("period"),
                          "DM: %.3f" % f32("dm"),
                          "ACC: %.3f" % f32("acc"),
                          "RA: %s" % radec_to_str(float(hdr.get("src_raj", "0") or 0)),
                          "DEC: %s" % radec_to_str(float(hdr.get("src_dej", "0") or 0))))

    def as_array(self) -> np.ndarray:
        dt = [("cand_num", "i4")] + [(t, "f8" if ty is float else "i8") for t, ty in self.fields]
        arr = np.zeros(len(self), dtype=dt)
        for i in range(len(self)):
            d = self.get_candidate(i)
            for k in arr.dtype.names:
                arr[i][k] = d[k]
        return arr


class CandidateFileParser:
    """Reads records of candidates.peasoup by byte offset."""

    def __init__(self, path: str):
        self.buf = open(path, "rb").read()

    def cand_from_offset(self, offset: int) -> Tuple[Optional[np.ndarray], np.ndarray]:
        b = self.buf
        fold = None
        if b[offset: offset + 4] == b"FOLD":
            nbins, nints = struct.unpack_from("<ii", b, offset + 4)
            off = offset + 12
            fold = np.frombuffer(b, dtype="<f4", count=nbins * nints, offset=off).reshape(nints, nbins)
            off += 4 * nbins * nints
        else:
            off = offset
        (count,) = struct.unpack_from("<i", b, off)
        hits = np.frombuffer(b, dtype=POD_DTYPE, count=count, offset=off + 4)
        return fold, hits

    def records(self) -> List[Tuple[int, Optional[np.ndarray], np.ndarray]]:
        out = []
        off = 0
        while off < len(self.buf):
            fold, hits = self.cand_from_offset(off)
            out.append((off, fold, hits))
            off += (12 + fold.size * 4 if fold is not None else 0) + 4 + hits.size * 24
        return out


@dataclass
class Candidate:
    info: Dict
    fold: Optional[np.ndarray]
    hits: np.ndarray


class PeasoupOutput:
    def __init__(self, overview_file: str, candidate_file: str):
        self.overview = OverviewFile(overview_file)
        self.cands = CandidateFileParser(candidate_file)

    def __len__(self) -> int:
        return len(self.overview)

    def get_candidate(self, idx: int) -> Candidate:
        d = self.overview.get_candidate(idx)
        fold, hits = self.cands.cand_from_offset(d["byte_offset"])
        return Candidate(d, fold, hits)

    def as_text(self) -> str:
        a = self.overview.as_array()
        lines = ["#cand period opt_period dm acc nh snr folded_snr is_adjacent is_physical ddm_count ddm_snr nassoc"]
        for r in a:
            lines.append(f"{r['cand_num']:d} {r['period']:.12f} {r['opt_period']:.12f} {r['dm']:.3f} {r['acc']:.3f} "
                         f"{r['nh']:d} {r['snr']:.2f} {r['folded_snr']:.2f} {r['is_adjacent']:d} {r['is_physical']:d} "
                         f"{r['ddm_count_ratio']:.4f} {r['ddm_snr_ratio']:.4f} {r['nassoc']:d}")
        return "\n".join(lines)
