"""Seeded synthetic filterbanks with injected (accelerated) pulsars.

Used by the tests and benchmarks (there is no network access to real data).
The generator produces quantised Gaussian noise plus a dispersed periodic
pulse train whose arrival times follow the same dispersion law the pipeline
searches for (delay_c = 4.15e3 * DM * (1/f_c^2 - 1/f_1^2) s), optionally with
a constant line-of-sight acceleration (phase = (t - a t^2/(2c)) / P, a > 0 away).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np

from .sigproc import pack_samples, write_filterbank

C_LIGHT = 299792458.0


@dataclass
class PulsarSpec:
    period: float = 0.25        # s
    dm: float = 30.0            # pc cm^-3
    duty: float = 0.05          # pulse FWHM as a fraction of the period
    amplitude: float = 1.0      # peak in units of the per-channel noise sigma
    accel: float = 0.0          # m/s^2
    phase: float = 0.0


def make_header(nchans: int = 64, nbits: int = 2, tsamp: float = 320e-6, fch1: float = 1510.0,
                foff: float = -1.09, nsamples: int = 0, source_name: str = "synthetic") -> Dict:
    return {"source_name": source_name, "tsamp": tsamp, "fch1": fch1, "foff": foff, "nchans": nchans,
            "nbits": nbits, "nifs": 1, "data_type": 1, "tstart": 50000.0, "nsamples": nsamples}


def generate(nsamps: int, header: Dict, pulsars=(), seed: int = 0, chunk: int = 1 << 16) -> np.ndarray:
    """Return [nsamps, nchans] uint8 quantised samples (values < 2^nbits)."""
    rng = np.random.default_rng(seed)
    nchans = int(header["nchans"])
    nbits = int(header["nbits"])
    tsamp = float(header["tsamp"])
    fch1 = float(header["fch1"])
    foff = float(header["foff"])
    freqs = fch1 + foff * np.arange(nchans)
    levels = (1 << nbits) - 1
    # Gaussian noise mapped to the quantiser: mean mid-scale, sigma ~ levels/4
    mean = levels / 2.0
    sigma = max(levels / 4.0, 0.5)
    out = np.empty((nsamps, nchans), dtype=np.uint8)
    for t0 in range(0, nsamps, chunk):
        t1 = min(nsamps, t0 + chunk)
        x = rng.standard_normal((t1 - t0, nchans)).astype(np.float32)
        t = (np.arange(t0, t1, dtype=np.float64) * tsamp)[:, None]
        for p in pulsars:
            delay = 4.15e3 * p.dm * (1.0 / freqs ** 2 - 1.0 / fch1 ** 2)  # seconds
            te = t - delay[None, :]
            # +ve acceleration = away from the observer (distiller.hpp:164):
            # the apparent spin frequency drifts down
            ph = (te - p.accel * te * te / (2 * C_LIGHT)) / p.period + p.phase
            ph = ph - np.floor(ph)
            d = np.minimum(ph, 1.0 - ph)
            w = p.duty / 2.3548
            x += p.amplitude * np.exp(-0.5 * (d / w) ** 2).astype(np.float32)
        q = np.rint(mean + sigma * x)
        out[t0:t1] = np.clip(q, 0, levels).astype(np.uint8)
    return out


def write(path: str, nsamps: int, header: Optional[Dict] = None, pulsars=(), seed: int = 0) -> Dict:
    hdr = dict(header or make_header())
    hdr["nsamples"] = nsamps
    vals = generate(nsamps, hdr, pulsars, seed)
    write_filterbank(path, hdr, vals)
    return hdr


def packed(nsamps: int, header: Dict, pulsars=(), seed: int = 0) -> np.ndarray:
    return pack_samples(generate(nsamps, header, pulsars, seed), int(header["nbits"]))


def generate_packed_torch(nsamps: int, header: Dict, pulsars=(), seed: int = 0, device=None,
                          chunk: int = 1 << 15, birdies=()):
    """GPU form of :func:`packed` (same noise model, quantiser, dispersion and
    acceleration law; torch's generator instead of NumPy's, so not the same
    noise samples): packed SIGPROC bytes as a uint8 tensor on ``device``.
    ``birdies``: (frequency Hz, amplitude) sinusoids added to every channel
    (periodic RFI: strong, undispersed, many harmonics of threshold crossings).
    Minutes-long 2^23-sample, 1024-channel filterbanks take seconds."""
    import torch

    dev = torch.device(device) if device is not None else torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    nchans = int(header["nchans"])
    nbits = int(header["nbits"])
    tsamp = float(header["tsamp"])
    fch1 = float(header["fch1"])
    foff = float(header["foff"])
    levels = (1 << nbits) - 1
    mean = levels / 2.0
    sigma = max(levels / 4.0, 0.5)
    per = 8 // nbits if nbits < 8 else 1
    assert nbits in (1, 2, 4, 8) and nchans % per == 0
    freqs = fch1 + foff * torch.arange(nchans, device=dev, dtype=torch.float64)
    out = torch.empty(nsamps * nchans * nbits // 8, dtype=torch.uint8, device=dev)
    row = nchans * nbits // 8
    for t0 in range(0, nsamps, chunk):
        n = min(chunk, nsamps - t0)
        x = torch.randn((n, nchans), device=dev, generator=g)
        t = (torch.arange(t0, t0 + n, device=dev, dtype=torch.float64) * tsamp)[:, None]
        for p in pulsars:
            delay = 4.15e3 * p.dm * (1.0 / freqs ** 2 - 1.0 / fch1 ** 2)
            te = t - delay[None, :]
            ph = (te - p.accel * te * te / (2 * C_LIGHT)) / p.period + p.phase
            ph = ph - torch.floor(ph)
            d = torch.minimum(ph, 1.0 - ph)
            w = p.duty / 2.3548
            x += (p.amplitude * torch.exp(-0.5 * (d / w) ** 2)).float()
        for f, amp in birdies:
            x += (amp * torch.sin(2 * np.pi * f * t)).float()
        q = torch.clamp(torch.round(mean + sigma * x), 0, levels).to(torch.uint8)
        if nbits == 8:
            packed = q.reshape(-1)
        else:
            q = q.view(n, nchans // per, per).to(torch.int32)
            acc = torch.zeros((n, nchans // per), dtype=torch.int32, device=dev)
            for k in range(per):
                acc |= q[..., k] << (k * nbits)
            packed = acc.to(torch.uint8).reshape(-1)
        out[t0 * row:(t0 + n) * row] = packed
    return out
