"""Antenna-delay finder by FFT cross-correlation (include/transforms/
correlator.hpp:33-92, DelayFinder; reference tool `accmap`).

Input: ``narrays`` complex 8-bit streams (interleaved int8 re/im, ``size``
complex samples each).  For every pair (i < j): C2C FFT both, conjugate X_i,
multiply into X_j, inverse FFT, and take the lag of max |.|^2 over
[-max_delay, max_delay).  The reference copies both ends of the correlation
to the host and argmaxes there; here the window is gathered on the device
and only the argmax returns.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch

from .. import ops
from ..ops.core import FFTPlanCache, _s


def _c2c(x: torch.Tensor, inverse: bool) -> torch.Tensor:
    n = x.shape[-1]
    out = torch.empty_like(x)
    FFTPlanCache.get("c2c_inv" if inverse else "c2c_fwd", n, 1).execute(x.data_ptr(), out.data_ptr(), _s())
    return out


def find_delays(arrays: np.ndarray, max_delay: int) -> Dict[Tuple[int, int], int]:
    """arrays: int8 [narrays, 2*size] (re, im interleaved).  Returns
    {(i, j): lag} where lag in [-max_delay, max_delay)."""
    a = torch.from_numpy(np.ascontiguousarray(arrays)).cuda()
    narr, twice = a.shape
    size = twice // 2
    spectra = []
    for i in range(narr):
        z = torch.view_as_complex(a[i].to(torch.float32).view(size, 2).contiguous()).contiguous()
        spectra.append(_c2c(z, inverse=False))
    out = {}
    for i in range(narr):
        xi = ops.conjugate(spectra[i].clone())
        for j in range(i + 1, narr):
            y = ops.cmul_(xi, spectra[j].clone())
            corr = _c2c(y, inverse=True)
            win = torch.cat([corr[:max_delay], corr[size - max_delay:]])
            k = int(torch.argmax(win.real ** 2 + win.imag ** 2).item())
            out[(i, j)] = k if k < max_delay else k - 2 * max_delay
    return out
