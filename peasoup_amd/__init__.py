"""peasoup_amd: MI355X-native pulsar acceleration search (peasoup capabilities).

C++/HIP core (``peasoup_amd._C``) for gfx950 + a PyTorch-ROCm facing Python
layer.  ``torch`` is imported first so that the extension binds to the HIP
runtime torch already loaded (one runtime per process).
"""
from __future__ import annotations

import torch  # noqa: F401  (must precede _C: share torch's HIP runtime)

__version__ = "0.1.0"

try:
    from . import _C  # noqa: F401
except ImportError as exc:  # pragma: no cover - exercised only when unbuilt
    raise ImportError(
        "peasoup_amd native extension is not built; run `python peasoup_amd/_build.py` "
        f"(hipcc/gfx950) first: {exc}"
    ) from exc

NativeError = _C.NativeError


DEDISP_KERNELS = ("auto", "mfma", "valu", "direct", "packed2")


def dedisp_kernel(name: str):
    """``--dedisp_kernel`` name -> ``_C.DedispKernel`` (the one map every
    driver uses; the names are the native parser's, cli.cpp)."""
    table = {"auto": _C.DedispKernel.Auto, "mfma": _C.DedispKernel.Mfma, "valu": _C.DedispKernel.Valu,
             "direct": _C.DedispKernel.Direct, "packed2": _C.DedispKernel.Packed2}
    try:
        return table[str(name).lower()]
    except KeyError:
        raise ValueError(f"unknown dedispersion kernel {name!r}; one of {', '.join(DEDISP_KERNELS)}") from None


def native_library_path() -> str:
    """Filesystem path of the loaded native extension."""
    return _C.__file__


def gpu_available() -> bool:
    """True when a HIP device is visible to this process."""
    return torch.cuda.is_available() and torch.cuda.device_count() > 0
