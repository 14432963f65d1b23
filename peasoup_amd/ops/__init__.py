"""PyTorch-ROCm facing wrappers of the hand-written HIP kernels.

Every op takes/returns ``torch`` tensors on the current HIP device and runs on
``torch.cuda.current_stream()``, so it composes with torch code and graph
capture.  The native extension must be loaded: there is no silent CPU
fallback (a missing/unbuilt extension raises at import).
"""
from .core import (  # noqa: F401
    FFTPlanCache,
    coincidence_counts,
    coincidence_mask,
    conjugate,
    cmul_,
    convert_pad,
    dedisperse,
    deredden,
    fft4_resample_interbin,
    fft4_spectrum_pass,
    spec_unblock,
    spec_pblk_index,
    fft4_resample_spectrum,
    fold_optimise,
    fold_series,
    form_amplitude,
    form_interbin,
    harmonic_peaks,
    harmonic_sums,
    interbin_normalise,
    interbin_stats,
    irfft,
    median_scrunch5,
    normalise,
    quantize_q8,
    r2c_interbin_normalise,
    resample,
    resample_v1,
    rfft,
    running_median,
    unpack_transpose,
)
