"""Op implementations (see package docstring)."""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import _C

K = _C.kernels


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a HIP (cuda) tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _cplx_ptr(t: torch.Tensor) -> int:
    _check(t, torch.complex64, "complex tensor")
    return t.data_ptr()


# ------------------------------------------------------------------ dedisp --
def unpack_transpose(packed: torch.Tensor, nsamps: int, nchans: int, nbits: int, bias: int = 0,
                     stride: Optional[int] = None) -> torch.Tensor:
    """Packed SIGPROC bytes -> int8 [nchans, stride] (value - bias)."""
    _check(packed, torch.uint8, "packed")
    stride = stride or nsamps
    out = torch.zeros((nchans, stride), dtype=torch.int8, device=packed.device)
    K.unpack_transpose(packed.data_ptr(), nsamps, nchans, nbits, out.data_ptr(), stride, bias, _s())
    return out


def dedisperse(chan_major: torch.Tensor, offsets: torch.Tensor, out_nsamps: int, scale: float, bias: int = 0,
               killmask: Optional[torch.Tensor] = None, kernel: str = "direct") -> torch.Tensor:
    """Brute-force dedispersion of an int8 [nchans, stride] block.

    offsets: int32 [ndm, nchans] sample delays.  Returns uint8 [ndm, out_nsamps].
    kernel: "direct" (VALU) or "mfma" (v_mfma_i32_32x32x32_i8 one-hot GEMM).
    """
    _check(chan_major, torch.int8, "chan_major")
    nchans, stride = chan_major.shape
    ndm = offsets.shape[0]
    dev = chan_major.device
    kill = killmask if killmask is not None else torch.ones(nchans, dtype=torch.int32, device=dev)
    nactive = int(kill.ne(0).sum())
    out = torch.empty((ndm, out_nsamps), dtype=torch.uint8, device=dev)
    if kernel == "direct":
        offs = offsets.to(dev, torch.int32).contiguous()
        K.dedisperse_direct(chan_major.data_ptr(), stride, nchans, offs.data_ptr(), kill.to(dev, torch.int32).contiguous().data_ptr(),
                            ndm, out_nsamps, out.data_ptr(), out_nsamps, float(scale), int(bias), nactive, _s())
        return out
    raise ValueError("mfma dedispersion is driven through _C.Dedisperser (needs padded rows)")


# ------------------------------------------------------------ time series --
def convert_pad(trial: torch.Tensor, n: int) -> torch.Tensor:
    """uint8 trial -> float32[n]: copy (truncate) or pad with the trial mean."""
    _check(trial, torch.uint8, "trial")
    out = torch.empty(n, dtype=torch.float32, device=trial.device)
    tmp = torch.zeros(1, dtype=torch.int64, device=trial.device)
    K.u8_to_f32_pad(trial.data_ptr(), min(trial.numel(), n), out.data_ptr(), n, tmp.data_ptr(), _s())
    return out


# ------------------------------------------------------------------ FFT -----
class FFTPlanCache:
    """rocFFT plan cache keyed by (type, n, batch)."""

    _plans: Dict[Tuple, object] = {}

    @classmethod
    def get(cls, kind: str, n: int, batch: int = 1):
        key = (kind, n, batch, torch.cuda.current_device())
        p = cls._plans.get(key)
        if p is None:
            t = {"r2c": _C.FftType.R2C, "c2r": _C.FftType.C2R, "c2c_fwd": _C.FftType.C2C_FWD,
                 "c2c_inv": _C.FftType.C2C_INV}[kind]
            p = _C.FftPlan(t, n, batch)
            cls._plans[key] = p
        return p


def rfft(x: torch.Tensor) -> torch.Tensor:
    """Unnormalised real-to-complex FFT over the last dim (rocFFT)."""
    _check(x, torch.float32, "x")
    n = x.shape[-1]
    batch = x.numel() // n
    out = torch.empty(x.shape[:-1] + (n // 2 + 1,), dtype=torch.complex64, device=x.device)
    FFTPlanCache.get("r2c", n, batch).execute(x.data_ptr(), out.data_ptr(), _s())
    return out


def irfft(X: torch.Tensor, n: int) -> torch.Tensor:
    """Unnormalised complex-to-real inverse FFT (cuFFT/rocFFT convention: x*n)."""
    Xc = X.contiguous().clone()  # C2R may overwrite its input
    batch = Xc.numel() // (n // 2 + 1)
    out = torch.empty(X.shape[:-1] + (n,), dtype=torch.float32, device=X.device)
    FFTPlanCache.get("c2r", n, batch).execute(_cplx_ptr(Xc), out.data_ptr(), _s())
    return out


# --------------------------------------------------------------- spectra ----
def form_amplitude(X: torch.Tensor) -> torch.Tensor:
    out = torch.empty(X.numel(), dtype=torch.float32, device=X.device)
    K.form_amplitude(_cplx_ptr(X), X.numel(), out.data_ptr(), _s())
    return out


def form_interbin(X: torch.Tensor) -> torch.Tensor:
    out = torch.empty(X.numel(), dtype=torch.float32, device=X.device)
    K.form_interbin(_cplx_ptr(X), X.numel(), out.data_ptr(), _s())
    return out


def normalise(x: torch.Tensor, mean: float, sigma: float) -> torch.Tensor:
    _check(x, torch.float32, "x")
    K.normalise(x.data_ptr(), x.numel(), float(mean), float(sigma), _s())
    return x


def median_scrunch5(x: torch.Tensor, from_complex: bool = False) -> torch.Tensor:
    n = x.numel()
    out = torch.empty(max(1, n // 5), dtype=torch.float32, device=x.device)
    if from_complex:
        K.median5_amp(_cplx_ptr(x), n, out.data_ptr(), _s())
    else:
        _check(x, torch.float32, "x")
        K.median5(x.data_ptr(), n, out.data_ptr(), _s())
    return out


def running_median(X: torch.Tensor):
    """The three median scrunches of Dereddener::calculate_median."""
    m5 = median_scrunch5(X, from_complex=True)
    m25 = median_scrunch5(m5)
    m125 = median_scrunch5(m25)
    return m5, m25, m125


def deredden(X: torch.Tensor, bin_width: float, zapmask: Optional[torch.Tensor] = None,
             boundary5: float = 0.05, boundary25: float = 0.5) -> torch.Tensor:
    """In place: X /= running median (bins < 5 -> 0), zapped bins -> 1+0i."""
    nb = X.numel()
    m5, m25, m125 = running_median(X)
    pos5 = int(float(torch.tensor(boundary5, dtype=torch.float32) / torch.tensor(bin_width, dtype=torch.float32)))
    pos25 = int(float(torch.tensor(boundary25, dtype=torch.float32) / torch.tensor(bin_width, dtype=torch.float32)))
    zp = 0
    if zapmask is not None:
        _check(zapmask, torch.int32, "zapmask")
        zp = zapmask.data_ptr()
    K.deredden_zap(_cplx_ptr(X), nb, m5.data_ptr(), nb // 5, m25.data_ptr(), max(1, nb // 25), m125.data_ptr(),
                   max(1, nb // 125), pos5, pos25, zp, _s())
    return X


def interbin_stats(X: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Interbinned spectrum + device stats {mean, rms, std}."""
    P = torch.empty(X.numel(), dtype=torch.float32, device=X.device)
    partials = torch.empty(2048, dtype=torch.float64, device=X.device)
    st = torch.empty(4, dtype=torch.float32, device=X.device)
    K.interbin_stats(_cplx_ptr(X), X.numel(), P.data_ptr(), partials.data_ptr(), 1024, st.data_ptr(), _s())
    return P, st


def interbin_normalise(X: torch.Tensor, stats: torch.Tensor, nscale: float, nbins_out: Optional[int] = None):
    """Batched: X complex [K, B] -> (interbin(X) - mean*nscale)/(std*nscale)."""
    Kb, nb = X.shape
    nbo = nbins_out or nb
    P = torch.empty((Kb, nbo), dtype=torch.float32, device=X.device)
    K.interbin_normalise_batch(_cplx_ptr(X), nb, nb, P.data_ptr(), nbo, Kb, nbo, stats.data_ptr(), float(nscale), _s())
    return P


def r2c_interbin_normalise(x: torch.Tensor, stats: torch.Tensor, nscale: float,
                           nbins_out: Optional[int] = None) -> torch.Tensor:
    """Batched real series x [K, N] (N even) -> same output as
    ``interbin_normalise(rfft(x))`` but via an N/2-point complex FFT of the
    packed series with the real-FFT post-processing fused into the kernel."""
    _check(x, torch.float32, "x")
    Kb, n = x.shape
    assert n % 2 == 0
    M = n // 2
    Z = torch.fft.fft(torch.view_as_complex(x.contiguous().view(Kb, M, 2)), dim=-1).contiguous()
    nbo = nbins_out or (M + 1)
    P = torch.empty((Kb, nbo), dtype=torch.float32, device=x.device)
    K.r2c_interbin_normalise_batch(_cplx_ptr(Z), M, M, M.bit_length() - 1, M, 8, 3, P.data_ptr(), nbo, Kb, nbo,
                                   stats.data_ptr(), float(nscale), _s())
    return P


# ---------------------------------------------------------- acceleration ---
def resample(x: torch.Tensor, accels: Sequence[float], tsamp: float) -> torch.Tensor:
    """Batched time-domain acceleration resampling (resampleII semantics)."""
    _check(x, torch.float32, "x")
    n = x.numel()
    af = torch.tensor([(float(torch.tensor(a, dtype=torch.float32)) * float(torch.tensor(tsamp, dtype=torch.float32)))
                       / (2 * 299792458.0) for a in accels], dtype=torch.float64, device=x.device)
    stride = (n + 3) // 4 * 4
    out = torch.empty((len(accels), stride), dtype=torch.float32, device=x.device)
    K.resample_batch(x.data_ptr(), n, out.data_ptr(), stride, af.data_ptr(), len(accels), _s())
    return out[:, :n]


def _accel_factors(accels: Sequence[float], tsamp: float, device) -> torch.Tensor:
    return torch.tensor([(float(torch.tensor(a, dtype=torch.float32)) * float(torch.tensor(tsamp, dtype=torch.float32)))
                         / (2 * 299792458.0) for a in accels], dtype=torch.float64, device=device)


def _fft4_padded(x: torch.Tensor, accels: Sequence[float], tsamp: float, nbins_out: int = 0):
    _check(x, torch.float32, "x")
    n = x.numel()
    g = K.fft4_geometry(n // 2)
    if not g.ok or n % 2:
        raise ValueError(f"fft4: unsupported length {n}")
    tab = torch.from_numpy(K.fft4_tables(g)).to(x.device)
    af = _accel_factors(accels, tsamp, x.device)
    Kb = len(accels)
    xp = torch.empty(g.insize, dtype=torch.float32, device=x.device)
    Y = torch.empty((Kb, g.ystride, 2), dtype=torch.float32, device=x.device)
    X = torch.empty((Kb, g.xstride, 2), dtype=torch.float32, device=x.device)
    K.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, _s())
    K.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), Kb, Y.data_ptr(), g, tab.data_ptr(), _s())
    K.fft4_rowpass(Y.data_ptr(), X.data_ptr(), Kb, g, tab.data_ptr(), _s(), nbins_out)
    return g, X


def fft4_x_layout(g):
    """(log2_row, row_pitch, blk_pitch, log2_blk, tiled) of the fused FFT's
    spectrum layout under the current kernel flags."""
    return K.fft4_x_layout(g)


def fft4_resample_spectrum(x: torch.Tensor, accels: Sequence[float], tsamp: float) -> torch.Tensor:
    """Fused resample + four-step FFT: returns Z [K, N/2] complex64 with
    Z[k] = FFT_{N/2}(z_k), z_k[m] = r_k[2m] + i r_k[2m+1], r_k = resample(x, accels[k])."""
    g, X = _fft4_padded(x, accels, tsamp)
    Kb = X.shape[0]
    M = g.n1 * g.n2
    log2_row, row, blk, lw, tiled = fft4_x_layout(g)
    k = torch.arange(M, device=x.device, dtype=torch.int64)
    k2 = k & (g.n2 - 1)
    k1 = k >> log2_row
    if tiled:
        addr = (k2 >> 3) * (8 * g.n1) + (k1 >> 3) * 64 + (k2 & 7) * 8 + (k1 & 7)
    else:
        addr = (k2 >> lw) * blk + k1 * row + (k2 & ((1 << lw) - 1))
    Xc = torch.view_as_complex(X)  # [K, xstride]
    return Xc[:, addr].contiguous()


def fft4_resample_interbin(x: torch.Tensor, accels: Sequence[float], tsamp: float, stats: torch.Tensor,
                           nscale: float, nbins_out: int | None = None, screen: bool = False):
    """The search hot path of fft_mode 2: fused resample + four-step FFT, then
    the paired real-FFT post-processing + interbin + normalise on the fused
    FFT's spectrum layout.  Returns P [K, N/2 + 1]; with ``nbins_out`` only
    bins below it are formed (pass B then stores only the spectrum rows the
    r2c step reads, as the search engine does) and the rest stay zero.  With
    ``screen`` (tiled layout only) returns (P, Q): Q [K, qstride] uint8 the
    screening bytes the r2c kernel writes for the harmonic sum."""
    M = (x.numel()) // 2
    nbo = M + 1 if nbins_out is None else int(nbins_out)
    g, X = _fft4_padded(x, accels, tsamp, nbins_out=0 if nbins_out is None else nbo)
    Kb = X.shape[0]
    log2_row, row, blk, lw, tiled = fft4_x_layout(g)
    P = torch.zeros((Kb, M + 1), dtype=torch.float32, device=x.device)
    if screen and not tiled:
        raise ValueError("screening bytes come from the tiled r2c kernel only")
    if tiled:
        qst = (M + 1 + 63) // 64 * 64
        Q = torch.zeros((Kb, qst), dtype=torch.uint8, device=x.device) if screen else None
        K.r2c_interbin_normalise_tiled(X.data_ptr(), g.n1, g.n2, g.xstride, P.data_ptr(), M + 1, Kb, nbo,
                                       stats.data_ptr(), float(nscale), _s(), Q.data_ptr() if screen else 0,
                                       qst if screen else 0)
        if screen:
            return P, Q
    else:
        K.r2c_interbin_normalise_batch(X.data_ptr(), M, g.xstride, log2_row, row, blk, lw, P.data_ptr(), M + 1, Kb,
                                       nbo, stats.data_ptr(), float(nscale), _s())
    return P


def fft4_spectrum_pass(x: torch.Tensor, accels: Sequence[float], tsamp: float, stats: torch.Tensor,
                       nscale: float, pair_y: bool | None = None, nbins: int = 0):
    """The search hot path with the fused spectrum pass (the default engine
    path): fused resample + pass A, then pass B forming the normalised
    interbinned spectrum and its screening bytes directly
    (kernels.hpp fft4_rowpass_spectrum).  Returns (Pb, Q, g): Pb [K, pstride]
    in the blocked layout (``spec_unblock`` gives natural order), Q [K,
    qstride] uint8 with bin b at column ``spec_q_shift`` + b.  ``pair_y``:
    pass A hands over Y in row pairs (default: where ``fft4_pair_y`` allows,
    as the search engine does).  ``nbins`` > 0: only bins below it are
    written (whole 4-bin groups; the rest of Pb / Q keeps its zeros)."""
    _check(x, torch.float32, "x")
    n = x.numel()
    g = K.fft4_geometry(n // 2)
    if not g.ok or n % 2:
        raise ValueError(f"fft4: unsupported length {n}")
    M = g.n1 * g.n2
    g.ypair = K.fft4_pair_y(g) if pair_y is None else bool(pair_y)
    tab = torch.from_numpy(K.fft4_tables(g)).to(x.device)
    af = _accel_factors(accels, tsamp, x.device)
    Kb = len(accels)
    xp = torch.empty(g.insize, dtype=torch.float32, device=x.device)
    Y = torch.empty((Kb, g.ystride, 2), dtype=torch.float32, device=x.device)
    K.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, _s())
    K.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), Kb, Y.data_ptr(), g, tab.data_ptr(), _s())
    pst = (M + 1 + 63) // 64 * 64
    qst = (M + 1 + K.spec_q_shift + 63) // 64 * 64
    Pb = torch.zeros((Kb, pst), dtype=torch.float32, device=x.device)
    Q = torch.zeros((Kb, qst), dtype=torch.uint8, device=x.device)
    K.fft4_rowpass_spectrum(Y.data_ptr(), Kb, g, tab.data_ptr(), Pb.data_ptr(), pst, Q.data_ptr(), qst,
                            stats.data_ptr(), float(nscale), _s(), 0, int(nbins))
    return Pb, Q, g


def spec_pblk_index(b: torch.Tensor, log2_n2: int, n1: int) -> torch.Tensor:
    """kernels.hpp spec_pblk_index, vectorised: position of bins b (int64,
    0..M) in the blocked spectrum of ``fft4_spectrum_pass``."""
    n2 = 1 << log2_n2
    M = n1 * n2
    r = b & (n2 - 1)
    prim = (r >= 1) & (r <= n2 // 2)
    ip = (((r - 1) >> 2) * 2 * n1 + (b >> log2_n2)) * 4 + ((r - 1) & 3)
    bm = M - b
    rm = bm & (n2 - 1)
    im = (((rm >> 2) * 2 + 1) * n1 + (bm >> log2_n2)) * 4 + (rm & 3)
    out = torch.where(prim, ip, im)
    return torch.where(b == 0, torch.full_like(b, M), out)


def spec_unblock(Pb: torch.Tensor, g) -> torch.Tensor:
    """Natural-order P [K, M + 1] from the blocked spectrum of ``fft4_spectrum_pass``."""
    M = g.n1 * g.n2
    b = torch.arange(M + 1, device=Pb.device, dtype=torch.int64)
    return Pb[:, spec_pblk_index(b, g.log2_xrow, g.n1)]


def resample_v1(x: torch.Tensor, accel: float, tsamp: float) -> torch.Tensor:
    _check(x, torch.float32, "x")
    af = (float(torch.tensor(accel, dtype=torch.float32)) * float(torch.tensor(tsamp, dtype=torch.float32))) / (2 * 299792458.0)
    out = torch.empty_like(x)
    K.resample_v1(x.data_ptr(), x.numel(), out.data_ptr(), af, _s())
    return out


def harmonic_sums(P: torch.Tensor, nlevels: int) -> torch.Tensor:
    """Materialised harmonic sums [nlevels, n] (debug/test path)."""
    _check(P, torch.float32, "P")
    out = torch.empty((max(1, nlevels), P.numel()), dtype=torch.float32, device=P.device)
    K.harmonic_sums(P.data_ptr(), P.numel(), nlevels, out.data_ptr(), _s())
    return out[:nlevels]


def quantize_q8(P: torch.Tensor) -> torch.Tensor:
    """Screening bytes (device_common.hpp dev::q8) of spectra P [K, n]:
    [K, qstride] uint8, qstride = n rounded up to 64."""
    _check(P, torch.float32, "P")
    Kb, n = P.shape
    qst = (n + 63) // 64 * 64
    Q = torch.zeros((Kb, qst), dtype=torch.uint8, device=P.device)
    K.quantize_q8(P.data_ptr(), n, n, Kb, Q.data_ptr(), qst, _s())
    return Q


def harmonic_peaks(P: torch.Tensor, nlevels: int, starts: Sequence[int], ends: Sequence[int], thresh: float,
                   capacity: int = 1 << 20, nbins: int | None = None, Q: torch.Tensor | None = None,
                   pblk=None):
    """Fused harmonic sum + threshold: P [K, n] -> records (trial, level, idx, snr)
    as int64/float32 tensors sorted by (trial, level, idx) (the kernel's chunk
    descriptors, kernels.hpp kPeakChunk, are dropped).  ``nbins``: bins per
    spectrum when the rows are padded (default n).  ``Q``: screening bytes of
    P ([K, qstride] uint8, ``quantize_q8``) -- the screened kernel, same
    records.  ``pblk`` = the geometry ``g`` of ``fft4_spectrum_pass``: P is
    its blocked spectrum and Q its screening rows (bins shifted by
    ``spec_q_shift``)."""
    _check(P, torch.float32, "P")
    Kb, n = P.shape
    rec = torch.empty((capacity, 3), dtype=torch.int32, device=P.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=P.device)
    nb = n if nbins is None else int(nbins)
    if Q is not None:
        if Q.dtype != torch.uint8 or Q.shape[0] != Kb or not Q.is_contiguous():
            raise ValueError("Q must be a contiguous [K, qstride] uint8 tensor")
    extra = {}
    if pblk is not None:
        extra = dict(pblk_log2_n2=pblk.log2_xrow, pblk_n1=pblk.n1, qshift=K.spec_q_shift)
    K.harmonic_peaks_batch(P.data_ptr(), nb, n, Kb, nlevels, list(starts), list(ends), float(thresh), capacity,
                           rec.data_ptr(), cnt.data_ptr(), _s(), 0 if Q is None else Q.data_ptr(),
                           0 if Q is None else Q.shape[1], **extra)
    c = int(cnt.item())
    if c > capacity:
        return harmonic_peaks(P, nlevels, starts, ends, thresh, capacity=c + 1024, nbins=nbins, Q=Q, pblk=pblk)
    r = rec[:c]
    r = r[r[:, 0] >= 0]  # drop the chunk descriptors (seg field with kPeakChunk, bit 31, set)
    seg = r[:, 0].to(torch.int64)
    idx = r[:, 1].to(torch.int64)
    snr = r[:, 2].view(torch.float32)
    order = torch.argsort(seg * (1 << 32) + idx)
    return seg[order] // 8, seg[order] % 8, idx[order], snr[order]


# --------------------------------------------------------------- folding ----
def fold_series(series: torch.Tensor, periods: Sequence[float], accels: Sequence[float], tsamp: float):
    """Fold + optimise a whitened series for several (period, accel) pairs.
    Returns native FoldResult objects (folded_snr, opt_period, fold[16*64], ...)."""
    _check(series, torch.float32, "series")
    fe = _C.FoldEngine(series.numel(), float(tsamp), _s())
    return fe.fold_series(series.data_ptr(), [float(p) for p in periods], [float(a) for a in accels])


def fold_optimise(folds: torch.Tensor):
    """Fused fold optimiser on [nfold, 16, 64] folds -> (opt_int[nfold,3], opt_fold, opt_prof)."""
    _check(folds, torch.float32, "folds")
    nf = folds.shape[0]
    dev = folds.device
    table = torch.empty((64, 16, 64), dtype=torch.complex64, device=dev)
    K.fold_shift_table(table.data_ptr(), 64, 16, _s())
    of = torch.empty_like(folds)
    op = torch.empty((nf, 64), dtype=torch.float32, device=dev)
    oi = torch.empty((nf, 3), dtype=torch.int32, device=dev)
    ov = torch.empty(nf, dtype=torch.float32, device=dev)
    K.fold_optimise(folds.data_ptr(), nf, table.data_ptr(), of.data_ptr(), op.data_ptr(), oi.data_ptr(), ov.data_ptr(), _s())
    return oi, of, op


# ----------------------------------------------------------- coincidence ----
def coincidence_counts(x: torch.Tensor, thresh: float, counts: Optional[torch.Tensor] = None) -> torch.Tensor:
    _check(x, torch.float32, "x")
    if counts is None:
        counts = torch.zeros(x.numel(), dtype=torch.uint8, device=x.device)
    K.count_above(x.data_ptr(), x.numel(), float(thresh), counts.data_ptr(), _s())
    return counts


def coincidence_mask(counts: torch.Tensor, beam_thresh: int) -> torch.Tensor:
    _check(counts, torch.uint8, "counts")
    mask = torch.empty(counts.numel(), dtype=torch.float32, device=counts.device)
    K.coincidence_mask(counts.data_ptr(), counts.numel(), int(beam_thresh), mask.data_ptr(), _s())
    return mask


# ----------------------------------------------------------- correlation ----
def conjugate(x: torch.Tensor) -> torch.Tensor:
    K.conjugate(_cplx_ptr(x), x.numel(), _s())
    return x


def cmul_(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """y <- x * y (complex, in place)."""
    K.cmul_inplace(_cplx_ptr(x), _cplx_ptr(y), y.numel(), _s())
    return y
