// Host-side launchers for every hand-written HIP kernel (gfx950 / CDNA4).
// All launchers are asynchronous on the given stream and never synchronise.
//
// Reference kernel map (src/kernels.cu):
//   K29 conversion_kernel, K9/K10 GPU_mean/GPU_fill   -> u8_sum + u8_to_f32_pad
//   K2 power_series / K3 bin_interbin / K4 normalise  -> form_amplitude,
//        form_interbin, normalise; fused into whiten_* and interbin_normalise_batch
//   K22/K23 median_scrunch5 + linear_stretch + K24 divide_c_by_f + K25 zap
//                                                      -> median5_amp, median5,
//                                                         deredden_zap (fused)
//   K8/K9 GPU_rms/GPU_mean                            -> interbin_stats (fused
//                                                         single-pass partials)
//   K5/K6 resample_kernel(II)                         -> resample_batch, resample_v1
//   K1 harmonic_sum + K7 device_find_peaks            -> harmonic_peaks_batch
//   K13 fold_time_series                              -> fold_accumulate + fold_reduce
//   K14-K21 fold optimiser chain                      -> fold_optimise (one fused kernel)
//   K26 coincidence_kernel                            -> coincidence_*
//   K27/K28 conjugate / cuCmulf_inplace               -> conjugate, cmul_inplace
//   dedisp (external library)                         -> unpack_transpose,
//                                                        dedisperse_direct, dedisperse_mfma
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace psoup {
namespace kern {

// ---------------------------------------------------------------- records ---
// harmonic_peaks_batch output: crossings {segment, idx, snr} (segment =
// batch_item * 8 + level), each run of one (wave, 64-bin group, level)
// preceded by a chunk descriptor {kPeakChunk | count << 16 | segment, first
// idx, position of its first crossing (as the snr bits)}.
constexpr uint32_t kPeakChunk = 0x80000000u;
// Record regions (HarmParams::region_log2 = g > 0): `out` is cut into 2^g
// regions of capacity >> g records; workgroup b emits into region
// b & (2^g - 1), whose counter is count[region * kPeakRegionStride] (one
// 128-byte line each).  Chunk positions stay absolute.  One counter took
// every wave's reservation atomic in turn: ~11 ns each, 8.8 ms for the 777k
// chunks of one peak-heavy 1024-trial batch; 64 counters 0.2 ms
// (tools/expt/atomic_bench.hip, profiles/r5_regions/).
constexpr uint32_t kPeakRegionStride = 32;
struct PeakRecord {
  uint32_t seg;  // batch_item * 8 + level, or a chunk descriptor (kPeakChunk)
  int32_t idx;
  float snr;
};
static_assert(sizeof(PeakRecord) == 12, "PeakRecord layout");

constexpr int kMaxHarmLevels = 5;  // 2,4,8,16,32 harmonics (kernels.cu:42-96)

// --------------------------------------------------------- unpack/dedisp ----
// packed time-major SIGPROC data (nbits in {1,2,4,8}, LSB-first) ->
// channel-major int8 rows: out[c*out_stride + t] = value - bias.
void unpack_transpose(const uint8_t* packed, uint64_t nsamps, int nchans, int nbits, int8_t* out,
                      uint64_t out_stride, int bias, hipStream_t s);

// Direct (VALU) brute-force dedispersion, exact integer sums.
//   out[d*out_stride + t] = clip(scale * (sum_{c: kill[c]} (x[c][t + off(c,d)] + bias)))
// for d in [0, ndm), t in [0, out_nsamps).  offsets: int32 [ndm][nchans].
void dedisperse_direct(const int8_t* chan_major, uint64_t chan_stride, int nchans, const int32_t* offsets,
                       const int32_t* killmask, int ndm, uint64_t out_nsamps, uint8_t* out, uint64_t out_stride,
                       float scale, int bias, int nactive, hipStream_t s);

// MFMA dedispersion (v_mfma_i32_32x32x32_i8 over one-hot shift matrices),
// bit-identical to dedisperse_direct.  The host builds, per tile of 32 DMs,
// the list of (channel, 16-sample shift block) pairs (two per MFMA step) and
// the per-lane one-hot positions; see dedisperse.hip.
struct MfmaDedispPlan {
  int ntiles = 0;
  int max_steps = 0;               // longest tile (informational)
  std::vector<int32_t> steps;      // [total steps][4] = {c0, sb0, c1, sb1}, tiles back to back
  std::vector<int8_t> deltas;      // [total steps][64] one-hot position per lane, -1 = none
  std::vector<int32_t> tile_info;  // [ntiles][2] = {first step, step count}
};
// offsets: host int32 [ndm][nchans]; killmask: host [nchans] (0 = killed)
void build_mfma_dedisp_plan(const int32_t* offsets, int ndm, int nchans, const int32_t* killmask,
                            MfmaDedispPlan& plan);
// Reads up to 560 bytes past out_nsamps + max offset in each channel row.
// d_skip: the first tile's leading DMs before the range (not stored); out is
// the range's first DM.
void dedisperse_mfma(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_steps, const int8_t* d_deltas,
                     const int32_t* d_tile_info, int ntiles, int ndm, uint64_t out_nsamps, uint8_t* out,
                     uint64_t out_stride, float scale, int bias_total, hipStream_t s, int d_skip = 0);

// LDS-fed one-hot MFMA dedispersion (dedisperse_mfma_lds_kernel): per
// 32-DM tile and group of kMfmaLdsGroup active channels, the channel windows
// are staged in LDS and the A fragments built from there.  Tiles whose
// per-channel offset spread does not fit the kMfmaLdsWindow-byte window are
// marked tile_ok = 0 (no steps; the VALU kernels take them).  Everything a
// step needs is staged in LDS with the windows, so the MFMA loop issues no
// global or scalar loads: a 32-bit step word (two 16-bit halves, one per
// K-half of the MFMA: bits 0-3 channel slot, 4-11 window byte offset rel,
// 12 = empty half) and per channel slot the 32 DMs' window-relative offsets
// (bytes); a lane's one-hot position is relo[slot][dm] - rel.
constexpr int kMfmaLdsGroup = 16;
constexpr int kMfmaLdsWindow = 1280;
constexpr int kMfmaLdsMaxSteps = 128;  // step words staged per channel group
struct MfmaLdsPlan {
  int ntiles = 0, ngroups = 0, nactive = 0;
  std::vector<int32_t> steps;       // [total + kMfmaLdsMaxSteps] packed step words (zero padded)
  std::vector<uint8_t> relo;        // [ntiles][ngroups][kMfmaLdsGroup][32] offset - window start per DM
  std::vector<int32_t> ginfo;       // [ntiles][ngroups][2] = {first step, step count}
  std::vector<int32_t> wmin;        // [ntiles][nactive]: window start (offset, 16-byte aligned) per channel
  std::vector<int32_t> tile_ok;     // [ntiles]
  std::vector<int32_t> tile_steps;  // [ntiles] MFMA steps of the tile (0 if not ok)
};
// Tiles [tile0, tile1) of the plan (tile1 < 0: to the end; the others are
// left not-ok); offsets[(d - d_first) * nchans + c] for the DMs they cover.
void build_mfma_lds_plan(const int32_t* offsets, int ndm, int nchans, const int32_t* killmask, MfmaLdsPlan& plan,
                         int tile0 = 0, int tile1 = -1, int d_first = 0);
// Tiles [tile0, tile0 + ntiles) of a plan (pointers already offset to tile0
// for ginfo, relo and wmin; ndm DMs from the range's first): bit-identical to
// dedisperse_direct.  Rows are read up to 1280 bytes past t + wmin.
void dedisperse_mfma_lds(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_active, int nactive,
                         const int32_t* d_steps, const uint8_t* d_relo, const int32_t* d_ginfo, int ngroups,
                         const int32_t* d_wmin, int ntiles, int ndm, uint64_t out_nsamps, uint8_t* out,
                         uint64_t out_stride, float scale, int bias_total, hipStream_t s, int d_skip = 0);

// Packed-byte VALU dedispersion (wide-spread DM tiles), bit-identical to
// dedisperse_direct.  d_offT: int32 [nactive][ldo] offsets of active channel
// ci for DM column d_base + k (k < ndm rounded up to the workgroup's DM count,
// padded columns must hold valid offsets); d_active: active channel indices.
void dedisperse_valu(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_active, int nactive,
                     const int32_t* d_offT, int ldo, int d_base, int ndm, uint64_t out_nsamps, uint8_t* out,
                     uint64_t out_stride, float scale, int nbits, int bias, hipStream_t s);

// LDS-staged packed-byte kernel: same contract as dedisperse_valu for the
// DMs [d0, d0 + ndm) of the offset table (any d0: workgroups start on their
// DM-count boundary below d0 and skip the DMs before it), plus d_wmin
// [absolute 32-DM tile][nactive] = each tile's smallest offset per channel
// rounded down to 16 and max_window = the largest (tile, channel) window
// 1024 + (max offset - wmin) + 32 bytes.
bool dedisperse_lds_fits(int nbits, int nactive, int max_window);
// Packed 2-bit rows for dedisperse_2bit: dword j of row r = samples 16 j ..
// 16 j + 15 of chan_major row r (values 0..3) at bits 2 (t & 15), for the
// samples [t0, t0 + ns) (t0 a multiple of 16).
void pack2_rows(const int8_t* chan_major, uint64_t chan_stride, int nrows, uint32_t* out, uint64_t stride2, uint64_t t0,
                uint64_t ns, hipStream_t s);
// Dedispersion of narrow data (nbits <= 2) from the packed 2-bit rows (VALU
// nibble-lane sums, dedisperse.hip): bit-identical to dedisperse_direct.
// max_spread: the largest (largest offset - window start) of the launch's
// 32-DM tiles, in samples (window start: wmin, 16-sample aligned); max_offset:
// the largest window start (rows are read to sample tiles * 2048 + max_offset
// + the window).
int dedisperse_2bit_window(int max_spread);  // staged dwords per channel
bool dedisperse_2bit_fits(int nactive, int max_spread);
void dedisperse_2bit(const uint32_t* x2, uint64_t stride2, const int32_t* d_active, int nactive, const int32_t* d_offT,
                     int ldo, int d0, int ndm, const int32_t* d_wmin, int max_spread, int max_offset,
                     uint64_t out_nsamps, uint8_t* out, uint64_t out_stride, float scale, hipStream_t s);
void dedisperse_lds(const int8_t* chan_major, uint64_t chan_stride, const int32_t* d_active, int nactive,
                    const int32_t* d_offT, int ldo, int d_base, int ndm, const int32_t* d_wmin, int max_window,
                    uint64_t out_nsamps, uint8_t* out, uint64_t out_stride, float scale, int nbits, int bias,
                    hipStream_t s);

// ------------------------------------------------------------ time series ---
// count > 1: rows b at in + b*in_stride, sums sum[b], outputs out + b*out_stride.
void u8_sum(const uint8_t* in, uint64_t n, unsigned long long* sum, hipStream_t s, int count = 1,
            uint64_t in_stride = 0);
// out[i] = i < nvalid ? in[i] : (float)(sum / nvalid)
void u8_to_f32_pad(const uint8_t* in, uint64_t nvalid, float* out, uint64_t n, const unsigned long long* sum,
                   hipStream_t s, int count = 1, uint64_t in_stride = 0, uint64_t out_stride = 0);
void f32_stats(const float* x, uint64_t n, double* partials, int npartials, float* stats_out, hipStream_t s);

// ----------------------------------------------------------------- spectra --
void form_amplitude(const float2* X, uint64_t nbins, float* out, hipStream_t s);
void form_interbin(const float2* X, uint64_t nbins, float* out, hipStream_t s);
// x = (x - mean)/sigma ; mean/sigma either host scalars or device pointer
// (stats = {mean, rms, std}) scaled by `scale`.
void normalise(float* x, uint64_t n, float mean, float sigma, hipStream_t s);
void normalise_dev(float* x, uint64_t n, const float* stats, float scale, hipStream_t s);

// running median (Dereddener::calculate_median): out_count = count/5
// batch > 1: item b at X + b*xstride / in + b*istride -> out + b*ostride
void median5_amp(const float2* X, uint64_t nbins, float* out, hipStream_t s, int batch = 1, uint64_t xstride = 0,
                 uint64_t ostride = 0);
void median5(const float* in, uint64_t count, float* out, hipStream_t s, int batch = 1, uint64_t istride = 0,
             uint64_t ostride = 0);
// X[k] /= median(k) (k<5 -> 0), then zapped bins -> 1+0i. median(k) is the
// piecewise linear stretch of m5/m25/m125 at boundaries pos5/pos25.
void deredden_zap(float2* X, uint64_t nbins, const float* m5, uint64_t n5, const float* m25, uint64_t n25,
                  const float* m125, uint64_t n125, int64_t pos5, int64_t pos25, const uint32_t* zapmask,
                  hipStream_t s, int batch = 1, uint64_t xstride = 0, uint64_t mstride = 0);
// P = interbin(X); per-block partial sums of P and P^2 -> stats {mean,rms,std}
// batch > 1 (P == nullptr): item b's spectrum at X + b*xstride, partials at
// partials + 2*npartials*b, stats at stats + 4*b
void interbin_stats(const float2* X, uint64_t nbins, float* P, double* partials, int npartials, float* stats,
                    hipStream_t s, int batch = 1, uint64_t xstride = 0);
// deredden_zap + interbin_stats (P == nullptr) in one pass, out of place:
// item b's X (stride xstride) -> out (stride ostride), the statistics
// bit-identical to the two-kernel sequence's.
void deredden_zap_stats(const float2* X, float2* out, uint64_t nbins, const float* m5, uint64_t n5, const float* m25,
                        uint64_t n25, const float* m125, uint64_t n125, int64_t pos5, int64_t pos25,
                        const uint32_t* zapmask, double* partials, int npartials, float* stats, hipStream_t s,
                        int batch, uint64_t xstride, uint64_t ostride, uint64_t mstride);

// ------------------------------------------------------------- resampling ---
// out[k][i] = in[clamp(rint(i + i*af_k*(i - n)))], af_k = acc_k*tsamp/(2c)
void resample_batch(const float* in, uint64_t n, float* out, uint64_t out_stride, const double* af, int K,
                    hipStream_t s);
// out[i] = in[clamp(rint(i + af*((i-n/2)^2 - (n/2)^2)))]
void resample_v1(const float* in, uint64_t n, float* out, double af, hipStream_t s);

// ----------------------------------------------------- search hot path ------
// P[k][i] = (interbin(X[k])[i] - stats.mean*nscale) / (stats.std*nscale), i < nbins_out
void interbin_normalise_batch(const float2* X, uint64_t nbins, uint64_t xstride, float* P, uint64_t pstride,
                              int K, uint64_t nbins_out, const float* stats, float nscale, hipStream_t s);

// Same output from the M = N/2 point complex FFT Z[K] of the packed real
// series (real-FFT post-processing fused in; saves the separate r2c pass).
// Bin k = k2 + 2^log2_row * k1 of Z lives at
// (k2 >> log2_blk)*blk_pitch + k1*row_pitch + (k2 & (2^log2_blk - 1))
// (plain array: log2_row = log2 M, row_pitch = M, log2_blk = 3, blk_pitch = 8;
// see fft4_x_layout for the fused FFT's layouts).  Each thread forms the bin
// pair (k, M-k) from one pair of loads.
void r2c_interbin_normalise_batch(const float2* Z, uint64_t M, uint64_t zstride, int log2_row, uint64_t row_pitch,
                                  uint64_t blk_pitch, int log2_blk, float* P, uint64_t pstride, int K,
                                  uint64_t nbins_out, const float* stats, float nscale, hipStream_t s,
                                  const uint32_t* tsrc = nullptr);
// The same from a row-major half spectrum Z[k2 * zp + k1] = FFT_M(z)[k2 + n2 k1]
// (n2 = 2^log2_n2 rows of n1, e.g. rocFFT's row pass of the long-series
// four-step FFT): LDS-tiled transpose, P in natural bin order; Q (optional):
// the screening bytes dev::q8(P) of the same bins (natural, qstride per trial).
void r2c_interbin_normalise_rows(const float2* Z, uint64_t zp, uint64_t zstride, int log2_n2, uint64_t n1, float* P,
                                 uint64_t pstride, int K, uint64_t nbins_out, const float* stats, float nscale,
                                 hipStream_t s, const uint32_t* tsrc = nullptr, uint8_t* Q = nullptr,
                                 uint64_t qstride = 0);

// Same output from the 8x8-tiled spectrum of fft4 pass B (kFft4TileX):
// bin k = k2 + n2*k1 at X[k2/8][k1/8][k2%8][k1%8]; 64-byte loads per thread.
// tsrc (device, optional): trial k normalises with stats + 4*tsrc[k] (batches
// mixing trials of several prepared series).
// With Q, also the screening bytes dev::q8(P) of every stored bin (row k at
// Q + k*qstride, qstride >= nbins_out) for harmonic_peaks_batch's screen; P
// may then be null (Q only).  Twiddles from rt = r2c_twiddle_table(n1 * n2)
// (nullptr: looked up): every bin's value depends on X and its index alone,
// so the screened harmonic sum can recompute any bin exactly (HarmFromX).
void r2c_interbin_normalise_tiled(const float2* X, int n1, int n2, uint64_t xstride, float* P, uint64_t pstride,
                                  int K, uint64_t nbins_out, const float* stats, float nscale, hipStream_t s,
                                  const uint32_t* tsrc = nullptr, uint8_t* Q = nullptr, uint64_t qstride = 0,
                                  const float2* rt = nullptr);
// Device table of e^{-i pi k / M} (k = 2048 a + b: [b < 2048] then
// [a <= M/2 >> 11]) on the current device, built on first use (synchronous
// copy) and cached for the process.
const float2* r2c_twiddle_table(uint64_t M);

// Fused resample + four-step FFT (fft4step.hip).  M = N/2 = n1*n2 with
// n1, n2 powers of two in [128, 4096], n2 <= n1 <= 2 n2.  Intermediates use
// padded row pitches (power-of-two strides would camp on one memory channel):
//   Y[k][k2*ypitch + i]  (pass A output),  X[k][k1*xpitch + k2] = FFT_M(z_k)[k2 + n2 k1].
struct Fft4Geom {
  int n1 = 0, n2 = 0;
  uint64_t ypitch = 0, ystride = 0;  // complex
  uint64_t xpitch = 0, xstride = 0;  // complex
  int log2_xrow = 0;                 // log2(n2): X index of bin k = (k >> log2_xrow)*xpitch + (k & (n2-1))
  uint64_t inpitch = 0, insize = 0;  // floats: padded input copy (room for either layout: row pitch or strips)
  bool ok = false;
  // Pass A input per trial k: in + k*in_tstride, in_pad + k*pad_tstride
  // (0 = every trial resamples the same series; the batched whitener sets n, insize).
  uint64_t in_tstride = 0, pad_tstride = 0;
  // optional device map trial -> series index (else trial k reads series k)
  const uint32_t* tsrc = nullptr;
  // Y in row pairs, Y_p[k2/2][i][k2%2], instead of 8x8 tiles (only where
  // fft4_pair_y(g) holds; read by fft4_rowpass_spectrum alone)
  bool ypair = false;
  // every trial is a plain FFT (af = 0: the whitener's forward and inverse
  // transforms): the one-exchange pass A reads the padded input in column
  // strips; the Stockham pass A can read the sources below directly
  bool zero_shift = false;
  // zero_shift, Stockham pass A only (fft4_direct_source(g)): read trial k's
  // series straight from its source instead of in_pad --
  //   u8: 8-bit rows at u8 + src * src_stride, sample i < u8_nvalid as is,
  //       then the row mean u8sum[src] / u8_nvalid up to n (the whitener's
  //       forward input: no f32 copy, no pad kernel);
  //   c2r: half spectra X (M + 1 bins at c2r + src * src_stride), turned into
  //       the C2R pre-processed series on the fly (fft4_c2r_pre's arithmetic,
  //       bit for bit: the whitener's inverse)
  const uint8_t* u8 = nullptr;
  const unsigned long long* u8sum = nullptr;
  uint64_t u8_nvalid = 0;
  const float2* c2r = nullptr;
  uint64_t src_stride = 0;
  //   f32_direct: the unpadded series in + src * in_tstride itself (no pad copy);
  //   strips_direct: in_pad in column strips (fft4_pad_input_u8's layout)
  bool f32_direct = false, strips_direct = false;
  // fft4_geometry_rows: rows longer than the fused passes take (n1 >= 8192)
  // are transformed outside (rocFFT); pass A writes natural Y rows
  // Y[k2 * ypitch + i] for it
  bool rows_ext = false;
};
Fft4Geom fft4_geometry(uint64_t M);
// Series of 2^26 points and more: columns of 4096 through the fused
// resample + Stockham pass A, rows of n1 = M / 4096 for an external FFT
// (ok = false below M = 2^25 or at M >= 2^31).
Fft4Geom fft4_geometry_rows(uint64_t M);
// Pass A of g can take the u8 / c2r direct sources (a zero-shift geometry
// whose column pass is the Stockham kernel).
bool fft4_direct_source(const Fft4Geom& g);
// fft4_pad_input writes g's padded input in column strips (fft4_pad_input_u8 needs it)
bool fft4_strip_layout(const Fft4Geom& g);
// Twiddle tables (upload once per plan): see fft4step.hip for the layout.
std::vector<float2> fft4_tables(const Fft4Geom& g);
// Padded copy of the (whitened) input series read by pass A; insize floats.
// count > 1: series b at in + b*in_stride -> in_pad + b*g.insize.
void fft4_pad_input(const float* in, uint64_t n, float* in_pad, const Fft4Geom& g, hipStream_t s, int count = 1,
                    uint64_t in_stride = 0);
// The same padded copy straight from 8-bit dedispersed rows (strip layouts
// only: fft4_strip_layout(g), or a direct-source geometry's strips_direct): sample i < nvalid is in[i], then
// the row mean (sum[b] / nvalid) up to n, zeros beyond -- u8_to_f32_pad and
// fft4_pad_input in one pass.  count rows at in + b * in_stride.
void fft4_pad_input_u8(const uint8_t* in, uint64_t nvalid, uint64_t n, const unsigned long long* sum, float* in_pad,
                       const Fft4Geom& g, hipStream_t s, int count, uint64_t in_stride);
// Pass A: Y[k][k2][i] = W_M^{i k2} sum_j z_k[n1 j + i] W_n2^{j k2}, where
// z_k[m] = x_k[2m] + i x_k[2m+1] and x_k = resampleII(in, af[k]); n = 2M.
void fft4_resample_colpass(const float* in, const float* in_pad, uint64_t n, const double* af, int K, float2* Y,
                           const Fft4Geom& g, const float2* tables, hipStream_t s);
// Pass B: X[k][k1][k2] = sum_i Y[k][k2][i] W_n1^{i k1}.  With the tiled
// spectrum layout and nbins_out > 0, only the k1 rows that
// r2c_interbin_normalise_tiled reads for bins < nbins_out are stored (the
// search needs bins below max_freq only: ~14% of the spectrum at 2^23).
void fft4_rowpass(const float2* Y, float2* X, int K, const Fft4Geom& g, const float2* tables, hipStream_t s,
                  uint64_t nbins_out = 0);
// Pass B fused with the search spectrum (fft4step.hip fft4_rowpass_spectrum_kernel):
// from the tiled Y of fft4_resample_colpass, the normalised interbinned
// spectrum P of every bin 0..M (as r2c_interbin_normalise_tiled forms it, to
// FFT rounding) and its screening bytes dev::q8(P), without the complex
// spectrum ever reaching memory.  P is stored workgroup-blocked
// (spec_pblk_index), Q in natural order: bin b of trial k at
// Q[k*qstride + kSpecQShift + b].  Trial k normalises with stats + 4*tsrc[k]
// (tsrc null: stats) scaled by nscale.
constexpr int kSpecQShift = 15;
struct SpecOut {
  float* P = nullptr;
  uint64_t pstride = 0;  // floats per trial, >= M + 1 (multiple of 4)
  uint8_t* Q = nullptr;
  uint64_t qstride = 0;  // bytes per trial, >= M + 1 + kSpecQShift (multiple of 16)
  const float* stats = nullptr;
  const uint32_t* tsrc = nullptr;
  float nscale = 1.f;
  // bins [0, nbins) are written (whole 4-bin groups; 0: all M + 1): the
  // search reads none at or above its highest harmonic bin (max_freq x
  // 2^nlevels: below M only for few harmonics -- 1100 Hz at 2^23 x 64 us is
  // 14% of the spectrum per harmonic doubling), so the rest of P and Q is
  // neither formed nor stored
  uint32_t nbins = 0;
};
// Position of bin b (0 <= b <= M = n1 << log2_n2) in the blocked P: rows
// r = b mod n2 in [1, n2/2] at ((2v) n1 + k1) 4 + j with v = (r-1)/4, j = (r-1)%4;
// the other bins b = M - (r + n2 k1) (r < n2/2) at ((2v+1) n1 + k1) 4 + j with
// v = r/4, j = r%4; bin 0 at M.
__host__ __device__ inline uint32_t spec_pblk_index(uint32_t b, int log2_n2, uint32_t n1) {
  const uint32_t n2 = 1u << log2_n2, M = n1 << log2_n2;
  if (b == 0) return M;
  const uint32_t r = b & (n2 - 1);
  if (r >= 1 && r <= n2 / 2) return (((r - 1) >> 2) * 2 * n1 + (b >> log2_n2)) * 4 + ((r - 1) & 3);
  const uint32_t bm = M - b, rm = bm & (n2 - 1);
  return (((rm >> 2) * 2 + 1) * n1 + (bm >> log2_n2)) * 4 + (rm & 3);
}
void fft4_rowpass_spectrum(const float2* Y, int K, const Fft4Geom& g, const float2* tables, const SpecOut& o,
                           hipStream_t s);
// Whether pass A can write the row-pair Y layout for the spectrum pass under
// the current flags (the one-exchange pass A, column length 2048): its lanes
// then load two rows per 16-byte vector, 1 KiB contiguous per wave.
bool fft4_pair_y(const Fft4Geom& g);
// Row-octet blocks (8 rows k1 each) r2c_interbin_normalise_tiled runs for
// bins < nbins_out; it reads spectrum rows k1 <= 8*ny and k1 >= n1 - 8*ny.
inline uint32_t r2c_tiled_row_blocks(uint64_t nbins_out, int n1, int n2) {
  const uint64_t full = static_cast<uint64_t>(n1) / 16;
  if (nbins_out == 0) return static_cast<uint32_t>(full);
  const uint64_t ny = (nbins_out - 1) / (8ull * static_cast<uint64_t>(n2)) + 1;
  return static_cast<uint32_t>(ny < full ? ny : full);
}
// Spectrum layout of fft4_rowpass under the current flags, as r2c parameters.
struct Fft4XLayout {
  int log2_row;
  uint64_t row_pitch, blk_pitch;
  int log2_blk;
  bool tiled;  // kFft4TileX: use r2c_interbin_normalise_tiled
};
Fft4XLayout fft4_x_layout(const Fft4Geom& g);
// Whitening real FFTs on the four-step passes (K = 1): spectrum layout of
// fft4_rowpass as kernel arguments; natural-order half spectrum <-> pass data.
struct XLayoutArgs {
  int tiled;           // kFft4TileX layout (taddr) else blocked/natural (zaddr)
  int log2_row;        // tiled: log2(n2)
  uint64_t n1;         // tiled
  uint64_t row_pitch, blk_pitch;
  int log2_blk;
};
inline XLayoutArgs xlayout_args(const Fft4Geom& g, const Fft4XLayout& l) {
  XLayoutArgs a{};
  a.tiled = l.tiled ? 1 : 0;
  a.log2_row = l.tiled ? g.log2_xrow : l.log2_row;
  a.n1 = static_cast<uint64_t>(g.n1);
  a.row_pitch = l.row_pitch;
  a.blk_pitch = l.blk_pitch;
  a.log2_blk = l.log2_blk;
  return a;
}
// X[k] (k = 0..M, natural) of the N = 2M real series whose half-length FFT Z
// (layout L) fft4_rowpass produced.
// Batched (count transforms): Z + b*zstride -> X + b*xstride (and likewise below).
void fft4_r2c_half(const float2* Z, uint64_t M, const XLayoutArgs& L, float2* X, hipStream_t s, int count = 1,
                   uint64_t zstride = 0, uint64_t xstride = 0);
// Natural-order M complex values whose forward FFT is the conjugate of the
// unnormalised C2R of X[0..M] (as pairs x[2m] + i x[2m+1]).
void fft4_c2r_pre(const float2* X, uint64_t M, float2* out, hipStream_t s, int count = 1, uint64_t xstride = 0,
                  uint64_t ostride = 0);
// x[2m] + i x[2m+1] = conj(Z[m]) (Z in layout L): the N-point unnormalised C2R.
void fft4_c2r_post(const float2* Z, uint64_t M, const XLayoutArgs& L, float* x, hipStream_t s, int count = 1,
                   uint64_t zstride = 0, uint64_t ostride = 0);
// The same inverse written straight into the search pass A's padded row input
// (fft4_pad_input's layout: rows of 2 gs.n1 floats at pitch gs.inpitch, each
// row's pad holding the next row's head, trial b at xpad + b * pstride).
// Returns false, writing nothing, where the layouts do not allow it (the
// strip layout, the external-row geometry, an untiled spectrum).
bool fft4_c2r_post_pad(const float2* Z, uint64_t M, const XLayoutArgs& L, float* xpad, const Fft4Geom& gs,
                       hipStream_t s, int count, uint64_t zstride, uint64_t pstride);
// Mixed-radix (n = m p, p a power of two, m odd) transforms on the four-step
// passes, for series whose length is not a power of two (the multi-beam
// coincidencer transforms the whole DM-0 series): z[n1][n2] = s(n1 + m n2),
// m batched p-point FFTs, then X[k] = sum_n1 W_n^(n1 k) Z_n1[k mod p].
// gather mode 0: s = real series x (imaginary 0); mode 1: s = conj of the
// Hermitian extension of the half spectrum X[0..n/2] (the C2R input).
void mixed_gather(const float* src, uint64_t n, uint32_t m, uint64_t p, int mode, float2* dst, hipStream_t s);
// Z_n1 in layout L at Z + n1*zstride; mode 0: out = float2 X[0..n/2]; mode 1:
// out = float Re X[0..n-1] (the unnormalised C2R when the gather was mode 1).
void mixed_combine(const float2* Z, uint64_t zstride, const XLayoutArgs& L, uint64_t n, uint32_t m, uint64_t p,
                   int mode, void* out, hipStream_t s);
// Kernel-shape switches (process-wide; the default is the fastest measured
// set, every bit of it in use; tests/test_kernels_gpu.py runs each prefix of
// the chain below).  Bit values are stable (flag sets are recorded in
// profiles and the run identity).
enum Fft4Flags : int {
  kFft4Cpt8 = 1,           // 8 transforms per thread, one thread group (else 4 per thread, two groups)
  kFft4NoRemap = 2,        // plain block order (no XCD-contiguous remap)
  kFft4Blocked = 256,      // blocked Y/X layouts: every lane stores its transforms' values contiguously
  kFft4TileY = 1024,       // with kFft4Blocked: 8x8-tiled Y between the passes (16-byte pass-B loads)
  kFft4TileX = 2048,       // with kFft4TileY: 8x8-tiled spectrum X (coalesced pass-B stores; tiled r2c)
  kFft4PairXcd = 4096,     // pass A: adjacent column blocks of a trial on one XCD (shared input lines)
  kFft4GroupXcd = 8192,    // pass A: 8 trials x 2 adjacent column blocks per XCD group (needs K % 8 == 0)
  kFft4UniformTw = 65536,  // pass A: four-step twiddles as per-thread x workgroup-uniform (SGPR) factors
  kFft4OneX = 131072,      // pass A (tiled Y, column length 2048): 2 columns x 32 points per thread,
                           // one LDS exchange, compile-time twiddles inside the two local DFTs
  kFft4PairY = 262144,     // the Stockham pass A (column lengths other than the one-exchange one) also
                           // hands the fused spectrum pass row-pair Y (Y_p[k2/2][i][k2%2])
  kFft4EarlyTw = 2097152,  // one-exchange pass A / fused spectrum pass: every twiddle and output constant
                           // loaded before the data (pass A) or staged in LDS (spectrum pass stages), no
                           // dependent global round trip after the loads
  kFft4WideY = 8388608,    // one-exchange pass A, row-pair Y: lane pairs swap halves (DPP) so every lane
                           // stores 16 bytes (half the store instructions)
  kFft4WhitenStrips = 16777216,  // whitener (plain FFTs, Fft4Geom::zero_shift): the one-exchange pass A reads
                                 // the 8-bit rows staged into strips; the Stockham pass A reads its inverse
                                 // input straight from the half spectra (C2R pre-processing fused) and
  kFft4WhitenU8 = 33554432,      // its forward input straight from the 8-bit rows,
  kFft4WhitenF32 = 67108864,     // or the unpadded f32 copy (neither: the 8-bit rows staged into strips).
                                 // 2^20 bench A/B (profiles/r6_whiten): strips / u8 / f32 all +1.5-2% over
                                 // the f32 copy + pad path, within noise of each other; u8 moves the fewest bytes
  kFft4StripInput = 1073741824,  // one-exchange pass A: the padded input in column strips (16 + 4 floats of
                                 // every row per strip, strips row-contiguous), so a wave's 16 rows are
                                 // one ~1.3 KiB contiguous range instead of 16 pieces 16 KiB apart
};
void fft4_set_flags(int flags);
// Debug: per-workgroup phase timestamps of the fft4 passes (12 x u64 per block), nullptr = off.
void fft4_set_trace(unsigned long long* d_events);
int fft4_flags();

struct HarmParams {
  int nlevels;             // number of harmonic-sum levels (0..5)
  int start[6];            // per level search range [start, end)
  int end[6];
  float thresh;
  uint32_t capacity;       // PeakRecord capacity of `out` (a multiple of 2^region_log2)
  uint32_t trial_base = 0; // added to the batch item of every record (sub-batch launches)
  int region_log2 = 0;     // record regions (kPeakRegionStride): 0 = one counter, count[0]
};
// Fused incoherent harmonic sum + threshold + compaction: never writes the
// summed spectra.  Records land unordered; count may exceed capacity (then
// the caller re-runs with a bigger buffer).
// With Q (the screening bytes of P, row k at Q + k*qstride, qstride >= the
// highest searched bin, 16-byte aligned rows) the sums are screened on Q:
// integer sums of the staged bytes (a quarter of P's gather traffic) against
// per-level integer bounds that no bin whose fp32 sum passes the pre-threshold
// can miss; only the bins that pass (or touch a saturated byte) are summed
// exactly from P.  Records are identical either way.
// With fx (and Q) the exact sums recompute their bins from the tiled
// spectrum X exactly as r2c_interbin_normalise_tiled forms them, so P need
// not be written at all (P is then ignored).
// With fx->pblk (and Q from fft4_rowpass_spectrum), P is the blocked spectrum
// of that pass (spec_pblk_index with fx->log2_n2, fx->n1; X unused) and the
// screening bytes of bin b are at Q[k*qstride + fx->qshift + b].
struct HarmFromX {
  int pblk = 0;
  int qshift = 0;
  const float2* X = nullptr;  // tiled pass-B spectra, trial k at X + k*xstride
  uint64_t xstride = 0;
  int log2_n2 = 0;
  uint32_t n1 = 0;
  const float2* rt = nullptr;       // r2c_twiddle_table(n1 << log2_n2)
  const float* stats = nullptr;     // whitening stats (mean at [0], sigma at [2]) per series
  const uint32_t* tsrc = nullptr;   // series of trial k (stats + 4*tsrc[k]); nullptr: stats itself
  float nscale = 1.f;
};
void harmonic_peaks_batch(const float* P, uint64_t nbins, uint64_t pstride, int K, const HarmParams& hp,
                          PeakRecord* out, uint32_t* count, hipStream_t s, const uint8_t* Q = nullptr,
                          uint64_t qstride = 0, const HarmFromX* fx = nullptr);
// Q[k*qstride + i] = dev::q8(P[k*pstride + i]), i < n (tests and tools; the
// search writes Q from the r2c kernel).
void quantize_q8(const float* P, uint64_t pstride, uint64_t n, int K, uint8_t* Q, uint64_t qstride, hipStream_t s);
// Peak clustering on the device (peakcluster.hip; peakfinder.hpp:24-55):
// the records of harmonic_peaks_batch (first min(*d_count, cap)) -- chunks
// of idx-ascending crossings, each behind its descriptor record (seg field
// kPeakChunk | count << 16 | segment, idx = first idx, snr bits = position
// of the first crossing) -- per segment (seg < nseg <= 65536) clustered with
// the reference's gap rule.  d_segtab[seg] = {first, count} of its cluster
// peaks in d_out (ascending idx; uint2 = {idx, snr bits}; segments packed in
// any order, *d_total in all), or {first, count | kClusterRaw} when the
// segment has more than kClusterCap crossings: then its raw, unsorted
// crossings are d_sorted[cap + first .. cap + first + count) for the host.
// d_work: 5 * nseg uint32; d_sorted: 2 * cap entries; d_out: cap entries.
// Timing (tools/expt/cluster_bench.py --trace): the large kernel's phase
// timestamps, 8 per workgroup (nullptr: off).
void peak_cluster_set_trace(unsigned long long* d_events);
constexpr uint32_t kClusterCap = 14000;
constexpr uint32_t kClusterRaw = 0x80000000u;
// region_log2 > 0: the records in regions as harmonic_peaks_batch wrote them
// (kPeakRegionStride; d_count = the region counters, cap >> region_log2 a
// multiple of 4096).
void peak_cluster_batch(const PeakRecord* d_peaks, const uint32_t* d_count, uint32_t cap, uint32_t nseg, int gap,
                        uint32_t* d_work, uint2* d_sorted, uint2* d_out, uint2* d_segtab, uint32_t* d_total,
                        hipStream_t s, int region_log2 = 0);
// *d_total = the records held in the 2^region_log2 regions of d_rcount, or,
// when one overflowed, 2^region_log2 x its count (more than cap).
void peak_regions_total(const uint32_t* d_rcount, int region_log2, uint32_t cap, uint32_t* d_total, hipStream_t s);
// Per-trial harmonic distillation on the device (harmdistill.hip;
// distiller.hpp:63-108, HarmonicDistiller(tol, max_harm, keep_related=false,
// fractional_harms=true) on the cluster peaks of every level of one trial).
// For trial k (segments 8k .. 8k + nlevels of peak_cluster_batch's table):
// d_ttab[k] = {first, count} of its unique candidates in d_out, in
// descending S/N order -- uint2 = {idx | level << 29, snr bits}; trials packed
// in any order, *d_total in all -- or {0, kHarmHost} when the host must
// distill the trial from its cluster peaks: a raw (over-capacity) segment,
// more than kHarmCap peaks, or two peaks with equal S/N (the reference's
// introsort order of ties is not reproduced on the device).
// Equal to the host distiller's output (candidates.cpp, fast relation path:
// tol <= 1e-3): same double-precision expressions, no contraction.
struct HarmDistillParams {
  int nlevels;          // levels 0..nlevels
  double factor[6];     // freq of bin idx at level h: float(idx * factor[h])
  float tol;            // freq_tol (float, as HarmonicDistiller::tol_)
  float max_harm;       // max_harm_match
  double lower_tol;     // 1 - tol
  double upper_tol;     // 1 + tol
};
constexpr uint32_t kHarmCap = 4096;
constexpr uint32_t kHarmHost = 0x80000000u;
void harm_distill_batch(const uint2* d_clust, const uint2* d_segtab, int ntrials, const HarmDistillParams& p,
                        uint2* d_out, uint2* d_ttab, uint32_t* d_total, hipStream_t s);
// Harmonic-sum switches (process-wide; default 1 | 8 | 32 | 64 | 10 << 8):
// bit 0 = XCD-per-trial block order; bit 1 = pre-threshold off (tests);
// engines built afterwards: bit 2 = the screened sum off, bit 3 = (without
// bit 6) its exact sums recomputed from the spectrum with no P stored, bit 6
// = the fused spectrum pass (fft4_rowpass_spectrum; needs the screen);
// bit 5 = the fp32 3-level kernel in two staging phases; bits 8-15 = that
// kernel's dynamic-LDS occupancy cap in KiB.
void harmonic_set_flags(int flags);
int harmonic_flags();
// Debug/test: materialise level-h sums [nlevels][nbins] for one spectrum.
void harmonic_sums(const float* P, uint64_t nbins, int nlevels, float* out, hipStream_t s);

// ------------------------------------------------------------------ folding --
struct FoldJob {
  double tsamp_by_period;  // tsamp / period
  double af;               // acc*tsamp/(2c) for the v1 resampler
  uint64_t series = 0;     // the job folds in + series * n (a batch of whitened DM trials)
};
// Partial fold sums: partial[(job*nints + subint)*nchunk + chunk][nbins] (sum),
// counts likewise.  n = samples per (whitened) series; job j reads series
// jobs[j].series of the batch at `in`.
void fold_accumulate(const float* in, uint64_t n, const FoldJob* jobs, int njobs, int nbins, int nints,
                     int chunk, float* psum, int32_t* pcount, hipStream_t s);
void fold_reduce(const float* psum, const int32_t* pcount, int njobs, int nbins, int nints, int nchunk,
                 float* fold, hipStream_t s);
// Shift-phase table [nshift][nints][nbins] complex (FoldOptimiser shift array)
void fold_shift_table(float2* table, int nbins, int nints, hipStream_t s);
// One workgroup per fold: shift/collapse/template search.  opt_int = {template, shift, bin}
void fold_optimise(const float* folds, int nfold, const float2* shift_table, float* opt_fold, float* opt_prof,
                   int32_t* opt_int, float* opt_val, hipStream_t s);

// ------------------------------------------------------------- coincidence --
// counts[i] += (x[i] > thresh)   (uint8 counts)
void count_above(const float* x, uint64_t n, float thresh, uint8_t* counts, hipStream_t s);
// mask[i] = counts[i] < beam_thresh
void coincidence_mask(const uint8_t* counts, uint64_t n, int beam_thresh, float* mask, hipStream_t s);
// acc[i] += a[i] (uint8 beam counts of two devices' beams)
void add_counts(const uint8_t* a, uint64_t n, uint8_t* acc, hipStream_t s);

// ------------------------------------------------------------- correlation --
void conjugate(float2* x, uint64_t n, hipStream_t s);
void cmul_inplace(const float2* x, float2* y, uint64_t n, hipStream_t s);
// Copy nrows scattered device rows of nbytes (16-byte aligned multiples) to
// dst + i * dst_stride, one launch per kGatherRows rows.
constexpr int kGatherRows = 64;
struct RowPtrs {
  const uint8_t* p[kGatherRows];
};
void gather_rows(const uint8_t* const* rows, int nrows, uint64_t nbytes, uint8_t* dst, uint64_t dst_stride,
                 hipStream_t s);

}  // namespace kern
}  // namespace psoup
