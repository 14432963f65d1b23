// FFA (Fast Folding Algorithm) periodicity search: the pipeline behind the
// reference's FFA options (include/utils/cmdline.hpp:35-50 FFACmdLineOptions,
// :211-292 read_ffa_cmdline_options; Makefile:41-42 `ffaster`, source not in
// the reference tree).  Kernels in csrc/kernels/ffa.hip, engine in
// csrc/src/ffa.cpp, CLI bin/ffaster (csrc/apps/ffa_main.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "psoup/cli.hpp"
#include "psoup/common.hpp"

namespace psoup {

// ------------------------------------------------------------- kernels ----
namespace kern {

struct FfaPeriod {
  int32_t p;       // base period in (downsampled) bins
  int32_t m;       // rows holding data (floor(nds / p))
  int32_t m2;      // rows after zero padding (power of two >= m)
  int32_t log2m2;
  uint64_t offset;       // floats into the arena
  uint64_t best_offset;  // profiles into the optional best-S/N output
};

constexpr int kFfaMaxWidths = 24;
struct FfaSnrParams {
  int32_t widths[kFfaMaxWidths];
  int32_t nwidths;
  float thresh;
  float var_per_bin;  // variance of one downsampled bin of the normalised series (= factor)
};

struct FfaPeak {
  int32_t period_idx;  // into the chunk's period table
  int32_t drift;       // FFA row: period = p + drift / (m2 - 1) bins
  float snr;
  int32_t width;       // boxcar width in bins
};
static_assert(sizeof(FfaPeak) == 16, "FfaPeak layout");

// Block means over `window` samples, x = in - (linear trend between block
// centres).  sums / block_means: ceil(n / window) elements (< 65536).
void ffa_detrend(const uint8_t* in, uint64_t n, uint64_t window, unsigned long long* sums, float* block_means,
                 float* out, hipStream_t s);
// out[j] = integral of x over [j f, (j+1) f), j < nout <= n / f (f >= 1).
void ffa_downsample(const float* x, uint64_t n, double f, float* out, uint64_t nout, hipStream_t s);
// Folded FFA planes of every period of a chunk (arena layout from FfaPeriod):
// the first min(4, log2m2) stages on LDS-resident row blocks (when the
// chunk's longest period fits), the rest as ping-pong passes of two stages.
bool ffa_uses_lds(int max_p);
// True when period pp's result lies in the second arena: an odd number of
// global passes, ceil((log2m2 - LDS stages) / 2).
__host__ __device__ inline bool ffa_result_in_second(const FfaPeriod& pp, int lds_stages) {
  const int g = pp.log2m2 - (pp.log2m2 < lds_stages ? pp.log2m2 : lds_stages);
  return (((g + 1) / 2) & 1) != 0;
}
void ffa_transform(const float* ds, const FfaPeriod* d_periods, int nper, int max_m2, int max_log2m2, int max_p,
                   float* arena0, float* arena1, hipStream_t s);
// Best boxcar S/N of every folded profile; records above sp.thresh are
// appended to out (count may exceed capacity).  best (optional): S/N per
// profile at FfaPeriod::best_offset + drift.
void ffa_snr(const FfaPeriod* d_periods, int nper, int max_m2, int max_p, const float* arena0, const float* arena1,
             const FfaSnrParams& sp, FfaPeak* out, uint32_t* count, uint32_t capacity, float* best, hipStream_t s);
int ffa_max_profile();

}  // namespace kern

// --------------------------------------------------------------- engine ----
struct FfaParams {
  double tsamp = 64e-6;
  double p_start = 0.8;   // s
  double p_end = 20.0;    // s
  float min_dc = 0.001f;  // minimum duty cycle -> base bins per period
  int nbins = 0;          // base bins nb0 (periods span [nb0, 2 nb0) bins); 0 = from min_dc
  float min_snr = 7.0f;
  double detrend_s = 0;   // trend window (s); 0 = 3 x p_end
  uint64_t arena_floats = uint64_t(1) << 27;  // per ping-pong buffer
  double cluster_tol = 2.0;                   // peak clustering, in units of 1/T_obs
  int min_rows = 8;                           // skip periods with fewer folded rows
};

struct FfaCandidate {
  double period = 0;  // s
  float snr = 0;
  int width = 0;      // bins
  int nbins = 0;      // bins across the period at its octave (folded profile length)
  float dm = 0;
  int dm_idx = 0;
  int octave = 0;
  double duty_cycle() const { return nbins > 0 ? static_cast<double>(width) / nbins : 0; }
  double freq() const { return 1.0 / period; }
};
using FfaCandidateList = std::vector<FfaCandidate>;

struct FfaChunk {
  std::vector<kern::FfaPeriod> periods;
  int max_m2 = 0, max_log2m2 = 0, max_p = 0;
  uint64_t arena = 0;  // floats used
  uint64_t nprof = 0;  // profiles (sum of m2)
};

struct FfaOctave {
  double factor = 1;  // downsampling factor
  uint64_t nds = 0;   // downsampled length
  int pa = 0, pb = 0; // base periods [pa, pb) in bins
  std::vector<FfaChunk> chunks;
};

// Octave plan for a series of n samples (host only; testable on CPU).
std::vector<FfaOctave> ffa_plan(const FfaParams& p, uint64_t n);
int ffa_base_bins(const FfaParams& p);
std::vector<int> ffa_widths(int nb0);

// Clusters candidates whose frequencies lie within tol_hz of a stronger one
// (greedy in S/N order, like the reference's distillers); returns the
// survivors sorted by S/N (descending).
FfaCandidateList ffa_cluster(FfaCandidateList cands, double tol_hz);

class FfaEngine {
 public:
  FfaEngine(const FfaParams& p, uint64_t nsamps, hipStream_t stream);
  ~FfaEngine();
  // d_trial: device u8 dedispersed series of nsamps samples.
  FfaCandidateList search(const uint8_t* d_trial, float dm, int dm_idx);
  const std::vector<FfaOctave>& plan() const { return plan_; }
  uint64_t nsamps() const { return n_; }
  double tobs() const { return static_cast<double>(n_) * p_.tsamp; }
  // Counters
  uint64_t profiles() const { return nprof_; }
  uint64_t peaks() const { return npeaks_; }

 private:
  FfaParams p_;
  uint64_t n_;
  hipStream_t stream_;
  std::vector<FfaOctave> plan_;
  DeviceBuffer<float> x_, ds_, means_, a0_, a1_;
  DeviceBuffer<unsigned long long> sums_;
  DeviceBuffer<double> partials_;
  DeviceBuffer<float> stats_;
  DeviceBuffer<kern::FfaPeak> d_peaks_;
  DeviceBuffer<uint32_t> d_count_;
  std::vector<kern::FfaPeak> h_peaks_;
  uint32_t cap_ = 1u << 16;
  uint64_t nprof_ = 0, npeaks_ = 0;
  kern::FfaSnrParams snr_{};
  std::vector<DeviceBuffer<kern::FfaPeriod>> tables_;
};

// ------------------------------------------------------------ pipeline ----
struct FfaResult {
  FfaCandidateList candidates;          // clustered over all DMs, S/N descending, limited
  std::vector<float> dm_list;
  std::vector<int> devices;
  std::map<std::string, double> timers;  // reading, dedispersion, searching, total (s)
  uint64_t nsamps = 0;                  // dedispersed series length searched
  double tobs = 0;
  int nb0 = 0;
  std::vector<FfaOctave> plan;
  uint64_t profiles = 0, peaks = 0;
};
FfaParams ffa_params_from(const FfaCmdLineOptions& args, double tsamp);
// Reads the filterbank, dedisperses (MFMA) on min(-t, devices) GPUs (one
// thread per GPU pulling DM chunks), runs the FFA on every trial.
FfaResult run_ffa_pipeline(const FfaCmdLineOptions& args);
// Text output (one candidate per line after a commented header).
void write_ffa_output(const std::string& path, const FfaCmdLineOptions& args, const FfaResult& res);

}  // namespace psoup
