// Command-line options.
//
// Parity: include/utils/cmdline.hpp:6-209 (CmdLineOptions + TCLAP parser with
// 25 options and their defaults; -h/--help and --version "1.0" come from
// TCLAP) and src/coincidencer.cpp:31-98 (coincidencer options).  The parser
// is a small in-repo replacement for the vendored TCLAP (no vendoring).
// Extra MI355X options are long-only and default to the reference behaviour
// except where noted.
#pragma once

#include <string>
#include <vector>

namespace psoup {

struct CmdLineOptions {
  std::string infilename;
  std::string outdir;
  std::string killfilename;
  std::string zapfilename;
  int max_num_threads = 14;
  int limit = 1000;
  unsigned int size = 0;
  float dm_start = 0.0f;
  float dm_end = 100.0f;
  float dm_tol = 1.10f;
  float dm_pulse_width = 64.0f;
  float acc_start = 0.0f;
  float acc_end = 0.0f;
  float acc_tol = 1.10f;
  float acc_pulse_width = 64.0f;
  float boundary_5_freq = 0.05f;
  float boundary_25_freq = 0.5f;
  int nharmonics = 4;
  int npdmp = 0;
  float min_snr = 9.0f;
  float min_freq = 0.1f;
  float max_freq = 1100.0f;
  int max_harm = 16;
  float freq_tol = 0.0001f;
  bool verbose = false;
  bool progress_bar = false;

  // ---- MI355X-native extensions (long options only) ----
  std::string accel_convention = "legacy";  // legacy | reference
  std::string dedisp_kernel = "auto";       // auto | mfma | direct
  int accel_batch = 0;                      // 0 = auto (sized for HBM)
  int engines_per_gpu = 0;                  // search engines (streams + host threads) per GPU, 0 = auto
  std::string dm_schedule = "auto";         // multi-rank DM distribution: dynamic | static | auto (dynamic with
                                            // >= 2 ranks and >= 4 32-DM chunks per rank, else static; an
                                            // explicit dynamic also runs the queue on one rank)
  int accel_slices = 0;                     // acceleration-trial slices per DM work unit of the multi-rank
                                            // Python driver (0 = auto: split when the job has fewer than 4 DM
                                            // chunks per rank; 1 = never)
  int sub_batch = -1;                       // -1 = auto
  int fft_mode = 2;                         // see SearchParams::fft_mode
  bool use_boundaries = false;              // honour --boundary_* (reference ignores them)
  std::string checkpoint_dir;               // per-DM candidate spill + resume
  std::string trace_json;                   // optional per-stage JSON trace
  int fault_after_dms = -1;                 // fault injection (testing)
  bool time_shards = false;                 // Python driver: time-sharded dedispersion (halo + all-to-all)
};

// Returns false on a parse error (message printed to stderr).  Sets
// *exit_now (and returns true) for --help / --version.
bool parse_cmdline(CmdLineOptions& args, int argc, const char* const* argv, bool* exit_now = nullptr);
bool parse_cmdline(CmdLineOptions& args, const std::vector<std::string>& argv, bool* exit_now = nullptr);
std::string cmdline_usage();

// Default outdir: "./%Y-%m-%d-%H:%M_peasoup/" in UTC (cmdline.hpp:53-59).
std::string default_outdir();

struct CoincidencerOptions {
  std::vector<std::string> filterbanks;
  std::string samp_outfilename = "rfi.eb_mask";
  std::string spec_outfilename = "birdies.txt";
  float boundary_5_freq = 0.05f;
  float boundary_25_freq = 0.5f;
  int nharmonics = 4;
  float threshold = 4.0f;
  int beam_threshold = 4;
  float min_freq = 0.1f;
  float max_freq = 1100.0f;
  int max_harm = 16;
  float freq_tol = 0.0001f;
  bool verbose = false;
};
bool parse_coincidencer_cmdline(CoincidencerOptions& args, int argc, const char* const* argv,
                                bool* exit_now = nullptr);

// FFA pipeline options (include/utils/cmdline.hpp:35-50 FFACmdLineOptions,
// :211-292 read_ffa_cmdline_options): same flags and defaults.
struct FfaCmdLineOptions {
  std::string infilename;
  std::string outfilename;
  std::string killfilename;
  int max_num_threads = 14;
  unsigned int nstreams = 16;
  float dm_start = 0.0f;
  float dm_end = 100.0f;
  float dm_tol = 1.10f;
  float dm_pulse_width = 64.0f;
  float p_start = 0.8f;
  float p_end = 20.0f;
  float min_dc = 0.001f;
  bool verbose = false;
  bool progress_bar = false;
  // MI355X-native extensions (long options only)
  float min_snr = 7.0f;
  int nbins = 0;
  int limit = 1000;
  double cluster_tol = 2.0;
  std::string dedisp_kernel = "auto";
};
// "%Y-%m-%d-%H:%M_ffaster.output" in UTC (cmdline.hpp:61-67).
std::string default_ffa_output_filename();
bool parse_ffa_cmdline(FfaCmdLineOptions& args, const std::vector<std::string>& argv, bool* exit_now = nullptr);

}  // namespace psoup
