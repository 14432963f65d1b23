// End-to-end peasoup pipeline (src/pipeline_multi.cu:262-419).
//
// Reference structure: host reads the .fil, dedisp dedisperses ALL DMs on
// the GPUs and copies the 8-bit trials back to host RAM; one pthread per GPU
// then pulls DM indices from a mutex queue, copies each trial back H2D and
// searches it; results are concatenated after pthread_join; folding runs on
// one device afterwards.
//
// Here: each GPU worker holds the filterbank resident in HBM (channel-major)
// and pulls CHUNKS of DMs from a lock-free queue; it dedisperses the chunk
// on the MFMA kernel straight into HBM and searches it there -- trials never
// leave the GPU.  Folding is distributed over the same workers (candidates
// grouped by DM, re-dedispersing only the DMs that hold fold candidates).
// Optional per-chunk candidate spill files give checkpoint/resume.
#pragma once

#include <functional>
#include <map>
#include <string>
#include <vector>

#include "psoup/candidates.hpp"
#include "psoup/cli.hpp"
#include "psoup/engine.hpp"
#include "psoup/plan.hpp"
#include "psoup/sigproc.hpp"

namespace psoup {

struct SearchSetup {
  SigprocHeader header;
  uint64_t nsamps = 0;        // filterbank samples
  std::vector<float> dm_list;
  std::vector<int> killmask;
  uint64_t fft_size = 0;
  AccelPlan accel_plan;
  SearchParams search;
  DedispKernel dedisp_kernel = DedispKernel::Auto;
  float cfreq = 0.f;
};

// Builds everything that follows from the CLI options and the header
// (DM list, killmask, fft size, acceleration plan, search parameters).
SearchSetup make_search_setup(const CmdLineOptions& args, const SigprocHeader& hdr);

// Global post-processing after the search (pipeline_multi.cu:353-369):
// DM distill (keep related), harmonic distill (keep related, integer
// harmonics only), scoring.
CandidateList global_distill_and_score(CandidateList cands, const CmdLineOptions& args, const SearchSetup& s);

// Fold selection of MultiFolder::fold_n (folder.hpp:424-434): the first n
// candidates with 1 ms < P < 10 s grouped by dm_idx.
std::map<int, std::vector<int>> select_fold_candidates(const CandidateList& cands, int n);

class ProgressBar {
 public:
  explicit ProgressBar(std::string title);
  ~ProgressBar();
  void start();
  void set(double frac);
  void stop();

 private:
  struct Impl;
  Impl* impl_;
};

struct PipelineResult {
  CandidateList candidates;                 // final, sorted, limited
  std::map<std::string, double> timers;     // reading/dedispersion/searching/folding/total (s)
  std::map<std::string, double> performance;
  std::vector<int> devices;
  SearchSetup setup;
  // per device: dedispersion_s, search_s, dm_trials, accel_trials, peaks,
  // peak_overflows, accel_loop_s, host_distill_s, fft_mode, accel_batch
  std::vector<std::map<std::string, double>> device_stats;
};

// Per-stage JSON trace (--trace_json): timers, performance, per-device
// counters and the search configuration.
std::string trace_json(const CmdLineOptions& args, const PipelineResult& res,
                       const std::map<std::string, double>& extra_performance = {});

// Runs the whole search in this process on `ndevices` GPUs (threads).
PipelineResult run_pipeline(const CmdLineOptions& args);

// Writes candidates.peasoup + overview.xml into args.outdir.
void write_outputs(const CmdLineOptions& args, const PipelineResult& res);

}  // namespace psoup
