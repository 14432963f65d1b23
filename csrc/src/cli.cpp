#include "psoup/cli.hpp"

#include <cstdlib>
#include <ctime>
#include <functional>
#include <iostream>
#include <sstream>

namespace psoup {

namespace {

struct Spec {
  std::string shortf;  // without '-'
  std::string longf;   // without '--'
  std::string help;
  bool is_switch;
  bool required;
  std::function<bool(const std::string&)> set;  // returns false on bad value
  std::function<void()> flip;                    // for switches
};

template <class T>
bool parse_num(const std::string& s, T& out) {
  std::istringstream ss(s);
  T v;
  ss >> v;
  if (ss.fail()) return false;
  std::string rest;
  ss >> rest;
  if (!rest.empty()) return false;
  out = v;
  return true;
}

bool parse_uint(const std::string& s, unsigned int& out) {
  if (!s.empty() && s[0] == '-') return false;
  unsigned long long v;
  if (!parse_num(s, v)) return false;
  out = static_cast<unsigned int>(v);
  return true;
}

Spec val_s(const char* s, const char* l, const char* help, std::string& dst, bool required = false) {
  return Spec{s, l, help, false, required, [&dst](const std::string& v) { dst = v; return true; }, nullptr};
}
template <class T>
Spec val_n(const char* s, const char* l, const char* help, T& dst) {
  return Spec{s, l, help, false, false, [&dst](const std::string& v) { return parse_num(v, dst); }, nullptr};
}
Spec val_u(const char* s, const char* l, const char* help, unsigned int& dst) {
  return Spec{s, l, help, false, false, [&dst](const std::string& v) { return parse_uint(v, dst); }, nullptr};
}
Spec sw(const char* s, const char* l, const char* help, bool& dst) {
  return Spec{s, l, help, true, false, nullptr, [&dst]() { dst = true; }};
}

std::string usage_of(const std::string& prog, const std::vector<Spec>& specs, const std::string& positional) {
  std::ostringstream os;
  os << "USAGE: \n\n   " << prog;
  for (const auto& s : specs) {
    os << " ";
    if (!s.required) os << "[";
    os << (s.shortf.empty() ? "--" + s.longf : "-" + s.shortf);
    if (!s.is_switch) os << " <value>";
    if (!s.required) os << "]";
  }
  if (!positional.empty()) os << " <" << positional << "> ...";
  os << "\n\nWhere: \n\n";
  for (const auto& s : specs) {
    os << "   ";
    if (!s.shortf.empty()) os << "-" << s.shortf << ",  ";
    os << "--" << s.longf << "\n     " << s.help << "\n\n";
  }
  os << "   -h,  --help\n     Displays usage information and exits.\n\n";
  os << "   --version\n     Displays version information and exits.\n";
  return os.str();
}

// Generic parser.  positional != nullptr collects unlabeled arguments.
bool run_parser(const std::vector<Spec>& specs, const std::vector<std::string>& argv, const std::string& title,
                std::vector<std::string>* positional, bool* exit_now) {
  if (exit_now) *exit_now = false;
  std::vector<bool> seen(specs.size(), false);
  auto find_short = [&](const std::string& f) -> int {
    for (size_t i = 0; i < specs.size(); ++i)
      if (!specs[i].shortf.empty() && specs[i].shortf == f) return static_cast<int>(i);
    return -1;
  };
  auto find_long = [&](const std::string& f) -> int {
    for (size_t i = 0; i < specs.size(); ++i)
      if (specs[i].longf == f) return static_cast<int>(i);
    return -1;
  };
  const std::string prog = argv.empty() ? "peasoup" : argv[0];
  for (size_t i = 1; i < argv.size(); ++i) {
    const std::string& a = argv[i];
    if (a == "-h" || a == "--help") {
      std::cout << title << "\n\n" << usage_of(prog, specs, positional ? "filterbanks" : "") << std::endl;
      if (exit_now) *exit_now = true;
      return true;
    }
    if (a == "--version") {
      std::cout << "\n" << prog << "  version: 1.0\n" << std::endl;
      if (exit_now) *exit_now = true;
      return true;
    }
    int idx = -1;
    std::string value;
    bool has_value = false;
    if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
      std::string name = a.substr(2);
      auto eq = name.find('=');
      if (eq != std::string::npos) {
        value = name.substr(eq + 1);
        name = name.substr(0, eq);
        has_value = true;
      }
      idx = find_long(name);
      if (idx < 0) {
        std::cerr << "Error: Couldn't find match for argument " << a << std::endl;
        return false;
      }
    } else if (a.size() > 1 && a[0] == '-' && !(std::isdigit(static_cast<unsigned char>(a[1])) || a[1] == '.')) {
      std::string name = a.substr(1);
      idx = find_short(name);
      if (idx < 0) {
        // combined switches, e.g. -vp
        bool all = true;
        for (char ch : name) {
          int k = find_short(std::string(1, ch));
          if (k < 0 || !specs[k].is_switch) {
            all = false;
            break;
          }
        }
        if (!all) {
          std::cerr << "Error: Couldn't find match for argument " << a << std::endl;
          return false;
        }
        for (char ch : name) {
          int k = find_short(std::string(1, ch));
          specs[k].flip();
          seen[k] = true;
        }
        continue;
      }
    } else {
      if (positional) {
        positional->push_back(a);
        continue;
      }
      std::cerr << "Error: Couldn't find match for argument " << a << std::endl;
      return false;
    }
    const Spec& s = specs[idx];
    if (s.is_switch) {
      if (has_value) {
        std::cerr << "Error: switch " << a << " takes no value" << std::endl;
        return false;
      }
      s.flip();
      seen[idx] = true;
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argv.size()) {
        std::cerr << "Error: Missing a value for this argument! for arg " << a << std::endl;
        return false;
      }
      value = argv[++i];
    }
    if (!s.set(value)) {
      std::cerr << "Error: Couldn't read argument value from string '" << value << "' for arg " << a << std::endl;
      return false;
    }
    seen[idx] = true;
  }
  for (size_t i = 0; i < specs.size(); ++i) {
    if (specs[i].required && !seen[i]) {
      std::cerr << "Error: Required argument missing: " << (specs[i].shortf.empty() ? "" : "-" + specs[i].shortf + ", ")
                << "--" << specs[i].longf << std::endl;
      return false;
    }
  }
  return true;
}

}  // namespace

std::string default_outdir() {
  char buf[128];
  std::time_t t = std::time(nullptr);
  std::strftime(buf, sizeof(buf), "./%Y-%m-%d-%H:%M_peasoup/", std::gmtime(&t));
  return std::string(buf);
}

static std::vector<Spec> peasoup_specs(CmdLineOptions& a) {
  return {
      val_s("i", "inputfile", "File to process (.fil)", a.infilename, true),
      val_s("o", "outdir", "The output directory", a.outdir),
      val_s("k", "killfile", "Channel mask file", a.killfilename),
      val_s("z", "zapfile", "Birdie list file", a.zapfilename),
      val_n("t", "num_threads", "The number of GPUs to use", a.max_num_threads),
      val_n("", "limit", "upper limit on number of candidates to write out", a.limit),
      val_u("", "fft_size", "Transform size to use (defaults to lower power of two)", a.size),
      val_n("", "dm_start", "First DM to dedisperse to", a.dm_start),
      val_n("", "dm_end", "Last DM to dedisperse to", a.dm_end),
      val_n("", "dm_tol", "DM smearing tolerance (1.11=10%)", a.dm_tol),
      val_n("", "dm_pulse_width", "Minimum pulse width for which dm_tol is valid", a.dm_pulse_width),
      val_n("", "acc_start", "First acceleration to resample to", a.acc_start),
      val_n("", "acc_end", "Last acceleration to resample to", a.acc_end),
      val_n("", "acc_tol", "Acceleration smearing tolerance (1.11=10%)", a.acc_tol),
      val_n("", "acc_pulse_width", "Minimum pulse width for which acc_tol is valid", a.acc_pulse_width),
      val_n("", "boundary_5_freq", "Frequency at which to switch from median5 to median25", a.boundary_5_freq),
      val_n("", "boundary_25_freq", "Frequency at which to switch from median25 to median125", a.boundary_25_freq),
      val_n("n", "nharmonics", "Number of harmonic sums to perform", a.nharmonics),
      val_n("", "npdmp", "Number of candidates to fold and pdmp", a.npdmp),
      val_n("m", "min_snr", "The minimum S/N for a candidate", a.min_snr),
      val_n("", "min_freq", "Lowest Fourier freqency to consider", a.min_freq),
      val_n("", "max_freq", "Highest Fourier freqency to consider", a.max_freq),
      val_n("", "max_harm_match", "Maximum harmonic for related candidates", a.max_harm),
      val_n("", "freq_tol", "Tolerance for distilling frequencies (0.0001 = 0.01%)", a.freq_tol),
      sw("v", "verbose", "verbose mode", a.verbose),
      sw("p", "progress_bar", "Enable progress bar for DM search", a.progress_bar),
      // MI355X-native extensions
      val_s("", "accel_convention", "Acceleration-plan unit convention: legacy (default, golden) | reference",
            a.accel_convention),
      val_s("", "dedisp_kernel", "Dedispersion kernel: auto | mfma | valu | direct | packed2", a.dedisp_kernel),
      val_n("", "accel_batch", "Acceleration trials per batched FFT (0 = auto)", a.accel_batch),
      val_n("", "engines_per_gpu",
            "Search engines per GPU, each on its own stream and host thread, dealt every N-th DM of a chunk "
            "(0 = auto: Python driver 3 when DMs have < 128 acceleration trials, else 1; native pipeline 1)",
            a.engines_per_gpu),
      val_s("", "dm_schedule",
            "Multi-rank DM distribution (python -m peasoup_amd under torchrun): dynamic = ranks claim DM chunks "
            "from a shared first-come queue, like the reference's DMDispenser; static = contiguous shards balanced "
            "by acceleration-trial count; auto = dynamic when the list has >= 4 chunks per rank",
            a.dm_schedule),
      val_n("", "accel_slices",
            "Multi-rank Python driver: acceleration-trial slices per DM work unit, so DMs with many trials "
            "spread over the ranks (0 = auto: split when the job has fewer than 4 DM chunks per rank; 1 = never)",
            a.accel_slices),
      val_n("", "sub_batch", "Fused-FFT trials per sub-batch on two alternating streams (0 = off, -1 = auto)",
            a.sub_batch),
      val_n("", "fft_mode", "Accel-trial FFT: 2 = fused resample + four-step FFT (default), 1 = rocFFT C2C(N/2), 0 = rocFFT R2C",
            a.fft_mode),
      sw("", "use_boundaries", "Honour --boundary_* in the running median (reference ignores them)",
         a.use_boundaries),
      val_s("", "checkpoint_dir", "Spill per-DM candidates here and resume from it", a.checkpoint_dir),
      val_s("", "trace_json", "Write per-stage timings as JSON to this file", a.trace_json),
      val_n("", "fault_after_dms", "Testing: abort after this many DM trials", a.fault_after_dms),
      sw("", "time_shards",
         "Python driver under torchrun: each rank holds only its time slice of the filterbank; ring halo exchange "
         "+ all-to-all corner turn to DM shards (series too long to replicate on every GPU)",
         a.time_shards),
  };
}

bool parse_cmdline(CmdLineOptions& args, const std::vector<std::string>& argv, bool* exit_now) {
  args.outdir = default_outdir();
  auto specs = peasoup_specs(args);
  return run_parser(specs, argv, "Peasoup - a GPU pulsar search pipeline", nullptr, exit_now);
}

bool parse_cmdline(CmdLineOptions& args, int argc, const char* const* argv, bool* exit_now) {
  std::vector<std::string> v(argv, argv + argc);
  return parse_cmdline(args, v, exit_now);
}

std::string cmdline_usage() {
  CmdLineOptions a;
  return usage_of("peasoup", peasoup_specs(a), "");
}

bool parse_coincidencer_cmdline(CoincidencerOptions& a, int argc, const char* const* argv, bool* exit_now) {
  std::vector<Spec> specs = {
      val_s("", "o", "Sample mask output filename", a.samp_outfilename),
      val_s("", "o2", "Birdie list output filename", a.spec_outfilename),
      val_n("l", "boundary_5_freq", "Frequency at which to switch from median5 to median25", a.boundary_5_freq),
      val_n("a", "boundary_25_freq", "Frequency at which to switch from median25 to median125", a.boundary_25_freq),
      val_n("n", "nharmonics", "Number of harmonic sums to perform", a.nharmonics),
      val_n("", "thresh", "The S/N threshold for a candidate to be considered for coincidencing matching",
            a.threshold),
      val_n("", "beam_thresh", "The number of beams a candidate must appear in to be considered multibeam",
            a.beam_threshold),
      val_n("L", "min_freq", "Lowest Fourier freqency to consider", a.min_freq),
      val_n("H", "max_freq", "Highest Fourier freqency to consider", a.max_freq),
      val_n("b", "max_harm", "Maximum harmonic for related candidates", a.max_harm),
      val_n("f", "freq_tol", "Tolerance for distilling frequencies (0.0001 = 0.01%)", a.freq_tol),
      sw("v", "verbose", "verbose mode", a.verbose),
  };
  std::vector<std::string> v(argv, argv + argc);
  if (!run_parser(specs, v, "Peasoup - a GPU pulsar search pipeline", &a.filterbanks, exit_now)) return false;
  if ((!exit_now || !*exit_now) && a.filterbanks.empty()) {
    std::cerr << "Error: Required argument missing: filterbanks" << std::endl;
    return false;
  }
  return true;
}

std::string default_ffa_output_filename() {
  char buf[128];
  std::time_t t = std::time(nullptr);
  std::strftime(buf, sizeof(buf), "%Y-%m-%d-%H:%M_ffaster.output", std::gmtime(&t));
  return std::string(buf);
}

bool parse_ffa_cmdline(FfaCmdLineOptions& a, const std::vector<std::string>& argv, bool* exit_now) {
  a.outfilename = default_ffa_output_filename();
  std::vector<Spec> specs = {
      val_s("i", "inputfile", "File to process (.fil)", a.infilename, true),
      val_s("o", "outfilename", "The output filename", a.outfilename),
      val_s("k", "killfile", "Channel mask file", a.killfilename),
      val_n("t", "num_threads", "The number of GPUs to use", a.max_num_threads),
      val_u("", "nstreams", "The number of CUDA streams to use", a.nstreams),
      val_n("", "dm_start", "First DM to dedisperse to", a.dm_start),
      val_n("", "dm_end", "Last DM to dedisperse to", a.dm_end),
      val_n("", "dm_tol", "DM smearing tolerance (1.11=10%)", a.dm_tol),
      val_n("", "dm_pulse_width", "Minimum pulse width for which dm_tol is valid", a.dm_pulse_width),
      val_n("", "p_start", "Start period for FFA search", a.p_start),
      val_n("", "p_end", "End period for FFA search", a.p_end),
      val_n("", "min_dc", "Minimum duty cycle", a.min_dc),
      sw("v", "verbose", "verbose mode", a.verbose),
      sw("p", "progress_bar", "Enable progress bar for DM search", a.progress_bar),
      // MI355X-native extensions
      val_n("m", "min_snr", "Minimum boxcar S/N of a folded profile", a.min_snr),
      val_n("", "bins", "Base bins per period (periods span [bins, 2 bins)); 0 = from --min_dc", a.nbins),
      val_n("", "limit", "Upper limit on the number of candidates written", a.limit),
      val_n("", "cluster_tol", "Peak clustering tolerance in units of 1/T_obs", a.cluster_tol),
      val_s("", "dedisp_kernel", "Dedispersion kernel: auto | mfma | valu | direct | packed2", a.dedisp_kernel),
  };
  return run_parser(specs, argv, "Peasoup/FFAster extension - a GPU FFA pulsar search pipeline", nullptr, exit_now);
}

}  // namespace psoup
