// `ffaster`: FFA periodicity search over DM trials -- the pipeline behind the
// reference's FFA options (include/utils/cmdline.hpp:35-50, 211-292;
// Makefile:41-42 target ${BIN_DIR}/ffaster, source not in the reference).
#include <iostream>

#include "psoup/cli.hpp"
#include "psoup/common.hpp"
#include "psoup/ffa.hpp"

using namespace psoup;

int main(int argc, char** argv) {
  FfaCmdLineOptions args;
  bool exit_now = false;
  std::vector<std::string> av(argv, argv + argc);
  if (!parse_ffa_cmdline(args, av, &exit_now)) return 1;
  if (exit_now) return 0;
  try {
    FfaResult res = run_ffa_pipeline(args);
    write_ffa_output(args.outfilename, args, res);
    if (args.verbose)
      std::cout << "FFA search: " << res.dm_list.size() << " DM trials, " << res.candidates.size()
                << " candidates -> " << args.outfilename << " (" << res.timers["total"] << " s)" << std::endl;
  } catch (const std::exception& e) {
    std::cerr << "ffaster: " << e.what() << std::endl;
    return 2;
  }
  return 0;
}
