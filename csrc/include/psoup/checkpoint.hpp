// Checkpoint / resume: per-DM-chunk candidate spill files bound to the run
// that wrote them.
//
// The reference has no checkpointing (outputs are written only
// at the end, pipeline_multi.cu:393-416).  Here both drivers (native
// run_pipeline and the Python RankSearcher) spill the candidate trees of every
// finished DM chunk to <dir>/dm_<d0>_<d1>.psoc and skip chunks whose spill is
// present on a rerun.  A spill is only reused when it was written by the same
// run: every file carries a 64-bit key hashed from the run identity (input
// file path, size and sampled content, header, every option that changes the
// per-DM candidates, killfile/zapfile contents, format version), plus a
// payload hash that catches truncated or corrupt files.  A mismatching or
// corrupt spill is ignored and recomputed; <dir>/manifest.txt records the
// identity text of the run that last used the directory.
#pragma once

#include <cstdint>
#include <string>

#include "psoup/candidates.hpp"
#include "psoup/cli.hpp"
#include "psoup/sigproc.hpp"

namespace psoup {

struct RunIdentity {
  std::string text;  // canonical, human-readable description (manifest.txt)
  uint64_t key = 0;  // FNV-1a 64 of text
};

// Identity of a search run.  `hdr` is the header the search uses (its
// nsamples included); the input file is read for its size and 16 sampled
// 4 KiB blocks when it exists (a synthetic input is identified by name).
RunIdentity make_run_identity(const CmdLineOptions& args, const SigprocHeader& hdr);

uint64_t fnv1a64(const void* data, size_t n, uint64_t h = 0xcbf29ce484222325ull);

// <dir>/dm_<d0>_<d1>.psoc
std::string spill_path(const std::string& dir, int d0, int d1);

// Creates the directory and (re)writes manifest.txt; logs a warning when the
// directory held spills of a different run (they are then ignored).
void prepare_checkpoint_dir(const std::string& dir, const RunIdentity& id);

enum class SpillStatus { Missing = 0, Loaded = 1, Mismatch = 2, Corrupt = 3 };

// Appends the spill's candidates to `out` only when it is Loaded.
SpillStatus load_spill(const std::string& path, uint64_t key, CandidateList& out);

// Writes atomically (unique temporary + rename); throws psoup::Error on any
// write or rename failure, so a bad spill is never committed.
void save_spill(const std::string& path, uint64_t key, const CandidateList& cands);

const char* spill_status_name(SpillStatus s);

}  // namespace psoup
