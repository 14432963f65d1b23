// Candidates and host-side candidate post-processing.
//
// Parity:
//   include/data_types/candidates.hpp:10-166   Candidate / CandidatePOD /
//       CandidateCollection / SpectrumCandidates
//   include/transforms/distiller.hpp:16-197    Base/Harmonic/Acceleration/DM
//       distillers (greedy O(n^2) after an S/N sort; the related-candidate
//       test does NOT skip already-absorbed candidates, and a candidate that
//       matches several (harmonic, fraction) pairs is appended once per
//       match -- reproduced exactly).
//   include/transforms/scorer.hpp:8-87         CandidateScorer
//   include/transforms/peakfinder.hpp:27-56    identify_unique_peaks
//       (the cluster gap is measured from the LAST MAXIMUM, not from the last
//       element of the run -- reproduced).
// The S/N sort is std::sort like the reference (same tie order for the same
// input order).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace psoup {

#pragma pack(push, 1)
struct CandidatePOD {
  float dm;
  int32_t dm_idx;
  float acc;
  int32_t nh;
  float snr;
  float freq;
};
#pragma pack(pop)
static_assert(sizeof(CandidatePOD) == 24, "CandidatePOD must be 24 bytes (on-disk format)");

struct Candidate {
  float dm = 0.f;
  int dm_idx = 0;
  float acc = 0.f;
  int nh = 0;
  float snr = 0.f;
  float freq = 0.f;
  float folded_snr = 0.f;
  double opt_period = 0.0;
  bool is_adjacent = false;
  bool is_physical = false;
  float ddm_count_ratio = 0.f;
  float ddm_snr_ratio = 0.f;
  std::vector<Candidate> assoc;
  std::vector<float> fold;  // [nints][nbins]
  int nbins = 0;
  int nints = 0;

  Candidate() = default;
  Candidate(float dm_, int dm_idx_, float acc_, int nh_, float snr_, float freq_)
      : dm(dm_), dm_idx(dm_idx_), acc(acc_), nh(nh_), snr(snr_), freq(freq_) {}

  void append(const Candidate& other) { assoc.push_back(other); }
  int count_assoc() const;
  void collect_candidates(std::vector<CandidatePOD>& out) const;
  void set_fold(const float* ar, int nbins_, int nints_);
  CandidatePOD pod() const { return CandidatePOD{dm, dm_idx, acc, nh, snr, freq}; }
  // 13 tab-separated columns (candidates.hpp:78-88), recursive.
  std::string print() const;
};

using CandidateList = std::vector<Candidate>;

// std::stable_sort by dm_idx (the order the reference merges its workers'
// lists in), as one permutation of the candidates instead of moving them
// (with their trees) at every step of the sort: same result.
void stable_sort_by_dm_idx(CandidateList& c);

// ------------------------------------------------------------ distillers ---
class HarmonicDistiller {
 public:
  HarmonicDistiller(float tol, float max_harm, bool keep_related, bool fractional_harms = true)
      : tol_(tol), max_harm_(max_harm), keep_related_(keep_related), fractional_(fractional_harms) {}
  CandidateList distill(CandidateList cands) const;
  // the reference's O(n^2) scan (tests compare the indexed path against it)
  CandidateList distill_reference(CandidateList cands) const { return run(std::move(cands), true); }

 private:
  CandidateList run(CandidateList cands, bool force_scan) const;
  float tol_, max_harm_;
  bool keep_related_, fractional_;
};

class AccelerationDistiller {
 public:
  AccelerationDistiller(float tobs, float tol, bool keep_related);
  CandidateList distill(CandidateList cands) const;
  CandidateList distill_reference(CandidateList cands) const { return run(std::move(cands), true); }

 private:
  CandidateList run(CandidateList cands, bool force_scan) const;
  float tobs_, tol_;
  double tobs_over_c_;
  bool keep_related_;
};

// Acceleration trials of one DM split over work units (SearchEngine::Job::
// raw, possibly searched on several ranks): `all` holds the units' raw lists
// (per-trial harmonic-distilled candidates, trial order within a unit),
// slice[i] the unit slice of top-level candidate i.  Per DM the slices are
// joined in slice (= acceleration plan) order and acceleration-distilled --
// the list SearchEngine distils for an unsplit DM, so the result is the same
// -- on `nthreads` threads; the output is ordered by DM index.
CandidateList accel_distill_slices(CandidateList all, const std::vector<int>& slice, const AccelerationDistiller& d,
                                   int nthreads);

class DMDistiller {
 public:
  DMDistiller(float tol, bool keep_related) : tol_(tol), keep_related_(keep_related) {}
  CandidateList distill(CandidateList cands) const;
  CandidateList distill_reference(CandidateList cands) const { return run(std::move(cands), true); }

 private:
  CandidateList run(CandidateList cands, bool force_scan) const;
  float tol_;
  bool keep_related_;
};

// ---------------------------------------------------------------- scorer ---
class CandidateScorer {
 public:
  CandidateScorer(float tsamp, float cfreq, float foff, float bw);
  void score(Candidate& c) const;
  void score_all(CandidateList& cands) const;

 private:
  float tsamp_, cfreq_, foff_;
  float tdm_chan_partial_, tdm_band_partial_;
};

// ---------------------------------------------------------- peak cluster ---
// idxs ascending; returns (peak idx, peak snr) pairs.
void identify_unique_peaks(const int* idxs, const float* snrs, size_t count, int min_gap,
                           std::vector<int>& peak_idxs, std::vector<float>& peak_snrs);

// Search-range bounds and frequency conversion of one harmonic level, exactly
// as PeakFinder::find_candidates (peakfinder.hpp:77-94) computes them.
struct PeakBounds {
  int start_idx;  // first bin searched
  int end_idx;    // one past the last bin searched (min(size, max_bin))
  double factor;  // freq = (float)(idx * factor)
};
PeakBounds peak_bounds(int nbins, float bin_width, int nh, float min_freq, float max_freq);

// ------------------------------------------------------------ sorting ------
// sort by max(snr, folded_snr) descending (folder.hpp:25-31), stable.
void sort_by_folded_snr(CandidateList& cands);

// --------------------------------------------------------- serialisation ---
// Compact binary encoding of candidate trees (used for the RCCL gather of
// per-rank candidates and for checkpoint spill files).
std::vector<uint8_t> serialize_candidates(const CandidateList& cands);
// the same encoding of candidates held elsewhere (no copy of their trees)
std::vector<uint8_t> serialize_candidates(const std::vector<const Candidate*>& cands);
CandidateList deserialize_candidates(const uint8_t* data, size_t nbytes);
// deserialised candidates appended to `out` (moved, no intermediate list)
void deserialize_candidates_into(const uint8_t* data, size_t nbytes, CandidateList& out);

}  // namespace psoup
