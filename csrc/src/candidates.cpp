#include "psoup/candidates.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "psoup/common.hpp"

namespace psoup {

static constexpr double kSpeedOfLight = 299792458.0;

int Candidate::count_assoc() const {
  int count = 0;
  for (const auto& a : assoc) {
    count++;
    count += a.count_assoc();
  }
  return count;
}

void Candidate::collect_candidates(std::vector<CandidatePOD>& out) const {
  out.push_back(pod());
  for (const auto& a : assoc) a.collect_candidates(out);
}

void Candidate::set_fold(const float* ar, int nbins_, int nints_) {
  nbins = nbins_;
  nints = nints_;
  fold.assign(ar, ar + static_cast<size_t>(nbins_) * nints_);
}

std::string Candidate::print() const {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%.15f\t%.15f\t%.15f\t%.2f\t%.2f\t%d\t%.1f\t%.1f\t%d\t%d\t%.4f\t%.4f\t%d\n",
                1.0 / freq, opt_period, static_cast<double>(freq), static_cast<double>(dm),
                static_cast<double>(acc), nh, static_cast<double>(snr), static_cast<double>(folded_snr),
                static_cast<int>(is_adjacent), static_cast<int>(is_physical),
                static_cast<double>(ddm_count_ratio), static_cast<double>(ddm_snr_ratio),
                static_cast<int>(assoc.size()));
  std::string s(buf);
  for (const auto& a : assoc) s += a.print();
  return s;
}

namespace {

// c[i] = old c[order[i]], each candidate moved once
void apply_order(CandidateList& c, const std::vector<uint32_t>& order) {
  CandidateList out;
  out.reserve(c.size());
  for (uint32_t i : order) out.push_back(std::move(c[i]));
  c = std::move(out);
}

// BaseDistiller::distill (distiller.hpp:27-59): sort by S/N, then every
// surviving candidate in turn (the "fundamental") marks the later candidates
// related to it as non-unique (appending them to its assoc list when
// keep_related).  The reference scans every later candidate for every
// fundamental -- O(n^2) relation tests, 128-512 ratio tests each for the
// harmonic distiller -- which becomes the host bottleneck on candidate-heavy
// data.  Each distiller here also gives, per
// fundamental, frequency windows that contain every candidate its relation
// can accept; above kIndexedMin candidates those windows are looked up in a
// frequency-sorted index and only the candidates found are tested, in
// ascending S/N-rank order with the reference's exact relation (same
// floating-point expressions, same append order and multiplicity), so the
// output is identical to the O(n^2) scan (tests: distill_reference).
constexpr size_t kIndexedMin = 64;

struct FreqIndex {
  std::vector<double> f;        // ascending
  std::vector<uint32_t> rank;   // S/N rank of f[i]
  explicit FreqIndex(const CandidateList& c) {
    std::vector<uint32_t> order(c.size());
    for (size_t i = 0; i < c.size(); ++i) order[i] = static_cast<uint32_t>(i);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
      return static_cast<double>(c[a].freq) < static_cast<double>(c[b].freq);
    });
    f.resize(order.size());
    rank.resize(order.size());
    for (size_t i = 0; i < order.size(); ++i) {
      f[i] = c[order[i]].freq;
      rank[i] = order[i];
    }
  }
  // ranks > idx with frequency in [lo, hi], appended to out
  void query(double lo, double hi, size_t idx, std::vector<uint32_t>& out) const {
    auto it = std::lower_bound(f.begin(), f.end(), lo);
    for (size_t i = static_cast<size_t>(it - f.begin()); i < f.size() && f[i] <= hi; ++i)
      if (rank[i] > idx) out.push_back(rank[i]);
  }
  // the same for windows sorted by lo (and hi): one forward pointer,
  // galloping to each window's start instead of a full binary search
  void query_sorted(const std::vector<std::pair<double, double>>& w, size_t idx, std::vector<uint32_t>& out) const {
    const size_t n = f.size();
    size_t p = 0;
    for (const auto& [lo, hi] : w) {
      if (p < n && f[p] < lo) {
        size_t q = p, step = 1;
        while (q + step < n && f[q + step] < lo) {
          q += step;
          step <<= 1;
        }
        const size_t e = std::min(q + step, n);
        p = static_cast<size_t>(std::lower_bound(f.begin() + static_cast<long>(q) + 1, f.begin() + static_cast<long>(e), lo) -
                                f.begin());
      }
      for (size_t i = p; i < n && f[i] <= hi; ++i)
        if (rank[i] > idx) out.push_back(rank[i]);
    }
  }
};

// windows(c, idx, push(lo, hi)) lists the fundamental's frequency windows;
// related(c, idx, ii) is the reference's inner-loop body for one later
// candidate: how many times the reference appends ii to idx's assoc list
// (0: unrelated; with keep_related off, 1 for related).
//
// keep_related: the reference copies each related candidate (with its own
// assoc tree) into the fundamental's list at once; here the appends are
// recorded and materialised after the scan, the last use of each candidate
// moved instead of copied.  The result is the same: an appended candidate is
// non-unique from then on, so it never becomes a fundamental and its
// contents never change after the first append (fundamentals are the only
// candidates whose lists grow, and they are never appended).  On the config-4
// candidate list (138k candidates carrying 1.56M associated ones) the DM
// distillation went 363 -> ~30 ms.
template <class Windows, class Related>
CandidateList base_distill(CandidateList cands, Windows&& windows, Related&& related, bool keep, bool force_scan = false,
                           bool sorted_windows = false) {
  const size_t size = cands.size();
  std::vector<char> unique(size, 1);
  // std::sort (not stable_sort) on purpose: with the same input order it breaks
  // S/N ties exactly as the reference's libstdc++ introsort does.  Sorted as
  // an index permutation (std::sort's result depends only on the comparison
  // outcomes), each candidate then moved once.
  {
    std::vector<uint32_t> order(size);
    for (size_t i = 0; i < size; ++i) order[i] = static_cast<uint32_t>(i);
    std::vector<float> snr(size);
    for (size_t i = 0; i < size; ++i) snr[i] = cands[i].snr;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return snr[a] > snr[b]; });
    apply_order(cands, order);
  }
  const bool indexed = !force_scan && size >= kIndexedMin;
  std::unique_ptr<FreqIndex> index;
  if (indexed) index = std::make_unique<FreqIndex>(cands);
  std::vector<uint32_t> hits;
  std::vector<std::pair<double, double>> wins;
  std::vector<std::pair<uint32_t, uint32_t>> appends;  // (fundamental, appended), in the reference's order
  std::vector<uint32_t> uses;                           // appends of each candidate
  if (keep) uses.assign(size, 0);
  auto relate = [&](size_t fi, size_t ii) {
    const int n = related(cands, fi, ii);
    if (n <= 0) return;
    unique[ii] = 0;
    if (keep)
      for (int r = 0; r < n; ++r) {
        appends.emplace_back(static_cast<uint32_t>(fi), static_cast<uint32_t>(ii));
        uses[ii]++;
      }
  };
  size_t start = 0;
  while (true) {
    long idx = -1;
    for (size_t ii = start; ii < size; ++ii) {
      if (unique[ii]) {
        start = ii + 1;
        idx = static_cast<long>(ii);
        break;
      }
    }
    if (idx < 0) break;
    const size_t fi = static_cast<size_t>(idx);
    if (!indexed) {
      for (size_t ii = fi + 1; ii < size; ++ii) relate(fi, ii);
      continue;
    }
    hits.clear();
    if (sorted_windows) {
      wins.clear();
      windows(cands, fi, [&](double lo, double hi) {
        const double m = 1e-9 * std::max(std::fabs(lo), std::fabs(hi));
        wins.emplace_back(lo - m, hi + m);
      });
      index->query_sorted(wins, fi, hits);
    } else {
      windows(cands, fi, [&](double lo, double hi) {
        // a relative 1e-9 margin covers the rounding of the window bounds; the
        // exact relation decides membership
        const double m = 1e-9 * std::max(std::fabs(lo), std::fabs(hi));
        index->query(lo - m, hi + m, fi, hits);
      });
    }
    std::sort(hits.begin(), hits.end());
    hits.erase(std::unique(hits.begin(), hits.end()), hits.end());
    for (uint32_t ii : hits) relate(fi, ii);
  }
  for (const auto& [fi, ii] : appends) {
    if (--uses[ii] == 0)
      cands[fi].assoc.push_back(std::move(cands[ii]));
    else
      cands[fi].assoc.push_back(cands[ii]);
  }
  CandidateList out;
  for (size_t ii = 0; ii < size; ++ii)
    if (unique[ii]) out.push_back(std::move(cands[ii]));
  return out;
}

}  // namespace

CandidateList HarmonicDistiller::distill(CandidateList cands) const { return run(std::move(cands), false); }

CandidateList HarmonicDistiller::run(CandidateList cands, bool force_scan) const {
  const double upper_tol = 1 + tol_;
  const double lower_tol = 1 - tol_;
  const float max_harm = max_harm_;
  const bool keep = keep_related_, frac = fractional_;
  int max_nh = 0;
  for (const auto& c : cands) max_nh = std::max(max_nh, c.nh);
  const float max_den_all = frac ? static_cast<float>(std::pow(2.0, max_nh)) : 1.f;
  // ratio = kk f / (jj fundi) in (lower, upper)  <=>  f in (lower, upper) * jj fundi / kk:
  // the distinct jj / kk ascending, so each fundamental's windows come sorted
  std::vector<double> ratios;
  for (int jj = 1; jj <= max_harm; ++jj)
    for (int kk = 1; kk <= max_den_all; ++kk) ratios.push_back(static_cast<double>(jj) / kk);
  std::sort(ratios.begin(), ratios.end());
  ratios.erase(std::unique(ratios.begin(), ratios.end(),
                           [](double a, double b) { return std::fabs(a - b) <= 1e-12 * b; }),
               ratios.end());
  auto windows = [&](const CandidateList& c, size_t idx, auto&& push) {
    const double fundi_freq = c[idx].freq;
    for (double r : ratios) push(lower_tol * r * fundi_freq, upper_tol * r * fundi_freq);
  };
  // the reference scan (force_scan) keeps the reference's full jj x kk loop
  const bool fast = !keep && tol_ <= 1e-3f && !force_scan;
  auto related = [&](const CandidateList& c, size_t idx, size_t ii) -> int {
    const double fundi_freq = c[idx].freq;
    const double freq = c[ii].freq;
    const int nh = c[ii].nh;
    const float max_denominator =
        frac ? (nh >= 0 && nh < 24 ? static_cast<float>(1u << nh) : static_cast<float>(std::pow(2.0, nh))) : 1.f;
    if (fast) {
      // Only the whole result matters: for each kk just the jj nearest
      // kk freq / fundi (|jj - that| <= 16 tol < 0.02 for any passing jj)
      // and its neighbours, tested with the exact expression.
      // (a multiply-and-round prefilter skips every kk whose kk freq / fundi
      // is not within 1.5 jj tol of an integer jj: only then the exact test)
      const double x1 = freq / fundi_freq;
      for (int kk = 1; kk <= max_denominator; ++kk) {
        const double x = kk * x1;
        if (!(x < max_harm + 2.0)) break;
        const int j0 = static_cast<int>(std::lround(x));
        if (j0 < 1 || j0 > max_harm || std::fabs(x - j0) > 1.5 * tol_ * j0 + 1e-9) continue;
        const double ratio = kk * freq / (j0 * fundi_freq);
        if (ratio > lower_tol && ratio < upper_tol) return 1;
      }
      return 0;
    }
    // every (jj, kk) match appends once (keep_related)
    int n = 0;
    for (int jj = 1; jj <= max_harm; ++jj) {
      for (int kk = 1; kk <= max_denominator; ++kk) {
        const double ratio = kk * freq / (jj * fundi_freq);
        if (ratio > lower_tol && ratio < upper_tol) ++n;
      }
    }
    return keep ? n : (n > 0 ? 1 : 0);
  };
  return base_distill(std::move(cands), windows, related, keep, force_scan, true);
}

AccelerationDistiller::AccelerationDistiller(float tobs, float tol, bool keep_related)
    : tobs_(tobs), tol_(tol), keep_related_(keep_related) {
  tobs_over_c_ = tobs_ / kSpeedOfLight;
}

CandidateList AccelerationDistiller::distill(CandidateList cands) const { return run(std::move(cands), false); }

CandidateList AccelerationDistiller::run(CandidateList cands, bool force_scan) const {
  const double toc = tobs_over_c_;
  const float tol = tol_;
  const bool keep = keep_related_;
  double acc_min = 0.0, acc_max = 0.0;
  for (size_t i = 0; i < cands.size(); ++i) {
    acc_min = i ? std::min(acc_min, static_cast<double>(cands[i].acc)) : cands[i].acc;
    acc_max = i ? std::max(acc_max, static_cast<double>(cands[i].acc)) : cands[i].acc;
  }
  auto windows = [&](const CandidateList& c, size_t idx, auto&& push) {
    // acc_freq spans fundi + (fundi_acc - acc) fundi toc over the candidates' accelerations
    const double fundi_freq = c[idx].freq, fundi_acc = c[idx].acc, edge = fundi_freq * tol;
    const double a1 = fundi_freq + (fundi_acc - acc_max) * fundi_freq * toc;
    const double a2 = fundi_freq + (fundi_acc - acc_min) * fundi_freq * toc;
    // acc_freq is rounded to float in the relation: widen by 1e-6 relative
    const double lo = std::min({fundi_freq, a1, a2}) - edge, hi = std::max({fundi_freq, a1, a2}) + edge;
    push(lo - 1e-6 * std::fabs(lo), hi + 1e-6 * std::fabs(hi));
  };
  auto related = [&](const CandidateList& c, size_t idx, size_t ii) -> int {
    const double fundi_freq = c[idx].freq;
    const double fundi_acc = c[idx].acc;
    const double edge = fundi_freq * tol;
    const double delta_acc = fundi_acc - c[ii].acc;
    // correct_for_acceleration returns float (distiller.hpp:120-122).
    const double acc_freq = static_cast<float>(fundi_freq + delta_acc * fundi_freq * toc);
    const double f = c[ii].freq;
    bool rel;
    if (acc_freq > fundi_freq)
      rel = (f > fundi_freq - edge && f < acc_freq + edge);
    else
      rel = (f < fundi_freq + edge && f > acc_freq - edge);
    return rel ? 1 : 0;
  };
  return base_distill(std::move(cands), windows, related, keep, force_scan);
}

CandidateList DMDistiller::distill(CandidateList cands) const { return run(std::move(cands), false); }

CandidateList DMDistiller::run(CandidateList cands, bool force_scan) const {
  const double upper_tol = 1 + tol_;
  const double lower_tol = 1 - tol_;
  const bool keep = keep_related_;
  auto windows = [&](const CandidateList& c, size_t idx, auto&& push) {
    const double fundi_freq = c[idx].freq;
    push(lower_tol * fundi_freq, upper_tol * fundi_freq);
  };
  auto related = [&](const CandidateList& c, size_t idx, size_t ii) -> int {
    const double ratio = c[ii].freq / static_cast<double>(c[idx].freq);
    return ratio > lower_tol && ratio < upper_tol ? 1 : 0;
  };
  return base_distill(std::move(cands), windows, related, keep, force_scan);
}

CandidateScorer::CandidateScorer(float tsamp, float cfreq, float foff, float bw)
    : tsamp_(tsamp), cfreq_(cfreq), foff_(foff) {
  float ftop = static_cast<float>(cfreq + bw / 2.0);
  float fbottom = static_cast<float>(cfreq - bw / 2.0);
  tdm_chan_partial_ = static_cast<float>(8300.0 * foff / std::pow(cfreq, 3.0));
  tdm_band_partial_ = static_cast<float>(4150.0 * (1.0 / std::pow(fbottom, 2) - 1.0 / std::pow(ftop, 2)));
}

void CandidateScorer::score(Candidate& cand) const {
  cand.is_physical = 1.0 / cand.freq > cand.dm * tdm_chan_partial_;
  {
    const int idx = cand.dm_idx;
    bool adjacent = false, unique = true;
    for (const auto& a : cand.assoc) {
      if (a.dm_idx != idx) unique = false;
      if (a.dm_idx == idx + 1 || a.dm_idx == idx - 1) {
        adjacent = true;
        break;
      }
    }
    cand.is_adjacent = adjacent || unique;
  }
  {
    int inside_count = 1, total_count = 1;
    float inside_snr = cand.snr, total_snr = cand.snr;
    float ddm = static_cast<float>(1.0 / (cand.freq * tdm_band_partial_));
    for (const auto& a : cand.assoc) {
      total_count++;
      total_snr += a.snr;
      if (std::fabs(cand.dm - a.dm) <= ddm) {
        inside_count++;
        inside_snr += a.snr;
      }
    }
    cand.ddm_count_ratio = static_cast<float>(inside_count) / total_count;
    cand.ddm_snr_ratio = inside_snr / total_snr;
  }
}

void CandidateScorer::score_all(CandidateList& cands) const {
  for (auto& c : cands) score(c);
}

void identify_unique_peaks(const int* idxs, const float* snrs, size_t count, int min_gap,
                           std::vector<int>& peak_idxs, std::vector<float>& peak_snrs) {
  size_t ii = 0;
  while (ii < count) {
    float cpeak = snrs[ii];
    int cpeakidx = idxs[ii];
    int lastidx = idxs[ii];
    ii++;
    while (ii < count && (idxs[ii] - lastidx) < min_gap) {
      if (snrs[ii] > cpeak) {
        cpeak = snrs[ii];
        cpeakidx = idxs[ii];
        lastidx = idxs[ii];
      }
      ii++;
    }
    peak_idxs.push_back(cpeakidx);
    peak_snrs.push_back(cpeak);
  }
}

PeakBounds peak_bounds(int size, float bin_width, int nh, float min_freq, float max_freq) {
  PeakBounds b;
  const float nyquist = bin_width * size;
  const int orig_size = static_cast<int>(2.0 * (size - 1.0));
  const double p2 = std::pow(2.0, nh);
  const int max_bin = static_cast<int>((max_freq / bin_width) * p2);
  b.start_idx = static_cast<int>(orig_size * (min_freq / nyquist) * p2);
  b.end_idx = std::min(size, max_bin);
  b.factor = 1.0 / size * nyquist / std::pow(2.0, static_cast<float>(nh));
  if (b.start_idx < 0) b.start_idx = 0;
  return b;
}

void stable_sort_by_dm_idx(CandidateList& c) {
  std::vector<uint32_t> order(c.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<uint32_t>(i);
  // std::stable_sort's permutation depends on the comparison outcomes alone
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return c[a].dm_idx < c[b].dm_idx; });
  apply_order(c, order);
}

CandidateList accel_distill_slices(CandidateList all, const std::vector<int>& slice, const AccelerationDistiller& d,
                                   int nthreads) {
  PSOUP_CHECK(slice.size() == all.size(), "accel_distill_slices: one slice index per candidate");
  // (dm_idx, slice) order, stable: a slice's candidates keep their trial order
  std::vector<uint32_t> order(all.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<uint32_t>(i);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return all[a].dm_idx != all[b].dm_idx ? all[a].dm_idx < all[b].dm_idx : slice[a] < slice[b];
  });
  apply_order(all, order);
  std::vector<std::pair<size_t, size_t>> runs;  // one DM each
  for (size_t i = 0; i < all.size();) {
    size_t j = i + 1;
    while (j < all.size() && all[j].dm_idx == all[i].dm_idx) ++j;
    runs.emplace_back(i, j);
    i = j;
  }
  std::vector<CandidateList> out(runs.size());
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex err_mu;
  auto work = [&] {
    try {
      for (size_t r; (r = next.fetch_add(1)) < runs.size();) {
        CandidateList one(std::make_move_iterator(all.begin() + static_cast<std::ptrdiff_t>(runs[r].first)),
                          std::make_move_iterator(all.begin() + static_cast<std::ptrdiff_t>(runs[r].second)));
        out[r] = d.distill(std::move(one));
      }
    } catch (...) {
      std::lock_guard<std::mutex> lk(err_mu);
      if (!err) err = std::current_exception();
      next.store(runs.size());
    }
  };
  const int nt = std::max(1, std::min<int>(nthreads, static_cast<int>(runs.size())));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  if (err) std::rethrow_exception(err);
  CandidateList res;
  for (auto& l : out)
    for (auto& c : l) res.push_back(std::move(c));
  return res;
}

void sort_by_folded_snr(CandidateList& cands) {
  std::sort(cands.begin(), cands.end(), [](const Candidate& x, const Candidate& y) {
    return std::max(x.snr, x.folded_snr) > std::max(y.snr, y.folded_snr);
  });
}

// ------------------------------------------------------------ serialise ----
// Two record forms.  The full one carries every field (folded candidates,
// checkpoints); the compact one (magic "PSOD") only what a candidate has
// before folding and scoring -- the DM, acceleration, harmonic, S/N and
// frequency of each node and its association count -- 28 instead of 55 bytes
// a node.  The multi-rank merge ships search-stage lists (peak-heavy ranks:
// ~15 MB a step in the full form), so the compact form halves what is
// gathered, and serialised and rebuilt on both ends.
namespace {
constexpr uint32_t kMagicFull = 0x50534F43u;     // "PSOC"
constexpr uint32_t kMagicCompact = 0x50534F44u;  // "PSOD"
#pragma pack(push, 1)
struct NodeRec {
  float dm;
  int32_t dm_idx;
  float acc;
  int32_t nh;
  float snr;
  float freq;
  float folded_snr;
  double opt_period;
  uint8_t is_adjacent;
  uint8_t is_physical;
  float ddm_count_ratio;
  float ddm_snr_ratio;
  int32_t nbins;
  int32_t nints;
  int32_t nfold;
  int32_t nassoc;
};
struct CompactRec {
  float dm;
  int32_t dm_idx;
  float acc;
  int32_t nh;
  float snr;
  float freq;
  int32_t nassoc;
};
#pragma pack(pop)

void put(std::vector<uint8_t>& out, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  out.insert(out.end(), b, b + n);
}

// no field beyond the compact record's set (bit patterns: -0.0 is not default)
template <typename T>
bool zero_bits(T v) {
  unsigned char b[sizeof(T)];
  std::memcpy(b, &v, sizeof(T));
  for (unsigned char x : b)
    if (x) return false;
  return true;
}
bool search_stage(const Candidate& c) {
  auto zero = [](float f) { return zero_bits(f); };
  return zero(c.folded_snr) && zero_bits(c.opt_period) && !c.is_adjacent && !c.is_physical &&
         zero(c.ddm_count_ratio) && zero(c.ddm_snr_ratio) && c.nbins == 0 && c.nints == 0 && c.fold.empty();
}
bool search_stage_tree(const Candidate& c) {
  if (!search_stage(c)) return false;
  for (const auto& a : c.assoc)
    if (!search_stage_tree(a)) return false;
  return true;
}

void ser_node(const Candidate& c, std::vector<uint8_t>& out) {
  NodeRec r{c.dm, c.dm_idx, c.acc, c.nh, c.snr, c.freq, c.folded_snr, c.opt_period,
            static_cast<uint8_t>(c.is_adjacent), static_cast<uint8_t>(c.is_physical), c.ddm_count_ratio,
            c.ddm_snr_ratio, c.nbins, c.nints, static_cast<int32_t>(c.fold.size()),
            static_cast<int32_t>(c.assoc.size())};
  put(out, &r, sizeof(r));
  if (!c.fold.empty()) put(out, c.fold.data(), c.fold.size() * sizeof(float));
  for (const auto& a : c.assoc) ser_node(a, out);
}

void ser_compact(const Candidate& c, std::vector<uint8_t>& out) {
  CompactRec r{c.dm, c.dm_idx, c.acc, c.nh, c.snr, c.freq, static_cast<int32_t>(c.assoc.size())};
  put(out, &r, sizeof(r));
  for (const auto& a : c.assoc) ser_compact(a, out);
}

size_t tree_nodes(const Candidate& c) {
  size_t n = 1;
  for (const auto& a : c.assoc) n += tree_nodes(a);
  return n;
}

struct Reader {
  const uint8_t* p;
  size_t n, off = 0;
  void get(void* dst, size_t k) {
    PSOUP_CHECK(off + k <= n, "truncated candidate stream");
    std::memcpy(dst, p + off, k);
    off += k;
  }
};

template <bool COMPACT>
Candidate de_node(Reader& r, int depth) {
  PSOUP_CHECK(depth < 64, "candidate tree too deep");
  if constexpr (COMPACT) {
    CompactRec rec;
    r.get(&rec, sizeof(rec));
    PSOUP_CHECK(rec.nassoc >= 0, "corrupt candidate record");
    Candidate c(rec.dm, rec.dm_idx, rec.acc, rec.nh, rec.snr, rec.freq);
    c.assoc.reserve(static_cast<size_t>(rec.nassoc));
    for (int i = 0; i < rec.nassoc; ++i) c.assoc.push_back(de_node<true>(r, depth + 1));
    return c;
  } else {
    NodeRec rec;
    r.get(&rec, sizeof(rec));
    Candidate c(rec.dm, rec.dm_idx, rec.acc, rec.nh, rec.snr, rec.freq);
    c.folded_snr = rec.folded_snr;
    c.opt_period = rec.opt_period;
    c.is_adjacent = rec.is_adjacent != 0;
    c.is_physical = rec.is_physical != 0;
    c.ddm_count_ratio = rec.ddm_count_ratio;
    c.ddm_snr_ratio = rec.ddm_snr_ratio;
    c.nbins = rec.nbins;
    c.nints = rec.nints;
    PSOUP_CHECK(rec.nfold >= 0 && rec.nassoc >= 0, "corrupt candidate record");
    if (rec.nfold > 0) {
      c.fold.resize(static_cast<size_t>(rec.nfold));
      r.get(c.fold.data(), c.fold.size() * sizeof(float));
    }
    c.assoc.reserve(static_cast<size_t>(rec.nassoc));
    for (int i = 0; i < rec.nassoc; ++i) c.assoc.push_back(de_node<false>(r, depth + 1));
    return c;
  }
}

// past one record and its subtree (headers only): the byte offsets of the
// top-level records, so their subtrees can be rebuilt in parallel
template <bool COMPACT>
void skip_node(Reader& r, int depth) {
  PSOUP_CHECK(depth < 64, "candidate tree too deep");
  if constexpr (COMPACT) {
    CompactRec rec;
    r.get(&rec, sizeof(rec));
    PSOUP_CHECK(rec.nassoc >= 0, "corrupt candidate record");
    for (int i = 0; i < rec.nassoc; ++i) skip_node<true>(r, depth + 1);
  } else {
    NodeRec rec;
    r.get(&rec, sizeof(rec));
    PSOUP_CHECK(rec.nfold >= 0 && rec.nassoc >= 0, "corrupt candidate record");
    PSOUP_CHECK(r.off + static_cast<size_t>(rec.nfold) * sizeof(float) <= r.n, "truncated candidate stream");
    r.off += static_cast<size_t>(rec.nfold) * sizeof(float);
    for (int i = 0; i < rec.nassoc; ++i) skip_node<false>(r, depth + 1);
  }
}

template <bool COMPACT>
void deserialize_body(const uint8_t* data, size_t nbytes, Reader& r, int64_t n, CandidateList& out) {
  const size_t base = out.size();
  // Large streams (a merge of 138k candidates carrying 1.6M associated ones:
  // ~100 MB) are rebuilt on several threads: one header-only pass finds each
  // top-level record, then contiguous ranges of records are deserialised in
  // parallel straight into their final positions.
  const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  if (nbytes < (8u << 20) || hw == 1 || n < 1024) {
    out.reserve(base + static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) out.push_back(de_node<COMPACT>(r, 0));
    PSOUP_CHECK(r.off == nbytes, "trailing bytes after the candidate stream");
    return;
  }
  std::vector<size_t> at(static_cast<size_t>(n) + 1);
  for (int64_t i = 0; i < n; ++i) {
    at[static_cast<size_t>(i)] = r.off;
    skip_node<COMPACT>(r, 0);
  }
  at[static_cast<size_t>(n)] = r.off;
  PSOUP_CHECK(r.off == nbytes, "trailing bytes after the candidate stream");
  out.resize(base + static_cast<size_t>(n));
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> err(hw);
  for (unsigned t = 0; t < hw; ++t)
    th.emplace_back([&, t] {
      try {
        // ranges balanced by bytes
        const size_t lo = nbytes / hw * t, hi = t + 1 == hw ? nbytes : nbytes / hw * (t + 1);
        size_t i0 = static_cast<size_t>(std::lower_bound(at.begin(), at.end() - 1, lo) - at.begin());
        size_t i1 = t + 1 == hw ? static_cast<size_t>(n)
                                : static_cast<size_t>(std::lower_bound(at.begin(), at.end() - 1, hi) - at.begin());
        for (size_t i = i0; i < i1; ++i) {
          Reader rr{data, nbytes, at[i]};
          out[base + i] = de_node<COMPACT>(rr, 0);
        }
      } catch (...) {
        err[t] = std::current_exception();
      }
    });
  for (auto& x : th) x.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}
}  // namespace

std::vector<uint8_t> serialize_candidates(const CandidateList& cands) {
  std::vector<const Candidate*> p;
  p.reserve(cands.size());
  for (const auto& c : cands) p.push_back(&c);
  return serialize_candidates(p);
}

std::vector<uint8_t> serialize_candidates(const std::vector<const Candidate*>& cands) {
  std::vector<uint8_t> out;
  bool compact = true;
  size_t nodes = 0;
  for (const Candidate* c : cands) {
    if (compact && !search_stage_tree(*c)) compact = false;
    nodes += tree_nodes(*c);
  }
  out.reserve(12 + nodes * (compact ? sizeof(CompactRec) : sizeof(NodeRec)));
  const uint32_t magic = compact ? kMagicCompact : kMagicFull;
  int64_t n = static_cast<int64_t>(cands.size());
  put(out, &magic, 4);
  put(out, &n, 8);
  for (const Candidate* c : cands) {
    if (compact)
      ser_compact(*c, out);
    else
      ser_node(*c, out);
  }
  return out;
}

void deserialize_candidates_into(const uint8_t* data, size_t nbytes, CandidateList& out) {
  if (nbytes == 0) return;
  Reader r{data, nbytes};
  uint32_t magic = 0;
  int64_t n = 0;
  r.get(&magic, 4);
  PSOUP_CHECK(magic == kMagicFull || magic == kMagicCompact, "bad candidate stream magic");
  r.get(&n, 8);
  PSOUP_CHECK(n >= 0, "bad candidate count");
  if (magic == kMagicCompact)
    deserialize_body<true>(data, nbytes, r, n, out);
  else
    deserialize_body<false>(data, nbytes, r, n, out);
}

CandidateList deserialize_candidates(const uint8_t* data, size_t nbytes) {
  CandidateList out;
  deserialize_candidates_into(data, nbytes, out);
  return out;
}

}  // namespace psoup
