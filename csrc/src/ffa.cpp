// FFA search engine, octave planning, clustering and the ffaster options.
// See psoup/ffa.hpp; reference: include/utils/cmdline.hpp:35-67, 211-292.
#include "psoup/ffa.hpp"

#include <algorithm>
#include <cmath>
#include <ctime>
#include <iostream>

#include <atomic>
#include <cstdio>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

#include "psoup/cli.hpp"
#include "psoup/engine.hpp"
#include "psoup/kernels.hpp"
#include "psoup/pipeline.hpp"
#include "psoup/plan.hpp"
#include "psoup/sigproc.hpp"

namespace psoup {

int ffa_base_bins(const FfaParams& p) {
  if (p.nbins > 0) return std::min(p.nbins, kern::ffa_max_profile() / 2);
  // periods span [nb0, 2 nb0) bins: the narrowest pulse (one bin) at the
  // octave top has duty cycle 1 / (2 nb0) = min_dc
  const double want = 0.5 / std::max(1e-6, static_cast<double>(p.min_dc));
  return static_cast<int>(std::min(1024.0, std::max(32.0, std::ceil(want))));
}

std::vector<int> ffa_widths(int nb0) {
  // geometric ladder (x ~1.5) from one bin to half of the smallest period
  std::vector<int> w;
  double v = 1.0;
  while (static_cast<int>(w.size()) < kern::kFfaMaxWidths) {
    const int iv = static_cast<int>(std::lround(v));
    if (iv > nb0 / 2) break;
    if (w.empty() || iv > w.back()) w.push_back(iv);
    v *= 1.5;
  }
  return w;
}

std::vector<FfaOctave> ffa_plan(const FfaParams& p, uint64_t n) {
  PSOUP_CHECK(p.tsamp > 0 && p.p_start > 0 && p.p_end > p.p_start, "ffa: bad period range");
  const int nb0 = ffa_base_bins(p);
  std::vector<FfaOctave> plan;
  for (int o = 0; o < 64; ++o) {
    const double plo = p.p_start * std::ldexp(1.0, o);
    if (plo >= p.p_end) break;
    FfaOctave oc;
    oc.factor = std::max(1.0, plo / (nb0 * p.tsamp));
    oc.nds = static_cast<uint64_t>(std::floor(static_cast<double>(n) / oc.factor));
    const double bin_s = oc.factor * p.tsamp;
    oc.pa = std::max(2, static_cast<int>(std::lround(plo / bin_s)));
    oc.pb = std::min(2 * oc.pa, static_cast<int>(std::ceil(p.p_end / bin_s)));
    oc.pb = std::min(oc.pb, kern::ffa_max_profile() + 1);
    FfaChunk ch;
    auto flush = [&]() {
      if (!ch.periods.empty()) oc.chunks.push_back(std::move(ch));
      ch = FfaChunk();
    };
    for (int P = oc.pa; P < oc.pb; ++P) {
      const uint64_t m = oc.nds / static_cast<uint64_t>(P);
      if (m < static_cast<uint64_t>(std::max(2, p.min_rows))) continue;
      int lg = 0;
      while ((uint64_t(1) << lg) < m) ++lg;
      const uint64_t m2 = uint64_t(1) << lg;
      const uint64_t need = m2 * static_cast<uint64_t>(P);
      PSOUP_CHECK(need <= p.arena_floats, "ffa: one period exceeds the arena (raise arena_floats)");
      if (ch.arena + need > p.arena_floats || ch.periods.size() >= 65535) flush();
      kern::FfaPeriod fp{};
      fp.p = P;
      fp.m = static_cast<int32_t>(m);
      fp.m2 = static_cast<int32_t>(m2);
      fp.log2m2 = lg;
      fp.offset = ch.arena;
      fp.best_offset = ch.nprof;
      ch.periods.push_back(fp);
      ch.arena += need;
      ch.nprof += m2;
      ch.max_m2 = std::max(ch.max_m2, static_cast<int>(m2));
      ch.max_log2m2 = std::max(ch.max_log2m2, lg);
      ch.max_p = std::max(ch.max_p, P);
    }
    flush();
    if (!oc.chunks.empty()) plan.push_back(std::move(oc));
  }
  return plan;
}

FfaCandidateList ffa_cluster(FfaCandidateList c, double tol_hz) {
  // greedy in S/N order; neighbours found through a frequency-sorted index
  // (O(n log n + n k) instead of the distillers' O(n^2))
  std::stable_sort(c.begin(), c.end(), [](const FfaCandidate& a, const FfaCandidate& b) { return a.snr > b.snr; });
  const size_t n = c.size();
  std::vector<size_t> by_f(n);
  for (size_t i = 0; i < n; ++i) by_f[i] = i;
  std::stable_sort(by_f.begin(), by_f.end(), [&](size_t a, size_t b) { return c[a].freq() < c[b].freq(); });
  std::vector<size_t> rank(n);
  for (size_t r = 0; r < n; ++r) rank[by_f[r]] = r;
  std::vector<char> dead(n, 0);
  FfaCandidateList out;
  for (size_t i = 0; i < n; ++i) {
    if (dead[i]) continue;
    const double fi = c[i].freq();
    for (size_t r = rank[i] + 1; r < n && c[by_f[r]].freq() - fi < tol_hz; ++r) dead[by_f[r]] = 1;
    for (size_t r = rank[i]; r-- > 0 && fi - c[by_f[r]].freq() < tol_hz;) dead[by_f[r]] = 1;
    dead[i] = 0;
    out.push_back(c[i]);
  }
  return out;
}

FfaEngine::FfaEngine(const FfaParams& p, uint64_t nsamps, hipStream_t stream) : p_(p), n_(nsamps), stream_(stream) {
  PSOUP_CHECK(n_ >= 64, "ffa: series too short");
  plan_ = ffa_plan(p_, n_);
  uint64_t arena = 0, maxds = 0;
  for (const auto& o : plan_) {
    maxds = std::max(maxds, o.nds);
    for (const auto& c : o.chunks) {
      arena = std::max(arena, c.arena);
      tables_.emplace_back(c.periods.size());
      PSOUP_HIP_CHECK(hipMemcpy(tables_.back().data(), c.periods.data(), c.periods.size() * sizeof(kern::FfaPeriod),
                                hipMemcpyHostToDevice));
    }
  }
  x_.resize(n_);
  ds_.resize(std::max<uint64_t>(1, maxds));
  a0_.resize(std::max<uint64_t>(1, arena));
  a1_.resize(std::max<uint64_t>(1, arena));
  uint64_t window = static_cast<uint64_t>(std::ceil((p_.detrend_s > 0 ? p_.detrend_s : 3.0 * p_.p_end) / p_.tsamp));
  window = std::min<uint64_t>(std::max<uint64_t>(window, 64), n_);
  means_.resize((n_ + window - 1) / window);
  sums_.resize((n_ + window - 1) / window);
  partials_.resize(2 * 1024);
  stats_.resize(4);
  cap_ = 1u << 14;
  const std::vector<int> w = ffa_widths(ffa_base_bins(p_));
  snr_.nwidths = static_cast<int32_t>(w.size());
  for (size_t i = 0; i < w.size(); ++i) snr_.widths[i] = w[i];
  snr_.thresh = p_.min_snr;
}

FfaEngine::~FfaEngine() { (void)hipStreamSynchronize(stream_); }

FfaCandidateList FfaEngine::search(const uint8_t* d_trial, float dm, int dm_idx) {
  hipStream_t s = stream_;
  uint64_t window = static_cast<uint64_t>(std::ceil((p_.detrend_s > 0 ? p_.detrend_s : 3.0 * p_.p_end) / p_.tsamp));
  window = std::min<uint64_t>(std::max<uint64_t>(window, 64), n_);
  kern::ffa_detrend(d_trial, n_, window, sums_.data(), means_.data(), x_.data(), s);
  kern::f32_stats(x_.data(), n_, partials_.data(), 1024, stats_.data(), s);
  kern::normalise_dev(x_.data(), n_, stats_.data(), 1.0f, s);
  // Every chunk of every octave is issued back to back (one S/N record
  // buffer and counter per chunk); the host synchronises once per DM.  A
  // record-buffer overflow (rare) grows the buffers and reruns the DM.
  size_t nchunks = 0;
  for (const auto& oc : plan_) nchunks += oc.chunks.size();
  std::vector<uint32_t> counts(nchunks);
  for (int attempt = 0; attempt < 3; ++attempt) {
    if (d_peaks_.size() < nchunks * cap_) d_peaks_.resize(nchunks * cap_);
    if (d_count_.size() < nchunks) d_count_.resize(nchunks);
    PSOUP_HIP_CHECK(hipMemsetAsync(d_count_.data(), 0, nchunks * sizeof(uint32_t), s));
    size_t t = 0;
    for (size_t o = 0; o < plan_.size(); ++o) {
      const FfaOctave& oc = plan_[o];
      kern::ffa_downsample(x_.data(), n_, oc.factor, ds_.data(), oc.nds, s);
      kern::FfaSnrParams sp = snr_;
      sp.var_per_bin = static_cast<float>(oc.factor);
      for (const FfaChunk& ch : oc.chunks) {
        const kern::FfaPeriod* dper = tables_[t].data();
        const int nper = static_cast<int>(ch.periods.size());
        kern::ffa_transform(ds_.data(), dper, nper, ch.max_m2, ch.max_log2m2, ch.max_p, a0_.data(), a1_.data(), s);
        kern::ffa_snr(dper, nper, ch.max_m2, ch.max_p, a0_.data(), a1_.data(), sp, d_peaks_.data() + t * cap_,
                      d_count_.data() + t, cap_, nullptr, s);
        ++t;
      }
    }
    PSOUP_HIP_CHECK(hipMemcpyAsync(counts.data(), d_count_.data(), nchunks * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PSOUP_HIP_CHECK(hipStreamSynchronize(s));
    const uint32_t mx = nchunks ? *std::max_element(counts.begin(), counts.end()) : 0;
    if (mx <= cap_) break;
    PSOUP_CHECK(attempt < 2, "ffa: peak buffer overflow persists");
    cap_ = mx + mx / 4;
  }
  FfaCandidateList raw;
  size_t t = 0;
  for (size_t o = 0; o < plan_.size(); ++o) {
    const FfaOctave& oc = plan_[o];
    const double bin_s = oc.factor * p_.tsamp;
    for (const FfaChunk& ch : oc.chunks) {
      const uint32_t cnt = counts[t];
      nprof_ += ch.nprof;
      npeaks_ += cnt;
      h_peaks_.resize(cnt);
      if (cnt)
        PSOUP_HIP_CHECK(hipMemcpy(h_peaks_.data(), d_peaks_.data() + t * cap_, cnt * sizeof(kern::FfaPeak),
                                  hipMemcpyDeviceToHost));
      for (const auto& pk : h_peaks_) {
        const kern::FfaPeriod& fp = ch.periods[static_cast<size_t>(pk.period_idx)];
        const double pbins = fp.m2 > 1 ? fp.p + static_cast<double>(pk.drift) / (fp.m2 - 1) : fp.p;
        FfaCandidate c;
        c.period = pbins * bin_s;
        c.snr = pk.snr;
        c.width = pk.width;
        c.nbins = fp.p;
        c.dm = dm;
        c.dm_idx = dm_idx;
        c.octave = static_cast<int>(o);
        raw.push_back(c);
      }
      ++t;
    }
  }
  return ffa_cluster(std::move(raw), p_.cluster_tol / tobs());
}

FfaParams ffa_params_from(const FfaCmdLineOptions& a, double tsamp) {
  FfaParams p;
  p.tsamp = tsamp;
  p.p_start = a.p_start;
  p.p_end = a.p_end;
  p.min_dc = a.min_dc;
  p.nbins = a.nbins;
  p.min_snr = a.min_snr;
  p.cluster_tol = a.cluster_tol;
  return p;
}

FfaResult run_ffa_pipeline(const FfaCmdLineOptions& args) {
  FfaResult res;
  Stopwatch t_total, t_read;
  t_total.start();
  if (args.verbose) set_log_level(LogLevel::Verbose);
  t_read.start();
  Filterbank fb = Filterbank::from_file(args.infilename);
  t_read.stop();
  const SigprocHeader& hdr = fb.header();
  res.dm_list = generate_dm_list(args.dm_start, args.dm_end, hdr.tsamp, args.dm_pulse_width, hdr.fch1, hdr.foff,
                                 hdr.nchans, args.dm_tol);
  std::vector<int> kill(static_cast<size_t>(hdr.nchans), 1);
  if (!args.killfilename.empty()) kill = read_killfile(args.killfilename, hdr.nchans);
  const int ndev = device_count();
  PSOUP_CHECK(ndev > 0, "no HIP devices visible");
  const int ngpu = std::max(1, std::min(ndev, args.max_num_threads));
  for (int i = 0; i < ngpu; ++i) res.devices.push_back(i);
  DedispGeometry geom = DedispGeometry::make(hdr, fb.nsamps(), res.dm_list, kill);
  res.nsamps = geom.out_nsamps;
  const FfaParams fp = ffa_params_from(args, hdr.tsamp);
  res.plan = ffa_plan(fp, res.nsamps);
  res.nb0 = ffa_base_bins(fp);
  res.tobs = static_cast<double>(res.nsamps) * hdr.tsamp;
  const DedispKernel dk = parse_dedisp_kernel(args.dedisp_kernel);
  const int ndm = static_cast<int>(res.dm_list.size());
  const int chunk = std::max(1, std::min(16, ndm / (4 * ngpu) + 1));
  std::atomic<int> next{0}, done{0};
  std::atomic<uint64_t> nprof{0}, npeaks{0};
  std::mutex mu;
  std::exception_ptr err;
  FfaCandidateList all;
  std::vector<double> dedisp_s(static_cast<size_t>(ngpu), 0.0), search_s(static_cast<size_t>(ngpu), 0.0);
  ProgressBar progress("FFA search over DM trials");
  if (args.progress_bar) progress.start();
  Stopwatch t_search;
  t_search.start();
  auto worker = [&](int dev) {
    try {
      PSOUP_HIP_CHECK(hipSetDevice(dev));
      Stream stream;
      DeviceFilterbank dfb(geom, stream.get());
      load_filterbank_fanout({&dfb}, {dev}, fb);
      Dedisperser dd(dfb, stream.get());
      FfaEngine eng(fp, geom.out_nsamps, stream.get());
      const uint64_t rs = Dedisperser::row_stride(geom.out_nsamps);
      DeviceBuffer<uint8_t> trials(rs * static_cast<uint64_t>(chunk));
      Stopwatch wd, ws;
      while (true) {
        const int d0 = next.fetch_add(chunk);
        if (d0 >= ndm) break;
        const int d1 = std::min(ndm, d0 + chunk);
        wd.start();
        dd.run(d0, d1, trials.data(), rs, dk);
        PSOUP_HIP_CHECK(hipStreamSynchronize(stream.get()));
        wd.stop();
        ws.start();
        FfaCandidateList local;
        for (int d = d0; d < d1; ++d) {
          FfaCandidateList c = eng.search(trials.data() + static_cast<uint64_t>(d - d0) * rs,
                                          res.dm_list[static_cast<size_t>(d)], d);
          log_verbose("FFA DM " + std::to_string(res.dm_list[static_cast<size_t>(d)]) + ": " +
                      std::to_string(c.size()) + " candidates");
          for (auto& x : c) local.push_back(x);
        }
        ws.stop();
        {
          std::lock_guard<std::mutex> lk(mu);
          for (auto& x : local) all.push_back(x);
        }
        const int dn = done.fetch_add(d1 - d0) + (d1 - d0);
        if (args.progress_bar) progress.set(static_cast<double>(dn) / ndm);
      }
      nprof += eng.profiles();
      npeaks += eng.peaks();
      dedisp_s[static_cast<size_t>(dev)] = wd.get_time();
      search_s[static_cast<size_t>(dev)] = ws.get_time();
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!err) err = std::current_exception();
      next.store(ndm + 1000000);
    }
  };
  std::vector<std::thread> th;
  for (int d = 0; d < ngpu; ++d) th.emplace_back(worker, d);
  for (auto& t : th) t.join();
  t_search.stop();
  if (args.progress_bar) progress.stop();
  if (err) std::rethrow_exception(err);
  // deterministic order before the cross-DM clustering
  std::stable_sort(all.begin(), all.end(), [](const FfaCandidate& a, const FfaCandidate& b) {
    return a.dm_idx != b.dm_idx ? a.dm_idx < b.dm_idx : a.period < b.period;
  });
  res.candidates = ffa_cluster(std::move(all), fp.cluster_tol / res.tobs);
  if (args.limit >= 0 && res.candidates.size() > static_cast<size_t>(args.limit))
    res.candidates.resize(static_cast<size_t>(args.limit));
  res.profiles = nprof.load();
  res.peaks = npeaks.load();
  t_total.stop();
  res.timers["reading"] = t_read.get_time();
  res.timers["dedispersion"] = *std::max_element(dedisp_s.begin(), dedisp_s.end());
  res.timers["searching"] = t_search.get_time();
  res.timers["total"] = t_total.get_time();
  return res;
}

void write_ffa_output(const std::string& path, const FfaCmdLineOptions& args, const FfaResult& res) {
  FILE* fo = std::fopen(path.c_str(), "w");
  PSOUP_CHECK(fo != nullptr, "cannot open FFA output " << path);
  std::fprintf(fo, "# peasoup_amd FFA search (ffaster)\n# input: %s\n", args.infilename.c_str());
  std::fprintf(fo, "# dm_trials: %zu (%.3f..%.3f)  period: %.6f..%.6f s  min_dc: %g  base_bins: %d  T_obs: %.3f s\n",
               res.dm_list.size(), res.dm_list.empty() ? 0.0 : res.dm_list.front(),
               res.dm_list.empty() ? 0.0 : res.dm_list.back(), static_cast<double>(args.p_start),
               static_cast<double>(args.p_end), static_cast<double>(args.min_dc), res.nb0, res.tobs);
  std::fprintf(fo, "# profiles: %llu  peaks: %llu  min_snr: %g  searching: %.3f s  total: %.3f s\n",
               static_cast<unsigned long long>(res.profiles), static_cast<unsigned long long>(res.peaks),
               static_cast<double>(args.min_snr), res.timers.count("searching") ? res.timers.at("searching") : 0.0,
               res.timers.count("total") ? res.timers.at("total") : 0.0);
  std::fprintf(fo, "#%5s %18s %16s %10s %7s %9s %7s %10s %6s %7s\n", "id", "period_s", "freq_hz", "dm", "dm_idx",
               "snr", "width", "duty_cycle", "nbins", "octave");
  for (size_t i = 0; i < res.candidates.size(); ++i) {
    const FfaCandidate& c = res.candidates[i];
    std::fprintf(fo, "%6zu %18.12f %16.10f %10.4f %7d %9.3f %7d %10.6f %6d %7d\n", i, c.period, c.freq(),
                 static_cast<double>(c.dm), c.dm_idx, static_cast<double>(c.snr), c.width, c.duty_cycle(), c.nbins,
                 c.octave);
  }
  std::fclose(fo);
}

}  // namespace psoup
