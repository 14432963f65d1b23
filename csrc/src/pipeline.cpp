#include "psoup/pipeline.hpp"

#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>
#include <tuple>

#include "psoup/checkpoint.hpp"
#include "psoup/output.hpp"
#include "psoup/scheduler.hpp"

namespace psoup {

SearchSetup make_search_setup(const CmdLineOptions& args, const SigprocHeader& hdr) {
  SearchSetup s;
  s.header = hdr;
  s.nsamps = static_cast<uint64_t>(hdr.nsamples);
  s.dm_list = generate_dm_list(args.dm_start, args.dm_end, hdr.tsamp, args.dm_pulse_width, hdr.fch1, hdr.foff,
                               hdr.nchans, args.dm_tol);
  s.killmask = std::vector<int>(static_cast<size_t>(hdr.nchans), 1);
  if (!args.killfilename.empty()) s.killmask = read_killfile(args.killfilename, hdr.nchans);
  s.fft_size = args.size == 0 ? prev_power_of_two(s.nsamps) : args.size;
  // cfreq as Filterbank::get_cfreq (float arithmetic)
  {
    float fch1 = static_cast<float>(hdr.fch1), foff = static_cast<float>(hdr.foff);
    float nch = static_cast<float>(static_cast<unsigned>(hdr.nchans));
    s.cfreq = foff < 0 ? fch1 + foff * nch / 2 : fch1 - foff * nch / 2;
  }
  s.accel_plan = AccelPlan(args.acc_start, args.acc_end, args.acc_tol, args.acc_pulse_width, s.fft_size,
                           static_cast<float>(hdr.tsamp), s.cfreq, static_cast<float>(hdr.foff),
                           parse_accel_convention(args.accel_convention));
  SearchParams& p = s.search;
  p.fft_size = s.fft_size;
  p.tsamp = static_cast<float>(hdr.tsamp);
  p.min_snr = args.min_snr;
  p.min_freq = args.min_freq;
  p.max_freq = args.max_freq;
  p.nharmonics = args.nharmonics;
  p.freq_tol = args.freq_tol;
  p.max_harm = args.max_harm;
  // The reference never passes --boundary_* to the dereddener (pipeline_multi.cu:182).
  p.boundary_5_freq = args.use_boundaries ? args.boundary_5_freq : 0.05f;
  p.boundary_25_freq = args.use_boundaries ? args.boundary_25_freq : 0.5f;
  if (!args.zapfilename.empty()) read_zapfile(args.zapfilename, p.zap_freqs, p.zap_widths);
  p.accel_batch = args.accel_batch;
  p.sub_batch = args.sub_batch;
  p.fft_mode = args.fft_mode;
  s.dedisp_kernel = parse_dedisp_kernel(args.dedisp_kernel);
  return s;
}

CandidateList global_distill_and_score(CandidateList cands, const CmdLineOptions& args, const SearchSetup& s) {
  DMDistiller dm_still(args.freq_tol, true);
  HarmonicDistiller harm_still(args.freq_tol, static_cast<float>(args.max_harm), true, false);
  cands = dm_still.distill(std::move(cands));
  cands = harm_still.distill(std::move(cands));
  CandidateScorer scorer(static_cast<float>(s.header.tsamp), s.cfreq, static_cast<float>(s.header.foff),
                         static_cast<float>(std::fabs(s.header.foff) * s.header.nchans));
  scorer.score_all(cands);
  return cands;
}

std::map<int, std::vector<int>> select_fold_candidates(const CandidateList& cands, int n) {
  std::map<int, std::vector<int>> m;
  const int count = std::min(n, static_cast<int>(cands.size()));
  for (int i = 0; i < count; ++i) {
    const float p = static_cast<float>(1.0 / cands[i].freq);
    if (p > 0.001f && p < 10.00f) m[cands[i].dm_idx].push_back(i);
  }
  return m;
}

// ---------------------------------------------------------------- progress --
struct ProgressBar::Impl {
  std::string title;
  std::atomic<double> frac{0.0};
  std::atomic<bool> running{false};
  std::thread th;
  Stopwatch sw;
};

ProgressBar::ProgressBar(std::string title) : impl_(new Impl) { impl_->title = std::move(title); }
ProgressBar::~ProgressBar() {
  stop();
  delete impl_;
}
void ProgressBar::start() {
  if (impl_->running.exchange(true)) return;
  impl_->sw.start();
  impl_->th = std::thread([this] {
    while (impl_->running.load()) {
      double f = impl_->frac.load();
      double el = impl_->sw.get_time();
      double eta = f > 0 ? el / f - el : 0.0;
      int w = 40, fill = static_cast<int>(f * w);
      std::fprintf(stderr, "\r%s [%s%s] %5.1f%%  ETA %6.1f s", impl_->title.c_str(), std::string(fill, '=').c_str(),
                   std::string(w - fill, ' ').c_str(), 100 * f, eta);
      std::fflush(stderr);
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
  });
}
void ProgressBar::set(double f) { impl_->frac.store(f); }
void ProgressBar::stop() {
  if (!impl_->running.exchange(false)) return;
  if (impl_->th.joinable()) impl_->th.join();
  std::fprintf(stderr, "\r%s complete (%.2f s)%40s\n", impl_->title.c_str(), impl_->sw.get_time(), "");
}

// ---------------------------------------------------------------- pipeline --
namespace {

struct Shared {
  const CmdLineOptions* args;
  const SearchSetup* setup;
  const Filterbank* fb;
  int chunk = 8;
  int ndm = 0;
  std::mutex mu;
  CandidateList cands;
  std::atomic<uint64_t> accel_trials{0};
  std::atomic<int> done_dms{0};
  std::vector<double> dedisp_s, search_s;
  std::vector<std::map<std::string, double>> dev_stats;
  std::exception_ptr error;
  ProgressBar* progress = nullptr;
};

}  // namespace

PipelineResult run_pipeline(const CmdLineOptions& args) {
  PipelineResult res;
  Stopwatch t_total, t_read, t_dedisp, t_search, t_fold;
  t_total.start();
  if (args.verbose) set_log_level(LogLevel::Verbose);
  // wall time of each phase in order (trace_json "performance": phase_<name>_s),
  // together the whole of "total"
  double t_mark = 0;
  auto mark = [&](const char* name) {
    const double now = t_total.get_time();
    res.performance[std::string("phase_") + name + "_s"] = now - t_mark;
    t_mark = now;
  };

  t_read.start();
  Filterbank fb = Filterbank::from_file(args.infilename);
  t_read.stop();

  mark("read");
  SearchSetup setup = make_search_setup(args, fb.header());
  res.setup = setup;
  const int ndev_avail = device_count();
  PSOUP_CHECK(ndev_avail > 0, "no HIP devices visible");
  // Device workers: one per GPU (the reference's Worker pool,
  // pipeline_multi.cu:276-277, 342-351).  PSOUP_OVERSUBSCRIBE=1 keeps -t
  // workers even beyond the visible devices, worker d on device d % ndev:
  // the multi-device feeder / queue / fold-distribution paths then run (and
  // are tested) on a one-GPU box.
  const char* ovs = std::getenv("PSOUP_OVERSUBSCRIBE");
  const bool oversub = ovs && std::atoi(ovs) != 0;
  const int ngpu = std::max(1, oversub ? args.max_num_threads : std::min(ndev_avail, args.max_num_threads));
  auto hip_dev = [ndev_avail](int d) { return d % ndev_avail; };
  for (int i = 0; i < ngpu; ++i) res.devices.push_back(hip_dev(i));
  // device start-up (code objects, memory state) counted in "total" only, as
  // the reference's context creation is: the stage timers hold stage work
  {
    double init_s = 0;
    for (int i = 0; i < ngpu && i < ndev_avail; ++i) {
      PSOUP_HIP_CHECK(hipSetDevice(hip_dev(i)));
      init_s = std::max(init_s, warm_device());
    }
    res.performance["device_init_s"] = init_s;
    const char* dl = std::getenv("HIP_ENABLE_DEFERRED_LOADING");
    res.performance["code_objects_deferred"] = dl && std::atoi(dl) == 0 ? 0 : 1;
  }
  mark("device_init");
  log_verbose("Using " + std::to_string(ngpu) + " GPU(s); " + std::to_string(setup.dm_list.size()) + " DM trials; fft " +
              std::to_string(setup.fft_size));

  DedispGeometry geom = DedispGeometry::make(fb.header(), fb.nsamps(), setup.dm_list, setup.killmask);
  RunIdentity ckid;
  if (!args.checkpoint_dir.empty()) {
    ckid = make_run_identity(args, fb.header());
    prepare_checkpoint_dir(args.checkpoint_dir, ckid);
  }

  Shared sh;
  sh.args = &args;
  sh.setup = &setup;
  sh.fb = &fb;
  sh.ndm = static_cast<int>(setup.dm_list.size());
  // DMs per chunk: 32, or 64 for lists of at least 8 x 64 DMs per GPU (an
  // engine's chunk ends with a wait for its last batch and the peaks' host
  // processing before the next chunk is issued: fewer, larger chunks leave
  // the GPU idle less often -- as the Python driver's static blocks); the
  // PSOUP_CHUNK_DMS environment variable overrides
  int cmax = sh.ndm / ngpu >= 8 * 64 ? 64 : 32;
  if (const char* e = std::getenv("PSOUP_CHUNK_DMS")) cmax = std::max(1, std::atoi(e));
  sh.chunk = std::max(1, std::min(cmax, sh.ndm / (4 * ngpu) + 1));
  sh.dedisp_s.assign(static_cast<size_t>(ngpu), 0.0);
  sh.dev_stats.assign(static_cast<size_t>(ngpu), {});
  sh.search_s.assign(static_cast<size_t>(ngpu), 0.0);
  ProgressBar progress("Searching DM trials");
  if (args.progress_bar) {
    sh.progress = &progress;
    progress.start();
  }

  // Per-device resident state is kept for the folding stage.
  struct DevState {
    std::unique_ptr<Stream> stream;
    std::unique_ptr<DeviceFilterbank> dfb;
    std::unique_ptr<Dedisperser> dd;
    std::vector<std::unique_ptr<Stream>> estreams;       // engines 1.. (engine 0 uses `stream`)
    std::vector<std::unique_ptr<SearchEngine>> engines;  // built with the resident data, outside the search timer
    std::unique_ptr<FoldEngine> fe;                       // --npdmp > 0: buffers allocated up front
  };
  std::vector<DevState> devs(static_cast<size_t>(ngpu));

  // Search engines per GPU: each has its own stream, dedispersion side stream
  // and host thread, and pulls DM chunks from the shared queue, so one
  // engine's small per-DM kernels and host distillation overlap another's.
  int neng = args.engines_per_gpu;
  if (const char* e = std::getenv("PSOUP_ENGINES")) neng = std::max(neng, std::atoi(e));
  if (neng <= 0) {
    // measured on the 2026-DM config 4 (13 trials per DM): 1 engine 0.52 s,
    // 3 engines 0.56 s of search here (the Python driver gains from 3)
    neng = 1;
  }
  res.performance["engines_per_gpu"] = neng;
  setup.search.engines_per_device = neng;  // the auto batch budget is shared among them
  // block pipeline (ops.issue below): two halves of prepared slots per engine
  const char* pipe_env = std::getenv("PSOUP_BLOCK_PIPELINE");
  const bool pipelined = pipe_env == nullptr || std::atoi(pipe_env) != 0;
  res.performance["block_pipeline"] = pipelined ? 1 : 0;

  // phase 1: resident filterbank per device: one host upload to the first
  // device and a chunk-pipelined device-to-device fan-out to the others
  // (load_filterbank_fanout) -- not one host upload per device -- then each
  // device's tables and engines in parallel.  "reading" stays the file read
  // alone (pipeline_multi.cu:287-289); the setup is charged to the stage it
  // serves, as the reference's timers do (its dedispersion timer covers the
  // H2D copy and plan work, its searching timer the worker allocations and
  // FFT plans): upload + dedispersion tables -> "dedispersion", engines ->
  // "searching", fold buffers -> "folding" (per-part times in performance).
  double setup_dd = 0, setup_eng = 0, setup_fold = 0, setup_load = 0;
  Stopwatch t_setup;
  t_setup.start();
  {
    std::vector<DeviceFilterbank*> fbs;
    std::vector<int> phys;
    for (int dev = 0; dev < ngpu; ++dev) {
      PSOUP_HIP_CHECK(hipSetDevice(hip_dev(dev)));
      DevState& ds = devs[static_cast<size_t>(dev)];
      ds.stream = std::make_unique<Stream>();
      ds.dfb = std::make_unique<DeviceFilterbank>(geom, ds.stream->get());
      fbs.push_back(ds.dfb.get());
      phys.push_back(hip_dev(dev));
    }
    // each device's tables, engines and fold buffers are built on a thread of
    // their own while this thread uploads the filterbank (none of them reads
    // its samples)
    std::vector<std::thread> lth;
    for (int dev = 0; dev < ngpu; ++dev)
      lth.emplace_back([&, dev] {
        try {
          PSOUP_HIP_CHECK(hipSetDevice(hip_dev(dev)));
          DevState& ds = devs[static_cast<size_t>(dev)];
          Stopwatch wl;
          wl.start();
          ds.dd = std::make_unique<Dedisperser>(*ds.dfb, ds.stream->get());
          ds.dd->warm();  // plan tables now, not at the first tile that needs them
          const double t_dd = wl.get_time();
          for (int e = 0; e < neng; ++e) {
            if (e > 0) ds.estreams.push_back(std::make_unique<Stream>());
            ds.engines.push_back(std::make_unique<SearchEngine>(
                setup.search, e > 0 ? ds.estreams.back()->get() : ds.stream->get()));
            ds.engines.back()->reserve(ds.engines.back()->max_prepare(), 0, pipelined);
          }
          const double t_eng = wl.get_time();
          if (args.npdmp > 0 && prev_power_of_two(geom.out_nsamps) >= 1024) {
            ds.fe = std::make_unique<FoldEngine>(prev_power_of_two(geom.out_nsamps), static_cast<float>(geom.tsamp),
                                                 ds.stream->get());
            ds.fe->reserve(args.npdmp);
          }
          wl.stop();
          // host-side times: building the tables and enqueueing their
          // uploads on ds.stream (the device work is not waited for here; the
          // stream is synchronised once, after the filterbank fan-out)
          std::lock_guard<std::mutex> lk(sh.mu);
          auto& st = sh.dev_stats[static_cast<size_t>(dev)];
          st["setup_host_s"] = wl.get_time();
          st["setup_dedisp_host_s"] = t_dd;
          st["setup_engines_host_s"] = t_eng - t_dd;
          st["setup_fold_host_s"] = wl.get_time() - t_eng;
          setup_dd = std::max(setup_dd, t_dd);
          setup_eng = std::max(setup_eng, t_eng - t_dd);
          setup_fold = std::max(setup_fold, wl.get_time() - t_eng);
        } catch (...) {
          std::lock_guard<std::mutex> lk(sh.mu);
          if (!sh.error) sh.error = std::current_exception();
        }
      });
    Stopwatch wf;
    wf.start();
    try {
      load_filterbank_fanout(fbs, phys, fb);
    } catch (...) {
      std::lock_guard<std::mutex> lk(sh.mu);
      if (!sh.error) sh.error = std::current_exception();
    }
    wf.stop();
    setup_load = wf.get_time();
    res.performance["filterbank_load_s"] = setup_load;
    res.performance["filterbank_devices"] = ngpu;
    for (auto& t : lth) t.join();
    for (int dev = 0; dev < ngpu; ++dev) {
      PSOUP_HIP_CHECK(hipSetDevice(hip_dev(dev)));
      PSOUP_HIP_CHECK(hipStreamSynchronize(devs[static_cast<size_t>(dev)].stream->get()));
    }
    if (sh.error) std::rethrow_exception(sh.error);
  }
  t_setup.stop();
  mark("setup");
  res.performance["setup_s"] = t_setup.get_time();
  // (host-side build + enqueue times, the slowest device's; setup_s is the
  // whole phase including the device work)
  res.performance["setup_dedisp_host_s"] = setup_dd;
  res.performance["setup_engines_host_s"] = setup_eng;
  res.performance["setup_fold_host_s"] = setup_fold;
  t_search.start();
  // PSOUP_SCHED_TRACE=<file>: the scheduler's host events as CSV (ms, thread,
  // event, chunk d0) -- where the feeder and the engines wait
  struct SchedTrace {
    std::mutex mu;
    std::vector<std::tuple<double, int, const char*, int>> ev;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    bool on = false;
    void add(int who, const char* what, int d0) {
      if (!on) return;
      const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::lock_guard<std::mutex> lk(mu);
      ev.emplace_back(t, who, what, d0);
    }
  } strace;
  const char* strace_path = std::getenv("PSOUP_SCHED_TRACE");
  strace.on = strace_path != nullptr;
  // phase 2, per device: a feeder thread dedisperses DM chunks (one ahead,
  // double-buffered, on its own stream) and publishes them; each of the
  // device's neng engine threads searches every neng-th DM row of each chunk
  // (whitened and searched as one flat trial list), so all engines work on the
  // same chunk and the feeder reuses a buffer once every engine released it.
  // The protocol itself (slots, hand-over, abort) is ChunkScheduler
  // (scheduler.hpp), which the host unit tests run under the thread sanitizer.
  struct DevSched {
    std::atomic<int> processed{0};
    std::unique_ptr<Stream> dstream;
    static_assert(kSchedSlots == 3, "one initialiser per slot below");
    std::unique_ptr<DeviceBuffer<uint8_t>> trials[kSchedSlots];
    Event ready[kSchedSlots] = {Event(true), Event(true), Event(true)},
          began[kSchedSlots] = {Event(true), Event(true), Event(true)};
    std::vector<std::unique_ptr<Event>> freed[kSchedSlots];
    bool used[kSchedSlots] = {};
    const uint8_t* rows[kSchedSlots] = {};  // the slot's dedispersed rows (row d at rows + (d - d0) * rstride)
    double dd_ms = 0.0;
    std::vector<Stopwatch> search_w;  // per engine
    // per engine: the next chunk's first rows whitened ahead (into the other
    // half of the prepared slots while this chunk's last batches run)
    struct Ahead {
      int d0 = -1;  // the chunk they belong to (-1: none)
      int first = 0;
      int half = 0;  // the half the next prepare writes
      std::exception_ptr err;  // a failure whitening ahead, reported by the next issue
    };
    std::vector<Ahead> ahead;
  };
  std::vector<std::unique_ptr<DevSched>> scheds;
  const uint64_t rstride = Dedisperser::row_stride(geom.out_nsamps);
  // Kept trials: each device dedisperses its chunks straight into a
  // DM-indexed store (row d at d * rstride) that outlives the search, so the
  // fold stage reads the rows instead of dedispersing them again (the
  // reference keeps its DispersionTrials in host memory for the folder).
  // On when folding is requested and the whole DM list fits in a quarter of
  // the free HBM of every device (PSOUP_KEEP_TRIALS=0/1 forces it).
  bool keep = args.npdmp > 0;
  {
    // every worker mapped to a physical device holds its own store
    const uint64_t need = rstride * static_cast<uint64_t>(sh.ndm);
    std::map<int, uint64_t> per_dev;
    for (int d = 0; d < ngpu; ++d) per_dev[hip_dev(d)] += need;
    for (const auto& [phys, bytes] : per_dev) {
      if (!keep) break;
      PSOUP_HIP_CHECK(hipSetDevice(phys));
      size_t free_b = 0, total_b = 0;
      PSOUP_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
      keep = bytes <= free_b / 4;
    }
    if (const char* e = std::getenv("PSOUP_KEEP_TRIALS")) keep = std::atoi(e) != 0;
  }
  std::vector<std::unique_ptr<DeviceBuffer<uint8_t>>> kept(static_cast<size_t>(ngpu));
  std::vector<int> row_owner(static_cast<size_t>(sh.ndm), -1);  // written by the feeders, disjoint chunks
  for (int d = 0; d < ngpu; ++d) {
    PSOUP_HIP_CHECK(hipSetDevice(hip_dev(d)));
    auto sc = std::make_unique<DevSched>();
    sc->dstream = std::make_unique<Stream>();
    for (int k = 0; k < kSchedSlots; ++k) {
      if (!keep) sc->trials[k] = std::make_unique<DeviceBuffer<uint8_t>>(rstride * static_cast<uint64_t>(sh.chunk));
      for (int e = 0; e < neng; ++e) sc->freed[k].push_back(std::make_unique<Event>());
    }
    if (keep) kept[static_cast<size_t>(d)] = std::make_unique<DeviceBuffer<uint8_t>>(rstride * static_cast<uint64_t>(sh.ndm));
    sc->search_w.resize(static_cast<size_t>(neng));
    sc->ahead.resize(static_cast<size_t>(neng));
    sh.dev_stats[static_cast<size_t>(d)]["kept_trials"] = keep ? 1.0 : 0.0;
    scheds.push_back(std::move(sc));
  }
  mark("scheduler_setup");
  using Pending = std::shared_ptr<SearchEngine::Pending>;
  SchedFns<Candidate, std::vector<Pending>> ops;
  using Chunk = SchedChunk<Candidate>;
  ops.bind = [&](int dev) { PSOUP_HIP_CHECK(hipSetDevice(hip_dev(dev))); };
  ops.prepare = [&](int dev, int k, Chunk& p) {
    DevSched& sc = *scheds[static_cast<size_t>(dev)];
    DevState& ds = devs[static_cast<size_t>(dev)];
    hipStream_t dst = sc.dstream->get();
    const std::string ck = args.checkpoint_dir.empty() ? std::string() : spill_path(args.checkpoint_dir, p.d0, p.d1);
    const SpillStatus st = ck.empty() ? SpillStatus::Missing : load_spill(ck, ckid.key, p.items);
    p.resumed = st == SpillStatus::Loaded;
    if (p.resumed) {
      log_verbose("resumed DMs [" + std::to_string(p.d0) + "," + std::to_string(p.d1) + ") from checkpoint");
      return;
    }
    if (st != SpillStatus::Missing)
      log_info("checkpoint spill " + ck + " is " + spill_status_name(st) + "; recomputing DMs [" +
               std::to_string(p.d0) + "," + std::to_string(p.d1) + ")");
    p.items.clear();
    strace.add(-1 - dev, "prep0", p.d0);
    uint8_t* rows = keep ? kept[static_cast<size_t>(dev)]->data() + static_cast<uint64_t>(p.d0) * rstride
                         : sc.trials[k]->data();
    if (sc.used[k] && !keep)
      for (auto& ev : sc.freed[k]) PSOUP_HIP_CHECK(hipStreamWaitEvent(dst, ev->get(), 0));
    sc.began[k].record(dst);
    ds.dd->run(p.d0, p.d1, rows, rstride, setup.dedisp_kernel, dst);
    sc.ready[k].record(dst);
    sc.used[k] = true;
    sc.rows[k] = rows;
    strace.add(-1 - dev, "prep1", p.d0);
    if (keep)
      for (int d = p.d0; d < p.d1; ++d) row_owner[static_cast<size_t>(d)] = dev;
  };
  // A chunk's searches are issued (search_prepared_many_async) and the
  // previous chunk is collected only after them, so its acceleration
  // distillation on the engine's host workers overlaps this chunk's GPU work
  // (the Python driver's RankSearcher does the same).  Block pipeline: the
  // last group of a chunk is issued in two halves (search_launch /
  // search_finish) with the next chunk's first rows -- when the feeder has
  // published it -- whitened in between into the other half of the prepared
  // slots, so that whitening runs behind this chunk's first batches instead
  // of after its last peaks were processed (Python: RankSearcher.search_iter's
  // prep; PSOUP_BLOCK_PIPELINE=0 turns it off in both).
  ops.issue = [&](int dev, int slot, int k, const Chunk& p, int kn,
                  const std::function<const Chunk*()>& peek_next) {
    DevSched& sc = *scheds[static_cast<size_t>(dev)];
    DevSched::Ahead& ah = sc.ahead[static_cast<size_t>(slot)];
    if (ah.err) {  // whitening this chunk ahead failed (the previous chunk was finished first)
      std::exception_ptr e = ah.err;
      ah.err = nullptr;
      std::rethrow_exception(e);
    }
    SearchEngine& engine = *devs[static_cast<size_t>(dev)].engines[static_cast<size_t>(slot)];
    hipStream_t st = engine.stream();
    Stopwatch& ws = sc.search_w[static_cast<size_t>(slot)];
    const int mp = engine.max_prepare();
    const int who = dev * 64 + slot;
    strace.add(who, "issue0", p.d0);
    auto rows_of = [&](const Chunk& c) {
      std::vector<int> r;
      for (int d = c.d0 + slot; d < c.d1; d += neng) r.push_back(d);
      return r;
    };
    // whiten rows rr[r0, r0 + cnt) of chunk c (slot kk) into the next half
    auto whiten = [&](int kk, const Chunk& c, const std::vector<int>& rr, size_t r0, int cnt) {
      const int before = sc.processed.fetch_add(cnt);
      if (args.fault_after_dms >= 0 && before + cnt > args.fault_after_dms)
        PSOUP_THROW("fault injection: device " << dev << " aborting after " << before << " DM trials");
      const int first = ah.half * mp;
      engine.prepare(sc.rows[kk] + static_cast<uint64_t>(rr[r0] - c.d0) * rstride,
                     static_cast<uint64_t>(neng) * rstride, geom.out_nsamps, cnt, first);
      if (pipelined) ah.half ^= 1;  // (else every group is whitened into the first half)
      return first;
    };
    std::vector<Pending> pend;
    PSOUP_HIP_CHECK(hipStreamWaitEvent(st, sc.ready[k].get(), 0));
    ws.start();
    const std::vector<int> rows = rows_of(p);
    for (size_t r0 = 0; r0 < rows.size(); r0 += static_cast<size_t>(mp)) {
      const int cnt = static_cast<int>(std::min(rows.size() - r0, static_cast<size_t>(mp)));
      int first;
      if (r0 == 0 && ah.d0 == p.d0) {
        first = ah.first;  // whitened ahead, during the previous chunk
      } else {
        first = whiten(k, p, rows, r0, cnt);
      }
      ah.d0 = -1;
      std::vector<SearchEngine::Job> jobs;
      for (int i = 0; i < cnt; ++i) {
        const int d = rows[r0 + static_cast<size_t>(i)];
        const float dm = setup.dm_list[static_cast<size_t>(d)];
        jobs.push_back(SearchEngine::Job{first + i, dm, d, setup.accel_plan.generate(dm)});
        log_verbose("Searching " + std::to_string(jobs.back().accs.size()) + " acceleration trials for DM " +
                    std::to_string(dm));
        sh.accel_trials += jobs.back().accs.size();
      }
      if (!pipelined || r0 + static_cast<size_t>(mp) < rows.size()) {
        // one flat trial list over these DMs (batches span DM boundaries)
        pend.push_back(engine.search_prepared_many_async(jobs));
        continue;
      }
      strace.add(who, "launch0", p.d0);
      auto h = engine.search_launch(jobs);
      try {
        // (waits for the feeder to publish it: this chunk's first batches
        // are already queued on the GPU)
        strace.add(who, "peek0", p.d0);
        const Chunk* next = peek_next();
        strace.add(who, "peek1", next != nullptr ? next->d0 : -1);
        const std::vector<int> nrows = next != nullptr ? rows_of(*next) : std::vector<int>();
        if (!nrows.empty()) {
          PSOUP_HIP_CHECK(hipStreamWaitEvent(st, sc.ready[kn].get(), 0));
          ah.first = whiten(kn, *next, nrows, 0, static_cast<int>(std::min(nrows.size(), static_cast<size_t>(mp))));
          ah.d0 = next->d0;
          strace.add(who, "ahead1", next->d0);
        }
      } catch (...) {
        // this chunk is still finished (and, once collected, checkpointed)
        // before the failure is reported, by the next chunk's issue
        ah.err = std::current_exception();
        ah.d0 = -1;
      }
      engine.search_finish(h);
      strace.add(who, "finish1", p.d0);
      pend.push_back(h);
    }
    ws.stop();
    sc.freed[k][static_cast<size_t>(slot)]->record(st);
    return pend;
  };
  ops.collect = [&](int dev, int slot, std::vector<Pending>& pend, std::vector<Candidate>& out) {
    DevSched& sc = *scheds[static_cast<size_t>(dev)];
    SearchEngine& engine = *devs[static_cast<size_t>(dev)].engines[static_cast<size_t>(slot)];
    Stopwatch& ws = sc.search_w[static_cast<size_t>(slot)];
    ws.start();
    strace.add(dev * 64 + slot, "coll0", -1);
    for (auto& h : pend)
      for (auto& c : engine.collect(h))
        for (auto& x : c) out.push_back(std::move(x));
    strace.add(dev * 64 + slot, "coll1", -1);
    ws.stop();
  };
  ops.handover = [&](int dev, int k, Chunk& p) {
    // every engine is done with this chunk: checkpoint and hand over
    DevSched& sc = *scheds[static_cast<size_t>(dev)];
    if (!p.resumed) {
      float ms = 0.f;
      PSOUP_HIP_CHECK(hipEventElapsedTime(&ms, sc.began[k].get(), sc.ready[k].get()));
      sc.dd_ms += ms;
      stable_sort_by_dm_idx(p.items);
      if (!args.checkpoint_dir.empty()) save_spill(spill_path(args.checkpoint_dir, p.d0, p.d1), ckid.key, p.items);
    }
    {
      std::lock_guard<std::mutex> lk(sh.mu);
      // moved, not copied (the chunk's list is cleared after the hand-over):
      // a copy duplicated every association tree under the lock
      const size_t need = sh.cands.size() + p.items.size();
      if (need > sh.cands.capacity()) sh.cands.reserve(std::max(need, 2 * sh.cands.capacity()));
      for (auto& x : p.items) sh.cands.push_back(std::move(x));
    }
    strace.add(-1 - dev, "hand1", p.d0);
    const int done = sh.done_dms.fetch_add(p.d1 - p.d0) + (p.d1 - p.d0);
    if (sh.progress) sh.progress->set(static_cast<double>(done) / sh.ndm);
  };
  ops.engine_exit = [&](int dev, int slot) {
    DevSched& sc = *scheds[static_cast<size_t>(dev)];
    SearchEngine& engine = *devs[static_cast<size_t>(dev)].engines[static_cast<size_t>(slot)];
    PSOUP_HIP_CHECK(hipStreamSynchronize(engine.stream()));
    const double wt = sc.search_w[static_cast<size_t>(slot)].get_time();
    const SearchCounters& c = engine.counters();
    std::lock_guard<std::mutex> lk(sh.mu);
    sh.search_s[static_cast<size_t>(dev)] += wt;
    auto& st_map = sh.dev_stats[static_cast<size_t>(dev)];
    st_map["search_s"] += wt;  // summed over the device's engines
    st_map["dm_trials"] += static_cast<double>(c.dm_trials);
    st_map["accel_trials"] += static_cast<double>(c.accel_trials);
    st_map["peaks"] += static_cast<double>(c.peaks);
    st_map["peak_overflows"] += static_cast<double>(c.overflows);
    st_map["accel_loop_s"] += c.accel_s;
    st_map["host_distill_s"] += c.host_s;
    st_map["trials_distilled_on_gpu"] += static_cast<double>(c.gpu_distilled);
    st_map["trials_distilled_on_host"] += static_cast<double>(c.host_distilled);
    st_map["accel_distill_s"] += c.accd_s;
    st_map["fft_mode"] = engine.fft_mode();
    st_map["accel_batch"] = engine.batch_size();
    st_map["sub_batch"] = engine.sub_batch();
  };
  {
    ChunkScheduler<decltype(ops)> sched(ops, ngpu, neng, sh.ndm, sh.chunk);
    try {
      sched.run();
    } catch (...) {
      sh.error = std::current_exception();
    }
  }
  if (strace.on) {
    std::ofstream f(strace_path);
    f << "# t0_ns " << std::chrono::duration_cast<std::chrono::nanoseconds>(strace.t0.time_since_epoch()).count()
      << " (steady_clock)\nms,thread,event,d0\n";
    for (const auto& [t, who, what, d0] : strace.ev) f << t << ',' << who << ',' << what << ',' << d0 << '\n';
  }
  for (int d = 0; d < ngpu; ++d) {
    PSOUP_HIP_CHECK(hipSetDevice(hip_dev(d)));
    scheds[static_cast<size_t>(d)]->dstream->sync();
    const double dd = scheds[static_cast<size_t>(d)]->dd_ms * 1e-3;  // GPU time of the (overlapped) kernels
    sh.dedisp_s[static_cast<size_t>(d)] = dd;
    sh.dev_stats[static_cast<size_t>(d)]["dedispersion_s"] = dd;
  }
  t_search.stop();
  mark("search");
  if (args.progress_bar) progress.stop();
  if (sh.error) std::rethrow_exception(sh.error);

  // Concatenation order of the reference depends on thread timing; sort by
  // DM index first so the global distillation is deterministic.
  Stopwatch t_gds;
  t_gds.start();
  stable_sort_by_dm_idx(sh.cands);
  CandidateList cands = global_distill_and_score(std::move(sh.cands), args, setup);
  t_gds.stop();
  mark("global_distill");
  res.performance["global_distill_s"] = t_gds.get_time();

  // ---- folding (distributed over the devices by DM)
  t_fold.start();
  if (args.npdmp > 0 && !cands.empty()) {
    auto groups = select_fold_candidates(cands, args.npdmp);
    const uint64_t fold_n = prev_power_of_two(geom.out_nsamps);
    std::vector<std::pair<int, std::vector<int>>> glist(groups.begin(), groups.end());
    std::vector<std::thread> fth;
    std::exception_ptr ferr;
    std::mutex fmu;
    for (int dev = 0; dev < ngpu; ++dev) {
      fth.emplace_back([&, dev] {
        try {
          PSOUP_HIP_CHECK(hipSetDevice(hip_dev(dev)));
          DevState& ds = devs[static_cast<size_t>(dev)];
          hipStream_t st = ds.stream->get();
          if (!ds.fe) ds.fe = std::make_unique<FoldEngine>(fold_n, static_cast<float>(geom.tsamp), st);
          FoldEngine& fe = *ds.fe;
          const uint64_t rstride = Dedisperser::row_stride(geom.out_nsamps);
          // this worker's DM groups, batched: every DM of a batch dedispersed
          // into one buffer (no host waits), then whitened and folded together
          // the device holding a DM's kept row folds it; DMs nobody kept
          // (resumed from a checkpoint, or keep off) go round-robin
          std::vector<size_t> mine;
          size_t nrest = 0;
          for (size_t g = 0; g < glist.size(); ++g) {
            const int own = row_owner[static_cast<size_t>(glist[g].first)];
            if (own >= 0) {
              if (own == dev) mine.push_back(g);
            } else if (nrest++ % static_cast<size_t>(ngpu) == static_cast<size_t>(dev)) {
              mine.push_back(g);
            }
          }
          const int B = fe.max_batch();
          DeviceBuffer<uint8_t> trials;  // dedispersion target of batches with rows nobody kept
          for (size_t b0 = 0; b0 < mine.size(); b0 += static_cast<size_t>(B)) {
            const size_t cnt = std::min<size_t>(static_cast<size_t>(B), mine.size() - b0);
            std::vector<std::vector<double>> periods(cnt);
            std::vector<std::vector<float>> accs(cnt);
            std::vector<int> dms(cnt);
            for (size_t t = 0; t < cnt; ++t) dms[t] = glist[mine[b0 + t]].first;
            bool all_kept = true;
            for (size_t t = 0; t < cnt; ++t) all_kept = all_kept && row_owner[static_cast<size_t>(dms[t])] == dev;
            std::vector<const uint8_t*> kept_rows;
            if (all_kept)  // rows kept from the search: gathered by the folder, no dedispersion
              for (size_t t = 0; t < cnt; ++t)
                kept_rows.push_back(kept[static_cast<size_t>(dev)]->data() + static_cast<uint64_t>(dms[t]) * rstride);
            else {
              trials.resize(rstride * static_cast<uint64_t>(B));
              ds.dd->run_list(dms, trials.data(), rstride, st);  // one launch for the batch's DMs
            }
            for (size_t t = 0; t < cnt; ++t) {
              const auto& grp = glist[mine[b0 + t]];
              for (int ci : grp.second) {
                periods[t].push_back(static_cast<double>(static_cast<float>(1.0 / cands[ci].freq)));
                accs[t].push_back(cands[ci].acc);
              }
            }
            auto fr = all_kept ? fe.fold_rows(kept_rows, geom.out_nsamps, periods, accs)
                               : fe.fold_trials(trials.data(), rstride, geom.out_nsamps, static_cast<int>(cnt), periods,
                                                accs);
            for (size_t t = 0; t < cnt; ++t) {
              const auto& grp = glist[mine[b0 + t]];
              for (size_t k = 0; k < fr[t].size(); ++k) {
                Candidate& c = cands[static_cast<size_t>(grp.second[k])];
                c.folded_snr = fr[t][k].folded_snr;
                c.set_fold(fr[t][k].fold.data(), FoldEngine::kNbins, FoldEngine::kNints);
                c.opt_period = fr[t][k].opt_period;
              }
            }
          }
        } catch (...) {
          std::lock_guard<std::mutex> lk(fmu);
          if (!ferr) ferr = std::current_exception();
        }
      });
    }
    for (auto& t : fth) t.join();
    if (ferr) std::rethrow_exception(ferr);
    sort_by_folded_snr(cands);
  }
  t_fold.stop();
  mark("fold");

  const size_t new_size = std::min(static_cast<size_t>(std::max(args.limit, 0)), cands.size());
  cands.resize(new_size);
  res.candidates = std::move(cands);

  double dmax = 0, smax = 0;
  for (int d = 0; d < ngpu; ++d) {
    dmax = std::max(dmax, sh.dedisp_s[static_cast<size_t>(d)]);
    smax = std::max(smax, sh.search_s[static_cast<size_t>(d)]);
  }
  t_total.stop();
  res.timers["reading"] = t_read.get_time();
  res.timers["dedispersion"] = dmax + setup_load + setup_dd;
  res.timers["searching"] = t_search.get_time() + setup_eng;
  res.timers["folding"] = t_fold.get_time() + setup_fold;
  res.timers["total"] = t_total.get_time();
  const double trials = static_cast<double>(sh.accel_trials.load());
  res.performance["dm_accel_trials"] = trials;
  res.performance["dm_accel_trials_per_sec"] = t_search.get_time() > 0 ? trials / t_search.get_time() : 0.0;
  res.performance["search_kernel_seconds_max_device"] = smax;
  res.performance["search_loop_s"] = t_search.get_time();
  res.performance["fold_s"] = t_fold.get_time();
  res.device_stats = sh.dev_stats;
  return res;
}

namespace {
std::string json_num(double v) {
  if (!std::isfinite(v)) return "null";
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.17g", v);
  return buf;
}
std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char ch : s) {
    if (ch == '"' || ch == '\\') o += '\\';
    if (static_cast<unsigned char>(ch) < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", ch);
      o += b;
      continue;
    }
    o += ch;
  }
  return o + "\"";
}
std::string json_map(const std::map<std::string, double>& m) {
  std::string o = "{";
  bool first = true;
  for (const auto& kv : m) {
    o += (first ? "" : ", ") + json_str(kv.first) + ": " + json_num(kv.second);
    first = false;
  }
  return o + "}";
}
}  // namespace

std::string trace_json(const CmdLineOptions& args, const PipelineResult& res,
                       const std::map<std::string, double>& extra_performance) {
  std::string o = "{\n";
  o += "  \"input\": " + json_str(args.infilename) + ",\n";
  o += "  \"config\": {\"fft_size\": " + json_num(static_cast<double>(res.setup.search.fft_size)) +
       ", \"nharmonics\": " + json_num(args.nharmonics) + ", \"ndm\": " +
       json_num(static_cast<double>(res.setup.dm_list.size())) + ", \"acc_start\": " + json_num(args.acc_start) +
       ", \"acc_end\": " + json_num(args.acc_end) + ", \"accel_convention\": " + json_str(args.accel_convention) +
       ", \"dedisp_kernel\": " + json_str(args.dedisp_kernel) + ", \"fft_mode\": " + json_num(args.fft_mode) +
       "},\n";
  o += "  \"timers_s\": " + json_map(res.timers) + ",\n";
  std::map<std::string, double> perf = res.performance;
  for (const auto& kv : extra_performance) perf[kv.first] = kv.second;
  o += "  \"performance\": " + json_map(perf) + ",\n";
  o += "  \"devices\": [";
  for (size_t d = 0; d < res.device_stats.size(); ++d) {
    auto m = res.device_stats[d];
    m["device"] = d < res.devices.size() ? res.devices[d] : static_cast<double>(d);
    o += (d ? ",\n    " : "\n    ") + json_map(m);
  }
  o += "\n  ],\n";
  o += "  \"candidates\": " + json_num(static_cast<double>(res.candidates.size())) + "\n}\n";
  return o;
}

void write_outputs(const CmdLineOptions& args, const PipelineResult& res) {
  Stopwatch tw;
  tw.start();
  CandidateFileWriter cf(args.outdir);
  cf.write_binary(res.candidates, "candidates.peasoup");
  OverviewWriter ow;
  ow.add_misc_info();
  ow.add_header(args.infilename);
  ow.add_search_parameters(args);
  ow.add_dm_list(res.setup.dm_list);
  ow.add_acc_list(res.setup.accel_plan.generate(0.0f));
  ow.add_gpu_info(res.devices);
  ow.add_candidates(res.candidates, cf.byte_mapping);
  ow.add_timing_info(res.timers);
  ow.add_performance(res.performance);
  ow.to_file(args.outdir + "/overview.xml");
  tw.stop();
  if (!args.trace_json.empty()) {
    std::ofstream f(args.trace_json);
    if (!f) PSOUP_THROW("cannot write trace file " << args.trace_json);
    f << trace_json(args, res, {{"write_outputs_s", tw.get_time()}});
  }
}

}  // namespace psoup
