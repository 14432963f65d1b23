// Native host-side unit tests for the C++ core (no GPU needed).  Built as
// `bin/psoup_unit_tests`; the sanitizer build (`python -m peasoup_amd._build
// --sanitize address|undefined|thread`) compiles these sources and the host
// components they exercise with -fsanitize=..., since GPU
// ASan is not available on the MI355X pool.
//
// usage: psoup_unit_tests [repo_root]   (repo_root locates the tutorial .fil)
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <map>
#include <mutex>
#include <random>
#include <cstring>
#include <array>
#include <functional>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "psoup/candidates.hpp"
#include "psoup/checkpoint.hpp"
#include "psoup/cli.hpp"
#include "psoup/common.hpp"
#include "psoup/output.hpp"
#include "psoup/plan.hpp"
#include "psoup/scheduler.hpp"
#include "psoup/sigproc.hpp"

using namespace psoup;

namespace {

int g_fail = 0, g_pass = 0;
std::string g_root = ".";

#define CHECK(cond)                                                                      \
  do {                                                                                   \
    if (!(cond)) {                                                                       \
      std::cerr << "  FAILED " << __FILE__ << ":" << __LINE__ << ": " #cond << "\n";     \
      ++g_fail;                                                                          \
      return;                                                                            \
    }                                                                                    \
  } while (0)

struct Case {
  const char* name;
  std::function<void()> fn;
};

void t_prev_power_of_two() {
  CHECK(prev_power_of_two(187520) == 131072);
  CHECK(prev_power_of_two(1u << 23) == (1u << 22));  // strictly less (utils.hpp:12-18)
  CHECK(prev_power_of_two(1000) == 512);
}

void t_accel_plan_conventions() {
  AccelPlan legacy(-5, 5, 1.1f, 64.f, 131072, 0.00032f, 1367.5f, -1.09f);
  auto l = legacy.generate(0.f);
  CHECK(l.size() == 3 && l[0] == 0.f && l[1] == -5.f && l[2] == 5.f);
  AccelPlan cur(-5, 5, 1.1f, 64.f, 131072, 0.00032f, 1367.5f, -1.09f, AccelConvention::Reference);
  CHECK(cur.generate(0.f).size() == 44);
  AccelPlan big(-500, 500, 1.1f, 64.f, 1u << 23, 64e-6f, 1400.f, -0.39f);
  const size_t nb = big.generate(0.f).size();
  CHECK(nb >= 680 && nb <= 690);
  CHECK(AccelPlan(0, 0, 1.1f, 64.f, 1024, 1e-4f, 1400.f, -1.f).generate(3.f) == std::vector<float>{0.f});
}

void t_dm_list_tutorial() {
  SigprocHeader h = read_header_file(g_root + "/tests/data/tutorial.fil");
  auto dms = generate_dm_list(0.f, 250.f, h.tsamp, 64.0, h.fch1, h.foff, h.nchans, 1.1f);
  CHECK(dms.size() == 59);  // golden overview.xml dedispersion_trials
  CHECK(dms.front() == 0.f);
  for (size_t i = 1; i < dms.size(); ++i) CHECK(dms[i] > dms[i - 1]);
  auto delays = generate_delay_table(h.nchans, h.tsamp, h.fch1, h.foff);
  CHECK(compute_max_delay(dms, delays) == 140);
}

void t_cli_parse() {
  CmdLineOptions a;
  bool exit_now = false;
  std::vector<std::string> argv = {"peasoup", "-i", "x.fil", "--dm_end", "250", "-n", "3", "--acc_start=-5",
                                   "--acc_end", "5", "-vp", "--fft_mode", "1", "--npdmp", "10"};
  CHECK(parse_cmdline(a, argv, &exit_now));
  CHECK(!exit_now && a.infilename == "x.fil" && a.dm_end == 250.f && a.nharmonics == 3);
  CHECK(a.acc_start == -5.f && a.acc_end == 5.f && a.verbose && a.progress_bar && a.fft_mode == 1 && a.npdmp == 10);
  CmdLineOptions b;
  CHECK(!parse_cmdline(b, std::vector<std::string>{"peasoup", "--dm_end", "1"}, &exit_now));  // -i required
  CHECK(!parse_cmdline(b, std::vector<std::string>{"peasoup", "-i", "f", "--bogus", "1"}, &exit_now));
}

void t_xml_format() {
  CHECK(xml::fmt(0.1) == "0.1");
  CHECK(xml::fmt(1.0 / 3.0) == "0.333333333333333");
  xml::Element e("cand");
  e.add_attribute("id", 3);
  e.add_attribute("name", std::string("a<b&c"));
  e.append(xml::Element("period", 0.25));
  const std::string s = e.to_string();
  CHECK(s.find("id='3'") != std::string::npos);
  CHECK(s.find("a&lt;b&amp;c") != std::string::npos);
  CHECK(s.find("<period>0.25</period>") != std::string::npos);
}

CandidateList synth_cands() {
  CandidateList c;
  c.emplace_back(10.f, 3, 0.f, 2, 20.f, 4.0f);
  c.emplace_back(10.f, 3, 0.f, 1, 12.f, 8.0f);        // 2nd harmonic of the first
  c.emplace_back(10.f, 3, 0.f, 1, 11.f, 2.0f);        // subharmonic
  c.emplace_back(10.f, 3, 0.f, 1, 15.f, 4.7312f);     // unrelated
  c.emplace_back(12.f, 4, 5.f, 1, 9.5f, 4.00001f);    // same signal, neighbour DM
  return c;
}

void t_distillers() {
  HarmonicDistiller hd(0.0001f, 16.f, true, true);
  auto out = hd.distill(synth_cands());
  CHECK(out.size() == 2);
  CHECK(out[0].snr == 20.f && out[0].count_assoc() >= 2);
  DMDistiller dd(0.0001f, true);
  auto out2 = dd.distill(synth_cands());
  CHECK(out2.size() < 5);
  AccelerationDistiller ad(537.f, 0.0001f, true);
  CHECK(!ad.distill(synth_cands()).empty());
}

void t_serialise_roundtrip() {
  CandidateList c = synth_cands();
  c[0].append(c[1]);
  c[0].assoc[0].append(c[2]);
  auto bytes = serialize_candidates(c);
  auto back = deserialize_candidates(bytes.data(), bytes.size());
  CHECK(back.size() == c.size());
  CHECK(back[0].count_assoc() == c[0].count_assoc());
  CHECK(back[3].freq == c[3].freq && back[4].dm_idx == 4);
  bool threw = false;
  try {
    deserialize_candidates(bytes.data(), bytes.size() / 2);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

void t_sigproc_roundtrip() {
  SigprocHeader h;
  h.source_name = "unit";
  h.nchans = 16;
  h.nbits = 8;
  h.tsamp = 1e-4;
  h.fch1 = 1500;
  h.foff = -1;
  h.nsamples = 7;
  h.nifs = 1;
  h.keys_present = {"source_name", "nchans", "nbits", "tsamp", "fch1", "foff", "nsamples", "nifs"};
  std::stringstream ss;
  write_header(ss, h);
  SigprocHeader r;
  ss.seekg(0);
  CHECK(read_header(ss, r));
  CHECK(r.source_name == "unit" && r.nchans == 16 && r.nbits == 8 && r.tsamp == 1e-4 && r.fch1 == 1500 &&
        r.foff == -1 && r.nsamples == 7);
}

void t_peaks_and_bounds() {
  // identify_unique_peaks: clusters separated by < min_gap merge (peakfinder.hpp:24-55)
  const int idx[] = {100, 101, 105, 200, 260, 261};
  const float snr[] = {9.5f, 12.f, 10.f, 11.f, 9.1f, 9.2f};
  std::vector<int> oi;
  std::vector<float> os;
  identify_unique_peaks(idx, snr, 6, 30, oi, os);
  CHECK(oi.size() == 3 && oi[0] == 101 && oi[1] == 200 && oi[2] == 261);
  PeakBounds b = peak_bounds(65537, 0.0238f, 3, 0.1f, 1100.f);
  CHECK(b.start_idx > 0 && b.end_idx == 65537);
}

void t_threads_shared_readonly() {
  // The per-GPU worker threads share the AccelPlan and DM list read-only
  // (SURVEY.md §5.2); hammer that under TSan/ASan builds.
  AccelPlan plan(-500, 500, 1.1f, 64.f, 1u << 20, 64e-6f, 1400.f, -0.39f);
  std::vector<size_t> counts(8);
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      size_t n = 0;
      for (int k = 0; k < 50; ++k) n += plan.generate(static_cast<float>(k)).size();
      counts[static_cast<size_t>(t)] = n;
    });
  for (auto& x : th) x.join();
  for (size_t c : counts) CHECK(c == counts[0] && c > 0);
}

// HostPool (engine host stages): every index runs exactly once per call,
// repeated generations reuse the workers, exceptions reach the caller
// (exercised under TSan by the sanitizer build).
void t_host_pool() {
  HostPool pool(5);
  CHECK(pool.size() == 6);
  for (int rep = 0; rep < 50; ++rep) {
    const int n = 1 + (rep * 37) % 200;
    std::vector<int> hits(static_cast<size_t>(n), 0);
    pool.parallel_for(n, [&](int i) { hits[static_cast<size_t>(i)] += 1; });
    for (int h : hits) CHECK(h == 1);
  }
  bool thrown = false;
  try {
    pool.parallel_for(64, [](int i) {
      if (i == 17) throw std::runtime_error("boom");
    });
  } catch (const std::runtime_error&) {
    thrown = true;
  }
  CHECK(thrown);
  std::vector<int> again(10, 0);
  pool.parallel_for(10, [&](int i) { again[static_cast<size_t>(i)] = i; });
  for (int i = 0; i < 10; ++i) CHECK(again[static_cast<size_t>(i)] == i);
}

}  // namespace

// Checkpoint spills: keyed, integrity-checked, atomic; concurrent writers of
// different chunks (the native pipeline's engines) leave only whole files.
void t_checkpoint_spills() {
  char tmpl[] = "/tmp/psoup_ck_XXXXXX";
  char* dir = ::mkdtemp(tmpl);
  CHECK(dir != nullptr);
  const std::string d = dir;
  CmdLineOptions a;
  a.infilename = g_root + "/tests/data/tutorial.fil";
  SigprocHeader h = read_header_file(a.infilename);
  const RunIdentity id = make_run_identity(a, h);
  prepare_checkpoint_dir(d, id);
  CandidateList c = synth_cands();
  std::vector<std::thread> th;
  for (int i = 0; i < 4; ++i) th.emplace_back([&, i] { save_spill(spill_path(d, 8 * i, 8 * i + 8), id.key, c); });
  for (auto& t : th) t.join();
  for (int i = 0; i < 4; ++i) {
    CandidateList back;
    CHECK(load_spill(spill_path(d, 8 * i, 8 * i + 8), id.key, back) == SpillStatus::Loaded);
    CHECK(back.size() == c.size() && back[3].freq == c[3].freq);
    CandidateList none;
    CHECK(load_spill(spill_path(d, 8 * i, 8 * i + 8), id.key + 1, none) == SpillStatus::Mismatch && none.empty());
  }
  CandidateList none;
  CHECK(load_spill(spill_path(d, 99, 100), id.key, none) == SpillStatus::Missing);
  a.nharmonics = 3;
  CHECK(make_run_identity(a, h).key != id.key);
  bool threw = false;
  try {
    save_spill(d + "/missing_subdir/x.psoc", id.key, c);
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  for (int i = 0; i < 4; ++i) std::remove(spill_path(d, 8 * i, 8 * i + 8).c_str());
  std::remove((d + "/manifest.txt").c_str());
  ::rmdir(d.c_str());
}

// The native pipeline's chunk scheduler (scheduler.hpp, run_pipeline's
// feeder / engine threads) on fake devices: the slot a feeder fills is plain
// memory that the engines read without a lock (as the real feeder's
// dedispersion target), so a protocol that let a feeder refill a slot an
// engine still reads, or two engines write one chunk's results unlocked, is
// a data race the thread-sanitizer build reports.  Random delays vary the
// interleavings; every DM must be handed over exactly once, resumed
// (checkpointed) chunks included, and an injected fault must end every
// thread of every device.
namespace {
struct FakeRun {
  int ndev, neng, ndm, chunk;
  int fault_after = -1;  // issue() throws once this many DMs were issued
  int fault_d0 = -1;     // prepare() (the feeder) throws on the chunk starting here
  bool racy = false;
  std::mutex mu;
  std::map<int, int> handed;                // DM -> times handed over
  std::vector<std::array<int, 4>> slot_of;  // [dev * 2 + slot] = {d0, d1, fill count, -}: plain, feeder-written
  std::atomic<int> issued{0};
  std::atomic<long> seed{1};
  void nap(int max_us) {
    thread_local std::mt19937 rng(static_cast<unsigned>(seed.fetch_add(7919)));
    std::this_thread::sleep_for(std::chrono::microseconds(rng() % static_cast<unsigned>(max_us + 1)));
  }
  static bool resumed_chunk(int d0, int chunk) { return (d0 / chunk) % 5 == 3; }
  void run() {
    slot_of.assign(static_cast<size_t>(ndev) * kSchedSlots, {-1, -1, 0, 0});
    SchedFns<int, std::vector<int>> ops;
    using Chunk = SchedChunk<int>;
    ops.prepare = [&](int dev, int k, Chunk& c) {
      nap(150);
      if (c.d0 == fault_d0) throw std::runtime_error("fault injection");
      if (resumed_chunk(c.d0, chunk)) {  // a spill: results without any search
        c.resumed = true;
        for (int d = c.d0; d < c.d1; ++d) c.items.push_back(d);
        return;
      }
      auto& sl = slot_of[static_cast<size_t>(dev) * kSchedSlots + k];
      sl[0] = c.d0;  // "dedisperse" into the slot
      sl[1] = c.d1;
      sl[2]++;
    };
    ops.issue = [&](int dev, int eng, int k, const Chunk& c, int kn, const std::function<const Chunk*()>& peek) {
      const auto& sl = slot_of[static_cast<size_t>(dev) * kSchedSlots + k];
      if (sl[0] != c.d0 || sl[1] != c.d1) throw std::runtime_error("slot refilled under a reading engine");
      std::vector<int> mine;
      for (int d = c.d0 + eng; d < c.d1; d += neng) mine.push_back(d);
      if (fault_after >= 0 && issued.fetch_add(static_cast<int>(mine.size())) > fault_after)
        throw std::runtime_error("fault injection");
      nap(200);
      const Chunk* next = peek();
      if (next != nullptr) {
        // "whiten the next chunk ahead": its slot holds it, and keeps it
        // while this engine reads it
        const auto& sn = slot_of[static_cast<size_t>(dev) * kSchedSlots + kn];
        if (next->resumed || next->d0 <= c.d0 || sn[0] != next->d0 || sn[1] != next->d1)
          throw std::runtime_error("look-ahead chunk is not the published next chunk");
        nap(100);
        if (sn[0] != next->d0 || sn[1] != next->d1) throw std::runtime_error("slot refilled under a reading engine");
      }
      return mine;
    };
    ops.collect = [&](int, int, std::vector<int>& t, std::vector<int>& out) {
      nap(200);
      out = t;
    };
    ops.handover = [&](int, int, Chunk& c) {
      nap(50);
      std::lock_guard<std::mutex> lk(mu);
      for (int d : c.items) handed[d]++;
    };
    ChunkScheduler<decltype(ops)> sched(ops, ndev, neng, ndm, chunk);
    sched.inject_race_for_test(racy);
    sched.run();
  }
};
}  // namespace

void t_scheduler_protocol() {
  for (int rep = 0; rep < 6; ++rep) {
    FakeRun r{1 + rep % 3, 1 + rep % 2 + (rep == 5 ? 1 : 0), 181 + 17 * rep, 3 + rep};
    r.run();
    CHECK(static_cast<int>(r.handed.size()) == r.ndm);
    for (const auto& [d, n] : r.handed) CHECK(d >= 0 && d < r.ndm && n == 1);
  }
}

void t_scheduler_fault_ends_every_thread() {
  for (int rep = 0; rep < 4; ++rep) {
    FakeRun r{3, 2, 400, 4};
    r.fault_after = 40 + 30 * rep;
    bool threw = false;
    try {
      r.run();  // returns (every thread joined) and rethrows the fault
    } catch (const std::runtime_error& e) {
      threw = std::string(e.what()) == "fault injection";
    }
    CHECK(threw);
    for (const auto& kv : r.handed) CHECK(kv.second == 1);
    // one engine per device: the chunk issued before the failing one was
    // still handed over (its checkpoint spill exists for a resume)
    FakeRun one{1, 1, 100, 10};
    one.fault_after = 15;
    try {
      one.run();
    } catch (const std::runtime_error&) {
    }
    CHECK(one.handed.count(0) == 1 && one.handed.count(19) == 1 && one.handed.count(20) == 0);
    // three engines per device: the feeder fails preparing chunk [60, 70).
    // It could only start that chunk once slot 0's previous chunk [30, 40)
    // was handed over, i.e. after every engine had issued [40, 50): so the
    // engines, seeing the abort, must still finalize [40, 50) and it is
    // handed over once.  [50, 60) may not have been issued by every engine
    // (kSchedSlots = 3): it is handed over whole or not at all.
    for (int k = 0; k < 6; ++k) {
      FakeRun three{1, 3, 100, 10};
      three.fault_d0 = 60;
      try {
        three.run();
      } catch (const std::runtime_error&) {
      }
      for (int d = 0; d < 50; ++d) CHECK(three.handed.count(d) == 1 && three.handed[d] == 1);
      const size_t tail = three.handed.count(50);
      for (int d = 50; d < 60; ++d) CHECK(three.handed.count(d) == tail && (tail == 0 || three.handed[d] == 1));
      CHECK(three.handed.count(60) == 0);
    }
  }
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "--inject-race") {
    // (tests/test_native_unit.py: the thread-sanitizer build must report this)
    for (int rep = 0; rep < 20; ++rep) {
      FakeRun r{2, 3, 300, 6};
      r.racy = true;
      r.run();
    }
    std::cout << "race injected\n";
    return 0;
  }
  if (argc > 1) g_root = argv[1];
  std::vector<Case> cases = {
      {"prev_power_of_two", t_prev_power_of_two},
      {"accel_plan_conventions", t_accel_plan_conventions},
      {"dm_list_tutorial", t_dm_list_tutorial},
      {"cli_parse", t_cli_parse},
      {"xml_format", t_xml_format},
      {"distillers", t_distillers},
      {"serialise_roundtrip", t_serialise_roundtrip},
      {"sigproc_roundtrip", t_sigproc_roundtrip},
      {"peaks_and_bounds", t_peaks_and_bounds},
      {"threads_shared_readonly", t_threads_shared_readonly},
      {"host_pool", t_host_pool},
      {"checkpoint_spills", t_checkpoint_spills},
      {"scheduler_protocol", t_scheduler_protocol},
      {"scheduler_fault_ends_every_thread", t_scheduler_fault_ends_every_thread},
  };
  for (auto& c : cases) {
    const int before = g_fail;
    try {
      c.fn();
    } catch (const std::exception& e) {
      std::cerr << "  EXCEPTION in " << c.name << ": " << e.what() << "\n";
      ++g_fail;
    }
    if (g_fail == before) ++g_pass;
    std::cout << (g_fail == before ? "[ OK ] " : "[FAIL] ") << c.name << "\n";
  }
  std::cout << g_pass << " passed, " << g_fail << " failed\n";
  return g_fail == 0 ? 0 : 1;
}
