// Per-device DM-chunk scheduler of the native pipeline (run_pipeline): the
// host-side concurrency protocol, separated from its GPU work so that it can
// run (and be checked by the thread sanitizer) with fake devices in the host
// unit tests.
//
// The reference's equivalent is the mutex-protected DMDispenser queue that
// every Worker thread pulls single DM trials from (src/pipeline_multi.cu:
// 33-81, 209-243).  Here, per device:
//   * one feeder thread pulls DM chunks [d0, d1) from the queue shared by all
//     devices (one atomic add), prepares each into one of kSchedSlots slots
//     (the dedispersion of the next chunk overlaps the search of this one; or
//     a checkpoint spill is loaded: a "resumed" chunk) and publishes it;
//   * neng engine threads take every published chunk in order, issue their
//     share of its searches (Ops::issue) and only then finalize the previous
//     chunk (Ops::collect), so each chunk's host tail overlaps the next
//     chunk's GPU work;
//   * the last engine to finalize a chunk hands it over (Ops::handover) with
//     the slot still held (pending = 1), then frees the slot for the feeder.
// A failure anywhere (an exception from any Ops call) aborts every thread of
// every device; run() rethrows the first error once all have exited.
//
// Ops provides (Chunk = SchedChunk<Item>):
//   using Item = ...;   // one result (a candidate)
//   using Token = ...;  // what issue() hands to collect() (default-constructible)
//   void bind(int dev);                         // first call of every scheduler thread (device binding)
//   void prepare(int dev, int slot, Chunk& c);  // fills c.resumed (and c.items when resumed)
//   Token issue(int dev, int engine, int slot, const Chunk& c,   // not called for resumed chunks
//               int next_slot, const std::function<const Chunk*()>& next);
//       next(): waits until the feeder has published the following chunk
//       and returns it (nullptr: there is none, it is resumed, or the run
//       aborts).  Its slot stays valid until this engine finalizes it, so
//       issue() may start on it (whiten it ahead).  The wait cannot deadlock:
//       that chunk needs the slot of chunk g - 2, which every engine has
//       finalized once it is issuing chunk g - 1 or later, so the slowest
//       engine's wait is always satisfiable.
//   void collect(int dev, int engine, Token& t, std::vector<Item>& out);
//   void handover(int dev, int slot, Chunk& c);  // c.items: every engine's results
//   void engine_exit(int dev, int engine);       // an engine thread's last call (not after a failure)
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace psoup {

// Chunk slots per device: with three, the feeder prepares chunk k + 1 (its
// dedispersion on the GPU beside chunk k's search) while chunk k - 1 is still
// being collected and handed over; with two it had to wait for that hand-over,
// which comes after chunk k's searches were issued, and the next chunk's
// dedispersion then ran alone on the GPU.
constexpr int kSchedSlots = 3;

template <class Item>
struct SchedChunk {
  int d0 = 0, d1 = 0;
  bool resumed = false;
  int pending = 0;  // engines that have not finalized it (0: the slot is free)
  std::vector<Item> items;
};

// Ops from callables (the pipeline's GPU work, the unit tests' fake devices).
template <class Item_, class Token_>
struct SchedFns {
  using Item = Item_;
  using Token = Token_;
  using Chunk = SchedChunk<Item>;
  std::function<void(int)> bind = [](int) {};
  std::function<void(int, int, Chunk&)> prepare;
  std::function<Token(int, int, int, const Chunk&, int, const std::function<const Chunk*()>&)> issue;
  std::function<void(int, int, Token&, std::vector<Item>&)> collect;
  std::function<void(int, int, Chunk&)> handover;
  std::function<void(int, int)> engine_exit = [](int, int) {};
};

template <class Ops>
class ChunkScheduler {
 public:
  using Item = typename Ops::Item;
  using Token = typename Ops::Token;
  using Chunk = SchedChunk<Item>;

  ChunkScheduler(Ops& ops, int ndev, int neng, int ndm, int chunk)
      : ops_(ops), ndev_(ndev), neng_(neng), ndm_(ndm), chunk_(std::max(1, chunk)) {
    for (int d = 0; d < ndev_; ++d) devs_.push_back(std::make_unique<Dev>());
  }

  // Test hook: finalize appends results to the shared chunk without its lock
  // (a deliberate data race, to check that the thread sanitizer sees one).
  void inject_race_for_test(bool on) { racy_ = on; }

  void run() {
    std::vector<std::thread> th;
    for (int d = 0; d < ndev_; ++d) {
      th.emplace_back([this, d] { feeder(d); });
      for (int e = 0; e < neng_; ++e) th.emplace_back([this, d, e] { worker(d, e); });
    }
    for (auto& t : th) t.join();
    if (err_) std::rethrow_exception(err_);
  }

  bool aborted() const { return abort_.load(); }

 private:
  struct Dev {
    std::mutex mu;
    std::condition_variable cv;
    Chunk pub[kSchedSlots];
    long published = 0;
    bool done = false;
  };

  void fail() {
    {
      std::lock_guard<std::mutex> lk(err_mu_);
      if (!err_) err_ = std::current_exception();
    }
    abort_.store(true);
    for (auto& dv : devs_) {
      std::lock_guard<std::mutex> lk(dv->mu);
      dv->cv.notify_all();
    }
  }

  void feeder(int dev) {
    Dev& dv = *devs_[static_cast<size_t>(dev)];
    try {
      ops_.bind(dev);
      int k = 0;
      while (!abort_.load()) {
        const int d0 = next_.fetch_add(chunk_);
        if (d0 >= ndm_) break;
        {
          std::unique_lock<std::mutex> lk(dv.mu);
          dv.cv.wait(lk, [&] { return dv.pub[k].pending == 0 || abort_.load(); });
        }
        if (abort_.load()) break;
        // the slot is free: no engine reads it until it is published below
        Chunk& c = dv.pub[k];
        c.d0 = d0;
        c.d1 = std::min(ndm_, d0 + chunk_);
        c.resumed = false;
        c.items.clear();
        ops_.prepare(dev, k, c);
        {
          std::lock_guard<std::mutex> lk(dv.mu);
          c.pending = neng_;
          dv.published++;
        }
        dv.cv.notify_all();
        k = (k + 1) % kSchedSlots;
      }
    } catch (...) {
      fail();
    }
    std::lock_guard<std::mutex> lk(dv.mu);
    dv.done = true;
    dv.cv.notify_all();
  }

  struct Issued {
    int slot = -1;
    Token token{};
  };

  void finalize(int dev, int eng, Issued& is) {
    Dev& dv = *devs_[static_cast<size_t>(dev)];
    Chunk& c = dv.pub[is.slot];
    std::vector<Item> local;
    if (!c.resumed) ops_.collect(dev, eng, is.token, local);
    bool last = false;
    if (racy_) {
      for (auto& x : local) c.items.push_back(std::move(x));  // (test hook: no lock)
      std::lock_guard<std::mutex> lk(dv.mu);
      last = c.pending == 1;
      if (!last) --c.pending;
    } else {
      // the last engine keeps pending at 1 until the chunk is handed over, so
      // the feeder cannot refill this slot while c.items is read
      std::lock_guard<std::mutex> lk(dv.mu);
      for (auto& x : local) c.items.push_back(std::move(x));
      last = c.pending == 1;
      if (!last) --c.pending;
    }
    if (last) {
      ops_.handover(dev, is.slot, c);
      std::lock_guard<std::mutex> lk(dv.mu);
      c.items.clear();
      c.pending = 0;
      dv.cv.notify_all();
    }
    is = Issued();
  }

  void worker(int dev, int eng) {
    Dev& dv = *devs_[static_cast<size_t>(dev)];
    try {
      ops_.bind(dev);
      Issued prev;
      for (long g = 0;; ++g) {
        {
          std::unique_lock<std::mutex> lk(dv.mu);
          dv.cv.wait(lk, [&] { return dv.published > g || dv.done || abort_.load(); });
          if (abort_.load() || dv.published <= g) break;
        }
        Issued cur;
        cur.slot = static_cast<int>(g % kSchedSlots);
        const Chunk& c = dv.pub[cur.slot];
        if (!c.resumed) {
          // the next chunk, once the feeder has published it: its slot is
          // not refilled before this engine has finalized it
          const int ns = static_cast<int>((g + 1) % kSchedSlots);
          const std::function<const Chunk*()> nx = [&, g, ns]() -> const Chunk* {
            std::unique_lock<std::mutex> lk(dv.mu);
            dv.cv.wait(lk, [&] { return dv.published > g + 1 || dv.done || abort_.load(); });
            if (abort_.load() || dv.published <= g + 1 || dv.pub[ns].resumed) return nullptr;
            return &dv.pub[ns];
          };
          try {
            cur.token = ops_.issue(dev, eng, cur.slot, c, ns, nx);
          } catch (...) {
            // the previous chunk was issued whole: finalize it (its checkpoint
            // spill) before the failure propagates, so a resume skips it
            if (prev.slot >= 0) {
              try {
                finalize(dev, eng, prev);
              } catch (...) {  // the first failure is the one reported
              }
            }
            throw;
          }
        }
        if (prev.slot >= 0) finalize(dev, eng, prev);
        prev = std::move(cur);
      }
      if (prev.slot >= 0) {
        if (!abort_.load()) {
          finalize(dev, eng, prev);
        } else {
          // another thread failed: this engine's share of the previous chunk
          // was issued whole, so finalize it too; the chunk is handed over
          // (checkpointed) once every engine has, whichever of them fails
          try {
            finalize(dev, eng, prev);
          } catch (...) {  // the first failure is the one reported
          }
        }
      }
      if (!abort_.load()) ops_.engine_exit(dev, eng);
    } catch (...) {
      fail();
    }
  }

  Ops& ops_;
  const int ndev_, neng_, ndm_, chunk_;
  std::vector<std::unique_ptr<Dev>> devs_;
  std::atomic<int> next_{0};
  std::atomic<bool> abort_{false};
  std::mutex err_mu_;
  std::exception_ptr err_;
  bool racy_ = false;
};

}  // namespace psoup
