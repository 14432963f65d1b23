#include "psoup/engine.hpp"

#include <thread>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <charconv>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <numeric>

namespace psoup {

static constexpr double kC = 299792458.0;

DedispKernel parse_dedisp_kernel(const std::string& s) {
  if (s == "auto") return DedispKernel::Auto;
  if (s == "direct") return DedispKernel::Direct;
  if (s == "mfma") return DedispKernel::Mfma;
  if (s == "valu") return DedispKernel::Valu;
  if (s == "packed2") return DedispKernel::Packed2;
  PSOUP_THROW("unknown dedispersion kernel '" << s << "' (auto|direct|mfma|valu|packed2)");
}

// ------------------------------------------------------------ geometry ------
DedispGeometry DedispGeometry::make(const SigprocHeader& hdr, uint64_t nsamps, const std::vector<float>& dm_list,
                                    const std::vector<int>& killmask) {
  DedispGeometry g;
  g.nchans = hdr.nchans;
  g.nbits = hdr.nbits;
  g.tsamp = hdr.tsamp;
  g.fch1 = hdr.fch1;
  g.foff = hdr.foff;
  g.nsamps = nsamps;
  g.dm_list = dm_list;
  g.delays = generate_delay_table(g.nchans, g.tsamp, g.fch1, g.foff);
  g.killmask = killmask.empty() ? std::vector<int>(static_cast<size_t>(g.nchans), 1) : killmask;
  PSOUP_CHECK(static_cast<int>(g.killmask.size()) == g.nchans, "killmask size != nchans");
  g.max_delay = compute_max_delay(g.dm_list, g.delays);
  PSOUP_CHECK(static_cast<uint64_t>(g.max_delay) < nsamps,
              "max dispersion delay (" << g.max_delay << " samples) exceeds the observation (" << nsamps << ")");
  g.out_nsamps = nsamps - static_cast<uint64_t>(g.max_delay);
  const double in_range = static_cast<double>((1 << g.nbits) - 1);
  g.out_scale = static_cast<float>(192.0 / (in_range * g.nchans));
  g.bias = (g.nbits == 8) ? 128 : 0;
  g.nactive = 0;
  for (int k : g.killmask) g.nactive += (k != 0);
  return g;
}

std::vector<int32_t> DedispGeometry::offsets(int d0, int d1) const {
  std::vector<int32_t> o(static_cast<size_t>(d1 - d0) * nchans);
  for (int d = d0; d < d1; ++d)
    for (int c = 0; c < nchans; ++c)
      o[static_cast<size_t>(d - d0) * nchans + c] = dm_delay_samples(dm_list[d], delays[c]);
  return o;
}

// -------------------------------------------------------- device filterbank -
DeviceFilterbank::DeviceFilterbank(const DedispGeometry& g, hipStream_t stream) : g_(g), stream_(stream) {
  // rows padded so the MFMA kernel's over-reads (<= 560 B past the last
  // output sample + its offset) stay inside the row; one spare row at the end
  stride_ = (g_.nsamps + 1024 + 255) / 256 * 256;
  chan_.resize(stride_ * static_cast<uint64_t>(g_.nchans + 1));
  chan_.zero_async(stream_);
  if (g_.nbits <= 2 && g_.bias == 0) {
    // 2-bit rows: 6144 + 2048 samples of zeros past the int8 row length (a
    // workgroup's staged window past its last sample)
    stride2_ = (stride_ + 8192) / 64 * 4;
    chan2_.resize(stride2_ * static_cast<uint64_t>(g_.nchans));
    chan2_.zero_async(stream_);
  }
}

void DeviceFilterbank::pack2(uint64_t t0, uint64_t ns, hipStream_t s) {
  if (chan2_.size())
    kern::pack2_rows(chan_.data(), stride_, g_.nchans, chan2_.data(), stride2_, t0, ns, s ? s : stream_);
}

void DeviceFilterbank::load_packed_device(const uint8_t* d_packed) {
  kern::unpack_transpose(d_packed, g_.nsamps, g_.nchans, g_.nbits, chan_.data(), stride_, g_.bias, stream_);
  pack2(0, g_.nsamps, stream_);
}

void DeviceFilterbank::load_packed_host(const uint8_t* h_packed) {
  const uint64_t bytes = g_.nsamps * static_cast<uint64_t>(g_.nchans) * g_.nbits / 8;
  // Chunked: H2D through two pinned staging buffers, unpack each chunk.
  const uint64_t bps = static_cast<uint64_t>(g_.nchans) * g_.nbits / 8;
  uint64_t chunk_samps = std::max<uint64_t>(256, ((64ull << 20) / bps) / 256 * 256);
  PinnedBuffer<uint8_t> stage[2];
  DeviceBuffer<uint8_t> dstage[2];
  Event ev[2];
  for (int i = 0; i < 2; ++i) {
    stage[i].resize(chunk_samps * bps);
    dstage[i].resize(chunk_samps * bps);
  }
  int slot = 0;
  bool used[2] = {false, false};
  for (uint64_t t0 = 0; t0 < g_.nsamps; t0 += chunk_samps) {
    const uint64_t ns = std::min(chunk_samps, g_.nsamps - t0);
    if (used[slot]) ev[slot].sync();
    std::memcpy(stage[slot].data(), h_packed + t0 * bps, ns * bps);
    PSOUP_HIP_CHECK(hipMemcpyAsync(dstage[slot].data(), stage[slot].data(), ns * bps, hipMemcpyHostToDevice, stream_));
    kern::unpack_transpose(dstage[slot].data(), ns, g_.nchans, g_.nbits, chan_.data() + t0, stride_, g_.bias, stream_);
    pack2(t0, ns, stream_);
    ev[slot].record(stream_);
    used[slot] = true;
    slot ^= 1;
  }
  (void)bytes;
  PSOUP_HIP_CHECK(hipStreamSynchronize(stream_));
}

void DeviceFilterbank::unpack_chunk(const uint8_t* d_packed, uint64_t t0, uint64_t ns, hipStream_t s) {
  PSOUP_CHECK(t0 + ns <= g_.nsamps, "unpack_chunk: samples past the filterbank");
  kern::unpack_transpose(d_packed, ns, g_.nchans, g_.nbits, chan_.data() + t0, stride_, g_.bias, s ? s : stream_);
  pack2(t0, ns, s);
}

void staged_upload(uint64_t bytes, uint64_t chunk, const HostReader& read, uint8_t* d_dst, hipStream_t s,
                   const std::function<void(uint64_t, uint64_t)>& on_chunk) {
  if (bytes == 0) return;
  chunk = std::max<uint64_t>(1, std::min(chunk, bytes));
  // two pinned stages: the host reads chunk k+1 while chunk k's copy runs
  // (pinning is ~0.1 ms per MB: 16 MB stages, not the whole file)
  PinnedBuffer<uint8_t> stage[2];
  Event staged[2];
  bool used[2] = {false, false};
  int slot = 0;
  for (uint64_t off = 0; off < bytes; off += chunk, slot ^= 1) {
    const uint64_t nb = std::min(chunk, bytes - off);
    if (stage[slot].size() < nb) stage[slot].resize(nb);
    if (used[slot]) staged[slot].sync();
    read(off, nb, stage[slot].data());
    PSOUP_HIP_CHECK(hipMemcpyAsync(d_dst + off, stage[slot].data(), nb, hipMemcpyHostToDevice, s));
    staged[slot].record(s);
    used[slot] = true;
    if (on_chunk) on_chunk(off, nb);
  }
  for (int i = 0; i < 2; ++i)
    if (used[i]) staged[i].sync();
}

namespace {
void fanout_impl(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices, const HostReader& read,
                 const uint8_t* h_direct) {
  PSOUP_CHECK(!fbs.empty() && fbs.size() == devices.size(), "load_filterbank_fanout: one device per filterbank");
  const DedispGeometry& g = fbs[0]->geometry();
  const uint64_t bps = static_cast<uint64_t>(g.nchans) * g.nbits / 8;  // bytes per sample
  const uint64_t bytes = g.nsamps * bps;
  const uint64_t chunk = std::max<uint64_t>(256, ((16ull << 20) / bps) / 256 * 256);  // samples per chunk
  int prev = 0;
  PSOUP_HIP_CHECK(hipGetDevice(&prev));
  const size_t n = fbs.size();
  // device i pulls each chunk from the first device: with peer access the
  // copy reads device 0's memory straight over xGMI instead of staging it
  // through host memory
  for (size_t i = 1; i < n; ++i) enable_peer_access(devices[i], devices[0]);
  // the packed bytes on every device (transient: freed on return)
  std::vector<DeviceBuffer<uint8_t>> packed(n);
  for (size_t i = 0; i < n; ++i) {
    PSOUP_HIP_CHECK(hipSetDevice(devices[i]));
    packed[i].resize(bytes);
  }
  PSOUP_HIP_CHECK(hipSetDevice(devices[0]));
  hipStream_t s0 = fbs[0]->stream();
  Event landed;
  auto on_chunk = [&](uint64_t off, uint64_t nb) {
    const uint64_t t0 = off / bps, ns = nb / bps;
    landed.record(s0);
    fbs[0]->unpack_chunk(packed[0].data() + off, t0, ns);
    for (size_t i = 1; i < n; ++i) {
      PSOUP_HIP_CHECK(hipSetDevice(devices[i]));
      hipStream_t si = fbs[i]->stream();
      PSOUP_HIP_CHECK(hipStreamWaitEvent(si, landed.get(), 0));
      PSOUP_HIP_CHECK(hipMemcpyPeerAsync(packed[i].data() + off, devices[i], packed[0].data() + off, devices[0], nb, si));
      fbs[i]->unpack_chunk(packed[i].data() + off, t0, ns);
    }
    PSOUP_HIP_CHECK(hipSetDevice(devices[0]));
  };
  if (h_direct && bytes <= chunk * bps) {
    // a file within one chunk goes up straight from its (mapped) pages:
    // pinning a stage costs more than the copy (tutorial.fil: 3 MB)
    PSOUP_HIP_CHECK(hipMemcpy(packed[0].data(), h_direct, bytes, hipMemcpyHostToDevice));
    on_chunk(0, bytes);
  } else {
    staged_upload(bytes, chunk * bps, read, packed[0].data(), s0, on_chunk);
  }
  for (size_t i = 0; i < n; ++i) {
    PSOUP_HIP_CHECK(hipSetDevice(devices[i]));
    PSOUP_HIP_CHECK(hipStreamSynchronize(fbs[i]->stream()));
  }
  // the transient copies are freed on their own devices
  for (size_t i = 0; i < n; ++i) {
    PSOUP_HIP_CHECK(hipSetDevice(devices[i]));
    packed[i] = DeviceBuffer<uint8_t>();
  }
  PSOUP_HIP_CHECK(hipSetDevice(prev));
}

}  // namespace

void load_filterbank_fanout(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices,
                            const HostReader& read) {
  fanout_impl(fbs, devices, read, nullptr);
}

void load_filterbank_fanout(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices,
                            const uint8_t* h_packed) {
  fanout_impl(
      fbs, devices, [h_packed](uint64_t off, uint64_t n, uint8_t* dst) { std::memcpy(dst, h_packed + off, n); },
      h_packed);
}

void load_filterbank_fanout(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices,
                            const Filterbank& fb) {
  fanout_impl(
      fbs, devices, [&fb](uint64_t off, uint64_t n, uint8_t* dst) { fb.read_data(off, n, dst); }, fb.data());
}

Dedisperser::Dedisperser(const DeviceFilterbank& fb, hipStream_t stream) : fb_(fb), stream_(stream) {
  const auto& g = fb_.geometry();
  std::vector<int32_t> kill(g.killmask.begin(), g.killmask.end());
  std::vector<int32_t> active;
  for (int c = 0; c < g.nchans; ++c)
    if (g.killmask[c]) active.push_back(c);
  d_kill_.resize(kill.size());
  PSOUP_HIP_CHECK(hipMemcpy(d_kill_.data(), kill.data(), kill.size() * 4, hipMemcpyHostToDevice));
  d_active_.resize(std::max<size_t>(1, active.size()));
  if (!active.empty())
    PSOUP_HIP_CHECK(hipMemcpy(d_active_.data(), active.data(), active.size() * 4, hipMemcpyHostToDevice));
}

void Dedisperser::warm(int d0, int d1) {
  // The tables Auto needs (VALU offsets and windows, LDS-fed MFMA plan) for
  // the tiles of [d0, d1) (a rank's static shard; default the whole list),
  // from one offset table, the two builds in parallel.  A later range outside
  // them rebuilds the whole list's (ensure_tables).  The whole-list
  // global-load MFMA plan (~380k steps on the 2026-DM config-4 list, 136 ms on
  // the host) serves only an explicit --dedisp_kernel mfma over tiles the LDS
  // kernel cannot take: built on first such use.
  const auto& g = fb_.geometry();
  const int ndm = static_cast<int>(g.dm_list.size());
  if (ndm == 0 || g.nactive == 0) return;
  if (d1 < 0 || d1 > ndm) d1 = ndm;
  d0 = std::max(0, std::min(d0, d1 - 1));
  const int t0 = d0 / kTileDms, t1 = (d1 - 1) / kTileDms + 1;
  if (tab_t0_ <= t0 && t1 <= tab_t1_) return;
  build_tables(t0, t1);
}

void Dedisperser::ensure_tables(int d0, int d1) {
  const int ndm = static_cast<int>(fb_.geometry().dm_list.size());
  const int t0 = d0 / kTileDms, t1 = (std::max(d0 + 1, d1) - 1) / kTileDms + 1;
  if (tab_t0_ <= t0 && t1 <= tab_t1_) return;
  build_tables(0, (ndm + kTileDms - 1) / kTileDms);
}

void Dedisperser::build_tables(int t0, int t1) {
  const auto& g = fb_.geometry();
  const int ndm = static_cast<int>(g.dm_list.size());
  // offsets of DMs [t0 * 32, (t1 + 1) * 32): the VALU tables' columns run one
  // tile past the last (a range from an unaligned DM reads up to 31 beyond it)
  const int e0 = t0 * kTileDms, e1 = std::min(ndm, (t1 + 1) * kTileDms);
  const std::vector<int32_t> offs = g.offsets(e0, e1);
  std::exception_ptr err;
  std::unique_ptr<kern::MfmaLdsPlan> plan;
  std::thread th;
  if (g.nactive > 0)
    th = std::thread([&] {
      try {
        std::vector<int32_t> kill(g.killmask.begin(), g.killmask.end());
        plan = std::make_unique<kern::MfmaLdsPlan>();
        kern::build_mfma_lds_plan(offs.data(), ndm, g.nchans, kill.data(), *plan, t0, t1, e0);
      } catch (...) {
        err = std::current_exception();
      }
    });
  try {
    build_valu_tables(offs, e0, t0, t1);
  } catch (...) {
    if (th.joinable()) th.join();
    throw;
  }
  if (th.joinable()) th.join();
  if (err) std::rethrow_exception(err);
  if (plan) upload_mfma_lds_tables(*plan);
  tab_t0_ = t0;
  tab_t1_ = t1;
}

void Dedisperser::build_resident_plan() {
  const auto& g = fb_.geometry();
  const int ndm = static_cast<int>(g.dm_list.size());
  std::vector<int32_t> offs = g.offsets(0, ndm);
  std::vector<int32_t> kill(g.killmask.begin(), g.killmask.end());
  kern::MfmaDedispPlan plan;
  kern::build_mfma_dedisp_plan(offs.data(), ndm, g.nchans, kill.data(), plan);
  r_steps_.resize(plan.steps.size());
  r_deltas_.resize(plan.deltas.size());
  r_tile_info_.resize(plan.tile_info.size());
  PSOUP_HIP_CHECK(hipMemcpy(r_steps_.data(), plan.steps.data(), plan.steps.size() * 4, hipMemcpyHostToDevice));
  PSOUP_HIP_CHECK(hipMemcpy(r_deltas_.data(), plan.deltas.data(), plan.deltas.size(), hipMemcpyHostToDevice));
  PSOUP_HIP_CHECK(
      hipMemcpy(r_tile_info_.data(), plan.tile_info.data(), plan.tile_info.size() * 4, hipMemcpyHostToDevice));
  resident_ = true;
}

void Dedisperser::build_valu_tables(const std::vector<int32_t>& offs, int e0, int t0, int t1) {
  // offsets transposed to [active channel][DM], columns padded (with the last
  // DM) past the last workgroup of any range; filled for the columns of tiles
  // [t0, t1 + 1) only (offs: rows of DMs [e0, ...))
  const auto& g = fb_.geometry();
  const int ndm = static_cast<int>(g.dm_list.size());
  std::vector<int> active;
  for (int c = 0; c < g.nchans; ++c)
    if (g.killmask[c]) active.push_back(c);
  ldo_ = (ndm + kTileDms - 1) / kTileDms * kTileDms + kTileDms;
  const int j0 = t0 * kTileDms, j1 = std::min(ldo_, (t1 + 1) * kTileDms), w = j1 - j0;
  const size_t na = std::max<size_t>(1, active.size());
  std::vector<int32_t> t(na * static_cast<size_t>(w), 0);
  for (size_t ci = 0; ci < active.size(); ++ci)
    for (int j = j0; j < j1; ++j)
      t[ci * w + (j - j0)] = offs[static_cast<size_t>(std::min(j, ndm - 1) - e0) * g.nchans + active[ci]];
  r_offT_.resize(na * static_cast<size_t>(ldo_));
  PSOUP_HIP_CHECK(hipMemcpy2D(r_offT_.data() + j0, static_cast<size_t>(ldo_) * 4, t.data(), static_cast<size_t>(w) * 4,
                              static_cast<size_t>(w) * 4, na, hipMemcpyHostToDevice));
  // LDS kernel windows: per 32-DM tile and channel, the smallest offset
  // (rounded down to 16 bytes) and the window length it must stage
  const int ntiles = ldo_ / kTileDms;
  std::vector<int32_t> wmin(static_cast<size_t>(t1 - t0) * na, 0);
  h_tile_win_.assign(static_cast<size_t>(ntiles), 0);
  // and the global-load MFMA plan's step count per tile (its 16-sample blocks
  // from each channel's smallest offset, two per step), which Auto weighs
  // against the VALU kernels without building that plan
  h_tile_steps_.assign(static_cast<size_t>(ntiles), 0);
  for (int T = t0; T < t1; ++T) {
    int64_t blocks = 0;
    for (size_t ci = 0; ci < active.size(); ++ci) {
      const int32_t* col = &t[ci * w + (T * kTileDms - j0)];
      int lo = col[0], hi = lo;
      for (int k = 1; k < kTileDms; ++k) {
        lo = std::min(lo, col[k]);
        hi = std::max(hi, col[k]);
      }
      const int w0 = lo & ~15;
      wmin[static_cast<size_t>(T - t0) * na + ci] = w0;
      h_tile_win_[static_cast<size_t>(T)] = std::max(h_tile_win_[static_cast<size_t>(T)], 1024 + (hi - w0) + 32);
      blocks += (hi - lo) / 16 + 1;
    }
    h_tile_steps_[static_cast<size_t>(T)] = static_cast<int32_t>((blocks + 1) / 2);
  }
  r_wmin_.resize(static_cast<size_t>(ntiles) * na);
  PSOUP_HIP_CHECK(hipMemcpy(r_wmin_.data() + static_cast<size_t>(t0) * na, wmin.data(), wmin.size() * 4,
                            hipMemcpyHostToDevice));
}

int Dedisperser::max_spread(int d0, int d1) const {
  int win = 0;
  for (int T = d0 / kTileDms; T <= (d1 - 1) / kTileDms; ++T) win = std::max(win, h_tile_win_[static_cast<size_t>(T)]);
  return std::max(0, win - 1056);  // h_tile_win_ = 1024 + (hi - w0) + 32
}

static double valu_ratio() {
  // MFMA steps per (tile, active channel) above which the VALU kernel is
  // faster (calibrated on MI355X with tools/dedisp_bench.py)
  return 1.85;
}

double Dedisperser::mfma_steps_per_channel(int d0, int d1) {
  const auto& g = fb_.geometry();
  PSOUP_CHECK(d0 >= 0 && d0 < d1 && d1 <= static_cast<int>(g.dm_list.size()), "bad DM range");
  ensure_tables(d0, d1);
  double steps = 0;
  const int t0 = d0 / kTileDms, t1 = (d1 - 1) / kTileDms;
  for (int T = t0; T <= t1; ++T) steps += h_tile_steps_[static_cast<size_t>(T)];
  return steps / ((t1 - t0 + 1) * static_cast<double>(std::max(1, g.nactive)));
}

DedispKernel Dedisperser::choose(int d0, int d1) {
  const auto& g = fb_.geometry();
  if (g.nactive == 0 || d0 >= d1) return DedispKernel::Mfma;
  // the LDS-staged packed-byte kernel (tile-aligned ranges, narrow samples)
  // beats the MFMA plan from ~1.0 steps per channel, the global-load one from 1.85
  ensure_tables(d0, d1);
  int win = 0;
  for (int T = d0 / kTileDms; T <= (d1 - 1) / kTileDms; ++T) win = std::max(win, h_tile_win_[static_cast<size_t>(T)]);
  const bool lds = kern::dedisperse_lds_fits(g.nbits, g.nactive, win);
  const double ratio = lds ? valu_ratio() * (1.0 / 1.85) : valu_ratio();
  return mfma_steps_per_channel(d0, d1) > ratio ? DedispKernel::Valu : DedispKernel::Mfma;
}

void Dedisperser::upload_mfma_lds_tables(const kern::MfmaLdsPlan& plan) {
  ml_ngroups_ = plan.ngroups;
  ml_tile_ok_ = plan.tile_ok;
  ml_tile_steps_ = plan.tile_steps;
  auto up = [](auto& dev, const auto& host) {
    using T = typename std::decay_t<decltype(host)>::value_type;
    dev.resize(std::max<size_t>(1, host.size()));
    if (!host.empty()) PSOUP_HIP_CHECK(hipMemcpy(dev.data(), host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
  };
  up(ml_steps_, plan.steps);
  up(ml_relo_, plan.relo);
  up(ml_ginfo_, plan.ginfo);
  up(ml_wmin_, plan.wmin);
}

static double mfma_lds_ratio(bool packed2) {
  // LDS-fed MFMA steps per (tile, active channel) up to which a tile takes the
  // MFMA kernel in Auto (each step is 2 x 16-shift blocks of one-hot GEMM;
  // the VALU kernels cost the same per channel whatever the spread).
  // Measured crossover on MI355X vs the byte kernel (profiles/r3_dedisp):
  // ~2.35 steps/channel; vs the 2-bit kernel none (1.11 vs 1.38 ms per
  // 32-DM chunk at DM 0, 1024 ch x 2^20, profiles/r5_dedisp); override with
  // PSOUP_MFMA_LDS_RATIO_2BIT
  if (packed2) {
    static const double r2 = [] {
      const char* e = std::getenv("PSOUP_MFMA_LDS_RATIO_2BIT");
      return e ? std::atof(e) : 0.0;  // the 2-bit kernel won every 32-DM chunk of the config-4 list
    }();
    return r2;
  }
  return 2.3;
}

int Dedisperser::mfma_lds_split(int d0, int d1) {
  const auto& g = fb_.geometry();
  if (g.nactive == 0) return d0;
  ensure_tables(d0, d1);
  const double ratio = mfma_lds_ratio(fb_.data2() != nullptr && kern::dedisperse_2bit_fits(g.nactive, max_spread(d0, d1)));
  if (ratio <= 0) return d0;
  int T = d0 / kTileDms;
  const int T1 = (d1 - 1) / kTileDms + 1;
  // the MFMA kernel computes whole 32-DM tiles, the VALU kernels only the
  // DMs asked for (8-DM workgroups for short ranges): a partial tile's MFMA
  // budget shrinks with its DM count (the bench's 8-DM chunk at DM 0:
  // MFMA 9.7 ms vs VALU 4.9 ms per step at 2^23)
  auto tile_dms = [&](int t) { return std::min(d1, (t + 1) * kTileDms) - std::max(d0, t * kTileDms); };
  while (T < T1 && ml_tile_ok_[static_cast<size_t>(T)] &&
         ml_tile_steps_[static_cast<size_t>(T)] <= ratio * g.nactive * tile_dms(T) / kTileDms)
    ++T;
  return std::min(d1, T * kTileDms);
}

void Dedisperser::run_mfma_lds(int d0, int d1, uint8_t* out, uint64_t out_stride, hipStream_t s) {
  const auto& g = fb_.geometry();
  ensure_tables(d0, d1);
  // whole tiles from the one holding d0; its DMs before d0 are not stored
  const int T0 = d0 / kTileDms, skip = d0 - T0 * kTileDms, nt = (d1 - T0 * kTileDms + kTileDms - 1) / kTileDms;
  kern::dedisperse_mfma_lds(fb_.data(), fb_.stride(), d_active_.data(), g.nactive, ml_steps_.data(),
                            ml_relo_.data() + static_cast<size_t>(T0) * ml_ngroups_ * kern::kMfmaLdsGroup * 32,
                            ml_ginfo_.data() + static_cast<size_t>(T0) * ml_ngroups_ * 2,
                            ml_ngroups_, ml_wmin_.data() + static_cast<size_t>(T0) * g.nactive, nt, d1 - d0,
                            g.out_nsamps, out, out_stride, g.out_scale, g.bias * g.nactive, s, skip);
}

void Dedisperser::run_list(const std::vector<int>& dms, uint8_t* out, uint64_t out_stride, hipStream_t s) {
  const auto& g = fb_.geometry();
  if (dms.empty()) return;
  if (!s) s = stream_;
  const int ndm_list = static_cast<int>(g.dm_list.size());
  for (int d : dms) PSOUP_CHECK(d >= 0 && d < ndm_list, "run_list: DM index " << d << " outside the list");
  if (g.nactive == 0) {  // every channel killed: the direct kernel writes the bias rows
    for (size_t i = 0; i < dms.size(); ++i)
      run(dms[i], dms[i] + 1, out + i * out_stride, out_stride, DedispKernel::Direct, s);
    return;
  }
  RoctxRange r("Dedisperse");
  const int n = static_cast<int>(dms.size());
  const int ldo = (n + kTileDms - 1) / kTileDms * kTileDms + kTileDms;  // padded like build_valu_tables
  std::vector<int> active;
  for (int c = 0; c < g.nchans; ++c)
    if (g.killmask[c]) active.push_back(c);
  std::vector<int32_t> t(active.size() * static_cast<size_t>(ldo));
  for (int j = 0; j < ldo; ++j) {
    const int d = dms[static_cast<size_t>(std::min(j, n - 1))];  // padded columns repeat the last DM
    const std::vector<int32_t> offs = g.offsets(d, d + 1);
    for (size_t ci = 0; ci < active.size(); ++ci) t[ci * ldo + j] = offs[static_cast<size_t>(active[ci])];
  }
  d_list_offT_.resize(t.size());
  PSOUP_HIP_CHECK(hipMemcpyAsync(d_list_offT_.data(), t.data(), t.size() * 4, hipMemcpyHostToDevice, s));
  PSOUP_HIP_CHECK(hipStreamSynchronize(s));
  kern::dedisperse_valu(fb_.data(), fb_.stride(), d_active_.data(), g.nactive, d_list_offT_.data(), ldo, 0, n,
                        g.out_nsamps, out, out_stride, g.out_scale, g.nbits, g.bias, s);
}

void Dedisperser::run(int d0, int d1, uint8_t* out, uint64_t out_stride, DedispKernel kind, hipStream_t s) {
  const auto& g = fb_.geometry();
  PSOUP_CHECK(d0 >= 0 && d1 <= static_cast<int>(g.dm_list.size()) && d0 <= d1, "bad DM range");
  if (d0 == d1) return;
  if (!s) s = stream_;
  RoctxRange r("Dedisperse");
  const int ndm_list = static_cast<int>(g.dm_list.size());
  (void)ndm_list;
  // Every kernel below takes any DM range: a range not starting on a 32-DM
  // tile computes its first tile (or workgroup) whole and stores from d0, so
  // every rank of a DM-sharded run dedisperses with the same kernels and no
  // per-call host tables.
  if (kind == DedispKernel::Auto && g.nactive > 0) {
    // hybrid: the leading narrow-spread tiles on the LDS-fed MFMA kernel, the
    // rest (tile-aligned from the split) on the VALU kernels
    const int split = mfma_lds_split(d0, d1);
    if (split > d0) {
      run_mfma_lds(d0, split, out, out_stride, s);
      if (split < d1) {
        const bool p2 = fb_.data2() && kern::dedisperse_2bit_fits(g.nactive, max_spread(split, d1));
        run(split, d1, out + static_cast<uint64_t>(split - d0) * out_stride, out_stride,
            p2 ? DedispKernel::Packed2 : DedispKernel::Valu, s);
      }
      return;
    }
  }
  if (kind == DedispKernel::Mfma && g.nactive > 0) {
    // explicit MFMA: the LDS-fed kernel where every tile fits its window
    ensure_tables(d0, d1);
    bool fit = true;
    for (int T = d0 / kTileDms; T <= (d1 - 1) / kTileDms; ++T) fit = fit && ml_tile_ok_[static_cast<size_t>(T)];
    if (fit) {
      run_mfma_lds(d0, d1, out, out_stride, s);
      return;
    }
  }
  if (kind == DedispKernel::Auto) {
    // past the MFMA-LDS tiles: the 2-bit kernel where the data allows (it
    // beats the global-load MFMA plan at any spread), else the byte / MFMA choice
    ensure_tables(d0, d1);
    kind = fb_.data2() && kern::dedisperse_2bit_fits(g.nactive, max_spread(d0, d1)) ? DedispKernel::Packed2
                                                                                   : choose(d0, d1);
  }
  if ((kind == DedispKernel::Valu || kind == DedispKernel::Packed2) && g.nactive == 0) kind = DedispKernel::Direct;
  const int ndm = d1 - d0;
  if (kind == DedispKernel::Packed2) {
    PSOUP_CHECK(fb_.data2(), "packed2 dedispersion needs nbits <= 2 data");
    ensure_tables(d0, d1);
    const int spread = max_spread(d0, d1);
    if (kern::dedisperse_2bit_fits(g.nactive, spread)) {
      kern::dedisperse_2bit(fb_.data2(), fb_.stride2(), d_active_.data(), g.nactive, r_offT_.data(), ldo_, d0, ndm,
                            r_wmin_.data(), spread, g.max_delay, g.out_nsamps, out, out_stride, g.out_scale, s);
      return;
    }
    kind = DedispKernel::Valu;  // a window too wide for the 2-bit kernel's LDS
  }
  if (kind == DedispKernel::Valu) {
    ensure_tables(d0, d1);
    int win = 0;
    for (int T = d0 / kTileDms; T <= (d1 - 1) / kTileDms; ++T) win = std::max(win, h_tile_win_[static_cast<size_t>(T)]);
    if (kern::dedisperse_lds_fits(g.nbits, g.nactive, win))
      kern::dedisperse_lds(fb_.data(), fb_.stride(), d_active_.data(), g.nactive, r_offT_.data(), ldo_, d0, ndm,
                           r_wmin_.data(), win, g.out_nsamps, out, out_stride, g.out_scale, g.nbits, g.bias, s);
    else
      kern::dedisperse_valu(fb_.data(), fb_.stride(), d_active_.data(), g.nactive, r_offT_.data(), ldo_, d0, ndm,
                            g.out_nsamps, out, out_stride, g.out_scale, g.nbits, g.bias, s);
    return;
  }
  if (kind == DedispKernel::Mfma) {
    // whole tiles of the resident plan from the one holding d0
    if (!resident_) build_resident_plan();
    const int T0 = d0 / kTileDms, skip = d0 - T0 * kTileDms;
    const int ntiles = (d1 - T0 * kTileDms + kTileDms - 1) / kTileDms;
    kern::dedisperse_mfma(fb_.data(), fb_.stride(), r_steps_.data(), r_deltas_.data(), r_tile_info_.data() + 2 * T0,
                          ntiles, ndm, g.out_nsamps, out, out_stride, g.out_scale, g.bias * g.nactive, s, skip);
  } else {
    std::vector<int32_t> offs = g.offsets(d0, d1);
    d_offsets_.resize(offs.size());
    PSOUP_HIP_CHECK(hipMemcpyAsync(d_offsets_.data(), offs.data(), offs.size() * 4, hipMemcpyHostToDevice, s));
    PSOUP_HIP_CHECK(hipStreamSynchronize(s));
    kern::dedisperse_direct(fb_.data(), fb_.stride(), g.nchans, d_offsets_.data(), d_kill_.data(), ndm, g.out_nsamps,
                            out, out_stride, g.out_scale, g.bias, g.nactive, s);
  }
}

// ---------------------------------------------------------------- whitener --
Whitener::Whitener(uint64_t n, float tsamp, hipStream_t stream, bool allow_fft4)
    : n_(n), tsamp_(tsamp), stream_(stream) {
  PSOUP_CHECK(n >= 250, "series too short for the running median (need >= 250 samples)");
  float tobs = static_cast<float>(static_cast<float>(n) * tsamp);
  bin_width_ = static_cast<float>(1.0 / tobs);
  const uint64_t nb = nbins();
  if (allow_fft4 && n % 2 == 0) {
    g4_ = kern::fft4_geometry(n / 2);
    g4_.zero_shift = (kern::fft4_flags() & kern::kFft4WhitenStrips) != 0;  // plain FFTs: strip-layout pass A
    // single-transform grids of both passes need n1/8 % 16 == 0 and n2/8 % 8 == 0
    f4_ = g4_.ok && g4_.n1 >= 128 && g4_.n2 >= 64;
  }
  if (const char* fs = std::getenv("PSOUP_WHITEN_FUSED_STATS")) fused_stats_ = std::atoi(fs) != 0;
  fser_.resize(nb);
  m5_.resize(nb / 5);
  m25_.resize(std::max<uint64_t>(1, nb / 5 / 5));
  m125_.resize(std::max<uint64_t>(1, nb / 5 / 5 / 5));
  partials_.resize(2 * 1024);
  stats_.resize(4);
  sum_.resize(1);
  if (f4_) {
    auto tab = kern::fft4_tables(g4_);
    tab4_.resize(tab.size());
    PSOUP_HIP_CHECK(hipMemcpy(tab4_.data(), tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));
    ensure_batch(1);
  } else if (allow_fft4) {
    // lengths with an odd factor (e.g. the coincidencer's whole DM-0 series,
    // 1114112 = 17 x 2^16): m batched power-of-two FFTs + a length-m pass
    const uint64_t p = n & (~n + 1);  // largest power of two dividing n
    const uint64_t m = n / p;
    if (m >= 3 && m <= 255) {
      gm_ = kern::fft4_geometry(p);
      gm_.zero_shift = (kern::fft4_flags() & kern::kFft4WhitenStrips) != 0;
      mixed_ = gm_.ok && gm_.n1 >= 128 && gm_.n2 >= 64;
    }
    if (mixed_) {
      mm_ = static_cast<uint32_t>(m);
      mp_ = p;
      auto tab = kern::fft4_tables(gm_);
      mtab_.resize(tab.size());
      PSOUP_HIP_CHECK(hipMemcpy(mtab_.data(), tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));
      mz_.resize(n);
      mpad_.resize(gm_.insize * m);
      my_.resize(gm_.ystride * m);
      mx_.resize(gm_.xstride * m);
      maf0_.resize(m);
      maf0_.zero_async(stream_);
    }
  }
}

void Whitener::mixed_fft(const float* src, int gather_mode, void* out, int combine_mode) {
  const uint64_t fl = 2 * mp_;  // floats per column (interleaved complex)
  const int K = static_cast<int>(mm_);
  kern::mixed_gather(src, n_, mm_, mp_, gather_mode, mz_.data(), stream_);
  const float* z = reinterpret_cast<const float*>(mz_.data());
  kern::Fft4Geom g = gm_;
  g.in_tstride = fl;
  g.pad_tstride = gm_.insize;
  kern::fft4_pad_input(z, fl, mpad_.data(), gm_, stream_, K, fl);
  kern::fft4_resample_colpass(z, mpad_.data(), fl, maf0_.data(), K, my_.data(), g, mtab_.data(), stream_);
  kern::fft4_rowpass(my_.data(), mx_.data(), K, gm_, mtab_.data(), stream_);
  kern::mixed_combine(mx_.data(), gm_.xstride, kern::xlayout_args(gm_, kern::fft4_x_layout(gm_)), n_, mm_, mp_,
                      combine_mode, out, stream_);
}

FftPlan& Whitener::r2c() {
  if (!r2c_) r2c_ = std::make_unique<FftPlan>(FftType::R2C, n_, 1);
  return *r2c_;
}

FftPlan& Whitener::c2r() {
  if (!c2r_) c2r_ = std::make_unique<FftPlan>(FftType::C2R, n_, 1);
  return *c2r_;
}

void Whitener::forward(const float* d_series, float2* d_spec) {
  if (mixed_) {
    mixed_fft(d_series, 0, d_spec, 0);
    return;
  }
  if (!f4_) {
    r2c().execute(const_cast<float*>(d_series), d_spec, stream_);
    return;
  }
  const uint64_t M = n_ / 2;
  kern::fft4_pad_input(d_series, n_, in4_.data(), g4_, stream_);
  kern::fft4_resample_colpass(d_series, in4_.data(), n_, af0_.data(), 1, y4_.data(), g4_, tab4_.data(), stream_);
  kern::fft4_rowpass(y4_.data(), x4_.data(), 1, g4_, tab4_.data(), stream_);
  kern::fft4_r2c_half(x4_.data(), M, kern::xlayout_args(g4_, kern::fft4_x_layout(g4_)), d_spec, stream_);
}

void Whitener::inverse(const float2* d_spec, float* d_series) {
  if (mixed_) {
    // C2R = Re FFT(conj of the Hermitian extension), unnormalised like rocFFT's
    mixed_fft(reinterpret_cast<const float*>(d_spec), 1, d_series, 1);
    return;
  }
  if (!f4_) {
    c2r().execute(const_cast<float2*>(d_spec), d_series, stream_);
    return;
  }
  const uint64_t M = n_ / 2;
  kern::fft4_c2r_pre(d_spec, M, tmp4_.data(), stream_);
  const float* t = reinterpret_cast<const float*>(tmp4_.data());
  kern::fft4_pad_input(t, n_, in4_.data(), g4_, stream_);
  kern::fft4_resample_colpass(t, in4_.data(), n_, af0_.data(), 1, y4_.data(), g4_, tab4_.data(), stream_);
  kern::fft4_rowpass(y4_.data(), x4_.data(), 1, g4_, tab4_.data(), stream_);
  kern::fft4_c2r_post(x4_.data(), M, kern::xlayout_args(g4_, kern::fft4_x_layout(g4_)), d_series, stream_);
}

void Whitener::load_trial(const uint8_t* d_trial, uint64_t nsamps, float* d_series) {
  const uint64_t nvalid = std::min(nsamps, n_);
  kern::u8_sum(d_trial, nvalid, sum_.data(), stream_);
  kern::u8_to_f32_pad(d_trial, nvalid, d_series, n_, sum_.data(), stream_);
}

void Whitener::dered_stats(float2* spec, const uint32_t* d_zapmask, float* d_stats, float boundary5,
                           float boundary25) {
  const uint64_t nb = nbins();
  const uint64_t n5 = nb / 5, n25 = n5 / 5, n125 = n25 / 5;
  kern::median5_amp(spec, nb, m5_.data(), stream_);
  kern::median5(m5_.data(), n5, m25_.data(), stream_);
  kern::median5(m25_.data(), n25, m125_.data(), stream_);
  const int64_t pos5 = static_cast<int64_t>(static_cast<int>(boundary5 / bin_width_));
  const int64_t pos25 = static_cast<int64_t>(static_cast<int>(boundary25 / bin_width_));
  kern::deredden_zap(spec, nb, m5_.data(), n5, m25_.data(), std::max<uint64_t>(1, n25), m125_.data(),
                     std::max<uint64_t>(1, n125), pos5, pos25, d_zapmask, stream_);
  if (d_stats) kern::interbin_stats(spec, nb, nullptr, partials_.data(), 1024, d_stats, stream_);
}

void Whitener::whiten(float* d_series, const uint32_t* d_zapmask, bool with_stats, float boundary5, float boundary25) {
  forward(d_series, fser_.data());
  dered_stats(fser_.data(), d_zapmask, with_stats ? stats_.data() : nullptr, boundary5, boundary25);
  inverse(fser_.data(), d_series);
}

uint64_t Whitener::batch_bytes_per_trial() const {
  if (!f4_) return 0;
  return g4_.ystride * 8 + g4_.xstride * 8 + nbins() * 8 + (n_ / 2) * 8 + g4_.insize * 4 +
         3 * (nbins() / 5 + 1) * 4 + 2 * 1024 * 8;
}

void Whitener::reserve_batch(int count) {
  if (f4_) ensure_batch(count);
}

void Whitener::ensure_batch(int count) {
  if (count <= bcap_) return;
  y4_.resize(g4_.ystride * count);
  x4_.resize(g4_.xstride * count);
  tmp4_.resize((n_ / 2) * count);
  in4_.resize(g4_.insize * count);
  bspec_.resize(nbins() * count);
  bsum_.resize(static_cast<uint64_t>(count));
  // running medians / stats partials of every batch item (stride: n5)
  const uint64_t ms = std::max<uint64_t>(1, nbins() / 5);
  m5_.resize(ms * count);
  m25_.resize(ms * count);
  m125_.resize(ms * count);
  partials_.resize(2 * 1024 * static_cast<uint64_t>(count));
  af0_.resize(static_cast<uint64_t>(count));
  af0_.zero_async(stream_);
  bcap_ = count;
}

bool Whitener::whiten_batch(const uint8_t* d_trials, uint64_t row_stride, uint64_t nsamps, int count, float* d_out,
                            uint64_t out_stride, const uint32_t* d_zapmask, float* d_stats, float boundary5,
                            float boundary25, float* pad_out, const kern::Fft4Geom* pad_g, uint64_t pad_stride) {
  PSOUP_CHECK(count >= 1, "whiten_batch: empty batch");
  if (!f4_) {
    for (int b = 0; b < count; ++b) {
      float* x = d_out + static_cast<uint64_t>(b) * out_stride;
      load_trial(d_trials + static_cast<uint64_t>(b) * row_stride, nsamps, x);
      forward(x, fser_.data());
      dered_stats(fser_.data(), d_zapmask, d_stats + 4 * b, boundary5, boundary25);
      inverse(fser_.data(), x);
    }
    return false;
  }
  ensure_batch(count);
  const uint64_t M = n_ / 2, nb = nbins();
  const uint64_t nvalid = std::min(nsamps, n_);
  const kern::XLayoutArgs L = kern::xlayout_args(g4_, kern::fft4_x_layout(g4_));
  kern::u8_sum(d_trials, nvalid, bsum_.data(), stream_, count, row_stride);
  // forward: K = count transforms, trial b reading series b, the 8-bit rows
  // converted (mean-padded) straight into pass A's strip layout; d_out is
  // first written by the inverse
  kern::Fft4Geom g = g4_;
  g.in_tstride = out_stride;
  g.pad_tstride = g4_.insize;
  const bool direct = kern::fft4_direct_source(g4_);
  const bool u8_aligned = (reinterpret_cast<uintptr_t>(d_trials) & 15) == 0 && (count == 1 || row_stride % 16 == 0);
  if (direct && u8_aligned && (kern::fft4_flags() & kern::kFft4WhitenU8)) {
    g.u8 = d_trials;  // pass A reads the 8-bit rows themselves
    g.u8sum = bsum_.data();
    g.u8_nvalid = nvalid;
    g.src_stride = row_stride;
  } else if (direct && u8_aligned && !(kern::fft4_flags() & kern::kFft4WhitenF32)) {
    // 8-bit rows -> column strips, which pass A reads with contiguous wave loads
    kern::fft4_pad_input_u8(d_trials, nvalid, n_, bsum_.data(), in4_.data(), g4_, stream_, count, row_stride);
    g.strips_direct = true;
  } else if (direct && out_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(d_out) & 15) == 0) {
    // pass A reads the f32 copy itself (no padded copy)
    kern::u8_to_f32_pad(d_trials, nvalid, d_out, n_, bsum_.data(), stream_, count, row_stride, out_stride);
    g.f32_direct = true;
  } else if (kern::fft4_strip_layout(g4_) && u8_aligned) {
    kern::fft4_pad_input_u8(d_trials, nvalid, n_, bsum_.data(), in4_.data(), g4_, stream_, count, row_stride);
  } else {
    kern::u8_to_f32_pad(d_trials, nvalid, d_out, n_, bsum_.data(), stream_, count, row_stride, out_stride);
    kern::fft4_pad_input(d_out, n_, in4_.data(), g4_, stream_, count, out_stride);
  }
  kern::fft4_resample_colpass(d_out, in4_.data(), n_, af0_.data(), count, y4_.data(), g, tab4_.data(), stream_);
  kern::fft4_rowpass(y4_.data(), x4_.data(), count, g4_, tab4_.data(), stream_);
  kern::fft4_r2c_half(x4_.data(), M, L, bspec_.data(), stream_, count, g4_.xstride, nb);
  {
    // running median, dereddening + zapping and interbin stats of all items
    const uint64_t n5 = nb / 5, n25 = n5 / 5, n125 = n25 / 5, ms = std::max<uint64_t>(1, n5);
    kern::median5_amp(bspec_.data(), nb, m5_.data(), stream_, count, nb, ms);
    kern::median5(m5_.data(), n5, m25_.data(), stream_, count, ms, ms);
    kern::median5(m25_.data(), n25, m125_.data(), stream_, count, ms, ms);
    const int64_t pos5 = static_cast<int64_t>(static_cast<int>(boundary5 / bin_width_));
    const int64_t pos25 = static_cast<int64_t>(static_cast<int>(boundary25 / bin_width_));
    PSOUP_CHECK(!fused_stats_ || g4_.xstride >= nb, "whiten_batch: X stride below the spectrum length");
    if (fused_stats_) {
      // one pass, out of place into x4_ (free after the r2c until the
      // inverse's pass B; xstride >= nb): its statistics equal the two
      // kernels' bit for bit
      kern::deredden_zap_stats(bspec_.data(), x4_.data(), nb, m5_.data(), n5, m25_.data(),
                               std::max<uint64_t>(1, n25), m125_.data(), std::max<uint64_t>(1, n125), pos5, pos25,
                               d_zapmask, partials_.data(), 1024, d_stats, stream_, count, nb, g4_.xstride, ms);
    } else {
      kern::deredden_zap(bspec_.data(), nb, m5_.data(), n5, m25_.data(), std::max<uint64_t>(1, n25), m125_.data(),
                         std::max<uint64_t>(1, n125), pos5, pos25, d_zapmask, stream_, count, nb, ms);
      kern::interbin_stats(bspec_.data(), nb, nullptr, partials_.data(), 1024, d_stats, stream_, count, nb);
    }
  }
  // inverse (direct: pass A applies the C2R pre-processing to the spectra as it reads them)
  const float2* wspec = fused_stats_ ? x4_.data() : bspec_.data();
  const uint64_t wstride = fused_stats_ ? g4_.xstride : nb;
  const float* t = reinterpret_cast<const float*>(tmp4_.data());
  g.in_tstride = n_;
  g.u8 = nullptr;
  g.f32_direct = g.strips_direct = false;
  if (direct) {
    g.c2r = wspec;
    g.src_stride = wstride;
  } else {
    kern::fft4_c2r_pre(wspec, M, tmp4_.data(), stream_, count, wstride, M);
    kern::fft4_pad_input(t, n_, in4_.data(), g4_, stream_, count, n_);
  }
  kern::fft4_resample_colpass(t, in4_.data(), n_, af0_.data(), count, y4_.data(), g, tab4_.data(), stream_);
  kern::fft4_rowpass(y4_.data(), x4_.data(), count, g4_, tab4_.data(), stream_);
  if (pad_out && pad_g && kern::fft4_c2r_post_pad(x4_.data(), M, L, pad_out, *pad_g, stream_, count, g4_.xstride,
                                                  pad_stride))
    return true;
  kern::fft4_c2r_post(x4_.data(), M, L, d_out, stream_, count, g4_.xstride, out_stride);
  return false;
}

std::vector<uint32_t> build_zap_mask(const std::vector<float>& freqs, const std::vector<float>& widths,
                                     float bin_width, uint64_t nbins) {
  std::vector<uint32_t> mask((nbins + 31) / 32, 0u);
  for (size_t i = 0; i < freqs.size() && i < widths.size(); ++i) {
    const float f = freqs[i], w = widths[i];
    long low = static_cast<long>(std::floor((f - w) / bin_width));
    long high = static_cast<long>(std::ceil((f + w) / bin_width));
    if (low < 0) low = 0;
    if (low >= static_cast<long>(nbins)) continue;
    if (high >= static_cast<long>(nbins)) high = static_cast<long>(nbins) - 1;
    for (long k = low; k < high; ++k) mask[static_cast<size_t>(k) >> 5] |= 1u << (k & 31);
  }
  return mask;
}

// ----------------------------------------------------------- search engine --
static int ilog2(uint64_t v) {
  int l = 0;
  while ((uint64_t(1) << (l + 1)) <= v) ++l;
  return l;
}

AccelerationDistiller search_accel_distiller(const SearchParams& p) {
  return AccelerationDistiller(static_cast<float>(static_cast<float>(p.fft_size) * p.tsamp), p.freq_tol, true);
}

SearchEngine::SearchEngine(const SearchParams& p, hipStream_t stream)
    : p_(p),
      stream_(stream),
      harm_(p.freq_tol, static_cast<float>(p.max_harm), false, true),
      accd_(search_accel_distiller(p)) {
  PSOUP_CHECK(p_.fft_size >= 250, "fft_size too small");
  n_ = p_.fft_size;
  nb_ = n_ / 2 + 1;
  tobs_ = static_cast<float>(static_cast<float>(n_) * p_.tsamp);
  bin_width_ = static_cast<float>(1.0 / tobs_);
  nlev_ = std::min(std::max(p_.nharmonics, 0), kern::kMaxHarmLevels);
  if (p_.nharmonics > kern::kMaxHarmLevels)
    log_info("warning: nharmonics > 5 is capped at 5 (32 harmonics), as the reference kernel only writes 5 levels");
  // PSOUP_WHITEN_ROCFFT=1 whitens with rocFFT (the fallback FFT path)
  const char* wr = std::getenv("PSOUP_WHITEN_ROCFFT");
  wh_ = std::make_unique<Whitener>(n_, p_.tsamp, stream_, p_.fft_mode == 2 && !(wr && std::atoi(wr) == 1));
  {
    // whitening batch: up to 3 GB of per-trial whitening state (>= 1 trial)
    const uint64_t per = wh_->batch_bytes_per_trial() + n_ * 4 + (p_.fft_mode == 2 ? n_ * 4 + 4096 : 0);
    max_prep_ = per ? static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(64, (3ull << 30) / per))) : 1;
    // PSOUP_MAX_PREPARE lowers it (tests: chunks of several whitening groups)
    if (const char* e = std::getenv("PSOUP_MAX_PREPARE")) max_prep_ = std::clamp(std::atoi(e), 1, max_prep_);
  }
  tim_.resize(n_);
  wstats_.resize(8 * static_cast<uint64_t>(max_prep_));  // two halves of prepared slots
  mode_ = (n_ % 2 == 0) ? std::min(std::max(p_.fft_mode, 0), 2) : 0;
  if (mode_ == 2) f4_ = kern::fft4_geometry(n_ / 2);
  if (mode_ == 2 && !f4_.ok) {
    // rows too long for the fused passes (2^26 and up): fused resample +
    // pass A over columns of 4096, rocFFT over the rows, then a transposing
    // r2c + interbin + normalise (PSOUP_ROWS_EXT=0: the plain rocFFT path)
    const char* re = std::getenv("PSOUP_ROWS_EXT");
    if (!(re && std::atoi(re) == 0)) f4_ = kern::fft4_geometry_rows(n_ / 2);
    rows_ext_ = f4_.ok;
  }
  if (mode_ == 2 && !f4_.ok) mode_ = 1;
  if (const char* pd = std::getenv("PSOUP_WHITEN_PAD_DIRECT")) pad_direct_ = std::atoi(pd) != 0;
  if (mode_ == 2) {
    auto tab = kern::fft4_tables(f4_);
    f4_tab_.resize(tab.size());
    PSOUP_HIP_CHECK(hipMemcpy(f4_tab_.data(), tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));
    f4_in_.resize(f4_.insize);
  }
  xs_ = mode_ == 2 ? f4_.xstride : nb_;
  if (!p_.zap_freqs.empty()) {
    auto mask = build_zap_mask(p_.zap_freqs, p_.zap_widths, bin_width_, nb_);
    zapmask_.resize(mask.size());
    PSOUP_HIP_CHECK(hipMemcpy(zapmask_.data(), mask.data(), mask.size() * 4, hipMemcpyHostToDevice));
    zap_ = true;
  }
  bounds_.clear();
  hp_.nlevels = nlev_;
  hp_.thresh = p_.min_snr;
  hi_ = 0;
  for (int h = 0; h <= 5; ++h) {
    if (h <= nlev_) {
      PeakBounds b = peak_bounds(static_cast<int>(nb_), bin_width_, h, p_.min_freq, p_.max_freq);
      bounds_.push_back(b);
      hp_.start[h] = b.start_idx;
      hp_.end[h] = std::max(b.start_idx, b.end_idx);
      hi_ = std::max(hi_, hp_.end[h]);
    } else {
      hp_.start[h] = hp_.end[h] = 0;
    }
  }
  // normalised spectra: bins below the search limit only (pass B prunes
  // its stores to the bins the r2c kernel reads for them).  (A pass B fused
  // with r2c + interbin + normalise was measured in round 3 and lost: the
  // harmonic sum reads its blocked layout at 2.1x the cost,
  // profiles/r3_fused/SUMMARY.md.)
  pst_ = std::max<uint64_t>(1, static_cast<uint64_t>(hi_));
  // screened harmonic sum on the bytes the r2c kernel writes (the tiled fused
  // layouts, or the transposing r2c of the external-row path)
  q8_ = mode_ == 2 && (rows_ext_ || kern::fft4_x_layout(f4_).tiled) && !(kern::harmonic_flags() & 4);
  // the fused spectrum pass (harmonic flag 64) writes every bin 0..M of P (blocked) and Q
  fused_ = q8_ && !rows_ext_ && (kern::harmonic_flags() & 64) && f4_.n2 >= 16 && f4_.n1 >= 128;
  fromx_ = q8_ && !fused_ && !rows_ext_ && (kern::harmonic_flags() & 8);
  if (fused_) pst_ = (n_ / 2 + 1 + 63) / 64 * 64;
  if (rows_ext_) pst_ = (pst_ + 63) / 64 * 64;  // 16-byte P / 4-byte Q groups
  qst_ = q8_ ? (pst_ + (fused_ ? kern::kSpecQShift : 0) + 63) / 64 * 64 : 0;
  if (mode_ == 2 && !rows_ext_) rt_ = kern::r2c_twiddle_table(n_ / 2);
  // batch size
  {
    // auto budget: capped by the device's free memory shared among its engines
    size_t budget = p_.batch_bytes;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
      budget = std::min(budget, free_b / 10 * 7 / static_cast<size_t>(std::max(1, p_.engines_per_device)));
    const size_t per = n_ * 4 + (fused_ ? 0 : nb_ * 8) + (fromx_ ? 0 : pst_ * 4) + qst_;  // Y/res + X/spec + P + Q per trial
    // at most 2048 trials per batch (within the budget).  Short series: a
    // list under k_small_ runs as one batch (2^20, 32 DMs x 13 trials: one
    // 416-trial batch 121.5k / 120.4k trials/s vs 256 + 160 114.5k / 116.3k)
    const size_t kmax = 2048;
    auto round_batch = [kmax](size_t k) {
      int K = static_cast<int>(std::min<size_t>(kmax, std::max<size_t>(1, k)));
      if (K >= 32) K = K / 16 * 16;  // halves stay multiples of 8 (XCD-grouped kernels)
      else if (K >= 16) K = K / 8 * 8;
      return K;
    };
    K_ = p_.accel_batch > 0 ? p_.accel_batch : round_batch(budget / per);
    k_small_ = std::min(K_, std::max(16, round_batch(budget / 8 / per)));  // 304 at 2^23
  }
  // Auto: sub-batches on alternating streams, half a batch but at most 2^28
  // samples -- below 2^22 samples only.  At 2^23 they were +4-5% in round 1
  // (20.81k at 16, 20.84k at 32 trials per sub-batch), but with the current
  // passes one stream wins on the same box: K = 256 without sub-batches
  // 21.98k/21.97k vs 21.0k/21.5k/21.5k/21.6k with 16/32/64/128; at 2^22
  // 44.0k vs 42.9k; at 2^20 they still win, 81.0k vs 78.2k
  // (profiles/r3_sub/, profiles/r3_k512/).
  int sub_auto = 0;
  if (K_ >= 16 && n_ < (uint64_t(1) << 22)) {
    const int cap = static_cast<int>(std::max<uint64_t>(8, (uint64_t(1) << 28) / n_)) / 8 * 8;
    sub_auto = std::min(K_ / 2, cap);
  }
  sub_ = mode_ != 2 ? 0 : p_.sub_batch >= 0 ? p_.sub_batch : sub_auto;
  if (sub_ >= K_) sub_ = 0;
  if (sub_ > 0) {  // (only the sub-batch pipeline uses them: a stream is a hardware queue, ~3-7 ms to create)
    const int ns = std::max(2, p_.sub_streams);
    for (int i = 1; i < ns; ++i) {
      aux_.push_back(std::make_unique<Stream>());
      joins_.push_back(std::make_unique<Event>());
    }
  }
  cap_ = static_cast<uint32_t>(std::max<uint64_t>(1u << 16, static_cast<uint64_t>(K_) * 4096));
  if (const char* e = std::getenv("PSOUP_GPU_CLUSTER")) gpu_cluster_ = std::atoi(e) != 0;
  gpu_cluster_ = gpu_cluster_ && p_.min_gap >= 1 && p_.min_gap <= 30;  // the device windows span 32 positions
  // record regions (kern::kPeakRegionStride) where the device clusters the
  // records; the host path and the peak dump read one contiguous run
  if (const char* e = std::getenv("PSOUP_PEAK_REGION_LOG2")) p_.peak_region_log2 = std::atoi(e);
  rlog2_ = gpu_cluster_ && !std::getenv("PSOUP_DUMP_PEAKS") ? std::clamp(p_.peak_region_log2, 0, 8) : 0;
  hp_.region_log2 = rlog2_;
  for (auto& s : slots_) {
    s.done = std::make_unique<Event>();
    s.copied = std::make_unique<Event>();
    // [0] records, [1] cluster peaks, [2] distilled candidates; region counters from [32]
    s.d_count.resize(rlog2_ ? kern::kPeakRegionStride * ((1u << rlog2_) + 1) : 3);
    s.h_count.resize(3);
  }
  // per-trial harmonic distillation on the device: needs the device clusters,
  // the fast relation's tolerance range, and bins that fit the record's 29 bits
  if (const char* e = std::getenv("PSOUP_GPU_DISTILL")) gpu_distill_ = std::atoi(e) != 0;
  gpu_distill_ = gpu_distill_ && gpu_cluster_ && p_.freq_tol <= 1e-3f && nb_ < (uint64_t(1) << 29);
  hdp_.nlevels = nlev_;
  for (int h = 0; h <= nlev_; ++h) hdp_.factor[h] = bounds_[static_cast<size_t>(h)].factor;
  hdp_.tol = p_.freq_tol;
  hdp_.max_harm = static_cast<float>(p_.max_harm);
  hdp_.lower_tol = 1 - hdp_.tol;  // HarmonicDistiller::run: double(1 -/+ float tol)
  hdp_.upper_tol = 1 + hdp_.tol;
  grow_capacity(cap_);
  int ht = p_.host_threads;
  if (const char* e = std::getenv("PSOUP_HOST_THREADS")) ht = std::atoi(e);
  if (ht < 0) ht = static_cast<int>(std::min(4u, std::max(1u, std::thread::hardware_concurrency() / 4)));
  if (ht > 1) pool_ = std::make_unique<HostPool>(ht - 1);
  // acceleration distillation of each DM as its last batch retires, on two
  // workers of their own (none: synchronous, in the calling thread)
  int aw = ht > 1 ? 2 : 0;
  if (const char* e = std::getenv("PSOUP_ACCD_THREADS")) aw = std::max(0, std::atoi(e));
  accq_ = std::make_unique<TaskQueue>(aw);
}

SearchEngine::~SearchEngine() {
  (void)hipStreamSynchronize(stream_);
  (void)hipStreamSynchronize(copy_stream_.get());
}

void SearchEngine::grow_capacity(uint32_t need) {
  // regions of whole 4096-record blocks (the clustering's hist/scatter blocks)
  const uint64_t q = rlog2_ ? uint64_t(4096) << rlog2_ : 1;
  const uint64_t c = (std::max<uint64_t>(cap_, need) + q - 1) / q * q;
  PSOUP_CHECK(c < (uint64_t(1) << 32), "peak record capacity beyond 32-bit positions");
  cap_ = static_cast<uint32_t>(c);
  for (auto& s : slots_) {
    s.d_peaks.resize(cap_);
    if (gpu_cluster_) {
      s.d_sorted.resize(2 * static_cast<size_t>(cap_));  // chunk descriptors, then raw segments' crossings
      s.d_clust.resize(cap_);
      if (gpu_distill_) s.d_hout.resize(cap_);
    }
    // (the pinned host copies grow on demand, to what a batch's counts ask
    // for: sized to the device capacity they were ~48 MB of pinning -- and
    // as much again to free -- per engine, most of a small run's setup)
  }
  hp_.capacity = cap_;
}

namespace {
// pinned host buffer b holds at least n entries (contents not kept)
template <typename T>
void ensure_host(PinnedBuffer<T>& b, size_t n) {
  if (b.size() < n) b.resize(std::max<size_t>(n, std::max<size_t>(2 * b.size(), 1u << 14)));
}
}  // namespace

void SearchEngine::ensure_batch_buffers(int k) {
  // sized for the largest batch actually launched (a short trial list never
  // allocates a whole K_-trial batch)
  if (k <= buf_k_) return;
  buf_k_ = k;
  if (gpu_cluster_)
    for (auto& s : slots_) {
      s.d_work.resize(5 * 8 * static_cast<size_t>(k));
      s.d_segtab.resize(8 * static_cast<size_t>(k));
      s.h_segtab.resize(8 * static_cast<size_t>(k));
      if (gpu_distill_) {
        s.d_ttab.resize(static_cast<size_t>(k));
        s.h_ttab.resize(static_cast<size_t>(k));
      }
    }
  const uint64_t rs = mode_ == 2 ? 2 * f4_.ystride : n_;  // floats per trial
  res_.resize(static_cast<uint64_t>(k) * rs);
  if (!fused_) spec_.resize(static_cast<uint64_t>(k) * xs_);
  if (!fromx_) P_.resize(static_cast<uint64_t>(k) * pst_);
  if (q8_) Q_.resize(static_cast<uint64_t>(k) * qst_);
}

FftPlan& SearchEngine::batch_plan(int count) {
  auto it = plans_.find(count);
  if (it != plans_.end()) return *it->second;
  std::unique_ptr<FftPlan> plan;
  if (mode_ == 1)  // N/2-point complex FFT of the packed real series (post-processing fused downstream)
    plan = std::make_unique<FftPlan>(FftType::C2C_FWD, n_ / 2, static_cast<uint64_t>(count), n_ / 2, nb_);
  else
    plan = std::make_unique<FftPlan>(FftType::R2C, n_, static_cast<uint64_t>(count), n_, nb_);
  FftPlan& ref = *plan;
  plans_[count] = std::move(plan);
  return ref;
}

void SearchEngine::launch_batch(Slot& s, int first, int count) {
  s.first = first;
  s.count = count;
  const uint64_t pst = pst_;
  const kern::Fft4XLayout xl = mode_ == 2 && !rows_ext_ ? kern::fft4_x_layout(f4_)
                                                        : kern::Fft4XLayout{ilog2(n_ / 2), n_ / 2, 8, 3, false};
  // the record counter(s): region r's at rcount(s)[r * kPeakRegionStride]
  PSOUP_HIP_CHECK(hipMemsetAsync(rcount(s), 0, (rlog2_ ? kern::kPeakRegionStride << rlog2_ : 1) * sizeof(uint32_t),
                                 stream_));
  // Trials [b, b + c) of the batch: spectrum, power spectrum, harmonic peaks.
  auto run = [&](int b, int c, hipStream_t st) {
    float* P = fromx_ ? nullptr : P_.data() + static_cast<uint64_t>(b) * pst;
    // (the kernel flags can change after construction: Q only where the tiled r2c writes it)
    uint8_t* Q = q8_ && mode_ == 2 && (xl.tiled || rows_ext_) ? Q_.data() + static_cast<uint64_t>(b) * qst_ : nullptr;
    PSOUP_CHECK(!fromx_ || Q, "fft4 kernel flags changed under an engine that recomputes spectra from X");
    kern::HarmFromX fx;
    if (mode_ == 2) {
      // res_ holds the four-step intermediates Y (complex, ystride per trial)
      float2* Y = reinterpret_cast<float2*>(res_.data()) + static_cast<uint64_t>(b) * f4_.ystride;
      // trial first+b+i resamples prepared series d_src_[first+b+i] and is
      // normalised with that series' whitening stats
      const uint32_t* src = d_src_.data() + first + b;
      kern::Fft4Geom g = f4_;
      g.in_tstride = n_;
      g.pad_tstride = f4_.insize;
      g.tsrc = src;
      g.ypair = fused_ && kern::fft4_pair_y(f4_);
      kern::fft4_resample_colpass(tim_.data(), f4_in_.data(), n_, af_.data() + first + b, c, Y, g, f4_tab_.data(),
                                  st);
      if (fused_) {
        PSOUP_CHECK(Q, "fft4 kernel flags changed under an engine with the fused spectrum pass");
        kern::SpecOut so;
        so.P = P;
        so.pstride = pst;
        so.Q = Q;
        so.qstride = qst_;
        so.stats = wstats_.data();
        so.tsrc = src;
        so.nscale = static_cast<float>(n_);
        so.nbins = static_cast<uint32_t>(hi_);  // the harmonic sum reads no bin at or above hi_
        kern::fft4_rowpass_spectrum(Y, c, g, f4_tab_.data(), so, st);
        fx.pblk = 1;
        fx.qshift = kern::kSpecQShift;
        fx.log2_n2 = ilog2(static_cast<uint64_t>(f4_.n2));
        fx.n1 = static_cast<uint32_t>(f4_.n1);
        RoctxRange r("Harmonic summing");
        kern::HarmParams hp = hp_;
        hp.trial_base = static_cast<uint32_t>(b);
        kern::harmonic_peaks_batch(P, nb_, pst, c, hp, s.d_peaks.data(), rcount(s), st, Q, qst_, &fx);
        return;
      }
      float2* X = spec_.data() + static_cast<uint64_t>(b) * xs_;
      if (rows_ext_) {
        // the rows (n1 >= 8192 points, contiguous in Y) by rocFFT, each row's
        // transform written contiguously (4.3 TB/s at 2^26; a natural-order
        // output stride ran at 1.0: tools/expt/rows_probe.py), then the
        // transposing r2c + interbin + normalise
        if (!rows_plan_)
          rows_plan_ = std::make_unique<FftPlan>(FftType::C2C_FWD, static_cast<uint64_t>(f4_.n1),
                                                 static_cast<uint64_t>(f4_.n2), f4_.ypitch, f4_.xpitch);
        for (int i = 0; i < c; ++i)
          rows_plan_->execute(Y + static_cast<uint64_t>(i) * f4_.ystride, X + static_cast<uint64_t>(i) * xs_, st);
        kern::r2c_interbin_normalise_rows(X, f4_.xpitch, xs_, ilog2(static_cast<uint64_t>(f4_.n2)),
                                          static_cast<uint64_t>(f4_.n1), P, pst, c, static_cast<uint64_t>(hi_),
                                          wstats_.data(), static_cast<float>(n_), st, src, Q, qst_);
        RoctxRange r("Harmonic summing");
        kern::HarmParams hp = hp_;
        hp.trial_base = static_cast<uint32_t>(b);
        kern::harmonic_peaks_batch(P, nb_, pst, c, hp, s.d_peaks.data(), rcount(s), st, Q, qst_, nullptr);
        return;
      }
      kern::fft4_rowpass(Y, X, c, f4_, f4_tab_.data(), st, static_cast<uint64_t>(hi_));
      if (xl.tiled) {
        kern::r2c_interbin_normalise_tiled(X, f4_.n1, f4_.n2, xs_, P, pst, c, static_cast<uint64_t>(hi_),
                                           wstats_.data(), static_cast<float>(n_), st, src, Q, qst_, rt_);
      } else {
        kern::r2c_interbin_normalise_batch(X, n_ / 2, xs_, xl.log2_row, xl.row_pitch, xl.blk_pitch, xl.log2_blk, P,
                                           pst, c, static_cast<uint64_t>(hi_), wstats_.data(),
                                           static_cast<float>(n_), st, src);
      }
      if (fromx_) {
        fx.X = X;
        fx.xstride = xs_;
        fx.log2_n2 = ilog2(static_cast<uint64_t>(f4_.n2));
        fx.n1 = static_cast<uint32_t>(f4_.n1);
        fx.rt = rt_;
        fx.stats = wstats_.data();
        fx.tsrc = src;
        fx.nscale = static_cast<float>(n_);
      }
    } else {
      kern::resample_batch(cur_tim_, n_, res_.data(), n_, af_.data() + first, c, st);
      batch_plan(c).execute(res_.data(), spec_.data(), st);
      if (mode_ == 1)
        kern::r2c_interbin_normalise_batch(spec_.data(), n_ / 2, xs_, xl.log2_row, xl.row_pitch, xl.blk_pitch,
                                           xl.log2_blk, P, pst, c, static_cast<uint64_t>(hi_), cur_stats_,
                                           static_cast<float>(n_), st);
      else
        kern::interbin_normalise_batch(spec_.data(), nb_, nb_, P, pst, c, static_cast<uint64_t>(hi_),
                                       cur_stats_, static_cast<float>(n_), st);
    }
    RoctxRange r("Harmonic summing");
    kern::HarmParams hp = hp_;
    hp.trial_base = static_cast<uint32_t>(b);
    kern::harmonic_peaks_batch(P, nb_, pst, c, hp, s.d_peaks.data(), rcount(s), st, Q, qst_,
                               fromx_ ? &fx : nullptr);
  };
  if (sub_ > 0 && count > sub_) {
    // Sub-batch pipeline: consecutive sub-batches alternate between two
    // streams, so one sub-batch's four kernels run while the other's are in
    // flight and each intermediate (Y, X, P) is re-read soon after it was
    // written, while it is still resident in the 256 MB Infinity Cache.
    fork_.record(stream_);
    for (auto& a : aux_) PSOUP_HIP_CHECK(hipStreamWaitEvent(a->get(), fork_.get(), 0));
    const int ns = static_cast<int>(aux_.size()) + 1;
    for (int b = 0, j = 0; b < count; b += sub_, ++j)
      run(b, std::min(sub_, count - b), j % ns == 0 ? stream_ : aux_[static_cast<size_t>(j % ns - 1)]->get());
    for (size_t i = 0; i < aux_.size(); ++i) {
      joins_[i]->record(aux_[i]->get());
      PSOUP_HIP_CHECK(hipStreamWaitEvent(stream_, joins_[i]->get(), 0));
    }
  } else {
    run(0, count, stream_);
  }
  // d_count[0]: the records held (or, after a region overflowed, the capacity that fits)
  if (rlog2_) kern::peak_regions_total(rcount(s), rlog2_, cap_, s.d_count.data(), stream_);
  if (const char* dump = std::getenv("PSOUP_DUMP_PEAKS")) {
    // diagnostics (tools/expt/cluster_replay.py): the first batch's raw peak
    // records with at least PSOUP_DUMP_PEAKS_MIN of them, for replaying the
    // clustering kernels on real data
    static std::atomic<bool> dumped{false};
    const char* mn = std::getenv("PSOUP_DUMP_PEAKS_MIN");
    uint32_t n = 0;
    PSOUP_HIP_CHECK(hipMemcpyAsync(&n, s.d_count.data(), 4, hipMemcpyDeviceToHost, stream_));
    PSOUP_HIP_CHECK(hipStreamSynchronize(stream_));
    if (n <= cap_ && n >= static_cast<uint32_t>(mn ? std::atoi(mn) : 1) && !dumped.exchange(true)) {
      std::vector<kern::PeakRecord> h(n);
      PSOUP_HIP_CHECK(hipMemcpy(h.data(), s.d_peaks.data(), n * sizeof(kern::PeakRecord), hipMemcpyDeviceToHost));
      if (FILE* f = std::fopen(dump, "wb")) {
        const uint32_t hdr[3] = {static_cast<uint32_t>(count) * 8, static_cast<uint32_t>(p_.min_gap), n};
        std::fwrite(hdr, 4, 3, f);
        std::fwrite(h.data(), sizeof(kern::PeakRecord), n, f);
        std::fclose(f);
      }
    }
  }
  if (gpu_cluster_) {
    // cluster on the device: only cluster peaks (and the rare over-capacity
    // segment's raw crossings) are copied out
    kern::peak_cluster_batch(s.d_peaks.data(), rcount(s), cap_, static_cast<uint32_t>(count) * 8, p_.min_gap,
                             s.d_work.data(), s.d_sorted.data(), s.d_clust.data(), s.d_segtab.data(),
                             s.d_count.data() + 1, stream_, rlog2_);
    PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_segtab.data(), s.d_segtab.data(), 8ull * count * sizeof(uint2),
                                   hipMemcpyDeviceToHost, stream_));
    if (gpu_distill_) {
      // per-trial harmonic distillation of the cluster peaks: only the
      // distilled candidates (and the rare host-flagged trials' peaks) go out
      kern::harm_distill_batch(s.d_clust.data(), s.d_segtab.data(), count, hdp_, s.d_hout.data(), s.d_ttab.data(),
                               s.d_count.data() + 2, stream_);
      PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_ttab.data(), s.d_ttab.data(), static_cast<size_t>(count) * sizeof(uint2),
                                     hipMemcpyDeviceToHost, stream_));
    }
  }
  PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_count.data(), s.d_count.data(), 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
  s.done->record(stream_);
}

void SearchEngine::process_slot(Slot& s, int first, int count, uint32_t npeaks,
                                std::vector<CandidateList>& out_by_job) {
  const uint32_t cnt = std::min(npeaks, cap_);
  ctr_.peaks += cnt;
  const int nseg = count * 8;
  seg_count_.assign(static_cast<size_t>(nseg) + 1, 0);
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint32_t seg = s.h_peaks[i].seg;
    if (seg & kern::kPeakChunk) continue;  // chunk descriptor (device clustering only)
    PSOUP_CHECK(seg < static_cast<uint32_t>(nseg), "peak record outside its batch (segment " << seg << ")");
    seg_count_[seg]++;
  }
  seg_off_.assign(static_cast<size_t>(nseg) + 1, 0);
  for (int i = 0; i < nseg; ++i) seg_off_[i + 1] = seg_off_[i] + seg_count_[i];
  sorted_.resize(cnt);
  {
    std::vector<uint32_t> fill(seg_off_.begin(), seg_off_.end() - 1);
    for (uint32_t i = 0; i < cnt; ++i)
      if (!(s.h_peaks[i].seg & kern::kPeakChunk)) sorted_[fill[s.h_peaks[i].seg]++] = s.h_peaks[i];
  }
  // Per-trial clustering + harmonic distillation.  Trials own disjoint
  // segments of sorted_, so peak-heavy batches (RFI) are spread over the
  // host pool; results are concatenated in trial order (deterministic).
  build_trials(first, count, cnt, [&](int k, int h, std::vector<int>& pidx, std::vector<float>& psnr) {
    thread_local std::vector<int> idxs;
    thread_local std::vector<float> snrs;
    const int seg = k * 8 + h;
    const uint32_t a = seg_off_[seg], b = seg_off_[seg + 1];
    if (a == b) return;
    std::sort(sorted_.begin() + a, sorted_.begin() + b,
              [](const kern::PeakRecord& x, const kern::PeakRecord& y) { return x.idx < y.idx; });
    idxs.resize(b - a);
    snrs.resize(b - a);
    for (uint32_t i = a; i < b; ++i) {
      idxs[i - a] = sorted_[i].idx;
      snrs[i - a] = sorted_[i].snr;
    }
    identify_unique_peaks(idxs.data(), snrs.data(), idxs.size(), p_.min_gap, pidx, psnr);
  }, out_by_job);
}

void SearchEngine::process_clustered(Slot& s, int first, int count, const std::vector<uint2>& segtab,
                                     const std::vector<uint2>* ttab, std::vector<CandidateList>& out_by_job) {
  size_t work = 0;
  for (int k = 0; k < count; ++k) {
    if (ttab && !((*ttab)[static_cast<size_t>(k)].y & kern::kHarmHost)) {
      work += (*ttab)[static_cast<size_t>(k)].y / 8;  // building the distilled list only
      continue;
    }
    for (int h = 0; h < 8; ++h) work += segtab[static_cast<size_t>(k) * 8 + h].y & ~kern::kClusterRaw;
  }
  // a device-distilled trial's list: {idx | level << 29, snr} in S/N order
  const std::function<bool(int, CandidateList&)> distilled = [&](int k, CandidateList& trial) {
    const uint2 e = (*ttab)[static_cast<size_t>(k)];
    if (e.y & kern::kHarmHost) return false;
    const size_t ft = static_cast<size_t>(first + k);
    const float acc = flat_acc_[ft];
    const Job& job = (*jobs_)[static_cast<size_t>(flat_job_[ft])];
    trial.reserve(e.y);
    for (uint32_t i = 0; i < e.y; ++i) {
      const uint2 v = s.h_hout[e.x + i];
      const int h = static_cast<int>(v.x >> 29);
      const int idx = static_cast<int>(v.x & ((1u << 29) - 1));
      float snr;
      std::memcpy(&snr, &v.y, 4);
      trial.emplace_back(job.dm, job.dm_idx, acc, h, snr,
                         static_cast<float>(idx * bounds_[static_cast<size_t>(h)].factor));
    }
    return true;
  };
  build_trials(first, count, work, [&](int k, int h, std::vector<int>& pidx, std::vector<float>& psnr) {
    const uint2 e = segtab[static_cast<size_t>(k * 8 + h)];
    if (e.y == 0) return;
    if (e.y & kern::kClusterRaw) {
      // a segment over the device's LDS capacity: the reference scan here
      thread_local std::vector<std::pair<int, float>> raw;
      thread_local std::vector<int> idxs;
      thread_local std::vector<float> snrs;
      const uint32_t n = e.y & ~kern::kClusterRaw;
      raw.resize(n);
      for (uint32_t i = 0; i < n; ++i) {
        const uint2 v = s.h_raw[e.x + i];
        float f;
        std::memcpy(&f, &v.y, 4);
        raw[i] = {static_cast<int>(v.x), f};
      }
      std::sort(raw.begin(), raw.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      idxs.resize(n);
      snrs.resize(n);
      for (uint32_t i = 0; i < n; ++i) {
        idxs[i] = raw[i].first;
        snrs[i] = raw[i].second;
      }
      identify_unique_peaks(idxs.data(), snrs.data(), n, p_.min_gap, pidx, psnr);
      return;
    }
    pidx.resize(e.y);
    psnr.resize(e.y);
    for (uint32_t i = 0; i < e.y; ++i) {
      const uint2 v = s.h_clust[e.x + i];
      pidx[i] = static_cast<int>(v.x);
      std::memcpy(&psnr[i], &v.y, 4);
    }
  }, out_by_job, ttab ? &distilled : nullptr);
}

void SearchEngine::build_trials(int first, int count, size_t work,
                                const std::function<void(int, int, std::vector<int>&, std::vector<float>&)>& peaks_of,
                                std::vector<CandidateList>& out_by_job,
                                const std::function<bool(int, CandidateList&)>* distilled) {
  const int L = nlev_ + 1;
  // per-trial results, appended to their jobs' lists in trial order below
  std::vector<CandidateList> per_trial(static_cast<size_t>(count));
  std::atomic<uint64_t> harm_in{0}, on_gpu{0};
  auto trial_range = [&](int k0, int k1) {
    std::vector<int> pidx;
    std::vector<float> psnr;
    for (int k = k0; k < k1; ++k) {
      if (distilled && (*distilled)(k, per_trial[static_cast<size_t>(k)])) {
        on_gpu++;
        continue;
      }
      const size_t ft = static_cast<size_t>(first + k);
      const float acc = flat_acc_[ft];
      const Job& job = (*jobs_)[static_cast<size_t>(flat_job_[ft])];
      const float dm = job.dm;
      const int dm_idx = job.dm_idx;
      CandidateList trial;
      for (int h = 0; h < L; ++h) {
        pidx.clear();
        psnr.clear();
        peaks_of(k, h, pidx, psnr);
        const double factor = bounds_[static_cast<size_t>(h)].factor;
        for (size_t i = 0; i < pidx.size(); ++i)
          trial.emplace_back(dm, dm_idx, acc, h, psnr[i], static_cast<float>(pidx[i] * factor));
      }
      harm_in += trial.size();
      if (!trial.empty()) per_trial[static_cast<size_t>(k)] = harm_.distill(std::move(trial));
    }
  };
  constexpr size_t kParallelPeaks = 8192;  // below this the serial loop is cheaper
  if (pool_ && work >= kParallelPeaks && count > 1) {
    const int nparts = std::min(count, 4 * pool_->size());
    pool_->parallel_for(nparts, [&](int j) {
      const int k0 = static_cast<int>(static_cast<int64_t>(count) * j / nparts);
      const int k1 = static_cast<int>(static_cast<int64_t>(count) * (j + 1) / nparts);
      trial_range(k0, k1);
    });
  } else {
    trial_range(0, count);
  }
  for (int k = 0; k < count; ++k) {
    CandidateList& dst = out_by_job[static_cast<size_t>(flat_job_[static_cast<size_t>(first + k)])];
    ctr_.harm_out += per_trial[static_cast<size_t>(k)].size();
    for (auto& c : per_trial[static_cast<size_t>(k)]) dst.push_back(std::move(c));
  }
  ctr_.harm_in += harm_in.load();
  ctr_.gpu_distilled += on_gpu.load();
  ctr_.host_distilled += static_cast<uint64_t>(count) - on_gpu.load();
}

void SearchEngine::prepare(const uint8_t* d_trials, uint64_t row_stride, uint64_t nsamps, int count, int first) {
  PSOUP_CHECK(count >= 1 && count <= max_prep_, "prepare: count " << count << " outside [1, " << max_prep_ << "]");
  PSOUP_CHECK(first == 0 || first == max_prep_, "prepare: first slot " << first << " (0 or max_prepare)");
  RoctxRange r("Whitening");
  // first == 0: the previous searches have retired (search_prepared waits on
  // every acceleration batch), so the buffers may be rewritten (and grown);
  // first == max_prepare: the other half of a reserve(.., two = true) layout,
  // written while the first half's search may still be in flight (the
  // kernels run after it in stream order; nothing is reallocated)
  const uint64_t end = static_cast<uint64_t>(first) + static_cast<uint64_t>(count);
  if (first == 0) {  // grow only: a reserve(.., two = true) keeps its second half
    if (tim_.size() < n_ * end) tim_.resize(n_ * end);
    if (mode_ == 2 && f4_in_.size() < f4_.insize * end) f4_in_.resize(f4_.insize * end);
  }
  PSOUP_CHECK(tim_.size() >= n_ * end && (mode_ != 2 || f4_in_.size() >= f4_.insize * end),
              "prepare: the second half of the prepared slots needs reserve(count, trials, true)");
  float* tim = tim_.data() + static_cast<uint64_t>(first) * n_;
  float* pad = mode_ == 2 ? f4_in_.data() + static_cast<uint64_t>(first) * f4_.insize : nullptr;
  // the padded rows of pass A's input written by the whitener's last kernel
  // (no unpadded copy and no pad kernel) where the layouts allow it
  pad_only_ = wh_->whiten_batch(d_trials, row_stride, nsamps, count, tim, n_, zap_ ? zapmask_.data() : nullptr,
                                wstats_.data() + 4 * static_cast<uint64_t>(first), p_.boundary_5_freq,
                                p_.boundary_25_freq, pad_direct_ ? pad : nullptr, &f4_, f4_.insize);
  if (mode_ == 2 && !pad_only_) kern::fft4_pad_input(tim, n_, pad, f4_, stream_, count, n_);
  prepared_ = static_cast<int>(end);
}

void SearchEngine::copy_whitened(float* dst) const {
  if (!pad_only_) {
    PSOUP_HIP_CHECK(hipMemcpy(dst, cur_tim_, n_ * sizeof(float), hipMemcpyDeviceToDevice));
    return;
  }
  // rows of 2 n1 floats at pitch inpitch
  const uint64_t row = 2 * static_cast<uint64_t>(f4_.n1);
  PSOUP_HIP_CHECK(hipMemcpy2D(dst, row * sizeof(float), cur_pad_, f4_.inpitch * sizeof(float), row * sizeof(float),
                              static_cast<size_t>(f4_.n2), hipMemcpyDeviceToDevice));
}

CandidateList SearchEngine::search_trial(const uint8_t* d_trial, uint64_t nsamps, float dm, int dm_idx,
                                         const std::vector<float>& accs) {
  prepare(d_trial, 0, nsamps, 1);
  return search_prepared(0, dm, dm_idx, accs);
}

CandidateList SearchEngine::search_prepared(int b, float dm, int dm_idx, const std::vector<float>& accs) {
  std::vector<Job> jobs(1);
  jobs[0] = Job{b, dm, dm_idx, accs};
  return std::move(search_prepared_many(jobs)[0]);
}

int SearchEngine::batch_for(int ntr) const {
  // Short trial lists (one DM at 2^23: 685 trials) keep at least min_batches
  // (SearchParams::min_batches, default 4) batches in the two-slot pipeline so
  // host clustering still overlaps the GPU, but never fall below k_small_
  // (the batch an eighth of the budget gives: 304 at 2^23 with the default
  // 128 GiB, rounded like K_).
  const int min_batches = std::max(1, p_.min_batches);
  if (p_.accel_batch <= 0 && ntr < min_batches * K_) {
    const int even = (ntr + min_batches - 1) / min_batches;
    return std::min(K_, std::max(k_small_, (even + 7) / 8 * 8));
  }
  return K_;
}

void SearchEngine::reserve(int count, int trials, bool two) {
  count = std::max(1, std::min(count, max_prep_));
  const uint64_t slots = two ? 2 * static_cast<uint64_t>(max_prep_) : static_cast<uint64_t>(count);
  if (tim_.size() < n_ * slots) tim_.resize(n_ * slots);  // grow only
  wh_->reserve_batch(count);
  if (mode_ == 2 && f4_in_.size() < f4_.insize * slots) f4_in_.resize(f4_.insize * slots);
  if (trials > 0) ensure_batch_buffers(std::min(batch_for(trials), trials));
}

std::vector<CandidateList> SearchEngine::search_prepared_many(const std::vector<Job>& jobs) {
  return collect(search_prepared_many_async(jobs));
}

std::vector<CandidateList> SearchEngine::collect(const std::shared_ptr<Pending>& pd) {
  Stopwatch w;
  w.start();
  std::unique_lock<std::mutex> lk(pd->mu);
  pd->cv.wait(lk, [&] { return pd->remaining == 0; });
  w.stop();
  ctr_.tail_s += w.get_time();
  if (pd->err) std::rethrow_exception(pd->err);
  for (double t : pd->accd_t) ctr_.accd_s += t;
  ctr_.accel_s += pd->accel_s + w.get_time();
  return std::move(pd->out);
}

std::shared_ptr<SearchEngine::Pending> SearchEngine::search_prepared_many_async(const std::vector<Job>& jobs) {
  auto pd = search_launch(jobs);
  search_finish(pd);
  return pd;
}

void SearchEngine::send_done(const std::shared_ptr<Pending>& pd, int processed) {
  const int njobs = static_cast<int>(pd->jobs.size());
  while (pd->jobs_sent < njobs && pd->job_end[static_cast<size_t>(pd->jobs_sent)] <= processed) {
    const int j = pd->jobs_sent++;
    if (pd->jobs[static_cast<size_t>(j)].raw) {  // a slice: distilled once the slices are joined
      pd->out[static_cast<size_t>(j)] = std::move(pd->by_job[static_cast<size_t>(j)]);
      continue;
    }
    {
      std::lock_guard<std::mutex> lk(pd->mu);
      pd->remaining++;
    }
    accq_->submit([this, j, pd] {
      Stopwatch w;
      w.start();
      std::exception_ptr err;
      try {
        pd->out[static_cast<size_t>(j)] = accd_.distill(std::move(pd->by_job[static_cast<size_t>(j)]));
      } catch (...) {
        err = std::current_exception();
      }
      w.stop();
      std::lock_guard<std::mutex> lk(pd->mu);
      pd->accd_t[static_cast<size_t>(j)] = w.get_time();
      if (err && !pd->err) pd->err = err;
      if (--pd->remaining == 0) pd->cv.notify_all();
    });
  }
}

std::shared_ptr<SearchEngine::Pending> SearchEngine::search_launch(const std::vector<Job>& jobs_in) {
  PSOUP_CHECK(!open_, "search_launch: the previous launch has not been finished (search_finish)");
  RoctxRange dm_range("DM-Loop");
  auto pd = std::make_shared<Pending>();
  pd->sw.start();
  pd->jobs = jobs_in;  // owned: the batches are processed after this call returns
  const std::vector<Job>& jobs = pd->jobs;
  const int njobs = static_cast<int>(jobs.size());
  pd->out.resize(static_cast<size_t>(njobs));
  pd->by_job.resize(static_cast<size_t>(njobs));
  pd->accd_t.assign(static_cast<size_t>(njobs), 0.0);
  std::vector<CandidateList>& by_job = pd->by_job;
  if (njobs == 0) return pd;
  if (mode_ != 2 && njobs > 1) {
    // the rocFFT paths resample one series per batch: one job at a time
    for (int j = 0; j < njobs; ++j) {
      const std::vector<Job> one(1, jobs[static_cast<size_t>(j)]);
      pd->out[static_cast<size_t>(j)] = std::move(search_prepared_many(one)[0]);
    }
    return pd;
  }
  // flat trial list: job j's trials in order, jobs in order
  flat_job_.clear();
  flat_acc_.clear();
  flat_src_.clear();
  af_host_.clear();
  for (int j = 0; j < njobs; ++j) {
    const Job& jb = jobs[static_cast<size_t>(j)];
    PSOUP_CHECK(jb.b >= 0 && jb.b < prepared_, "search_prepared: trial " << jb.b << " was not prepared");
    for (float a : jb.accs) {
      flat_job_.push_back(j);
      flat_acc_.push_back(a);
      flat_src_.push_back(static_cast<uint32_t>(jb.b));
      af_host_.push_back((static_cast<double>(a) * p_.tsamp) / (2 * kC));
    }
  }
  ctr_.dm_trials += static_cast<uint64_t>(njobs);
  const Job& j0 = jobs[0];
  cur_tim_ = tim_.data() + static_cast<uint64_t>(j0.b) * n_;
  cur_pad_ = mode_ == 2 ? f4_in_.data() + static_cast<uint64_t>(j0.b) * f4_.insize : nullptr;
  cur_stats_ = wstats_.data() + 4 * static_cast<uint64_t>(j0.b);
  const int ntr = static_cast<int>(flat_acc_.size());
  if (ntr == 0) return pd;
  jobs_ = &pd->jobs;
  // previous batches have all retired (their events were waited on), so the
  // device copies of the trial tables may be rewritten
  af_.resize(af_host_.size());
  d_src_.resize(flat_src_.size());
  PSOUP_HIP_CHECK(hipMemcpyAsync(af_.data(), af_host_.data(), af_host_.size() * sizeof(double),
                                 hipMemcpyHostToDevice, stream_));
  PSOUP_HIP_CHECK(hipMemcpyAsync(d_src_.data(), flat_src_.data(), flat_src_.size() * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, stream_));
  RoctxRange acc_range("Acceleration-Loop");
  // Acceleration distillation (pipeline_multi.cu:243) of each DM as soon as
  // the batch holding its last trial has been processed, on accq_'s workers
  // while the GPU runs the next batches; the tasks own their data through
  // the Pending record, so the last DMs' distillation may outlive this call
  // (collect() waits for it).
  pd->job_end.resize(static_cast<size_t>(njobs));
  for (int j = 0, e = 0; j < njobs; ++j)
    pd->job_end[static_cast<size_t>(j)] = e += static_cast<int>(jobs[static_cast<size_t>(j)].accs.size());
  send_done(pd, 0);
  std::deque<int>& inflight = pd->inflight;  // slot indices
  int& next = pd->next;
  int slot = slot_next_;
  // Short trial lists (one DM at 2^23: 685 trials) keep at least min_batches
  // (SearchParams::min_batches, default 4) batches in the two-slot pipeline so
  // host clustering still overlaps the GPU, but never fall below k_small_
  // (the batch an eighth of the budget gives: 304 at 2^23 with the default
  // 128 GiB, rounded like K_).
  const int kc = batch_for(ntr);
  last_kc_ = kc;
  pd->kc = kc;
  pd->ntr = ntr;
  ensure_batch_buffers(std::min(kc, ntr));
  while (inflight.size() < 2 && next < ntr) {
    issue_batch(*pd, slot);
    slot ^= 1;
  }
  slot_next_ = slot;
  pd->open = true;
  open_ = true;
  pd->launch_s = pd->sw.get_time();
  return pd;
}

void SearchEngine::issue_batch(Pending& pd, int sl) {
  const int c = std::min(pd.kc, pd.ntr - pd.next);
  launch_batch(slots_[sl], pd.next, c);
  pd.inflight.push_back(sl);
  pd.next += c;
}

void SearchEngine::search_finish(const std::shared_ptr<Pending>& pd) {
  if (!pd->open) {  // nothing deferred (an empty list, or the rocFFT paths' job-by-job search)
    pd->accel_s = pd->sw.get_time();
    return;
  }
  pd->open = false;
  open_ = false;
  Stopwatch fsw;
  fsw.start();
  RoctxRange acc_range("Acceleration-Loop");
  std::vector<CandidateList>& by_job = pd->by_job;
  std::deque<int>& inflight = pd->inflight;
  const int ntr = pd->ntr;
  jobs_ = &pd->jobs;
  Stopwatch host;
  while (!inflight.empty()) {
    const int sl = inflight.front();
    Slot& s = slots_[sl];
    s.done->sync();
    uint32_t cnt = s.h_count[0];
    if (cnt > cap_) {
      // Peak buffer overflow: drain, grow, recompute every in-flight batch.
      ctr_.overflows++;
      PSOUP_HIP_CHECK(hipStreamSynchronize(stream_));
      uint32_t need = cnt;
      for (int q : inflight) need = std::max(need, slots_[q].h_count[0]);
      grow_capacity(need + need / 2 + 1024);
      for (int q : inflight) launch_batch(slots_[q], slots_[q].first, slots_[q].count);
      continue;
    }
    inflight.pop_front();
    // The batch's identity: the slot is re-issued below (launch_batch
    // overwrites first/count/h_count) before its records are processed.
    const int b_first = s.first, b_count = s.count;
    if (gpu_cluster_) {
      // snapshot the segment table (the re-issued launch rewrites it) and
      // copy the cluster peaks plus any raw over-capacity segments
      segtab_.assign(s.h_segtab.data(), s.h_segtab.data() + 8 * static_cast<size_t>(b_count));
      // host copies sized to this batch (the slot's previous copies retired:
      // s.copied was waited on before its records were processed)
      if (gpu_distill_) ttab_.assign(s.h_ttab.data(), s.h_ttab.data() + b_count);
      {
        size_t n_raw = 0, n_clust = gpu_distill_ ? 0 : s.h_count[1];
        for (int k = 0; k < b_count; ++k) {
          // with device distillation only the host-flagged trials' segments come out
          if (gpu_distill_ && !(ttab_[static_cast<size_t>(k)].y & kern::kHarmHost)) continue;
          for (int h = 0; h < 8; ++h) {
            const uint2& e = segtab_[static_cast<size_t>(k) * 8 + h];
            if (e.y & kern::kClusterRaw)
              n_raw = std::max<size_t>(n_raw, static_cast<size_t>(e.x) + (e.y & ~kern::kClusterRaw));
            else
              n_clust = std::max<size_t>(n_clust, static_cast<size_t>(e.x) + e.y);
          }
        }
        ensure_host(s.h_raw, n_raw);
        ensure_host(s.h_clust, n_clust);
        if (gpu_distill_) ensure_host(s.h_hout, s.h_count[2]);
      }
      auto copy_seg = [&](const uint2& e) {
        if (e.y & kern::kClusterRaw)
          PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_raw.data() + e.x, s.d_sorted.data() + cap_ + e.x,
                                         (e.y & ~kern::kClusterRaw) * sizeof(uint2), hipMemcpyDeviceToHost,
                                         copy_stream_.get()));
        else if (e.y > 0)
          PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_clust.data() + e.x, s.d_clust.data() + e.x, e.y * sizeof(uint2),
                                         hipMemcpyDeviceToHost, copy_stream_.get()));
      };
      if (gpu_distill_) {
        // the distilled candidates, plus the cluster peaks of the trials the
        // device left to the host
        const uint32_t tot2 = s.h_count[2];
        if (tot2 > 0)
          PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_hout.data(), s.d_hout.data(), tot2 * sizeof(uint2),
                                         hipMemcpyDeviceToHost, copy_stream_.get()));
        // the host trials' cluster segments: one copy of their hull when
        // there are more than a few (each copy is a blit launch; peak-heavy
        // batches left ~40 trials x 4 levels to the host)
        uint64_t lo = ~0ull, hi = 0;
        int nseg_h = 0;
        for (int k = 0; k < b_count; ++k)
          if (ttab_[static_cast<size_t>(k)].y & kern::kHarmHost)
            for (int h = 0; h <= nlev_; ++h) {
              const uint2& e = segtab_[static_cast<size_t>(k) * 8 + h];
              if (e.y & kern::kClusterRaw) {
                copy_seg(e);
              } else if (e.y > 0) {
                lo = std::min<uint64_t>(lo, e.x);
                hi = std::max<uint64_t>(hi, static_cast<uint64_t>(e.x) + e.y);
                ++nseg_h;
              }
            }
        if (nseg_h > 4) {
          PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_clust.data() + lo, s.d_clust.data() + lo, (hi - lo) * sizeof(uint2),
                                         hipMemcpyDeviceToHost, copy_stream_.get()));
        } else if (nseg_h > 0) {
          for (int k = 0; k < b_count; ++k)
            if (ttab_[static_cast<size_t>(k)].y & kern::kHarmHost)
              for (int h = 0; h <= nlev_; ++h) {
                const uint2& e = segtab_[static_cast<size_t>(k) * 8 + h];
                if (!(e.y & kern::kClusterRaw)) copy_seg(e);
              }
        }
      } else {
        const uint32_t tot = s.h_count[1];
        if (tot > 0)
          PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_clust.data(), s.d_clust.data(), tot * sizeof(uint2),
                                         hipMemcpyDeviceToHost, copy_stream_.get()));
        for (const uint2& e : segtab_)
          if (e.y & kern::kClusterRaw) copy_seg(e);
      }
    } else if (cnt > 0) {
      ensure_host(s.h_peaks, cnt);
      PSOUP_HIP_CHECK(hipMemcpyAsync(s.h_peaks.data(), s.d_peaks.data(), cnt * sizeof(kern::PeakRecord),
                                     hipMemcpyDeviceToHost, copy_stream_.get()));
    }
    s.copied->record(copy_stream_.get());
    // the next batch that reuses this slot must wait for the copy-out
    PSOUP_HIP_CHECK(hipStreamWaitEvent(stream_, s.copied->get(), 0));
    if (pd->next < ntr) issue_batch(*pd, sl);
    s.copied->sync();
    host.start();
    if (gpu_cluster_) {
      ctr_.peaks += std::min(cnt, cap_);
      process_clustered(s, b_first, b_count, segtab_, gpu_distill_ ? &ttab_ : nullptr, by_job);
    } else {
      process_slot(s, b_first, b_count, cnt, by_job);
    }
    host.stop();
    ctr_.accel_trials += static_cast<uint64_t>(b_count);
    send_done(pd, b_first + b_count);
  }
  ctr_.host_s += host.get_time();
  send_done(pd, ntr);
  jobs_ = nullptr;
  fsw.stop();
  pd->accel_s = pd->launch_s + fsw.get_time();
}

// ---------------------------------------------------------------- folding ---
void fold_calculate_sn(const float* prof, int bin, int width, int nbins, float* sn1, float* sn2) {
  const int edge = static_cast<int>(width * 0.3 + 0.5);
  const int width_by_2 = static_cast<int>(width / 2.0 + 0.5);
  std::vector<float> on_pulse, off_pulse, rprof;
  for (int ii = 0; ii < nbins; ++ii) {
    int jj = ((bin - nbins / 2 + ii) % nbins + nbins) % nbins;
    rprof.push_back(prof[jj]);
  }
  bin = nbins / 2 - 1;
  const int upper_edge = bin + (width_by_2 + edge);
  const int lower_edge = bin - (width_by_2 + edge);
  for (int ii = 0; ii < nbins; ++ii) {
    if (ii <= upper_edge && ii >= lower_edge) on_pulse.push_back(rprof[ii]);
    else off_pulse.push_back(rprof[ii]);
  }
  auto mean_of = [](const std::vector<float>& v) -> float {
    if (v.empty()) return std::nanf("");
    double a = 0.0;  // std::accumulate(..., 0.0) accumulates in double
    for (float x : v) a += x;
    return static_cast<float>(a / v.size());
  };
  const float on_mean = mean_of(on_pulse);
  const float off_mean = mean_of(off_pulse);
  float acc = 0;
  for (float x : off_pulse) acc = static_cast<float>(acc + std::pow(x - off_mean, 2.0));
  const float off_std = std::sqrt(acc / off_pulse.size());
  *sn1 = static_cast<float>((on_mean - off_mean) * std::sqrt(static_cast<double>(width)) / off_std);
  double tot = 0.0;
  for (int ii = 0; ii < nbins; ++ii) {
    float v = rprof[ii] - off_mean;
    v = v / off_std;
    tot += v;
  }
  *sn2 = static_cast<float>(tot / std::sqrt(static_cast<double>(width)));
  if (*sn1 > 99999) *sn1 = 0.0f;
  if (*sn2 > 99999) *sn2 = 0.0f;
}

FoldEngine::FoldEngine(uint64_t nsamps, float tsamp, hipStream_t stream) : n_(nsamps), tsamp_(tsamp), stream_(stream) {
  PSOUP_CHECK(n_ >= 1024, "fold series too short");
  wh_ = std::make_unique<Whitener>(n_, tsamp_, stream_);
  // whitening batch: up to ~2 GB of per-trial state, at most 64 trials
  const uint64_t per = wh_->batch_bytes_per_trial() + n_ * 4;
  max_batch_ = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(64, (2ull << 30) / std::max<uint64_t>(1, per))));
  tim_.resize(n_);
  shift_table_.resize(static_cast<uint64_t>(kNbins) * kNbins * kNints);
  kern::fold_shift_table(shift_table_.data(), kNbins, kNints, stream_);
  chunk_ = static_cast<int>(std::min<uint64_t>(4096, n_ / kNints));
}

std::vector<FoldResult> FoldEngine::fold_trial(const uint8_t* d_trial, uint64_t trial_nsamps,
                                               const std::vector<double>& periods, const std::vector<float>& accs) {
  wh_->load_trial(d_trial, trial_nsamps, tim_.data());
  wh_->whiten(tim_.data(), nullptr, false, 0.05f, 0.5f);
  return fold_series(tim_.data(), periods, accs);
}

std::vector<std::vector<FoldResult>> FoldEngine::fold_trials(const uint8_t* d_trials, uint64_t row_stride,
                                                             uint64_t trial_nsamps, int ntrials,
                                                             const std::vector<std::vector<double>>& periods,
                                                             const std::vector<std::vector<float>>& accs) {
  PSOUP_CHECK(ntrials >= 0 && static_cast<int>(periods.size()) == ntrials && static_cast<int>(accs.size()) == ntrials,
              "fold_trials: one candidate list per trial");
  std::vector<std::vector<FoldResult>> out(static_cast<size_t>(ntrials));
  for (int t0 = 0; t0 < ntrials; t0 += max_batch_) {
    const int cnt = std::min(max_batch_, ntrials - t0);
    tim_.resize(static_cast<uint64_t>(cnt) * n_);
    bstats_.resize(4 * static_cast<uint64_t>(cnt));
    // the fold's whitening: no zap mask, default boundaries (pipeline_multi.cu
    // ignores --boundary_*), stats unused
    wh_->whiten_batch(d_trials + static_cast<uint64_t>(t0) * row_stride, row_stride, trial_nsamps, cnt, tim_.data(),
                      n_, nullptr, bstats_.data(), 0.05f, 0.5f);
    std::vector<kern::FoldJob> jobs;
    std::vector<double> ps;
    for (int t = 0; t < cnt; ++t) {
      const auto& P = periods[static_cast<size_t>(t0 + t)];
      const auto& A = accs[static_cast<size_t>(t0 + t)];
      PSOUP_CHECK(P.size() == A.size(), "fold_trials: periods/accs size mismatch");
      for (size_t i = 0; i < P.size(); ++i) {
        kern::FoldJob j;
        j.tsamp_by_period = static_cast<double>(tsamp_) / P[i];
        j.af = (static_cast<double>(A[i]) * tsamp_) / (2 * kC);
        j.series = static_cast<uint64_t>(t);
        jobs.push_back(j);
        ps.push_back(P[i]);
      }
    }
    std::vector<FoldResult> r = fold_jobs(tim_.data(), jobs, ps);
    size_t k = 0;
    for (int t = 0; t < cnt; ++t)
      for (size_t i = 0; i < periods[static_cast<size_t>(t0 + t)].size(); ++i)
        out[static_cast<size_t>(t0 + t)].push_back(std::move(r[k++]));
  }
  return out;
}

std::vector<std::vector<FoldResult>> FoldEngine::fold_rows(const std::vector<const uint8_t*>& rows,
                                                           uint64_t trial_nsamps,
                                                           const std::vector<std::vector<double>>& periods,
                                                           const std::vector<std::vector<float>>& accs) {
  const int ntrials = static_cast<int>(rows.size());
  PSOUP_CHECK(static_cast<int>(periods.size()) == ntrials && static_cast<int>(accs.size()) == ntrials,
              "fold_rows: one candidate list per row");
  const uint64_t rstride = (trial_nsamps + 255) / 256 * 256;
  std::vector<std::vector<FoldResult>> out;
  out.reserve(static_cast<size_t>(ntrials));
  for (int t0 = 0; t0 < ntrials; t0 += max_batch_) {
    const int cnt = std::min(max_batch_, ntrials - t0);
    gathered_.resize(rstride * static_cast<uint64_t>(max_batch_));
    kern::gather_rows(rows.data() + t0, cnt, rstride, gathered_.data(), rstride, stream_);
    std::vector<std::vector<double>> p(periods.begin() + t0, periods.begin() + t0 + cnt);
    std::vector<std::vector<float>> a(accs.begin() + t0, accs.begin() + t0 + cnt);
    auto r = fold_trials(gathered_.data(), rstride, trial_nsamps, cnt, p, a);
    for (auto& x : r) out.push_back(std::move(x));
  }
  return out;
}

void FoldEngine::reserve(int njobs_hint) {
  const int b = max_batch_;
  wh_->reserve_batch(b);
  tim_.resize(static_cast<uint64_t>(b) * n_);
  bstats_.resize(4 * static_cast<uint64_t>(b));
  const uint64_t nj = static_cast<uint64_t>(std::max(1, njobs_hint));
  const uint64_t nps = n_ / kNints;
  const uint64_t nchunk = (nps + chunk_ - 1) / chunk_;
  const uint64_t nfold = nj * kNints * kNbins;
  jobs_.resize(nj);
  psum_.resize(nfold * nchunk);
  pcount_.resize(nfold * nchunk);
  folds_.resize(nfold);
  opt_fold_.resize(nfold);
  opt_prof_.resize(nj * kNbins);
  opt_int_.resize(nj * 3);
  opt_val_.resize(nj);
  PSOUP_HIP_CHECK(hipStreamSynchronize(stream_));
}

std::vector<FoldResult> FoldEngine::fold_series(const float* d_series, const std::vector<double>& periods,
                                                const std::vector<float>& accs) {
  std::vector<kern::FoldJob> jobs(periods.size());
  for (size_t i = 0; i < periods.size(); ++i) {
    jobs[i].tsamp_by_period = static_cast<double>(tsamp_) / periods[i];
    jobs[i].af = (static_cast<double>(accs[i]) * tsamp_) / (2 * kC);
    jobs[i].series = 0;
  }
  return fold_jobs(d_series, jobs, periods);
}

std::vector<FoldResult> FoldEngine::fold_jobs(const float* d_series, const std::vector<kern::FoldJob>& jobs,
                                              const std::vector<double>& periods) {
  const int nj = static_cast<int>(jobs.size());
  std::vector<FoldResult> res(static_cast<size_t>(nj));
  if (nj == 0) return res;
  const uint64_t nps = n_ / kNints;
  const int nchunk = static_cast<int>((nps + chunk_ - 1) / chunk_);
  jobs_.resize(jobs.size());
  PSOUP_HIP_CHECK(hipMemcpyAsync(jobs_.data(), jobs.data(), jobs.size() * sizeof(kern::FoldJob), hipMemcpyHostToDevice,
                                 stream_));
  const size_t nfold = static_cast<size_t>(nj) * kNints * kNbins;
  psum_.resize(nfold * nchunk);
  pcount_.resize(nfold * nchunk);
  folds_.resize(nfold);
  opt_fold_.resize(nfold);
  opt_prof_.resize(static_cast<size_t>(nj) * kNbins);
  opt_int_.resize(static_cast<size_t>(nj) * 3);
  opt_val_.resize(static_cast<size_t>(nj));
  kern::fold_accumulate(d_series, n_, jobs_.data(), nj, kNbins, kNints, chunk_, psum_.data(), pcount_.data(), stream_);
  kern::fold_reduce(psum_.data(), pcount_.data(), nj, kNbins, kNints, nchunk, folds_.data(), stream_);
  kern::fold_optimise(folds_.data(), nj, shift_table_.data(), opt_fold_.data(), opt_prof_.data(), opt_int_.data(),
                      opt_val_.data(), stream_);
  std::vector<float> h_fold(nfold), h_prof(static_cast<size_t>(nj) * kNbins);
  std::vector<int32_t> h_int(static_cast<size_t>(nj) * 3);
  PSOUP_HIP_CHECK(hipMemcpyAsync(h_fold.data(), opt_fold_.data(), nfold * 4, hipMemcpyDeviceToHost, stream_));
  PSOUP_HIP_CHECK(hipMemcpyAsync(h_prof.data(), opt_prof_.data(), h_prof.size() * 4, hipMemcpyDeviceToHost, stream_));
  PSOUP_HIP_CHECK(hipMemcpyAsync(h_int.data(), opt_int_.data(), h_int.size() * 4, hipMemcpyDeviceToHost, stream_));
  PSOUP_HIP_CHECK(hipStreamSynchronize(stream_));
  const float tobs = static_cast<float>(static_cast<double>(n_) * tsamp_);
  for (int i = 0; i < nj; ++i) {
    FoldResult& r = res[i];
    const int opt_template = h_int[3 * i + 0];
    const int opt_shift = h_int[3 * i + 1];
    const int opt_bin = h_int[3 * i + 2] - opt_template / 2;
    float sn1 = 0, sn2 = 0;
    fold_calculate_sn(h_prof.data() + static_cast<size_t>(i) * kNbins, opt_bin, opt_template, kNbins, &sn1, &sn2);
    r.folded_snr = std::max(sn1, sn2);
    const double p = periods[i];
    // FoldedSubints::get_opt_period returns float (folded.hpp)
    r.opt_period = static_cast<float>(p * ((((32.0 - opt_shift) * p) / (kNbins * tobs)) + 1));
    r.opt_width = opt_template + 1;
    r.opt_bin = opt_bin;
    r.fold.assign(h_fold.begin() + static_cast<long>(i) * kNints * kNbins,
                  h_fold.begin() + static_cast<long>(i + 1) * kNints * kNbins);
    r.prof.assign(h_prof.begin() + static_cast<long>(i) * kNbins, h_prof.begin() + static_cast<long>(i + 1) * kNbins);
  }
  return res;
}

// ------------------------------------------------------------ coincidencer --
void coincidencer_beam(const uint8_t* d_trial, uint64_t n, float tsamp, BeamProducts& out, hipStream_t stream) {
  Whitener wh(n, tsamp, stream);
  out.series.resize(n);
  out.spectrum.resize(wh.nbins());
  wh.load_trial(d_trial, n, out.series.data());
  // whiten without the C2R so the dereddened spectrum can be formed first
  const uint64_t nb = wh.nbins();
  wh.forward(out.series.data(), wh.spectrum());
  DeviceBuffer<float> m5(nb / 5), m25(std::max<uint64_t>(1, nb / 25)), m125(std::max<uint64_t>(1, nb / 125));
  const uint64_t n5 = nb / 5, n25 = n5 / 5, n125 = n25 / 5;
  kern::median5_amp(wh.spectrum(), nb, m5.data(), stream);
  kern::median5(m5.data(), n5, m25.data(), stream);
  kern::median5(m25.data(), n25, m125.data(), stream);
  const float bw = wh.bin_width();
  kern::deredden_zap(wh.spectrum(), nb, m5.data(), n5, m25.data(), std::max<uint64_t>(1, n25), m125.data(),
                     std::max<uint64_t>(1, n125), static_cast<int>(0.05f / bw), static_cast<int>(0.5f / bw), nullptr,
                     stream);
  DeviceBuffer<double> partials(2 * 1024);
  DeviceBuffer<float> st(4);
  kern::interbin_stats(wh.spectrum(), nb, out.spectrum.data(), partials.data(), 1024, st.data(), stream);
  kern::normalise_dev(out.spectrum.data(), nb, st.data(), 1.0f, stream);
  wh.inverse(wh.spectrum(), out.series.data());
  kern::f32_stats(out.series.data(), n, partials.data(), 1024, st.data(), stream);
  kern::normalise_dev(out.series.data(), n, st.data(), 1.0f, stream);
  PSOUP_HIP_CHECK(hipStreamSynchronize(stream));
}

void write_samp_mask(const std::vector<float>& mask, const std::string& filename) {
  // "%d\n" per sample (coincidencer.cpp), formatted into one buffer
  std::string buf = "#0 1\n";
  buf.reserve(buf.size() + mask.size() * 3);
  char tmp[16];
  for (float v : mask) {
    const auto r = std::to_chars(tmp, tmp + sizeof(tmp), static_cast<int>(v));
    buf.append(tmp, r.ptr);
    buf.push_back('\n');
  }
  FILE* fo = std::fopen(filename.c_str(), "w");
  if (!fo) PSOUP_THROW("cannot write " << filename);
  const bool ok = std::fwrite(buf.data(), 1, buf.size(), fo) == buf.size();
  if (std::fclose(fo) != 0 || !ok) PSOUP_THROW("failed writing " << filename);
}

void write_birdie_list(const std::vector<float>& mask, float bin_width, const std::string& filename) {
  std::vector<std::pair<float, float>> birdies;
  const long size = static_cast<long>(mask.size());
  long ii = 0;
  while (ii < size) {
    if (mask[ii] == 0) {
      int count = 0;
      while (ii < size && mask[ii] == 0) {
        count++;
        ii++;
      }
      birdies.emplace_back(static_cast<float>(((ii - 1) - (count / 2.0)) * bin_width),
                           static_cast<float>(count * bin_width));
    } else {
      ii++;
    }
  }
  FILE* fo = std::fopen(filename.c_str(), "w");
  if (!fo) PSOUP_THROW("cannot write " << filename);
  bool ok = true;
  for (const auto& b : birdies) ok = ok && std::fprintf(fo, "%.9f\t%.6f\n", b.first, b.second) > 0;
  if (std::fclose(fo) != 0 || !ok) PSOUP_THROW("failed writing " << filename);
}

}  // namespace psoup
