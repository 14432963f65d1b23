// `peasoup_tools`: the reference's stand-alone test/diagnostic drivers as
// subcommands of one executable, on real inputs instead of hard-coded paths.
//
//   harmsum    harmonic_sum_test.cpp   comb spectrum, repeated harmonic sums, exactness check
//   resample   resampling_test.cpp     resampler v1 vs II on the sawtooth pattern
//   fft        hcfft.cpp               R2C+C2R timing (rocFFT) and the fused four-step FFT
//   dedisp     dedisp_test.cpp         DM list + dedispersion of a .fil, optional dumps
//   fold       folder_test.cpp         fold + optimise a .tim at a period (dumps the fold)
//   rednoise   rednoise_test.cpp       whitening chain of a .tim with intermediate dumps
//   filterbank filterbank_test.cpp     header accessors and write/read round trip
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "psoup/common.hpp"
#include "psoup/engine.hpp"
#include "psoup/fft.hpp"
#include "psoup/kernels.hpp"
#include "psoup/plan.hpp"
#include "psoup/sigproc.hpp"

using namespace psoup;

namespace {

struct Args {
  std::map<std::string, std::string> kv;
  std::vector<std::string> pos;
  std::string get(const std::string& k, const std::string& d) const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
  double num(const std::string& k, double d) const {
    auto it = kv.find(k);
    return it == kv.end() ? d : std::stod(it->second);
  }
  bool has(const std::string& k) const { return kv.count(k) > 0; }
};

Args parse(int argc, char** argv, int first) {
  Args a;
  for (int i = first; i < argc; ++i) {
    std::string s = argv[i];
    if (s.rfind("--", 0) == 0) {
      std::string key = s.substr(2), val = "1";
      auto eq = key.find('=');
      if (eq != std::string::npos) {
        val = key.substr(eq + 1);
        key = key.substr(0, eq);
      } else if (i + 1 < argc && std::string(argv[i + 1]).rfind("--", 0) != 0) {
        val = argv[++i];
      }
      a.kv[key] = val;
    } else {
      a.pos.push_back(s);
    }
  }
  return a;
}

template <class T>
void dump(const std::string& path, const T* d_ptr, size_t n) {
  std::vector<T> h(n);
  PSOUP_HIP_CHECK(hipMemcpy(h.data(), d_ptr, n * sizeof(T), hipMemcpyDeviceToHost));
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(h.data()), static_cast<std::streamsize>(n * sizeof(T)));
  std::cout << "wrote " << path << " (" << n << " x " << sizeof(T) << " B)\n";
}

// ------------------------------------------------------------------ harmsum --
int cmd_harmsum(const Args& a) {
  const uint64_t nbins = static_cast<uint64_t>(a.num("nbins", 10000000));
  const int nlev = static_cast<int>(a.num("nlevels", 4));
  const int reps = static_cast<int>(a.num("reps", 100));
  std::vector<float> h(nbins);
  for (uint64_t i = 0; i < nbins; ++i) h[i] = (i % 32 == 0) ? 1.f : 0.f;
  Stream st;
  DeviceBuffer<float> p(nbins), sums(nbins * nlev);
  PSOUP_HIP_CHECK(hipMemcpy(p.data(), h.data(), nbins * 4, hipMemcpyHostToDevice));
  GpuTimer t;
  t.start(st.get());
  for (int r = 0; r < reps; ++r) kern::harmonic_sums(p.data(), nbins, nlev, sums.data(), st.get());
  t.stop(st.get());
  const double ms = t.elapsed_ms() / reps;
  std::vector<float> out(nbins * nlev);
  PSOUP_HIP_CHECK(hipMemcpy(out.data(), sums.data(), out.size() * 4, hipMemcpyDeviceToHost));
  // host check on a sample of bins (reference recurrence, kernels.cu:42-96)
  static const double scale[6] = {1.0, 0.70710678118654752440, 0.5, 0.35355339059327376220, 0.25,
                                  0.17677669529663688110};
  uint64_t bad = 0, checked = 0;
  for (uint64_t i = 0; i < nbins; i += 997) {
    float v = h[i];
    const long long li = static_cast<long long>(i);
    for (int lev = 1; lev <= nlev; ++lev) {
      if (lev == 1) {
        v += h[(li + 1) >> 1];
      } else if (lev == 2) {
        v += h[(li * 3 + 2) >> 2];
        v += h[(li + 2) >> 2];
      } else {
        const int den = 1 << lev;
        for (int m = 1; m < den; m += 2) v += h[(li * m + den / 2) >> lev];
      }
      const float e = static_cast<float>(static_cast<double>(v) * scale[lev]);
      bad += out[static_cast<uint64_t>(lev - 1) * nbins + i] != e;
      ++checked;
    }
  }
  std::cout << "harmonic_sums: nbins=" << nbins << " levels=" << nlev << " " << ms << " ms/call, "
            << (nbins * 4.0 * (1 + nlev) / (ms * 1e-3) / 1e9) << " GB/s written+read; mismatches " << bad << "/"
            << checked << "\n";
  return bad == 0 ? 0 : 1;
}

// ----------------------------------------------------------------- resample --
int cmd_resample(const Args& a) {
  const uint64_t n = static_cast<uint64_t>(a.num("n", 4194304));
  const float tsamp = static_cast<float>(a.num("tsamp", 0.000064));
  const float acc = static_cast<float>(a.num("acc", 125.5));
  std::vector<float> h(n);
  for (uint64_t i = 0; i < n; ++i) h[i] = static_cast<float>(i % 451);
  Stream st;
  DeviceBuffer<float> in(n), r0(n), r1(n);
  DeviceBuffer<double> af(1);
  PSOUP_HIP_CHECK(hipMemcpy(in.data(), h.data(), n * 4, hipMemcpyHostToDevice));
  const double afv = (static_cast<double>(acc) * tsamp) / (2 * 299792458.0);
  PSOUP_HIP_CHECK(hipMemcpy(af.data(), &afv, 8, hipMemcpyHostToDevice));
  kern::resample_v1(in.data(), n, r0.data(), afv, st.get());
  kern::resample_batch(in.data(), n, r1.data(), n, af.data(), 1, st.get());
  st.sync();
  std::vector<float> b0(n), b1(n);
  PSOUP_HIP_CHECK(hipMemcpy(b0.data(), r0.data(), n * 4, hipMemcpyDeviceToHost));
  PSOUP_HIP_CHECK(hipMemcpy(b1.data(), r1.data(), n * 4, hipMemcpyDeviceToHost));
  uint64_t wrong = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (std::fabs(b0[i] - b1[i]) > 0.0001f) {
      if (wrong < 10) std::printf("[WRONG (%llu)] %f != %f\n", static_cast<unsigned long long>(i), b0[i], b1[i]);
      ++wrong;
    }
  std::cout << "resample v1 vs II: " << wrong << " of " << n << " samples differ (index rounding ties)\n";
  return 0;
}

// ---------------------------------------------------------------------- fft --
int cmd_fft(const Args& a) {
  const uint64_t n = static_cast<uint64_t>(a.num("n", 8388608));
  const int loops = static_cast<int>(a.num("loops", 100));
  const int K = static_cast<int>(a.num("batch", 32));
  Stream st;
  DeviceBuffer<float> tim(n), res(n);
  DeviceBuffer<float2> spec(n / 2 + 1);
  tim.zero_async(st.get());
  FftPlan fwd(FftType::R2C, n), inv(FftType::C2R, n);
  GpuTimer t;
  fwd.execute(tim.data(), spec.data(), st.get());
  t.start(st.get());
  for (int i = 0; i < loops; ++i) {
    fwd.execute(tim.data(), spec.data(), st.get());
    inv.execute(spec.data(), res.data(), st.get());
  }
  t.stop(st.get());
  std::cout << "rocFFT R2C+C2R n=" << n << ": " << t.elapsed_ms() / loops << " ms per pair\n";
  const kern::Fft4Geom g = kern::fft4_geometry(n / 2);
  if (!g.ok) {
    std::cout << "fused four-step FFT: unsupported length\n";
    return 0;
  }
  auto tab = kern::fft4_tables(g);
  DeviceBuffer<float2> d_tab(tab.size()), Y(static_cast<size_t>(K) * g.ystride), X(static_cast<size_t>(K) * g.xstride);
  DeviceBuffer<float> pad(g.insize);
  DeviceBuffer<double> af(static_cast<size_t>(K));
  std::vector<double> afh(static_cast<size_t>(K));
  for (int k = 0; k < K; ++k) afh[static_cast<size_t>(k)] = (-500.0 + 1000.0 * k / std::max(1, K - 1)) * 64e-6 / 6e8;
  PSOUP_HIP_CHECK(hipMemcpy(d_tab.data(), tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice));
  PSOUP_HIP_CHECK(hipMemcpy(af.data(), afh.data(), afh.size() * 8, hipMemcpyHostToDevice));
  kern::fft4_pad_input(tim.data(), n, pad.data(), g, st.get());
  GpuTimer t2;
  t2.start(st.get());
  for (int i = 0; i < loops; ++i) {
    kern::fft4_resample_colpass(tim.data(), pad.data(), n, af.data(), K, Y.data(), g, d_tab.data(), st.get());
    kern::fft4_rowpass(Y.data(), X.data(), K, g, d_tab.data(), st.get());
  }
  t2.stop(st.get());
  std::cout << "fused resample + four-step FFT (" << g.n1 << " x " << g.n2 << "), batch " << K << ": "
            << t2.elapsed_ms() / loops / K << " ms per trial\n";
  return 0;
}

// ------------------------------------------------------------------- dedisp --
int cmd_dedisp(const Args& a) {
  if (!a.has("i")) PSOUP_THROW("dedisp: -i/--i <file.fil> required");
  Filterbank fb = Filterbank::from_file(a.get("i", ""));
  auto dms = generate_dm_list(static_cast<float>(a.num("dm_start", 0)), static_cast<float>(a.num("dm_end", 100)),
                              fb.tsamp(), static_cast<float>(a.num("dm_pulse_width", 40)), fb.fch1(), fb.foff(),
                              fb.nchans(), static_cast<float>(a.num("dm_tol", 1.1)));
  std::cout << dms.size() << " DM trials\n";
  for (size_t i = 0; i < dms.size(); ++i) std::cout << i << "\t" << dms[i] << "\n";
  Stream st;
  auto g = DedispGeometry::make(fb.header(), fb.nsamps(), dms, {});
  DeviceFilterbank dfb(g, st.get());
  dfb.load_packed_host(fb.data());
  Dedisperser dd(dfb, st.get());
  const uint64_t stride = Dedisperser::row_stride(g.out_nsamps);
  DeviceBuffer<uint8_t> out(stride * dms.size());
  Stopwatch sw;
  sw.start();
  dd.run(0, static_cast<int>(dms.size()), out.data(), stride, DedispKernel::Auto);
  st.sync();
  sw.stop();
  std::cout << "dedispersed " << dms.size() << " x " << g.out_nsamps << " samples in " << sw.get_time() << " s\n";
  if (a.has("dump")) {
    std::vector<uint8_t> h(stride * dms.size());
    PSOUP_HIP_CHECK(hipMemcpy(h.data(), out.data(), h.size(), hipMemcpyDeviceToHost));
    std::ofstream f(a.get("dump", ""), std::ios::binary);
    for (size_t d = 0; d < dms.size(); ++d)
      f.write(reinterpret_cast<const char*>(h.data() + d * stride), static_cast<std::streamsize>(g.out_nsamps));
    std::cout << "wrote " << a.get("dump", "") << "\n";
  }
  return 0;
}

// --------------------------------------------------------------------- fold --
int cmd_fold(const Args& a) {
  if (a.pos.empty()) PSOUP_THROW("fold: <file.tim> required");
  TimeSeriesFile tf = read_tim(a.pos[0]);
  const double period = a.num("period", 0.007453099228);
  const float acc = static_cast<float>(a.num("acc", 0));
  const uint64_t n = prev_power_of_two(tf.data.size() + 1);
  Stream st;
  DeviceBuffer<float> d(n);
  PSOUP_HIP_CHECK(hipMemcpy(d.data(), tf.data.data(), n * 4, hipMemcpyHostToDevice));
  FoldEngine fe(n, static_cast<float>(tf.header.tsamp), st.get());
  Stopwatch sw;
  sw.start();
  auto res = fe.fold_series(d.data(), {period}, {acc});
  sw.stop();
  const FoldResult& r = res.at(0);
  std::cout << "fold of " << n << " samples at P=" << period << " s: folded S/N " << r.folded_snr << ", opt period "
            << r.opt_period << " (" << sw.get_time() << " s)\n";
  if (a.has("dump")) {
    std::ofstream f(a.get("dump", "original_fold.bin"), std::ios::binary);
    f.write(reinterpret_cast<const char*>(r.fold.data()), static_cast<std::streamsize>(r.fold.size() * 4));
  }
  return 0;
}

// ----------------------------------------------------------------- rednoise --
int cmd_rednoise(const Args& a) {
  if (a.pos.empty()) PSOUP_THROW("rednoise: <file.tim> required");
  TimeSeriesFile tf = read_tim(a.pos[0]);
  const uint64_t n = a.has("size") ? static_cast<uint64_t>(a.num("size", 0)) : prev_power_of_two(tf.data.size() + 1);
  const float tsamp = static_cast<float>(tf.header.tsamp);
  const float acc = static_cast<float>(a.num("acc", 222.51));
  const int nlev = static_cast<int>(a.num("nharmonics", 4));
  const std::string od = a.get("outdir", ".");
  Stream st;
  Whitener wh(n, tsamp, st.get());
  DeviceBuffer<float> series(n), res(n), P(n / 2 + 1), sums(static_cast<size_t>(n / 2 + 1) * std::max(nlev, 1));
  std::vector<float> h(n, 0.f);
  std::copy(tf.data.begin(), tf.data.begin() + static_cast<std::ptrdiff_t>(std::min<uint64_t>(n, tf.data.size())),
            h.begin());
  PSOUP_HIP_CHECK(hipMemcpy(series.data(), h.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> zap;
  DeviceBuffer<uint32_t> d_zap;
  if (a.has("zapfile")) {
    std::vector<float> fr, wd;
    read_zapfile(a.get("zapfile", ""), fr, wd);
    zap = build_zap_mask(fr, wd, wh.bin_width(), wh.nbins());
    d_zap.resize(zap.size());
    PSOUP_HIP_CHECK(hipMemcpy(d_zap.data(), zap.data(), zap.size() * 4, hipMemcpyHostToDevice));
  }
  wh.whiten(series.data(), zap.empty() ? nullptr : d_zap.data(), true, 0.05f, 0.5f);
  std::vector<float> stats(3);
  st.sync();
  PSOUP_HIP_CHECK(hipMemcpy(stats.data(), wh.stats(), 12, hipMemcpyDeviceToHost));
  std::cout << "whitened: interbin mean " << stats[0] << " rms " << stats[1] << " std " << stats[2] << "\n";
  DeviceBuffer<double> af(1);
  const double afv = (static_cast<double>(acc) * tsamp) / (2 * 299792458.0);
  PSOUP_HIP_CHECK(hipMemcpy(af.data(), &afv, 8, hipMemcpyHostToDevice));
  kern::resample_batch(series.data(), n, res.data(), n, af.data(), 1, st.get());
  dump(od + "/tim_r.bin", res.data(), n);
  DeviceBuffer<float2> X(n / 2 + 1);
  FftPlan r2c(FftType::R2C, n);
  r2c.execute(res.data(), X.data(), st.get());
  kern::form_amplitude(X.data(), n / 2 + 1, P.data(), st.get());
  dump(od + "/non_interp_spec.bin", P.data(), n / 2 + 1);
  kern::form_interbin(X.data(), n / 2 + 1, P.data(), st.get());
  dump(od + "/interp_spec.bin", P.data(), n / 2 + 1);
  kern::normalise_dev(P.data(), n / 2 + 1, wh.stats(), static_cast<float>(n), st.get());
  dump(od + "/pspec_post.bin", P.data(), n / 2 + 1);
  if (nlev > 0) {
    kern::harmonic_sums(P.data(), n / 2 + 1, nlev, sums.data(), st.get());
    for (int l = 0; l < nlev; ++l)
      dump(od + "/harm" + std::to_string(l + 1) + ".bin", sums.data() + static_cast<size_t>(l) * (n / 2 + 1),
           n / 2 + 1);
  }
  return 0;
}

// --------------------------------------------------------------- filterbank --
int cmd_filterbank(const Args& a) {
  SigprocHeader hdr;
  hdr.nchans = 1024;
  hdr.nbits = 2;
  hdr.fch1 = 1560.0;
  hdr.foff = 0.39;
  hdr.tsamp = 0.000054;
  hdr.nsamples = 1000;
  hdr.nifs = 1;
  hdr.data_type = 1;
  hdr.keys_present = {"nchans", "nbits", "fch1", "foff", "tsamp", "nsamples", "nifs", "data_type"};
  std::vector<uint8_t> data(static_cast<size_t>(hdr.nsamples) * hdr.nchans * hdr.nbits / 8);
  for (size_t i = 0; i < data.size(); ++i) data[i] = static_cast<uint8_t>(i * 2654435761u >> 24);
  Filterbank fb = Filterbank::from_memory(hdr, data);
  bool ok = fb.nsamps() == 1000 && fb.nchans() == 1024 && fb.nbits() == 2 && fb.tsamp() == 0.000054 &&
            fb.foff() == 0.39 && fb.fch1() == 1560.0;
  const std::string path = a.get("o", "/tmp/peasoup_tools_fb.fil");
  fb.write(path);
  Filterbank rb = Filterbank::from_file(path);
  ok = ok && rb.nsamps() == fb.nsamps() && rb.nchans() == fb.nchans() && rb.data_bytes() == fb.data_bytes() &&
       std::equal(data.begin(), data.end(), rb.data());
  if (a.has("i")) {
    Filterbank in = Filterbank::from_file(a.get("i", ""));
    std::cout << a.get("i", "") << ": nsamps " << in.nsamps() << " nchans " << in.nchans() << " nbits " << in.nbits()
              << " tsamp " << in.tsamp() << " fch1 " << in.fch1() << " foff " << in.foff() << "\n";
  }
  std::cout << "filterbank accessors + write/read round trip: " << (ok ? "OK" : "FAILED") << "\n";
  return ok ? 0 : 1;
}

void usage() {
  std::cerr << "usage: peasoup_tools <harmsum|resample|fft|dedisp|fold|rednoise|filterbank> [options]\n"
               "  harmsum    [--nbins N] [--nlevels L] [--reps R]\n"
               "  resample   [--n N] [--tsamp T] [--acc A]\n"
               "  fft        [--n N] [--loops L] [--batch K]\n"
               "  dedisp     --i file.fil [--dm_start --dm_end --dm_pulse_width --dm_tol] [--dump out.bin]\n"
               "  fold       file.tim [--period P] [--acc A] [--dump fold.bin]\n"
               "  rednoise   file.tim [--size N] [--acc A] [--nharmonics L] [--zapfile f] [--outdir d]\n"
               "  filterbank [--i file.fil] [--o tmp.fil]\n";
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    usage();
    return 2;
  }
  const std::string cmd = argv[1];
  const Args a = parse(argc, argv, 2);
  try {
    if (cmd == "harmsum") return cmd_harmsum(a);
    if (cmd == "resample") return cmd_resample(a);
    if (cmd == "fft") return cmd_fft(a);
    if (cmd == "dedisp") return cmd_dedisp(a);
    if (cmd == "fold") return cmd_fold(a);
    if (cmd == "rednoise") return cmd_rednoise(a);
    if (cmd == "filterbank") return cmd_filterbank(a);
    usage();
    return 2;
  } catch (const std::exception& e) {
    std::cerr << "peasoup_tools " << cmd << ": " << e.what() << "\n";
    return 1;
  }
}
