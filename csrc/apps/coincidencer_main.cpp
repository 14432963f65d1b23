// `peasoup_coincidencer`: multi-beam RFI coincidence masks
// (src/coincidencer.cpp:46-215).  Each beam is dedispersed at DM 0,
// whitened and normalised; a time sample / Fourier bin is masked when it
// exceeds --thresh in at least --beam_thresh beams.  Beams are spread over
// the visible GPUs; per-GPU uint8 indicator counts are summed on device 0
// (peer copies + kernels) and thresholded there.
#include <algorithm>
#include <memory>
#include <iostream>
#include <mutex>
#include <thread>

#include "psoup/cli.hpp"
#include "psoup/common.hpp"
#include "psoup/engine.hpp"
#include "psoup/plan.hpp"
#include "psoup/sigproc.hpp"

using namespace psoup;

int main(int argc, char** argv) {
  CoincidencerOptions args;
  bool exit_now = false;
  if (!parse_coincidencer_cmdline(args, argc, argv, &exit_now)) return 1;
  if (exit_now) return 0;
  try {
    const int nfiles = static_cast<int>(args.filterbanks.size());
    // per-sample beam counts are uint8 (kern::count_above): more beams would wrap
    PSOUP_CHECK(nfiles <= 255, nfiles << " beams: the coincidencer counts beams in uint8, at most 255");
    std::vector<Filterbank> fbs;
    for (const auto& f : args.filterbanks) fbs.push_back(Filterbank::from_file(f));
    std::vector<uint64_t> lens;
    for (auto& fb : fbs) {
      auto dms = generate_dm_list(0.f, 0.f, fb.tsamp(), 0.4, fb.fch1(), fb.foff(), fb.nchans(), 1.1);
      auto g = DedispGeometry::make(fb.header(), fb.nsamps(), dms, {});
      lens.push_back(g.out_nsamps);
    }
    const uint64_t size = lens[0];
    for (auto l : lens)
      if (l != size) PSOUP_THROW("Not all filterbanks the same length");
    const float tsamp = static_cast<float>(fbs[0].tsamp());
    const uint64_t nb = size / 2 + 1;
    const int ngpu = std::max(1, std::min(device_count(), nfiles));
    // per device: its stream and the uint8 beam counts of its beams
    struct DevCounts {
      std::unique_ptr<Stream> st;
      DeviceBuffer<uint8_t> tc, sc;
    };
    std::vector<DevCounts> dc(static_cast<size_t>(ngpu));
    std::vector<std::thread> th;
    std::exception_ptr err;
    std::mutex mu;
    for (int dev = 0; dev < ngpu; ++dev) {
      th.emplace_back([&, dev] {
        try {
          PSOUP_HIP_CHECK(hipSetDevice(dev));
          DevCounts& d = dc[static_cast<size_t>(dev)];
          d.st = std::make_unique<Stream>();
          Stream& st = *d.st;
          d.tc.resize(size);
          d.sc.resize(nb);
          DeviceBuffer<uint8_t>& tc = d.tc;
          DeviceBuffer<uint8_t>& sc = d.sc;
          tc.zero_async(st.get());
          sc.zero_async(st.get());
          for (int b = dev; b < nfiles; b += ngpu) {
            if (args.verbose) log_info("Baselining beam " + std::to_string(b));
            auto dms = generate_dm_list(0.f, 0.f, fbs[b].tsamp(), 0.4, fbs[b].fch1(), fbs[b].foff(), fbs[b].nchans(), 1.1);
            auto g = DedispGeometry::make(fbs[b].header(), fbs[b].nsamps(), dms, {});
            DeviceFilterbank dfb(g, st.get());
            dfb.load_packed_host(fbs[b].data());
            Dedisperser dd(dfb, st.get());
            DeviceBuffer<uint8_t> trial(Dedisperser::row_stride(g.out_nsamps));
            dd.run(0, 1, trial.data(), trial.size(), DedispKernel::Direct);
            BeamProducts bp;
            coincidencer_beam(trial.data(), size, tsamp, bp, st.get());
            kern::count_above(bp.series.data(), size, args.threshold, tc.data(), st.get());
            kern::count_above(bp.spectrum.data(), nb, args.threshold, sc.data(), st.get());
            PSOUP_HIP_CHECK(hipStreamSynchronize(st.get()));
          }
        } catch (...) {
          std::lock_guard<std::mutex> lk(mu);
          if (!err) err = std::current_exception();
        }
      });
    }
    for (auto& t : th) t.join();
    if (err) std::rethrow_exception(err);
    if (args.verbose) log_info("Performing cross beam coincidence matching");
    // every device's counts summed on device 0 (peer copies over xGMI where
    // the pair allows), thresholded there into the two masks
    PSOUP_HIP_CHECK(hipSetDevice(0));
    hipStream_t s0 = dc[0].st->get();
    DeviceBuffer<uint8_t> stage_t, stage_s;
    if (ngpu > 1) {
      stage_t.resize(size);
      stage_s.resize(nb);
    }
    for (int d = 1; d < ngpu; ++d) {
      enable_peer_access(0, d);
      PSOUP_HIP_CHECK(hipMemcpyPeerAsync(stage_t.data(), 0, dc[static_cast<size_t>(d)].tc.data(), d, size, s0));
      kern::add_counts(stage_t.data(), size, dc[0].tc.data(), s0);
      PSOUP_HIP_CHECK(hipMemcpyPeerAsync(stage_s.data(), 0, dc[static_cast<size_t>(d)].sc.data(), d, nb, s0));
      kern::add_counts(stage_s.data(), nb, dc[0].sc.data(), s0);
    }
    DeviceBuffer<float> d_samp(size), d_spec(nb);
    kern::coincidence_mask(dc[0].tc.data(), size, args.beam_threshold, d_samp.data(), s0);
    kern::coincidence_mask(dc[0].sc.data(), nb, args.beam_threshold, d_spec.data(), s0);
    std::vector<float> samp_mask(size), spec_mask(nb);
    PSOUP_HIP_CHECK(hipMemcpyAsync(samp_mask.data(), d_samp.data(), size * sizeof(float), hipMemcpyDeviceToHost, s0));
    PSOUP_HIP_CHECK(hipMemcpyAsync(spec_mask.data(), d_spec.data(), nb * sizeof(float), hipMemcpyDeviceToHost, s0));
    PSOUP_HIP_CHECK(hipStreamSynchronize(s0));
    const float bin_width = static_cast<float>(1.0 / static_cast<float>(size * tsamp));
    write_samp_mask(samp_mask, args.samp_outfilename);
    write_birdie_list(spec_mask, bin_width, args.spec_outfilename);
  } catch (const std::exception& e) {
    std::cerr << "peasoup_coincidencer: error: " << e.what() << std::endl;
    return 2;
  }
  return 0;
}
