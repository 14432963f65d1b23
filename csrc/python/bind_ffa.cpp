// pybind11 bindings of the FFA search (ffa.hpp): options, plan, engine,
// pipeline, and a self-contained kernel driver for numerics tests.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "psoup/cli.hpp"
#include "psoup/common.hpp"
#include "psoup/ffa.hpp"

namespace py = pybind11;
using namespace psoup;

void bind_ffa(py::module_& m) {
  py::class_<FfaCmdLineOptions>(m, "FfaCmdLineOptions")
      .def(py::init<>())
      .def_readwrite("infilename", &FfaCmdLineOptions::infilename)
      .def_readwrite("outfilename", &FfaCmdLineOptions::outfilename)
      .def_readwrite("killfilename", &FfaCmdLineOptions::killfilename)
      .def_readwrite("max_num_threads", &FfaCmdLineOptions::max_num_threads)
      .def_readwrite("nstreams", &FfaCmdLineOptions::nstreams)
      .def_readwrite("dm_start", &FfaCmdLineOptions::dm_start)
      .def_readwrite("dm_end", &FfaCmdLineOptions::dm_end)
      .def_readwrite("dm_tol", &FfaCmdLineOptions::dm_tol)
      .def_readwrite("dm_pulse_width", &FfaCmdLineOptions::dm_pulse_width)
      .def_readwrite("p_start", &FfaCmdLineOptions::p_start)
      .def_readwrite("p_end", &FfaCmdLineOptions::p_end)
      .def_readwrite("min_dc", &FfaCmdLineOptions::min_dc)
      .def_readwrite("verbose", &FfaCmdLineOptions::verbose)
      .def_readwrite("progress_bar", &FfaCmdLineOptions::progress_bar)
      .def_readwrite("min_snr", &FfaCmdLineOptions::min_snr)
      .def_readwrite("nbins", &FfaCmdLineOptions::nbins)
      .def_readwrite("limit", &FfaCmdLineOptions::limit)
      .def_readwrite("cluster_tol", &FfaCmdLineOptions::cluster_tol)
      .def_readwrite("dedisp_kernel", &FfaCmdLineOptions::dedisp_kernel);
  m.def("parse_ffa_cmdline", [](const std::vector<std::string>& argv) {
    FfaCmdLineOptions a;
    bool exit_now = false;
    bool ok = parse_ffa_cmdline(a, argv, &exit_now);
    return py::make_tuple(ok, exit_now, a);
  });
  m.def("default_ffa_output_filename", &default_ffa_output_filename);

  py::class_<FfaParams>(m, "FfaParams")
      .def(py::init<>())
      .def_readwrite("tsamp", &FfaParams::tsamp)
      .def_readwrite("p_start", &FfaParams::p_start)
      .def_readwrite("p_end", &FfaParams::p_end)
      .def_readwrite("min_dc", &FfaParams::min_dc)
      .def_readwrite("nbins", &FfaParams::nbins)
      .def_readwrite("min_snr", &FfaParams::min_snr)
      .def_readwrite("detrend_s", &FfaParams::detrend_s)
      .def_readwrite("arena_floats", &FfaParams::arena_floats)
      .def_readwrite("cluster_tol", &FfaParams::cluster_tol)
      .def_readwrite("min_rows", &FfaParams::min_rows);
  m.def("ffa_params_from", &ffa_params_from);

  py::class_<FfaCandidate>(m, "FfaCandidate")
      .def(py::init<>())
      .def_readwrite("period", &FfaCandidate::period)
      .def_readwrite("snr", &FfaCandidate::snr)
      .def_readwrite("width", &FfaCandidate::width)
      .def_readwrite("nbins", &FfaCandidate::nbins)
      .def_readwrite("dm", &FfaCandidate::dm)
      .def_readwrite("dm_idx", &FfaCandidate::dm_idx)
      .def_readwrite("octave", &FfaCandidate::octave)
      .def_property_readonly("freq", &FfaCandidate::freq)
      .def_property_readonly("duty_cycle", &FfaCandidate::duty_cycle);

  m.def("ffa_base_bins", &ffa_base_bins);
  m.def("ffa_widths", &ffa_widths);
  m.def("ffa_cluster", &ffa_cluster);
  m.def("ffa_plan", [](const FfaParams& p, uint64_t n) {
    py::list out;
    for (const FfaOctave& o : ffa_plan(p, n)) {
      py::dict d;
      d["factor"] = o.factor;
      d["nds"] = o.nds;
      d["pa"] = o.pa;
      d["pb"] = o.pb;
      py::list chunks;
      for (const FfaChunk& c : o.chunks) {
        py::dict cd;
        py::list per;
        for (const auto& fp : c.periods) per.append(py::make_tuple(fp.p, fp.m, fp.m2, fp.log2m2, fp.offset));
        cd["periods"] = per;
        cd["arena"] = c.arena;
        cd["max_m2"] = c.max_m2;
        cd["max_p"] = c.max_p;
        cd["nprof"] = c.nprof;
        chunks.append(cd);
      }
      d["chunks"] = chunks;
      out.append(d);
    }
    return out;
  });

  py::class_<FfaEngine>(m, "FfaEngine")
      .def(py::init([](const FfaParams& p, uint64_t nsamps, uintptr_t stream) {
             return new FfaEngine(p, nsamps, reinterpret_cast<hipStream_t>(stream));
           }),
           py::arg("params"), py::arg("nsamps"), py::arg("stream") = 0)
      .def("search",
           [](FfaEngine& e, uintptr_t trial, float dm, int dm_idx) {
             py::gil_scoped_release nogil;
             return e.search(reinterpret_cast<const uint8_t*>(trial), dm, dm_idx);
           })
      .def_property_readonly("nsamps", &FfaEngine::nsamps)
      .def_property_readonly("tobs", &FfaEngine::tobs)
      .def_property_readonly("profiles", &FfaEngine::profiles)
      .def_property_readonly("peaks", &FfaEngine::peaks);

  py::class_<FfaResult>(m, "FfaResult")
      .def(py::init<>())
      .def_readwrite("candidates", &FfaResult::candidates)
      .def_readwrite("dm_list", &FfaResult::dm_list)
      .def_readwrite("devices", &FfaResult::devices)
      .def_readwrite("timers", &FfaResult::timers)
      .def_readwrite("nsamps", &FfaResult::nsamps)
      .def_readwrite("tobs", &FfaResult::tobs)
      .def_readwrite("nb0", &FfaResult::nb0)
      .def_readwrite("profiles", &FfaResult::profiles)
      .def_readwrite("peaks", &FfaResult::peaks);
  m.def("run_ffa_pipeline", [](const FfaCmdLineOptions& a) {
    py::gil_scoped_release nogil;
    return run_ffa_pipeline(a);
  });
  m.def("write_ffa_output", &write_ffa_output);

  // Kernel driver for tests: FFA planes + per-profile best S/N of the
  // given base periods over a host series (ds, unit-variance bins of
  // variance `var_per_bin`), on the current device.
  m.def(
      "ffa_fold_planes",
      [](py::array_t<float, py::array::c_style> ds, const std::vector<int>& periods, float var_per_bin,
         float thresh) {
        const uint64_t nds = static_cast<uint64_t>(ds.size());
        std::vector<kern::FfaPeriod> tab;
        uint64_t arena = 0, nprof = 0;
        int max_m2 = 0, max_lg = 0, max_p = 0;
        for (int P : periods) {
          const uint64_t mrows = nds / static_cast<uint64_t>(P);
          PSOUP_CHECK(P >= 2 && mrows >= 1, "ffa_fold_planes: period longer than the series");
          int lg = 0;
          while ((uint64_t(1) << lg) < mrows) ++lg;
          kern::FfaPeriod fp{};
          fp.p = P;
          fp.m = static_cast<int32_t>(mrows);
          fp.m2 = 1 << lg;
          fp.log2m2 = lg;
          fp.offset = arena;
          fp.best_offset = nprof;
          arena += static_cast<uint64_t>(fp.m2) * P;
          nprof += static_cast<uint64_t>(fp.m2);
          max_m2 = std::max(max_m2, fp.m2);
          max_lg = std::max(max_lg, lg);
          max_p = std::max(max_p, P);
          tab.push_back(fp);
        }
        DeviceBuffer<float> d_ds(nds), a0(arena), a1(arena), best(nprof);
        DeviceBuffer<kern::FfaPeriod> d_tab(tab.size());
        DeviceBuffer<kern::FfaPeak> peaks(1u << 16);
        DeviceBuffer<uint32_t> cnt(1);
        PSOUP_HIP_CHECK(hipMemcpy(d_ds.data(), ds.data(), nds * 4, hipMemcpyHostToDevice));
        PSOUP_HIP_CHECK(
            hipMemcpy(d_tab.data(), tab.data(), tab.size() * sizeof(kern::FfaPeriod), hipMemcpyHostToDevice));
        PSOUP_HIP_CHECK(hipMemset(cnt.data(), 0, 4));
        const std::vector<int> w = ffa_widths(*std::min_element(periods.begin(), periods.end()));
        kern::FfaSnrParams sp{};
        sp.nwidths = static_cast<int32_t>(w.size());
        for (size_t i = 0; i < w.size(); ++i) sp.widths[i] = w[i];
        sp.thresh = thresh;
        sp.var_per_bin = var_per_bin;
        kern::ffa_transform(d_ds.data(), d_tab.data(), static_cast<int>(tab.size()), max_m2, max_lg, max_p, a0.data(),
                            a1.data(), nullptr);
        kern::ffa_snr(d_tab.data(), static_cast<int>(tab.size()), max_m2, max_p, a0.data(), a1.data(), sp,
                      peaks.data(), cnt.data(), 1u << 16, best.data(), nullptr);
        PSOUP_HIP_CHECK(hipDeviceSynchronize());
        std::vector<float> h0(arena), h1(arena), hb(nprof);
        PSOUP_HIP_CHECK(hipMemcpy(h0.data(), a0.data(), arena * 4, hipMemcpyDeviceToHost));
        PSOUP_HIP_CHECK(hipMemcpy(h1.data(), a1.data(), arena * 4, hipMemcpyDeviceToHost));
        PSOUP_HIP_CHECK(hipMemcpy(hb.data(), best.data(), nprof * 4, hipMemcpyDeviceToHost));
        const bool lds = kern::ffa_uses_lds(max_p);
        py::list out;
        for (const auto& fp : tab) {
          const bool in1 = kern::ffa_result_in_second(fp, lds ? 4 : 0);
          const float* src = (in1 ? h1.data() : h0.data()) + fp.offset;
          py::array_t<float> plane({fp.m2, fp.p});
          std::copy(src, src + static_cast<size_t>(fp.m2) * fp.p, plane.mutable_data());
          py::array_t<float> b(fp.m2);
          std::copy(hb.data() + fp.best_offset, hb.data() + fp.best_offset + fp.m2, b.mutable_data());
          out.append(py::make_tuple(fp.p, fp.m, fp.m2, plane, b));
        }
        return py::make_tuple(out, w);
      },
      py::arg("ds"), py::arg("periods"), py::arg("var_per_bin") = 1.0f, py::arg("thresh") = 1e30f);
}
