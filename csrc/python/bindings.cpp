// pybind11 bindings of the native core (module peasoup_amd._C).
// Device memory crosses the boundary as raw addresses (torch tensors'
// data_ptr()) and streams as hipStream_t handles (torch.cuda.Stream.cuda_stream),
// so no torch headers are needed and the extension builds in seconds.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "psoup/candidates.hpp"
#include "psoup/checkpoint.hpp"
#include "psoup/cli.hpp"
#include "psoup/common.hpp"
#include "psoup/engine.hpp"
#include "psoup/ffa.hpp"
#include "psoup/fft.hpp"
#include "psoup/kernels.hpp"
#include "psoup/output.hpp"
#include "psoup/pipeline.hpp"
#include "psoup/plan.hpp"
#include "psoup/sigproc.hpp"

namespace py = pybind11;
using namespace psoup;

namespace {

// the Python-facing native candidate list (see the CandidateBag class below)
struct CandidateBag {
  CandidateList c;
};


template <class T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::dict header_to_dict(const SigprocHeader& h) {
  py::dict d;
  d["source_name"] = h.source_name;
  d["rawdatafile"] = h.rawdatafile;
  d["az_start"] = h.az_start;
  d["za_start"] = h.za_start;
  d["src_raj"] = h.src_raj;
  d["src_dej"] = h.src_dej;
  d["tstart"] = h.tstart;
  d["tsamp"] = h.tsamp;
  d["period"] = h.period;
  d["fch1"] = h.fch1;
  d["foff"] = h.foff;
  d["nchans"] = h.nchans;
  d["telescope_id"] = h.telescope_id;
  d["machine_id"] = h.machine_id;
  d["data_type"] = h.data_type;
  d["ibeam"] = h.ibeam;
  d["nbeams"] = h.nbeams;
  d["nbits"] = h.nbits;
  d["barycentric"] = h.barycentric;
  d["pulsarcentric"] = h.pulsarcentric;
  d["nbins"] = h.nbins;
  d["nsamples"] = h.nsamples;
  d["nifs"] = h.nifs;
  d["npuls"] = h.npuls;
  d["refdm"] = h.refdm;
  d["signed"] = static_cast<int>(h.signed_data);
  d["size"] = h.size;
  return d;
}

SigprocHeader dict_to_header(const py::dict& d) {
  SigprocHeader h;
  auto gd = [&](const char* k, double& v) {
    if (d.contains(k)) {
      v = d[k].cast<double>();
      h.keys_present.push_back(k);
    }
  };
  auto gi = [&](const char* k, int& v) {
    if (d.contains(k)) {
      v = d[k].cast<int>();
      h.keys_present.push_back(k);
    }
  };
  if (d.contains("source_name")) h.source_name = d["source_name"].cast<std::string>();
  if (d.contains("rawdatafile")) h.rawdatafile = d["rawdatafile"].cast<std::string>();
  gd("az_start", h.az_start);
  gd("za_start", h.za_start);
  gd("src_raj", h.src_raj);
  gd("src_dej", h.src_dej);
  gd("tstart", h.tstart);
  gd("tsamp", h.tsamp);
  gd("period", h.period);
  gd("fch1", h.fch1);
  gd("foff", h.foff);
  gi("nchans", h.nchans);
  gi("telescope_id", h.telescope_id);
  gi("machine_id", h.machine_id);
  gi("data_type", h.data_type);
  gi("ibeam", h.ibeam);
  gi("nbeams", h.nbeams);
  gi("nbits", h.nbits);
  gi("barycentric", h.barycentric);
  gi("pulsarcentric", h.pulsarcentric);
  gi("nbins", h.nbins);
  gi("nsamples", h.nsamples);
  gi("nifs", h.nifs);
  gi("npuls", h.npuls);
  gd("refdm", h.refdm);
  if (d.contains("signed")) {
    h.signed_data = static_cast<unsigned char>(d["signed"].cast<int>());
    h.keys_present.push_back("signed");
  }
  return h;
}

}  // namespace

void bind_ffa(py::module_& m);  // bind_ffa.cpp

PYBIND11_MODULE(_C, m) {
  m.doc() = "peasoup_amd native core (C++/HIP for gfx950)";
  py::register_exception<psoup::Error>(m, "NativeError", PyExc_RuntimeError);

  // ------------------------------------------------------------ platform --
  m.def("device_count", &device_count);
  m.def("device_info", [](int d) {
    DeviceInfo i = device_info(d);
    py::dict r;
    r["id"] = i.id;
    r["name"] = i.name;
    r["arch"] = i.arch;
    r["major"] = i.major;
    r["minor"] = i.minor;
    r["multiprocessors"] = i.multiprocessors;
    r["total_mem"] = i.total_mem;
    return r;
  });
  m.def("runtime_version", &runtime_version);
  m.def("driver_version", &driver_version);
  m.def("set_log_rank", &set_log_rank);
  m.def("set_log_level", [](int l) { set_log_level(static_cast<LogLevel>(l)); });
  m.def("prev_power_of_two", &prev_power_of_two);
  m.def("roctx_push", [](const std::string& name) { roctx_push(name.c_str()); });
  m.def("roctx_pop", &roctx_pop);

  // ---------------------------------------------------------------- io ----
  m.def("read_header", [](const std::string& f) { return header_to_dict(read_header_file(f)); });
  m.def("read_killfile", [](const std::string& f, int nchans) {
    bool ok = true;
    auto v = read_killfile(f, nchans, &ok);
    return py::make_tuple(v, ok);
  });
  m.def("read_zapfile", [](const std::string& f) {
    std::vector<float> a, b;
    read_zapfile(f, a, b);
    return py::make_tuple(a, b);
  });
  m.def("read_dada_header", [](const std::string& f) {
    DadaHeader h = read_dada_header(f);
    py::dict d;
    d["header_version"] = h.header_version;
    d["header_size"] = h.header_size;
    d["bw"] = h.bw;
    d["freq"] = h.freq;
    d["nant"] = h.nant;
    d["nchan"] = h.nchan;
    d["ndim"] = h.ndim;
    d["npol"] = h.npol;
    d["nbit"] = h.nbit;
    d["tsamp"] = h.tsamp;
    d["osamp_ratio"] = h.osamp_ratio;
    d["source_name"] = h.source_name;
    d["ra"] = h.ra;
    d["dec"] = h.dec;
    d["proc_file"] = h.proc_file;
    d["mode"] = h.mode;
    d["observer"] = h.observer;
    d["pid"] = h.pid;
    d["obs_offset"] = h.obs_offset;
    d["telescope"] = h.telescope;
    d["instrument"] = h.instrument;
    d["dsb"] = h.dsb;
    d["filesize"] = h.filesize;
    d["dada_filesize"] = h.dada_filesize;
    d["nsamples"] = h.nsamples;
    d["bytes_per_sec"] = h.bytes_per_sec;
    d["utc_start"] = h.utc_start;
    d["ant_id"] = h.ant_id;
    d["file_no"] = h.file_no;
    return d;
  });
  m.def("write_filterbank", [](const std::string& f, const py::dict& hdr, py::array_t<uint8_t, py::array::c_style> data) {
    SigprocHeader h = dict_to_header(hdr);
    std::vector<uint8_t> v(data.data(), data.data() + data.size());
    Filterbank fb = Filterbank::from_memory(h, std::move(v));
    fb.write(f);
  });
  m.def("read_tim", [](const std::string& f) {
    TimeSeriesFile t = read_tim(f);
    return py::make_tuple(header_to_dict(t.header), py::array_t<float>(t.data.size(), t.data.data()));
  });
  m.def("write_tim", [](const std::string& f, const py::dict& hdr, const std::vector<float>& data) {
    write_tim(f, dict_to_header(hdr), data);
  });

  py::class_<Filterbank>(m, "Filterbank")
      .def_static("from_file", &Filterbank::from_file)
      .def_property_readonly("header", [](const Filterbank& fb) { return header_to_dict(fb.header()); })
      .def_property_readonly("nsamps", &Filterbank::nsamps)
      .def_property_readonly("nchans", &Filterbank::nchans)
      .def_property_readonly("nbits", &Filterbank::nbits)
      .def_property_readonly("tsamp", &Filterbank::tsamp)
      .def_property_readonly("fch1", &Filterbank::fch1)
      .def_property_readonly("foff", &Filterbank::foff)
      .def_property_readonly("data_bytes", &Filterbank::data_bytes)
      .def_property_readonly("data_address", [](const Filterbank& fb) { return reinterpret_cast<uintptr_t>(fb.data()); })
      .def("cfreq", &Filterbank::cfreq)
      .def(
          "read_into",
          [](const Filterbank& fb, uint64_t off, uint64_t n, uintptr_t dst, int nthreads) {
            fb.read_data(off, n, P<uint8_t>(dst), nthreads);
          },
          py::arg("off"), py::arg("n"), py::arg("dst"), py::arg("nthreads") = 4, py::call_guard<py::gil_scoped_release>())
      .def(
          "upload",
          [](const Filterbank& fb, uintptr_t dptr, uint64_t nbytes, uint64_t dst_bytes, uintptr_t stream) {
            // the first nbytes of the data block -> a device buffer of
            // dst_bytes (threaded pread into two pinned 16 MB stages, copies
            // overlapping the reads); returns when it landed.  0 bytes: no-op
            PSOUP_CHECK(nbytes <= fb.data_bytes(), "upload: more bytes than the data block");
            PSOUP_CHECK(nbytes <= dst_bytes, "upload: more bytes than the destination holds");
            if (nbytes == 0) return;
            auto s = reinterpret_cast<hipStream_t>(stream);
            staged_upload(nbytes, 16ull << 20, [&fb](uint64_t o, uint64_t k, uint8_t* d) { fb.read_data(o, k, d); },
                          P<uint8_t>(dptr), s);
            PSOUP_HIP_CHECK(hipStreamSynchronize(s));
          },
          py::arg("dptr"), py::arg("nbytes"), py::arg("dst_bytes"), py::arg("stream") = 0,
          py::call_guard<py::gil_scoped_release>())
      .def("data", [](const Filterbank& fb) {
        // zero-copy read-only view of the mmapped data block
        py::array_t<uint8_t> a({static_cast<py::ssize_t>(fb.data_bytes())}, {1}, fb.data(), py::cast(fb));
        py::detail::array_proxy(a.ptr())->flags &= ~py::detail::npy_api::NPY_ARRAY_WRITEABLE_;
        return a;
      });

  // -------------------------------------------------------------- plans ---
  m.def("generate_dm_list", &generate_dm_list, py::arg("dm_start"), py::arg("dm_end"), py::arg("tsamp"),
        py::arg("pulse_width_us"), py::arg("fch1"), py::arg("foff"), py::arg("nchans"), py::arg("tol"));
  m.def("generate_delay_table", &generate_delay_table);
  m.def("compute_max_delay", &compute_max_delay);
  py::enum_<AccelConvention>(m, "AccelConvention")
      .value("Legacy", AccelConvention::Legacy)
      .value("Reference", AccelConvention::Reference);
  py::class_<AccelPlan>(m, "AccelPlan")
      .def(py::init<float, float, float, float, uint64_t, float, float, float, AccelConvention>(), py::arg("acc_lo"),
           py::arg("acc_hi"), py::arg("tol"), py::arg("pulse_width"), py::arg("nsamps"), py::arg("tsamp"),
           py::arg("cfreq"), py::arg("bw"), py::arg("convention") = AccelConvention::Legacy)
      .def("generate", &AccelPlan::generate)
      .def("step", &AccelPlan::step);

  // --------------------------------------------------------- candidates ---
  py::class_<Candidate>(m, "Candidate")
      .def(py::init<>())
      .def(py::init<float, int, float, int, float, float>(), py::arg("dm"), py::arg("dm_idx"), py::arg("acc"),
           py::arg("nh"), py::arg("snr"), py::arg("freq"))
      .def_readwrite("dm", &Candidate::dm)
      .def_readwrite("dm_idx", &Candidate::dm_idx)
      .def_readwrite("acc", &Candidate::acc)
      .def_readwrite("nh", &Candidate::nh)
      .def_readwrite("snr", &Candidate::snr)
      .def_readwrite("freq", &Candidate::freq)
      .def_readwrite("folded_snr", &Candidate::folded_snr)
      .def_readwrite("opt_period", &Candidate::opt_period)
      .def_readwrite("is_adjacent", &Candidate::is_adjacent)
      .def_readwrite("is_physical", &Candidate::is_physical)
      .def_readwrite("ddm_count_ratio", &Candidate::ddm_count_ratio)
      .def_readwrite("ddm_snr_ratio", &Candidate::ddm_snr_ratio)
      .def_readwrite("assoc", &Candidate::assoc)
      .def_readwrite("fold", &Candidate::fold)
      .def_readwrite("nbins", &Candidate::nbins)
      .def_readwrite("nints", &Candidate::nints)
      .def("set_fold_array",
           [](Candidate& c, py::array_t<float, py::array::c_style | py::array::forcecast> a, int nbins, int nints) {
             c.fold.assign(a.data(), a.data() + a.size());  // one copy, no per-element conversion
             c.nbins = nbins;
             c.nints = nints;
           },
           py::arg("fold"), py::arg("nbins") = 64, py::arg("nints") = 16)
      .def("count_assoc", &Candidate::count_assoc)
      .def("print", &Candidate::print)
      .def("pods", [](const Candidate& c) {
        std::vector<CandidatePOD> v;
        c.collect_candidates(v);
        py::list out;
        for (auto& p : v) out.append(py::make_tuple(p.dm, p.dm_idx, p.acc, p.nh, p.snr, p.freq));
        return out;
      })
      .def("__repr__", [](const Candidate& c) {
        char b[256];
        std::snprintf(b, sizeof b, "<Candidate P=%.9f dm=%.3f acc=%.2f nh=%d snr=%.2f fsnr=%.2f nassoc=%d>",
                      1.0 / c.freq, c.dm, c.acc, c.nh, c.snr, c.folded_snr, c.count_assoc());
        return std::string(b);
      });
  // A candidate list that stays native: the search's per-DM results, the
  // merged list and the written outputs pass through Python as one handle
  // instead of a Python list of Candidate objects (each conversion of a list
  // deep-copied every candidate's association tree: 1.7M candidates in the
  // config-4 list).  Indexing and iteration give references into the bag
  // (writes such as folded_snr land in it); len, extend (moves the other
  // bag's candidates), permute, truncate and sort_by_dm are native.
  py::class_<CandidateBag, std::shared_ptr<CandidateBag>>(m, "CandidateBag")
      .def(py::init<>())
      .def(py::init([](const py::sequence& seq) {
        auto b = std::make_shared<CandidateBag>();
        b->c.reserve(seq.size());
        for (auto h : seq) b->c.push_back(h.cast<const Candidate&>());
        return b;
      }))
      .def("__len__", [](const CandidateBag& b) { return b.c.size(); })
      .def(
          "__getitem__",
          [](CandidateBag& b, long i) -> Candidate& {
            const long n = static_cast<long>(b.c.size());
            if (i < 0) i += n;
            if (i < 0 || i >= n) throw py::index_error("CandidateBag index out of range");
            return b.c[static_cast<size_t>(i)];
          },
          py::return_value_policy::reference_internal)
      .def(
          "__iter__", [](CandidateBag& b) { return py::make_iterator(b.c.begin(), b.c.end()); },
          py::keep_alive<0, 1>())
      .def("extend",
           [](CandidateBag& b, CandidateBag& o) {
             if (&b == &o) throw std::invalid_argument("CandidateBag.extend: a bag into itself");
             // geometric growth: an exact reserve per call reallocated (and
             // moved every candidate already held) on every extend, so a run
             // that extends a growing bag once per DM block paid O(total) per
             // block (config 4: 1 -> 5 ms of host time per block over the run)
             const size_t need = b.c.size() + o.c.size();
             if (need > b.c.capacity()) b.c.reserve(std::max(need, 2 * b.c.capacity()));
             for (auto& x : o.c) b.c.push_back(std::move(x));
             o.c.clear();
           },
           py::arg("other"), "move every candidate of `other` (left empty) to the end of this bag")
      .def("permute",
           [](CandidateBag& b, const std::vector<int>& order) {
             CandidateList out;
             out.reserve(order.size());
             std::vector<char> seen(b.c.size(), 0);
             for (int i : order) {
               PSOUP_CHECK(i >= 0 && static_cast<size_t>(i) < b.c.size() && !seen[static_cast<size_t>(i)],
                           "CandidateBag.permute: not a permutation");
               seen[static_cast<size_t>(i)] = 1;
               out.push_back(std::move(b.c[static_cast<size_t>(i)]));
             }
             PSOUP_CHECK(out.size() == b.c.size(), "CandidateBag.permute: not a permutation");
             b.c = std::move(out);
           },
           py::arg("order"), "reorder: new[i] = old[order[i]]")
      .def("truncate", [](CandidateBag& b, size_t n) { b.c.resize(std::min(n, b.c.size())); })
      .def("sort_by_dm",
           [](CandidateBag& b) {
             py::gil_scoped_release nogil;
             stable_sort_by_dm_idx(b.c);
           },
           "stable sort by DM index (the merge order of the reference, pipeline_multi.cu:356-365)")
      .def("to_list", [](const CandidateBag& b) { return b.c; });
  m.def("collect_bags", [](SearchEngine& e, const std::shared_ptr<SearchEngine::Pending>& h) {
    std::vector<CandidateList> v;
    {
      py::gil_scoped_release nogil;
      v = e.collect(h);
    }
    std::vector<std::shared_ptr<CandidateBag>> out;
    out.reserve(v.size());
    for (auto& l : v) out.push_back(std::make_shared<CandidateBag>(CandidateBag{std::move(l)}));
    return out;
  }, py::arg("engine"), py::arg("handle"),
     "SearchEngine.collect, the per-job candidate lists as CandidateBags (nothing copied)");
  py::class_<HarmonicDistiller>(m, "HarmonicDistiller")
      .def(py::init<float, float, bool, bool>(), py::arg("tol"), py::arg("max_harm"), py::arg("keep_related"),
           py::arg("fractional_harms") = true)
      .def("distill", &HarmonicDistiller::distill)
      .def("distill_reference", &HarmonicDistiller::distill_reference);
  m.def("accel_distill_slices",
        [](CandidateList all, const std::vector<int>& slices, float tobs, float tol, int nthreads) {
          return accel_distill_slices(std::move(all), slices, AccelerationDistiller(tobs, tol, true), nthreads);
        },
        py::arg("cands"), py::arg("slices"), py::arg("tobs"), py::arg("tol"), py::arg("nthreads") = 4,
        py::call_guard<py::gil_scoped_release>(),
        "join each DM's acceleration slices in slice order and acceleration-distil them (keep related)");
  py::class_<AccelerationDistiller>(m, "AccelerationDistiller")
      .def(py::init<float, float, bool>(), py::arg("tobs"), py::arg("tol"), py::arg("keep_related"))
      .def("distill", &AccelerationDistiller::distill)
      .def("distill_reference", &AccelerationDistiller::distill_reference);
  py::class_<DMDistiller>(m, "DMDistiller")
      .def(py::init<float, bool>(), py::arg("tol"), py::arg("keep_related"))
      .def("distill", &DMDistiller::distill)
      .def("distill_reference", &DMDistiller::distill_reference);
  py::class_<CandidateScorer>(m, "CandidateScorer")
      .def(py::init<float, float, float, float>(), py::arg("tsamp"), py::arg("cfreq"), py::arg("foff"), py::arg("bw"))
      .def("score_all", [](const CandidateScorer& s, CandidateList c) {
        s.score_all(c);
        return c;
      });
  m.def("identify_unique_peaks", [](const std::vector<int>& idxs, const std::vector<float>& snrs, int min_gap) {
    std::vector<int> pi;
    std::vector<float> ps;
    identify_unique_peaks(idxs.data(), snrs.data(), std::min(idxs.size(), snrs.size()), min_gap, pi, ps);
    return py::make_tuple(pi, ps);
  });
  m.def("peak_bounds", [](int nbins, float bin_width, int nh, float min_freq, float max_freq) {
    PeakBounds b = peak_bounds(nbins, bin_width, nh, min_freq, max_freq);
    return py::make_tuple(b.start_idx, b.end_idx, b.factor);
  });
  m.def("sort_by_folded_snr", [](CandidateList c) {
    sort_by_folded_snr(c);
    return c;
  });
  // The permutation sort_by_folded_snr applies, from the keys max(snr,
  // folded_snr) alone: std::sort's result depends only on the comparison
  // outcomes, so reordering a Python list by it equals sorting the list
  // (without converting candidates and their association trees).
  m.def("sort_order_by_folded_snr", [](const std::vector<float>& snr, const std::vector<float>& folded) {
    PSOUP_CHECK(snr.size() == folded.size(), "sort_order_by_folded_snr: size mismatch");
    struct K {
      float v;
      int i;
    };
    std::vector<K> k(snr.size());
    for (size_t i = 0; i < k.size(); ++i) k[i] = K{std::max(snr[i], folded[i]), static_cast<int>(i)};
    std::sort(k.begin(), k.end(), [](const K& x, const K& y) { return x.v > y.v; });
    std::vector<int> order(k.size());
    for (size_t i = 0; i < k.size(); ++i) order[i] = k[i].i;
    return order;
  });
  m.def("serialize_candidates", [](const CandidateBag& b) {
    std::vector<uint8_t> v;
    {
      py::gil_scoped_release nogil;
      v = serialize_candidates(b.c);
    }
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
  });
  // a sequence of Candidate objects, serialised in place: no copy of the
  // trees into a temporary C++ list (candidate-heavy searches carry large
  // keep_related trees)
  m.def("serialize_candidates", [](const py::sequence& seq) {
    std::vector<const Candidate*> p;
    p.reserve(seq.size());
    for (auto h : seq) p.push_back(&h.cast<const Candidate&>());
    std::vector<uint8_t> v;
    {
      py::gil_scoped_release nogil;
      v = serialize_candidates(p);
    }
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
  });
  // The multi-rank merge (pipeline_multi.cu:353-369) in one native call:
  // every rank's serialised candidates (rank order), a stable sort by DM
  // index, then the global DM + harmonic distillation and scoring -- no
  // intermediate Python lists.
  m.def("merge_candidate_blobs", [](const std::vector<py::bytes>& blobs, const CmdLineOptions& args,
                                    const py::dict& hdr) {
    std::vector<std::string> raw;
    raw.reserve(blobs.size());
    for (const auto& b : blobs) raw.push_back(static_cast<std::string>(b));
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    auto out = std::make_shared<CandidateBag>();
    {
      py::gil_scoped_release nogil;
      CandidateList all;
      for (const auto& r : raw) deserialize_candidates_into(reinterpret_cast<const uint8_t*>(r.data()), r.size(), all);
      stable_sort_by_dm_idx(all);
      out->c = global_distill_and_score(std::move(all), args, s);
    }
    return out;
  });
  // The merge from raw buffers ((address, size) of host memory, e.g. the
  // uint8 tensors a gather delivered): no Python bytes objects in between.
  m.def("merge_candidate_buffers", [](const std::vector<std::pair<uintptr_t, size_t>>& bufs,
                                      const CmdLineOptions& args, const py::dict& hdr) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    auto out = std::make_shared<CandidateBag>();
    {
      py::gil_scoped_release nogil;
      CandidateList all;
      for (const auto& [addr, n] : bufs) deserialize_candidates_into(reinterpret_cast<const uint8_t*>(addr), n, all);
      stable_sort_by_dm_idx(all);
      out->c = global_distill_and_score(std::move(all), args, s);
    }
    return out;
  });
  // The merge when DMs' acceleration trials were split over work units
  // (--accel_slices): every buffer holds raw slice lists, slices[i] their
  // per-candidate slice indices (int32, (address, count) of host memory);
  // the slices of each DM are joined in plan order and acceleration-distilled
  // (accel_distill_slices), then the usual global distillation and scoring.
  m.def("merge_split_buffers", [](const std::vector<std::pair<uintptr_t, size_t>>& bufs,
                                  const std::vector<std::pair<uintptr_t, size_t>>& slices, const CmdLineOptions& args,
                                  const py::dict& hdr, int nthreads) {
    PSOUP_CHECK(bufs.size() == slices.size(), "merge_split_buffers: one slice array per buffer");
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    auto out = std::make_shared<CandidateBag>();
    {
      py::gil_scoped_release nogil;
      CandidateList all;
      std::vector<int> sl;
      for (size_t i = 0; i < bufs.size(); ++i) {
        const size_t before = all.size();
        deserialize_candidates_into(reinterpret_cast<const uint8_t*>(bufs[i].first), bufs[i].second, all);
        PSOUP_CHECK(all.size() - before == slices[i].second, "merge_split_buffers: slice count mismatch");
        const int32_t* si = reinterpret_cast<const int32_t*>(slices[i].first);
        sl.insert(sl.end(), si, si + slices[i].second);
      }
      all = accel_distill_slices(std::move(all), sl, search_accel_distiller(s.search), nthreads);
      stable_sort_by_dm_idx(all);
      out->c = global_distill_and_score(std::move(all), args, s);
    }
    return out;
  }, py::arg("bufs"), py::arg("slices"), py::arg("args"), py::arg("header"), py::arg("nthreads") = 8);
  m.def("merge_split_local", [](CandidateBag& local, const std::vector<int>& slices, const CmdLineOptions& args,
                                const py::dict& hdr, int nthreads) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    auto out = std::make_shared<CandidateBag>();
    {
      py::gil_scoped_release nogil;
      CandidateList all = std::move(local.c);
      local.c.clear();
      all = accel_distill_slices(std::move(all), slices, search_accel_distiller(s.search), nthreads);
      stable_sort_by_dm_idx(all);
      out->c = global_distill_and_score(std::move(all), args, s);
    }
    return out;
  }, py::arg("local"), py::arg("slices"), py::arg("args"), py::arg("header"), py::arg("nthreads") = 8);
  // serialised into a uint8 numpy array that owns the bytes (torch.from_numpy
  // takes it without a copy)
  m.def("serialize_candidates_array", [](const CandidateBag& b) {
    auto* v = new std::vector<uint8_t>();
    {
      py::gil_scoped_release nogil;
      *v = serialize_candidates(b.c);
    }
    py::capsule owner(v, [](void* p) { delete static_cast<std::vector<uint8_t>*>(p); });
    return py::array_t<uint8_t>({static_cast<py::ssize_t>(v->size())}, {static_cast<py::ssize_t>(1)}, v->data(),
                                owner);
  });
  // The same merge of one rank's own candidates (a world of one): no
  // serialisation; `local` is consumed (left empty).
  m.def("merge_local", [](CandidateBag& local, const CmdLineOptions& args, const py::dict& hdr) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    auto out = std::make_shared<CandidateBag>();
    {
      py::gil_scoped_release nogil;
      CandidateList all = std::move(local.c);
      local.c.clear();
      stable_sort_by_dm_idx(all);
      out->c = global_distill_and_score(std::move(all), args, s);
    }
    return out;
  });
  m.def("deserialize_candidates", [](py::buffer b) {
    py::buffer_info info = b.request();
    return deserialize_candidates(static_cast<const uint8_t*>(info.ptr), static_cast<size_t>(info.size * info.itemsize));
  });
  m.def("deserialize_candidates_at", [](uintptr_t addr, size_t n) {
    return deserialize_candidates(reinterpret_cast<const uint8_t*>(addr), n);
  });

  // ----------------------------------------------------------------- cli --
  py::class_<CmdLineOptions>(m, "CmdLineOptions")
      .def(py::init<>())
      .def_readwrite("infilename", &CmdLineOptions::infilename)
      .def_readwrite("outdir", &CmdLineOptions::outdir)
      .def_readwrite("killfilename", &CmdLineOptions::killfilename)
      .def_readwrite("zapfilename", &CmdLineOptions::zapfilename)
      .def_readwrite("max_num_threads", &CmdLineOptions::max_num_threads)
      .def_readwrite("limit", &CmdLineOptions::limit)
      .def_readwrite("size", &CmdLineOptions::size)
      .def_readwrite("dm_start", &CmdLineOptions::dm_start)
      .def_readwrite("dm_end", &CmdLineOptions::dm_end)
      .def_readwrite("dm_tol", &CmdLineOptions::dm_tol)
      .def_readwrite("dm_pulse_width", &CmdLineOptions::dm_pulse_width)
      .def_readwrite("acc_start", &CmdLineOptions::acc_start)
      .def_readwrite("acc_end", &CmdLineOptions::acc_end)
      .def_readwrite("acc_tol", &CmdLineOptions::acc_tol)
      .def_readwrite("acc_pulse_width", &CmdLineOptions::acc_pulse_width)
      .def_readwrite("boundary_5_freq", &CmdLineOptions::boundary_5_freq)
      .def_readwrite("boundary_25_freq", &CmdLineOptions::boundary_25_freq)
      .def_readwrite("nharmonics", &CmdLineOptions::nharmonics)
      .def_readwrite("npdmp", &CmdLineOptions::npdmp)
      .def_readwrite("min_snr", &CmdLineOptions::min_snr)
      .def_readwrite("min_freq", &CmdLineOptions::min_freq)
      .def_readwrite("max_freq", &CmdLineOptions::max_freq)
      .def_readwrite("max_harm", &CmdLineOptions::max_harm)
      .def_readwrite("freq_tol", &CmdLineOptions::freq_tol)
      .def_readwrite("verbose", &CmdLineOptions::verbose)
      .def_readwrite("progress_bar", &CmdLineOptions::progress_bar)
      .def_readwrite("accel_convention", &CmdLineOptions::accel_convention)
      .def_readwrite("dedisp_kernel", &CmdLineOptions::dedisp_kernel)
      .def_readwrite("accel_batch", &CmdLineOptions::accel_batch)
      .def_readwrite("engines_per_gpu", &CmdLineOptions::engines_per_gpu)
      .def_readwrite("dm_schedule", &CmdLineOptions::dm_schedule)
      .def_readwrite("accel_slices", &CmdLineOptions::accel_slices)
      .def_readwrite("sub_batch", &CmdLineOptions::sub_batch)
      .def_readwrite("fft_mode", &CmdLineOptions::fft_mode)
      .def_readwrite("use_boundaries", &CmdLineOptions::use_boundaries)
      .def_readwrite("checkpoint_dir", &CmdLineOptions::checkpoint_dir)
      .def_readwrite("trace_json", &CmdLineOptions::trace_json)
      .def_readwrite("fault_after_dms", &CmdLineOptions::fault_after_dms)
      .def_readwrite("time_shards", &CmdLineOptions::time_shards);
  m.def("parse_cmdline", [](const std::vector<std::string>& argv) {
    CmdLineOptions a;
    bool exit_now = false;
    bool ok = parse_cmdline(a, argv, &exit_now);
    return py::make_tuple(ok, exit_now, a);
  });
  m.def("cmdline_usage", &cmdline_usage);
  m.def("default_outdir", &default_outdir);
  py::class_<CoincidencerOptions>(m, "CoincidencerOptions")
      .def(py::init<>())
      .def_readwrite("filterbanks", &CoincidencerOptions::filterbanks)
      .def_readwrite("samp_outfilename", &CoincidencerOptions::samp_outfilename)
      .def_readwrite("spec_outfilename", &CoincidencerOptions::spec_outfilename)
      .def_readwrite("threshold", &CoincidencerOptions::threshold)
      .def_readwrite("beam_threshold", &CoincidencerOptions::beam_threshold)
      .def_readwrite("nharmonics", &CoincidencerOptions::nharmonics)
      .def_readwrite("verbose", &CoincidencerOptions::verbose);
  m.def("parse_coincidencer_cmdline", [](const std::vector<std::string>& argv) {
    CoincidencerOptions a;
    bool exit_now = false;
    std::vector<const char*> cv;
    for (auto& s : argv) cv.push_back(s.c_str());
    bool ok = parse_coincidencer_cmdline(a, static_cast<int>(cv.size()), cv.data(), &exit_now);
    return py::make_tuple(ok, exit_now, a);
  });

  // -------------------------------------------------------------- output --
  m.def("xml_fmt_float", [](float v) { return xml::fmt(v); });
  m.def("xml_fmt_double", [](double v) { return xml::fmt(v); });
  m.def("write_candidates_binary", [](const std::string& outdir, const CandidateBag& b, const std::string& fname) {
    CandidateFileWriter w(outdir);
    w.write_binary(b.c, fname);
    std::map<unsigned, long> bm = w.byte_mapping;
    return bm;
  });
  m.def("write_candidates_binary", [](const std::string& outdir, const CandidateList& c, const std::string& fname) {
    CandidateFileWriter w(outdir);
    w.write_binary(c, fname);
    std::map<unsigned, long> bm = w.byte_mapping;
    return bm;
  });
  m.def("write_candidates_binaries", [](const std::string& outdir, const CandidateList& c) {
    CandidateFileWriter w(outdir);
    if (!w.write_binaries(c)) throw std::runtime_error("write_binaries failed in " + outdir);
    std::map<unsigned, std::string> names = w.filenames;
    return names;
  });
  m.def("write_candidate_text_files", &write_candidate_text_files);
  m.def("write_candidate_file", &write_candidate_file);
  m.def(
      "write_overview",
      [](const std::string& path, const CmdLineOptions& args, const py::object& header_file, const std::vector<float>& dms,
         const std::vector<float>& accs, const std::vector<int>& devices, const py::object& cands_obj,
         const std::map<unsigned, long>& byte_map, const std::map<std::string, double>& timers,
         const std::map<std::string, double>& perf) {
        OverviewWriter ow;
        ow.add_misc_info();
        if (py::isinstance<py::str>(header_file)) ow.add_header(header_file.cast<std::string>());
        else ow.add_header(dict_to_header(header_file.cast<py::dict>()));
        ow.add_search_parameters(args);
        ow.add_dm_list(dms);
        ow.add_acc_list(accs);
        if (!devices.empty()) ow.add_gpu_info(devices);
        if (py::isinstance<CandidateBag>(cands_obj))
          ow.add_candidates(cands_obj.cast<const CandidateBag&>().c, byte_map);
        else
          ow.add_candidates(cands_obj.cast<CandidateList>(), byte_map);
        ow.add_timing_info(timers);
        if (!perf.empty()) ow.add_performance(perf);
        ow.to_file(path);
      },
      py::arg("path"), py::arg("args"), py::arg("header"), py::arg("dms"), py::arg("accs"), py::arg("devices"),
      py::arg("cands"), py::arg("byte_map"), py::arg("timers"), py::arg("perf"));

  // ------------------------------------------------------------- kernels --
  bind_ffa(m);

  py::module_ k = m.def_submodule("kernels", "raw HIP kernel launchers (addresses + stream handles)");
  k.def("unpack_transpose", [](uintptr_t packed, uint64_t nsamps, int nchans, int nbits, uintptr_t out,
                               uint64_t out_stride, int bias, uintptr_t s) {
    kern::unpack_transpose(P<const uint8_t>(packed), nsamps, nchans, nbits, P<int8_t>(out), out_stride, bias, S(s));
  });
  k.def("dedisperse_direct", [](uintptr_t x, uint64_t stride, int nchans, uintptr_t offsets, uintptr_t kill, int ndm,
                                uint64_t out_nsamps, uintptr_t out, uint64_t out_stride, float scale, int bias,
                                int nactive, uintptr_t s) {
    kern::dedisperse_direct(P<const int8_t>(x), stride, nchans, P<const int32_t>(offsets), P<const int32_t>(kill), ndm,
                            out_nsamps, P<uint8_t>(out), out_stride, scale, bias, nactive, S(s));
  });
  k.def("u8_to_f32_pad", [](uintptr_t in, uint64_t nvalid, uintptr_t out, uint64_t n, uintptr_t sum, uintptr_t s) {
    kern::u8_sum(P<const uint8_t>(in), nvalid, P<unsigned long long>(sum), S(s));
    kern::u8_to_f32_pad(P<const uint8_t>(in), nvalid, P<float>(out), n, P<const unsigned long long>(sum), S(s));
  });
  k.def("f32_stats", [](uintptr_t x, uint64_t n, uintptr_t partials, int np, uintptr_t stats, uintptr_t s) {
    kern::f32_stats(P<const float>(x), n, P<double>(partials), np, P<float>(stats), S(s));
  });
  k.def("form_amplitude", [](uintptr_t X, uint64_t nb, uintptr_t out, uintptr_t s) {
    kern::form_amplitude(P<const float2>(X), nb, P<float>(out), S(s));
  });
  k.def("form_interbin", [](uintptr_t X, uint64_t nb, uintptr_t out, uintptr_t s) {
    kern::form_interbin(P<const float2>(X), nb, P<float>(out), S(s));
  });
  k.def("normalise", [](uintptr_t x, uint64_t n, float mean, float sigma, uintptr_t s) {
    kern::normalise(P<float>(x), n, mean, sigma, S(s));
  });
  k.def("median5_amp", [](uintptr_t X, uint64_t nb, uintptr_t out, uintptr_t s) {
    kern::median5_amp(P<const float2>(X), nb, P<float>(out), S(s));
  });
  k.def("median5", [](uintptr_t in, uint64_t count, uintptr_t out, uintptr_t s) {
    kern::median5(P<const float>(in), count, P<float>(out), S(s));
  });
  k.def("deredden_zap", [](uintptr_t X, uint64_t nb, uintptr_t m5, uint64_t n5, uintptr_t m25, uint64_t n25,
                           uintptr_t m125, uint64_t n125, int64_t pos5, int64_t pos25, uintptr_t zap, uintptr_t s) {
    kern::deredden_zap(P<float2>(X), nb, P<const float>(m5), n5, P<const float>(m25), n25, P<const float>(m125), n125,
                       pos5, pos25, P<const uint32_t>(zap), S(s));
  });
  k.def("interbin_stats", [](uintptr_t X, uint64_t nb, uintptr_t Pout, uintptr_t partials, int np, uintptr_t stats,
                             uintptr_t s) {
    kern::interbin_stats(P<const float2>(X), nb, P<float>(Pout), P<double>(partials), np, P<float>(stats), S(s));
  });
  k.def("resample_batch", [](uintptr_t in, uint64_t n, uintptr_t out, uint64_t ostride, uintptr_t af, int K,
                             uintptr_t s) {
    kern::resample_batch(P<const float>(in), n, P<float>(out), ostride, P<const double>(af), K, S(s));
  });
  k.def("resample_v1", [](uintptr_t in, uint64_t n, uintptr_t out, double af, uintptr_t s) {
    kern::resample_v1(P<const float>(in), n, P<float>(out), af, S(s));
  });
  k.def("interbin_normalise_batch", [](uintptr_t X, uint64_t nb, uint64_t xstride, uintptr_t Pout, uint64_t pstride,
                                       int K, uint64_t nbo, uintptr_t stats, float nscale, uintptr_t s) {
    kern::interbin_normalise_batch(P<const float2>(X), nb, xstride, P<float>(Pout), pstride, K, nbo,
                                   P<const float>(stats), nscale, S(s));
  });
  k.def("r2c_interbin_normalise_batch", [](uintptr_t Z, uint64_t M, uint64_t zstride, int log2_row,
                                           uint64_t row_pitch, uint64_t blk_pitch, int log2_blk, uintptr_t Pout,
                                           uint64_t pstride, int K, uint64_t nbo, uintptr_t stats, float nscale,
                                           uintptr_t s) {
    kern::r2c_interbin_normalise_batch(P<const float2>(Z), M, zstride, log2_row, row_pitch, blk_pitch, log2_blk,
                                       P<float>(Pout), pstride, K, nbo, P<const float>(stats), nscale, S(s));
  });
  k.def(
      "r2c_interbin_normalise_rows",
      [](uintptr_t Z, uint64_t zp, uint64_t zstride, int log2_n2, uint64_t n1, uintptr_t Pout, uint64_t pstride, int K,
         uint64_t nbo, uintptr_t stats, float nscale, uintptr_t s, uintptr_t q, uint64_t qstride) {
        kern::r2c_interbin_normalise_rows(P<const float2>(Z), zp, zstride, log2_n2, n1, P<float>(Pout), pstride, K,
                                          nbo, P<const float>(stats), nscale, S(s), nullptr, P<uint8_t>(q), qstride);
      },
      py::arg("Z"), py::arg("zp"), py::arg("zstride"), py::arg("log2_n2"), py::arg("n1"), py::arg("P"),
      py::arg("pstride"), py::arg("K"), py::arg("nbo"), py::arg("stats"), py::arg("nscale"), py::arg("s"),
      py::arg("q") = 0, py::arg("qstride") = 0);
  k.def("fft4_x_layout", [](const kern::Fft4Geom& g) {
    kern::Fft4XLayout l = kern::fft4_x_layout(g);
    return py::make_tuple(l.log2_row, l.row_pitch, l.blk_pitch, l.log2_blk, l.tiled);
  });
  k.def(
      "r2c_interbin_normalise_tiled",
      [](uintptr_t X, int n1, int n2, uint64_t xstride, uintptr_t Pout, uint64_t pstride, int K, uint64_t nbo,
         uintptr_t stats, float nscale, uintptr_t s, uintptr_t q, uint64_t qstride) {
        kern::r2c_interbin_normalise_tiled(P<const float2>(X), n1, n2, xstride, P<float>(Pout), pstride, K, nbo,
                                           P<const float>(stats), nscale, S(s), nullptr, P<uint8_t>(q), qstride);
      },
      py::arg("X"), py::arg("n1"), py::arg("n2"), py::arg("xstride"), py::arg("P"), py::arg("pstride"), py::arg("K"),
      py::arg("nbo"), py::arg("stats"), py::arg("nscale"), py::arg("s"), py::arg("q") = 0, py::arg("qstride") = 0);
  m.def("warm_device", &warm_device,
        "load every kernel module's code object on the current device (a no-op launch each); seconds taken");
  k.def("quantize_q8", [](uintptr_t Pin, uint64_t pstride, uint64_t n, int K, uintptr_t q, uint64_t qstride,
                          uintptr_t s) { kern::quantize_q8(P<const float>(Pin), pstride, n, K, P<uint8_t>(q), qstride, S(s)); });
  py::class_<kern::Fft4Geom>(k, "Fft4Geom")
      .def_readonly("ok", &kern::Fft4Geom::ok)
      .def_readonly("n1", &kern::Fft4Geom::n1)
      .def_readonly("n2", &kern::Fft4Geom::n2)
      .def_readonly("ypitch", &kern::Fft4Geom::ypitch)
      .def_readonly("ystride", &kern::Fft4Geom::ystride)
      .def_readonly("xpitch", &kern::Fft4Geom::xpitch)
      .def_readonly("xstride", &kern::Fft4Geom::xstride)
      .def_readonly("log2_xrow", &kern::Fft4Geom::log2_xrow)
      .def_readonly("inpitch", &kern::Fft4Geom::inpitch)
      .def_readonly("insize", &kern::Fft4Geom::insize)
      .def_readwrite("ypair", &kern::Fft4Geom::ypair)
      .def_readonly("rows_ext", &kern::Fft4Geom::rows_ext);
  k.def("fft4_pair_y", &kern::fft4_pair_y);
  k.def("fft4_geometry", &kern::fft4_geometry);
  k.def("fft4_geometry_rows", &kern::fft4_geometry_rows);
  k.def("fft4_set_flags", &kern::fft4_set_flags);
  k.def("peak_cluster_set_trace",
        [](uintptr_t p) { kern::peak_cluster_set_trace(reinterpret_cast<unsigned long long*>(p)); });
  k.def("fft4_set_trace", [](uintptr_t p) { kern::fft4_set_trace(reinterpret_cast<unsigned long long*>(p)); });
  k.def("fft4_flags", &kern::fft4_flags);
  k.def("fft4_tables", [](const kern::Fft4Geom& g) {
    auto t = kern::fft4_tables(g);
    py::array_t<float> a({static_cast<py::ssize_t>(t.size()), static_cast<py::ssize_t>(2)});
    std::memcpy(a.mutable_data(), t.data(), t.size() * sizeof(float2));
    return a;
  });
  k.def("fft4_pad_input", [](uintptr_t in, uint64_t n, uintptr_t out, const kern::Fft4Geom& g, uintptr_t s) {
    kern::fft4_pad_input(P<const float>(in), n, P<float>(out), g, S(s));
  });
  k.def("fft4_resample_colpass", [](uintptr_t in, uintptr_t in_pad, uint64_t n, uintptr_t af, int K, uintptr_t Y,
                                    const kern::Fft4Geom& g, uintptr_t tab, uintptr_t s) {
    kern::fft4_resample_colpass(P<const float>(in), P<const float>(in_pad), n, P<const double>(af), K, P<float2>(Y),
                                g, P<const float2>(tab), S(s));
  });
  k.def(
      "fft4_rowpass",
      [](uintptr_t Y, uintptr_t X, int K, const kern::Fft4Geom& g, uintptr_t tab, uintptr_t s, uint64_t nbins_out) {
        kern::fft4_rowpass(P<const float2>(Y), P<float2>(X), K, g, P<const float2>(tab), S(s), nbins_out);
      },
      py::arg("Y"), py::arg("X"), py::arg("K"), py::arg("g"), py::arg("tab"), py::arg("s"), py::arg("nbins_out") = 0);
  k.def(
      "fft4_rowpass_spectrum",
      [](uintptr_t Y, int K, const kern::Fft4Geom& g, uintptr_t tab, uintptr_t Pout, uint64_t pstride, uintptr_t q,
         uint64_t qstride, uintptr_t stats, float nscale, uintptr_t s, uintptr_t tsrc, uint32_t nbins) {
        kern::SpecOut o;
        o.nbins = nbins;
        o.P = P<float>(Pout);
        o.pstride = pstride;
        o.Q = P<uint8_t>(q);
        o.qstride = qstride;
        o.stats = P<const float>(stats);
        o.tsrc = P<const uint32_t>(tsrc);
        o.nscale = nscale;
        kern::fft4_rowpass_spectrum(P<const float2>(Y), K, g, P<const float2>(tab), o, S(s));
      },
      py::arg("Y"), py::arg("K"), py::arg("g"), py::arg("tab"), py::arg("P"), py::arg("pstride"), py::arg("q"),
      py::arg("qstride"), py::arg("stats"), py::arg("nscale"), py::arg("s"), py::arg("tsrc") = 0,
      py::arg("nbins") = 0);
  k.attr("spec_q_shift") = kern::kSpecQShift;
  k.def("spec_pblk_index", &kern::spec_pblk_index);
  k.def("r2c_tiled_row_blocks", &kern::r2c_tiled_row_blocks);
  k.def("harmonic_peaks_batch", [](uintptr_t Pin, uint64_t nb, uint64_t pstride, int K, int nlevels,
                                   const std::vector<int>& start, const std::vector<int>& end, float thresh,
                                   uint32_t capacity, uintptr_t out, uintptr_t count, uintptr_t s, uintptr_t q,
                                   uint64_t qstride, int pblk_log2_n2, uint32_t pblk_n1, int qshift, int region_log2) {
    kern::HarmParams hp{};
    hp.region_log2 = region_log2;
    hp.nlevels = nlevels;
    for (int i = 0; i < 6; ++i) {
      hp.start[i] = i < static_cast<int>(start.size()) ? start[i] : 0;
      hp.end[i] = i < static_cast<int>(end.size()) ? end[i] : 0;
    }
    hp.thresh = thresh;
    hp.capacity = capacity;
    kern::HarmFromX fx;
    fx.pblk = pblk_n1 > 0 ? 1 : 0;
    fx.log2_n2 = pblk_log2_n2;
    fx.n1 = pblk_n1;
    fx.qshift = qshift;
    kern::harmonic_peaks_batch(P<const float>(Pin), nb, pstride, K, hp, P<kern::PeakRecord>(out), P<uint32_t>(count),
                               S(s), P<const uint8_t>(q), qstride, pblk_n1 > 0 ? &fx : nullptr);
  }, py::arg("P"), py::arg("nb"), py::arg("pstride"), py::arg("K"), py::arg("nlevels"), py::arg("start"),
     py::arg("end"), py::arg("thresh"), py::arg("capacity"), py::arg("out"), py::arg("count"), py::arg("s"),
     py::arg("q") = 0, py::arg("qstride") = 0, py::arg("pblk_log2_n2") = 0, py::arg("pblk_n1") = 0,
     py::arg("qshift") = 0, py::arg("region_log2") = 0);
  k.def("peak_cluster_batch", [](uintptr_t peaks, uintptr_t count, uint32_t cap, uint32_t nseg, int gap,
                                 uintptr_t work, uintptr_t sorted, uintptr_t out, uintptr_t segtab, uintptr_t total,
                                 uintptr_t s, int region_log2) {
    kern::peak_cluster_batch(P<const kern::PeakRecord>(peaks), P<const uint32_t>(count), cap, nseg, gap,
                             P<uint32_t>(work), P<uint2>(sorted), P<uint2>(out), P<uint2>(segtab), P<uint32_t>(total),
                             S(s), region_log2);
  }, py::arg("peaks"), py::arg("count"), py::arg("cap"), py::arg("nseg"), py::arg("gap"), py::arg("work"),
     py::arg("sorted"), py::arg("out"), py::arg("segtab"), py::arg("total"), py::arg("s"), py::arg("region_log2") = 0);
  k.def("peak_regions_total", [](uintptr_t rcount, int region_log2, uint32_t cap, uintptr_t total, uintptr_t s) {
    kern::peak_regions_total(P<const uint32_t>(rcount), region_log2, cap, P<uint32_t>(total), S(s));
  });
  k.attr("peak_region_stride") = kern::kPeakRegionStride;
  k.attr("cluster_cap") = kern::kClusterCap;
  k.def("harm_distill_batch", [](uintptr_t clust, uintptr_t segtab, int ntrials, int nlevels,
                                 const std::vector<double>& factor, float tol, float max_harm, uintptr_t out,
                                 uintptr_t ttab, uintptr_t total, uintptr_t s) {
    kern::HarmDistillParams p{};
    p.nlevels = nlevels;
    PSOUP_CHECK(static_cast<int>(factor.size()) >= nlevels + 1, "harm_distill_batch: one factor per level");
    for (int h = 0; h <= nlevels; ++h) p.factor[h] = factor[static_cast<size_t>(h)];
    p.tol = tol;
    p.max_harm = max_harm;
    p.lower_tol = 1 - tol;
    p.upper_tol = 1 + tol;
    kern::harm_distill_batch(P<const uint2>(clust), P<const uint2>(segtab), ntrials, p, P<uint2>(out), P<uint2>(ttab),
                             P<uint32_t>(total), S(s));
  });
  k.attr("harm_cap") = kern::kHarmCap;
  k.def("harmonic_sums", [](uintptr_t Pin, uint64_t nb, int nlevels, uintptr_t out, uintptr_t s) {
    kern::harmonic_sums(P<const float>(Pin), nb, nlevels, P<float>(out), S(s));
  });
  k.def("harmonic_set_flags", &kern::harmonic_set_flags);
  k.def("harmonic_flags", &kern::harmonic_flags);
  k.def("ffa_downsample", [](uintptr_t x, uint64_t n, double f, uintptr_t out, uint64_t nout, uintptr_t s) {
    kern::ffa_downsample(P<const float>(x), n, f, P<float>(out), nout, S(s));
  });
  k.def("ffa_detrend", [](uintptr_t in, uint64_t n, uint64_t window, uintptr_t sums, uintptr_t means, uintptr_t out,
                          uintptr_t s) {
    kern::ffa_detrend(P<const uint8_t>(in), n, window, P<unsigned long long>(sums), P<float>(means), P<float>(out),
                      S(s));
  });
  k.def("fold_shift_table", [](uintptr_t table, int nbins, int nints, uintptr_t s) {
    kern::fold_shift_table(P<float2>(table), nbins, nints, S(s));
  });
  k.def("fold_optimise", [](uintptr_t folds, int nfold, uintptr_t table, uintptr_t opt_fold, uintptr_t opt_prof,
                            uintptr_t opt_int, uintptr_t opt_val, uintptr_t s) {
    kern::fold_optimise(P<const float>(folds), nfold, P<const float2>(table), P<float>(opt_fold), P<float>(opt_prof),
                        P<int32_t>(opt_int), P<float>(opt_val), S(s));
  });
  k.def("count_above", [](uintptr_t x, uint64_t n, float thresh, uintptr_t counts, uintptr_t s) {
    kern::count_above(P<const float>(x), n, thresh, P<uint8_t>(counts), S(s));
  });
  k.def("coincidence_mask", [](uintptr_t counts, uint64_t n, int beam_thresh, uintptr_t mask, uintptr_t s) {
    kern::coincidence_mask(P<const uint8_t>(counts), n, beam_thresh, P<float>(mask), S(s));
  });
  k.def("conjugate", [](uintptr_t x, uint64_t n, uintptr_t s) { kern::conjugate(P<float2>(x), n, S(s)); });
  k.def("cmul_inplace", [](uintptr_t x, uintptr_t y, uint64_t n, uintptr_t s) {
    kern::cmul_inplace(P<const float2>(x), P<float2>(y), n, S(s));
  });

  // ------------------------------------------------------------- fft ------
  py::enum_<FftType>(m, "FftType")
      .value("R2C", FftType::R2C)
      .value("C2R", FftType::C2R)
      .value("C2C_FWD", FftType::C2C_FWD)
      .value("C2C_INV", FftType::C2C_INV);
  py::class_<FftPlan>(m, "FftPlan")
      .def(py::init<FftType, uint64_t, uint64_t, uint64_t, uint64_t, bool, uint64_t, uint64_t>(), py::arg("type"),
           py::arg("n"), py::arg("batch") = 1, py::arg("in_dist") = 0, py::arg("out_dist") = 0,
           py::arg("inplace") = false, py::arg("in_stride") = 1, py::arg("out_stride") = 1)
      .def("execute", [](FftPlan& p, uintptr_t in, uintptr_t out, uintptr_t s) { p.execute(P<void>(in), P<void>(out), S(s)); })
      .def_property_readonly("work_bytes", &FftPlan::work_bytes);

  // ------------------------------------------------------------- engine ---
  py::enum_<DedispKernel>(m, "DedispKernel")
      .value("Auto", DedispKernel::Auto)
      .value("Direct", DedispKernel::Direct)
      .value("Mfma", DedispKernel::Mfma)
      .value("Valu", DedispKernel::Valu)
      .value("Packed2", DedispKernel::Packed2);
  py::class_<DedispGeometry>(m, "DedispGeometry")
      .def_static("make", [](const py::dict& hdr, uint64_t nsamps, const std::vector<float>& dms,
                             const std::vector<int>& kill) { return DedispGeometry::make(dict_to_header(hdr), nsamps, dms, kill); })
      .def_readonly("nchans", &DedispGeometry::nchans)
      .def_readonly("nbits", &DedispGeometry::nbits)
      .def_readonly("nsamps", &DedispGeometry::nsamps)
      .def_readonly("dm_list", &DedispGeometry::dm_list)
      .def_readonly("delays", &DedispGeometry::delays)
      .def_readonly("killmask", &DedispGeometry::killmask)
      .def_readonly("max_delay", &DedispGeometry::max_delay)
      .def_readonly("out_nsamps", &DedispGeometry::out_nsamps)
      .def_readonly("out_scale", &DedispGeometry::out_scale)
      .def_readonly("bias", &DedispGeometry::bias)
      .def_readonly("nactive", &DedispGeometry::nactive)
      .def("offsets", &DedispGeometry::offsets);
  py::class_<DeviceFilterbank>(m, "DeviceFilterbank")
      .def(py::init([](const DedispGeometry& g, uintptr_t s) { return new DeviceFilterbank(g, S(s)); }),
           py::keep_alive<1, 2>())
      .def("load_packed_device", [](DeviceFilterbank& f, uintptr_t p) { f.load_packed_device(P<const uint8_t>(p)); })
      .def("load_packed_host", [](DeviceFilterbank& f, uintptr_t p) { f.load_packed_host(P<const uint8_t>(p)); },
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("data_address", [](const DeviceFilterbank& f) { return reinterpret_cast<uintptr_t>(f.data()); })
      .def_property_readonly("stride", &DeviceFilterbank::stride);
  // Native stream / event handles: ordering between the engine's stream and a
  // side stream is expressed with these (HIP semantics end to end) rather than
  // through torch's stream objects.
  py::class_<Stream>(m, "GpuStream")
      .def(py::init<>())
      .def_property_readonly("handle", [](const Stream& s) { return reinterpret_cast<uintptr_t>(s.get()); })
      .def("synchronize", &Stream::sync, py::call_guard<py::gil_scoped_release>());
  m.def("stream_synchronize", [](uintptr_t s) { PSOUP_HIP_CHECK(hipStreamSynchronize(S(s))); },
        py::call_guard<py::gil_scoped_release>());
  py::class_<Event>(m, "GpuEvent")
      .def(py::init<bool>(), py::arg("timing") = false)
      .def("record", [](Event& e, uintptr_t s) { e.record(S(s)); })
      .def("wait", [](Event& e, uintptr_t s) { PSOUP_HIP_CHECK(hipStreamWaitEvent(S(s), e.get(), 0)); },
           py::arg("stream"), "make `stream` wait for the last record of this event")
      .def("synchronize", &Event::sync, py::call_guard<py::gil_scoped_release>())
      .def("elapsed_ms", [](const Event& a, const Event& b) {
        float ms = 0.f;
        PSOUP_HIP_CHECK(hipEventElapsedTime(&ms, a.get(), b.get()));
        return ms;
      });
  py::class_<Dedisperser>(m, "Dedisperser")
      .def(py::init([](const DeviceFilterbank& fb, uintptr_t s) { return new Dedisperser(fb, S(s)); }),
           py::keep_alive<1, 2>())
      .def("run", [](Dedisperser& d, int d0, int d1, uintptr_t out, uint64_t ostride, DedispKernel k, uintptr_t s) {
        d.run(d0, d1, P<uint8_t>(out), ostride, k, S(s));
      }, py::arg("d0"), py::arg("d1"), py::arg("out"), py::arg("out_stride"), py::arg("kind") = DedispKernel::Auto,
           py::arg("stream") = 0, py::call_guard<py::gil_scoped_release>())
      .def("run_list", [](Dedisperser& d, const std::vector<int>& dms, uintptr_t out, uint64_t ostride, uintptr_t s) {
        d.run_list(dms, P<uint8_t>(out), ostride, S(s));
      }, py::arg("dms"), py::arg("out"), py::arg("out_stride"), py::arg("stream") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def_static("row_stride", &Dedisperser::row_stride)
      .def("choose", &Dedisperser::choose, py::arg("d0"), py::arg("d1"))
      .def("mfma_steps_per_channel", &Dedisperser::mfma_steps_per_channel, py::arg("d0"), py::arg("d1"))
      .def("mfma_lds_split", &Dedisperser::mfma_lds_split, py::arg("d0"), py::arg("d1"))
      .def("warm", &Dedisperser::warm, py::arg("d0") = 0, py::arg("d1") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly_static("tile_dms", [](py::object) { return Dedisperser::kTileDms; });

  py::class_<Whitener>(m, "Whitener")
      .def(py::init([](uint64_t n, float tsamp, uintptr_t s, bool f4) { return new Whitener(n, tsamp, S(s), f4); }),
           py::arg("n"), py::arg("tsamp"), py::arg("stream"), py::arg("allow_fft4") = true)
      .def("forward", [](Whitener& w, uintptr_t x, uintptr_t X) { w.forward(P<const float>(x), P<float2>(X)); })
      .def("inverse", [](Whitener& w, uintptr_t X, uintptr_t x) { w.inverse(P<const float2>(X), P<float>(x)); })
      .def("whiten", [](Whitener& w, uintptr_t x, bool stats) { w.whiten(P<float>(x), nullptr, stats, 0.05f, 0.5f); },
           py::arg("series"), py::arg("with_stats") = true)
      .def_property_readonly("uses_fft4", &Whitener::uses_fft4)
      .def_property_readonly("mixed_radix", &Whitener::mixed_radix)
      .def_property_readonly("nbins", &Whitener::nbins);
  py::class_<SearchParams>(m, "SearchParams")
      .def(py::init<>())
      .def_readwrite("fft_size", &SearchParams::fft_size)
      .def_readwrite("tsamp", &SearchParams::tsamp)
      .def_readwrite("min_snr", &SearchParams::min_snr)
      .def_readwrite("host_threads", &SearchParams::host_threads)
      .def_readwrite("min_freq", &SearchParams::min_freq)
      .def_readwrite("max_freq", &SearchParams::max_freq)
      .def_readwrite("nharmonics", &SearchParams::nharmonics)
      .def_readwrite("freq_tol", &SearchParams::freq_tol)
      .def_readwrite("max_harm", &SearchParams::max_harm)
      .def_readwrite("boundary_5_freq", &SearchParams::boundary_5_freq)
      .def_readwrite("boundary_25_freq", &SearchParams::boundary_25_freq)
      .def_readwrite("zap_freqs", &SearchParams::zap_freqs)
      .def_readwrite("zap_widths", &SearchParams::zap_widths)
      .def_readwrite("accel_batch", &SearchParams::accel_batch)
      .def_readwrite("sub_batch", &SearchParams::sub_batch)
      .def_readwrite("sub_streams", &SearchParams::sub_streams)
      .def_readwrite("batch_bytes", &SearchParams::batch_bytes)
      .def_readwrite("engines_per_device", &SearchParams::engines_per_device)
      .def_readwrite("min_batches", &SearchParams::min_batches)
      .def_readwrite("peak_region_log2", &SearchParams::peak_region_log2)
      .def_readwrite("min_gap", &SearchParams::min_gap)
      .def_readwrite("fft_mode", &SearchParams::fft_mode);
  py::class_<SearchEngine::Pending, std::shared_ptr<SearchEngine::Pending>>(m, "PendingSearch");
  py::class_<SearchEngine>(m, "SearchEngine")
      .def(py::init([](const SearchParams& p, uintptr_t s) { return new SearchEngine(p, S(s)); }))
      .def("search_trial", [](SearchEngine& e, uintptr_t trial, uint64_t nsamps, float dm, int dm_idx,
                              const std::vector<float>& accs) {
        return e.search_trial(P<const uint8_t>(trial), nsamps, dm, dm_idx, accs);
      }, py::call_guard<py::gil_scoped_release>())
      .def("prepare", [](SearchEngine& e, uintptr_t trials, uint64_t row_stride, uint64_t nsamps, int count,
                         int first) { e.prepare(P<const uint8_t>(trials), row_stride, nsamps, count, first); },
           py::arg("trials"), py::arg("row_stride"), py::arg("nsamps"), py::arg("count"), py::arg("first") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("reserve", &SearchEngine::reserve, py::arg("count"), py::arg("trials"), py::arg("two") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("batch_for", &SearchEngine::batch_for, py::arg("ntr"))
      .def("search_prepared", [](SearchEngine& e, int b, float dm, int dm_idx, const std::vector<float>& accs) {
        return e.search_prepared(b, dm, dm_idx, accs);
      }, py::call_guard<py::gil_scoped_release>())
      .def("search_prepared_many", [](SearchEngine& e, const std::vector<std::tuple<int, float, int, std::vector<float>>>& jobs) {
        std::vector<SearchEngine::Job> js;
        js.reserve(jobs.size());
        for (const auto& j : jobs) js.push_back(SearchEngine::Job{std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j)});
        return e.search_prepared_many(js);
      }, py::arg("jobs"), py::call_guard<py::gil_scoped_release>(),
         "jobs: [(prepared index, dm, dm_idx, accs)] -> one candidate list per job")
      .def("search_prepared_many_async",
           [](SearchEngine& e, const std::vector<std::tuple<int, float, int, std::vector<float>, bool>>& jobs) {
             std::vector<SearchEngine::Job> js;
             js.reserve(jobs.size());
             for (const auto& j : jobs)
               js.push_back(SearchEngine::Job{std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j),
                                              std::get<4>(j)});
             return e.search_prepared_many_async(js);
           }, py::arg("jobs"), py::call_guard<py::gil_scoped_release>(),
           "jobs: [(prepared index, dm, dm_idx, accs, raw)]; raw: an acceleration slice, its per-trial "
           "harmonic-distilled list returned undistilled (accel_distill_slices joins the slices)")
      .def("search_prepared_many_async", [](SearchEngine& e, const std::vector<std::tuple<int, float, int, std::vector<float>>>& jobs) {
        std::vector<SearchEngine::Job> js;
        js.reserve(jobs.size());
        for (const auto& j : jobs) js.push_back(SearchEngine::Job{std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j)});
        return e.search_prepared_many_async(js);
      }, py::arg("jobs"), py::call_guard<py::gil_scoped_release>(),
         "as search_prepared_many, returning once the batches have retired; collect(handle) waits for the "
         "per-DM acceleration distillation still running on the engine's workers")
      .def("search_launch",
           [](SearchEngine& e, const std::vector<std::tuple<int, float, int, std::vector<float>, bool>>& jobs) {
             std::vector<SearchEngine::Job> js;
             js.reserve(jobs.size());
             for (const auto& j : jobs)
               js.push_back(SearchEngine::Job{std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j),
                                              std::get<4>(j)});
             return e.search_launch(js);
           }, py::arg("jobs"), py::call_guard<py::gil_scoped_release>(),
           "search_prepared_many_async's first half: issues the first batches and returns (search_finish next)")
      .def("search_finish", &SearchEngine::search_finish, py::arg("handle"),
           py::call_guard<py::gil_scoped_release>(),
           "waits for a launched search's batches, issues the rest, processes the peaks (then collect)")
      .def("collect", &SearchEngine::collect, py::arg("handle"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("max_prepare", &SearchEngine::max_prepare)
      .def_property_readonly("batch_size", &SearchEngine::batch_size)
      .def_property_readonly("last_batch", &SearchEngine::last_batch)
      .def_property_readonly("sub_batch", &SearchEngine::sub_batch)
      .def_property_readonly("fft_mode", &SearchEngine::fft_mode)
      .def_property_readonly("rows_ext", &SearchEngine::rows_ext)
      .def_property_readonly("stream", [](const SearchEngine& e) { return reinterpret_cast<uintptr_t>(e.stream()); })
      .def_property_readonly("tobs", &SearchEngine::tobs)
      .def_property_readonly("stats_address", [](const SearchEngine& e) { return reinterpret_cast<uintptr_t>(e.trial_stats()); })
      .def("copy_whitened", [](const SearchEngine& e, uintptr_t dst) { e.copy_whitened(P<float>(dst)); })
      .def("copy_stats", [](const SearchEngine& e, uintptr_t dst) {
        PSOUP_HIP_CHECK(hipMemcpy(P<void>(dst), e.trial_stats(), 3 * sizeof(float), hipMemcpyDeviceToDevice));
      })
      .def("counters", [](const SearchEngine& e) {
        const SearchCounters& c = e.counters();
        py::dict d;
        d["dm_trials"] = c.dm_trials;
        d["accel_trials"] = c.accel_trials;
        d["peaks"] = c.peaks;
        d["overflows"] = c.overflows;
        d["harm_in"] = c.harm_in;
        d["harm_out"] = c.harm_out;
        d["accel_s"] = c.accel_s;
        d["host_s"] = c.host_s;
        d["accd_s"] = c.accd_s;
        d["tail_s"] = c.tail_s;
        d["gpu_distilled"] = c.gpu_distilled;
        d["host_distilled"] = c.host_distilled;
        return d;
      })
      .def("reset_counters", &SearchEngine::reset_counters);
  m.def("build_zap_mask", &build_zap_mask);
  m.def("fold_calculate_sn", [](const std::vector<float>& prof, int bin, int width) {
    float a = 0, b = 0;
    fold_calculate_sn(prof.data(), bin, width, static_cast<int>(prof.size()), &a, &b);
    return py::make_tuple(a, b);
  });
  py::class_<FoldResult>(m, "FoldResult")
      .def_readonly("folded_snr", &FoldResult::folded_snr)
      .def_readonly("opt_period", &FoldResult::opt_period)
      .def_readonly("opt_width", &FoldResult::opt_width)
      .def_readonly("opt_bin", &FoldResult::opt_bin)
      .def_readonly("fold", &FoldResult::fold)
      .def_property_readonly("fold_array", [](const FoldResult& r) {  // float32 copy, no per-element conversion
        py::array_t<float> a(static_cast<py::ssize_t>(r.fold.size()));
        std::copy(r.fold.begin(), r.fold.end(), a.mutable_data());
        return a;
      })
      .def_readonly("prof", &FoldResult::prof);
  py::class_<FoldEngine>(m, "FoldEngine")
      .def(py::init([](uint64_t n, float tsamp, uintptr_t s) { return new FoldEngine(n, tsamp, S(s)); }))
      .def("fold_trial", [](FoldEngine& f, uintptr_t trial, uint64_t nsamps, const std::vector<double>& periods,
                            const std::vector<float>& accs) { return f.fold_trial(P<const uint8_t>(trial), nsamps, periods, accs); },
           py::call_guard<py::gil_scoped_release>())
      .def("fold_trials", [](FoldEngine& f, uintptr_t trials, uint64_t row_stride, uint64_t nsamps,
                             const std::vector<std::vector<double>>& periods,
                             const std::vector<std::vector<float>>& accs) {
        return f.fold_trials(P<const uint8_t>(trials), row_stride, nsamps, static_cast<int>(periods.size()), periods,
                             accs);
      })
      .def("fold_rows", [](FoldEngine& f, const std::vector<uintptr_t>& rows, uint64_t nsamps,
                           const std::vector<std::vector<double>>& periods,
                           const std::vector<std::vector<float>>& accs) {
        std::vector<const uint8_t*> r;
        for (uintptr_t v : rows) r.push_back(P<const uint8_t>(v));
        return f.fold_rows(r, nsamps, periods, accs);
      })
      .def("reserve", &FoldEngine::reserve, py::arg("njobs_hint"))
      .def_property_readonly("max_batch", &FoldEngine::max_batch)
      .def("fold_series", [](FoldEngine& f, uintptr_t series, const std::vector<double>& periods,
                             const std::vector<float>& accs) { return f.fold_series(P<const float>(series), periods, accs); },
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("nsamps", &FoldEngine::nsamps);
  m.def("coincidencer_beam", [](uintptr_t trial, uint64_t n, float tsamp, uintptr_t series_out, uintptr_t spec_out,
                                uintptr_t s) {
    BeamProducts bp;
    coincidencer_beam(P<const uint8_t>(trial), n, tsamp, bp, S(s));
    PSOUP_HIP_CHECK(hipMemcpyAsync(P<float>(series_out), bp.series.data(), n * 4, hipMemcpyDeviceToDevice, S(s)));
    PSOUP_HIP_CHECK(hipMemcpyAsync(P<float>(spec_out), bp.spectrum.data(), (n / 2 + 1) * 4, hipMemcpyDeviceToDevice, S(s)));
    PSOUP_HIP_CHECK(hipStreamSynchronize(S(s)));
  });
  m.def("write_samp_mask", &write_samp_mask);
  m.def("write_birdie_list", &write_birdie_list);
  // host float32 buffers by address (a 1M-sample mask without a Python list)
  m.def("write_samp_mask_ptr", [](uintptr_t mask, uint64_t n, const std::string& fn) {
    const float* f = P<const float>(mask);
    write_samp_mask(std::vector<float>(f, f + n), fn);
  });
  m.def("write_birdie_list_ptr", [](uintptr_t mask, uint64_t n, float bin_width, const std::string& fn) {
    const float* f = P<const float>(mask);
    write_birdie_list(std::vector<float>(f, f + n), bin_width, fn);
  });

  // ----------------------------------------------------------- pipeline ---
  m.def("run_pipeline_native", [](const CmdLineOptions& args) {
    PipelineResult r;
    {
      py::gil_scoped_release nogil;
      r = run_pipeline(args);
      write_outputs(args, r);
    }
    py::dict d;
    d["candidates"] = r.candidates;
    d["timers"] = r.timers;
    d["performance"] = r.performance;
    d["dm_list"] = r.setup.dm_list;
    d["fft_size"] = r.setup.fft_size;
    return d;
  });
  m.def("accel_list_for", [](const CmdLineOptions& args, const py::dict& hdr, float dm) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    return s.accel_plan.generate(dm);
  });
  m.def("accel_plan_from_args", [](const CmdLineOptions& args, const py::dict& hdr) {
    return make_search_setup(args, dict_to_header(hdr)).accel_plan;
  });
  m.def("global_distill_and_score", [](CandidateBag& b, const CmdLineOptions& args, const py::dict& hdr) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    auto out = std::make_shared<CandidateBag>();
    py::gil_scoped_release nogil;
    CandidateList all = std::move(b.c);
    b.c.clear();
    out->c = global_distill_and_score(std::move(all), args, s);
    return out;
  });
  m.def("global_distill_and_score", [](CandidateList c, const CmdLineOptions& args, const py::dict& hdr) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    return global_distill_and_score(std::move(c), args, s);
  });
  // ----------------------------------------------------- checkpoint/resume --
  m.def("checkpoint_identity", [](const CmdLineOptions& args, const py::dict& hdr) {
    RunIdentity id = make_run_identity(args, dict_to_header(hdr));
    return py::make_tuple(id.key, id.text);
  });
  m.def("prepare_checkpoint_dir", [](const std::string& dir, const CmdLineOptions& args, const py::dict& hdr) {
    RunIdentity id = make_run_identity(args, dict_to_header(hdr));
    prepare_checkpoint_dir(dir, id);
    return id.key;
  });
  m.def("spill_path", &spill_path);
  m.def("load_spill", [](const std::string& path, uint64_t key) {
    CandidateList c;
    SpillStatus st = load_spill(path, key, c);
    return py::make_tuple(std::string(spill_status_name(st)), c);
  });
  m.def("save_spill", [](const std::string& path, uint64_t key, const CandidateBag& b) { save_spill(path, key, b.c); },
        py::arg("path"), py::arg("key"), py::arg("cands"));
  m.def("save_spill", &save_spill, py::arg("path"), py::arg("key"), py::arg("cands"));
  m.def("load_spill_bag", [](const std::string& path, uint64_t key) {
    auto b = std::make_shared<CandidateBag>();
    SpillStatus st = load_spill(path, key, b->c);
    return py::make_tuple(std::string(spill_status_name(st)), b);
  });
  m.def("search_params_from_args", [](const CmdLineOptions& args, const py::dict& hdr) {
    SearchSetup s = make_search_setup(args, dict_to_header(hdr));
    return py::make_tuple(s.search, s.dm_list, s.killmask, s.fft_size, s.cfreq);
  });
}
