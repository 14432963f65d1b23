// Output writers.
//
// Parity:
//   include/utils/xml_util.hpp:9-92      XML::Element (setprecision(15),
//       single-quoted attributes in sorted-map order, 2-space indentation,
//       ISO-8859-1 declaration) -- byte-compatible.
//   include/utils/output_stats.hpp:17-218 OutputFileWriter (overview.xml:
//       misc_info, header_parameters, search_parameters, dedispersion_trials,
//       acceleration_trials, cuda_device_parameters, candidates,
//       execution_times).  Tag names are kept for tool compatibility; the
//       device section is filled from the HIP runtime.
//   include/utils/output_stats.hpp:221-270 CandidateFileWriter::write_binary
//       (candidates.peasoup: ["FOLD" i32 nbins i32 nints f32[nints*nbins]]
//       i32 ndets CandidatePOD[ndets] per candidate).
#pragma once

#include <cstdint>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "psoup/candidates.hpp"
#include "psoup/cli.hpp"
#include "psoup/sigproc.hpp"

namespace psoup {
namespace xml {

std::string fmt(double v);
std::string fmt(float v);
std::string fmt(int v);
std::string fmt(unsigned v);
std::string fmt(long v);
std::string fmt(long long v);
std::string fmt(unsigned long v);
std::string fmt(unsigned long long v);
std::string fmt(bool v);
std::string fmt(const std::string& v);
std::string fmt(const char* v);

class Element {
 public:
  explicit Element(std::string name) : name_(std::move(name)) {}
  template <class X>
  Element(std::string name, const X& value) : name_(std::move(name)) {
    text_ = fmt(value);
  }
  void append(Element child) { children_.push_back(std::move(child)); }
  template <class X>
  void set_text(const X& v) {
    text_ = fmt(v);
  }
  template <class X>
  void add_attribute(const std::string& key, const X& v) {
    attributes_[key] = "'" + fmt(v) + "'";
  }
  std::string to_string(bool header = false, int level = 0) const;
  void write(std::string& out, int level) const;  // appends this element's text
  const std::string& name() const { return name_; }
  const std::vector<Element>& children() const { return children_; }

 private:
  std::string name_;
  std::string text_;
  std::map<std::string, std::string> attributes_;
  std::vector<Element> children_;
};

}  // namespace xml

struct GpuStageTimes {
  std::map<std::string, double> seconds;  // optional per-stage breakdown
};

class OverviewWriter {
 public:
  OverviewWriter() : root_("peasoup_search") {}
  void add_misc_info();
  void add_header(const std::string& filename);  // re-reads the header (as the reference)
  void add_header(const SigprocHeader& hdr);
  void add_search_parameters(const CmdLineOptions& args);
  void add_dm_list(const std::vector<float>& dms);
  void add_acc_list(const std::vector<float>& accs);
  void add_gpu_info(const std::vector<int>& device_ids);
  void add_candidates(const CandidateList& cands, const std::map<unsigned, long>& byte_map);
  void add_timing_info(const std::map<std::string, double>& seconds);
  // MI355X extension (separate element so <execution_times> keeps its shape).
  void add_performance(const std::map<std::string, double>& values);
  void add_element(xml::Element e) { root_.append(std::move(e)); }
  std::string to_string() const { return root_.to_string(true); }
  void to_file(const std::string& filename) const;

 private:
  xml::Element root_;
};

class CandidateFileWriter {
 public:
  explicit CandidateFileWriter(std::string outdir);
  // Returns false (after perror) when the file cannot be opened.
  bool write_binary(const CandidateList& cands, const std::string& filename);
  // One file per candidate, cand_%04d_<P %.5f>_<DM %.1f>_<acc %.1f>.peasoup, same
  // record format (output_stats.hpp:272-307 write_binaries); fills `filenames`
  // with the absolute paths.  Returns false (after perror) on the first failure.
  bool write_binaries(const CandidateList& cands);
  std::map<unsigned, long> byte_mapping;
  std::map<unsigned, std::string> filenames;
  const std::string& outdir() const { return outdir_; }

 private:
  std::string outdir_;
};

// Text candidate dumps (candidates.hpp:120-150): one Candidate::print file per
// candidate (cand_%04d_..., CandidateCollection::generate_candidate_binaries)
// and a single annotated listing (write_candidate_file).
bool write_candidate_text_files(const CandidateList& cands, const std::string& outdir);
bool write_candidate_file(const CandidateList& cands, const std::string& path);

// Recursive mkdir -p (0777 & ~umask); returns false on failure.
bool make_dirs(const std::string& path);

}  // namespace psoup
