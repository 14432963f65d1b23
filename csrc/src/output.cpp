#include <climits>
#include <cstdlib>
#include "psoup/output.hpp"

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <fstream>
#include <iomanip>

#include "psoup/common.hpp"

namespace psoup {
namespace xml {

namespace {
// the digits `ostream << setprecision(15) << v` gives (%.15g; integers as
// they are), without a stream per value
std::string num_fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string num_fmt(const char* f, ...) {
  char buf[64];
  va_list ap;
  va_start(ap, f);
  const int n = std::vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return std::string(buf, static_cast<size_t>(std::max(0, std::min(n, static_cast<int>(sizeof(buf)) - 1))));
}

std::string escape(const std::string& s) {
  std::string o;
  o.reserve(s.size());
  for (char c : s) {
    if (c == '&') o += "&amp;";
    else if (c == '<') o += "&lt;";
    else if (c == '>') o += "&gt;";
    else o += c;
  }
  return o;
}
}  // namespace

std::string fmt(double v) { return num_fmt("%.15g", v); }
std::string fmt(float v) { return num_fmt("%.15g", static_cast<double>(v)); }
std::string fmt(int v) { return num_fmt("%d", v); }
std::string fmt(unsigned v) { return num_fmt("%u", v); }
std::string fmt(long v) { return num_fmt("%ld", v); }
std::string fmt(long long v) { return num_fmt("%lld", v); }
std::string fmt(unsigned long v) { return num_fmt("%lu", v); }
std::string fmt(unsigned long long v) { return num_fmt("%llu", v); }
std::string fmt(bool v) { return v ? "1" : "0"; }
std::string fmt(const std::string& v) { return escape(v); }
std::string fmt(const char* v) { return escape(v ? std::string(v) : std::string()); }

void Element::write(std::string& o, int level) const {
  o.append(2 * static_cast<size_t>(level), ' ');
  o += '<';
  o += name_;
  for (const auto& kv : attributes_) {
    o += ' ';
    o += kv.first;
    o += '=';
    o += kv.second;
  }
  o += '>';
  if (children_.empty()) {
    o += text_;
  } else {
    o += '\n';
    for (const auto& c : children_) c.write(o, level + 1);
    o.append(2 * static_cast<size_t>(level), ' ');
  }
  o += "</";
  o += name_;
  o += ">\n";
}

std::string Element::to_string(bool header, int level) const {
  std::string o;
  if (header) o = "<?xml version='1.0' encoding='ISO-8859-1'?>\n";
  write(o, level);
  return o;
}

}  // namespace xml

void OverviewWriter::add_misc_info() {
  xml::Element info("misc_info");
  char buf[128];
  std::string user;
  if (getlogin_r(buf, sizeof(buf)) == 0) user = buf;
  else if (const char* u = std::getenv("USER")) user = u;
  else user = "unknown";
  info.append(xml::Element("username", user));
  std::time_t t = std::time(nullptr);
  std::strftime(buf, sizeof(buf), "%Y-%m-%d-%H:%M", std::localtime(&t));
  info.append(xml::Element("local_datetime", std::string(buf)));
  std::strftime(buf, sizeof(buf), "%Y-%m-%d-%H:%M", std::gmtime(&t));
  info.append(xml::Element("utc_datetime", std::string(buf)));
  root_.append(info);
}

void OverviewWriter::add_header(const std::string& filename) { add_header(read_header_file(filename)); }

void OverviewWriter::add_header(const SigprocHeader& hdr) {
  xml::Element h("header_parameters");
  h.append(xml::Element("source_name", hdr.source_name));
  h.append(xml::Element("rawdatafile", hdr.rawdatafile));
  h.append(xml::Element("az_start", hdr.az_start));
  h.append(xml::Element("za_start", hdr.za_start));
  h.append(xml::Element("src_raj", hdr.src_raj));
  h.append(xml::Element("src_dej", hdr.src_dej));
  h.append(xml::Element("tstart", hdr.tstart));
  h.append(xml::Element("tsamp", hdr.tsamp));
  h.append(xml::Element("period", hdr.period));
  h.append(xml::Element("fch1", hdr.fch1));
  h.append(xml::Element("foff", hdr.foff));
  h.append(xml::Element("nchans", hdr.nchans));
  h.append(xml::Element("telescope_id", hdr.telescope_id));
  h.append(xml::Element("machine_id", hdr.machine_id));
  h.append(xml::Element("data_type", hdr.data_type));
  h.append(xml::Element("ibeam", hdr.ibeam));
  h.append(xml::Element("nbeams", hdr.nbeams));
  h.append(xml::Element("nbits", hdr.nbits));
  h.append(xml::Element("barycentric", hdr.barycentric));
  h.append(xml::Element("pulsarcentric", hdr.pulsarcentric));
  h.append(xml::Element("nbins", hdr.nbins));
  h.append(xml::Element("nsamples", hdr.nsamples));
  h.append(xml::Element("nifs", hdr.nifs));
  h.append(xml::Element("npuls", hdr.npuls));
  h.append(xml::Element("refdm", hdr.refdm));
  h.append(xml::Element("signed", static_cast<int>(hdr.signed_data)));
  root_.append(h);
}

void OverviewWriter::add_search_parameters(const CmdLineOptions& a) {
  xml::Element s("search_parameters");
  s.append(xml::Element("infilename", a.infilename));
  s.append(xml::Element("outdir", a.outdir));
  s.append(xml::Element("killfilename", a.killfilename));
  s.append(xml::Element("zapfilename", a.zapfilename));
  s.append(xml::Element("max_num_threads", a.max_num_threads));
  s.append(xml::Element("size", a.size));
  s.append(xml::Element("dm_start", a.dm_start));
  s.append(xml::Element("dm_end", a.dm_end));
  s.append(xml::Element("dm_tol", a.dm_tol));
  s.append(xml::Element("dm_pulse_width", a.dm_pulse_width));
  s.append(xml::Element("acc_start", a.acc_start));
  s.append(xml::Element("acc_end", a.acc_end));
  s.append(xml::Element("acc_tol", a.acc_tol));
  s.append(xml::Element("acc_pulse_width", a.acc_pulse_width));
  s.append(xml::Element("boundary_5_freq", a.boundary_5_freq));
  s.append(xml::Element("boundary_25_freq", a.boundary_25_freq));
  s.append(xml::Element("nharmonics", a.nharmonics));
  s.append(xml::Element("npdmp", a.npdmp));
  s.append(xml::Element("min_snr", a.min_snr));
  s.append(xml::Element("min_freq", a.min_freq));
  s.append(xml::Element("max_freq", a.max_freq));
  s.append(xml::Element("max_harm", a.max_harm));
  s.append(xml::Element("freq_tol", a.freq_tol));
  s.append(xml::Element("verbose", a.verbose));
  s.append(xml::Element("progress_bar", a.progress_bar));
  root_.append(s);
}

void OverviewWriter::add_dm_list(const std::vector<float>& dms) {
  xml::Element e("dedispersion_trials");
  e.add_attribute("count", static_cast<unsigned long>(dms.size()));
  for (size_t i = 0; i < dms.size(); ++i) {
    xml::Element t("trial");
    t.add_attribute("id", static_cast<int>(i));
    t.set_text(dms[i]);
    e.append(t);
  }
  root_.append(e);
}

void OverviewWriter::add_acc_list(const std::vector<float>& accs) {
  xml::Element e("acceleration_trials");
  e.add_attribute("count", static_cast<unsigned long>(accs.size()));
  e.add_attribute("DM", 0);
  for (size_t i = 0; i < accs.size(); ++i) {
    xml::Element t("trial");
    t.add_attribute("id", static_cast<int>(i));
    t.set_text(accs[i]);
    e.append(t);
  }
  root_.append(e);
}

void OverviewWriter::add_gpu_info(const std::vector<int>& device_ids) {
  xml::Element g("cuda_device_parameters");
  g.append(xml::Element("runtime", runtime_version()));
  g.append(xml::Element("driver", driver_version()));
  for (int id : device_ids) {
    xml::Element d("cuda_device");
    d.add_attribute("id", id);
    DeviceInfo info = device_info(id);
    d.append(xml::Element("name", info.name));
    d.append(xml::Element("major_cc", info.major));
    d.append(xml::Element("minor_cc", info.minor));
    d.append(xml::Element("arch", info.arch));
    d.append(xml::Element("compute_units", info.multiprocessors));
    g.append(d);
  }
  root_.append(g);
}

void OverviewWriter::add_candidates(const CandidateList& cands, const std::map<unsigned, long>& byte_map) {
  xml::Element e("candidates");
  std::vector<int> nassoc(cands.size());  // (tree walks, on several threads)
  parallel_each(cands.size(), 8, [&](size_t i) { nassoc[i] = cands[i].count_assoc(); });
  for (size_t i = 0; i < cands.size(); ++i) {
    const Candidate& c = cands[i];
    xml::Element x("candidate");
    x.add_attribute("id", static_cast<int>(i));
    x.append(xml::Element("period", 1.0 / c.freq));
    x.append(xml::Element("opt_period", c.opt_period));
    x.append(xml::Element("dm", c.dm));
    x.append(xml::Element("acc", c.acc));
    x.append(xml::Element("nh", c.nh));
    x.append(xml::Element("snr", c.snr));
    x.append(xml::Element("folded_snr", c.folded_snr));
    x.append(xml::Element("is_adjacent", c.is_adjacent));
    x.append(xml::Element("is_physical", c.is_physical));
    x.append(xml::Element("ddm_count_ratio", c.ddm_count_ratio));
    x.append(xml::Element("ddm_snr_ratio", c.ddm_snr_ratio));
    x.append(xml::Element("nassoc", nassoc[i]));
    auto it = byte_map.find(static_cast<unsigned>(i));
    x.append(xml::Element("byte_offset", it == byte_map.end() ? 0L : it->second));
    e.append(x);
  }
  root_.append(e);
}

void OverviewWriter::add_timing_info(const std::map<std::string, double>& seconds) {
  xml::Element e("execution_times");
  for (const auto& kv : seconds) e.append(xml::Element(kv.first, kv.second));
  root_.append(e);
}

void OverviewWriter::add_performance(const std::map<std::string, double>& values) {
  xml::Element e("performance");
  for (const auto& kv : values) e.append(xml::Element(kv.first, kv.second));
  root_.append(e);
}

void OverviewWriter::to_file(const std::string& filename) const {
  std::ofstream out(filename, std::ios::binary);
  if (!out) PSOUP_THROW("cannot write " << filename);
  out << to_string();
  if (!out) PSOUP_THROW("write failed for " << filename);
}

bool make_dirs(const std::string& path) {
  if (path.empty()) return true;
  std::string cur;
  size_t pos = 0;
  while (pos != std::string::npos) {
    pos = path.find('/', pos + 1);
    cur = path.substr(0, pos);
    if (cur.empty()) continue;
    struct stat st;
    if (stat(cur.c_str(), &st) == -1) {
      if (mkdir(cur.c_str(), 0777) != 0 && errno != EEXIST) return false;
    }
  }
  return true;
}

CandidateFileWriter::CandidateFileWriter(std::string outdir) : outdir_(std::move(outdir)) {
  if (!make_dirs(outdir_)) perror(outdir_.c_str());
}

bool CandidateFileWriter::write_binary(const CandidateList& cands, const std::string& filename) {
  std::string path = outdir_ + "/" + filename;
  FILE* fo = std::fopen(path.c_str(), "wb");
  if (!fo) {
    perror(path.c_str());
    return false;
  }
  byte_mapping.clear();
  // each candidate's record (fold, then its association tree flattened) built
  // on several threads -- config 4's 1000 candidates carry ~1.2M associated
  // ones (42 MB), whose tree walk cost more than the write -- then written in
  // order
  const size_t n = cands.size();
  std::vector<std::string> rec(n);
  parallel_each(n, 8, [&](size_t i) {
    thread_local std::vector<CandidatePOD> dets;
    {
      const Candidate& c = cands[i];
      dets.clear();
      c.collect_candidates(dets);
      const int32_t ndets = static_cast<int32_t>(dets.size());
      const size_t nf = c.fold.empty() ? 0 : static_cast<size_t>(c.nbins) * c.nints;
      std::string& r = rec[i];
      r.reserve((nf ? 12 + 4 * nf : 0) + 4 + dets.size() * sizeof(CandidatePOD));
      if (nf) {
        const int32_t nb = c.nbins, ni = c.nints;
        r.append("FOLD", 4);
        r.append(reinterpret_cast<const char*>(&nb), 4);
        r.append(reinterpret_cast<const char*>(&ni), 4);
        r.append(reinterpret_cast<const char*>(c.fold.data()), 4 * nf);
      }
      r.append(reinterpret_cast<const char*>(&ndets), 4);
      r.append(reinterpret_cast<const char*>(dets.data()), dets.size() * sizeof(CandidatePOD));
    }
  });
  long off = std::ftell(fo);
  bool ok = true;
  for (size_t i = 0; i < n; ++i) {
    byte_mapping[static_cast<unsigned>(i)] = off;
    ok = ok && std::fwrite(rec[i].data(), 1, rec[i].size(), fo) == rec[i].size();
    off += static_cast<long>(rec[i].size());
  }
  ok = (std::fclose(fo) == 0) && ok;
  if (!ok) perror(path.c_str());
  return ok;
}

namespace {
std::string cand_filename(size_t i, const Candidate& c) {
  char buf[160];
  std::snprintf(buf, sizeof(buf), "cand_%04d_%.5f_%.1f_%.1f.peasoup", static_cast<int>(i), 1.0 / c.freq, c.dm,
                c.acc);
  return buf;
}

void write_record(FILE* fo, const Candidate& c, std::vector<CandidatePOD>& dets) {
  if (!c.fold.empty()) {
    std::fwrite("FOLD", 1, 4, fo);
    int32_t nb = c.nbins, ni = c.nints;
    std::fwrite(&nb, sizeof(int32_t), 1, fo);
    std::fwrite(&ni, sizeof(int32_t), 1, fo);
    std::fwrite(c.fold.data(), sizeof(float), static_cast<size_t>(nb) * ni, fo);
  }
  dets.clear();
  c.collect_candidates(dets);
  int32_t ndets = static_cast<int32_t>(dets.size());
  std::fwrite(&ndets, sizeof(int32_t), 1, fo);
  std::fwrite(dets.data(), sizeof(CandidatePOD), dets.size(), fo);
}
}  // namespace

bool CandidateFileWriter::write_binaries(const CandidateList& cands) {
  filenames.clear();
  std::vector<CandidatePOD> dets;
  for (size_t i = 0; i < cands.size(); ++i) {
    const std::string path = outdir_ + "/" + cand_filename(i, cands[i]);
    FILE* fo = std::fopen(path.c_str(), "wb");
    if (!fo) {
      perror(path.c_str());
      return false;
    }
    write_record(fo, cands[i], dets);
    std::fclose(fo);
    char real[PATH_MAX];
    filenames[static_cast<unsigned>(i)] = realpath(path.c_str(), real) ? std::string(real) : path;
  }
  return true;
}

bool write_candidate_text_files(const CandidateList& cands, const std::string& outdir) {
  if (!make_dirs(outdir)) return false;
  for (size_t i = 0; i < cands.size(); ++i) {
    const std::string path = outdir + "/" + cand_filename(i, cands[i]);
    FILE* fo = std::fopen(path.c_str(), "w");
    if (!fo) {
      perror(path.c_str());
      return false;
    }
    const std::string txt = cands[i].print();
    std::fwrite(txt.data(), 1, txt.size(), fo);
    std::fclose(fo);
  }
  return true;
}

bool write_candidate_file(const CandidateList& cands, const std::string& path) {
  FILE* fo = std::fopen(path.c_str(), "w");
  if (!fo) {
    perror(path.c_str());
    return false;
  }
  std::fprintf(fo, "#Period...Optimal period...Frequency...DM...Acceleration...Harmonic number...S/N...Folded S/N\n");
  for (size_t i = 0; i < cands.size(); ++i) {
    std::fprintf(fo, "#Candidate %d\n", static_cast<int>(i));
    const std::string txt = cands[i].print();
    std::fwrite(txt.data(), 1, txt.size(), fo);
  }
  std::fclose(fo);
  return true;
}

}  // namespace psoup
