#include "psoup/sigproc.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iostream>
#include <mutex>
#include <sstream>
#include <thread>
#include <vector>

#include "psoup/common.hpp"

namespace psoup {

bool SigprocHeader::has(const std::string& key) const {
  return std::find(keys_present.begin(), keys_present.end(), key) != keys_present.end();
}

namespace {

bool read_string(std::istream& in, std::string& s) {
  int32_t len = 0;
  in.read(reinterpret_cast<char*>(&len), sizeof(len));
  if (!in || len <= 0 || len >= 80) return false;
  char buf[80];
  in.read(buf, len);
  if (!in) return false;
  s.assign(buf, static_cast<size_t>(len));
  return true;
}

template <class T>
void read_value(std::istream& in, T& v) {
  in.read(reinterpret_cast<char*>(&v), sizeof(T));
}

void write_string(std::ostream& out, const std::string& s) {
  int32_t len = static_cast<int32_t>(s.size());
  out.write(reinterpret_cast<const char*>(&len), sizeof(len));
  out.write(s.data(), len);
}

template <class T>
void write_kv(std::ostream& out, const char* key, T v) {
  write_string(out, key);
  out.write(reinterpret_cast<const char*>(&v), sizeof(T));
}

}  // namespace

bool read_header(std::istream& in, SigprocHeader& hdr) {
  std::string s;
  std::streampos start = in.tellg();
  if (!read_string(in, s) || s != "HEADER_START") {
    in.clear();
    in.seekg(start);
    return false;
  }
  bool expect_source = false, expect_raw = false;
  hdr.keys_present.clear();
  while (true) {
    if (!read_string(in, s)) PSOUP_THROW("corrupt SIGPROC header (bad key length)");
    if (s == "HEADER_END") break;
    bool known = true;
    if (s == "source_name") expect_source = true;
    else if (s == "rawdatafile") expect_raw = true;
    else if (s == "az_start") read_value(in, hdr.az_start);
    else if (s == "za_start") read_value(in, hdr.za_start);
    else if (s == "src_raj") read_value(in, hdr.src_raj);
    else if (s == "src_dej") read_value(in, hdr.src_dej);
    else if (s == "tstart") read_value(in, hdr.tstart);
    else if (s == "tsamp") read_value(in, hdr.tsamp);
    else if (s == "period") read_value(in, hdr.period);
    else if (s == "fch1") read_value(in, hdr.fch1);
    else if (s == "foff") read_value(in, hdr.foff);
    else if (s == "nchans") read_value(in, hdr.nchans);
    else if (s == "telescope_id") read_value(in, hdr.telescope_id);
    else if (s == "machine_id") read_value(in, hdr.machine_id);
    else if (s == "data_type") read_value(in, hdr.data_type);
    else if (s == "ibeam") read_value(in, hdr.ibeam);
    else if (s == "nbeams") read_value(in, hdr.nbeams);
    else if (s == "nbits") read_value(in, hdr.nbits);
    else if (s == "barycentric") read_value(in, hdr.barycentric);
    else if (s == "pulsarcentric") read_value(in, hdr.pulsarcentric);
    else if (s == "nbins") read_value(in, hdr.nbins);
    else if (s == "nsamples") read_value(in, hdr.nsamples);
    else if (s == "nifs") read_value(in, hdr.nifs);
    else if (s == "npuls") read_value(in, hdr.npuls);
    else if (s == "refdm") read_value(in, hdr.refdm);
    else if (s == "signed") read_value(in, hdr.signed_data);
    else if (expect_source) {
      hdr.source_name = s;
      expect_source = false;
      known = false;
    } else if (expect_raw) {
      hdr.rawdatafile = s;
      expect_raw = false;
      known = false;
    } else {
      std::cerr << "Warning: read_header: unknown parameter " << s << std::endl;
      known = false;
    }
    if (known) hdr.keys_present.push_back(s);
    if (!in) PSOUP_THROW("truncated SIGPROC header while reading " << s);
  }
  hdr.size = static_cast<uint64_t>(in.tellg() - start);
  if (hdr.nsamples == 0 && hdr.nchans > 0 && hdr.nbits > 0) {
    std::streampos here = in.tellg();
    in.seekg(0, std::ios::end);
    uint64_t total = static_cast<uint64_t>(in.tellg() - start);
    hdr.nsamples = static_cast<int>((total - hdr.size) / hdr.nchans * 8 / hdr.nbits);
    in.seekg(here);
  }
  return true;
}

SigprocHeader read_header_file(const std::string& filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) PSOUP_THROW("cannot open " << filename);
  SigprocHeader hdr;
  if (!read_header(in, hdr)) PSOUP_THROW(filename << " is not a SIGPROC file (no HEADER_START)");
  return hdr;
}

void write_header(std::ostream& out, const SigprocHeader& h) {
  auto want = [&](const char* key, bool nonzero) { return nonzero || h.has(key); };
  write_string(out, "HEADER_START");
  if (want("telescope_id", h.telescope_id != 0)) write_kv(out, "telescope_id", h.telescope_id);
  if (want("machine_id", h.machine_id != 0)) write_kv(out, "machine_id", h.machine_id);
  write_kv(out, "data_type", h.data_type == 0 ? 1 : h.data_type);
  if (!h.rawdatafile.empty()) {
    write_string(out, "rawdatafile");
    write_string(out, h.rawdatafile);
  }
  if (!h.source_name.empty()) {
    write_string(out, "source_name");
    write_string(out, h.source_name);
  }
  if (want("barycentric", h.barycentric != 0)) write_kv(out, "barycentric", h.barycentric);
  if (want("pulsarcentric", h.pulsarcentric != 0)) write_kv(out, "pulsarcentric", h.pulsarcentric);
  if (want("az_start", h.az_start != 0.0)) write_kv(out, "az_start", h.az_start);
  if (want("za_start", h.za_start != 0.0)) write_kv(out, "za_start", h.za_start);
  if (want("src_raj", h.src_raj != 0.0)) write_kv(out, "src_raj", h.src_raj);
  if (want("src_dej", h.src_dej != 0.0)) write_kv(out, "src_dej", h.src_dej);
  if (want("tstart", h.tstart != 0.0)) write_kv(out, "tstart", h.tstart);
  write_kv(out, "tsamp", h.tsamp);
  write_kv(out, "nbits", h.nbits);
  if (want("nsamples", h.nsamples != 0)) write_kv(out, "nsamples", h.nsamples);
  write_kv(out, "fch1", h.fch1);
  write_kv(out, "foff", h.foff);
  write_kv(out, "nchans", h.nchans);
  write_kv(out, "nifs", h.nifs == 0 ? 1 : h.nifs);
  if (want("ibeam", h.ibeam != 0)) write_kv(out, "ibeam", h.ibeam);
  if (want("nbeams", h.nbeams != 0)) write_kv(out, "nbeams", h.nbeams);
  if (want("refdm", h.refdm != 0.0)) write_kv(out, "refdm", h.refdm);
  if (want("period", h.period != 0.0)) write_kv(out, "period", h.period);
  if (want("nbins", h.nbins != 0)) write_kv(out, "nbins", h.nbins);
  if (want("npuls", h.npuls != 0)) write_kv(out, "npuls", h.npuls);
  if (want("signed", h.signed_data != 0)) write_kv(out, "signed", h.signed_data);
  write_string(out, "HEADER_END");
}

Filterbank Filterbank::from_file(const std::string& filename) {
  Filterbank fb;
  {
    std::ifstream in(filename, std::ios::binary);
    if (!in) PSOUP_THROW("cannot open filterbank " << filename);
    if (!read_header(in, fb.hdr_)) PSOUP_THROW(filename << " is not a SIGPROC filterbank");
  }
  PSOUP_CHECK(fb.hdr_.nchans > 0 && fb.hdr_.nbits > 0, "bad header in " << filename);
  PSOUP_CHECK(fb.hdr_.nbits == 1 || fb.hdr_.nbits == 2 || fb.hdr_.nbits == 4 || fb.hdr_.nbits == 8,
              "unsupported nbits=" << fb.hdr_.nbits << " (1/2/4/8 supported)");
  int fd = ::open(filename.c_str(), O_RDONLY);
  if (fd < 0) PSOUP_THROW("cannot open " << filename);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    PSOUP_THROW("cannot stat " << filename);
  }
  uint64_t file_size = static_cast<uint64_t>(st.st_size);
  uint64_t want = static_cast<uint64_t>(fb.hdr_.nsamples) * fb.hdr_.nbits * fb.hdr_.nchans / 8;
  if (fb.hdr_.size + want > file_size) {
    // Truncated file: keep only whole samples.
    uint64_t avail = file_size > fb.hdr_.size ? file_size - fb.hdr_.size : 0;
    uint64_t bps = fb.bytes_per_sample();
    fb.hdr_.nsamples = static_cast<int>(avail / bps);
    want = static_cast<uint64_t>(fb.hdr_.nsamples) * bps;
  }
  void* map = nullptr;
  if (file_size > 0) {
    map = ::mmap(nullptr, file_size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (map == MAP_FAILED) {
      ::close(fd);
      PSOUP_THROW("mmap failed for " << filename);
    }
    ::madvise(map, file_size, MADV_SEQUENTIAL);
  }
  ::close(fd);
  fb.owner_ = std::shared_ptr<void>(map, [file_size](void* p) {
    if (p) ::munmap(p, file_size);
  });
  fb.data_ = static_cast<const uint8_t*>(map) + fb.hdr_.size;
  fb.data_bytes_ = want;
  fb.path_ = filename;
  fb.data_offset_ = static_cast<uint64_t>(fb.hdr_.size);
  return fb;
}

void Filterbank::read_data(uint64_t off, uint64_t n, uint8_t* dst, int nthreads) const {
  PSOUP_CHECK(off + n <= data_bytes_, "read_data: past the data block");
  if (path_.empty()) {
    std::memcpy(dst, data_ + off, n);
    return;
  }
  // pread from the page cache: ~3x the rate of copying out of the fresh
  // mapping (whose first touch faults every page in), more with threads
  int fd = ::open(path_.c_str(), O_RDONLY);
  if (fd < 0) PSOUP_THROW("cannot open " << path_);
  std::exception_ptr err;
  std::mutex mu;
  auto part = [&](uint64_t a, uint64_t b) {
    try {
      while (a < b) {
        const ssize_t r = ::pread(fd, dst + a, static_cast<size_t>(b - a), static_cast<off_t>(data_offset_ + off + a));
        if (r <= 0) PSOUP_THROW("read failed on " << path_);
        a += static_cast<uint64_t>(r);
      }
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!err) err = std::current_exception();
    }
  };
  const int nt = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(static_cast<uint64_t>(std::max(1, nthreads)),
                                                                          n >> 21)));  // >= 2 MB each
  const uint64_t step = (n + nt - 1) / nt;
  std::vector<std::thread> th;
  for (int i = 1; i < nt; ++i) th.emplace_back(part, std::min(n, i * step), std::min(n, (i + 1) * step));
  part(0, std::min(n, step));
  for (auto& t : th) t.join();
  ::close(fd);
  if (err) std::rethrow_exception(err);
}

Filterbank Filterbank::from_memory(const SigprocHeader& hdr, std::vector<uint8_t> data) {
  Filterbank fb;
  fb.hdr_ = hdr;
  auto vec = std::make_shared<std::vector<uint8_t>>(std::move(data));
  fb.data_ = vec->data();
  fb.data_bytes_ = vec->size();
  uint64_t bps = fb.bytes_per_sample();
  PSOUP_CHECK(bps > 0, "bytes per sample must be >0 (nchans*nbits >= 8)");
  if (fb.hdr_.nsamples == 0) fb.hdr_.nsamples = static_cast<int>(fb.data_bytes_ / bps);
  PSOUP_CHECK(fb.data_bytes_ >= static_cast<uint64_t>(fb.hdr_.nsamples) * bps, "data block too small");
  fb.owner_ = vec;
  return fb;
}

float Filterbank::cfreq() const {
  float fch1 = static_cast<float>(hdr_.fch1);
  float foff = static_cast<float>(hdr_.foff);
  float nch = static_cast<float>(static_cast<unsigned>(hdr_.nchans));
  if (foff < 0) return fch1 + foff * nch / 2;
  return fch1 - foff * nch / 2;
}

void Filterbank::write(const std::string& filename) const {
  std::ofstream out(filename, std::ios::binary);
  if (!out) PSOUP_THROW("cannot write " << filename);
  write_header(out, hdr_);
  out.write(reinterpret_cast<const char*>(data_), static_cast<std::streamsize>(data_bytes_));
  if (!out) PSOUP_THROW("write failed for " << filename);
}

TimeSeriesFile read_tim(const std::string& filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) PSOUP_THROW("cannot open " << filename);
  TimeSeriesFile t;
  if (!read_header(in, t.header)) PSOUP_THROW(filename << " is not a SIGPROC time series");
  const int nbits = t.header.nbits;
  const uint64_t n = static_cast<uint64_t>(t.header.nsamples);
  t.data.resize(n);
  if (nbits == 32) {
    in.read(reinterpret_cast<char*>(t.data.data()), static_cast<std::streamsize>(n * 4));
  } else if (nbits == 8) {
    std::vector<uint8_t> raw(n);
    in.read(reinterpret_cast<char*>(raw.data()), static_cast<std::streamsize>(n));
    bool sgn = t.header.signed_data != 0;
    for (uint64_t i = 0; i < n; ++i)
      t.data[i] = sgn ? static_cast<float>(static_cast<int8_t>(raw[i])) : static_cast<float>(raw[i]);
  } else {
    PSOUP_THROW("unsupported .tim nbits=" << nbits);
  }
  return t;
}

void write_tim(const std::string& filename, const SigprocHeader& hdr_in, const std::vector<float>& data) {
  SigprocHeader hdr = hdr_in;
  hdr.nbits = 32;
  hdr.nchans = 1;
  hdr.nsamples = static_cast<int>(data.size());
  hdr.data_type = 2;
  std::ofstream out(filename, std::ios::binary);
  if (!out) PSOUP_THROW("cannot write " << filename);
  write_header(out, hdr);
  out.write(reinterpret_cast<const char*>(data.data()), static_cast<std::streamsize>(data.size() * 4));
}

std::vector<int> read_killfile(const std::string& filename, int nchans, bool* ok) {
  std::ifstream in(filename);
  if (!in) PSOUP_THROW("cannot open killfile " << filename);
  std::vector<int> mask;
  std::string line;
  int ii = 0;
  while (ii < nchans && std::getline(in, line)) {
    mask.push_back(std::atoi(line.c_str()));
    ++ii;
  }
  if (static_cast<int>(mask.size()) != nchans) {
    std::cerr << "WARNING: killmask is not the same size as nchans" << std::endl;
    std::cerr << mask.size() << " != " << nchans << std::endl;
    if (ok) *ok = false;
    return std::vector<int>(static_cast<size_t>(nchans), 1);
  }
  if (ok) *ok = true;
  return mask;
}

void read_zapfile(const std::string& filename, std::vector<float>& freqs, std::vector<float>& widths) {
  std::ifstream in(filename);
  if (!in) PSOUP_THROW("cannot open zapfile " << filename);
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string a, b;
    if (!(ss >> a)) continue;
    if (!(ss >> b)) continue;
    freqs.push_back(static_cast<float>(std::atof(a.c_str())));
    widths.push_back(static_cast<float>(std::atof(b.c_str())));
  }
}

// ------------------------------------------------------------------ DADA ---
namespace {
std::string dada_value(const std::string& text, const std::string& key) {
  const size_t pos = text.find(key + " ");
  if (pos == std::string::npos) return "";
  std::istringstream is(text.substr(pos + key.size() + 1));
  std::string v;
  is >> v;
  return v;
}
}  // namespace

DadaHeader parse_dada_header(const std::string& text, size_t payload_bytes) {
  DadaHeader h;
  auto s = [&](const char* k) { return dada_value(text, k); };
  auto i = [&](const char* k) { return std::atoi(s(k).c_str()); };
  auto f = [&](const char* k) { return std::atof(s(k).c_str()); };
  h.filesize = payload_bytes;
  h.header_version = static_cast<float>(f("HDR_VERSION"));
  h.header_size = static_cast<unsigned>(i("HDR_SIZE"));
  h.bw = i("BW");  // integer parse, as the reference
  h.freq = f("FREQ");
  h.nant = static_cast<unsigned>(i("NANT"));
  h.nchan = static_cast<unsigned>(i("NCHAN"));
  h.ndim = static_cast<unsigned>(i("NDIM"));
  h.npol = static_cast<unsigned>(i("NPOL"));
  h.nbit = static_cast<unsigned>(i("NBIT"));
  h.tsamp = f("TSAMP");
  h.osamp_ratio = f("OSAMP_RATIO");
  h.source_name = s("SOURCE");
  h.ra = s("RA");
  h.dec = s("DEC");
  h.proc_file = s("PROC_FILE");
  h.mode = s("MODE");
  h.observer = s("OBSERVER");
  h.pid = s("PID");
  h.obs_offset = static_cast<size_t>(i("OBS_OFFSET"));
  h.telescope = s("TELESCOPE");
  h.instrument = s("INSTRUMENT");
  h.dsb = static_cast<size_t>(i("DSB"));
  h.dada_filesize = static_cast<size_t>(i("FILE_SIZE"));
  const double denom = static_cast<double>(h.nchan) * h.nant * h.npol * 2.0;
  h.nsamples = denom > 0 ? static_cast<size_t>(static_cast<double>(payload_bytes) / denom) : 0;
  h.bytes_per_sec = static_cast<size_t>(i("BYTES_PER_SECOND"));
  h.utc_start = s("UTC_START");
  h.ant_id = static_cast<unsigned>(i("ANT_ID"));
  h.file_no = static_cast<unsigned>(i("FILE_NUMBER"));
  return h;
}

DadaHeader read_dada_header(const std::string& filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) PSOUP_THROW("cannot open DADA file " << filename);
  std::string buf(kDadaHeaderSize, '\0');
  in.read(&buf[0], static_cast<std::streamsize>(kDadaHeaderSize));
  const size_t got = static_cast<size_t>(in.gcount());
  buf.resize(got);
  in.seekg(0, std::ios::end);
  const size_t total = static_cast<size_t>(in.tellg());
  return parse_dada_header(buf, total > kDadaHeaderSize ? total - kDadaHeaderSize : 0);
}

}  // namespace psoup
