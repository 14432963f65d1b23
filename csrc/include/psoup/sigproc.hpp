// SIGPROC filterbank / time-series I/O.
//
// Parity: include/data_types/header.hpp:171-403 (SigprocHeader, header_write
// overloads, detail::header_read with 1..79-byte keys, read_header with the
// nsamples-from-file-size derivation) and include/data_types/filterbank.hpp:
// 44-238 (Filterbank metadata, get_cfreq, SigprocFilterbank reading the whole
// file into host RAM).  Here the data block is memory-mapped instead of copied,
// so a multi-GB filterbank costs no host copy before its H2D transfer.
#pragma once

#include <cstdint>
#include <istream>
#include <memory>
#include <ostream>
#include <string>
#include <vector>

namespace psoup {

struct SigprocHeader {
  std::string source_name;
  std::string rawdatafile;
  double az_start = 0.0;
  double za_start = 0.0;
  double src_raj = 0.0;
  double src_dej = 0.0;
  double tstart = 0.0;
  double tsamp = 0.0;
  double period = 0.0;
  double fch1 = 0.0;
  double foff = 0.0;
  int nchans = 0;
  int telescope_id = 0;
  int machine_id = 0;
  int data_type = 0;
  int ibeam = 0;
  int nbeams = 0;
  int nbits = 0;
  int barycentric = 0;
  int pulsarcentric = 0;
  int nbins = 0;
  int nsamples = 0;
  int nifs = 0;
  int npuls = 0;
  double refdm = 0.0;
  unsigned char signed_data = 0;
  uint64_t size = 0;  // header size in bytes
  // Which keys were present in the file (for a faithful re-write).
  std::vector<std::string> keys_present;
  bool has(const std::string& key) const;
};

// Parses a header; returns false (and rewinds) when the stream does not start
// with HEADER_START. Unknown keys produce a warning on stderr, like the
// reference. If nsamples is absent/zero it is derived from the stream size.
bool read_header(std::istream& in, SigprocHeader& hdr);
SigprocHeader read_header_file(const std::string& filename);

// Writes HEADER_START ... HEADER_END with the given header. Only keys that
// are "meaningful" are written: all numeric keys that are non-zero plus the
// mandatory ones (nchans, nbits, tsamp, fch1, foff, nifs, data_type), plus
// any key listed in hdr.keys_present.
void write_header(std::ostream& out, const SigprocHeader& hdr);

// A filterbank: metadata + packed data (time-major, nchans*nbits/8 bytes per
// sample, sub-byte samples packed LSB-first).
class Filterbank {
 public:
  Filterbank() = default;
  // Memory-maps `filename` (read-only). Throws on error.
  static Filterbank from_file(const std::string& filename);
  // Wraps an in-memory copy (used by the synthetic generator and tests).
  static Filterbank from_memory(const SigprocHeader& hdr, std::vector<uint8_t> data);

  const SigprocHeader& header() const { return hdr_; }
  const uint8_t* data() const { return data_; }
  uint64_t data_bytes() const { return data_bytes_; }
  uint64_t nsamps() const { return static_cast<uint64_t>(hdr_.nsamples); }
  int nchans() const { return hdr_.nchans; }
  int nbits() const { return hdr_.nbits; }
  double tsamp() const { return hdr_.tsamp; }
  double fch1() const { return hdr_.fch1; }
  double foff() const { return hdr_.foff; }
  uint64_t bytes_per_sample() const { return static_cast<uint64_t>(hdr_.nchans) * hdr_.nbits / 8; }
  // filterbank.hpp:190-196, evaluated in float like the reference.
  float cfreq() const;
  void write(const std::string& filename) const;
  // Bytes [off, off + n) of the data block into dst: pread() from the file on
  // up to nthreads threads when file-backed (the device upload's staging
  // reads), else a copy.
  void read_data(uint64_t off, uint64_t n, uint8_t* dst, int nthreads = 4) const;

 private:
  SigprocHeader hdr_;
  std::shared_ptr<void> owner_;  // munmap / vector owner
  const uint8_t* data_ = nullptr;
  uint64_t data_bytes_ = 0;
  std::string path_;  // file-backed: the file and its data block's offset
  uint64_t data_offset_ = 0;
};

// SIGPROC .tim time series (8-bit unsigned or 32-bit float samples).
struct TimeSeriesFile {
  SigprocHeader header;
  std::vector<float> data;
};
TimeSeriesFile read_tim(const std::string& filename);
void write_tim(const std::string& filename, const SigprocHeader& hdr, const std::vector<float>& data);

// Killfile: one integer per line, 0 = channel killed.  Mirrors
// dedisperser.hpp:71-95: at most nchans lines are read; if the count does not
// equal nchans a warning is printed and an all-ones mask is returned.
std::vector<int> read_killfile(const std::string& filename, int nchans, bool* ok = nullptr);

// Zapfile (birdie list): whitespace-separated "freq width" per line
// (birdiezapper.hpp:34-45).  Lines with fewer than 2 fields are skipped
// (the reference would read out of bounds on such lines).
void read_zapfile(const std::string& filename, std::vector<float>& freqs, std::vector<float>& widths);

// PSRDADA ASCII header (the first 4096 bytes of a .dada file), with the
// field set and parse semantics of DadaHeader::fromfile (header.hpp:52-161):
// first occurrence of "KEY " anywhere in the header, BW read as an integer,
// nsamples = payload bytes / nchan / nant / npol / 2.
constexpr size_t kDadaHeaderSize = 4096;
struct DadaHeader {
  float header_version = 0.f;
  unsigned header_size = 0;
  double bw = 0, freq = 0;
  unsigned nant = 0, nchan = 0, ndim = 0, npol = 0, nbit = 0;
  double tsamp = 0, osamp_ratio = 0;
  std::string source_name, ra, dec, proc_file, mode, observer, pid, telescope, instrument, utc_start;
  size_t obs_offset = 0, dsb = 0, filesize = 0, dada_filesize = 0, nsamples = 0, bytes_per_sec = 0;
  unsigned ant_id = 0, file_no = 0;
};
DadaHeader parse_dada_header(const std::string& text, size_t payload_bytes);
DadaHeader read_dada_header(const std::string& filename);

}  // namespace psoup
